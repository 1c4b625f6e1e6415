"""The world > 1 path of the headline bench with the real kernels (SURVEY.md §8e,
BASELINE configs[3]: B = 512 windows strong-sharded over ranks).

RCCL refuses two ranks on one device, so two fresh processes share the one GPU of the
test box and talk over gloo (which all-reduces CUDA tensors through host memory): the
sharded exact path 512 -> 2 x 256, the per-step MLL rows all-reduced once by
ObjectiveAccumulator.reduce, the barrier and the MAX all-reduce of the timed region --
bench.py's own code, launched by torch.distributed.run. The parent process makes no GPU
call before it spawns the ranks. Not a scaling measurement.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--strong", "--B", "512", "--steps", "4", "--warmup", "2", "--no-var", "--no-var3",
          "--no-grad", "--no-e2e", "--no-cfg2", "--no-cpu-baseline"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench_line(cmd):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_world2_strong_sharded_exact_matches_single_process():
    single = _bench_line([sys.executable, "bench.py"] + COMMON)
    two = _bench_line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                       "--backend", "gloo", "--share-device"] + COMMON)
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 512
    assert two["config"]["windows_per_gpu"] == 256 and two["config"]["process_group"] == "gloo"
    assert single["config"]["global_batch"] == 512
    # the all-reduced mean MLL of the two shards equals the one-process value (the windows
    # are the same; the 256-window launches may use the small-batch layout, so allow
    # fp32 rounding)
    assert abs(two["mean_mll"] - single["mean_mll"]) <= 1e-5 * abs(single["mean_mll"]), (two["mean_mll"], single["mean_mll"])
    # the reported times are the MAX over the ranks' own times
    rt = two["rank_times"]
    assert len(rt["ms_per_step"]) == 2 and len(rt["kernel_ms"]) == 2
    assert abs(two["ms_per_step"] - max(rt["ms_per_step"])) <= 1e-9 * max(rt["ms_per_step"])
    assert abs(two["roofline"]["kernel_ms"] - max(rt["kernel_ms"])) <= 1e-9 * max(rt["kernel_ms"])
    assert two["value"] > 0
