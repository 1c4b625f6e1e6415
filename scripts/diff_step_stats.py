"""GP share of a graphed training step by kernel: rocprofv3 kernel stats of
scripts/gp_step.py <cfg> <steps> graph-gp minus graph-nogp (per step).
    python scripts/diff_step_stats.py gpurun_out/<dir> [steps=23] [top=40]"""
import csv
import glob
import sys


def load(d, kind):
    f = glob.glob(f"{d}/step_{kind}/**/step_kernel_stats.csv", recursive=True)[0]
    return {x["Name"]: (int(x["Calls"]), float(x["TotalDurationNs"])) for x in csv.DictReader(open(f))}


d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 23
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
a, b = load(d, "graph-gp"), load(d, "graph-nogp")
ta, tb = sum(v[1] for v in a.values()), sum(v[1] for v in b.values())
print(f"kernel time per step: gp {ta / 1e6 / steps:.3f} ms, no-gp {tb / 1e6 / steps:.3f} ms, "
      f"difference {(ta - tb) / 1e6 / steps:.3f} ms")
rows = sorted(((a.get(k, (0, 0))[1] - b.get(k, (0, 0))[1], k) for k in set(a) | set(b)), reverse=True)
for dlt, k in rows[:top]:
    ca, cb = a.get(k, (0, 0))[0], b.get(k, (0, 0))[0]
    avg = a.get(k, (0, 0))[1] / max(ca, 1) / 1e3
    print(f"{dlt / 1e6 / steps:8.3f} ms/step  calls/step {(ca - cb) / steps:6.1f}  avg {avg:7.1f} us  {k[:80]}")
