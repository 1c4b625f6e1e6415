"""End-of-round evidence: gpurun_out/<tag> (scripts/r06/gpu_final.sh) -> profiles/rNN_*.

Writes
  profiles/rNN_kernel_stats.csv          rocprofv3 --kernel-trace --stats of bench.py (verbatim)
  profiles/rNN_var3_{192,96}_kernel_stats.csv   the same for the cfg-3 variational legs
  profiles/rNN_step_graph_gp_kernel_stats.csv   the graphed cfg-3 train step with / without GP
  profiles/rNN_pmc.json                  per-kernel FETCH_SIZE / WRITE_SIZE per launch
  profiles/pmc_summary.json              HBM bytes per launch read by bench.py's `traffic` fields
  profiles/rNN_bench.json, rNN_pytest_gpu.log, rNN_exact_stamps.txt, rNN_exact_timeline.txt

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports 1/2 of a wide (16 B/lane) coalesced read -> x2 (the raw value beside it).
    python scripts/summarize_round.py [round] [tag]      (default: r06 r06final)
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RND = sys.argv[1] if len(sys.argv) > 1 else "r06"
TAG = sys.argv[2] if len(sys.argv) > 2 else f"{RND}final"
SRC = os.path.join(ROOT, "gpurun_out", TAG)
OUT = os.path.join(ROOT, "profiles")


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def one(pattern):
    hits = glob.glob(os.path.join(SRC, pattern), recursive=True)
    return hits[0] if hits else None


def pmc(path, counter):
    acc = defaultdict(list)
    if path is None:
        return acc
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[(short(row["Kernel_Name"]), int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    return acc


def table(fetch, write):
    rows = {}
    for key in sorted(set(fetch) | set(write)):
        if "gpk" not in key[0]:
            continue
        f = fetch.get(key, [0.0])
        w = write.get(key, [0.0])
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        rows[f"{key[0]} grid={key[1]}"] = {
            "launches": len(f), "fetch_kib": fk, "write_kib": wk, "fetch_bytes_raw": fk * 1024,
            "fetch_bytes_x2": fk * 1024 * 2, "write_bytes": wk * 1024,
            "hbm_bytes_per_launch": fk * 1024 * 2 + wk * 1024}
    return rows


VAR3_FWD = ("gpk_var_fwd_l_kernel",)
# the saved-state adjoint: adjs (fp32 dK since round 6) -> kgram -> red (partials | G') -> fin (+ dL^-1 blocks)
VAR3_ADJ = ("gpk_var_adjs_l_kernel", "gpk_var_kgram_l_kernel", "gpk_var_red_kernel", "gpk_var_fin_kernel")


def main():
    os.makedirs(OUT, exist_ok=True)
    copies = [("prof/**/bench_kernel_stats.csv", f"{RND}_kernel_stats.csv"),
              ("prof_var3_192/**/var3_kernel_stats.csv", f"{RND}_var3_192_kernel_stats.csv"),
              ("prof_var3_96/**/var3_kernel_stats.csv", f"{RND}_var3_96_kernel_stats.csv"),
              ("step_graph-gp/**/step_kernel_stats.csv", f"{RND}_step_graph_gp_kernel_stats.csv")]
    for pat, dst in copies:
        src = one(pat)
        if src:
            shutil.copy(src, os.path.join(OUT, dst))
    for src, dst in (("pytest_gpu.log", f"{RND}_pytest_gpu.log"), ("stamps.txt", f"{RND}_exact_stamps.txt"),
                     ("stamps_col.txt", f"{RND}_exact_timeline.txt")):
        if os.path.exists(os.path.join(SRC, src)):
            shutil.copy(os.path.join(SRC, src), os.path.join(OUT, dst))
    bj = os.path.join(SRC, "bench.json")
    if os.path.exists(bj):
        lines = [ln for ln in open(bj).read().splitlines() if ln.startswith("{")]
        if lines:
            with open(os.path.join(OUT, f"{RND}_bench.json"), "w") as f:
                json.dump(json.loads(lines[-1]), f, indent=1)
    rows = table(pmc(one("pmc_fetch/**/bench_counter_collection.csv"), "FETCH_SIZE"),
                 pmc(one("pmc_write/**/bench_counter_collection.csv"), "WRITE_SIZE"))
    var3 = {n: table(pmc(one(f"pmc_fetch_var3_{n}/**/var3_counter_collection.csv"), "FETCH_SIZE"),
                     pmc(one(f"pmc_write_var3_{n}/**/var3_counter_collection.csv"), "WRITE_SIZE"))
            for n in (192, 96)}
    with open(os.path.join(OUT, f"{RND}_pmc.json"), "w") as fo:
        json.dump({"bench": rows, **{f"var3_N{n}": r for n, r in var3.items()}}, fo, indent=1)
    old = {}
    p = os.path.join(OUT, "pmc_summary.json")
    if os.path.exists(p):
        old = json.load(open(p))
    summary = dict(old)
    for k, v in rows.items():
        if k.startswith("gpk_exact_kernel<16, 8, false, true") and k.endswith("grid=262144"):   # B=512 N=256
            summary["exact_B512_N256_D32"] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                              "fetch_bytes_x2": v["fetch_bytes_x2"], "write_bytes": v["write_bytes"],
                                              "source": f"profiles/{RND}_pmc.json bench " + k}
        if k.startswith("gpk_var_fwd_r_kernel<32>"):
            summary["var_B1024_N256_M64_D32"] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                                 "fetch_raw_bytes": v["fetch_bytes_raw"],
                                                 "source": f"profiles/{RND}_pmc.json bench " + k}
    # cfg 5 (M = 64): the adjoint with the K-Gram folded in, ONE reduction of its
    # [adjoint | K-Gram] rows (155 blocks) and the output launch (4 dZ blocks + totals + dL^-1)
    adj = [v for k, v in rows.items() if k.startswith("gpk_var_adj_r_kernel<32")
           or k == "gpk_var_red_kernel grid=39680" or k == "gpk_var_fin_kernel grid=1536"]
    if adj:
        summary["var_adjoint_B1024_N256_M64_D32"] = {
            "hbm_bytes_per_launch": sum(v["hbm_bytes_per_launch"] for v in adj),
            "hbm_bytes_per_launch_raw": sum(v["fetch_bytes_raw"] + v["write_bytes"] for v in adj),
            "algorithmic_bytes": 4 * (2 * 1024 * 256 * 32 + 2 * 1024 * 256),
            "source": f"profiles/{RND}_pmc.json bench gpk_var_adj_r<32, 8, true> / red / fin"}
    for n, r in var3.items():
        fwd = [v for k, v in r.items() if k.split("<")[0].split(" ")[0] in VAR3_FWD]
        ad = [v for k, v in r.items() if k.split("<")[0].split(" ")[0] in VAR3_ADJ]
        if fwd:
            summary[f"var_B256_N{n}_M256_D32"] = {
                "hbm_bytes_per_launch": sum(v["hbm_bytes_per_launch"] for v in fwd),
                "source": f"profiles/{RND}_pmc.json var3_N{n} gpk_var_fwd_l_kernel"}
        if ad:
            summary[f"var_adjoint_B256_N{n}_M256_D32"] = {
                "hbm_bytes_per_launch": sum(v["hbm_bytes_per_launch"] for v in ad),
                "hbm_bytes_per_launch_raw": sum(v["fetch_bytes_raw"] + v["write_bytes"] for v in ad),
                "algorithmic_bytes": 4 * (2 * 256 * n * 32 + 2 * 256 * n),
                "note": "includes the forward's saved fp32 A read twice (adjs, kgram): 4 B N M per window",
                "source": f"profiles/{RND}_pmc.json var3_N{n} adjs / kgram / red / fin"}
    with open(p, "w") as fo:
        json.dump(summary, fo, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
