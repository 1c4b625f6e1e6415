"""Turn rocprofv3 outputs under gpurun_out/ into the committed profiles/ summaries.

python scripts/summarize_profiles.py --round r01 [--src gpurun_out] [--B 512 --N 256 --D 32]

Writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim copy)
  profiles/<round>_pmc.json           per-kernel FETCH_SIZE / WRITE_SIZE averages (raw + corrected)
  profiles/pmc_exact_summary.json     {"B512_N256_D32": {"hbm_bytes_per_launch": ...}} read by bench.py

Units / corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide
coalesced read (16 B/lane) -> x2; WRITE_SIZE is exact for 16 B/lane stores. The
exact kernel's global traffic is exactly those two shapes (float4 X/y loads,
float4 L stores, scalar mll/info stores that are negligible).
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def pmc_avg(path: str, counter: str):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r01")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--D", type=int, default=32)
    a = ap.parse_args()
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)

    stats = os.path.join(a.src, "prof_exact", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{a.round}_kernel_stats.csv"))
    kstats = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            kstats[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                                          "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])}

    fetch, nf = pmc_avg(os.path.join(a.src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, nw = pmc_avg(os.path.join(a.src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    per = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("gpk_"):
            continue
        fb = fetch.get(k, 0.0) * 1024 * 2       # KiB, x2 gfx950 wide-read correction
        wb = write.get(k, 0.0) * 1024
        per[k] = {"fetch_kib_raw": fetch.get(k), "write_kib_raw": write.get(k),
                  "launches": [nf.get(k, 0), nw.get(k, 0)],
                  "fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                  "kernel_stats": kstats.get(k)}
    meta = {"workload": f"bench.py B={a.B} N={a.N} D={a.D}",
            "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count of 16B/lane reads); WRITE_SIZE KiB x1024",
            "kernels": per}
    with open(os.path.join(out, f"{a.round}_pmc.json"), "w") as f:
        json.dump(meta, f, indent=1)
    exact = [v for k, v in per.items() if k.startswith("gpk_exact_kernel")]
    if exact:
        summ = {f"B{a.B}_N{a.N}_D{a.D}": {"hbm_bytes_per_launch": exact[0]["hbm_bytes_per_launch"],
                                           "source": f"profiles/{a.round}_pmc.json"}}
        with open(os.path.join(out, "pmc_exact_summary.json"), "w") as f:
            json.dump(summ, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
