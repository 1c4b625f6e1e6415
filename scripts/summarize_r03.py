"""Round-3 profile summaries: gpurun_out/r03q (scripts/gpu_r03q.sh) -> profiles/.

Writes
  profiles/r03_kernel_stats.csv        rocprofv3 --kernel-trace --stats of `bench.py` (verbatim)
  profiles/r03_var3_kernel_stats.csv   the same for the cfg-3 variational legs (scripts/var3_leg.py)
  profiles/r03_pmc.json                per-kernel FETCH_SIZE / WRITE_SIZE per launch (raw KiB and
                                       corrected bytes) from separate --pmc passes
  profiles/pmc_summary.json            HBM bytes per launch read by bench.py's `roofline.traffic`
  profiles/r03_bench.json              the bench line of the kernel-stats run

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports 1/2 of a wide (16 B/lane) coalesced read -> x2 (reported beside the raw
value: kernels with narrower loads sit between the two).
"""
import csv
import glob
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "r03q")
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
            "launches": len(f), "fetch_kib": fk, "write_kib": wk,
            "fetch_bytes_raw": fk * 1024, "fetch_bytes_x2": fk * 1024 * 2, "write_bytes": wk * 1024,
            "hbm_bytes_per_launch": fk * 1024 * 2 + wk * 1024}
    return rows


def main():
    os.makedirs(OUT, exist_ok=True)
    for pat, dst in (("prof/**/bench_kernel_stats.csv", "r03_kernel_stats.csv"),
                     ("prof_var3/**/var3_kernel_stats.csv", "r03_var3_kernel_stats.csv")):
        src = one(pat)
        if src:
            shutil.copy(src, os.path.join(OUT, dst))
    bj = os.path.join(SRC, "bench.json")
    if os.path.exists(bj):
        with open(bj) as f:
            line = f.read().strip().splitlines()
        if line:
            with open(os.path.join(OUT, "r03_bench.json"), "w") as f:
                json.dump(json.loads(line[-1]), f, indent=1)
    rows = table(pmc(one("pmc_fetch/**/bench_counter_collection.csv"), "FETCH_SIZE"),
                 pmc(one("pmc_write/**/bench_counter_collection.csv"), "WRITE_SIZE"))
    rows3 = table(pmc(one("pmc_fetch_var3/**/var3_counter_collection.csv"), "FETCH_SIZE"),
                  pmc(one("pmc_write_var3/**/var3_counter_collection.csv"), "WRITE_SIZE"))
    with open(os.path.join(OUT, "r03_pmc.json"), "w") as fo:
        json.dump({"bench": rows, "var3_leg": rows3}, fo, indent=1)
    summary = {}
    for k, v in rows.items():
        if k.startswith("gpk_exact_kernel<16, 8, false, true") and k.endswith("grid=262144"):   # B=512 N=256
            summary["exact_B512_N256_D32"] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                              "source": "profiles/r03_pmc.json bench " + k}
        if k.startswith("gpk_var_fwd_r_kernel<32>"):
            summary["var_B1024_N256_M64_D32"] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                                 "fetch_raw_bytes": v["fetch_bytes_raw"],
                                                 "source": "profiles/r03_pmc.json bench " + k}
    adj = [v for k, v in rows.items() if k.split(" grid")[0] in (
        "gpk_var_adj_r_kernel<32>", "gpk_var_kgram_r_kernel<32>", "gpk_var_gdl_kernel", "gpk_var_fin_kernel")
        or (k.startswith("gpk_var_red_kernel") and not k.endswith("grid=596736"))]
    if adj:
        summary["var_adjoint_B1024_N256_M64_D32"] = {
            "hbm_bytes_per_launch": sum(v["hbm_bytes_per_launch"] for v in adj),
            "hbm_bytes_per_launch_raw": sum(v["fetch_bytes_raw"] + v["write_bytes"] for v in adj),
            "hbm_bytes_per_launch_x2": sum(v["hbm_bytes_per_launch"] for v in adj),
            "algorithmic_bytes": 4 * (2 * 1024 * 256 * 32 + 2 * 1024 * 256),
            "source": "profiles/r03_pmc.json bench gpk_var_adj_r / kgram_r / red / gdl / fin"}
    with open(os.path.join(OUT, "pmc_summary.json"), "w") as fo:
        json.dump(summary, fo, indent=1)
    print(json.dumps(summary, indent=1))
    for name, rr in (("bench", rows), ("var3_leg", rows3)):
        print(f"--- {name}")
        for k, v in rr.items():
            print(f"{k:70s} fetch raw {v['fetch_bytes_raw'] / 1e6:9.2f} MB  x2 {v['fetch_bytes_x2'] / 1e6:9.2f} MB"
                  f"  write {v['write_bytes'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
