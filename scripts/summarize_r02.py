"""Round-2 profile summaries: gpurun_out/r02 (scripts/gpu_r02e.sh) -> profiles/.

Writes
  profiles/r02_kernel_stats.csv     rocprofv3 --kernel-trace --stats of `bench.py` (verbatim)
  profiles/r02_pmc.json             per-kernel FETCH_SIZE / WRITE_SIZE per launch (raw KiB and
                                    corrected bytes) from separate --pmc passes of the same bench
  profiles/pmc_summary.json         HBM bytes per launch read by bench.py's `roofline.traffic`
  profiles/r02_bench.json           the bench line of that run
  profiles/r02_gp_step_cfg{1,3}.json  scripts/gp_step.py (end-to-end step, GP share)

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports 1/2 of a wide (16 B/lane) coalesced read -> x2 for the exact kernel,
whose loads are all 16 B/lane; the variational forward reads X with 4 B/lane loads
(uncalibrated width), so its fetch is reported raw and x2 side by side.
"""
import csv
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "r02")
OUT = os.path.join(ROOT, "profiles")


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def pmc(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[(short(row["Kernel_Name"]), int(row["Grid_Size"]))].append(float(row["Counter_Value"]))
    return acc


def main():
    os.makedirs(OUT, exist_ok=True)
    shutil.copy(os.path.join(SRC, "prof", "bench_kernel_stats.csv"), os.path.join(OUT, "r02_kernel_stats.csv"))
    for name in ["bench.json", "gp_step_cfg3.json", "gp_step_cfg1.json"]:
        src = os.path.join(SRC, name)
        if os.path.exists(src):
            with open(src) as f:
                d = json.loads(f.read().strip().splitlines()[-1])
            with open(os.path.join(OUT, f"r02_{name}"), "w") as f:
                json.dump(d, f, indent=1)
    fetch = pmc(os.path.join(SRC, "pmc_fetch", "bench_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(SRC, "pmc_write", "bench_counter_collection.csv"), "WRITE_SIZE")
    rows = {}
    for key in sorted(set(fetch) | set(write)):
        if "gpk" not in key[0]:
            continue
        f = fetch.get(key, [0.0])
        w = write.get(key, [0.0])
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        rows[f"{key[0]} grid={key[1]}"] = {
            "launches": len(f), "fetch_kib": fk, "write_kib": wk,
            "fetch_bytes_x2": fk * 1024 * 2, "write_bytes": wk * 1024,
            "hbm_bytes_per_launch": fk * 1024 * 2 + wk * 1024}
    with open(os.path.join(OUT, "r02_pmc.json"), "w") as fo:
        json.dump(rows, fo, indent=1)
    summary = {}
    for k, v in rows.items():
        if k.startswith("gpk_exact_kernel<16, 8, false, true>"):   # N=256 (not the cfg-2 leg)
            summary["exact_B512_N256_D32"] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                              "source": "profiles/r02_pmc.json " + k}
        if k.startswith("gpk_var_fwd_r_kernel<32>") or k.startswith("gpk_var_fwd_kernel<4>"):
            summary["var_B1024_N256_M64_D32"] = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"],
                                                 "fetch_raw_bytes": v["fetch_kib"] * 1024,
                                                 "source": "profiles/r02_pmc.json " + k}
    with open(os.path.join(OUT, "pmc_summary.json"), "w") as fo:
        json.dump(summary, fo, indent=1)
    print(json.dumps(summary, indent=1))
    for k, v in rows.items():
        print(f"{k:50s} fetch x2 {v['fetch_bytes_x2'] / 1e6:9.2f} MB  write {v['write_bytes'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
