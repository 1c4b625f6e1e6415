"""Per-kernel register / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

    python scripts/resource_usage.py fine_grained_gaussian_process_forcasting_amd/csrc/gpk_variational.hip [filter]
"""
import re
import subprocess
import sys

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ""
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                    "-I", f"{ROOT}/include", "-c", src, "-o", "/tmp/_ru.o",
                    "-Rpass-analysis=kernel-resource-usage"] + defs, capture_output=True, text=True)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
print(f"{'kernel':60s} {'VGPR':>5s} {'AGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'occ':>4s}")
for row in rows:
    n = row["name"]
    if flt and flt not in n:
        continue
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)[:60]
    print(f"{n:60s} {row.get('VGPRs', 0):5d} {row.get('AGPRs', 0):5d} {row.get('VGPRs Spill', 0):6d} "
          f"{row.get('SGPRs Spill', 0):6d} {row.get('Occupancy [waves/SIMD]', 0):4d}")
if r.returncode:
    print(r.stderr[-3000:])
