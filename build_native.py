"""Build libgpk.so (HIP kernels + C ABI) for gfx950 in-tree.

Usage: python build_native.py [--force]
The .so lands in fine_grained_gaussian_process_forcasting_amd/_lib/ (git-ignored, but it
travels to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "fine_grained_gaussian_process_forcasting_amd")
CSRC = os.path.join(PKG, "csrc")
OUT_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(OUT_DIR, "libgpk.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall",
         "-Wno-unused-variable", "-Wno-unused-function", "-munsafe-fp-atomics"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(ROOT, "include", "gpk.h"))
    return sorted(hs)


def included(path, seen=None):
    """Local headers a source pulls in (quoted #include, transitively): the object digest
    covers exactly these, so editing one kernel's header does not rebuild every kernel."""
    import re
    seen = set() if seen is None else seen
    base = os.path.dirname(path)
    with open(path) as f:
        for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
            h = os.path.normpath(os.path.join(base, m.group(1)))
            if os.path.exists(h) and h not in seen:
                seen.add(h)
                included(h, seen)
    return seen


def _digest(paths, extra=""):
    h = hashlib.sha256(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = True, defines=(), out_dir: str = OUT_DIR) -> str:
    """Compile every csrc/*.hip for gfx950 and link libgpk.so into out_dir.
    `defines` (e.g. ["GPK_SPLIT_UPDATE=0"]) and a non-default out_dir are for
    A/B experiments only (load such a build with GPK_LIB=<path>)."""
    os.makedirs(out_dir, exist_ok=True)
    lib_path = os.path.join(out_dir, "libgpk.so")
    flags = FLAGS + [f"-D{d}" for d in defines]
    flag_str = " ".join(flags)
    objs = []
    jobs = []
    for src in sources():
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        stamp = obj + ".sha"
        dig = _digest([src] + sorted(included(src)), flag_str)
        objs.append(obj)
        if not force and os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == dig:
            continue
        jobs.append((src, obj, stamp, dig))

    def compile_one(job):
        src, obj, stamp, dig = job
        cmd = [HIPCC, *flags, "-I", os.path.join(ROOT, "include"), "-c", src, "-o", obj]
        if verbose:
            print("[build]", " ".join(os.path.basename(c) if c.startswith(ROOT) else c for c in cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        if r.stderr.strip() and verbose:
            print(r.stderr, file=sys.stderr)
        with open(stamp, "w") as f:
            f.write(dig)

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(compile_one, jobs))
    if jobs or not os.path.exists(lib_path):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib_path + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(lib_path + ".tmp", lib_path)
        if verbose:
            print("[build] linked", os.path.relpath(lib_path, ROOT), flush=True)
    return lib_path


# Measurement-only variant builds of the exact kernel (bench.py's "fp32_update" note: the
# pure-fp32 MFMA trailing update beside the split-f16 product path). Only gpk_exact.hip is
# recompiled (N = 128 / 256 instantiations); the other objects of the main build are linked in.
VARIANTS = {"f32update": ["GPK_SPLIT_UPDATE=0", "GPK_EXACT_DEV=1"]}


def build_variant(name: str, verbose: bool = True) -> str:
    main_lib = build(force=False, verbose=verbose)
    out_dir = os.path.join(PKG, "_lib_variants", name)
    os.makedirs(out_dir, exist_ok=True)
    lib_path = os.path.join(out_dir, "libgpk.so")
    src = os.path.join(CSRC, "gpk_exact.hip")
    obj = os.path.join(out_dir, "gpk_exact.hip.o")
    flags = FLAGS + [f"-D{d}" for d in VARIANTS[name]]
    objs = [os.path.join(OUT_DIR, os.path.basename(x) + ".o") for x in sources() if not x.endswith("gpk_exact.hip")]
    # the digest covers the variant's own source + flags AND the main-build objects it links
    # in (their .sha stamps), so a change to any other kernel relinks the variant too
    linked = "".join(open(o + ".sha").read() if os.path.exists(o + ".sha") else o for o in objs)
    dig = _digest([src] + sorted(included(src)), " ".join(flags) + main_lib + linked)
    stamp = obj + ".sha"
    if os.path.exists(lib_path) and os.path.exists(stamp) and open(stamp).read() == dig:
        return lib_path
    cmd = [HIPCC, *flags, "-I", os.path.join(ROOT, "include"), "-c", src, "-o", obj]
    if verbose:
        print("[build variant]", name, " ".join(VARIANTS[name]), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for the {name} variant:\n{r.stderr}")
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, obj, "-o", lib_path],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed for the {name} variant:\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(dig)
    return lib_path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D for A/B builds")
    ap.add_argument("--out-dir", default=OUT_DIR)
    args = ap.parse_args()
    build(force=args.force, defines=args.defines, out_dir=args.out_dir)
