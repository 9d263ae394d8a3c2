#!/usr/bin/env python3
"""Build libsae_attn.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed).

Usage: python build.py [--force] [--debug] [--dev] [--stamps]

--dev builds the development library libsae_attn_dev.so (schedule-variant knobs read from the
environment, SAE_DEV_KNOBS); tools load it through SAE_ATTN_LIB.  --stamps builds
libsae_attn_stamp.so (the dev knobs plus in-kernel s_memtime stamps, tools/stamps.py).  The release library
libsae_attn.so never reads the environment on a launch path.
"""
import argparse
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "self-attention-experiments-vision_amd")
SRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "libsae_attn.so")
OUT_DEV = os.path.join(PKG, "libsae_attn_dev.so")
OUT_STAMP = os.path.join(PKG, "libsae_attn_stamp.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SAE_ARCH", "gfx950")


def sources():
    return sorted(os.path.join(SRC, f) for f in os.listdir(SRC) if f.endswith((".hip", ".h")))


def up_to_date(out=OUT):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    deps = sources() + [os.path.join(ROOT, "include", "sae_attn.h")]
    return all(os.path.getmtime(p) <= t for p in deps)


def unit_deps(path, seen=None):
    """The translation unit and every local header it includes (recursively)."""
    seen = set() if seen is None else seen
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    for line in open(path):
        line = line.strip()
        if line.startswith("#include \""):
            inc = line.split('"')[1]
            for d in (os.path.dirname(path), os.path.join(ROOT, "include")):
                if os.path.exists(os.path.join(d, inc)):
                    unit_deps(os.path.join(d, inc), seen)
                    break
    return seen


# translation units: (source, extra flags).  capi.hip keeps every MFMA accumulator in VGPRs
# (-amdgpu-mfma-vgpr-form: the exp / rescale VALU reads them directly); bwd_agpr.hip holds the
# one-wave-per-SIMD kernels, whose dK / dV accumulators go to the AGPR half of the register file.
UNITS = [("capi.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]), ("bwd_agpr.hip", [])]


def build(force=False, debug=False, verbose=True, dev=False, stamps=False):
    out = OUT_STAMP if stamps else (OUT_DEV if dev else OUT)
    if not force and up_to_date(out):
        if verbose:
            print(f"[build] {out} is up to date")
        return out
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
              "-fno-honor-nans", "-fno-slp-vectorize", "-I", os.path.join(ROOT, "include")]
    if debug:
        common.append("-g")
    if dev or stamps:
        common.append("-DSAE_DEV_KNOBS")
    if stamps:
        common.append("-DSAE_STAMPS")
    tag = os.path.basename(out).replace(".so", "") + ("_g" if debug else "")
    # objects cached per library flavour and compile command (compiler, arch, flags: a change of
    # any of them is a different directory): a unit is recompiled only when it or a header it
    # includes changed (capi.hip takes ~2 minutes; the attention units seconds)
    key = hashlib.sha1(repr((common, UNITS)).encode()).hexdigest()[:12]
    objdir = os.path.join(ROOT, "build", f"{tag}_{ARCH}_{key}")
    os.makedirs(objdir, exist_ok=True)
    objs, procs = [], []
    for src, extra in UNITS:
        path = os.path.join(SRC, src)
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and all(
                os.path.getmtime(d) <= os.path.getmtime(obj) for d in unit_deps(path)):
            continue
        cmd = common + extra + ["-c", path, "-o", obj + ".tmp"]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), obj))
    failed = None
    for p, obj in procs:   # wait for every child before reporting a failure
        if p.wait() != 0:
            failed = failed or p.returncode
        else:
            os.replace(obj + ".tmp", obj)
    if failed is not None:
        raise subprocess.CalledProcessError(failed, "hipcc")
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"]
    if verbose:
        print("[build]", " ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--dev", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="diagnostic build with in-kernel cycle stamps")
    a = ap.parse_args()
    build(a.force, a.debug, dev=a.dev, stamps=a.stamps)
    sys.exit(0)
