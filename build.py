#!/usr/bin/env python3
"""Build libsae_attn.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed).

Usage: python build.py [--force] [--debug] [--dev]

--dev builds the development library libsae_attn_dev.so (schedule-variant knobs read from the
environment, SAE_DEV_KNOBS); tools load it through SAE_ATTN_LIB.  The release library
libsae_attn.so never reads the environment on a launch path.
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "self-attention-experiments-vision_amd")
SRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "libsae_attn.so")
OUT_DEV = os.path.join(PKG, "libsae_attn_dev.so")
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


def build(force=False, debug=False, verbose=True, dev=False):
    out = OUT_DEV if dev else OUT
    if not force and up_to_date(out):
        if verbose:
            print(f"[build] {out} is up to date")
        return out
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-function", "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-honor-nans", "-fno-slp-vectorize", "-I", os.path.join(ROOT, "include"),
           os.path.join(SRC, "capi.hip"), "-o", out + ".tmp"]
    if debug:
        cmd.insert(3, "-g")
    if dev:
        cmd.insert(3, "-DSAE_DEV_KNOBS")
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--dev", action="store_true")
    a = ap.parse_args()
    build(a.force, a.debug, dev=a.dev)
    sys.exit(0)
