#!/usr/bin/env python3
"""Build libsae_attn.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed).

Usage: python build.py [--force] [--debug]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "self-attention-experiments-vision_amd")
SRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "libsae_attn.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SAE_ARCH", "gfx950")


def sources():
    return sorted(os.path.join(SRC, f) for f in os.listdir(SRC) if f.endswith((".hip", ".h")))


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    deps = sources() + [os.path.join(ROOT, "include", "sae_attn.h")]
    return all(os.path.getmtime(p) <= t for p in deps)


def build(force=False, debug=False, verbose=True):
    if not force and up_to_date():
        if verbose:
            print(f"[build] {OUT} is up to date")
        return OUT
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-function", "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-honor-nans", "-I", os.path.join(ROOT, "include"),
           os.path.join(SRC, "capi.hip"), "-o", OUT + ".tmp"]
    if debug:
        cmd.insert(3, "-g")
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    build(a.force, a.debug)
    sys.exit(0)
