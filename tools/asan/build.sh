#!/bin/bash
# Host AddressSanitizer build + run of the C ABI (tools/asan/capi_asan.cpp).  Device code is
# compiled as in build.py; only the host side is instrumented (GPU ASan is unavailable on the
# pool).  CPU only: no GPU is touched.  Usage: tools/asan/build.sh [outdir]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${1:-/tmp/sae_asan}
mkdir -p "$OUT"
SRC="$ROOT/self-attention-experiments-vision_amd/csrc"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
COMMON=(--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -fno-honor-nans -fno-slp-vectorize -I "$ROOT/include"
        -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer)
"$HIPCC" "${COMMON[@]}" -mllvm -amdgpu-mfma-vgpr-form=1 -c "$SRC/capi.hip" -o "$OUT/capi.o" &
"$HIPCC" "${COMMON[@]}" -c "$SRC/bwd_agpr.hip" -o "$OUT/bwd_agpr.o" &
"$HIPCC" -O1 -g -std=c++17 -I "$ROOT/include" -Xarch_host -fsanitize=address -x c++ \
  -c "$ROOT/tools/asan/capi_asan.cpp" -o "$OUT/driver.o" &
wait %1 && wait %2 && wait %3
"$HIPCC" --offload-arch=gfx950 -fsanitize=address -fno-gpu-sanitize "$OUT/capi.o" "$OUT/bwd_agpr.o" \
  "$OUT/driver.o" -o "$OUT/capi_asan"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 "$OUT/capi_asan"
