#!/bin/bash
# Build the library from a git revision's csrc (default HEAD) as <pkg>/libsae_attn_base.so, for
# same-box A/B runs against the working tree (load it with SAE_ATTN_LIB=<that path>).
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
tmp=$(mktemp -d)
git archive "$rev" self-attention-experiments-vision_amd/csrc include | tar -x -C "$tmp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form=1 \
  -fno-honor-nans -fno-slp-vectorize -I "$tmp/include" "$tmp/self-attention-experiments-vision_amd/csrc/capi.hip" \
  -o self-attention-experiments-vision_amd/libsae_attn_base.so
rm -rf "$tmp"
echo "built libsae_attn_base.so from $rev"
