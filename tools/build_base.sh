#!/bin/bash
# Build the library from a git revision's csrc (default HEAD) as <pkg>/libsae_attn_base.so, for
# same-box A/B runs against the working tree (load it with SAE_ATTN_LIB=<that path>).  Every
# translation unit of that revision's csrc is compiled (capi.hip with the VGPR-form MFMA flag,
# the others without), as build.py does.
set -e
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
tmp=$(mktemp -d)
git archive "$rev" self-attention-experiments-vision_amd/csrc include | tar -x -C "$tmp"
src="$tmp/self-attention-experiments-vision_amd/csrc"
common=(/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
        -fno-honor-nans -fno-slp-vectorize -I "$tmp/include")
objs=()
for f in "$src"/*.hip; do
  extra=()
  [ "$(basename "$f")" = capi.hip ] && extra=(-mllvm -amdgpu-mfma-vgpr-form=1)
  "${common[@]}" "${extra[@]}" -c "$f" -o "$f.o" &
  objs+=("$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o self-attention-experiments-vision_amd/libsae_attn_base.so
rm -rf "$tmp"
echo "built libsae_attn_base.so from $rev"
