#!/bin/bash
# A/B of attention schedule variants on the development library (build.py --dev) + PMC passes.
# usage (on the GPU box): tools/gpu_ab.sh <tag> <shapes> <bwd-variants> [fwd-variants]
set -e
tag=$1; shapes=$2; bv=$3; fv=${4:-0}
export TMPDIR=/tmp
export SAE_ATTN_LIB=$PWD/self-attention-experiments-vision_amd/libsae_attn_dev.so
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/attn_bench.py --shapes $shapes --bwd-variants $bv --fwd-variants $fv > gpurun_out/ab_$tag.log 2>&1
cat gpurun_out/ab_$tag.log | grep -v amdgpu.ids
if [ -n "$PMC" ]; then
  tools/pmc.sh gpurun_out/pmc_$tag python3 tools/attn_bench.py --shapes $PMC --iters 3 --bwd-variants $bv --fwd-variants $fv
  python tools/pmc_summary.py gpurun_out/pmc_$tag bwd > gpurun_out/pmc_$tag.txt
  cat gpurun_out/pmc_$tag.txt
fi
