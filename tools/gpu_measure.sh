#!/bin/bash
# One-box measurement of a round (run on the GPU box from the repo root):
#   bench JSON, rocprofv3 kernel stats of the SAME build (training loop and attention bench),
#   PMC passes for the DeiT-S training step and the ViT-B@384 attention headline.
# usage: tools/gpu_measure.sh <tag>     -> gpurun_out/<tag>_*
set -e
tag=${1:-r02g}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-headline --model vit_b_patch16 --img-size 384 --batch 32 > gpurun_out/${tag}_bench_vitb16_384.json 2>> gpurun_out/${tag}_bench.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-headline --model cait_s_24 > gpurun_out/${tag}_bench_cait_s24.json 2>> gpurun_out/${tag}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_train -o run -- python3 bench.py --profile --steps 5 --warmup 3 > gpurun_out/${tag}_prof_train.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_attn -o run -- python3 tools/attn_bench.py --iters 10 > gpurun_out/${tag}_prof_attn.log 2>&1
timeout -k 10 300 python3 tools/attn_bench.py --iters 20 > gpurun_out/${tag}_attn_bench.txt 2>&1
timeout -k 10 300 python3 tools/attn_bench.py --shapes bot14,bot7 --rel --iters 20 >> gpurun_out/${tag}_attn_bench.txt 2>&1
timeout -k 10 300 python3 tools/attn_bench.py --shapes cait_s24,cait_m24 --th --iters 20 >> gpurun_out/${tag}_attn_bench.txt 2>&1
tools/pmc.sh gpurun_out/${tag}_pmc_b384 python3 tools/attn_bench.py --shapes vitb384 --iters 3
tools/pmc.sh gpurun_out/${tag}_pmc_th python3 tools/attn_bench.py --shapes cait_s24 --th --iters 3
tools/pmc.sh gpurun_out/${tag}_pmc_th_m24 python3 tools/attn_bench.py --shapes cait_m24 --th --iters 3
tools/pmc.sh gpurun_out/${tag}_pmc_deit python3 tools/attn_bench.py --shapes deit_s --iters 3
echo ALL_DONE
