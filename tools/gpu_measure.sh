set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- python3 bench.py --profile --steps 5 --warmup 3 > gpurun_out/prof_train.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn -o run -- python3 tools/attn_bench.py --iters 10 > gpurun_out/prof_attn.log 2>&1
tools/pmc.sh gpurun_out/pmc_train python3 bench.py --profile --eager --steps 3 --warmup 2
tools/pmc.sh gpurun_out/pmc_b384 python3 tools/attn_bench.py --shapes vitb384 --iters 3
echo ALL_DONE
