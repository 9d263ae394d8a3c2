#!/bin/bash
# Validation pass on the GPU box (run from the repo root): GPU suite, smoke(), default bench.
#   tools/gpu_validate.sh <tag>   -> gpurun_out/<tag>_{tests.log,smoke.log,bench.json,bench.err}
set -o pipefail
tag=${1:-val}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
  || { echo "BENCH FAILED"; tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
