#!/bin/bash
# PMC passes (one rocprofv3 run per pass, <= 8 SQ / 4 TCC counters each) over a program.
# usage (on the GPU box): tools/pmc.sh <outdir> <program args...>
# e.g.  tools/pmc.sh gpurun_out/pmc python3 tools/attn_bench.py --shapes vitb384 --iters 5
set -e
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE GRBM_COUNT"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$out/pass$i" -o run -- "$@" > "$out/pass$i.log" 2>&1
  i=$((i+1))
done
echo PMC_DONE
