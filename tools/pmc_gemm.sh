#!/bin/bash
# PMC passes for a GEMM investigation (one rocprofv3 run per pass; <= 8 SQ / 4 TCC counters each)
# usage (GPU box): tools/pmc_gemm.sh <outdir> <program args...>
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE GRBM_COUNT"
  "TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAIT_INST_LDS"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$out/pass$i" -o run -- "$@" > "$out/pass$i.log" 2>&1 || echo "pass $i rc $?" >> "$out/fail.log"
  i=$((i+1))
done
echo PMC_DONE
