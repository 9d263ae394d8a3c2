#!/bin/bash
# Exact read bytes by request size (gfx950: TCC_EA0_RDREQ_{32,64,128}B) and L2 hit / miss counts
# over a program, one rocprofv3 run per pass.  usage (GPU box): tools/pmc_bytes.sh <outdir> <program args...>
set -e
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
passes=(
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$out/pass$i" -o run -- "$@" > "$out/pass$i.log" 2>&1
  i=$((i+1))
done
echo PMC_BYTES_DONE
