#!/bin/bash
# Same-box A/B of two builds of the HIP library on the DeiT-S training step (run on the GPU box):
#   tools/ab_lib.sh <lib A .so> <lib B .so> [extra bench.py args]
# alternates A, B, A, B and prints img/s and ms/step of each run.
A=$1; B=$2; shift 2
for L in "$A" "$B" "$A" "$B"; do
  echo -n "$(basename "$L") "
  SAE_ATTN_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-headline "$@" 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
