#!/bin/bash
# Same-box A/B of the training loss on the DeiT-S step: torch's cross entropy (A) vs the two-launch
# HIP loss (B), alternating A B A B (run on the GPU box from the repo root).
for M in torch hip torch hip; do
  echo -n "loss=$M "
  timeout -k 10 200 python -u -c "
import sys, runpy
sys.path.insert(0, '.')
import torch.nn.functional as F
import sae_vision_amd.train as t
if '$M' == 'torch':
    t.smoothed_cross_entropy = lambda x, y, s=0.1: F.cross_entropy(x.float(), y, label_smoothing=s)
sys.argv = ['bench.py', '--no-cpu-baseline', '--no-headline']
runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['e2e']['final_loss'])"
done
