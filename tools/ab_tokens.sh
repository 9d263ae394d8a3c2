#!/bin/bash
# Same-box A/B of the encoder input on the DeiT-S step: the torch composition (cat + upcast + add,
# autograd's residual sum; A) vs sae_tokens_fwd/_bwd + the LayerNorm pass (B), alternating A B A B.
for M in torch hip torch hip; do
  echo -n "tokens=$M "
  timeout -k 10 200 python -u -c "
import sys, runpy
sys.path.insert(0, '.')
import sae_vision_amd.ops as o
if '$M' == 'torch':
    o.encoder_tokens_ok = lambda *a: False
    o.layer_norm_pass = lambda x, g, b, eps=o.LN_EPS: (x, o.layer_norm(x, g, b, eps))
sys.argv = ['bench.py', '--no-cpu-baseline', '--no-headline']
runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['e2e']['final_loss'])"
done
