#!/bin/bash
# Same-box A/B of the final LayerNorm on the DeiT-S step: over every token then token 0 selected (A)
# vs on the class-token rows only (ops.cls_add_layer_norm; B), alternating A B A B.
for M in full cls full cls; do
  echo -n "clsln=$M "
  timeout -k 10 200 python -u -c "
import sys, runpy
sys.path.insert(0, '.')
import sae_vision_amd.ops as o
if '$M' == 'full':
    o.cls_add_layer_norm = lambda x, f, g, b, eps=o.LN_EPS: o.add_layer_norm(x, f, g, b, eps)[1][:, 0]
sys.argv = ['bench.py', '--no-cpu-baseline', '--no-headline']
runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['e2e']['final_loss'])"
done
