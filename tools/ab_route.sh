# same-box A/B of the GEMM routing: narrow deep input gradients on the library (A) vs sae_gemm_nt (B)
for K in 0 1536 0 1536; do
  echo -n "narrow_max_k=$K "
  timeout -k 10 200 python -u -c "
import sys, runpy
sys.path.insert(0, '.')
import sae_vision_amd.ops as o
o.GEMM_NT_NARROW_MAX_K = $K
sys.argv = ['bench.py', '--no-cpu-baseline', '--no-headline']
runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
