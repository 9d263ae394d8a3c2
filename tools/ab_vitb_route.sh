# same-box A/B of the ViT-B/16@384 training step (B 32): round-2 GEMM routing on the HEAD library
# (A), round-2 routing on the working-tree library (B: 256-token GELU / GELU' tiles), every GEMM on
# sae_gemm_nt (C), sae_gemm_nt up to K = 768 (D); VARIANTS picks them.  Writes one line per run to gpurun_out/${TAG}_vitb_route.txt.
P=$PWD/self-attention-experiments-vision_amd
out=gpurun_out/${TAG:-ab}_vitb_route.txt
run() {  # $1 label, $2 lib, $3 routing (old|new)
  echo -n "$1 " >> $out
  SAE_ATTN_LIB=$2 timeout -k 10 240 python -u -c "
import sys, runpy
sys.path.insert(0, '.')
import sae_vision_amd.ops as o
if '$3' != 'new':
    o.GEMM_NT_ALL = False
    o.FF_NT_MAX_HIDDEN = 2048
if '$3' == 'k768':
    o.GEMM_NT_MAX_K = 768
sys.argv = ['bench.py', '--no-cpu-baseline', '--no-headline', '--model', 'vit_b_patch16', '--img-size', '384', '--batch', '32']
runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> $out
}
for r in 1 2; do
  for v in ${VARIANTS:-A B C}; do
    case $v in
      A) run A $P/libsae_attn_base.so old || exit 1 ;;
      B) run B $P/libsae_attn.so old || exit 1 ;;
      C) run C $P/libsae_attn.so new || exit 1 ;;
      D) run D $P/libsae_attn.so k768 || exit 1 ;;
    esac
  done
done
cat $out
