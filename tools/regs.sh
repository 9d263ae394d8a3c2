#!/bin/bash
# Per-kernel register / spill / occupancy report for the HIP library (hipcc resource remarks).
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-mfma-vgpr-form=1 -fno-honor-nans -fno-slp-vectorize $REGS_FLAGS -I include \
  self-attention-experiments-vision_amd/csrc/capi.hip -o /tmp/_regs.so -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys,re,subprocess
cur=None; rows={}
for line in sys.stdin:
    if 'error' in line: print(line.rstrip())
    m=re.search(r'remark: (.*?) \[-Rpass',line)
    if not m: continue
    t=m.group(1)
    if t.startswith('Function Name:'):
        cur=t.split(':',1)[1].strip(); rows[cur]={}
    elif cur:
        k,v=t.split(':',1); rows[cur][k.strip()]=v.strip()
pat=sys.argv[1] if len(sys.argv)>1 else ''
for k,v in rows.items():
    name=subprocess.run(['c++filt',k],capture_output=True,text=True).stdout.strip().replace('sae::','')
    if pat and not re.search(pat,name): continue
    print(f\"{name[:75]:75s} V={v.get('VGPRs')} A={v.get('AGPRs')} spill={v.get('VGPRs Spill')} occ={v.get('Occupancy [waves/SIMD]')} lds={v.get('LDS Size [bytes/block]')}\")
" "$1"
