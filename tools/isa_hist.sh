#!/bin/bash
# Instruction histogram of one kernel (mangled-name substring) of the HIP library.
cd "$(dirname "$0")/.." && mkdir -p /tmp/isa && cd /tmp/isa && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
  -mllvm -amdgpu-mfma-vgpr-form=1 -fno-honor-nans -fno-slp-vectorize -I /root/repo/include /root/repo/self-attention-experiments-vision_amd/csrc/capi.hip \
  -save-temps -o /tmp/isa/x.so 2>/dev/null
python3 - "$1" <<'PY'
import sys, re
from collections import Counter
s = open('/tmp/isa/capi-hip-amdgcn-amd-amdhsa-gfx950.s').read()
names = re.findall(r'^(_Z\S+):', s, re.M)
pat = sys.argv[1]
for name in names:
    if pat not in name: continue
    i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
    lines = [l.strip() for l in s[i:j].split('\n') if l.strip() and not l.strip().startswith(('.', ';', '_Z'))]
    c = Counter(l.split()[0] for l in lines)
    print(name, 'total', len(lines))
    print('  ', ', '.join(f'{k}:{v}' for k, v in c.most_common(45)))
PY
