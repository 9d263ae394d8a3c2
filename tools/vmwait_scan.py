#!/usr/bin/env python3
"""List `s_waitcnt vmcnt(N)` inside loops of each kernel in the compiled .s (tools/isa_hist.sh
writes /tmp/isa/capi-hip-amdgcn-amd-amdhsa-gfx950.s): a vmcnt wait in a loop body that guards
an MFMA operand loaded before the loop drains the loop's own prefetch on every trip."""
import re
import subprocess
import sys

s = open('/tmp/isa/capi-hip-amdgcn-amd-amdhsa-gfx950.s').read()
pat = sys.argv[1] if len(sys.argv) > 1 else ''
for name in re.findall(r'^(_Z\S+):', s, re.M):
    if pat not in name:
        continue
    i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
    lines = s[i:j].split('\n')
    labels = {}
    for n, l in enumerate(lines):
        m = re.match(r'^(\.LBB\S+):', l.strip())
        if m:
            labels[m.group(1)] = n
    loops = []
    for n, l in enumerate(lines):
        m = re.search(r's_(?:c?branch\S*)\s+(\.LBB\S+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < n:
            loops.append((labels[m.group(1)], n))
    hits = []
    for a, b in loops:
        for n in range(a, b):
            if 'vmcnt' in lines[n]:
                nxt = next((lines[k].strip() for k in range(n + 1, min(b, n + 4)) if lines[k].strip()), '')
                hits.append(f'    {lines[n].strip():40s} -> {nxt}')
    dn = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
    print(f'{dn[:90]}  loops={len(loops)} vmcnt-in-loop={len(hits)}')
    for h in hits[:12]:
        print(h)
