#!/usr/bin/env python3
"""Static instruction mix of the gfx950 kernels of one source file (VALU / LDS /
SALU / VMEM per kernel, VGPR count, spills), a proxy for issue cost when
comparing variants of the same kernel:
  python tools/isa_count.py <file.hip> [kernel-substring ...] [-D...]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, 'acoustic-echo-cancellation_amd', 'csrc')
args = sys.argv[1:]
defs = [a for a in args if a.startswith('-D')]
rest = [a for a in args if not a.startswith('-D')]
src = rest[0] if os.path.isabs(rest[0]) else os.path.join(CSRC, rest[0])
pats = rest[1:]
with tempfile.TemporaryDirectory() as d:
    out = os.path.join(d, 'k.s')
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fno-slp-vectorize',
                    '--cuda-device-only', '-S', f'-I{CSRC}', os.path.join(REPO, 'include') and f'-I{os.path.join(REPO, "include")}',
                    *defs, src, '-o', out], check=True, capture_output=True)
    lines = open(out).read().split('\n')
res = collections.OrderedDict()
meta = {}
ents = []
cur = None
for l in lines:
    m = re.match(r'^(_Z\w+):', l)
    if m:
        cur = m.group(1)
        res[cur] = collections.Counter()
        continue
    if l.strip().startswith('.Lfunc_end'):
        cur = None
        continue
    if re.match(r'\s+- \.', l):                      # a new kernel entry of the amdhsa metadata
        ent = {}
        ents.append(ent)
    m = re.match(r'\s+-?\s*\.(name|vgpr_count|vgpr_spill_count|sgpr_count):\s+(\S+)', l)
    if m and ents:
        ents[-1][m.group(1)] = m.group(2)
    if cur:
        t = l.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':'):
            continue
        op = t.split()[0]
        if op.startswith('v_'):
            c = 'valu'
        elif op.startswith('ds_'):
            c = 'lds'
        elif op.startswith(('buffer_', 'global_', 'flat_')):
            c = 'vmem'
        elif op.startswith(('s_waitcnt', 's_nop', 's_barrier')):
            c = 'wait'
        elif op.startswith('s_'):
            c = 'salu'
        else:
            c = 'other'
        res[cur][c] += 1
for e in ents:
    if 'name' in e:
        meta[e['name']] = e
for k, c in res.items():
    if pats and not any(p in k for p in pats):
        continue
    mt = meta.get(k, {})
    print(f'{k[:70]:70s} valu {c["valu"]:5d} lds {c["lds"]:4d} vmem {c["vmem"]:4d} salu {c["salu"]:4d} '
          f'vgpr {mt.get("vgpr_count", "?")} spill {mt.get("vgpr_spill_count", "?")}')
