#!/usr/bin/env python3
"""profiles/pmc_latest_c5.json from a tools/crn_pmc_summary.py JSON of the
tools/c5_pmc.sh passes (tools/c5_prof.py: 256 streams, 10 warm-up + HOPS
timed hops).  bench.py reads `hbm_bytes_per_hop` as the c5_stream_fp8
roofline's `traffic`: the HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, gfx950
correction) of every kernel the hop launches, per hop.

usage: c5_pmc_latest.py <summary.json> <source tag>"""
import json
import sys

summ = json.load(open(sys.argv[1]))
tag = sys.argv[2]
# the 256-stream hops: the front kernel at the largest grid (c5_prof.py also runs a 1-stream
# latency probe, whose hops are more numerous); that configuration's kernels launch once or twice
# per hop
grid = lambda k: int(k.rsplit('grid', 1)[1]) if 'grid' in k else 0
fk = max((k for k in summ if 'stream_front' in k or 'stream_enc' in k), key=grid)
hops = summ[fk]['launches']
per_hop = {k: v for k, v in summ.items()
           if v['launches'] in (hops, 2 * hops) and grid(k) >= grid(fk) // 2
           and not k.startswith(('__amd_rocclr', 'at::native'))}
total = sum(v['hbm_bytes_per_launch'] * v['launches'] for v in per_hop.values()) / hops
out = dict(pipeline='c5_stream', dtype='fp8', B=256, hops_counted=hops,
           source=f'rocprofv3 --pmc passes (tools/c5_pmc.sh {tag}) over tools/c5_prof.py',
           formula='hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE = half of streamed bytes)',
           hbm_bytes_per_hop=int(total), hop_kernels=per_hop)
json.dump(out, open('profiles/pmc_latest_c5.json', 'w'), indent=1)
print('C5 HBM bytes per hop', out['hbm_bytes_per_hop'], 'from', len(per_hop), 'kernels over', hops, 'hops')
