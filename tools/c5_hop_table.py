#!/usr/bin/env python3
"""Per-launch table of one C5 hop (median over hops) from rocprofv3 kernel traces:
python tools/c5_hop_table.py gpurun_out/c5pab_1 gpurun_out/c5pab_2 ..."""
import csv
import os
import statistics
import sys


def hops(d):
    rows = list(csv.DictReader(open(os.path.join(d, 'trace', 'run_kernel_trace.csv'))))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    # the hops at the largest stream count (tools/c5_prof.py also steps a 1-stream latency probe)
    front = [r for r in rows if 'stream_front' in r['Kernel_Name'] or 'stream_enc' in r['Kernel_Name']]
    gmax = max(int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) for r in front)
    idx = [i for i, r in enumerate(rows) if ('stream_front' in r['Kernel_Name'] or 'stream_enc' in r['Kernel_Name'])
           and int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) == gmax]
    out = []
    for a, b in zip(idx[5:-1], idx[6:]):
        seq = rows[a:b]
        out.append([(r['Kernel_Name'].split('(')[0].replace('void crn::', '')[:60],
                     int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) // int(r['Workgroup_Size_X']),
                     (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in seq
                    if 'rocclr' not in r['Kernel_Name']])
        out[-1].append(('hop', 0, (int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3))
    return out


cols = [hops(d) for d in sys.argv[1:]]
names = [open(os.path.join(d, 'cfg.txt')).read().strip() if os.path.exists(os.path.join(d, 'cfg.txt')) else d
         for d in sys.argv[1:]]
print(' ' * 72 + ''.join(f'{n[-14:]:>15}' for n in names))
base = cols[0]
n = min(len(h) for h in base)
for k in range(len(base[0])):
    name, blocks, _ = base[0][k]
    vals = []
    for c in cols:
        v = [h[k][2] for h in c if len(h) > k]
        vals.append(statistics.median(v))
    print(f'{name:60s} {blocks:8d}  ' + ''.join(f'{v:15.2f}' for v in vals))
