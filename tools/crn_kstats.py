#!/usr/bin/env python3
"""Per-kernel summary of a tools/crn_prof.sh trace (grouped by kernel and grid)."""
import collections
import csv
import sys

d = sys.argv[1]
r = list(csv.DictReader(open(f'{d}/trace/run_kernel_trace.csv')))
agg = collections.defaultdict(lambda: [0, 0.0])
for x in r:
    n = x['Kernel_Name'].split('(')[0].replace('void ', '').replace('crn::', '')[:70]
    key = (n, x['Grid_Size_X'], x['Grid_Size_Y'])
    agg[key][0] += 1
    agg[key][1] += (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3
tot = sum(v[1] for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f'{k[0]:70s} grid {k[1]:>10s}x{k[2]:<4s} n={v[0]:5d} avg {v[1]/v[0]:9.1f} us  tot {v[1]/1e3:8.2f} ms  {100*v[1]/tot:5.1f}%')
