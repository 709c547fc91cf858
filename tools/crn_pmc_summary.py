#!/usr/bin/env python3
"""Summarise tools/crn_pmc.sh: per kernel (largest grid) MFMA utilisation and
HBM bytes per launch.  MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs); HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB x
1024, gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]


def load(i):
    f = glob.glob(f'{d}/pmc_{i}/**/*counter_collection.csv', recursive=True)
    rows = list(csv.DictReader(open(f[0]))) if f else []
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in rows:
        name = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('crn::', '')[:60]
        key = (name, r.get('Grid_Size', r.get('Grid_Size_X', '')))
        agg[key][r['Counter_Name']] += float(r['Counter_Value'])
        cnt[key].add(r['Dispatch_Id'])
    return agg, cnt


m, mc = load(1)
f, fc = load(2)
w, wc = load(3)
out = {}
for key in m:
    n = len(mc[key])
    busy = m[key].get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / n
    grbm = m[key].get('GRBM_GUI_ACTIVE', 0) / n
    util = busy / (1024 * grbm / 8) if grbm else None
    fk = f.get(key, {}).get('FETCH_SIZE', 0) / max(len(fc.get(key, [])), 1)
    wk = w.get(key, {}).get('WRITE_SIZE', 0) / max(len(wc.get(key, [])), 1)
    out[f'{key[0]} grid {key[1]}'] = dict(launches=n, mfma_util=round(util, 4) if util is not None else None,
                                          hbm_bytes_per_launch=int(2 * fk * 1024 + wk * 1024))
for k, v in sorted(out.items(), key=lambda kv: -(kv[1]['mfma_util'] or 0)):
    print(f'{k:90s} {v}')
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], 'w'), indent=1)
