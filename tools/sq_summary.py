#!/usr/bin/env python3
"""Per-kernel averages of tools/sq_pmc.sh counters (per launch) and derived
ratios: VALU busy = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES-share, instructions
per wave, LDS conflict share."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f'{d}/pmc_*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'].split('(')[0].replace('void ', '')[:70]
        tot[name][r['Counter_Name']] += float(r['Counter_Value'])
        disp[(name, r['Counter_Name'])].add(r['Dispatch_Id'])
out = {}
for name, c in tot.items():
    avg = {k: v / max(len(disp[(name, k)]), 1) for k, v in c.items()}
    der = {}
    if avg.get('SQ_WAVE_CYCLES'):
        w = avg['SQ_WAVE_CYCLES']
        for k in ('SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_LDS', 'SQ_WAIT_INST_ANY', 'SQ_WAIT_ANY',
                  'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_SCA', 'SQ_WAIT_INST_LDS'):
            if k in avg:
                der[k + '/wave_cycles'] = round(avg[k] / w, 4)
    if avg.get('SQ_LDS_IDX_ACTIVE'):
        der['lds_bank_conflict_share'] = round(avg.get('SQ_LDS_BANK_CONFLICT', 0) / avg['SQ_LDS_IDX_ACTIVE'], 4)
    if avg.get('SQ_WAVES'):
        for k in ('SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_INSTS_SALU', 'SQ_INSTS_VMEM'):
            if k in avg:
                der[k + '/wave'] = round(avg[k] / avg['SQ_WAVES'], 1)
    out[name] = dict(avg={k: int(v) for k, v in avg.items()}, derived=der)
print(json.dumps(out, indent=1))
