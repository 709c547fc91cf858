#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/ (build host).

  python tools/summarize_profile.py gpurun_out/prof_r01 r01

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats table (verbatim)
  profiles/<tag>_bench_trace.json   the bench line printed under the tracer
  profiles/<tag>_hbm.csv            per kernel: FETCH_SIZE, WRITE_SIZE (KiB) and
                                    HBM bytes per launch
  profiles/pmc_latest_<pipeline>.json   read by bench.py for roofline.traffic

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950
FETCH_SIZE counts half the bytes of wide coalesced streaming reads and
WRITE_SIZE is exact for 16-B-per-lane stores (MI355X_MICROARCH.md, HBM
section); both counters are in KiB.  Only the launches at the bench's own grid
(the largest grid seen per kernel) are averaged.
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    return name.split('(')[0].split('<')[0].replace('void ', '').replace('aec::', '').replace('_kernel', '')


def main():
    src, tag = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dst = os.path.join(repo, 'profiles')
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'), os.path.join(dst, f'{tag}_kernel_stats.csv'))
    log = open(os.path.join(src, 'trace_bench.log')).read().splitlines()
    js = [l for l in log if l.startswith('{')]
    pipeline = None
    if js:
        open(os.path.join(dst, f'{tag}_bench_trace.json'), 'w').write(js[-1] + '\n')
        pipeline = json.loads(js[-1])['config'].get('pipeline')
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, 'run_counter_collection.csv')
        if not d.startswith('pmc_') or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = short(r['Kernel_Name'])
            if 'rocclr' in k:
                continue
            vals[k][(int(r['Grid_Size']), r['Counter_Name'])].append(float(r['Counter_Value']))
    out = {'pipeline': pipeline, 'source': f'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tools/profile.sh ({tag})',
           'formula': 'hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE = half of streamed bytes)',
           'kernels': {}}
    rows = []
    for k, d in sorted(vals.items()):
        grid = max(g for g, _ in d)
        fe = d.get((grid, 'FETCH_SIZE'), [])
        wr = d.get((grid, 'WRITE_SIZE'), [])
        if not fe or not wr:
            continue
        f_kib = sum(fe) / len(fe)
        w_kib = sum(wr) / len(wr)
        hbm = 2 * f_kib * 1024 + w_kib * 1024
        out['kernels'][k] = dict(grid=grid, fetch_kib=round(f_kib, 1), write_kib=round(w_kib, 1),
                                 hbm_bytes_per_launch=int(hbm), launches=len(fe))
        rows.append([k, grid, round(f_kib, 1), round(w_kib, 1), int(hbm)])
    with open(os.path.join(dst, f'{tag}_hbm.csv'), 'w', newline='') as fh:
        w = csv.writer(fh)
        w.writerow(['kernel', 'grid', 'FETCH_SIZE_KiB', 'WRITE_SIZE_KiB', 'hbm_bytes_per_launch'])
        w.writerows(rows)
    json.dump(out, open(os.path.join(dst, f'pmc_latest_{pipeline}.json'), 'w'), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
