#!/usr/bin/env python3
"""How the C2 pipeline's kernels pack on the GPU, from a rocprofv3 kernel trace.

  python tools/c2_timeline.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv

Takes the launches of the C2 kernels at the bench grid (the largest grid seen per kernel),
keeps the last `--steps` batches (the timed region of tools/profile.sh) and prints, over
that span: the time each kernel type is running (union of its launches), the time two
types overlap, and the time no C2 kernel runs at all.  Two batches in flight on two
streams should leave the moments pass (HBM-bound) under the compute kernels of the other
batch; this shows how much of it does.
"""
import argparse
import collections
import csv


def short(name):
    return name.split('(')[0].split('<')[0].replace('void ', '').replace('aec::', '').replace('_kernel', '')


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    keep = ('moments', 'moments_lds', 'norm_finalize', 'nlms_analysis', 'gru_synth')
    by = collections.defaultdict(list)
    for r in rows:
        k = short(r['Kernel_Name'])
        if k in keep:
            by[k].append((int(r['Grid_Size_X']), int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    ana = by['nlms_analysis']
    gmax = max(g for g, _, _ in ana)
    ana = sorted(x for x in ana if x[0] == gmax)[-a.steps:]
    t0 = ana[0][1]
    gru = sorted(x for x in by['gru_synth'] if x[0] == max(g for g, _, _ in by['gru_synth']))
    t1 = max(e for _, s, e in gru if s >= t0)
    iv = {}
    for k, v in by.items():
        g = max(x[0] for x in v)
        iv[k] = [(max(s, t0), min(e, t1)) for gg, s, e in v if gg == g and e > t0 and s < t1]
    span = t1 - t0
    print(f'span {span / 1e6:.3f} ms over {len(ana)} analysis launches: {span / 1e6 / len(ana):.4f} ms per batch')
    for k, v in iv.items():
        u = union(v)
        print(f'  {k:14s} launches {len(v):3d}  busy {u / 1e6:7.3f} ms ({u / span:5.1%})  '
              f'mean launch {sum(e - s for s, e in v) / max(1, len(v)) / 1e3:7.1f} us')
    # pairwise overlap and idle time via an event sweep
    ev = []
    for k, v in iv.items():
        for s, e in v:
            ev.append((s, 1, k))
            ev.append((e, -1, k))
    ev.sort(key=lambda x: (x[0], x[1]))
    act = collections.Counter()
    last = t0
    state_time = collections.Counter()
    for t, d, k in ev:
        if t > last:
            state_time[tuple(sorted(x for x in act if act[x] > 0))] += t - last
            last = t
        act[k] += d
    if t1 > last:
        state_time[tuple(sorted(x for x in act if act[x] > 0))] += t1 - last
    print('time by set of running kernel types:')
    for st, t in sorted(state_time.items(), key=lambda x: -x[1]):
        print(f'  {" + ".join(st) or "(none)":50s} {t / 1e6:7.3f} ms ({t / span:5.1%})')


if __name__ == '__main__':
    main()
