#!/usr/bin/env python3
"""Benchmark of the Stage-2 AEC hot path on MI355X (one process per GPU).

Metric (BASELINE.json): 16 kHz frames/s (one frame = one 256-sample hop), batched
AEC, plus RTF at batch 1.  Workload at N=1 = BASELINE config C2's shape: 256
concurrent 10 s streams (N = 160,000 samples, T = 626 frames each) through the
whole per-frame loop STFT -> ERB-GRU post-filter -> iSTFT, synthetic seeded
scenes (aec_amd.synth), seed-0 reference weights, inputs resident in HBM.
N>1 (torchrun): every rank runs its own 256 streams (weak scaling, no data-path
collective); timing = max over ranks.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))

HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector (= f32 MFMA) peak
KERNELS = ['moments', 'analysis', 'gru', 'synthesis']
# Algorithmic work per frame: bytes that must cross HBM and
# FLOPs of the FFT-based algorithm, for B streams with near (loss) enabled.
RFFT = 11520                   # 2.5 N log2 N, N = 512
ANA_SIG = RFFT + 512 + 3 * 257 + 2 * 483          # window, rFFT, |X|, sparse ERB
NLMS_FLOPS = 257 * (16 * 4 + 10)                  # SURVEY.md §8(d), 4 taps
SYN_TAIL = RFFT + 512 + 2 * 483 + 6 * 257 + 3 * 256   # gains, irFFT, window, WOLA
GRU = dict(bytes=3 * 32 * 4 + 32 * 4, flops=2 * 96 * 64 + 2 * 96 * 32 + 2 * (32 * 64 + 32 * 32) + 400)
ALG = {
    'postfilter': {
        'moments': dict(bytes=3 * 256 * 4, flops=3 * 256 * 4),
        'analysis': dict(bytes=3 * 256 * 4 + 3 * 32 * 4, flops=3 * ANA_SIG),
        'gru': GRU,
        'synthesis': dict(bytes=256 * 4 + 32 * 4 + 256 * 4, flops=RFFT + 512 + SYN_TAIL),
    },
    'full': {
        'moments': dict(bytes=3 * 256 * 4, flops=3 * 256 * 4),
        # + the error spectrum E written for K4 (2 KiB) and |E| -> ERB
        'analysis': dict(bytes=3 * 256 * 4 + 3 * 32 * 4 + 256 * 8, flops=3 * ANA_SIG + NLMS_FLOPS + 3 * 257 + 2 * 483),
        'gru': GRU,
        # E (2 KiB) instead of the mic samples; no forward transform
        'synthesis': dict(bytes=256 * 8 + 32 * 4 + 256 * 4, flops=SYN_TAIL),
    },
}
WORKLOAD = {
    'full': 'C2 (BASELINE configs[1]) shape: 256 concurrent 10 s 16 kHz streams per GPU through '
            'STFT -> FD-NLMS (4 taps/bin) -> ERB-GRU post-filter -> iSTFT',
    'postfilter': 'C2 shape: 256 concurrent 10 s 16 kHz streams per GPU, STFT -> ERB-GRU post-filter '
                  '-> iSTFT (reference Little_net path, FD-NLMS bypass)',
}
# the NLMS path runs K3 + K4 as one kernel (aec_gru_synth.hip) unless AEC_FUSED_SYNTH=0
ALG['full']['gru_synthesis'] = {k: GRU[k] + ALG['full']['synthesis'][k] for k in ('bytes', 'flops')}
PIPE = dict(bytes=4096, flops=82000)      # whole path, per frame
SURVEY_NLMS_FLOPS = 257 * (16 * 4 + 10)    # FD-NLMS adds 257 (16 L + 10) FLOP/frame, L = 4 taps


def path_flops(pipeline):
    """SURVEY.md §8(d) algorithmic FLOP per frame of the whole path."""
    return PIPE['flops'] + (SURVEY_NLMS_FLOPS if pipeline == 'full' else 0)


# The driver contract: `value` is the whole job's throughput (all ranks' frames / the
# max-over-ranks time), from which the driver computes the scaling efficiency itself;
# BASELINE's metric is per GPU, which is `value_per_gpu` (= value / n_gpus).
MIN_WARM_STEPS = 40   # C2 warm-up floor (untimed), see run(): the clock ramp of the first ~20 ms of load
WARM_MS = 30.0        # time-based untimed warm-up floor for the short C5 / training timed regions
VALUE_SEMANTICS = ('value = aggregate frames/s of all ranks (frames of every rank / max-over-ranks time); '
                   'value_per_gpu = value / n_gpus (the metric\'s per-GPU figure)')


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100,
                    help='timed steps (C2: 100 x ~0.54 ms; the fill and drain of three batches in flight are ~1.5 ms, '
                         '~15 %% of a 20-step region, profiles/r05z_steps_ab.log)')
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--streams', type=int, default=256)
    ap.add_argument('--seconds', type=float, default=10.0)
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='bounded CPU-baseline sample (wall s)')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--pipeline', choices=['full', 'postfilter', 'crn'], default='full',
                    help='full = STFT -> FD-NLMS -> ERB-GRU post-filter -> iSTFT (north_star); '
                         'postfilter = the reference Little_net path alone (NLMS bypass); '
                         'crn = BASELINE config 3: the DCCRN (dccrn2.py, configs.net_conf) post-filter')
    ap.add_argument('--crn-dtype', choices=['bf16', 'f32', 'fp8'], default='bf16',
                    help='--pipeline crn compute type (fp8 = bf16 with MX-fp8 LSTM input projections and wide conv layers)')
    ap.add_argument('--crn-version', type=int, choices=[1, 2], default=2, help='1 = dccrn.py, 2 = dccrn2.py')
    ap.add_argument('--crn-nlms', action='store_true',
                    help='--pipeline crn: feed the DCCRN the FD-NLMS error spectrum (C5, include/aec_crn.h)')
    ap.add_argument('--no-rtf', action='store_true', help='skip the batch-1 latency probe (profiling runs)')
    ap.add_argument('--no-sweep', action='store_true',
                    help='skip the batch sweep (B = 1 ... 4096 streams, 3 calls each, after the timed region)')
    ap.add_argument('--lookahead', type=int, default=1,
                    help='C2: step k queues the normaliser pass of batch k + LOOKAHEAD on a side stream (aec_prepare); '
                         '0 = off')
    ap.add_argument('--lookahead-cus', type=int, default=0,
                    help='C2: the look-ahead side stream runs on this many CUs only (hipExtStreamCreateWithCUMask; '
                         'every (256 / N)-th CU), so the HBM-bound pass holds few CUs; 0 = all CUs')
    ap.add_argument('--inflight', type=int, default=3,
                    help='C2 batches in flight (HIP streams, one handle each; 1 = strictly sequential; 3 measured '
                         '1-2 %% faster than 2, profiles/r05_notes.md r05t)')
    ap.add_argument('--crn-inflight', type=int, default=2,
                    help='CRN (C3 / C4 / --pipeline crn) batches in flight')
    ap.add_argument('--no-c3', action='store_true', help='skip the BASELINE config 3 (DCCRN bf16) figure')
    ap.add_argument('--c3-steps', type=int, default=10, help='timed steps of the config 3 figure')
    ap.add_argument('--no-train', action='store_true', help='skip the training-step figure')
    ap.add_argument('--no-near-leg', action='store_true',
                    help='skip the near=None (no loss) timed leg reported beside the headline')
    ap.add_argument('--train-steps', type=int, default=10, help='timed steps of the training-step figure')
    return ap.parse_args()


# knobs that only an A/B build reads (csrc/aec_knobs.h AEC_AB_KNOB): timing experiments and
# work-skipping switches.  The product library ignores them; a bench line is refused when one is
# set, so that no driver line can be read as having run a timing-only mode.
AB_ONLY_KNOBS = ('AEC_MOM_CFG', 'AEC_MOM_GRID', 'AEC_GRU_MODE', 'AEC_GRU_WMAP', 'AEC_NLMS_PRIO', 'AEC_NLMS_ERB', 'AEC_FUSED_MODE',
                 'AEC_CRN_ENC_FR', 'AEC_CRN_SPLITK', 'CRN_PERSIST_RA', 'AEC_CRN_ENC_MX_RERUN', 'CRN_DEC_FUSE',
                 'CRN_GEMM_XCD', 'CRN_GEMM_DMA', 'CRN_GEMM_BIG', 'CRN_GEMM_SQ', 'CRN_GEMM_RB64', 'CRN_GEMM_MODE',
                 'CRN_GEMM_PIPE', 'CRN_STEP_MODE', 'CRN_STEP_CFG', 'CRN_MX_STEP_MODE', 'AEC_CRN_PERSIST_WAVES')
# test hooks (fault injection) of the product library: never in a bench run
TEST_ONLY_KNOBS = ('AEC_CRN_PERSIST_STALL', 'AEC_CRN_SPIN_LIMIT', 'AEC_SMALLB_PIPE_STALL')


def knob_provenance():
    """Every AEC_* / CRN_* environment variable set, and the library's build
    description (aec_build_info); raises when a timing-only / test-only knob
    is set or the loaded library is an A/B build."""
    from aec_amd import _lib
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith(('AEC_', 'CRN_'))}
    # AEC_BENCH_AB=1: an A/B timing run (tools/*_ab.sh) of a variant build; its line says so
    ab_run = env.get('AEC_BENCH_AB') == '1'
    bad = [k for k in env if k in AB_ONLY_KNOBS or k in TEST_ONLY_KNOBS]
    if bad and not ab_run:
        raise SystemExit(f'bench.py: timing-only / test-only knobs set {bad}: refusing to produce a bench line')
    info = _lib.build_info()
    if info['ab_knobs'] and not ab_run:
        raise SystemExit(f'bench.py: {_lib.LIB_PATH} is an A/B build ({info["text"]}): refusing')
    unknown = [k for k in env if k not in info['mode_knobs'] and k not in ('AEC_HIP_LIB', 'AEC_BENCH_BACKEND',
                                                                          'AEC_BENCH_AB')]
    return dict(env=env, library=os.path.relpath(_lib.LIB_PATH, REPO), build_info=info['text'],
                defaults=not env, ab_timing_run=ab_run, unknown_names=unknown)


def cu_masked_stream(dev, ncu):
    """A HIP stream whose kernels run on `ncu` CUs only (every (n_cu / ncu)-th), wrapped for torch."""
    import ctypes
    import torch
    total = torch.cuda.get_device_properties(dev).multi_processor_count
    step = max(1, total // ncu)
    words = [0] * ((total + 31) // 32)
    for c in range(0, total, step)[:ncu]:
        words[c // 32] |= 1 << (c % 32)
    hip = ctypes.CDLL('libamdhip64.so')
    st = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    with torch.cuda.device(dev):
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(len(words)), arr)
    if rc != 0:
        raise RuntimeError(f'hipExtStreamCreateWithCUMask failed: {rc}')
    return torch.cuda.ExternalStream(st.value, device=dev)


def roofline(pipeline, kernel, ms_per_launch, frames_per_launch, pmc):
    """Dominant kernel vs the MI355X roofline.  `achieved` = the kernel's own
    algorithmic work per frame (its share of the path, DESIGN.md §5: the
    bytes it must move and the FLOPs of the FFT-based algorithm for the part
    of the path it implements) x the frames one launch processes / the
    launch's time (HIP events); `bound` is the larger of the HBM and FP32
    fractions.  `path_priced` repeats the figure with SURVEY.md §8(d)'s
    whole-path per-frame figures (4,096 B; 82 kFLOP + the NLMS's 19 kFLOP),
    which charges the whole path to this one kernel (an upper bound)."""
    t = ms_per_launch * 1e-3
    fl = path_flops(pipeline)
    traffic = None
    kname = {'analysis': 'nlms_analysis', 'gru_synthesis': 'gru_synth'}.get(kernel, kernel) \
        if pipeline == 'full' else kernel
    if pmc and pmc.get('pipeline') == pipeline and kname in pmc.get('kernels', {}):
        traffic = pmc['kernels'][kname].get('hbm_bytes_per_launch')
    a = ALG[pipeline].get(kernel, dict(bytes=PIPE['bytes'], flops=fl))
    gbs = a['bytes'] * frames_per_launch / t / 1e9
    tfl = a['flops'] * frames_per_launch / t / 1e12
    pg = PIPE['bytes'] * frames_per_launch / t / 1e9
    pt = fl * frames_per_launch / t / 1e12
    path = dict(alg_bytes_per_frame=PIPE['bytes'], alg_flops_per_frame=fl, achieved_gbs=round(pg, 1),
                achieved_tflops=round(pt, 3), frac=round(max(pg / HBM_PEAK_GBS, pt / FP32_PEAK_TFLOPS), 4))
    common = dict(traffic=traffic, traffic_alg_bytes_per_launch=a['bytes'] * frames_per_launch, kernel=kernel,
                  frac_basis='kernel_share: this kernel\'s own algorithmic bytes / FLOPs (DESIGN.md §5); '
                             'path_priced.frac charges the whole path to it (the pre-round-4 definition)',
                  alg_bytes_per_frame=a['bytes'], alg_flops_per_frame=a['flops'],
                  frames_per_launch=frames_per_launch, ms_per_launch=round(ms_per_launch, 4),
                  hbm_frac=round(gbs / HBM_PEAK_GBS, 4), fp32_frac=round(tfl / FP32_PEAK_TFLOPS, 4),
                  path_priced=path)
    if gbs / HBM_PEAK_GBS >= tfl / FP32_PEAK_TFLOPS:
        return dict(bound='hbm', achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit='GB/s',
                    frac=round(gbs / HBM_PEAK_GBS, 4), **common)
    return dict(bound='valu_fp32', achieved=round(tfl, 3), peak=FP32_PEAK_TFLOPS, unit='TFLOP/s',
                frac=round(tfl / FP32_PEAK_TFLOPS, 4), **common)


SQ_KERNEL = {'analysis': 'nlms_analysis_kernel', 'gru_synthesis': 'gru_synth_kernel', 'moments': 'moments_lds_kernel'}


def sq_limiter(kernel, path=None):
    """What limits a C2 kernel, from the committed SQ counter pass of the same build
    (profiles/sq_latest_full.json; counters in quad-cycles).  A wave64 VALU
    instruction holds one wave for a quad-cycle and the SIMD-32 issues two per
    quad-cycle from different waves (MI355X_MICROARCH.md, cycle constants), so
    the SIMD's VALU pipe use = waves per SIMD x VALU-active per wave / 2.
    limiter: 'valu-issue' at >= 0.8 of that pipe, else 'latency' with the
    stall split (dependency / issue stalls vs s_waitcnt + barrier waits)."""
    path = path or os.path.join(REPO, 'profiles', 'sq_latest_full.json')
    name = SQ_KERNEL.get(kernel)
    if not name or not os.path.exists(path):
        return None
    d = json.load(open(path))
    row = next((v for k, v in d.get('kernels', d).items() if name in k and isinstance(v, dict) and 'derived' in v),
               None)
    if row is None:
        return None
    dv, av = row['derived'], row['avg']
    waves_per_simd = d.get('waves_per_simd', {}).get(kernel, 3)
    pipe = waves_per_simd * dv['SQ_ACTIVE_INST_VALU/wave_cycles'] / 2
    out = dict(source=os.path.relpath(path, REPO), waves_per_simd=waves_per_simd,
               valu_active_per_wave=dv['SQ_ACTIVE_INST_VALU/wave_cycles'], valu_pipe_use=round(pipe, 3),
               issue_stall_per_wave=dv['SQ_WAIT_INST_ANY/wave_cycles'], waitcnt_barrier_per_wave=dv['SQ_WAIT_ANY/wave_cycles'],
               valu_instr_per_wave=dv['SQ_INSTS_VALU/wave'])
    out['limiter'] = 'valu-issue' if pipe >= 0.8 else (
        'latency: dependency / issue stalls %.0f %%, s_waitcnt + barrier waits %.0f %% of wave cycles'
        % (100 * dv['SQ_WAIT_INST_ANY/wave_cycles'], 100 * dv['SQ_WAIT_ANY/wave_cycles']))
    return out


def cpu_baseline(seconds, B=256, n=160000):
    """The reference op mix on host cores (oracle/torch_port.py), bounded
    sample: B = 256 x 10 s streams, then a few batch-1 calls."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    from torch_port import TorchPort
    from aec_amd import synth, erb_matrix
    w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
    port = TorchPort(w, erb_matrix())
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    mic, ref, near = (torch.from_numpy(a) for a in synth.batch(B, n, seed0=5000))
    port(mic[:2, :16000], ref[:2, :16000], near[:2, :16000])      # warm-up
    frames = 0
    t0 = time.perf_counter()
    reps = 0
    while True:
        port(mic, ref, near)
        reps += 1
        frames += B * (n // 256 + 1)
        el = time.perf_counter() - t0
        if el >= seconds and reps >= 2:
            break
    lat = []
    for i in range(3):
        t1 = time.perf_counter()
        port(mic[i:i + 1], ref[i:i + 1], near[i:i + 1])
        lat.append(time.perf_counter() - t1)
    b1 = float(np.median(lat))
    return dict(value=round(frames / el, 1), unit='frames/s', cores=threads, kind='port',
                sample=f'{reps} x [{B} streams x {n} samples] through oracle/torch_port.py '
                       f'(reference op mix: conv1d DFT, nn.GRU, conv_transpose1d), {el:.1f} s wall; '
                       f'batch 1: median of 3 single 10 s streams',
                batch1_frames_per_s=round((n // 256 + 1) / b1, 1), rtf_batch1=round(b1 / (n / 16000), 6))


BF16_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
FP8_PEAK_TFLOPS = 5000.0      # MI355X_MICROARCH.md: dense FP8 (block-scaled e4m3: 2x the bf16 rate)
CRN_STAGES = ['front', 'encoder', 'lstm', 'decoder', 'back']


def crn_flops_per_frame(conf, version):
    """Algorithmic MACs x 2 of the DCCRN per 256-sample frame (dense convs as
    GEMMs, LSTMs), SURVEY.md §8(d)."""
    ch = conf['conv_channels']
    L = len(ch) - 1
    enc = sum(2 * (256 >> (i + 1)) * ch[i + 1] * 5 * ch[i] for i in range(L))
    dec = sum(2 * (256 >> c) * (2 * ch[c]) * (ch[c - 1] if c != 1 else 2) * 5 for c in range(L, 0, -1))
    if version == 1:
        H = ch[-1] * 4
        rnn = 2 * 4 * H * (H + H)
    else:
        H = conf['hidden_dim'] * ch[-1] // 2
        rnn = conf['rnn_layers'] * 4 * 2 * 4 * H * (H + H)
    return dict(encoder=enc, decoder=dec, lstm=rnn, total=enc + dec + rnn)


def cpu_baseline_crn(seconds, conf, version, n=160000, B=1, nlms=None):
    """The reference op mix (oracle/torch_crn_port.py: conv2d / conv_transpose2d /
    nn.LSTM, float32; with nlms, the FD-NLMS front end in front) on host cores,
    bounded sample."""
    import torch
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import crn_oracle
    from torch_crn_port import TorchCrnPort
    from aec_amd import synth
    port = TorchCrnPort(crn_oracle.make_weights(conf, version, 1), conf, version, nlms=nlms)
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    mic, far, _ = (torch.from_numpy(a) for a in synth.batch(B, n, seed0=7000))
    port(mic[:, :16000], far[:, :16000])             # warm-up
    frames, reps = 0, 0
    t0 = time.perf_counter()
    while True:
        port(mic, far)
        reps += 1
        frames += B * (n // 256 + 1)
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 50:
            break
    return dict(value=round(frames / el, 1), unit='frames/s', cores=threads, kind='port',
                sample=f'{reps} x [{B} stream x {n} samples] through oracle/torch_crn_port.py '
                       f'(reference op mix: conv2d / conv_transpose2d / nn.LSTM, float32'
                       f'{", FD-NLMS front end" if nlms else ""}), {el:.1f} s wall')


def erle_check(run_gpu, run_ref, n, streams=2):
    """ERLE (10 log10(sum mic^2 / sum out^2), first 0.5 s
    skipped) of the GPU path and of the CPU reference restatement on the same
    far-end single-talk scenes; delta = GPU - reference (north_star: <= 0.1 dB)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    from aec_oracle import erle_db
    from aec_amd import synth
    g, r = [], []
    for i in range(streams):
        mic, ref, near = synth.scene(n, 90000 + i, double_talk=False)
        g.append(erle_db(mic, run_gpu(mic, ref, near)))
        r.append(erle_db(mic, run_ref(mic, ref, near)))
    return dict(gpu_db=round(float(np.mean(g)), 4), reference_db=round(float(np.mean(r)), 4),
                delta_db=round(float(np.mean(g) - np.mean(r)), 5), streams=streams,
                scene='far-end single talk (near = 0), 10 s, synthetic RIR echo')


def _init_dist(torch, dist, world, local):
    """One process per GPU over RCCL (backend "nccl").  AEC_BENCH_BACKEND=gloo
    rehearses the multi-rank flow (barriers, max-over-ranks, rank-0 line) with
    several ranks sharing the GPUs of a smaller box; never used for numbers."""
    if world > 1:
        backend = os.environ.get('AEC_BENCH_BACKEND', 'nccl')
        if backend == 'gloo':
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == 'gloo':
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    return local


def run_crn(args, dev, rank, world, dtype, steps, warmup, B, n, with_cpu, nlms=None, with_erle=None):
    """BASELINE config 3: the DCCRN post-filter (dccrn2.py, configs.net_conf) on
    B streams x n samples; returns the measurements (timing = max over ranks).
    nlms: the FD-NLMS front end (C5: NLMS -> CRN, include/aec_crn.h), timed
    in the 'front' stage."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import aec_amd
    from aec_amd import shard, synth
    if with_erle is None:
        with_erle = with_cpu
    conf = dict(aec_amd.net_conf)
    T = n // 256 + 1
    torch.manual_seed(0)                         # the reference's own init (random weights, no checkpoint ships)
    mod = aec_amd.dccrn if args.crn_version == 1 else aec_amd.dccrn2
    net = mod.DCCRN(conf, dtype=dtype, nlms=nlms).eval().to(dev)
    mic, far, _ = (torch.from_numpy(a).to(dev) for a in synth.batch(B, n, seed0=1000 * rank))
    lens = [n] * B

    inflight = max(1, args.crn_inflight)
    nets = [net]
    for _ in range(inflight - 1):
        extra = mod.DCCRN(conf, dtype=dtype, nlms=nlms).eval()
        extra.load_state_dict(net.state_dict())
        nets.append(extra.to(dev))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(inflight - 1)]
    kstep = [0]

    def step():
        k = kstep[0] % inflight
        kstep[0] += 1
        with torch.cuda.stream(streams[k]):
            return nets[k].forward_ragged(mic, far, lens, want_spec=False)

    with torch.no_grad():
        for _ in range(max(warmup, inflight)):
            step()
        torch.cuda.synchronize(dev)
        # stage times: HIP events over a sequential pass (one batch in flight)
        h = net._handle(dev)
        prof_steps = max(1, min(steps, 5))
        h.profile_enable(True)
        h.profile_read()
        for _ in range(prof_steps):
            net.forward_ragged(mic, far, lens, want_spec=False)
        torch.cuda.synchronize(dev)
        sms, calls = h.profile_read()
        h.profile_enable(False)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        el = shard.max_over_ranks(el)
        lat = []
        for _ in range(0 if args.no_rtf else 3):
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            net.forward_ragged(mic[:1], far[:1], [n], want_spec=False)
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - t1)
        rtf1 = float(np.median(lat)) / (n / 16000) if lat else None
    value = world * B * T * steps / el
    ms_step = el / steps * 1e3
    stage_ms = {k: sms[i] / max(calls, 1) for i, k in enumerate(CRN_STAGES)}
    fl = crn_flops_per_frame(conf, args.crn_version)
    # fp8 runs only the LSTM input projections on the scaled fp8 MFMA; everything else is bf16,
    # so it is priced against the bf16 peak (conservative for the input-GEMM half of the LSTM stage)
    peak = FP32_PEAK_TFLOPS if dtype == 'f32' else BF16_PEAK_TFLOPS
    dom = max(stage_ms, key=stage_ms.get)
    dom_fl = fl.get(dom, 0)
    ach = dom_fl * B * T / (stage_ms[dom] * 1e-3) / 1e12 if dom_fl else 0.0
    dom_peak, peak_note = peak, None
    if dtype == 'fp8' and dom == 'lstm':
        # the fp8 LSTM stage: the input projections (half the stage's FLOPs: W_ih x) run on the scaled
        # MX-fp8 MFMA (dense fp8 peak), the batch recurrence (W_hh h, the other half) stays bf16
        t_pk = (dom_fl / 2) / FP8_PEAK_TFLOPS + (dom_fl / 2) / BF16_PEAK_TFLOPS
        dom_peak = round(dom_fl / t_pk, 1)
        peak_note = ('blended: input-projection half (MX-fp8) at %.0f TF/s, recurrence half (bf16) at %.0f TF/s'
                     % (FP8_PEAK_TFLOPS, BF16_PEAK_TFLOPS))
    whole = fl['total'] * B * T / (ms_step * 1e-3) / 1e12
    # HBM bytes of the LSTM stage per batch from the committed PMC passes
    # (profiles/pmc_latest_crn.json, tools/crn_pmc.sh + tools/crn_pmc_latest.py), same shape and dtype only
    traffic = None
    pp = os.path.join(REPO, 'profiles', 'pmc_latest_crn.json')
    if dom == 'lstm' and not nlms and os.path.exists(pp):
        pj = json.load(open(pp))
        if pj.get('dtype') == dtype and pj.get('B') == B and pj.get('N') == n:
            traffic = pj.get('lstm_stage_hbm_bytes_per_batch')
    res = dict(value=round(value, 1), value_per_gpu=round(value / world, 1), ms_per_step=round(ms_step, 3),
               batches_in_flight=inflight,
               rtf_batch1=rtf1, stage_ms_per_step={k: round(v, 3) for k, v in stage_ms.items()},
               roofline={'bound': 'mfma', 'achieved': round(ach, 1), 'peak': dom_peak, 'unit': 'TFLOP/s',
                         'frac': round(ach / dom_peak, 4), 'traffic': traffic, 'peak_note': peak_note,
                         'kernel': f'{dom} stage ({"input GEMM + per-frame recurrence steps + combine per layer" if dom == "lstm" else "GEMM launches"})',
                         'alg_flops_per_frame': dom_fl, 'frames_per_launch': B * T},
               pipeline_roofline={'alg_flops_per_frame': fl['total'], 'achieved_tflops': round(whole, 1),
                                  'mfma_frac': round(whole / peak, 4)},
               erle=None, cpu_baseline=None)
    if with_erle and rank == 0 and world == 1:
        if with_cpu:
            res['cpu_baseline'] = cpu_baseline_crn(args.cpu_seconds, conf, args.crn_version, n=n, nlms=nlms)
        sys.path.insert(0, os.path.join(REPO, 'oracle'))
        from torch_crn_port import TorchCrnPort
        wref = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
        port = TorchCrnPort(wref, conf, args.crn_version, nlms=nlms)

        def gpu1(m_, f_, _n):
            with torch.no_grad():
                o, _, _ = net.forward_ragged(torch.from_numpy(m_)[None].to(dev), torch.from_numpy(f_)[None].to(dev),
                                             [len(m_)], want_spec=False)
            return o[0].cpu().numpy()

        res['erle'] = erle_check(gpu1, lambda m_, f_, _n: port(torch.from_numpy(m_)[None],
                                                               torch.from_numpy(f_)[None])[0].numpy(), n)
        res['erle']['reference'] = ('oracle/torch_crn_port.py TorchCrnPort (the reference op mix, f32' +
                                    (', with the same FD-NLMS front end' if nlms else '') + ')')
    del net, nets
    torch.cuda.empty_cache()
    return res




def c5_flop_split(conf):
    """Algorithmic FLOP per frame of the per-hop DCCRN v2 step
    split by the MFMA type the fp8 step runs them on: MX-fp8 = the LSTM layers
    (W_ih and W_hh, lstm_step_mx8_kernel), encoder layers 4-5 and decoder
    levels 4-6 (conv_mx8 / the fused-parity MX levels, crn_api.hip); bf16 =
    the narrow conv layers.  Fixed to configs.net_conf's layout."""
    ch = conf['conv_channels']
    fl = crn_flops_per_frame(conf, 2)
    enc = lambda i: 2 * (256 >> (i + 1)) * ch[i + 1] * 5 * ch[i]
    dec = lambda c: 2 * (256 >> c) * (2 * ch[c]) * (ch[c - 1] if c != 1 else 2) * 5
    fp8 = fl['lstm'] + enc(4) + enc(5) + dec(4) + dec(5) + dec(6)
    return dict(total=fl['total'], fp8=fp8, bf16=fl['total'] - fp8)


def c5_roofline(conf, B, ms_per_hop, pmc):
    """The whole hop (the step's 7 kernel launches) against the
    MFMA roofline: time at peak = the MX-fp8 FLOPs at the dense fp8 peak + the
    bf16 FLOPs at the dense bf16 peak; frac = that time / the measured hop."""
    sp = c5_flop_split(conf)
    t = ms_per_hop * 1e-3
    t_peak = B * (sp['fp8'] / (FP8_PEAK_TFLOPS * 1e12) + sp['bf16'] / (BF16_PEAK_TFLOPS * 1e12))
    ach = sp['total'] * B / t / 1e12
    blended = sp['total'] * B / t_peak / 1e12
    traffic = None
    if pmc and pmc.get('B') == B:
        traffic = pmc.get('hbm_bytes_per_hop')
    return dict(bound='mfma', achieved=round(ach, 1), peak=round(blended, 1), unit='TFLOP/s',
                frac=round(t_peak / t, 4), traffic=traffic,
                kernel='the per-hop step (7 launches: front, NLMS, encoder GEMMs, 2 MX LSTM layer '
                       'steps, decoder GEMMs, back)',
                alg_flops_per_frame=sp['total'], fp8_flops_per_frame=sp['fp8'], bf16_flops_per_frame=sp['bf16'],
                frames_per_launch=B,
                peak_note='blended: MX-fp8 share at %.0f TF/s, bf16 share at %.0f TF/s' % (FP8_PEAK_TFLOPS,
                                                                                          BF16_PEAK_TFLOPS),
                frac_vs_bf16_peak=round(ach / BF16_PEAK_TFLOPS, 4), frac_vs_fp8_peak=round(ach / FP8_PEAK_TFLOPS, 4),
                traffic_source='profiles/pmc_latest_c5.json (FETCH_SIZE / WRITE_SIZE passes of tools/c5_step.py, '
                               '2 FETCH + WRITE KiB per the gfx950 correction)' if traffic else None)


def cpu_baseline_c5(seconds, net, conf, nlms, B=256):
    """The per-hop step with the reference op mix on host cores
    (oracle/torch_crn_port.py TorchCrnStreamPort: one 256-sample hop per
    stream per call, LSTM / NLMS / overlap-add state carried), bounded sample."""
    import torch
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    from torch_crn_port import TorchCrnStreamPort
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    w = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    port = TorchCrnStreamPort(w, conf, 2, nlms=nlms)
    port.stream_open(B)
    g = torch.Generator().manual_seed(5)
    mic = 0.1 * torch.randn(B, 256, generator=g)
    far = 0.1 * torch.randn(B, 256, generator=g)
    port.step(mic, far)
    hops, t0 = 0, time.perf_counter()
    while True:
        port.step(mic, far)
        hops += 1
        el = time.perf_counter() - t0
        if el >= seconds or hops >= 2000:
            break
    return dict(value=round(B * hops / el, 1), unit='frames/s', cores=threads, kind='port',
                ms_per_hop=round(el / hops * 1e3, 3),
                sample=f'{hops} hops x {B} streams through oracle/torch_crn_port.py TorchCrnStreamPort '
                       f'(reference op mix: conv1d DFT frame, conv2d / conv_transpose2d, nn.LSTM with carried '
                       f'state, FD-NLMS per bin, float32), {el:.1f} s wall')


def c5_erle(net, dev, conf, nlms, streams=2, n=160000):
    """ERLE of the per-hop step (10 s far-end single-talk scenes stepped one hop
    per call, step k emitting hop k-1) against the reference op mix on the
    same signals (oracle/torch_crn_port.py TorchCrnPort with the same FD-NLMS
    front end, f32 CPU)."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    from aec_oracle import erle_db
    from torch_crn_port import TorchCrnPort
    from aec_amd import synth
    sc = [synth.scene(n, 90000 + i, double_talk=False) for i in range(streams)]
    nh = n // 256 + 1
    M = torch.zeros(streams, 256 * (nh + 1), device=dev)
    F = torch.zeros_like(M)
    M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sc])).to(dev)
    F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sc])).to(dev)
    net.stream_open(streams, device=dev)
    with torch.no_grad():
        outs = [net.stream_step(M[:, 256 * k:256 * (k + 1)], F[:, 256 * k:256 * (k + 1)]).clone() for k in range(nh)]
    torch.cuda.synchronize(dev)
    got = torch.cat(outs[1:], dim=1)[:, :256 * (n // 256)].cpu().numpy()
    w = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    port = TorchCrnPort(w, conf, 2, nlms=nlms)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = port(torch.from_numpy(np.stack([s[0] for s in sc])), torch.from_numpy(np.stack([s[1] for s in sc]))).numpy()
    g = [erle_db(sc[i][0], got[i]) for i in range(streams)]
    r = [erle_db(sc[i][0], ref[i]) for i in range(streams)]
    return dict(gpu_db=round(float(np.mean(g)), 4), reference_db=round(float(np.mean(r)), 4),
                delta_db=round(float(np.mean(g) - np.mean(r)), 5), streams=streams,
                scene='far-end single talk (near = 0), 10 s, synthetic RIR echo, stepped one hop per call',
                reference='oracle/torch_crn_port.py TorchCrnPort (reference op mix, f32, same FD-NLMS front end)')


def run_c5_stream(dev, B=256, hops=200, dtype='fp8', world=1, with_cpu=False, sweep=(1024, 4096),
                  cpu_seconds=10.0, with_erle=False):
    """BASELINE config 5: the per-hop step of the DCCRN (7 launches; timed launched directly and
    replayed from its hipGraphs)
    (MX-fp8 LSTM input projections, recurrence and wide conv layers) fed by the FD-NLMS,
    B concurrent streams per GPU, one 256-sample hop per stream per step
    (aec_crn_stream_step).  With world > 1 every rank steps its own B streams
    (no data-path collective); the timed region is bracketed by barriers and
    the time is the max over ranks.  Input: one random hop pair per stream,
    resident in the same device buffers every step (the graph's input nodes
    keep their pointers; parity of the step on real audio, and graph replay ==
    direct launches bit for bit, is tests/test_gpu_bench_shapes.py)."""
    import torch
    import torch.distributed as dist
    import aec_amd
    from aec_amd import shard
    torch.manual_seed(0)
    conf = dict(aec_amd.net_conf)
    net = aec_amd.dccrn2.DCCRN(conf, dtype=dtype, nlms=aec_amd.nlms_conf).eval().to(dev)

    def time_hops(bb, nhops, barrier, graph=False):
        net.stream_open(bb, device=dev, graph=graph)
        g = torch.Generator(device=dev).manual_seed(5)
        mic = 0.1 * torch.randn(bb, 256, device=dev, generator=g)
        far = 0.1 * torch.randn(bb, 256, device=dev, generator=g)
        out = torch.empty(bb, 256, device=dev)
        with torch.no_grad():
            # untimed warm-up of at least WARM_MS of back-to-back hops: the chip's clocks ramp over
            # the first ~20 ms of continuous load, longer than 200 hops at B=1
            tw = time.perf_counter()
            nw = 0
            while nw < 10 or (time.perf_counter() - tw) * 1e3 < WARM_MS:
                for _ in range(10):
                    net.stream_step(mic, far, out)
                nw += 10
                torch.cuda.synchronize(dev)
            if barrier and world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(nhops):
                net.stream_step(mic, far, out)
            torch.cuda.synchronize(dev)
            if barrier and world > 1:
                dist.barrier()
            el = time.perf_counter() - t0
        return shard.max_over_ranks(el) / nhops if barrier else el / nhops

    dt = time_hops(B, hops, True)
    # BASELINE configs[4] names the hipGraph-captured per-hop step: the same hops replayed from the
    # per-parity graphs (bit-identical, tests/test_gpu_bench_shapes.py), timed the same way; the
    # library's counters prove every timed hop was a replay
    dt_graph = time_hops(B, hops, True, graph=True)
    gstats = net.stream_stats()
    if gstats['graph_mode'] != 1 or gstats['direct_hops'] != 0 or gstats['graph_replays'] < hops:
        raise RuntimeError(f'C5 graph mode did not replay every hop: {gstats}')
    streams_sweep = None
    lat_b1 = None
    if world == 1:
        # the drop-in's own operating point is one stream (test.py:139): per-hop latency of a single
        # stream, host-synchronous per hop (submit, wait) and back-to-back (the graph replay rate)
        lat_b1 = dict(ms_per_hop_back_to_back=round(time_hops(1, hops, False) * 1e3, 4))
        net.stream_open(1, device=dev)
        g1 = torch.Generator(device=dev).manual_seed(6)
        m1 = 0.1 * torch.randn(1, 256, device=dev, generator=g1)
        f1 = 0.1 * torch.randn(1, 256, device=dev, generator=g1)
        o1 = torch.empty(1, 256, device=dev)
        sync_lat = []
        with torch.no_grad():
            for k in range(60):
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                net.stream_step(m1, f1, o1)
                torch.cuda.synchronize(dev)
                if k >= 10:
                    sync_lat.append(time.perf_counter() - t1)
        sync_lat.sort()
        lat_b1['ms_per_hop_synchronous_median'] = round(sync_lat[len(sync_lat) // 2] * 1e3, 4)
        lat_b1['rtf'] = round(lat_b1['ms_per_hop_synchronous_median'] / 16.0, 6)
    if world == 1 and sweep:
        streams_sweep = {'1': round(1e3 / lat_b1['ms_per_hop_back_to_back'], 1), str(B): round(B / dt, 1)}
        for bb in sweep:
            d2 = time_hops(bb, max(20, hops // 4), False)
            streams_sweep[str(bb)] = round(bb / d2, 1)
    erle = None
    if with_erle and world == 1:
        erle = c5_erle(net, dev, conf, aec_amd.nlms_conf)
    time_hops(B, 1, False)                           # leave the bench shape's streams open
    pmc = None
    pp = os.path.join(REPO, 'profiles', 'pmc_latest_c5.json')
    if os.path.exists(pp):
        pmc = json.load(open(pp))
    res = dict(workload=f'C5 (BASELINE configs[4]): {world} GPU(s) x {B} concurrent streams, one 256-sample hop per '
                        f'stream per step through the per-hop STFT -> FD-NLMS (4 taps) -> DCCRN v2 '
                        f'(net_conf, {dtype}' + (': bf16 + MX-fp8 LSTM input projections, LSTM recurrence (W_ih, W_hh, '
                        'x, h) and encoder 4-5 / decoder 4-6 convs'
                        if dtype == 'fp8' else '') + ') -> iSTFT step; input = one random hop pair per stream, '
                        'resident in the same device buffers every step',
               dtype=dtype, n_gpus=world, streams=B * world, hops=hops, ms_per_hop=round(dt * 1e3, 4),
               launch_mode='direct launches (the library default; ms_per_hop)',
               graph_ms_per_hop=round(dt_graph * 1e3, 4),
               graph_frames_per_s_per_gpu=round(B / dt_graph, 1),
               graph_stats=dict(gstats, note='aec_crn_stream_stats after the graph-mode timing (warm-up + timed hops)'),
               frames_per_s=round(world * B / dt, 1), frames_per_s_per_gpu=round(B / dt, 1),
               rtf=round(dt / 0.016, 5), roofline=c5_roofline(conf, B, dt * 1e3, pmc),
               latency_ms_per_hop_b1=lat_b1['ms_per_hop_synchronous_median'] if lat_b1 else None,
               batch1=lat_b1, streams_sweep_frames_per_s_per_gpu=streams_sweep, erle=erle, cpu_baseline=None)
    if lat_b1:
        # what limits the hop: one stream's back-to-back hop against B streams' (a latency chain of 7
        # launches when the two are about equal, not MFMA or HBM throughput)
        r1 = lat_b1['ms_per_hop_back_to_back'] / (dt * 1e3)
        res['roofline']['limiter'] = (f'latency: one stream\'s hop takes {r1:.2f} of {B} streams\' '
                                      f'({lat_b1["ms_per_hop_back_to_back"]} vs {round(dt * 1e3, 4)} ms back to '
                                      f'back), the 7-launch chain, not throughput')
    if with_cpu and world == 1:
        res['cpu_baseline'] = cpu_baseline_c5(cpu_seconds, net, conf, aec_amd.nlms_conf, B)
    del net
    torch.cuda.empty_cache()
    return res


def cpu_baseline_train(seconds, B=16, n=160000):
    """Training iteration (train1.py:199-218) with the reference's CPU op mix
    and autograd (oracle/torch_port.py TorchTrainPort), bounded sample."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    from torch_port import TorchTrainPort
    from aec_amd import synth, erb_matrix
    w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
    port = TorchTrainPort(w, erb_matrix())
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    mic, ref, near = (torch.from_numpy(a) for a in synth.batch(B, n, seed0=6000))
    port.step(mic[:2, :16000], ref[:2, :16000], near[:2, :16000])
    reps, t0 = 0, time.perf_counter()
    while True:
        port.step(mic, ref, near)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 20:
            break
    return dict(value=round(reps * B * (n // 256 + 1) / el, 1), unit='frames/s', cores=threads, kind='port',
                ms_per_step=round(el / reps * 1e3, 1),
                sample=f'{reps} training iterations on [{B} x {n}] through oracle/torch_port.py TorchTrainPort '
                       f'(reference op mix + autograd + torch Adam), {el:.1f} s wall')


def run_train(dev, B=16, n=160000, steps=10, warmup=2, with_cpu=False):
    """Training iteration of scripts/train1.py:199-218 on the drop-in:
    Little_net.train() forward on the padded [B, n] batch, loss.backward()
    (aec_train_backward), Adam.step() (aec_adam_step); inputs resident."""
    import numpy as np
    import torch
    import aec_amd
    from aec_amd import synth
    from aec_amd.train import Adam
    w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
    net = aec_amd.Little_net(aec_amd.speech_conf, 32)
    sd = net.state_dict()
    for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
              'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']:
        sd[k] = torch.from_numpy(w[k])
    net.load_state_dict(sd)
    net = net.to(dev).train()
    erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
    mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(B, n, seed0=7000))
    opt = Adam(net.parameters(), lr=aec_amd.train_conf['lr'])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    stage = np.zeros(3)

    def one(timed=False):
        opt.zero_grad()
        if timed:
            ev[0].record()
        _, loss = net(mic, ref, near, erb)
        if timed:
            ev[1].record()
        loss.backward()
        if timed:
            ev[2].record()
        opt.step()
        if timed:
            ev[3].record()
        return loss

    tw = time.perf_counter()
    nw = 0
    while nw < warmup or (time.perf_counter() - tw) * 1e3 < WARM_MS:   # clock-ramp floor, as time_hops
        one()
        nw += 1
        if nw % 8 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    for _ in range(3):                        # stage split: a separate, event-bracketed pass
        one(True)
        torch.cuda.synchronize(dev)
        stage += [ev[i].elapsed_time(ev[i + 1]) for i in range(3)]
    stage /= 3
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = one()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    T = n // 256 + 1
    res = dict(workload=f'one training iteration (train1.py:199-218): Little_net forward on a padded [{B} x {n}] '
                        'batch (batch-global normaliser), loss.backward() (head + BPTT on the device), Adam.step()',
               batch=B, steps=steps, ms_per_step=round(el / steps * 1e3, 3),
               frames_per_s=round(B * T * steps / el, 1),
               stage_ms={'forward': round(stage[0], 3), 'backward': round(stage[1], 3), 'adam': round(stage[2], 3)},
               loss=round(float(loss), 5))
    if with_cpu:
        res['cpu_baseline'] = cpu_baseline_train(10.0, B, n)
    return res


def crn_workload(args, dtype, B):
    return (f'C3 (BASELINE configs[2]): DCCRN v{args.crn_version} '
            f'({"dccrn2.py" if args.crn_version == 2 else "dccrn.py"}, configs.net_conf, {dtype} MFMA) on {B} '
            'concurrent 10 s 16 kHz streams per GPU, reference init (torch.manual_seed(0))')


def main_crn(args):
    """--pipeline crn: BASELINE config 3 as the headline line."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = _init_dist(torch, dist, world, int(os.environ.get('LOCAL_RANK', '0')))
    dev = torch.device('cuda', local)
    B = args.streams
    n = int(round(args.seconds * 16000))
    import aec_amd
    prov = knob_provenance()
    nl = aec_amd.nlms_conf if args.crn_nlms else None
    r = run_crn(args, dev, rank, world, args.crn_dtype, args.steps, args.warmup, B, n, not args.no_cpu, nl)
    if rank == 0:
        line = {
            'metric': '16kHz frames/sec/GPU (batched AEC) + RTF@batch=1; ERLE delta vs reference',
            'value': r['value'], 'unit': 'frames/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': r['ms_per_step'], 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': args.crn_dtype, 'data': 'synthetic',
            'config': {'workload': crn_workload(args, args.crn_dtype, B) + (' fed by the FD-NLMS error spectrum (C5)'
                                                                            if nl else ''),
                       'streams_per_gpu': B, 'samples_per_stream': n, 'frames_per_stream': n // 256 + 1,
                       'frame': '256-sample hop', 'pipeline': 'crn', 'batches_in_flight': r['batches_in_flight'],
                       'parallelism': f'streams sharded, {world} rank(s)'},
            'value_per_gpu': r['value_per_gpu'],
            'aggregate_frames_per_s': r['value'],
            'value_semantics': VALUE_SEMANTICS,
            'xRT': round(r['value'] * 256 / 16000, 1),
        }
        line.update({k: r[k] for k in ('rtf_batch1', 'stage_ms_per_step', 'roofline', 'pipeline_roofline',
                                       'erle', 'cpu_baseline')})
        line['knobs'] = prov
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.pipeline == 'crn':
        return main_crn(args)
    import numpy as np
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    local = _init_dist(torch, dist, world, local)
    dev = torch.device('cuda', local)
    import aec_amd
    from aec_amd import shard, synth
    prov = knob_provenance()

    B = args.streams
    n = int(round(args.seconds * 16000))
    T = n // 256 + 1
    w = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz')))
    nlms = aec_amd.nlms_conf if args.pipeline == 'full' else None
    net = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=nlms).eval()
    sd = net.state_dict()
    for k in ['gru1.weight_ih_l0', 'gru1.weight_hh_l0', 'gru1.bias_ih_l0', 'gru1.bias_hh_l0',
              'linear1.weight', 'linear1.bias', 'linear2.weight', 'linear2.bias']:
        sd[k] = torch.from_numpy(w[k])
    net.load_state_dict(sd)
    net = net.to(dev)
    erb = torch.tensor(aec_amd.erb_matrix(), dtype=torch.float32, device=dev)
    mic, ref, near = (torch.from_numpy(a).to(dev) for a in synth.batch(B, n, seed0=1000 * rank))
    lens = [n] * B

    # batches in flight: step k runs on HIP stream k % inflight with its own handle
    # (each aec_handle owns its workspace), so one batch's latency-bound GRU +
    # synthesis kernel overlaps the next batch's moments pass; every batch is
    # processed whole
    inflight = max(1, args.inflight)
    nets = [net]
    for _ in range(inflight - 1):
        extra = aec_amd.Little_net(aec_amd.speech_conf, 32, nlms=nlms).eval()
        extra.load_state_dict(net.state_dict())
        nets.append(extra.to(dev))
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(inflight - 1)]
    kstep = [0]
    # look-ahead (aec_prepare): step k queues the normaliser pass of batch k + LOOKAHEAD on a side
    # stream before its own kernels, so that HBM-bound pass runs under the compute of the batches
    # in flight instead of in front of that batch's analysis.  Every step still runs one pass (the
    # timed region's first batches take the passes queued by the last warm-up steps).
    side = None
    if args.lookahead:
        side = cu_masked_stream(dev, args.lookahead_cus) if args.lookahead_cus > 0 else torch.cuda.Stream(dev)

    tokens = {}                                  # step index -> look-ahead token of its batch

    def step(nr=near):
        # nr: the near-end signal (the loss target); None = the deployment form (no clean near-end
        # exists outside synthetic data; test.py:157 discards the loss): no near transform, no loss
        n_ = kstep[0]
        k = n_ % inflight
        kstep[0] += 1
        if side is not None:
            with torch.cuda.stream(side):
                tokens[n_ + args.lookahead] = nets[(k + args.lookahead) % inflight].prepare_ragged(mic, ref, nr,
                                                                                                  lens)
        with torch.cuda.stream(streams[k]):
            return nets[k].forward_ragged(mic, ref, nr, erb, lens, lookahead=tokens.pop(n_, None))

    with torch.no_grad():
        for _ in range(2):
            nets[0].forward_ragged(mic, ref, near, erb, lens)
        torch.cuda.synchronize(dev)
        # per-kernel times (roofline): HIP events around each kernel over a
        # sequential pass (one batch in flight, so no event interval contains
        # another batch's kernels; no look-ahead, so the moments pass is inside)
        h0 = nets[0]._handle(dev)[0]
        prof_steps = max(1, min(args.steps, 10))
        h0.profile_enable(True)
        torch.cuda.synchronize(dev)
        for _ in range(prof_steps):
            nets[0].forward_ragged(mic, ref, near, erb, lens)
        torch.cuda.synchronize(dev)
        kms, calls = h0.profile_read()
        h0.profile_enable(False)
        # warm-up steps in the timed loop's own form (the last one queues the first timed batch's
        # look-ahead pass): at least MIN_WARM_STEPS of them (~20 ms of continuous load).  The chip
        # clocks up over its first ~20 ms under this load: after 5 warm-up steps the first ~20
        # timed batches run ~15 % slower than the rest (tools/c2_step_events.py,
        # profiles/r05z6_warmup_ab.log), so a short timed region would price that ramp, not the path.
        warm_steps = max(args.warmup, inflight, args.lookahead, MIN_WARM_STEPS)
        for _ in range(warm_steps):
            step()
        torch.cuda.synchronize(dev)
        # the timed region: K steps, `inflight` batches in flight
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        el = shard.max_over_ranks(el)              # all_reduce(MAX) of one scalar, outside the timed region
        # the same pipelined step without the near-end signal (reported beside `value`, never as it):
        # the enhanced waveform only, as the reference's inference entry point uses it (test.py:157
        # keeps out_wav and discards the loss); the look-ahead queue is drained and refilled first,
        # since a token is tied to the signals it was prepared for
        no_near = None
        if not args.no_near_leg:
            torch.cuda.synchronize(dev)
            tokens.clear()
            kstep[0] = 0
            if side is not None:
                for j in range(args.lookahead):
                    with torch.cuda.stream(side):
                        tokens[j] = nets[j % inflight].prepare_ragged(mic, ref, None, lens)
            for _ in range(warm_steps):
                step(None)
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            for _ in range(args.steps):
                step(None)
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            el2 = shard.max_over_ranks(time.perf_counter() - t2)
            no_near = {'frames_per_s': round(world * B * T * args.steps / el2, 1),
                       'ms_per_step': round(el2 / args.steps * 1e3, 4), 'steps': args.steps,
                       'what': 'the same 256-stream pipelined step with near=None: mic / ref moments, no near-end '
                               'transform, no loss (the enhanced waveform is bit-identical to the headline path, '
                               'tests/test_gpu_nlms.py::test_no_near_waveform_bit_exact); not the headline, which '
                               'runs the reference forward whole (ERB.py:252-334, loss included)'}
        # RTF at batch 1: one 10 s utterance, synchronous latency (median of 7)
        lat = []
        for _ in range(0 if args.no_rtf else 7):
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            net.forward_ragged(mic[:1], ref[:1], near[:1], erb, [n])
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - t1)
        rtf1 = float(np.median(lat)) / args.seconds if lat else None
        sweep = None
        if not args.no_sweep and world == 1:
            # frames/s at B concurrent streams per call (one batch in flight, 5 synchronous calls
            # after two warm-ups); the drop-in's own operating point is B = 1 (test.py:139)
            sweep = {}
            for bb in [1, 16, 64, 256, 1024, 4096]:
                if bb > B:
                    mm, rr, nn_ = (x.repeat((bb + B - 1) // B, 1)[:bb] for x in (mic, ref, near))
                else:
                    mm, rr, nn_ = mic[:bb], ref[:bb], near[:bb]
                for _ in range(2):                     # warm-up: workspace growth, work lists
                    net.forward_ragged(mm, rr, nn_, erb, [n] * bb)
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                for _ in range(5):
                    net.forward_ragged(mm, rr, nn_, erb, [n] * bb)
                torch.cuda.synchronize(dev)
                sweep[str(bb)] = round(bb * T * 5 / (time.perf_counter() - t1), 1)
                del mm, rr, nn_
            torch.cuda.empty_cache()

    frames_total = world * B * T * args.steps
    value = frames_total / el
    ms_step = el / args.steps * 1e3
    # `calls` counts aec_process calls (profile marks per call; one launch of each
    # kernel per call here: 256 streams, no sub-batching)
    calls_per_step = max(calls, 1) / prof_steps
    per_kernel_ms = {k: kms[i] / prof_steps for i, k in enumerate(KERNELS)}
    per_launch_ms = {k: kms[i] / max(calls, 1) for i, k in enumerate(KERNELS)}
    if args.pipeline == 'full' and os.environ.get('AEC_FUSED_SYNTH', '1') != '0':
        # one fused launch: its time is in the 'gru' slot, the 'synthesis' slot is an empty interval
        kernels_per_call = ['moments_lds_kernel', 'norm_finalize_kernel', 'nlms_analysis_kernel', 'gru_synth_kernel']
        for d in (per_kernel_ms, per_launch_ms):
            d['gru_synthesis'] = d.pop('gru') + d.pop('synthesis')
    else:
        kernels_per_call = ['moments_lds_kernel', 'norm_finalize_kernel', 'analysis_kernel', 'gru_kernel',
                            'synthesis_kernel']
    launches_per_step = calls_per_step * len(kernels_per_call)
    dom = max(per_kernel_ms, key=per_kernel_ms.get)
    pmc = None
    pmc_path = os.path.join(REPO, 'profiles', f'pmc_latest_{args.pipeline}.json')
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path))
    roof = roofline(args.pipeline, dom, per_launch_ms[dom], int(round(B * T / calls_per_step)), pmc)
    if args.pipeline == 'full':
        roof['sq'] = sq_limiter(dom)
        roof['limiter'] = roof['sq']['limiter'] if roof['sq'] else None
    # every kernel of the step against its own roofline (the fused GRU + synthesis kernel runs two
    # streams per block on half the CUs, so the longest launch is not the one holding the most CU
    # time): the same figures as `roofline`, per kernel
    kernel_rooflines = {}
    for k in per_launch_ms:
        if per_launch_ms[k] > 0 and k in ALG[args.pipeline]:
            r = roofline(args.pipeline, k, per_launch_ms[k], int(round(B * T / calls_per_step)), pmc)
            kernel_rooflines[k] = {x: r[x] for x in ('bound', 'frac', 'hbm_frac', 'fp32_frac', 'ms_per_launch',
                                                     'traffic', 'traffic_alg_bytes_per_launch')}
            # `bound` is the roofline the kernel's algorithmic work is priced against; `sq` says what
            # the counters show limits it (C2's kernels: latency, not HBM or VALU throughput)
            kernel_rooflines[k]['sq'] = sq_limiter(k) if args.pipeline == 'full' else None
    pipe_t = ms_step * 1e-3
    pipe_gbs = PIPE['bytes'] * B * T / pipe_t / 1e9
    pipe_tfl = path_flops(args.pipeline) * B * T / pipe_t / 1e12
    cpu = None
    erle = None
    erle_bypass = None
    c3 = None
    if world == 1 and not args.no_c3:
        # BASELINE config 3 (DCCRN bf16, 256 x 10 s) in the same driver-timed run
        c3 = run_crn(args, dev, rank, world, 'bf16', args.c3_steps, 2, 256, 160000, not args.no_cpu)
        c3 = dict(workload=crn_workload(args, 'bf16', 256), dtype='bf16', steps=args.c3_steps,
                  batches_in_flight=c3['batches_in_flight'],
                  frames_per_s=c3['value'], ms_per_step=c3['ms_per_step'], rtf_batch1=c3['rtf_batch1'],
                  stage_ms_per_step=c3['stage_ms_per_step'], roofline=c3['roofline'],
                  pipeline_roofline=c3['pipeline_roofline'], erle=c3['erle'], cpu_baseline=c3['cpu_baseline'])
    c3f = None
    if world == 1 and not args.no_c3:
        # the same C3 batch with dtype fp8 (MX-fp8 LSTM input projections and wide conv layers,
        # e4m3 operands written by the producing epilogues)
        c3f = run_crn(args, dev, rank, world, 'fp8', args.c3_steps, 2, 256, 160000, False,
                      with_erle=not args.no_cpu)
        if c3 and c3.get('cpu_baseline'):
            # the CPU reference path is the same f32 op mix whatever the GPU dtype: C3's sample, reported here too
            c3f['cpu_baseline'] = dict(c3['cpu_baseline'], note='same CPU sample as c3_crn_bf16.cpu_baseline (the '
                                                                 'reference op mix is f32 for every GPU dtype)')
        c3f = dict(workload=crn_workload(args, 'fp8', 256), dtype='fp8', steps=args.c3_steps,
                   batches_in_flight=c3f['batches_in_flight'], frames_per_s=c3f['value'],
                   ms_per_step=c3f['ms_per_step'], stage_ms_per_step=c3f['stage_ms_per_step'],
                   roofline=c3f['roofline'], pipeline_roofline=c3f['pipeline_roofline'], erle=c3f['erle'],
                   cpu_baseline=c3f['cpu_baseline'])
    c4 = None
    if world == 1 and not args.no_c3:
        # C4's per-GPU leg: FD-NLMS + DCCRN post-filter (bf16) on one GPU's shard of utterances
        c4 = run_crn(args, dev, rank, world, 'bf16', args.c3_steps, 2, 256, 160000, not args.no_cpu,
                     aec_amd.nlms_conf, with_erle=not args.no_cpu)
        c4 = dict(workload='C4 (BASELINE configs[3]) per-GPU leg: end-to-end STFT -> FD-NLMS (4 taps) -> DCCRN v2 '
                           'post-filter (dccrn2.py, configs.net_conf, bf16 MFMA) -> iSTFT on one GPU\'s shard of 256 '
                           'concurrent 10 s 16 kHz utterances (the 8-GPU job runs this per rank, no data-path '
                           'collective)',
                  dtype='bf16', steps=args.c3_steps, batches_in_flight=c4['batches_in_flight'],
                  frames_per_s=c4['value'], ms_per_step=c4['ms_per_step'],
                  stage_ms_per_step=c4['stage_ms_per_step'], roofline=c4['roofline'],
                  pipeline_roofline=c4['pipeline_roofline'], erle=c4['erle'], cpu_baseline=c4['cpu_baseline'])
    c5s = None
    if not args.no_c3:
        # C5 is quoted on 8 GPUs: the per-hop step runs on every rank (streams sharded, weak scaling)
        c5s = run_c5_stream(dev, world=world, with_cpu=rank == 0 and world == 1 and not args.no_cpu,
                            sweep=() if args.no_sweep else (1024, 4096),
                            with_erle=rank == 0 and world == 1 and not args.no_cpu)
    tr = None
    if world == 1 and not args.no_train:
        tr = run_train(dev, 16, 160000, args.train_steps, with_cpu=not args.no_cpu)
        tr['batch256'] = {k: v for k, v in run_train(dev, 256, 160000, max(2, args.train_steps // 2)).items()
                          if k in ('ms_per_step', 'frames_per_s', 'stage_ms')}
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_seconds)
        sys.path.insert(0, os.path.join(REPO, 'oracle'))
        import aec_oracle
        erb_np = aec_amd.erb_matrix().astype(np.float32)

        def gpu1(m_, r_, n_):
            with torch.no_grad():
                o, _ = net.forward_ragged(*(torch.from_numpy(x)[None].to(dev) for x in (m_, r_, n_)), erb, [len(m_)])
            return o[0].cpu().numpy()

        erle = erle_check(gpu1, lambda m_, r_, n_: aec_oracle.aec_forward(m_, r_, n_, erb_np, w, nlms)[0], n)
        erle['note'] = ('GPU vs the float64 oracle of the same pipeline; the oracle\'s FD-NLMS is the build\'s own '
                        '(the reference has none), so this delta is GPU-vs-oracle; erle_bypass is the reference pin')
        # the one ERLE the reference pins: the Little_net path (NLMS bypass) vs the reference restatement
        # (aec_oracle.little_net_forward, pinned to the reference goldens), 10 s far-end single talk
        pf = aec_amd.Little_net(aec_amd.speech_conf, 32).eval()
        pf.load_state_dict(net.state_dict())
        pf = pf.to(dev)

        def gpu_pf(m_, r_, n_):
            with torch.no_grad():
                o, _ = pf.forward_ragged(*(torch.from_numpy(x)[None].to(dev) for x in (m_, r_, n_)), erb, [len(m_)])
            return o[0].cpu().numpy()

        erle_bypass = erle_check(gpu_pf, lambda m_, r_, n_: aec_oracle.little_net_forward(m_, r_, n_, erb_np, w)[0], n)
        erle_bypass['path'] = ('reference Little_net (ERB.py:252-334, NLMS bypass) on the GPU vs its float64 '
                               'restatement pinned by the reference goldens')
        del pf
    if rank == 0:
        line = {
            'metric': '16kHz frames/sec/GPU (batched AEC) + RTF@batch=1; ERLE delta vs reference',
            'value': round(value, 1), 'unit': 'frames/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'warmup_requested': args.warmup, 'warmup_steps_run': warm_steps,
            'warmup_note': f'warmup = the --warmup argument (driver contract); {warm_steps} untimed steps ran '
                           f'(floor {MIN_WARM_STEPS}: the clock ramp)',
            'ms_per_step': round(ms_step, 4), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': {'workload': WORKLOAD[args.pipeline],
                       'streams_per_gpu': B, 'samples_per_stream': n, 'frames_per_stream': T,
                       'frame': '256-sample hop', 'pipeline': args.pipeline, 'batches_in_flight': inflight,
                       'normaliser_lookahead_batches': args.lookahead if args.pipeline != 'crn' else 0,
                       'normaliser_lookahead_cus': args.lookahead_cus if args.pipeline != 'crn' else 0,
                       'parallelism': f'streams sharded, {world} rank(s)'},
            'value_per_gpu': round(value / world, 1),
            'aggregate_frames_per_s': round(value, 1),
            'value_semantics': VALUE_SEMANTICS,
            'xRT': round(value * 256 / 16000, 1),
            'rtf_batch1': rtf1,
            'kernel_ms_per_step': {k: round(v, 4) for k, v in per_kernel_ms.items()},
            'kernel_timing': f'HIP events around each kernel, sequential pass of {prof_steps} steps (1 batch in flight)',
            'kernels_per_step': kernels_per_call,
            'launches_per_step': launches_per_step,
            'roofline': roof,
            'kernel_rooflines': kernel_rooflines,
            'pipeline_roofline': {'alg_bytes_per_frame': PIPE['bytes'],
                                  'alg_flops_per_frame': path_flops(args.pipeline),
                                  'hbm_frac': round(pipe_gbs / HBM_PEAK_GBS, 4),
                                  'fp32_frac': round(pipe_tfl / FP32_PEAK_TFLOPS, 4)},
            'no_near': no_near,
            'erle': erle,
            'erle_bypass': erle_bypass,
            'cpu_baseline': cpu,
            'c3_crn_bf16': c3,
            'c3_crn_fp8': c3f,
            'c4_nlms_crn_bf16_per_gpu': c4,
            'c5_stream_fp8': c5s,
            'train_step': tr,
            'knobs': prov,
        }
        if sweep:
            line['batch_sweep_frames_per_s'] = sweep
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
