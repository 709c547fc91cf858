"""Debug: C5 fp8 stream step with the MX level-4 fold (AEC_CRN_STREAM_FUSE 15 vs 31, with and without
the level-4 GEMM re-run): finite outputs and differences.  GPU box only."""
import os, sys, copy, subprocess, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys, copy, json
import numpy as np, torch
sys.path.insert(0, os.path.join(%r, 'acoustic-echo-cancellation_amd')); sys.path.insert(0, os.path.join(%r, 'oracle'))
import aec_amd, crn_oracle as C
from aec_amd import synth
conf = copy.deepcopy(aec_amd.net_conf)
net = aec_amd.dccrn2.DCCRN(conf, dtype='fp8').eval()
sd = net.state_dict()
for k, v in C.make_weights(conf, 2, 1).items(): sd[k] = torch.from_numpy(v)
net.load_state_dict(sd); net = net.cuda()
B, n = 3, 2304
sig = [synth.scene(n, 60 + b) for b in range(B)]
nh = n // 256 + 1
M = torch.zeros(B, 256 * (nh + 1), device='cuda:0'); F = torch.zeros_like(M)
M[:, :n] = torch.from_numpy(np.stack([s[0] for s in sig])).cuda(); F[:, :n] = torch.from_numpy(np.stack([s[1] for s in sig])).cuda()
net.stream_open(B)
outs = []
with torch.no_grad():
    for k in range(nh):
        outs.append(net.stream_step(M[:, 256*k:256*(k+1)], F[:, 256*k:256*(k+1)]).clone())
torch.cuda.synchronize()
o = torch.stack(outs).cpu().numpy()
np.save(sys.argv[1], o)
print(json.dumps(dict(finite=bool(np.isfinite(o).all()), first_nan_hop=int(np.argmax(~np.isfinite(o).reshape(nh, -1).all(1))) if not np.isfinite(o).all() else -1)))
''' % (REPO, REPO)
res = {}
for tag, env in [('f15', dict(AEC_CRN_STREAM_FUSE='15')), ('f31', dict(AEC_CRN_STREAM_FUSE='31')),
                 ('f31r', dict(AEC_CRN_STREAM_FUSE='31', AEC_CRN_ENC_MX_RERUN='1'))]:
    e = dict(os.environ, **env)
    out = os.path.join(REPO, 'gpurun_out', f'encmx_{tag}.npy')
    r = subprocess.run([sys.executable, '-c', code, out], env=e, capture_output=True, text=True, timeout=300)
    print(tag, r.stdout.strip()[-300:], r.stderr.strip()[-300:] if r.returncode else '')
    res[tag] = np.load(out) if os.path.exists(out) else None
for a, b in [('f15', 'f31'), ('f15', 'f31r')]:
    if res[a] is not None and res[b] is not None:
        d = np.abs(np.nan_to_num(res[a], nan=1e9) - np.nan_to_num(res[b], nan=1e9))
        print(a, b, 'max abs diff', float(d.max()), 'equal', bool(np.array_equal(res[a], res[b])))
