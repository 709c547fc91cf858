"""Persistent LSTM recurrence probe: golden v2E_2125 bf16 input, NaN map per
output hop, then a second call (it reports a timeout flag left by the first)."""
import copy
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'acoustic-echo-cancellation_amd'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))
import aec_amd  # noqa: E402
import crn_oracle as C  # noqa: E402

meta = json.load(open(os.path.join(REPO, 'tests', 'golden', 'crn_meta.json')))
name = sys.argv[1] if len(sys.argv) > 1 else 'v2E_2125'
m = meta[name]
conf = copy.deepcopy(aec_amd.net_conf)
conf.update(m['overrides'])
net = aec_amd.dccrn2.DCCRN(conf, dtype='bf16').eval()
sd = net.state_dict()
for k, v in C.make_weights(conf, 2, m['weight_seed']).items():
    sd[k] = torch.from_numpy(v)
net.load_state_dict(sd)
net = net.cuda()
d = np.load(os.path.join(REPO, 'tests', 'golden', f'crn_{name}.npz'))
x = lambda a: torch.as_tensor(a, device='cuda')[None]
with torch.no_grad():
    out, _, mask = net.forward_ragged(x(d['mic']), x(d['far']), [m['n']], want_spec=False, want_mask=True)
    torch.cuda.synchronize()
    o = out[0].cpu().numpy()
    mk = mask[0].cpu().numpy()
    print('nan per hop:', [int(np.isnan(o[i:i + 256]).sum()) for i in range(0, len(o), 256)])
    print('mask nan per frame:', [int(np.isnan(mk[..., t]).sum()) for t in range(mk.shape[-1])])
    print('mask rel err per frame:', [round(float(np.sqrt(np.mean((mk[..., t] - d['mask'][..., t]) ** 2)) /
                                             np.sqrt(np.mean(d['mask'][..., t] ** 2))), 4) for t in range(mk.shape[-1])])
    try:
        net.forward_ragged(x(d['mic']), x(d['far']), [m['n']], want_spec=False)
        torch.cuda.synchronize()
        print('second call ok')
    except RuntimeError as e:
        print('second call:', e)
