#!/bin/bash
# round 5 batch w: where the window-in-overlap-add build differs from HEAD (arrays compared on the box)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
LIB_BITCMP_DUMP=/tmp/r05w_tree.npz timeout -k 10 120 python $R/tools/lib_bitcmp.py || exit 1
AEC_HIP_LIB=$AB/olawin.so LIB_BITCMP_DUMP=/tmp/r05w_olawin.npz timeout -k 10 120 python $R/tools/lib_bitcmp.py || exit 1
python - <<'PY'
import numpy as np
a=np.load('/tmp/r05w_tree.npz'); b=np.load('/tmp/r05w_olawin.npz')
for k in ('out','loss'):
    x,y=a[k],b[k]
    d=np.abs(x.astype(np.float64)-y)
    nz=np.argwhere(x!=y)
    print(k, 'differing', len(nz), 'of', x.size, 'max abs', d.max(), 'max rel', (d/np.maximum(np.abs(x),1e-30)).max())
    if len(nz):
        print(' first', nz[:8].tolist())
        rows=np.unique(nz[:,0]) if x.ndim>1 else nz
        print(' rows', rows[:20].tolist())
        if x.ndim>1:
            cols=nz[:,1]
            print(' cols % 256 histogram', np.bincount(cols % 256, minlength=256).nonzero()[0][:20].tolist())
            i,j=nz[0]; print(' sample', x[i,j], y[i,j])
PY
