#!/bin/bash
# Step-kernel decomposition (CRN_STEP_MODE, timing only): median step time per mode
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for m in "$@"; do
  CRN_STEP_MODE=$m bash $R/tools/crn_prof.sh mode$m --B 256 --N 160000 > /dev/null 2>&1 || exit 1
  python3 - $R/gpurun_out/prof_mode$m $m <<'PY'
import csv, statistics as st, sys
r=[x for x in csv.DictReader(open(sys.argv[1]+'/trace/run_kernel_trace.csv')) if 'lstm_step' in x['Kernel_Name']]
d=[(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3 for x in r]
print('mode', sys.argv[2], 'median step us', round(st.median(d),2), 'min', round(min(d),2))
PY
done
