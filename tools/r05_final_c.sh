#!/bin/bash
# round-5 end-of-round evidence (3/3): C5 per-hop trace (hop table), C3 kernel traces (bf16, fp8),
# C5 / C3 PMC passes, and the C3 LSTM input GEMM's HBM bytes with the XCD-aware tile order
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
bash $R/tools/c5_prof.sh r05z_c5 > $O/r05z_c5prof.log 2>&1 || { echo "c5 trace failed"; tail $O/r05z_c5prof.log; exit 1; }
python $R/tools/c5_hop_table.py $O/prof_r05z_c5 > $O/r05z_c5_hop_table.txt 2>&1 || { echo "hop table failed"; tail $O/r05z_c5_hop_table.txt; exit 1; }
head -20 $O/r05z_c5_hop_table.txt
bash $R/tools/crn_prof.sh r05z_c3_bf16 > $O/r05z_c3prof.log 2>&1 || { echo "c3 trace failed"; exit 1; }
bash $R/tools/crn_prof.sh r05z_c3_fp8 --dtype fp8 >> $O/r05z_c3prof.log 2>&1 || { echo "c3 fp8 trace failed"; exit 1; }
for t in bf16 fp8; do
  python $R/tools/crn_kstats.py $O/prof_r05z_c3_$t > $O/r05z_c3_${t}_kernel_table.txt 2>&1 || exit 1
  head -8 $O/r05z_c3_${t}_kernel_table.txt
done
bash $R/tools/c5_pmc.sh r05z_c5pmc > $O/r05z_c5pmc.log 2>&1 || { echo "c5 pmc failed"; tail -5 $O/r05z_c5pmc.log; exit 1; }
echo "c5 pmc done"
bash $R/tools/crn_pmc.sh r05z_crnpmc > $O/r05z_crnpmc.log 2>&1 || { echo "crn pmc failed"; tail -5 $O/r05z_crnpmc.log; exit 1; }
echo "crn pmc done"
CRN_GEMM_XCD=8 bash $R/tools/crn_pmc.sh r05z_crnpmc_xcd8 > $O/r05z_crnpmc_xcd8.log 2>&1 || { echo "crn pmc xcd failed"; tail -5 $O/r05z_crnpmc_xcd8.log; exit 1; }
echo "crn pmc xcd8 done"
timeout -k 10 500 python $R/bench.py > $O/r05z_bench100.log 2>&1 || { echo "bench failed"; tail -20 $O/r05z_bench100.log; exit 1; }
tail -1 $O/r05z_bench100.log | head -c 400; echo
