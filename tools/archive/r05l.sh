#!/bin/bash
# round 5 batch l: synthesis inverse FFT on the packed core (AEC_FFT_PK_INV) and the pre-scaled
# synthesis window (AEC_SYN_HANN_PRE, must be bit-identical): bit identity, C2 A/B, gru tick
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
AB=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p $O
for lib in tree $AB/hpre.so $AB/pkinv.so $AB/pkinv_hpre.so; do
  if [ "$lib" = tree ]; then unset AEC_HIP_LIB; else export AEC_HIP_LIB=$lib; fi
  echo "$(basename $lib): $(timeout -k 10 120 python $R/tools/lib_bitcmp.py 2>&1 | grep sha1)" >> $O/r05l_bitcmp.log || { echo "bitcmp failed"; exit 1; }
done
unset AEC_HIP_LIB
cat $O/r05l_bitcmp.log
bash $R/tools/libs_ab.sh 3 tree acoustic-echo-cancellation_amd/aec_amd/ab/hpre.so acoustic-echo-cancellation_amd/aec_amd/ab/pkinv.so acoustic-echo-cancellation_amd/aec_amd/ab/pkinv_hpre.so > $O/r05l_ab.log 2>&1 || { echo "ab failed"; tail $O/r05l_ab.log; exit 1; }
cat $O/r05l_ab.log
AEC_HIP_LIB=$AB/tick_pkinv.so timeout -k 10 120 python $R/tools/gru_tick_prof.py > $O/r05l_gru_tick_pkinv.txt 2>&1 || { echo "gru tick failed"; tail $O/r05l_gru_tick_pkinv.txt; exit 1; }
head -14 $O/r05l_gru_tick_pkinv.txt
for i in 1 2; do for f in 2 3; do
  timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --inflight $f > $O/r05l_inflight_${f}_$i.log 2>&1 || { echo "inflight $f failed"; exit 1; }
  echo "inflight $f #$i: $(tail -1 $O/r05l_inflight_${f}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done
