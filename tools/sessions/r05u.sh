#!/bin/bash
# Round-5 session U: Cholesky multipliers broadcast before the pivot scaling
# (chol_mult) -- bitwise outputs at N = 20 and 40, alternating A/B at config 3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05u; mkdir -p $OUT
for N in 20 40; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/base.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base$N.npz - 512 5 $N > $OUT/out_base$N.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base$N.log; exit 1; }
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/chol_mu.so timeout -k 10 200 python tools/ab_outputs.py $OUT/mu$N.npz $OUT/base$N.npz 512 5 $N > $OUT/out_mu$N.log 2>&1 || { echo "mu outputs failed"; cat $OUT/out_mu$N.log; exit 1; }
  tail -1 $OUT/out_mu$N.log
done
bash tools/ab_alt.sh r05u 3 openkite_amd/lib/ab/base.so openkite_amd/lib/ab/chol_mu.so || { echo "ab failed"; exit 1; }
echo done
