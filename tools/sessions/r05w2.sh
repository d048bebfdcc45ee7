#!/bin/bash
# Round-5 session W2: bitwise outputs of the prologue split vs HEAD over 60
# closed-loop steps (N = 20 and 40), NaN-aware comparison.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05w; mkdir -p $OUT
for N in 20 40; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/base.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base$N.npz - 256 60 $N > $OUT/out_base$N.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base$N.log; exit 1; }
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/light.so timeout -k 10 200 python tools/ab_outputs.py $OUT/light$N.npz $OUT/base$N.npz 256 60 $N > $OUT/out_light$N.log 2>&1 || { echo "light outputs failed"; cat $OUT/out_light$N.log; exit 1; }
  tail -1 $OUT/out_light$N.log
  rm -f $OUT/*.npz
done
echo done
