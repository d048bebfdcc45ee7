#!/bin/bash
# Round-5 session R: k_qp_ric with the forward sweep's column gather on
# permlane swaps instead of ds_bpermute -- bitwise outputs at N = 40 and an
# alternating config-5 A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05r; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/base.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 256 5 40 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base.log; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/ric_perm.so timeout -k 10 200 python tools/ab_outputs.py $OUT/perm.npz $OUT/base.npz 256 5 40 > $OUT/out_perm.log 2>&1 || { echo "perm outputs failed"; cat $OUT/out_perm.log; exit 1; }
tail -1 $OUT/out_perm.log
bash tools/ab_alt.sh r05r 3 openkite_amd/lib/ab/base.so openkite_amd/lib/ab/ric_perm.so -- --horizon 40 --ekf || { echo "ab failed"; exit 1; }
echo done
