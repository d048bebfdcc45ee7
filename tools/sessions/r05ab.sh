#!/bin/bash
# Round-5 session AB: k_condense20 with branch-free C-row stores (the wait for
# the next node's [A_k | B_k] loads no longer covers them) vs HEAD -- bitwise
# outputs at N = 20, GPU suite, kernel traces, alternating A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ab; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base20.npz - 256 60 20 > $OUT/out_base20.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base20.log; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/cstore.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new20.npz $OUT/base20.npz 256 60 20 > $OUT/out_new20.log 2>&1 || { echo "new outputs failed"; cat $OUT/out_new20.log; exit 1; }
tail -1 $OUT/out_new20.log
rm -f $OUT/*.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
bash tools/trace_ab.sh r05ab openkite_amd/lib/ab/head.so openkite_amd/lib/ab/cstore.so 2>&1 | grep -v rocclr || { echo "trace failed"; exit 1; }
bash tools/ab_alt.sh r05ab 3 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/cstore.so || { echo "ab failed"; exit 1; }
echo done
