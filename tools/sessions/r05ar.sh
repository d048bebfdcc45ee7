#!/bin/bash
# Round-5 session AR: the QP dispatch order computed by an extra block of the
# warm prologue (k_qp_order's launch gone on warm steps; the cold list emptied
# by the sensitivity kernel) vs HEAD -- outputs, GPU suite, traces, A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ar; mkdir -p $OUT
for N in 20 40; do
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base$N.npz - 256 40 $N > $OUT/out_base$N.log 2>&1 || { echo "base outputs failed"; exit 1; }
  KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/merge.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new$N.npz $OUT/base$N.npz 256 40 $N > $OUT/out_new$N.log 2>&1 || { echo "new outputs failed"; exit 1; }
  echo "N=$N: $(tail -1 $OUT/out_new$N.log)"
  rm -f $OUT/*.npz
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
bash tools/trace_ab.sh r05ar openkite_amd/lib/ab/head.so openkite_amd/lib/ab/merge.so 2>&1 | grep -E "==|k_prologue|k_qp_order|k_rk4" || { echo "trace failed"; exit 1; }
bash tools/ab_alt.sh r05ar 3 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/merge.so || { echo "ab failed"; exit 1; }
echo done
