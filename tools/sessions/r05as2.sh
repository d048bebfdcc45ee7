#!/bin/bash
# Round-5 session AS2: k_qp_tiled init with only the control scalings picked by
# selects (no lane-indexed kernel-argument loads; the other loads as at HEAD) vs
# HEAD -- outputs, GPU suite, kernel traces, alternating A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05as2; mkdir -p $OUT
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/head.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 512 30 20 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/init.so timeout -k 10 200 python tools/ab_outputs.py $OUT/new.npz $OUT/base.npz 512 30 20 > $OUT/out_new.log 2>&1 || { echo "new outputs failed"; exit 1; }
echo "512 kites x 30 steps vs HEAD: $(tail -1 $OUT/out_new.log)"
rm -f $OUT/*.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
bash tools/trace_ab.sh r05as2 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/init.so 2>&1 | grep -E "==|k_qp_tiled" || { echo "trace failed"; exit 1; }
bash tools/ab_alt.sh r05as2 3 openkite_amd/lib/ab/head.so openkite_amd/lib/ab/init.so || { echo "ab failed"; exit 1; }
echo done
