#!/bin/bash
# Round-5 session F: k_condense20 with scalar (SGPR) loads of A_k vs the LDS-staged base:
# bitwise outputs, condensing parity tests, alternating bench A/B.
set -o pipefail
OUT=gpurun_out/r05f; mkdir -p $OUT
export TMPDIR=/tmp
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/base.so timeout -k 10 120 python tools/ab_outputs.py $OUT/base.npz > $OUT/out_base.log 2>&1 || { echo "base out failed"; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/cd_scalar.so timeout -k 10 120 python tools/ab_outputs.py $OUT/cd.npz $OUT/base.npz > $OUT/out_cd.log 2>&1 || { echo "cd out failed"; exit 1; }
cat $OUT/out_cd.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "condensed or rti_steps or config3" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 900 bash tools/ab_alt.sh r05f 3 openkite_amd/lib/ab/base.so openkite_amd/lib/ab/cd_scalar.so || { echo "ab failed"; exit 1; }
echo done
