#!/bin/bash
# Round-5 session L: k_condense20 with the propagation on v_fmac_f64_dpp
# (row_newbcast from registers, no LDS broadcast of A_k) against the LDS form:
# bitwise outputs, the condensing / RTI GPU tests on the variant, A/B bench.
set -o pipefail
OUT=gpurun_out/r05l; mkdir -p $OUT
export TMPDIR=/tmp
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/base.so timeout -k 10 200 python tools/ab_outputs.py $OUT/base.npz - 512 6 > $OUT/out_base.log 2>&1 || { echo "base outputs failed"; cat $OUT/out_base.log; exit 1; }
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/cd_dpp.so timeout -k 10 200 python tools/ab_outputs.py $OUT/dpp.npz $OUT/base.npz 512 6 > $OUT/out_dpp.log 2>&1 || { echo "dpp outputs failed"; cat $OUT/out_dpp.log; exit 1; }
tail -3 $OUT/out_dpp.log
KITE_NMPC_LIB=$PWD/openkite_amd/lib/ab/cd_dpp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "condens or rti or config or long or full_batch or ragged or qp_kernels" > $OUT/pytest_dpp.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_dpp.log; exit 1; }
tail -2 $OUT/pytest_dpp.log
bash tools/ab_alt.sh r05l 3 openkite_amd/lib/ab/base.so openkite_amd/lib/ab/cd_dpp.so || { echo "ab failed"; exit 1; }
echo done
