#!/bin/bash
# A/B of two builds of the library on config 5 (N = 40 + EKF): variant A =
# openkite_amd/lib/libkite_nmpc_a.so, variant B = the default library, plus the
# multiple-shooting parity tests on B.   Usage (GPU box): bash tools/ab2_ric.sh
set -o pipefail
OUT=gpurun_out/ab2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ric_kkt.py tests/test_gpu_parity.py tests/test_path.py -x -q --timeout 300 -k "ric or config5 or horizons or fourier or Nh" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in a b; do
  if [ $v = a ]; then export KITE_NMPC_LIB=$PWD/openkite_amd/lib/libkite_nmpc_a.so; else unset KITE_NMPC_LIB; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --horizon 40 --ekf > $OUT/b40_$v.json 2> $OUT/b40_$v.err || { echo "bench $v failed"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b40_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['kernel_ms_per_step']['qp'], d['status_nan'], d['qp_converged_frac'])"
done
