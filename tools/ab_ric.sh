set -o pipefail
OUT=gpurun_out/ab1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ric_kkt.py tests/test_gpu_parity.py tests/test_path.py -x -q --timeout 300 -k "ric or config5 or horizons or fourier or Nh" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --horizon 40 --ekf > $OUT/b40.json 2> $OUT/b40.err || { echo "bench failed"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/b40.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['status_nan'], d['qp_converged_frac'], d['roofline']['achieved'])"
timeout -k 10 300 python tools/ric_phase_profile.py 4096 40 > $OUT/phase.txt 2>&1 && grep -v amdgpu.ids $OUT/phase.txt
