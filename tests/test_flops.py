"""The FLOP model behind bench.py's roofline (openkite_amd/flops.py): the frozen
RHS op counts are re-derived from the device template by tools/flopcount.cpp
(hipcc host build with a counting scalar), and the per-kernel formulas give
the per-instance figures DESIGN.md quotes."""
import json
import os
import subprocess

import pytest

from openkite_amd import flops

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rhs_op_counts_rederived(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not present")
    exe = str(tmp_path / "flopcount")
    subprocess.run([hipcc, "-O1", "-std=c++17", "-o", exe, os.path.join(REPO, "tools", "flopcount.cpp")],
                   check=True, capture_output=True)
    out = json.loads(subprocess.run([exe], check=True, capture_output=True, text=True).stdout)
    assert out == {"F_f": flops.F_F, "F_t": flops.F_T}


def test_per_instance_figures():
    # N = 20, M = 2
    assert flops.rk4_sens_per_interval(2) == 79512
    assert abs(flops.rk4_sens(20, 2) / 1e6 - 1.59) < 0.01
    assert abs(flops.condense_dense(20) / 1e6 - 0.78) < 0.01
    assert abs(flops.condense(20) / 1e6 - 0.401) < 0.001
    assert abs(flops.qp_per_iteration_dense(20) / 1e6 - 0.383) < 0.001
    assert abs(flops.qp_per_iteration(20) / 1e6 - 0.2616) < 0.0001
    assert abs(flops.qp_per_iteration_survey(20) - 345165.33) < 0.01    # 345 k
    d = flops.rti(20, 2, 10.687)
    assert abs(d["total"] - (d["rk4_sens"] + d["condense"] + d["qp"])) < 1e-6


def test_causal_counts_match_structure():
    """The causal counts are the dense formulas evaluated on the structural
    nonzeros: C (row k: 3k kite-control columns) and the residual Jacobian
    (node k: 4k + 3 columns) built explicitly for small N."""
    import numpy as np
    for N in (2, 5, 20):
        n = 4 * N + 2
        C = np.zeros((N, n), bool)
        for k in range(1, N + 1):
            C[k - 1, :3 * k] = True                  # GPU column order: kite controls first
        assert C.sum() == flops.c_nnz(N)
        outer = sum(int(r.sum()) * (int(r.sum()) + 1) for r in C)   # symmetric half x 2 flops
        normal = n * (n + 1) / 2 + outer
        expect = 2 * n * n + 4 * C.sum() + normal + n ** 3 / 3 + 2 * (2 * n * n + 4 * C.sum())
        assert abs(flops.qp_per_iteration(N) - expect) < 1e-6
        cols = [4 * k + 3 for k in range(N + 1)]
        syrk = sum((4 if k < N else 3) * c * (c + 1) for k, c in enumerate(cols))
        assert abs(flops.condense(N) - flops._propagation(N) - syrk) < 1e-6
        assert flops.qp_per_iteration(N) < flops.qp_per_iteration_dense(N)
