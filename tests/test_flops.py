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
    assert flops.rk4_sens_per_interval(2) == 82080
    assert abs(flops.rk4_sens(20, 2) / 1e6 - 1.64) < 0.01
    assert abs(flops.condense(20) / 1e6 - 0.78) < 0.01
    assert abs(flops.qp_per_iteration(20) / 1e6 - 0.383) < 0.001
    d = flops.rti(20, 2, 10.687)
    assert abs(d["total"] - (d["rk4_sens"] + d["condense"] + d["qp"])) < 1e-6
