"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
symbol include/kite_nmpc/kite_nmpc.h declares, and its host-only entry points
(parameter file loader, default configuration, error reporting) behave like
the reference (kite.cpp:7-76, nmpf_node.cpp:30-69).  No compute call is made
here; without a gfx950 device kite_nmpc_create must fail loudly."""
import ctypes
import math
import os
import re
import subprocess

import numpy as np
import pytest

import openkite_amd as ok
from openkite_amd import nmpc
from oracle import ffi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "kite_nmpc",
                      "kite_nmpc.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kite_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = ok.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    # and the Python binding covers all of them
    assert set(names) <= set(nmpc._SIGNATURES)


def test_struct_layouts_match_header():
    assert ctypes.sizeof(ok.KiteParams) == 52 * 8
    assert ctypes.sizeof(ok.MpcDiagnostic) == 6 * 8
    # kite_nmpc_config: 8 int32 + 91 doubles + 2 int32 + 2 int32 + 51 doubles (API 3: Fourier path)
    assert ctypes.sizeof(ok.NmpcConfig) == 12 * 4 + (1 + 3 + 4 + 1 + 15 + 4 + 15 + 15 + 4 + 4 + 1 + 2 + 4 + 2 + 1 + 2 + 51) * 8
    assert ok.lib().kite_nmpc_api_version() == 7


@pytest.mark.parametrize("cname,py", [("kite_nmpc_config", "NmpcConfig"), ("kite_colloc_config", "CollocConfig")])
def test_config_layout_matches_c_compiler(tmp_path, cname, py):
    """sizeof / offsetof of the config structs from a C compiler == the ctypes mirrors."""
    S = getattr(ok.nmpc, py)
    src = tmp_path / "lay.c"
    fields = [f for f, _ in S._fields_]
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "kite_nmpc/kite_nmpc.h"\nint main(void){'
                   + f'printf("%zu\\n", sizeof({cname}));'
                   + "".join(f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields) + "return 0;}")
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ok.nmpc.REPO, "include"), "-o", str(exe), str(src)], check=True)
    out = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert out[0] == ctypes.sizeof(S)
    assert out[1:] == [getattr(S, f).offset for f in fields]


def test_load_properties_matches_yaml_and_oracle():
    p = ok.load_properties()
    np.testing.assert_array_equal(p.as_array(), ffi.load_params())
    assert p.mass == 0.044 and p.Lt == 2.81 and p.Ixz == -3.5e-5


def test_load_properties_missing_tether_arm_defaults_to_zero(tmp_path):
    """The shipped umx_radian.yaml lacks tether.rx/ry/rz."""
    src = open(ok.nmpc.DEFAULT_PARAMS).read()
    stripped = "\n".join(l for l in src.splitlines() if not re.match(r"\s+r[xyz]:", l))
    f = tmp_path / "noarm.yaml"
    f.write_text(stripped)
    p = ok.load_properties(str(f))
    assert (p.rx, p.ry, p.rz) == (0.0, 0.0, 0.0)


def test_load_properties_errors(tmp_path):
    with pytest.raises(ok.KiteNmpcError) as e:
        ok.load_properties(str(tmp_path / "does_not_exist.yaml"))
    assert e.value.code == nmpc.KITE_EIO
    src = open(ok.nmpc.DEFAULT_PARAMS).read().replace("    Cmq:", "    Cmq_typo:")
    f = tmp_path / "bad.yaml"
    f.write_text(src)
    with pytest.raises(ok.KiteNmpcError) as e:
        ok.load_properties(str(f))
    assert e.value.code == nmpc.KITE_EPARSE


def test_default_config_is_the_reference_node():
    c = ok.default_config()
    ref = ffi.node_config()
    assert (c.N, c.M, c.qp_iters, c.shift) == (20, 2, 16, 1)
    np.testing.assert_allclose(list(c.Q), ref["Q"]); np.testing.assert_allclose(list(c.R), ref["R"])
    assert c.W == ref["W"] and c.vref == 4.0 and c.dt == 0.05
    np.testing.assert_allclose(list(c.Sx), ref["Sx"]); np.testing.assert_allclose(list(c.Su), ref["Su"])
    np.testing.assert_allclose(list(c.lbu), ref["lbu"]); np.testing.assert_allclose(list(c.ubu), ref["ubu"])
    np.testing.assert_array_equal(list(c.lbx), ref["lbx"]); np.testing.assert_array_equal(list(c.ubx), ref["ubx"])
    np.testing.assert_allclose(list(c.path_q), ref["path_q"])
    assert c.path_radius == 2.65 and c.theta_flex == 0.78 and c.min_speed == 2.1


def test_strerror_codes():
    L = ok.lib()
    for code in range(0, -8, -1):
        assert L.kite_nmpc_strerror(code)
    assert L.kite_nmpc_strerror(-99) == b"unknown error"


def _gpu_present():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_create_fails_loudly_without_device_and_validates():
    p = ok.load_properties()
    bad = ok.default_config(N=0)
    with pytest.raises(ok.KiteNmpcError) as e:
        ok.BatchNMPC(p, bad, 4)
    assert e.value.code == nmpc.KITE_EINVAL
    for b in (0, -3):                      # empty / negative batch: rejected before any device work
        with pytest.raises(ok.KiteNmpcError) as e:
            ok.BatchNMPC(p, ok.default_config(), b)
        assert e.value.code == nmpc.KITE_EINVAL
    bad = ok.default_config(N=21)          # beyond the fused kernels' horizon
    with pytest.raises(ok.KiteNmpcError):
        ok.BatchNMPC(p, bad, 4)
    for i, lo, hi in ((13, -1.0, float("inf")), (14, -float("inf"), 3.0), (3, 1.0, -1.0), (5, float("nan"), 1.0)):
        bad = ok.default_config()          # finite theta/thetadot bounds (not enforced) or a bad box: refused
        bad.lbx[i], bad.ubx[i] = lo, hi
        with pytest.raises(ok.KiteNmpcError) as e:
            ok.BatchNMPC(p, bad, 4)
        assert e.value.code == nmpc.KITE_EINVAL, i
    if not _gpu_present():
        with pytest.raises(ok.KiteNmpcError) as e:
            ok.BatchNMPC(p, ok.default_config(), 4)
        assert e.value.code == nmpc.KITE_ENODEV


def test_two_wave_ric_hand_overs_are_ds_only():
    """The two-wave k_qp_ric raises its LDS counters without an lgkmcnt wait
    (qp_ric.inc, ric_publish): that relies on every LDS access of the kernel
    being a DS instruction, executed in issue order.  A flat (generic-address)
    load or store could reach LDS out of that order, so the built kernels must
    contain none."""
    import sys
    sys.path.insert(0, os.path.join(ok.nmpc.REPO, "tools"))
    from kernel_resources import code_objects
    cos = [co for triple, co in code_objects(nmpc.LIB_PATH) if "gfx950" in triple]
    assert cos
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not in this image")
    import tempfile
    kernels = []
    for co in cos:                                   # one code object per translation unit
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            asm = subprocess.run([objdump, "-d", "--no-show-raw-insn", f.name], check=True, capture_output=True,
                                 text=True).stdout
        kernels += re.split(r"\n(?=[0-9a-f]+ <)", asm)
    ric = [k for k in kernels if re.match(r"[0-9a-f]+ <_ZN4kite8k_qp_ric", k)]
    assert len(ric) >= 2
    for k in ric:
        assert "flat_" not in k, k.splitlines()[0]
