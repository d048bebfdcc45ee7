import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libkite_nmpc.so")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kite_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kp():
    from oracle import ffi
    return ffi.load_params()


@pytest.fixture(scope="session")
def cfgv():
    from oracle import ffi
    return ffi.cfg_vector(ffi.node_config())
