"""openkite_amd -- MI355X-native batched NMPC (RTI) for the openKITE kite.

The product is libkite_nmpc.so (HIP kernels for gfx950 behind the C ABI in
include/kite_nmpc/kite_nmpc.h); this package is its Python host side.
"""
from .nmpc import (BatchNMPC, CollocConfig, KiteEKF, KiteNMPF, KiteNmpcError, KiteParams, NmpcConfig, MpcDiagnostic,  # noqa: F401
                   colloc_default_config, default_config, ekf_default_covariances, load_properties, lib, LIB_PATH, DIAG_FIELDS,
                   path_eval, resolve_qp_kernel)

__version__ = "0.1.0"
