// ric_kernels.hip -- the multiple-shooting QP of the RTI step on gfx950
// (qp_ric.inc): one wavefront per kite, Mehrotra interior point with a
// Riccati recursion on fp64 MFMA tiles.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kite_model.hpp"
#include "rti_kernels.hpp"
#include "rti_device.hpp"

namespace kite {
#include "qp_ric.inc"
}  // namespace kite
