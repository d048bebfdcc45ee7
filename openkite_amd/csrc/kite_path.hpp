// kite_path.hpp -- the unrotated path curve p(theta) and dp/dtheta, host and
// device.  The reference node builds P(theta) = vec(q^-1 (x) [0, p] (x) q) from
// the circle p = [R cos, R sin, alt] (nmpf_node.cpp:30-40); KiteNMPF itself
// takes any closed path (kiteNMPF.h:14), represented here by a truncated
// Fourier series per axis (kite_nmpc_config.path_harmonics / path_fourier).
// The callers apply the rotation.
#pragma once
#include <hip/hip_runtime.h>

#define KITE_PATH_HMAX 8
#define KITE_PATH_NC (2 * KITE_PATH_HMAX + 1)

namespace kite {

// c = cos(theta), s = sin(theta).  K = 0: the circle (R, alt), else
// p_a = F[a][0] + sum_{k <= K} F[a][2k-1] cos k theta + F[a][2k] sin k theta with
// (cos, sin)(k theta) from the angle-addition recurrence.  The harmonic loop is
// unrolled to KITE_PATH_HMAX so every coefficient index is a compile-time
// constant (a runtime index into a by-value kernel argument forces a private
// copy of the argument).
__host__ __device__ inline void path_curve(int K, double R, double alt, const double (*F)[KITE_PATH_NC],
                                           double c, double s, double p[3], double dp[3]) {
    if (K == 0) {
        p[0] = R * c; p[1] = R * s; p[2] = alt;
        dp[0] = -R * s; dp[1] = R * c; dp[2] = 0.0;
        return;
    }
    for (int a = 0; a < 3; ++a) { p[a] = F[a][0]; dp[a] = 0.0; }
    double ck = c, sk = s;
#pragma unroll
    for (int k = 1; k <= KITE_PATH_HMAX; ++k) {
        if (k > K) break;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double ak = F[a][2 * k - 1], bk = F[a][2 * k];
            p[a] += ak * ck + bk * sk;
            dp[a] += k * (bk * ck - ak * sk);
        }
        const double cn = ck * c - sk * s, sn = sk * c + ck * s;
        ck = cn; sk = sn;
    }
}

}  // namespace kite
