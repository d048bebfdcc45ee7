// flopcount.cpp -- op-count the kite RHS once (host build of the device
// template in openkite_amd/csrc/kite_model.hpp with a counting scalar) and
// print the algorithmic FLOP constants used by bench.py's roofline
// (FMA = 2 flops, transcendental / sqrt / reciprocal = 1).
//
//   F_f : primal RHS evaluation
//   F_t : one forward-mode tangent direction through the same RHS
//         (a+b: 1, a*b: 3, a*c: 1, 1/a: 3, sqrt: 2, exp: 1, asin: 1, atan2: 4)
//
// Build & run:  hipcc -O1 -std=c++17 -o /tmp/flopcount tools/flopcount.cpp && /tmp/flopcount
#include <cstdio>

#include "../openkite_amd/csrc/kite_model.hpp"

namespace {
long g_primal = 0, g_tangent = 0;

struct Op {
    double v = 0;
    bool act = false;
    Op() = default;
    Op(double a) : v(a), act(false) {}
    Op(double a, bool b) : v(a), act(b) {}
};
Op operator+(Op a, Op b) { g_primal++; if (a.act && b.act) g_tangent += 1; return Op(a.v + b.v, a.act || b.act); }
Op operator-(Op a, Op b) { g_primal++; if (a.act && b.act) g_tangent += 1; return Op(a.v - b.v, a.act || b.act); }
Op operator-(Op a) { return Op(-a.v, a.act); }
Op operator*(Op a, Op b) {
    g_primal++;
    if (a.act && b.act) g_tangent += 3; else if (a.act || b.act) g_tangent += 1;
    return Op(a.v * b.v, a.act || b.act);
}
Op operator+(Op a, double b) { g_primal++; return Op(a.v + b, a.act); }
Op operator+(double b, Op a) { g_primal++; return Op(a.v + b, a.act); }
Op operator-(Op a, double b) { g_primal++; return Op(a.v - b, a.act); }
Op operator-(double b, Op a) { g_primal++; return Op(b - a.v, a.act); }
Op operator*(Op a, double b) { g_primal++; if (a.act) g_tangent += 1; return Op(a.v * b, a.act); }
Op operator*(double b, Op a) { return a * b; }
Op rcp(Op a) { g_primal++; if (a.act) g_tangent += 3; return Op(1.0 / a.v, a.act); }
Op dsqrt(Op a) { g_primal++; if (a.act) g_tangent += 2; return Op(std::sqrt(a.v), a.act); }
Op dexp(Op a) { g_primal++; if (a.act) g_tangent += 1; return Op(std::exp(a.v), a.act); }
Op dasin(Op x, Op) { g_primal++; if (x.act) g_tangent += 1; return Op(std::asin(x.v), x.act); }
Op datan2(Op y, Op x, Op) { g_primal++; if (x.act || y.act) g_tangent += 4; return Op(std::atan2(y.v, x.v), x.act || y.act); }
}  // namespace

int main() {
    kite::ModelConst P{};
    P.inv_mass = 1; P.S = 1; P.b = 1; P.c = 1; P.half_rho = 1;
    P.rx = P.ry = P.rz = 0.0;    // umx_radian: no tether arm -- still counted (constants)
    Op x[13], u[3], f[13];
    const double xv[13] = {4.4, 0.44, 1.73, 0.81, -1.73, -1.53, -0.46, -2.68, 0.64, -0.0289, 0.1587, 0.4304, 0.8881};
    for (int i = 0; i < 13; ++i) x[i] = Op(xv[i], true);
    for (int i = 0; i < 3; ++i) u[i] = Op(0.1, true);
    kite::kite_rhs<Op>(P, x, u, f);
    std::printf("{\"F_f\": %ld, \"F_t\": %ld}\n", g_primal, g_tangent);
    return 0;
}
