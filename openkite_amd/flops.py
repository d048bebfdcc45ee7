"""Algorithmic FLOP model of one RTI step (DESIGN.md 'Roofline').

Convention: FMA = 2 flops, add/mul = 1, sqrt / reciprocal / transcendental = 1.
F_F and F_T are op counts of the device RHS template (openkite_amd/csrc/
kite_model.hpp), produced by tools/flopcount.cpp and frozen here
(tests/test_flops.py re-derives them with tools/flopcount.cpp).

Per instance:
  rk4_sens : N * M * 4 * (F_F + NDIR*F_T + 4*NK*(NDIR+1))
             value + NDIR = 16 forward tangents (13 kite states + 3 kite
             controls) through each RHS, plus the RK4 stage updates of
             value and tangents.  The primal is counted ONCE per stage (the
             kernel recomputes it on each of the 16 lanes: that redundancy is
             an implementation cost, not algorithmic work).
  condense : G-column propagation  sum_k (3k+1) * 2*NK^2  (+ defects)
             + H_ext = W^T W on the (4N+3) x (n+1) residual Jacobian,
               symmetric half: rows * (n+1)(n+2)/2 * 2
  qp       : per interior-point iteration, n = 4N+2, m = N:
             H w 2n^2, C w and C^T z 4mn, normal matrix n(n+1)/2 * (2m+1),
             Cholesky n^3/3, two solves 2 * (2n^2 + 4mn)
"""
from __future__ import annotations

F_F = 320      # primal RHS (tools/flopcount.cpp)
F_T = 566      # one tangent direction through the RHS
NK = 13
NDIR = 16


def rk4_sens_per_interval(M: int) -> float:
    return M * 4 * (F_F + NDIR * F_T + 4 * NK * (NDIR + 1))


def rk4_sens(N: int, M: int) -> float:
    return N * rk4_sens_per_interval(M)


def condense(N: int) -> float:
    n = 4 * N + 2
    prop = sum((3 * k + 1) * 2 * NK * NK + NK for k in range(N))
    rows = 4 * N + 3
    syrk = rows * (n + 1) * (n + 2) / 2 * 2
    return prop + syrk


def qp_per_iteration(N: int) -> float:
    n, m = 4 * N + 2, N
    return 2 * n * n + 4 * m * n + n * (n + 1) / 2 * (2 * m + 1) + n ** 3 / 3 + 2 * (2 * n * n + 4 * m * n)


def qp(N: int, iterations: float) -> float:
    # the final residual evaluation is one more H w / C w pass
    n, m = 4 * N + 2, N
    return iterations * qp_per_iteration(N) + 2 * n * n + 4 * m * n


def rti(N: int, M: int, mean_qp_iterations: float) -> dict:
    d = dict(rk4_sens=rk4_sens(N, M), condense=condense(N), qp=qp(N, mean_qp_iterations))
    d["total"] = sum(d.values())
    return d
