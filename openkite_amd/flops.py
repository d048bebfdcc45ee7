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
  qp_ric   : the multiple-shooting QP (qp_kernel 3, no condensing), per
             interior-point iteration and stage (nx = 15 states, nu = 4
             controls, the kite block Z = [A | B] is 13 x 16):
               factorisation  P Z for the kite and theta rows   2*15*13*16
                              Z' (P Z), symmetric half            16*17/2*13*2
                              theta border (W' P_bb W, M_xi,beta) 3*16*2 + 40
                              4x4 Cholesky + L^-1 M_ux            30 + 15*16
                              rank-4 update, symmetric half       15*16/2*4*2
               two solves     backward Z'p 13*16*2 + S's 15*4*2 + L^-1 g 16
                              forward  S x 15*4*2 + L^-T 16 + Z xi 13*16*2
               adjoint        Z' lambda 13*16*2 (stationarity test)
               elementwise    R_ROW flops per bound row: residual, Sigma and
                              rhs, two step directions, two ratio tests,
                              mu_aff, update (counted from qp_ric.inc)
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


# ---- multiple-shooting QP (qp_kernel 3, openkite_amd/csrc/qp_ric.inc) --------
RIC_FACT = 2 * 15 * 13 * 16 + 16 * 17 // 2 * 13 * 2 + (3 * 16 * 2 + 40) + (30 + 15 * 16) + 15 * 16 // 2 * 4 * 2
RIC_SOLVE = (13 * 16 * 2 + 15 * 4 * 2 + 16) + (15 * 4 * 2 + 16 + 13 * 16 * 2)
RIC_ADJ = 13 * 16 * 2
R_ROW = 80           # per bound row and iteration, each quantity counted once: residual 8, Sigma + rhs 16,
                     # affine direction 12 + ratio 4 + mu_aff 6, corrector rhs 10, direction 12 + ratio 4, update 8
ROWS_PER_STAGE = 23  # node configuration: 8 control rows + 15 state rows (nmpf_node.cpp:45-63)


def qp_ric_per_iteration(N: int, rows_per_stage: int = ROWS_PER_STAGE) -> float:
    return N * (RIC_FACT + 2 * RIC_SOLVE + RIC_ADJ) + (N + 1) * rows_per_stage * R_ROW


def qp_ric(N: int, iterations: float) -> float:
    # start: forward simulation (Z xi per stage); final residual: one adjoint sweep
    return iterations * qp_ric_per_iteration(N) + N * (13 * 16 * 2 + RIC_ADJ)


def rti_ric(N: int, M: int, mean_qp_iterations: float) -> dict:
    d = dict(rk4_sens=rk4_sens(N, M), condense=0.0, qp=qp_ric(N, mean_qp_iterations))
    d["total"] = sum(d.values())
    return d
