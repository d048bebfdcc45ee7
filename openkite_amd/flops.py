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
             + H_ext = W^T W, causal: the residual rows of node k (4, the
               Mayer node 3) reach only the c_k = 4k + 3 columns of the
               controls of intervals < k, theta0, thetadot0 and the affine
               column, so node k adds rows_k * c_k (c_k + 1) / 2 * 2
               (condense_dense: the dense (4N+3) x (n+1) Jacobian,
               rows * (n+1)(n+2)/2 * 2)
  qp       : per interior-point iteration, n = 4N+2, m = N vx rows; C is
             causal: the vx row of node k reaches only the 3k kite controls
             of intervals < k, nnz(C) = 3N(N+1)/2 (630 of m n = 1640 at N = 20):
             H w 2n^2, C w and C^T z 4 nnz(C), normal matrix H + C^T Sigma C
             n(n+1)/2 + sum_k 3k(3k+1) (symmetric half of each row's outer
             product), Cholesky n^3/3, two solves 2 * (2n^2 + 4 nnz(C)).
             Two other counts are kept beside it (qp_models): the dense count
             (C as a dense m x n matrix: 4mn and n(n+1)/2 (2m+1)) and
             SURVEY.md 8(d)'s F_qp = n^3/3 + 4 n^2 + m n^2 per iteration.
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

F_F = 303      # primal RHS (tools/flopcount.cpp)
F_T = 547      # one tangent direction through the RHS
NK = 13
NDIR = 16


def rk4_sens_per_interval(M: int) -> float:
    return M * 4 * (F_F + NDIR * F_T + 4 * NK * (NDIR + 1))


def rk4_sens(N: int, M: int) -> float:
    return N * rk4_sens_per_interval(M)


def _propagation(N: int) -> float:
    return sum((3 * k + 1) * 2 * NK * NK + NK for k in range(N))


def condense(N: int) -> float:
    syrk = sum((4 if k < N else 3) * (4 * k + 3) * (4 * k + 4) for k in range(N + 1))
    return _propagation(N) + syrk


def condense_dense(N: int) -> float:
    n = 4 * N + 2
    rows = 4 * N + 3
    return _propagation(N) + rows * (n + 1) * (n + 2) / 2 * 2


def c_nnz(N: int) -> int:
    """Structural nonzeros of the condensed vx rows C (row k: 3k kite controls)."""
    return 3 * N * (N + 1) // 2


def qp_per_iteration(N: int) -> float:
    n, c = 4 * N + 2, c_nnz(N)
    normal = n * (n + 1) / 2 + sum(3 * k * (3 * k + 1) for k in range(1, N + 1))
    return 2 * n * n + 4 * c + normal + n ** 3 / 3 + 2 * (2 * n * n + 4 * c)


def qp_per_iteration_dense(N: int) -> float:
    n, m = 4 * N + 2, N
    return 2 * n * n + 4 * m * n + n * (n + 1) / 2 * (2 * m + 1) + n ** 3 / 3 + 2 * (2 * n * n + 4 * m * n)


def qp_per_iteration_survey(N: int) -> float:
    """F_qp / K = n^3/3 + 4 n^2 + n_c n^2 (n_c = N rows)."""
    n = 4 * N + 2
    return n ** 3 / 3 + 4 * n * n + N * n * n


def qp_residual(N: int) -> float:
    """One exact residual evaluation: H w and C w, C^T z (causal C)."""
    n = 4 * N + 2
    return 2 * n * n + 4 * c_nnz(N)


def qp(N: int, iterations: float, recursive: bool = False) -> float:
    """Per instance.  The final residual evaluation is one more H w / C w
    pass.  recursive (k_qp_tiled: recursive residuals above 1e-6):
    only the residual evaluations that are certainly exact are counted -- the
    first iteration's and the final one -- a lower bound (the oracle's closed
    loop evaluates 29 % of them exactly), so the roofline is not overstated."""
    if recursive:
        return iterations * (qp_per_iteration(N) - qp_residual(N)) + 2 * qp_residual(N)
    return iterations * qp_per_iteration(N) + qp_residual(N)


def qp_models(N: int, iterations: float, recursive: bool = False) -> dict:
    """The condensed QP's flops per instance under the three counts: causal
    (`qp`, what bench.py's roofline uses), dense C, and SURVEY 8(d)'s F_qp."""
    n = 4 * N + 2
    return dict(causal=qp(N, iterations, recursive),
                dense=iterations * qp_per_iteration_dense(N) + 2 * n * n + 4 * N * n,
                survey=iterations * qp_per_iteration_survey(N))


def rti(N: int, M: int, mean_qp_iterations: float, recursive: bool = False) -> dict:
    d = dict(rk4_sens=rk4_sens(N, M), condense=condense(N), qp=qp(N, mean_qp_iterations, recursive))
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
