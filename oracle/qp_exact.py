"""Exact dense QP solver for the oracle (TEST INFRASTRUCTURE ONLY).

Solves   min 1/2 x'Px + q'x   s.t.   l <= A x <= u
with P positive semidefinite (positive definite on the null space of the
working set), by a textbook primal active-set method with exact dense KKT
solves, followed by a final direct solve of the optimal working set and a KKT
certificate.

Why an active-set method: the reference hands every subproblem to OSQP through
``ca.qpsol("solver", "osqp", ...)`` (``casadi/main.py:96,146``).  OSQP stops at
eps_abs = eps_rel = 1e-3 and the reference then rounds to 4 decimals
(``casadi/main.py:103,153``), so the reference's own answers are only
~1e-3 accurate.  Parity is therefore defined against the *exact* minimiser of
the same convex QP, which is unique (P is positive definite in the control
variables) and certified here by KKT residuals.  This algorithm is deliberately
different from the build's GPU solver (ADMM + active-set polish), so the two
agreeing is evidence about both.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this.
"""
from __future__ import annotations

import numpy as np


class QPError(RuntimeError):
    pass


def kkt_residuals(P, q, A, l, u, x, y):
    """Return (stationarity, primal infeasibility, dual sign/complementarity) maxima.

    Sign convention: P x + q + A' y = 0, y_i > 0 only at the upper bound,
    y_i < 0 only at the lower bound.
    """
    Ax = A @ x
    stat = np.max(np.abs(P @ x + q + A.T @ y)) if x.size else 0.0
    infeas = max(np.max(Ax - u, initial=0.0), np.max(l - Ax, initial=0.0))
    comp = 0.0
    for i in range(A.shape[0]):
        if y[i] > 0:
            comp = max(comp, y[i] * abs(u[i] - Ax[i]) if np.isfinite(u[i]) else abs(y[i]))
        elif y[i] < 0:
            comp = max(comp, -y[i] * abs(Ax[i] - l[i]) if np.isfinite(l[i]) else abs(y[i]))
    return float(stat), float(infeas), float(comp)


def solve(P, q, A, l, u, x0, tol=1e-12, max_iter=2000, W0=None):
    """Primal active-set QP.  ``x0`` must be feasible.  Returns (x, y, working_set).

    ``working_set`` is a list of (row, side) with side +1 (upper) / -1 (lower).
    """
    P = np.asarray(P, np.float64)
    q = np.asarray(q, np.float64)
    A = np.asarray(A, np.float64)
    n, m = q.size, A.shape[0]
    x = np.array(x0, np.float64, copy=True)
    scale = 1.0 + np.max(np.abs(np.concatenate([l[np.isfinite(l)], u[np.isfinite(u)], [0.0]])))
    feas_tol = 1e-12 * scale
    Ax = A @ x
    if np.any(Ax > u + 1e-9 * scale) or np.any(Ax < l - 1e-9 * scale):
        raise QPError("starting point infeasible")

    W: list[tuple[int, int]] = []
    row_norm = np.linalg.norm(A, axis=1)

    def independent(rows, cand):
        if not rows:
            return np.any(A[cand] != 0)
        M = A[rows + [cand]]
        return np.linalg.matrix_rank(M, tol=1e-10) == len(rows) + 1

    cand = W0 if W0 is not None else []
    if W0 is None:
        for i in range(m):
            if u[i] - Ax[i] <= feas_tol:
                cand.append((i, +1))
            elif Ax[i] - l[i] <= feas_tol:
                cand.append((i, -1))
    for (i, s) in cand:
        if len(W) < n and independent([r for r, _ in W], i):
            W.append((i, s))

    at_eqp_min = False
    degenerate = False      # the last step had length 0: use Bland's rule to avoid cycling
    for _ in range(max_iter):
        rows = [r for r, _ in W]
        k = len(rows)
        AW = A[rows] if k else np.zeros((0, n))
        g = P @ x + q
        K = np.zeros((n + k, n + k))
        K[:n, :n] = P
        K[:n, n:] = AW.T
        K[n:, :n] = AW
        rhs = np.concatenate([-g, np.zeros(k)])
        try:
            sol = np.linalg.solve(K, rhs)
        except np.linalg.LinAlgError as exc:
            raise QPError(f"singular KKT with |W|={k}") from exc
        p, lam = sol[:n], sol[n:]
        if at_eqp_min or np.max(np.abs(p), initial=0.0) <= 1e-13 * (1.0 + np.max(np.abs(x))):
            # stationary on the working set: check multiplier signs
            worst, wj = -1e-12 * (1.0 + np.max(np.abs(lam), initial=0.0)), -1
            thr = worst
            for j, (r, s) in enumerate(W):
                v = lam[j] * s
                if degenerate:
                    # Bland: the wrong-signed row of lowest index
                    if v < thr and (wj < 0 or r < W[wj][0]):
                        wj = j
                elif v < worst:
                    worst, wj = v, j
            if wj < 0:
                # optimal working set: re-solve it directly for full accuracy
                x, y = _solve_eqp(P, q, A, l, u, W)
                return x, y, W
            W.pop(wj)
            at_eqp_min = False
            continue
        Ap = A @ p
        Ax = A @ x
        alpha, block = 1.0, None
        inW = set(rows)
        pn = np.linalg.norm(p)
        for i in range(m):
            # rows with A_i p ~ 0 (relative) do not move along p; a row that is
            # linearly dependent on the working set is one of them (degenerate vertex)
            if i in inW or abs(Ap[i]) <= 1e-10 * row_norm[i] * pn:
                continue
            if Ap[i] > 0 and np.isfinite(u[i]):
                t = (u[i] - Ax[i]) / Ap[i]
                if t < alpha and independent(rows, i):
                    alpha, block = max(t, 0.0), (i, +1)
            elif Ap[i] < 0 and np.isfinite(l[i]):
                t = (l[i] - Ax[i]) / Ap[i]
                if t < alpha and independent(rows, i):
                    alpha, block = max(t, 0.0), (i, -1)
        x = x + alpha * p
        if block is not None:
            W.append(block)
        degenerate = block is not None and alpha <= 0.0
        at_eqp_min = block is None    # full step: x minimises the EQP of W
    raise QPError("active-set iteration limit")


def _solve_eqp(P, q, A, l, u, W):
    n = q.size
    rows = [r for r, _ in W]
    k = len(rows)
    AW = A[rows] if k else np.zeros((0, n))
    bW = np.array([u[r] if s > 0 else l[r] for r, s in W])
    K = np.zeros((n + k, n + k))
    K[:n, :n] = P
    K[:n, n:] = AW.T
    K[n:, :n] = AW
    rhs = np.concatenate([-q, bW])
    sol = np.linalg.solve(K, rhs)
    # one step of iterative refinement
    sol += np.linalg.solve(K, np.concatenate([-q, bW]) - K @ sol)
    x, lam = sol[:n], sol[n:]
    y = np.zeros(A.shape[0])
    for j, r in enumerate(rows):
        y[r] = lam[j]
    return x, y
