"""Exact dense QP solver for the oracle (TEST INFRASTRUCTURE ONLY).

Solves   min 1/2 x'Px + q'x   s.t.   l <= A x <= u
with P positive semidefinite, by a textbook null-space primal active-set method with exact
dense linear algebra, followed by a direct solve of the final working set and a complete KKT
certificate.  ``solve`` never returns an answer that fails the certificate: it raises
:class:`QPError` instead.

Why an active-set method: the reference hands every subproblem to OSQP through
``ca.qpsol("solver", "osqp", ...)`` (``casadi/main.py:96,146``).  OSQP stops at
eps_abs = eps_rel = 1e-3 and the reference then rounds to 4 decimals
(``casadi/main.py:103,153``), so the reference's own answers are only
~1e-3 accurate.  Parity is therefore defined against the *exact* minimiser of
the same convex QP, which is unique (P is positive definite in the control
variables) and certified here by KKT residuals.  This algorithm is deliberately
different from the build's GPU solver (a dual active set on the hinge form), so the two
agreeing is evidence about both.

The method (Nocedal & Wright, Algorithm 16.3, null-space form, for a positive SEMIdefinite P):
  * the working set W is kept linearly independent: the null-space basis Z of A_W comes from a
    complete QR of the row-normalised A_W', and a row enters W only as the blocking row of a
    step p with A_W p = 0 and |a_i'p| above rounding, so it is never in span(A_W);
  * the step is the minimiser of the quadratic on x + null(A_W) when Z'PZ is positive
    definite along Z'g, and a descent ray of zero curvature otherwise (the pair QP's slack
    variables: a slack with neither of its rows in W), of unbounded length;
  * every row outside W enters the ratio test (round 4's solver skipped rows it judged
    dependent on W and could leave the feasible set);
  * at a stationary point the multipliers come from A_W'y = -g; the most negative is dropped
    (Bland's rule -- lowest row index -- after a step of length zero, against cycling on
    degenerate vertices);
  * the optimal working set is re-solved directly (one refinement step), and the answer is
    certified: stationarity, feasibility of EVERY row, dual signs and complementarity, all at
    1e-9 relative (:func:`certify`).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this.
"""
from __future__ import annotations

import numpy as np

CERT_TOL = 1e-9


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


def certify(P, q, A, l, u, x, y, tol=CERT_TOL):
    """Complete KKT certificate at ``tol`` relative; returns the relative residuals
    (stationarity, infeasibility, complementarity incl. dual signs) or raises QPError.

    stationarity   |P x + q + A'y|_inf <= tol * (1 + max(|q|, |Px|, |A'y|))
    feasibility    every row: l_i - tol (1 + |l_i|) <= a_i'x <= u_i + tol (1 + |u_i|)
    dual signs     y_i > 0 only on a finite upper bound, y_i < 0 only on a finite lower bound
    complementarity |y_i| * slack_i <= tol * (1 + |y|_inf) * (1 + |bound_i|)
    """
    Ax = A @ x
    Px, Aty = P @ x, A.T @ y
    ssc = 1.0 + max(np.max(np.abs(q), initial=0.0), np.max(np.abs(Px), initial=0.0),
                    np.max(np.abs(Aty), initial=0.0))
    stat = float(np.max(np.abs(Px + q + Aty), initial=0.0)) / ssc
    fu = np.isfinite(u)
    fl = np.isfinite(l)
    vu = np.where(fu, (Ax - np.where(fu, u, 0.0)) / (1.0 + np.abs(np.where(fu, u, 0.0))), -np.inf)
    vl = np.where(fl, (np.where(fl, l, 0.0) - Ax) / (1.0 + np.abs(np.where(fl, l, 0.0))), -np.inf)
    infeas = float(max(np.max(vu, initial=0.0), np.max(vl, initial=0.0)))
    ysc = 1.0 + float(np.max(np.abs(y), initial=0.0))
    comp = 0.0
    for i in np.nonzero(y)[0]:
        if y[i] > 0:
            if not fu[i]:
                comp = max(comp, y[i] / ysc)
            else:
                comp = max(comp, y[i] * abs(u[i] - Ax[i]) / (ysc * (1.0 + abs(u[i]))))
        else:
            if not fl[i]:
                comp = max(comp, -y[i] / ysc)
            else:
                comp = max(comp, -y[i] * abs(Ax[i] - l[i]) / (ysc * (1.0 + abs(l[i]))))
    if not (stat <= tol and infeas <= tol and comp <= tol):
        raise QPError(f"KKT certificate failed: stationarity {stat:.2e}, infeasibility {infeas:.2e}, "
                      f"complementarity {comp:.2e} (tol {tol:.0e})")
    return stat, infeas, comp


def _null_space(AWn, n):
    """Orthonormal basis of null(A_W) from a complete QR of the (independent) normalised rows."""
    k = AWn.shape[0]
    if k == 0:
        return np.eye(n)
    Q, _ = np.linalg.qr(AWn.T, mode="complete")
    return Q[:, k:]


def solve(P, q, A, l, u, x0, tol=1e-12, max_iter=20000, W0=None):
    """Primal active-set QP.  ``x0`` must be feasible.  Returns (x, y, working_set), certified.

    ``working_set`` is a list of (row, side) with side +1 (upper) / -1 (lower).
    """
    P = np.asarray(P, np.float64)
    q = np.asarray(q, np.float64)
    A = np.asarray(A, np.float64)
    l = np.asarray(l, np.float64)
    u = np.asarray(u, np.float64)
    n, m = q.size, A.shape[0]
    x = np.array(x0, np.float64, copy=True)
    rn = np.linalg.norm(A, axis=1)
    rn_safe = np.where(rn > 0, rn, 1.0)
    An = A / rn_safe[:, None]
    bsc_u = 1.0 + np.abs(np.where(np.isfinite(u), u, 0.0))
    bsc_l = 1.0 + np.abs(np.where(np.isfinite(l), l, 0.0))
    Ax = A @ x
    if np.any(Ax - u > 1e-9 * bsc_u) or np.any(l - Ax > 1e-9 * bsc_l):
        raise QPError("starting point infeasible")

    def rank_ok(rows):
        if not rows:
            return True
        s = np.linalg.svd(An[rows], compute_uv=False)
        return s[-1] > 1e-9 * s[0]

    W: list[tuple[int, int]] = []
    cand = list(W0) if W0 is not None else []
    if W0 is None:
        for i in range(m):
            if rn[i] == 0:
                continue
            if np.isfinite(u[i]) and u[i] - Ax[i] <= 1e-13 * bsc_u[i]:
                cand.append((i, +1))
            elif np.isfinite(l[i]) and Ax[i] - l[i] <= 1e-13 * bsc_l[i]:
                cand.append((i, -1))
    for (i, s) in cand:
        if len(W) < n and rank_ok([r for r, _ in W] + [i]):
            W.append((i, s))

    degenerate = False      # the last step had length 0: Bland's rule against cycling
    at_eqp_min = False      # the last step was a full Newton step: x minimises the EQP of W
    for _ in range(max_iter):
        rows = [r for r, _ in W]
        k = len(rows)
        g = P @ x + q
        Z = _null_space(An[rows], n)
        p = np.zeros(n)
        ray = False
        if Z.shape[1]:
            Zg = Z.T @ g
            Hr = Z.T @ P @ Z
            w, V = np.linalg.eigh(0.5 * (Hr + Hr.T))
            wmax = max(float(np.max(np.abs(w))), 1e-300)
            gh = V.T @ Zg
            gsc = 1.0 + float(np.max(np.abs(g)))
            zero = w <= 1e-12 * wmax
            if np.any(zero & (np.abs(gh) > 1e-12 * gsc)):
                # a descent direction of zero curvature: an unbounded ray until a row blocks
                d = np.where(zero, -gh, 0.0)
                p = Z @ (V @ d)
                ray = True
            else:
                d = np.where(zero, 0.0, -gh / np.where(zero, 1.0, w))
                p = Z @ (V @ d)
        xsc = 1.0 + float(np.max(np.abs(x)))
        pn = float(np.linalg.norm(p))
        if at_eqp_min or (not ray and pn <= 1e-13 * xsc):
            at_eqp_min = False
            # stationary on the working set: multipliers from A_W' y = -g
            if k:
                lam = np.linalg.lstsq(A[rows].T, -g, rcond=None)[0]
            else:
                lam = np.zeros(0)
            thr = -1e-12 * (1.0 + float(np.max(np.abs(lam), initial=0.0)))
            wj, worst = -1, thr
            for j, (r, s) in enumerate(W):
                v = lam[j] * s
                if degenerate:
                    if v < thr and (wj < 0 or r < W[wj][0]):
                        wj = j
                elif v < worst:
                    worst, wj = v, j
            if wj < 0:
                x, y = _solve_eqp(P, q, A, l, u, W)
                certify(P, q, A, l, u, x, y)
                return x, y, W
            W.pop(wj)
            continue
        # ratio test over EVERY row outside the working set
        Ap = A @ p
        Ax = A @ x
        inW = np.zeros(m, bool)
        inW[rows] = True
        eps = 1e-11 * rn * pn
        alpha, block = (np.inf if ray else 1.0), None
        for i in range(m):
            if inW[i]:
                continue
            if Ap[i] > eps[i] and np.isfinite(u[i]):
                t = max((u[i] - Ax[i]) / Ap[i], 0.0)
                side = +1
            elif Ap[i] < -eps[i] and np.isfinite(l[i]):
                t = max((l[i] - Ax[i]) / Ap[i], 0.0)
                side = -1
            else:
                continue
            if t < alpha:          # ties keep the lowest row index (Bland)
                alpha, block = t, (i, side)
        if block is None and ray:
            raise QPError("unbounded QP (descent ray with no blocking row)")
        x = x + alpha * p
        if block is not None:
            if len(W) >= n:
                raise QPError("working set overflow")
            W.append(block)
        degenerate = block is not None and alpha <= 0.0
        at_eqp_min = block is None
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
    try:
        sol = np.linalg.solve(K, rhs)
    except np.linalg.LinAlgError as exc:
        raise QPError(f"singular KKT system of the final working set (|W|={k})") from exc
    # one step of iterative refinement
    sol += np.linalg.solve(K, rhs - K @ sol)
    x, lam = sol[:n], sol[n:]
    y = np.zeros(A.shape[0])
    for j, r in enumerate(rows):
        y[r] = lam[j]
    return x, y
