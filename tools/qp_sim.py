"""Algorithm prototype for the GPU QP solver (development tool, not shipped, not the oracle).

Generalised QP   min 1/2 x'Px + q'x + sum_i phi_i(a_i'x)
  BOX rows   : phi = indicator[l_i, u_i]
  HINGE rows : phi = beta * max(0, h_i - z)
solved by OSQP-style ADMM (scaled) + primal-dual active-set (PDAS) polish.
Used to choose the kernel's parameters; the kernel follows this file's math.
"""
from __future__ import annotations

import numpy as np

FREE, LOWER, UPPER = 0, 1, 2          # BOX
ZERO, KINK, LINEAR = 0, 1, 2          # HINGE


class GQP:
    def __init__(self, P, q, A, l, u, hinge_mask, beta):
        self.P, self.q, self.A = P, q, A
        self.l, self.u = l, u               # for hinge rows l = h, u = +inf
        self.hinge = hinge_mask.astype(bool)
        self.beta = beta
        self.n, self.m = q.size, A.shape[0]

    @staticmethod
    def from_edge_slack(P, q, A, l, u, H, beta):
        """Convert the oracle's slack form (3H vars) to hinge form (2H vars)."""
        n2 = 2 * H
        m1 = 2 * (2 * H - 1)
        rowsA = [A[:m1, :n2], A[m1 + H:, :n2]]
        Ah = np.vstack(rowsA)
        lh = np.concatenate([l[:m1], l[m1 + H:]])
        uh = np.concatenate([u[:m1], np.full(H, np.inf)])
        mask = np.concatenate([np.zeros(m1, bool), np.ones(H, bool)])
        return GQP(P[:n2, :n2], q[:n2], Ah, lh, uh, mask, beta)


def prox(gq, v, rho):
    """z = prox_{phi/rho}(v) row-wise."""
    z = np.clip(v, gq.l, gq.u)
    h = gq.l
    hm = gq.hinge
    zh = np.where(v[hm] >= h[hm], v[hm],
                  np.where(v[hm] <= h[hm] - gq.beta / rho[hm], v[hm] + gq.beta / rho[hm], h[hm]))
    z[hm] = zh
    return z


def classify(gq, w, rho):
    """Active-set labels from the prox input w = a'x + y/rho."""
    s = np.zeros(gq.m, np.int8)
    b = ~gq.hinge
    s[b & (w <= gq.l)] = LOWER
    s[b & (w >= gq.u)] = UPPER
    hm = gq.hinge
    s[hm & (w > gq.l - gq.beta / rho) & (w < gq.l)] = KINK
    s[hm & (w <= gq.l - gq.beta / rho)] = LINEAR
    return s


REG = [1e-13, 1]   # relative regularisation of S, refinement steps
DEP_TOL = [1e-10]  # relative pivot below which a working-set row counts as dependent


def reduced_solve(gq, Pinv, sets):
    """Equality-constrained QP of a label vector via the Schur complement on P^-1."""
    hm = gq.hinge
    qt = gq.q - gq.beta * gq.A[hm & (sets == LINEAR)].sum(axis=0)
    Wb = (~hm & (sets != FREE)) | (hm & (sets == KINK))
    rows = np.nonzero(Wb)[0]
    x0 = -Pinv @ qt
    y = np.zeros(gq.m)
    y[hm & (sets == LINEAR)] = -gq.beta
    if rows.size == 0:
        return x0, y, True
    AW = gq.A[rows]
    b = np.where(gq.hinge[rows], gq.l[rows], np.where(sets[rows] == LOWER, gq.l[rows], gq.u[rows]))
    V = Pinv @ AW.T
    S = AW @ V
    # Cholesky that drops rows linearly dependent on the earlier ones (pivot collapse)
    m = rows.size
    L = np.zeros((m, m))
    keep = np.ones(m, bool)
    for k in range(m):
        d = S[k, k] - L[k, :k] @ L[k, :k]
        if d <= DEP_TOL[0] * S[k, k]:
            keep[k] = False
            continue
        L[k, k] = np.sqrt(d)
        L[k + 1:, k] = (S[k + 1:, k] - L[k + 1:, :k] @ L[k, :k]) / L[k, k]
    rhs = AW @ x0 - b
    idx = np.nonzero(keep)[0]
    Lk = L[np.ix_(idx, idx)]
    lam = np.zeros(m)
    lam[idx] = np.linalg.solve(Lk.T, np.linalg.solve(Lk, rhs[idx]))
    for _ in range(REG[1]):
        r = rhs[idx] - S[np.ix_(idx, idx)] @ lam[idx]
        lam[idx] += np.linalg.solve(Lk.T, np.linalg.solve(Lk, r))
    x = x0 - V @ lam
    y[rows] = lam
    return x, y, True


def kkt_ok(gq, x, y, sets, tol):
    ax = gq.A @ x
    hm = gq.hinge
    b = ~hm
    sc = 1.0 + np.abs(gq.l[np.isfinite(gq.l)]).max()
    ok = True
    f = b & (sets == FREE)
    ok &= np.all(ax[f] >= gq.l[f] - tol * sc) and np.all(ax[f] <= gq.u[f] + tol * sc)
    ys = tol * (1 + np.abs(y).max())
    ok &= np.all(y[b & (sets == LOWER)] <= ys) and np.all(y[b & (sets == UPPER)] >= -ys)
    ok &= np.all(ax[hm & (sets == ZERO)] >= gq.l[hm & (sets == ZERO)] - tol * sc)
    ok &= np.all(ax[hm & (sets == LINEAR)] <= gq.l[hm & (sets == LINEAR)] + tol * sc)
    kk = hm & (sets == KINK)
    ok &= np.all(y[kk] <= ys) and np.all(y[kk] >= -gq.beta - ys)
    return bool(ok)


def pdas(gq, Pinv, sets, c, max_steps=8, tol=1e-9):
    for k in range(max_steps):
        x, y, good = reduced_solve(gq, Pinv, sets)
        if not good:
            return x, y, sets, False, k + 1
        if kkt_ok(gq, x, y, sets, tol):
            return x, y, sets, True, k + 1
        new = classify(gq, gq.A @ x + y / c, c)
        if np.array_equal(new, sets):
            return x, y, sets, False, k + 1
        sets = new
    return x, y, sets, False, max_steps


def scale_problem(gq, mode):
    """Diagonal scaling x = D xs, rows E: returns scaled P, q, A and (D, E)."""
    n, m = gq.n, gq.m
    D = np.ones(n)
    E = np.ones(m)
    if mode == "none":
        pass
    elif mode == "jacobi":
        D = 1.0 / np.sqrt(np.diag(gq.P))
        E = 1.0 / np.maximum(np.linalg.norm(gq.A * D, axis=1), 1e-12)
    elif mode == "ruiz":
        P, A = gq.P.copy(), gq.A.copy()
        for _ in range(15):
            cn = np.maximum(np.abs(P).max(axis=0), np.abs(A).max(axis=0))
            rn = np.abs(A).max(axis=1)
            # the kernel's clamp_norm: a (near-)zero row or column keeps scale 1
            dd = 1.0 / np.sqrt(np.where(cn > 1e-6, np.minimum(cn, 1e6), 1.0))
            ee = 1.0 / np.sqrt(np.where(rn > 1e-6, np.minimum(rn, 1e6), 1.0))
            P = dd[:, None] * P * dd[None, :]
            A = ee[:, None] * A * dd[None, :]
            D *= dd
            E *= ee
    return D, E


def admm(gq, rho_s, sigma, alpha, iters, D, E, state=None, Pinv=None, polish_every=10,
         rho_scale=None, adapt_every=0, stats=None):
    """OSQP iteration in the scaled space.  Returns (x, y, its, polished_ok, pdas_steps)."""
    Ps = D[:, None] * gq.P * D[None, :]
    qs = D * gq.q
    As = E[:, None] * gq.A * D[None, :]
    ls, us = E * gq.l, E * gq.u
    rho = np.full(gq.m, rho_s) if rho_scale is None else rho_s * rho_scale
    gs = GQP(Ps, qs, As, ls, us, gq.hinge, 0.0)
    beta_s = gq.beta * E        # hinge weight per row in scaled units: phi(z_s) = beta max(0, h - z_s/E)
    K = Ps + sigma * np.eye(gq.n) + As.T @ (rho[:, None] * As)
    Kinv = np.linalg.inv(K)
    if state is None:
        xs = np.zeros(gq.n)
        zs = As @ xs
        ys = np.zeros(gq.m)
    else:
        xs, zs, ys = state
    for it in range(1, iters + 1):
        xt = Kinv @ (sigma * xs - qs + As.T @ (rho * zs - ys))
        zt = As @ xt
        xs = alpha * xt + (1 - alpha) * xs
        v = alpha * zt + (1 - alpha) * zs + ys / rho
        zn = np.clip(v, ls, us)
        hm = gq.hinge
        hh = ls[hm]
        bb = (gq.beta / E[hm]) / rho[hm]     # scaled hinge weight beta/E, prox threshold /rho
        zn[hm] = np.where(v[hm] >= hh, v[hm], np.where(v[hm] <= hh - bb, v[hm] + bb, hh))
        ys = ys + rho * (v - ys / rho - zn)
        zs = zn
        if adapt_every and it % adapt_every == 0:
            # OSQP adaptive rho (scaled space): sqrt(prim/dual) of normalised residuals
            Ax = As @ xs
            rp = np.max(np.abs(Ax - zs)) / max(np.max(np.abs(Ax)), np.max(np.abs(zs)), 1e-30)
            Px = Ps @ xs
            Aty = As.T @ ys
            rd = np.max(np.abs(Px + qs + Aty)) / max(np.max(np.abs(Px)), np.max(np.abs(Aty)), np.max(np.abs(qs)), 1e-30)
            ratio = np.sqrt(rp / max(rd, 1e-30))
            if ratio > 5.0 or ratio < 0.2:
                rho = np.clip(rho * ratio, 1e-6, 1e6)
                K = Ps + sigma * np.eye(gq.n) + As.T @ (rho[:, None] * As)
                Kinv = np.linalg.inv(K)
                if stats is not None:
                    stats['refac'] = stats.get('refac', 0) + 1
        if Pinv is not None and it % polish_every == 0:
            # unscale: x = D xs, y = E ys, prox input w = a'x + y/c with c = rho E^2 in unscaled units
            x = D * xs
            y = E * ys
            c = rho * E * E
            sets = classify(gq, gq.A @ x + y / c, c)
            xp, yp, sets, ok, st = pdas(gq, Pinv, sets, c)
            if ok:
                return xp, yp, it, True, st
    return D * xs, E * ys, iters, False, 0
