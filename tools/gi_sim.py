"""Development tool (not shipped, not the oracle): Goldfarb-Idnani dual active set on the pair QP (hinge form), Schur/Cholesky form.
Constraint ids: 2*r (lower side of row r: a'x >= l), 2*r+1 (upper side: -a'x >= -u); hinge rows
only lower side with multiplier cap beta."""
import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import qp_sim as Q

def gi(gq, Pinv, max_steps=300, tol=1e-9, stats=None):
    n, m = gq.n, gq.m
    A, l, u, hm, beta = gq.A, gq.l, gq.u, gq.hinge, gq.beta
    qt = gq.q.copy()
    x = -Pinv @ qt
    W = []            # active constraint ids
    uW = []           # multipliers (>= 0)
    lin = np.zeros(m, bool)
    nsteps = 0; nadd = 0; ndrop = 0; ncap = 0
    def normal(c):
        r = c >> 1
        return (A[r] if (c & 1) == 0 else -A[r]), (l[r] if (c & 1) == 0 else -u[r])
    while True:
        ax = A @ x
        sc = 1.0 + np.abs(l[np.isfinite(l)]).max()
        # most violated constraint
        best, p = -tol * sc, -1
        inW = set(W)
        for r in range(m):
            if hm[r]:
                if lin[r]:
                    if ax[r] - l[r] > tol * sc:
                        if stats is not None: stats['linviol'] = stats.get('linviol', 0) + 1
                        return x, None, False, nsteps
                    continue
                c = 2 * r
                if c in inW: continue
                s = ax[r] - l[r]
                if s < best: best, p = s, c
            else:
                for c, s in ((2 * r, ax[r] - l[r]), (2 * r + 1, u[r] - ax[r])):
                    if c in inW: continue
                    if s < best: best, p = s, c
        if p < 0:
            # done: y in kernel convention
            y = np.zeros(m)
            for c, uu in zip(W, uW):
                r = c >> 1
                y[r] = -uu if (c & 1) == 0 else uu
            y[lin] = -beta
            if stats is not None:
                stats['add'] = stats.get('add', 0) + nadd; stats['drop'] = stats.get('drop', 0) + ndrop; stats['cap'] = stats.get('cap', 0) + ncap
            return x, y, True, nsteps
        npv, bp = normal(p)
        up = 0.0
        while True:
            nsteps += 1
            if nsteps > max_steps:
                return x, None, False, nsteps
            N = np.array([normal(c)[0] for c in W]).reshape(len(W), n)
            yp = Pinv @ npv
            if len(W):
                S = N @ Pinv @ N.T
                r_ = np.linalg.solve(S, N @ yp)
                z = yp - (Pinv @ N.T) @ r_
            else:
                r_ = np.zeros(0); z = yp
            znp = z @ npv
            sp = npv @ x - bp
            t2 = -sp / znp if znp > 1e-12 * (npv @ yp) else np.inf
            t1, k1, kind = np.inf, -1, None
            for k, c in enumerate(W):
                if r_[k] > 0:
                    t = uW[k] / r_[k]
                    if t < t1: t1, k1, kind = t, k, 'drop'
                if hm[c >> 1] and r_[k] < 0:
                    t = (beta - uW[k]) / (-r_[k])
                    if t < t1: t1, k1, kind = t, k, 'cap'
            t3 = (beta - up) if hm[p >> 1] else np.inf
            t = min(t1, t2, t3)
            if not np.isfinite(t):
                return x, None, False, nsteps
            if np.isfinite(t2) or t != t1:
                pass
            x = x + t * z if np.isfinite(t2) else x
            uW = [uu - t * rr for uu, rr in zip(uW, r_)]
            up += t
            if t == t2:
                W.append(p); uW.append(up); nadd += 1
                break
            if t == t3:
                lin[p >> 1] = True; ncap += 1
                qt = qt - beta * A[p >> 1]
                break
            # partial step: drop / cap constraint k1
            c = W.pop(k1); uu = uW.pop(k1)
            if kind == 'cap':
                lin[c >> 1] = True; ncap += 1
            else:
                ndrop += 1

if __name__ == '__main__':
    rec = list(np.load('/tmp/pair_qps.npy', allow_pickle=True))
    H = 30
    st = {}; its = []; errs = []; fails = 0
    for i, r in enumerate(rec):
        gq = Q.GQP.from_edge_slack(r['P'], r['q'], r['A'], r['lo'], r['hi'], H, 1000.0)
        Pinv = np.linalg.inv(gq.P)
        x, y, ok, ns = gi(gq, Pinv, stats=st)
        if not ok:
            fails += 1; continue
        its.append(ns); errs.append(np.abs(x - r['x'][:2*H]).max())
    its = np.array(its)
    print('fails', fails, 'of', len(rec), 'steps mean', its.mean(), 'p95', np.percentile(its, 95), 'max', its.max(), 'max err', max(errs), st)
