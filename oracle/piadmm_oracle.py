"""PI-ADMM oracle -- CPU fp64 NumPy restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker (or as the timed CPU baseline).  The product path (the HIP library
behind include/piadmm.h) never calls it and fails loudly without its extension.

What it restates (all paths relative to the reference root):
  * rollouts        ``casadi/PI_ADMM_class.py:45-70`` (linearised, numeric branch) and
                    ``:77-105`` (numeric branch = nonlinear Euler unicycle), literal
                    expression order; MATLAB numeric local rollout
                    ``matlab_old_files/ADMM_CVX_two_veh_intesection_PI_antiwindup.m:312-330``
  * x-step QP       ``casadi/PI_ADMM_class.py:114-135`` (cost), ``:172-192`` (constraints),
                    solved as in ``casadi/main.py:81-106``
  * collision test  ``casadi/main.py:110-118`` (MATLAB ``:107-118``)
  * z-step QP       ``casadi/PI_ADMM_class.py:145-169`` with the heading frozen at xt as in
                    MATLAB ``:276-304,378-397`` (quirk B3), ``casadi/main.py:121-158``
  * dual update     plain ``casadi/main.py:161-162``; PI + back-calculation
                    ``ADMM_CVX_..._PI_antiwindup.m:152-188``
  * residuals       ``casadi/main.py:164-181`` (MATLAB ``:191-210``)
  * MPC propagation ``casadi/main.py:185-192``, seeds ``:48-49``

Pinned bit for bit to the reference's own statements, executed (tests/test_oracle.py):
the rollouts (``oracle/gen_ref_rollouts.py`` -> ``tests/golden/ref_rollouts.npz``) and the
loop's NumPy statements -- seeds, collision test, pair hat rollout, plain dual update, residual
sums, propagation (``oracle/gen_ref_mainloop.py`` -> ``tests/golden/ref_mainloop.npz``).

Parity pinning: the reference cannot run here (casadi, bunch and OSQP are
absent) and its repository holds no tests, fixtures or outputs for
this path.  The oracle is pinned (a) by executing the reference's own NumPy code
on seeded inputs -- the numeric rollouts (oracle/gen_ref_rollouts.py) and every
non-solver statement of the casadi/main.py loop (oracle/gen_ref_mainloop.py), bit
for bit -- and (b) by KKT certificates of every QP it solves (the reference's
solver output is not available anywhere).  What stays "parity unpinned" against
reference outputs: the QP assembly (cost_function_primal / _edge need CasADi) and
the MATLAB PI update (MATLAB is absent); see DESIGN.md section 3.

Generalisation from the reference's two vehicles to N agents:
static candidate pairs (the AL sum runs over candidate neighbours, B8),
per-directed-edge PI accumulators (B10) and per-component termination (B9).
For one pair these reduce exactly to the reference.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from . import qp_exact


def around(x, decimals: int):
    """``np.around(x, 4)`` as used on every solver output (``casadi/main.py:103,153``)."""
    return np.around(x, decimals) if decimals >= 0 else x


# ----------------------------------------------------------------------------- rollouts
def rollout_linear(xt, u, s, dt, L):
    """``PI_ADMM_CASADI.dynamic_update_local`` numeric branch (``PI_ADMM_class.py:56-70``)."""
    H = u.shape[-1]
    x = np.zeros(H + 1)
    y = np.zeros(H + 1)
    th = np.zeros(H + 1)
    x[0], y[0], th[0] = xt[0], xt[1], xt[2]
    s0, c0 = np.sin(xt[2]), np.cos(xt[2])
    for k in range(H):
        x_dot = -s * s0 * th[k] + (s * c0 + s * xt[2] * s0)
        x[k + 1] = x[k] + x_dot * dt
        y_dot = s * c0 * th[k] + (s * s0 - s * xt[2] * c0)
        y[k + 1] = y[k] + y_dot * dt
        theta_dot = s / L * u[k]
        th[k + 1] = th[k] + theta_dot * dt
    return x, y, th


def rollout_nonlinear(xt, u, s, dt, L):
    """``PI_ADMM_CASADI.dynamic_update_edge`` numeric branch (``PI_ADMM_class.py:88-105``).

    Also the MATLAB numeric ``dynamic_update_local`` (``ADMM_CVX_...:312-330``).
    """
    H = u.shape[-1]
    x = np.zeros(H + 1)
    y = np.zeros(H + 1)
    th = np.zeros(H + 1)
    x[0], y[0], th[0] = xt[0], xt[1], xt[2]
    for k in range(H):
        sk, ck = np.sin(th[k]), np.cos(th[k])
        x_dot = -s * sk * th[k] + (s * ck + s * th[k] * sk)
        x[k + 1] = x[k] + x_dot * dt
        y_dot = s * ck * th[k] + (s * sk - s * th[k] * ck)
        y[k + 1] = y[k] + y_dot * dt
        theta_dot = s / L * u[k]
        th[k + 1] = th[k] + theta_dot * dt
    return x, y, th


def rollout_affine(xt, s, dt, L, H):
    """Affine form p = c + M u of the symbolic linearised rollout (``PI_ADMM_class.py:59-69``).

    Propagates (constant, coefficient-vector) pairs through the same recursion the
    reference builds as a CasADi SX graph.  Returns c (2, H+1) and M (2, H+1, H).
    """
    c = np.zeros((2, H + 1))
    M = np.zeros((2, H + 1, H))
    c[0, 0], c[1, 0] = xt[0], xt[1]
    s0, c0 = np.sin(xt[2]), np.cos(xt[2])
    th_c = xt[2]
    th_m = np.zeros(H)
    for k in range(H):
        c[0, k + 1] = c[0, k] + (-s * s0 * th_c + (s * c0 + s * xt[2] * s0)) * dt
        M[0, k + 1] = M[0, k] + (-s * s0 * dt) * th_m
        c[1, k + 1] = c[1, k] + (s * c0 * th_c + (s * s0 - s * xt[2] * c0)) * dt
        M[1, k + 1] = M[1, k] + (s * c0 * dt) * th_m
        th_m = th_m.copy()
        th_m[k] += s / L * dt
    return c, M


# ----------------------------------------------------------------------------- QPs
def box_rate_rows(H, u_max, du_max):
    """``nonlcon_function`` (``PI_ADMM_class.py:172-192``) as l <= A u <= u: [I; D1]."""
    A = np.zeros((2 * H - 1, H))
    A[:H] = np.eye(H)
    for k in range(H - 1):
        A[H + k, k + 1] = 1.0
        A[H + k, k] = -1.0
    lo = np.concatenate([np.full(H, -u_max), np.full(H - 1, -du_max)])
    hi = -lo
    return A, lo, hi


def xstep_qp(cfg, xt_i, s_i, ref_i, nbr_terms):
    """Per-agent QP of ``cost_function_primal`` (``PI_ADMM_class.py:114-135``).

    J(u) = Pnorm||c+Mu-r||^2 + ||D2 u||^2 + rho/2 sum_j ||c+Mu-hat_ij+lam_ij||^2 + Pcost||u||^2
    -> P = (2 Pnorm + rho |N|) M'M + 2 D2'D2 + 2 Pcost I,
       q = M'(2 Pnorm (c - r) + rho sum_j (c - hat_ij + lam_ij)).
    ``nbr_terms`` is a list of (hat_ij, lam_ij), each (2, H+1), or (hat_ij, lam_ij, rho_ij) with a
    per-pair penalty (global PI, ``casadi_old_PI_ADMM/main.py:139``: rho |N| becomes sum_j rho_ij).
    """
    H = cfg.H
    c, M = rollout_affine(xt_i, s_i, cfg.dt, cfg.L, H)
    Mf = M.reshape(2 * (H + 1), H)
    cf = c.reshape(-1)
    D2 = np.zeros((max(H - 2, 0), H))
    for k in range(H - 2):
        D2[k, k:k + 3] = (1.0, -2.0, 1.0)
    nN = len(nbr_terms)
    rhos = [t[2] if len(t) > 2 else cfg.rho for t in nbr_terms]
    rsum = cfg.rho * nN
    if any(len(t) > 2 for t in nbr_terms):
        rsum = 0.0
        for r in rhos:
            rsum = rsum + r
    P = (2.0 * cfg.Pnorm + rsum) * (Mf.T @ Mf) + 2.0 * (D2.T @ D2) + 2.0 * cfg.Pcost * np.eye(H)
    v = 2.0 * cfg.Pnorm * (cf - ref_i.reshape(-1))
    for t, r in zip(nbr_terms, rhos):
        v = v + r * (cf - t[0].reshape(-1) + t[1].reshape(-1))
    q = Mf.T @ v
    A, lo, hi = box_rate_rows(H, cfg.u_max, cfg.du_max)
    return P, q, A, lo, hi


def edge_qp(cfg, xt1, s1, xt2, s2, p1, p2, lam1, lam2, seed1, seed2, d_eff=None, rho=None):
    """Pair z-step of ``cost_function_edge`` (``PI_ADMM_class.py:145-169``), slack form.

    Heading frozen at xt (MATLAB symbolic branch ``ADMM_CVX_...:378-397``, quirk B3) so
    the edge positions are affine: e_v = c_v + M_v uhat_v.  Variables
    [uhat_1 (H), uhat_2 (H), s (H)]; the hinge beta*max(0, D^2 - dis_k) becomes
    beta*s_k with s_k >= 0 and s_k >= D^2 - dis_k,
    dis_k = 2 dbar'(e_2k - e_1k) - ||dbar||^2, k = 1..H, dbar = seed_2 - seed_1.
    """
    H = cfg.H
    rho = cfg.rho if rho is None else rho     # the pair's adaptive penalty (global PI)
    c1, M1 = rollout_affine(xt1, s1, cfg.dt, cfg.L, H)
    c2, M2 = rollout_affine(xt2, s2, cfg.dt, cfg.L, H)
    dbar = np.asarray(seed2, np.float64) - np.asarray(seed1, np.float64)
    dd = np.sum(np.power(dbar, 2))
    n = 3 * H
    P = np.zeros((n, n))
    q = np.zeros(n)
    for v, (c, M, p, lam) in enumerate(((c1, M1, p1, lam1), (c2, M2, p2, lam2))):
        Mf = M.reshape(2 * (H + 1), H)
        b = p.reshape(-1) + lam.reshape(-1) - c.reshape(-1)
        sl = slice(v * H, (v + 1) * H)
        P[sl, sl] = rho * (Mf.T @ Mf) + 2.0 * cfg.Pcost * np.eye(H)
        q[sl] = -rho * (Mf.T @ b)
    q[2 * H:] = cfg.beta
    Ab, lob, hib = box_rate_rows(H, cfg.u_max, cfg.du_max)
    m1 = Ab.shape[0]
    A = np.zeros((2 * m1 + 2 * H, n))
    A[:m1, :H] = Ab
    A[m1:2 * m1, H:2 * H] = Ab
    lo = np.concatenate([lob, lob, np.zeros(H), np.zeros(H)])
    hi = np.concatenate([hib, hib, np.full(H, np.inf), np.full(H, np.inf)])
    r0 = 2 * m1
    A[r0:r0 + H, 2 * H:] = np.eye(H)
    h0, G = hinge_rows(cfg, c1, M1, c2, M2, dbar, dd, d_eff)
    A[r0 + H:, :2 * H] = G
    A[r0 + H:, 2 * H:] = np.eye(H)
    lo[r0 + H:] = h0
    return P, q, A, lo, hi


def hinge_rows(cfg, c1, M1, c2, M2, dbar, dd, d_eff=None):
    """g_k(uhat) = D^2 - dis_k = h0_k - G_k uhat for k = 1..H (``PI_ADMM_class.py:149-156``).

    D = dis_thres, or the delay-tightened d_eff of the pair (``tighten``, :func:`safety_distance`)."""
    H = cfg.H
    D2 = (cfg.dis_thres if d_eff is None else d_eff) ** 2
    h0 = np.empty(H)
    G = np.zeros((H, 2 * H))
    for k in range(1, H + 1):
        h0[k - 1] = D2 + dd - 2.0 * (dbar[0] * (c2[0, k] - c1[0, k]) + dbar[1] * (c2[1, k] - c1[1, k]))
        G[k - 1, :H] = -2.0 * (dbar[0] * M1[0, k] + dbar[1] * M1[1, k])
        G[k - 1, H:] = 2.0 * (dbar[0] * M2[0, k] + dbar[1] * M2[1, k])
    return h0, G


def solve_xstep(cfg, xt_i, s_i, ref_i, nbr_terms):
    P, q, A, lo, hi = xstep_qp(cfg, xt_i, s_i, ref_i, nbr_terms)
    x, y, _ = qp_exact.solve(P, q, A, lo, hi, np.zeros(cfg.H))
    return x, (P, q, A, lo, hi, y)


def solve_edge(cfg, xt1, s1, xt2, s2, p1, p2, lam1, lam2, seed1, seed2, d_eff=None, rho=None):
    P, q, A, lo, hi = edge_qp(cfg, xt1, s1, xt2, s2, p1, p2, lam1, lam2, seed1, seed2, d_eff, rho)
    H = cfg.H
    x0 = np.zeros(3 * H)
    x0[2 * H:] = np.maximum(0.0, lo[-H:])          # feasible: s = max(0, g(0))
    x, y, _ = qp_exact.solve(P, q, A, lo, hi, x0)
    return x[:2 * H].reshape(2, H), (P, q, A, lo, hi, x, y)


def delay_offset(cfg, xt_i, s_i):
    """Delay offset of ``compute_square_halfspaces_ca_prob`` (``decentralized/util.py:81-96``):
    delta = avg_delay v (cos, sin) + sqrt(p/(1-p)) ((var_delay v cos)^2, (var_delay v sin)^2),
    with v = the agent's speed and the heading of its state at the start of the MPC step."""
    th = xt_i[2]
    dx_avg = cfg.avg_delay * s_i * np.cos(th)
    dy_avg = cfg.avg_delay * s_i * np.sin(th)
    dx_var = (cfg.var_delay * s_i * np.cos(th)) * (cfg.var_delay * s_i * np.cos(th))
    dy_var = (cfg.var_delay * s_i * np.sin(th)) * (cfg.var_delay * s_i * np.sin(th))
    kappa = np.sqrt(cfg.tight_p / (1.0 - cfg.tight_p))
    return np.array([dx_avg + kappa * dx_var, dy_avg + kappa * dy_var])


def safety_distance(cfg, xt, spd, v1, v2):
    """Pair safety distance: dis_thres, or with ``tighten`` the reference's
    delay offsets applied to the QP path as d_eff = dis_thres + |delta_1| + |delta_2|."""
    if not cfg.tighten:
        return cfg.dis_thres
    return cfg.dis_thres + np.hypot(*delay_offset(cfg, xt[v1], spd[v1])) + np.hypot(*delay_offset(cfg, xt[v2], spd[v2]))


def collides(cfg, p1, p2, d_eff):
    """Collision test of one candidate pair (``casadi/main.py:110-113``): any horizon point with
    d^2 below the threshold (Python compares d^2 with the unsquared dis_thres, quirk B2)."""
    d2 = np.square(p1[0] - p2[0]) + np.square(p1[1] - p2[1])
    return bool(np.max(d2 < cfg.collide_thr(d_eff)))


def pair_residuals(cfg, p_v1, hat_v1v2, last_v1v2):
    """One pair's terms of ``casadi/main.py:170-173`` (the v1 side only, times 2, quirk B5):
    (primal, dual) = (2 |p_v1 - hat_v1v2|_F, 2 |rho (last_hat_v1v2 - hat_v1v2)|_F)."""
    sk = 2 * np.sqrt(np.sum((cfg.rho * (last_v1v2 - hat_v1v2)) ** 2))
    rk = 2 * np.sqrt(np.sum((p_v1 - hat_v1v2) ** 2))
    return rk, sk


def propagate(cfg, xt, u, spd):
    """MPC propagation (``casadi/main.py:185-192``): every agent's state one step along the
    nonlinear rollout of its plan."""
    new_xt = np.array(xt, np.float64, copy=True)
    for i in range(new_xt.shape[0]):
        x, y, th = rollout_nonlinear(xt[i], u[i], spd[i], cfg.dt, cfg.L)
        new_xt[i] = (x[1], y[1], th[1])
    return new_xt


def shift_horizon(a):
    """Receding-horizon shift along the last axis: drop slot 0, duplicate the last slot
    (``iterate_next_state``, ``decentralized/optimizer.py:337-344``)."""
    return np.concatenate([a[..., 1:], a[..., -1:]], axis=-1)


# ----------------------------------------------------------------------------- near ties
# Kinds of include/piadmm.h (PIADMM_TIE_*): the reference's discrete decisions.
TIE_ROUND_U, TIE_ROUND_UHAT, TIE_ROUND_SEED, TIE_COLLIDE, TIE_STOP, TIE_DIST = range(6)


def round_margins(x, decimals):
    """Signed distance of each x to the nearest rounding boundary (k + 1/2) 10^-d of np.around
    (casadi/main.py:48-49,103,153), computed as the kernels do: (x 10^d - (floor(x 10^d) + 1/2)) / 10^d."""
    f = 10.0 ** decimals
    y = np.asarray(x, np.float64) * f
    return (y - (np.floor(y) + 0.5)) / f


class TieLog:
    """Near-tie log of the oracle: the mirror of piadmm_get_near_ties (same kinds, ids, margins)."""

    def __init__(self, tol=1e-9):
        self.tol = float(tol)
        self.events = []          # (step, iter, kind, id, index, margin)

    def rounding(self, t, it, kind, ident, x, decimals, idx0=0):
        if decimals < 0:
            return
        m = round_margins(x, decimals)
        for k in np.nonzero(np.abs(m) * 10.0 ** decimals <= self.tol * 10.0 ** decimals)[0]:
            self.events.append((t, it, kind, ident, idx0 + int(k), float(m[k])))

    def collide(self, t, it, e, d2, thr):
        lo = np.any(d2 < thr * (1.0 - self.tol))
        near = np.any(d2 <= thr * (1.0 + self.tol))
        if not lo and near:
            k = int(np.argmin(d2))
            self.events.append((t, it, TIE_COLLIDE, e, k, float((d2[k] - thr) / thr)))

    def scalar(self, t, it, kind, ident, idx, v, thr):
        if abs(v - thr) <= self.tol * abs(thr):
            self.events.append((t, it, kind, ident, idx, float((v - thr) / thr)))


# ----------------------------------------------------------------------------- state
@dataclasses.dataclass
class StepRecord:
    xt: np.ndarray            # (N,3) state after propagation
    u: np.ndarray             # (N,H) primal_u used for propagation
    iters: np.ndarray         # (C,) outer iterations executed per component
    resid: list               # per component: list of (rk, sk) per executed iteration
    pos_old: np.ndarray       # (N,2,H+1) final x-step positions
    hat: np.ndarray           # (E,2,2,H+1) final edge positions (dir 0: hat_{v1v2})
    lam: np.ndarray           # (E,2,2,H+1) final duals
    edge_active: np.ndarray   # (E,) collision flag of the last executed iteration
    global_resid: list = dataclasses.field(default_factory=list)   # term_global: summed (rk, sk)


class Oracle:
    """Runs the reference loop (``casadi/main.py:43-201``) on a :class:`Scenario`."""

    def __init__(self, cfg, scn, owned=None, counted=None):
        """``owned`` / ``counted`` (one rank of a job whose pairs cross ranks, piadmm.dist.Shard):
        only owned agents solve their x-step (the others are ghosts filled by the ``exchange``
        hook of :meth:`mpc_step`), and only counted pairs enter the residual sums."""
        self.cfg = cfg
        self.scn = scn
        self.owned = None if owned is None else np.asarray(owned, bool)
        self.counted = None if counted is None else np.asarray(counted, bool)
        self.N, self.E, self.H = scn.n_agents, scn.n_edges, cfg.H
        self.comp, self.n_comp = scn.components()
        self.xt = scn.xt0.astype(np.float64).copy()
        self.primal_u = np.zeros((self.N, self.H))
        self.comp_agents = [np.nonzero(self.comp == c)[0] for c in range(self.n_comp)]
        ecomp = self.comp[scn.edges[:, 0]] if self.E else np.zeros(0, np.int32)
        self.comp_edges = [np.nonzero(ecomp == c)[0] for c in range(self.n_comp)]
        self.nbrs = [[] for _ in range(self.N)]     # (edge, dir) per agent, sorted by neighbour
        for e, (v1, v2) in enumerate(scn.edges):
            self.nbrs[int(v1)].append((int(v2), e, 0))
            self.nbrs[int(v2)].append((int(v1), e, 1))
        for a in range(self.N):
            self.nbrs[a].sort()
        self.t = 0
        self.edge_state = None      # (hat, lam, S, D, last_hat) after the last step (warm_duals)
        # global PI: the pair's adaptive penalty, kept across MPC steps like PI_ADMM.param.rho
        # (casadi_old_PI_ADMM/main.py:139 is never reset)
        self.rho_pi = np.full(self.E, float(cfg.rho))
        self.ties = TieLog()        # near ties of the discrete decisions (piadmm_get_near_ties)

    def seeds(self):
        """``casadi/main.py:48-49``."""
        c, xt = self.cfg, self.xt
        sx = around(xt[:, 0] + c.dt * self.scn.spd * np.cos(xt[:, 2]), c.round_decimals)
        sy = around(xt[:, 1] + c.dt * self.scn.spd * np.sin(xt[:, 2]), c.round_decimals)
        return np.stack([sx, sy], axis=1)

    def mpc_step(self, components=None, reduce=None, exchange=None, on_iter=None) -> StepRecord:
        """One ``num_step`` body of ``casadi/main.py:43-201``.

        Iteration-major: every outer iteration runs the x-steps of all agents, the
        collision test, the z-steps and dual updates of the active pairs and the residual
        test, per termination group -- one group per connected component (``term_global``
        off) or one group of all agents (``term_global`` on: the reference's
        global ``flag`` and ``rk, sk`` sums, quirk B9).  Components are independent, so the
        per-component results do not depend on the order.

        ``reduce`` (term_global only) maps this process's termination partials
        [rk, sk, active pairs, pairs with a distance check, pairs failing it] to the sums over
        all processes: the all-reduce of the sharded path (tests/test_dist.py runs it on gloo).
        ``exchange(pos_old, primal_u)`` (a rank of a job whose pairs cross ranks) fills the ghost
        agents' rows in place after the x-steps: the boundary all-reduce of the sharded path.
        ``on_iter(it, state)`` is called after every outer iteration with copies of pos_old, hat,
        lam, S, D and ``stop`` (every termination group has stopped): the per-iteration state of
        ``casadi/main.py:78-181`` / ``ADMM_CVX_..._PI_antiwindup.m:160-188`` that
        ``piadmm_outer_iter`` exposes.
        """
        cfg, H, N, E = self.cfg, self.H, self.N, self.E
        if exchange is not None and not cfg.term_global:
            raise ValueError("pairs across ranks need term_global")
        own = (lambda i: True) if self.owned is None else (lambda i: bool(self.owned[i]))
        cnt = (lambda e: True) if self.counted is None else (lambda e: bool(self.counted[e]))
        t = self.t
        seeds = self.seeds()
        for i in range(N):
            raw = (self.xt[i, 0] + cfg.dt * self.scn.spd[i] * np.cos(self.xt[i, 2]),
                   self.xt[i, 1] + cfg.dt * self.scn.spd[i] * np.sin(self.xt[i, 2]))
            self.ties.rounding(t, -1, TIE_ROUND_SEED, i, np.array(raw), cfg.round_decimals)
        pos_old = np.zeros((N, 2, H + 1))
        if cfg.warm_duals and self.edge_state is not None:
            # a12: the previous step's duals, edge positions and PI accumulators, shifted
            hat, lam, S, D, last_hat = (shift_horizon(a) for a in self.edge_state)
        else:
            # casadi/main.py:52-63: reset every MPC step (the adaptive-gain script starts hat and
            # lam at 1e-4, ADMM_CVX_..._adp_PI_antiwindup1.m:58-61: cfg.dual_init)
            hat, lam, S, D, last_hat = (np.zeros((E, 2, 2, H + 1)) for _ in range(5))
            if cfg.dual_init != 0.0:
                hat[...] = cfg.dual_init
                lam[...] = cfg.dual_init
                last_hat[...] = cfg.dual_init
        active = np.zeros(E, bool)
        iters = np.zeros(self.n_comp, np.int32)
        resid = [[] for _ in range(self.n_comp)]
        d_eff = np.array([safety_distance(cfg, self.xt, self.scn.spd, int(v1), int(v2))
                          for v1, v2 in self.scn.edges]) if E else np.zeros(0)
        dis_chk = np.full(E, np.nan)
        comps = list(range(self.n_comp)) if components is None else list(components)
        groups = [comps] if cfg.term_global else [[c] for c in comps]
        g_flag = [0] * len(groups)
        g_alias = [False] * len(groups)
        g_done = [False] * len(groups)
        global_resid = []
        for it in range(cfg.max_outer):
            if all(g_done):
                break
            for g, gcomps in enumerate(groups):
                if g_done[g]:
                    continue
                agents = np.concatenate([self.comp_agents[c] for c in gcomps])
                edges = np.concatenate([self.comp_edges[c] for c in gcomps]).astype(np.int64)
                for c in gcomps:
                    iters[c] = it + 1
                # ---- x-step, casadi/main.py:81-106
                gpi = cfg.dual_mode == 2
                for i in agents:
                    if not own(i):
                        continue          # a ghost: its owner rank solves it (exchange below)
                    terms = [(hat[e, d], lam[e, d], self.rho_pi[e]) if gpi else (hat[e, d], lam[e, d])
                             for (_, e, d) in self.nbrs[i]]
                    u_star, _ = solve_xstep(cfg, self.xt[i], self.scn.spd[i],
                                            self.scn.ref[i, :, t:t + H + 1], terms)
                    u = around(u_star, cfg.round_decimals)
                    self.ties.rounding(t, it, TIE_ROUND_U, int(i), u_star, cfg.round_decimals)
                    roll = rollout_linear if cfg.pos_model == 0 else rollout_nonlinear
                    px, py, _ = roll(self.xt[i], u, self.scn.spd[i], cfg.dt, cfg.L)
                    pos_old[i, 0], pos_old[i, 1] = px, py
                    self.primal_u[i] = u
                if exchange is not None:
                    exchange(pos_old, self.primal_u)
                # ---- collision graph, casadi/main.py:110-118
                for e in edges:
                    v1, v2 = self.scn.edges[e]
                    active[e] = True if cfg.no_collision_gate else collides(cfg, pos_old[v1], pos_old[v2], d_eff[e])
                    if not cfg.no_collision_gate:
                        d2 = np.square(pos_old[v1][0] - pos_old[v2][0]) + np.square(pos_old[v1][1] - pos_old[v2][1])
                        self.ties.collide(t, it, int(e), d2, cfg.collide_thr(d_eff[e]))
                act = [e for e in edges if active[e]]
                # ---- z-step + dual update, casadi/main.py:121-162 (none when no pair is active)
                for e in act:
                    v1, v2 = (int(a) for a in self.scn.edges[e])
                    uh, _ = solve_edge(cfg, self.xt[v1], self.scn.spd[v1], self.xt[v2], self.scn.spd[v2],
                                       pos_old[v1], pos_old[v2], lam[e, 0], lam[e, 1], seeds[v1], seeds[v2],
                                       d_eff[e], self.rho_pi[e] if gpi else None)
                    for d in range(2):
                        self.ties.rounding(t, it, TIE_ROUND_UHAT, int(e), uh[d], cfg.round_decimals, idx0=d * H)
                    uh = around(uh, cfg.round_decimals)
                    for d, v in enumerate((v1, v2)):
                        hx, hy, _ = rollout_nonlinear(self.xt[v], uh[d], self.scn.spd[v], cfg.dt, cfg.L)
                        hat[e, d, 0], hat[e, d, 1] = hx, hy
                    if gpi:
                        dis_chk[e] = dual_update_global_pi(cfg, self.xt, self.scn.spd, self.primal_u, v1, v2,
                                                           pos_old, hat[e], lam[e], S[e], D[e], self.rho_pi, e)
                        if cfg.term_dist_check:
                            self.ties.scalar(t, it, TIE_DIST, int(e), 0, dis_chk[e], d_eff[e])
                        continue
                    dvec = pos_old[v1] - pos_old[v2]
                    dist = np.sqrt(np.sum(dvec * dvec, axis=0))
                    dual_update(cfg, pos_old[v1], pos_old[v2], hat[e], lam[e], S[e], D[e], dist)
                    dis_chk[e] = dist[1]
                    if cfg.term_dist_check:
                        self.ties.scalar(t, it, TIE_DIST, int(e), 0, dis_chk[e], d_eff[e])
                # ---- residuals, casadi/main.py:164-178 (per component; summed over the group)
                comp_r = []
                for c in gcomps:
                    rk = sk = 0.0
                    for e in self.comp_edges[c]:
                        if not active[e] or not cnt(e):
                            continue
                        v1, v2 = (int(a) for a in self.scn.edges[e])
                        if gpi:
                            rk_e, sk_e = pair_residuals_global_pi(pos_old[v1], pos_old[v2], hat[e], last_hat[e],
                                                                  self.rho_pi[e])
                        else:
                            rk_e, sk_e = pair_residuals(cfg, pos_old[v1], hat[e, 0], last_hat[e, 0])
                        if not g_alias[g]:
                            sk += sk_e
                        rk += rk_e
                    comp_r.append((rk, sk))
                seen = [e for e in edges if np.isfinite(dis_chk[e]) and cnt(e)]
                part = np.array([sum(r for r, _ in comp_r), sum(q for _, q in comp_r),
                                 float(sum(1 for e in act if cnt(e))),
                                 float(len(seen)), float(sum(1 for e in seen if not dis_chk[e] > d_eff[e]))])
                if cfg.term_global and reduce is not None:
                    part = np.asarray(reduce(part), np.float64)     # the all-reduce of the sharded path
                rk_g, sk_g, n_act, n_seen, n_bad = part
                if n_act == 0 and g_flag[g] == 0 and not cfg.fixed_iters:
                    g_done[g] = True        # no pair ever collided: stop before the residuals (:115-116)
                    continue
                g_flag[g] = 1
                for c, r in zip(gcomps, comp_r):
                    resid[c].append(r)
                if cfg.term_global:
                    global_resid.append((rk_g, sk_g))
                dist_ok = n_seen > 0 and n_bad == 0
                if not cfg.fixed_iters:
                    gid = -1 if cfg.term_global else int(gcomps[0])
                    self.ties.scalar(t, it, TIE_STOP, gid, 0, rk_g, cfg.eps_pri)
                    self.ties.scalar(t, it, TIE_STOP, gid, 1, sk_g, cfg.eps_dual)
                if (not cfg.fixed_iters and rk_g <= cfg.eps_pri and sk_g <= cfg.eps_dual
                        and (not cfg.term_dist_check or dist_ok)):
                    g_done[g] = True
                    continue
                # casadi/main.py:180 (alias, B4) / MATLAB :207 (copy)
                if cfg.alias_dual_residual:
                    g_alias[g] = True
                else:
                    last_hat[edges] = hat[edges]
            if on_iter is not None:
                on_iter(it, dict(pos_old=pos_old.copy(), hat=hat.copy(), lam=lam.copy(), S=S.copy(), D=D.copy(),
                                 stop=all(g_done)))
        self.edge_state = (hat.copy(), lam.copy(), S.copy(), D.copy(), last_hat.copy())
        # ---- propagation, casadi/main.py:185-192 (of the components that ran)
        new_xt = self.xt.copy()
        prop = np.arange(N) if components is None else np.concatenate([self.comp_agents[ci] for ci in comps])
        new_xt[prop] = propagate(cfg, self.xt[prop], self.primal_u[prop], self.scn.spd[prop])
        self.xt = new_xt
        self.t += 1
        return StepRecord(xt=new_xt.copy(), u=self.primal_u.copy(), iters=iters, resid=resid,
                          pos_old=pos_old, hat=hat, lam=lam, edge_active=active.copy(),
                          global_resid=global_resid)

    def run(self, n_steps=None):
        n_steps = self.scn.n_steps if n_steps is None else n_steps
        return [self.mpc_step() for _ in range(n_steps)]


def dual_update(cfg, p1, p2, hat_e, lam_e, S_e, D_e, dist):
    """In-place dual update of one pair (both directions).

    plain: ``casadi/main.py:161-162``; PI: ``ADMM_CVX_..._PI_antiwindup.m:160-166``;
    saturation / back-calculation: ``:169-188``.
    """
    ps = (p1, p2)
    if cfg.dual_mode == 0:
        for d in range(2):
            lam_e[d] += cfg.rho * (ps[d] - hat_e[d])
    else:
        kP = cfg.theta1 - cfg.theta2 / (1 + np.exp(-np.min(dist)))
        for d in range(2):
            err = ps[d] - hat_e[d]
            S_e[d] = S_e[d] + cfg.kI * err + D_e[d]
            lam_e[d] = S_e[d] + kP * err
    if cfg.windup:
        W = cfg.windup_sat
        for d in range(2):
            orig = lam_e[d].copy()
            lam_e[d] = np.minimum(W, np.maximum(lam_e[d], -W))
            if np.sum(orig != lam_e[d]) > 0:
                D_e[d] = lam_e[d] - orig
            else:
                D_e[d] = 0.0


def dual_update_global_pi(cfg, xt, spd, primal_u, v1, v2, pos_old, hat_e, lam_e, S_e, D_e, rho_pi, e):
    """Global PI with adaptive rho and K_P (``casadi_old_PI_ADMM/main.py:128-151``) for one pair,
    in place.  d = the pair's distances along the nonlinear rollouts of the x-step controls
    (``x_curr_pred``, :128-133); K_I = 3 (:135), K_P = min(theta1/d_min, theta2) (:136, 5 and
    2.5), the penalty rho = max(rho_min, min(rho_max, rho_num/d_min)) (:137); lam = S + K_P e,
    S += K_I e + 2 D (:141-142, S before its update); saturation with back-calculation over the
    pair (:145-151, ``np.sum(orig != sat) > 0`` over the whole dual array).  Returns dis_vec[1]
    (the stop check, :157).

    The adaptive-gain variant (``matlab_old_files/ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m:
    121-147``, preset matlab_adp_pi): K_I = K_I_coeff / d_min (``ki_adapt``, :127), K_P = min(5/d_min,
    3) (:128), S += K_I e + D (``d_gain`` 1, :135).  Both scripts' ``trad == 1`` branch
    (``pi_trad``; casadi_old :139-140, adp :131-132): lam += rho e + D with the updated rho, then
    the same saturation."""
    x1, y1, _ = rollout_nonlinear(xt[v1], primal_u[v1], spd[v1], cfg.dt, cfg.L)
    x2, y2, _ = rollout_nonlinear(xt[v2], primal_u[v2], spd[v2], cfg.dt, cfg.L)
    dx, dy = x1 - x2, y1 - y2
    dist = np.sqrt(dx * dx + dy * dy)
    dmin = np.min(dist)
    kI = cfg.kI / dmin if cfg.ki_adapt else cfg.kI
    kP = min(cfg.theta1 / dmin, cfg.theta2)
    rho_pi[e] = max(cfg.rho_min, min(cfg.rho_max, cfg.rho_num / dmin))
    raw = np.empty_like(lam_e)
    for d, v in enumerate((v1, v2)):
        err = pos_old[v] - hat_e[d]
        if cfg.pi_trad:
            raw[d] = lam_e[d] + rho_pi[e] * err + D_e[d]
            continue
        raw[d] = S_e[d] + kP * err
        S_e[d] = S_e[d] + kI * err + cfg.d_gain * D_e[d]
    if cfg.windup:
        W = cfg.windup_sat
        sat = np.minimum(W, np.maximum(raw, -W))
        D_e[...] = (sat - raw) if np.sum(raw != sat) > 0 else 0.0
        lam_e[...] = sat
    else:
        lam_e[...] = raw
    return dist[1]


def pair_residuals_global_pi(p_v1, p_v2, hat_e, last_e, rho):
    """One pair's terms of ``casadi_old_PI_ADMM/main.py:153-154``: (primal, dual) =
    (|[p_1; p_2] - [hat_12; hat_21]|_F, |rho ([last_12; last_21] - [hat_12; hat_21])|_F) -- both
    sides, no factor 2 (unlike casadi/main.py:170-173), rho the pair's updated penalty."""
    pos = np.concatenate([p_v1, p_v2])                 # (4, H+1): the script's 2N x (H+1) layout
    hat = hat_e.reshape(4, -1)
    sk = np.sqrt(np.sum((rho * (last_e.reshape(4, -1) - hat)) ** 2))
    rk = np.sqrt(np.sum((pos - hat) ** 2))
    return rk, sk


def candidate_pairs(xy, radius, block=2048):
    """All pairs i < j with |xy_i - xy_j|^2 <= (r_i + r_j)^2 in (i, j) order -- the brute-force
    statement of the candidate graph (the all-pairs loop of casadi/main.py:110-113 over the
    reach discs; checker of piadmm_candidate_pairs), same fp64 operations as the kernel."""
    xy = np.asarray(xy, np.float64).reshape(-1, 2)
    r = np.asarray(radius, np.float64).reshape(-1)
    n = xy.shape[0]
    out = []
    for a in range(0, n, block):
        i = np.arange(a, min(n, a + block))
        dx = xy[None, :, 0] - xy[i, None, 0]
        dy = xy[None, :, 1] - xy[i, None, 1]
        d2 = dx * dx + dy * dy
        rr = (r[i, None] + r[None, :]) * (r[i, None] + r[None, :])
        ok = (d2 <= rr) & (np.arange(n)[None, :] > i[:, None])
        ii, jj = np.nonzero(ok)
        out.append(np.stack([i[ii], jj], 1))
    return np.concatenate(out).astype(np.int32) if out else np.zeros((0, 2), np.int32)
