"""Candidate-pair graph for large N.

The reference collision-tests every pair of vehicles in every outer iteration
(``casadi/main.py:110-113``, O(N^2 H)).  The solver takes a static candidate graph; this module
builds it in O(N) on the GPU (``piadmm_candidate_pairs``, a uniform grid hash): all pairs whose
reach discs overlap, |p_i - p_j| <= r_i + r_j, with r_i a bound on how far agent i's planned
positions can get from its current position within the horizon plus half the collision
distance.  No pair outside the graph can then collide within the horizon, so the per-iteration
collision test over the candidates finds every colliding pair the all-pairs test would.  A
receding-horizon planner rebuilds the graph every MPC step from the current states
(:meth:`PI_ADMM_MI355X.set_candidate_graph`).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

from . import _lib


def reach_radii(cfg, spd, theta=None) -> np.ndarray:
    """Per-agent reach radius for the candidate test.

    pos_old is the x-step's rollout (``pos_model`` 0: the linearised ``dynamic_update_local``,
    PI_ADMM_class.py:59-69, whose step k has length dt s sqrt(1 + (theta_k - theta_0)^2) with
    |theta_k - theta_0| <= k dt s u_max / L; 1: the nonlinear model, step length dt s), so
    |p_k - p_0| <= sum_k dt s sqrt(1 + (k dt s u_max / L)^2).  Plus half the collision distance
    (sqrt(dis_thres) for the Python test d^2 < dis_thres, quirk B2; dis_thres for MATLAB's) and,
    with ``tighten``, the agent's delay offset |delta| (decentralized/util.py:81-96) at heading
    ``theta`` (the worst heading when None): MATLAB's test adds |delta_i| per agent; the Python
    test's distance sqrt(dis_thres + |delta_i| + |delta_j|) is bounded by half of
    sqrt(dis_thres + 2 max |delta|) per agent."""
    spd = np.asarray(spd, np.float64)
    H, dt = cfg.H, cfg.dt
    k = np.arange(H, dtype=np.float64)
    if cfg.pos_model == 0:
        w = dt * spd[:, None] * k[None, :] * cfg.u_max / cfg.L
        reach = np.sum(dt * spd[:, None] * np.sqrt(1.0 + w * w), axis=1)
    else:
        reach = H * dt * spd
    dcol = cfg.dis_thres if cfg.collide_sq_thres else math.sqrt(cfg.dis_thres)
    r = reach + 0.5 * dcol
    if cfg.tighten:
        kap = math.sqrt(cfg.tight_p / (1.0 - cfg.tight_p))
        if theta is None:
            d = np.hypot(cfg.avg_delay * spd + kap * (cfg.var_delay * spd) ** 2,
                         cfg.avg_delay * spd + kap * (cfg.var_delay * spd) ** 2)
        else:
            c, s = np.cos(theta), np.sin(theta)
            d = np.hypot(cfg.avg_delay * spd * c + kap * (cfg.var_delay * spd * c) ** 2,
                         cfg.avg_delay * spd * s + kap * (cfg.var_delay * spd * s) ** 2)
        if cfg.collide_sq_thres:
            r = r + d               # MATLAB test d < d_eff = dis_thres + |delta_i| + |delta_j|
        else:
            # Python test d^2 < d_eff (quirk B2): the collision distance sqrt(dis_thres + |delta_i| +
            # |delta_j|) is at most sqrt(dis_thres + 2 max |delta|), split evenly over the pair (the
            # per-agent 0.5 sqrt(dis_thres) + |delta_i| bounds it only when 2 sqrt(dis_thres) + delta >= 1)
            r = reach + 0.5 * math.sqrt(cfg.dis_thres + 2.0 * float(np.max(d)) if d.size else cfg.dis_thres)
    # a little slack over the rounding of the positions (u rounded to 1e-4, B6)
    return r * (1.0 + 1e-9) + 1e-9


def candidate_pairs(solver, xy: np.ndarray, radius: np.ndarray, with_time: bool = False):
    """All pairs i < j with |xy_i - xy_j| <= radius_i + radius_j, (E, 2) int32 in (i, j) order,
    computed on the solver's GPU (piadmm_candidate_pairs).  ``with_time``: also the device time
    (ms) of the detection kernels."""
    lib, h = solver.lib, solver._h
    xy = np.ascontiguousarray(xy, np.float64).reshape(-1, 2)
    radius = np.ascontiguousarray(radius, np.float64).reshape(-1)
    n = xy.shape[0]
    if radius.shape[0] != n:
        raise ValueError("one radius per point")
    cap = max(4 * n, 16)
    for _ in range(2):
        out = np.empty((cap, 2), np.int32)
        tot = ctypes.c_int32()
        ms = ctypes.c_float()
        _lib.check(lib.piadmm_candidate_pairs(h, _lib.dptr(xy), _lib.dptr(radius), n, _lib.iptr(out), cap,
                                              ctypes.byref(tot), ctypes.byref(ms)), h)
        if tot.value <= cap:
            pairs = out[:tot.value].copy()
            return (pairs, float(ms.value)) if with_time else pairs
        cap = tot.value
    raise RuntimeError("candidate pair count changed between calls")
