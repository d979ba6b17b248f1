"""Golden runs of the NumPy oracle on coupled jobs whose pair QPs need more than 63 active rows
(TEST INFRASTRUCTURE), at H = 40, matlab_pi preset, per-component termination, 12 MPC steps:

  run_matlab_pi_H40_crossing4  the 4-vehicle all-pairs crossing -- saturated pair QPs (both
                               vehicles' controls and rates at their bounds plus hinge kinks:
                               78-79 active rows at some optima) from step 0 on
  run_matlab_pi_H40_mixed      tests/test_gpu_graph.py::test_mixed_components_and_horizons[40]:
                               two intersection tiles, a 3-vehicle chain (a pair QP beyond 63
                               rows at step 5), the two-vehicle intersection, a lone vehicle
  run_matlab_pi_H63_tiled2     the lane limit H = 63 (tests/test_gpu_parity.py
                               test_largest_horizon_against_the_oracle): two seeded intersection
                               tiles, 8 MPC steps (pair QPs of 189 variables in slack form)

Every QP of these runs is certified: oracle/qp_exact.py's solve() raises unless its answer passes
the complete KKT certificate (stationarity, feasibility of every row, dual signs, complementarity
at 1e-9 relative).  Round 4's solver did not certify, and this crossing's step-5 pair QP came out
infeasible: the fixture was regenerated with the certifying solver (steps 5-11 changed; B-opt
now equals it at 1e-8 on every step, tests/test_cpu_bopt.py).

The oracle takes minutes for them, too long for a live GPU test; tests/test_gpu_graph.py
compares libpiadmm's wide dual active set (csrc/pd_qp.h gi_solve_wide) against these files,
and tests/test_oracle_golden.py re-derives the crossing's first step from the oracle.

  tests/golden/<name>.npz
    xt (K, N, 3), u (K, N, H), iters (K, C), resid (K, C, max_outer, 2) (NaN beyond iters),
    pos_old / hat / lam / edge_active after the last step

Usage: python oracle/gen_golden_wide.py [name ...]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))

from oracle import piadmm_oracle as O  # noqa: E402
from piadmm import config, scenario  # noqa: E402

H, K = 40, 12
NAME = "run_matlab_pi_H40_crossing4"
MIXED = "run_matlab_pi_H40_mixed"
H63 = "run_matlab_pi_H63_tiled2"
STEPS = {NAME: K, MIXED: K, H63: 8}


def make(name=NAME):
    if name == H63:
        return config.matlab_pi(H=63), scenario.tiled(2, 63, n_steps=12, seed=1)
    if name == NAME:
        return config.matlab_pi(H=H), scenario.crossing(4, H, n_steps=K + 2, seed=1)
    if name == MIXED:
        scn = scenario.concat([scenario.tiled(2, H, n_steps=K + 2, seed=3),
                               scenario.crossing(3, H, n_steps=K + 2, pairs="chain"),
                               scenario.intersection(H, n_steps=K + 2), scenario.crossing(1, H, n_steps=K + 2)])
        return config.matlab_pi(H=H), scn
    raise KeyError(name)


def run(name=NAME, n_steps=None):
    cfg, scn = make(name)
    n_steps = STEPS[name] if n_steps is None else n_steps
    H = cfg.H
    orc = O.Oracle(cfg, scn)
    M = cfg.max_outer
    out = {k: [] for k in ("xt", "u", "iters", "resid")}
    for _ in range(n_steps):
        r = orc.mpc_step()
        out["xt"].append(r.xt.copy())
        out["u"].append(r.u.copy())
        out["iters"].append(np.asarray(r.iters, np.int32).copy())
        rs = np.full((orc.n_comp, M, 2), np.nan)
        for c in range(orc.n_comp):
            if len(r.resid[c]):
                rs[c, :len(r.resid[c])] = np.asarray(r.resid[c])
        out["resid"].append(rs)
    res = {k: np.stack(v) for k, v in out.items()}
    res.update(pos_old=r.pos_old.copy(), hat=r.hat.copy(), lam=r.lam.copy(),
               edge_active=np.asarray(r.edge_active, np.uint8).copy(), H=np.int32(H), n_steps=np.int32(n_steps))
    return res


if __name__ == "__main__":
    for name in sys.argv[1:] or [NAME, MIXED, H63]:
        res = run(name)
        path = os.path.join(ROOT, "tests", "golden", name + ".npz")
        np.savez_compressed(path, **res)
        print("wrote", path, {k: v.shape for k, v in res.items()}, flush=True)
