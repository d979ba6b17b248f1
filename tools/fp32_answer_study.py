"""configs[4] fp32 tolerance study of the ANSWER path (CPU, oracle-based; not shipped).

What would fp32 arithmetic in the QP answers do to the planner at 256 agents x H = 50 with delay
tightening?  For every QP of the loop the oracle finds the exact fp64 working set; the answer on
that working set is then computed three ways and fed to the rest of the loop (rounding, rollouts,
collision test, dual update, residuals, termination -- all fp64 as on the GPU):
  fp64        the KKT system of the working set solved in fp64 (= the oracle / GPU answer)
  fp32        the same KKT system assembled and solved in fp32 (an fp32 answer path)
  fp32+ir     fp32 solve + one step of fp64 iterative refinement (residual in fp64, correction
              solved with the fp32 factorisation) -- the mixed-precision design
Reports max |du|, max relative dxt and the outer-iteration-count changes against fp64 over
sampled tiles of the bench's H = 50 tightening workload.

usage: python tools/fp32_answer_study.py [tiles=6] [steps=10] [H=50] > profiles/fp32_answer_study_r02.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
import numpy as np  # noqa: E402

from oracle import piadmm_oracle as O  # noqa: E402
from piadmm import config, scenario  # noqa: E402

tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 6
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H = int(sys.argv[3]) if len(sys.argv) > 3 else 50

_solve_x, _solve_e = O.solve_xstep, O.solve_edge
MODE = ["fp64"]
STATS = {"qps": 0, "max_rel_err_fp32": 0.0, "max_rel_err_ir": 0.0}


def kkt_answer(P, q, A, lo, hi, x, y):
    """x on x's working set (rows at a bound with a nonzero multiplier, or at a bound) in MODE."""
    ax = A @ x
    scale = 1.0 + np.abs(lo[np.isfinite(lo)]).max(initial=0.0)
    at = (np.abs(ax - lo) <= 1e-9 * scale) | (np.abs(ax - hi) <= 1e-9 * scale)
    rows = np.nonzero(at)[0]
    b = np.where(np.abs(ax[rows] - lo[rows]) <= np.abs(ax[rows] - hi[rows]), lo[rows], hi[rows])
    n, m = P.shape[0], rows.size
    K = np.zeros((n + m, n + m))
    K[:n, :n] = P
    K[:n, n:] = A[rows].T
    K[n:, :n] = A[rows]
    rhs = np.concatenate([-q, b])
    z64 = np.linalg.lstsq(K, rhs, rcond=None)[0]
    if MODE[0] == "fp64":
        return z64[:n]
    K32, r32 = K.astype(np.float32), rhs.astype(np.float32)
    z = np.linalg.lstsq(K32, r32, rcond=None)[0].astype(np.float64)
    err = np.max(np.abs(z[:n] - z64[:n])) / (1.0 + np.max(np.abs(z64[:n])))
    STATS["max_rel_err_fp32"] = max(STATS["max_rel_err_fp32"], float(err))
    if MODE[0] == "fp32+ir":
        res = rhs - K @ z                                   # fp64 residual
        z = z + np.linalg.lstsq(K32, res.astype(np.float32), rcond=None)[0].astype(np.float64)
        err = np.max(np.abs(z[:n] - z64[:n])) / (1.0 + np.max(np.abs(z64[:n])))
        STATS["max_rel_err_ir"] = max(STATS["max_rel_err_ir"], float(err))
    STATS["qps"] += 1
    return z[:n]


def solve_xstep(cfg, xt_i, s_i, ref_i, nbr_terms):
    x, data = _solve_x(cfg, xt_i, s_i, ref_i, nbr_terms)
    P, q, A, lo, hi, y = data
    return kkt_answer(P, q, A, lo, hi, x, y), data


def solve_edge(*a, **k):
    uh, data = _solve_e(*a, **k)
    P, q, A, lo, hi, x, y = data
    xx = kkt_answer(P, q, A, lo, hi, x, y)
    H_ = uh.shape[1]
    return xx[:2 * H_].reshape(2, H_), data


O.solve_xstep, O.solve_edge = solve_xstep, solve_edge
cfg = config.matlab_pi(H=H, tighten=1)
full = scenario.tiled(128, H, n_steps=steps + 1, seed=0)
pick = np.linspace(0, 127, tiles).astype(int)
runs = {}
t0 = time.time()
for mode in ("fp64", "fp32", "fp32+ir"):
    MODE[0] = mode
    xs, us, its = [], [], []
    for k in pick:
        sub = scenario.Scenario(spd=full.spd[2 * k:2 * k + 2], xt0=full.xt0[2 * k:2 * k + 2],
                                ref=full.ref[2 * k:2 * k + 2], edges=np.array([[0, 1]], np.int32),
                                n_steps=full.n_steps)
        orc = O.Oracle(cfg, sub)
        for _ in range(steps):
            r = orc.mpc_step()
            xs.append(r.xt)
            us.append(r.u)
            its.append(int(r.iters[0]))
    runs[mode] = (np.array(xs), np.array(us), np.array(its))
a = runs["fp64"]
out = {"workload": f"{tiles} of 128 tiles of the H={H} tightening workload (configs[4]), MPC steps 0..{steps - 1}, "
                   "natural termination, matlab_pi + tighten", "qps_per_mode": STATS["qps"] // 2,
       "max_rel_answer_err": {"fp32": STATS["max_rel_err_fp32"], "fp32+ir": STATS["max_rel_err_ir"]},
       "seconds": time.time() - t0}
for mode in ("fp32", "fp32+ir"):
    b = runs[mode]
    out[mode] = {"max_abs_du": float(np.max(np.abs(a[1] - b[1]))),
                 "max_rel_dxt": float(np.max(np.abs(a[0] - b[0]) / (1 + np.abs(a[0])))),
                 "iteration_count_changes": int(np.sum(a[2] != b[2])),
                 "steps": int(a[2].size)}
out["contract"] = "north_star: 1e-5 relative on state/control vectors"
print(json.dumps(out, indent=1))
