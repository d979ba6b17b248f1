"""Development diagnostic (not shipped): per-step comparison of the GPU (graph mode) with the
oracle on an N-vehicle crossing -- iteration counts, QP status, work counters, deviations.

usage: python tools/graph_diag.py [n] [preset] [pairs] [H] [steps] [seed] [--no-oracle]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
import numpy as np  # noqa: E402

from oracle import piadmm_oracle as O  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
use_orc = "--no-oracle" not in sys.argv
n = int(args[0]) if len(args) > 0 else 3
preset = args[1] if len(args) > 1 else "matlab_pi"
pairs = args[2] if len(args) > 2 else "all"
H = int(args[3]) if len(args) > 3 else 15
steps = int(args[4]) if len(args) > 4 else 12
cfg = config.PRESETS[preset](H=H)
seed = int(args[5]) if len(args) > 5 else None
scn = scenario.crossing(n, H, n_steps=30, pairs=pairs, seed=seed)
orc = O.Oracle(cfg, scn) if use_orc else None
with PI_ADMM_MI355X(cfg, scn) as s:
    for k in range(steps):
        s.reset_counters()
        rg = s.mpc_step()
        cnt = s.counters()
        line = f"step {k}: gpu iters {rg.iters.tolist()} status {rg.status.tolist()} cnt {cnt}"
        if orc is not None:
            ro = orc.mpc_step()
            dx = float(np.max(np.abs(ro.xt - rg.xt)))
            du = float(np.max(np.abs(ro.u - rg.u)))
            line += f" | oracle iters {ro.iters.tolist()} dxt {dx:.2e} du {du:.2e}"
        print(line, flush=True)
        if orc is not None:
            st = s.state()
            print("   edge_active gpu", st["edge_active"].tolist(), "oracle", ro.edge_active.astype(int).tolist(),
                  "dhat %.2e dlam %.2e dpos %.2e" % (np.max(np.abs(st["hat"] - ro.hat)), np.max(np.abs(st["lam"] - ro.lam)),
                                                     np.max(np.abs(st["pos_old"] - ro.pos_old))), flush=True)
