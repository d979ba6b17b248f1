"""Development diagnostic (not shipped): per-step comparison of the GPU (graph mode) with the
oracle on an N-vehicle crossing -- iteration counts, QP status, work counters, deviations."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
import numpy as np  # noqa: E402

from oracle import piadmm_oracle as O  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
preset = sys.argv[2] if len(sys.argv) > 2 else "matlab_pi"
pairs = sys.argv[3] if len(sys.argv) > 3 else "all"
H = int(sys.argv[4]) if len(sys.argv) > 4 else 15
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 12
cfg = config.PRESETS[preset](H=H)
scn = scenario.crossing(n, H, n_steps=30, pairs=pairs)
orc = O.Oracle(cfg, scn)
with PI_ADMM_MI355X(cfg, scn) as s:
    for k in range(steps):
        s.reset_counters()
        ro, rg = orc.mpc_step(), s.mpc_step()
        cnt = s.counters()
        dx = float(np.max(np.abs(ro.xt - rg.xt)))
        du = float(np.max(np.abs(ro.u - rg.u)))
        print(f"step {k}: iters oracle {ro.iters.tolist()} gpu {rg.iters.tolist()} status {rg.status.tolist()} "
              f"dxt {dx:.2e} du {du:.2e} cnt {cnt}", flush=True)
        st = s.state()
        print("   edge_active gpu", st["edge_active"].tolist(), "oracle", ro.edge_active.astype(int).tolist(),
              "dhat %.2e dlam %.2e dpos %.2e" % (np.max(np.abs(st["hat"] - ro.hat)), np.max(np.abs(st["lam"] - ro.lam)),
                                                 np.max(np.abs(st["pos_old"] - ro.pos_old))), flush=True)
