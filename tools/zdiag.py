"""Per-tile pair-QP work at MPC step 0 (development tool)."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd'))
import numpy as np
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = 30
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=1)
scn = scenario.tiled(128, H, n_steps=3)
s = PI_ADMM_MI355X(cfg, scn)
s.reset_counters()
r = s.mpc_step(0)
cc = s.component_counters()
order = np.argsort(-cc[:, 4])
print("per-tile [outer, xqp, zqp, admm_x, admm_z, pdas_x, pdas_z, inexact] worst by admm_z:")
for i in order[:8]:
    print(i, cc[i].tolist())
print("mean admm_z", cc[:, 4].mean(), "mean pdas_z", cc[:, 6].mean(), "status", np.unique(r.status).tolist())
np.save(os.path.join(ROOT, 'gpurun_out', 'zdiag_u.npy'), r.u)
