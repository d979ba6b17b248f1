"""Per-MPC-step work and QP status of the bench workload (development tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd'))
import numpy as np
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = int(sys.argv[1]) if len(sys.argv) > 1 else 30
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=100)
scn = scenario.tiled(128, H, n_steps=steps + 2, perturb=True, seed=0)
s = PI_ADMM_MI355X(cfg, scn)
for t in range(steps):
    s.reset_counters()
    ms = s.time_steps(t, 1)
    cc = s.component_counters()   # outer, x_qps, z_qps, admm_x, admm_z, pdas_x, pdas_z, inexact
    bad = np.nonzero(cc[:, 7])[0]
    print(f"t={t:2d} {ms:7.2f} ms  zqp {cc[:,2].sum():4d}  admm_x max {cc[:,3].max():6d} admm_z max {cc[:,4].max():5d} "
          f"pdas_z max {cc[:,6].max():3d} inexact {cc[:,7].sum():3d} comps {bad[:8].tolist()}", flush=True)
