"""Per-step, per-tile pair-QP work for the bench workload (development tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd'))
import numpy as np
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = 30
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=100)
scn = scenario.tiled(128, H, n_steps=12)
s = PI_ADMM_MI355X(cfg, scn)
for t in range(10):
    s.reset_counters()
    ms = s.time_steps(t, 1)
    cc = s.component_counters()
    w = int(np.argmax(cc[:, 4] + 50 * cc[:, 6]))
    print(f"step {t}: {ms:.2f} ms  zqp tot {cc[:,2].sum()}  admm_z mean {cc[:,4].mean():.1f} max {cc[:,4].max()}  pdas_z max {cc[:,6].max()}  admm_x max {cc[:,3].max()} pdas_x max {cc[:,5].max()} inexact {cc[:,7].sum()}  worst tile {w}: {cc[w].tolist()}")
