"""Step time against the outer-iteration count M (fixed iterations, bench workload): where in the
step the time goes (the collision event, the first iterations, the steady state)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd'))
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = 30
K = 10
prev = 0.0
for M in (1, 2, 3, 4, 5, 6, 8, 10, 20, 50, 100):
    cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=M, term_global=1)
    scn = scenario.tiled(128, H, n_steps=K + 2, perturb=True, seed=0)
    with PI_ADMM_MI355X(cfg, scn) as s:
        s.steps_async(0, 2); s.sync()
        s.set_xt(scn.xt0)
        s.reset_counters()
        ms = s.time_steps(0, K)
        cnt = s.counters()
    print(f"M={M:4d} step ms {ms / K:.4f}  delta {ms / K - prev:+.4f}  z_qps/comp/step {cnt['z_qps'] / 128 / K:.2f} "
          f"pdas_x/xqp {cnt['pdas_x'] / max(cnt['x_qps'], 1):.3f} admm_x {cnt['admm_x']} inexact {cnt['inexact']}", flush=True)
    prev = ms / K
