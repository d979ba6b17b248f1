"""Per-outer-iteration cost of the x-step path without pair QPs (dis_thres tiny: the collision
test never fires) and with them: (time at max_outer=200 - time at 100) / 100 per step."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd'))
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = int(sys.argv[1]) if len(sys.argv) > 1 else 30
K = 10
for thres in (1e-9, None):
    res = {}
    for M in (100, 200):
        kw = dict(H=H, fixed_iters=1, max_outer=M, term_global=1)
        if thres is not None:
            kw["dis_thres"] = thres
        cfg = config.matlab_pi(**kw)
        scn = scenario.tiled(128, H, n_steps=K + 2, perturb=True, seed=0)
        with PI_ADMM_MI355X(cfg, scn) as s:
            s.steps_async(0, 2); s.sync()
            s.set_xt(scn.xt0)
            s.reset_counters()
            ms = s.time_steps(0, K)
            res[M] = (ms / K, s.counters())
    per_it_us = (res[200][0] - res[100][0]) / 100 * 1e3
    print(f"dis_thres={thres}: step ms M=100 {res[100][0]:.3f}  M=200 {res[200][0]:.3f}  "
          f"per outer iteration {per_it_us:.2f} us = {per_it_us*2.4e3:.0f} cycles @2.4GHz; z_qps {res[100][1]['z_qps']}", flush=True)
