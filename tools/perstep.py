import os, sys
sys.path.insert(0, 'distributed-local-planner-pi-admm_amd')
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = 30; K = 10
for M in (1, 100):
    cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=M, term_global=1)
    scn = scenario.tiled(128, H, n_steps=K + 2, perturb=True, seed=0)
    with PI_ADMM_MI355X(cfg, scn) as s:
        s.steps_async(0, 2); s.sync()
        s.set_xt(scn.xt0)
        prev = None
        for t in range(K):
            s.reset_counters()
            ms = s.time_steps(t, 1)
            c = s.counters()
            print(M, t, f"{ms:.4f}", {k: v for k, v in c.items() if k not in ('outer_iters',)}, flush=True)
