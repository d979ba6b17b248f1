"""Development diagnostic (not shipped): one connected chain split over workgroups vs the single-
workgroup run vs the B-opt CPU baseline."""
import os
import sys
sys.path[:0] = ['.', 'distributed-local-planner-pi-admm_amd']
import numpy as np  # noqa: E402
from oracle import cpu_bopt  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X as S  # noqa: E402
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
H = int(sys.argv[2]) if len(sys.argv) > 2 else 30
M = int(sys.argv[3]) if len(sys.argv) > 3 else 100
cfg = config.matlab_pi(H=H, term_global=1, fixed_iters=1, max_outer=M)
scn = scenario.crossing(N, H, n_steps=4, seed=2, pairs="chain")
rc = cpu_bopt.run(cfg, scn, 2, threads=4)
print("bopt counters", rc["counters"], flush=True)
s1 = S(cfg, scn)
os.environ["PIADMM_GRAPH_BLOCK"] = "0"
s2 = S(cfg, scn)
del os.environ["PIADMM_GRAPH_BLOCK"]
for k in range(2):
    r1, r2 = s1.mpc_step(), s2.mpc_step()
    d1 = np.max(np.abs(r1.u - rc["u"][k]), axis=1)
    d2 = np.max(np.abs(r2.u - rc["u"][k]), axis=1)
    print(k, "split vs bopt", d1.max(), np.nonzero(d1 > 1e-8)[0][:20], "status", np.nonzero(r1.status)[0][:10], flush=True)
    print(k, "single vs bopt", d2.max(), np.nonzero(d2 > 1e-8)[0][:20], "status", np.nonzero(r2.status)[0][:10],
          r2.status[np.nonzero(r2.status)[0][:10]], flush=True)
print(s1.counters(), s2.counters())
