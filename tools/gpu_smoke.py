"""Quick GPU-vs-oracle comparison (development tool)."""
import sys, time
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/distributed-local-planner-pi-admm_amd')
import numpy as np
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
from oracle import piadmm_oracle as O

def compare(name, cfg, scn, n_steps):
    orc = O.Oracle(cfg, scn)
    gpu = PI_ADMM_MI355X(cfg, scn)
    worst = 0.0; itmis = 0
    for s in range(n_steps):
        ro = orc.mpc_step(); rg = gpu.mpc_step()
        dx = np.abs(ro.xt - rg.xt).max() / (1 + np.abs(ro.xt).max())
        du = np.abs(ro.u - rg.u).max()
        worst = max(worst, dx, du)
        itmis += int(np.sum(ro.iters != rg.iters))
        if s < 3 or dx > 1e-6 or du > 1e-6:
            print(f"  {name} step {s}: dxt {dx:.2e} du {du:.2e} iters o={ro.iters[:4].tolist()} g={rg.iters[:4].tolist()} status={np.unique(rg.status).tolist()}")
    print(f"{name}: worst rel {worst:.3e}, iteration mismatches {itmis}")
    gpu.close()
    return worst

if __name__ == '__main__':
    compare('casadi_default H10', config.casadi_default(H=10), scenario.intersection(10), 40)
    compare('matlab_pi H10', config.matlab_pi(H=10), scenario.intersection(10), 40)
    compare('matlab_pi H30 tiled4', config.matlab_pi(H=30), scenario.tiled(4, 30), 20)
    cfg = config.matlab_pi(H=30, fixed_iters=1, max_outer=20)
    compare('matlab_pi H30 tiled2 fixed20', cfg, scenario.tiled(2, 30), 12)
