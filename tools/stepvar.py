"""Per-step, per-component kernel cycles (stamps build): how much a persistent multi-step
launch could save (sum over steps of the per-step max vs the max over components of the sum)."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd'))
os.environ.setdefault('PIADMM_LIB', os.path.join(ROOT, 'distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_stamps.so'))
import numpy as np
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
H = int(sys.argv[1]) if len(sys.argv) > 1 else 30
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=100)
scn = scenario.tiled(128, H, n_steps=steps + 2)
s = PI_ADMM_MI355X(cfg, scn)
buf = (ctypes.c_uint64 * (s.C * 64))()
prev = np.zeros(s.C)
rows = []
for t in range(steps):
    ms = s.time_steps(t, 1)
    s._check(s.lib.piadmm_debug_stamps(s._h, buf, s.C * 64))
    k = np.array(buf, dtype=np.float64).reshape(s.C, 64)[:, 9]
    rows.append(k - prev)
    prev = k
    print(f"t={t:2d} {ms:6.2f} ms  max {rows[-1].max():10.0f} mean {rows[-1].mean():10.0f} argmax {rows[-1].argmax()}", flush=True)
R = np.array(rows)
print(f"sum_t max_c = {R.max(1).sum():.4g}   max_c sum_t = {R.sum(0).max():.4g}   mean_c sum_t = {R.sum(0).mean():.4g}")
print(f"ratio (persistent gain bound) = {R.max(1).sum() / R.sum(0).max():.3f}")
