"""Development diagnostic (not shipped): per-phase cycle breakdown of k_graph_step on the
1024-agent chain (bench.py --chain), the blocks' stamps of steps t0 .. t0+n-1 only (the stamps
accumulated over the earlier steps are subtracted), diagnostic stamps build.

    PIADMM_LIB=.../libpiadmm_stamps.so python tools/chain_stamps.py [t0] [n]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"), os.path.join(ROOT, "tools")]
os.environ.setdefault("PIADMM_LIB", os.path.join(ROOT, "distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_stamps.so"))
import numpy as np  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

t0 = int(sys.argv[1]) if len(sys.argv) > 1 else 17
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H = 30
NAMES = {2: "X phase", 3: "x qp", 6: "Z phase", 7: "z qp", 9: "kernel", 29: "gi_search", 30: "gi_solve",
         31: "gi_upd", 21: "zr_gemv/warm", 22: "zr_S/warmfeas", 23: "zr_chol", 24: "zr_x", 25: "zr_solve",
         27: "zkkt", 1: "setup_z", 20: "sz_pre"}
COUNTS = {40: "gi steps z", 42: "z qps", 49: "z drops", 50: "z appends", 51: "z warm rows", 52: "z sum m",
          53: "z sum m end", 54: "z gi ok"}
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=100, term_global=1)
scn = scenario.crossing(1024, H, n_steps=t0 + n + 2, seed=1, pairs="chain")
s = PI_ADMM_MI355X(cfg, scn)


def stamps():
    buf = (ctypes.c_uint64 * (s.C * 64))()
    s._check(s.lib.piadmm_debug_stamps(s._h, buf, s.C * 64))
    return np.array(buf, dtype=np.float64).reshape(s.C, 64)


for _ in range(t0):
    s.mpc_step()
a = stamps()
c0 = s.component_counters().astype(np.int64)
for _ in range(n):
    s.mpc_step()
st = stamps() - a
cc = s.component_counters().astype(np.int64) - c0
print(f"chain 1024 H={H} steps {t0}..{t0 + n - 1}, blocks={s.C}")
for i, nm in NAMES.items():
    print(f"  {nm:14s} mean cycles/block/step {st[:, i].mean() / n:12.0f}  max {st[:, i].max() / n:12.0f}")
for i, nm in COUNTS.items():
    print(f"  {nm:14s} sum over blocks /step {st[:, i].sum() / n:10.1f}  max block {st[:, i].max() / n:8.1f}")
order = np.argsort(-st[:, 7])
print("blocks with the most z-qp cycles (per step): zqp giz_steps zqps drops appends warm sum_m | z_qps pdas_z")
for k in order[:8]:
    print(f"  block {k:4d}: " + " ".join(f"{st[k, j] / n:10.0f}" for j in (7, 40, 42, 49, 50, 51, 52)) +
          f" | {cc[k, 2] / n:5.1f} {cc[k, 6] / n:5.1f}")
s.close()
