"""Development diagnostic (not shipped): per-phase cycle breakdown of k_graph_step on the
coupling-heavy crossing workload (diagnostic stamps build, libpiadmm_stamps.so).

  python tools/graph_stamps.py [n_crossings] [H] [steps] [fixed|natural] [all|chain]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
os.environ.setdefault("PIADMM_LIB", os.path.join(ROOT, "distributed-local-planner-pi-admm_amd/piadmm/libpiadmm_stamps.so"))
import numpy as np  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

NAMES = {0: "setup_x", 1: "setup_z", 2: "X phase", 3: "x qp", 6: "Z phase", 7: "z qp", 9: "kernel",
         16: "T phase", 29: "gi_search", 30: "gi_solve", 31: "gi_upd", 21: "zr_gemv/warm", 22: "zr_S/warmfeas",
         23: "zr_chol", 24: "zr_x", 25: "zr_solve", 26: "xr_solve", 27: "zkkt", 28: "xkkt", 10: "red_gemv",
         11: "red_S", 12: "red_chol", 13: "red_x", 14: "admm", 32: "sync after X", 34: "sync after Z",
         35: "rsx_pre", 18: "sz_kmat", 19: "sz_gj", 20: "sz_pre", 17: "sz_ruiz"}
NAMES.update({45: "gi fwd (z)", 46: "gi bwd (z)", 47: "gi Ypass (z)", 48: "gi drop (z)"})
COUNTS = {40: "gi steps z", 41: "gi steps x", 42: "z qps", 43: "z inexact", 44: "x setup rebuilds",
          49: "z drops", 50: "z appends", 51: "z warm rows", 52: "z sum m/step", 53: "z sum m end", 54: "z gi ok"}

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H = int(sys.argv[2]) if len(sys.argv) > 2 else 30
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
natural = len(sys.argv) > 4 and sys.argv[4] == "natural"
pairs = sys.argv[5] if len(sys.argv) > 5 else "all"
cfg = config.matlab_pi(H=H, fixed_iters=0 if natural else 1, max_outer=100, term_global=int(natural))
scn = scenario.concat([scenario.crossing(4, H, n_steps=steps + 2, seed=k, pairs=pairs) for k in range(n)])
s = PI_ADMM_MI355X(cfg, scn)
s.reset_counters()
ms = s.time_steps(0, steps)
cnt = s.counters()
buf = (ctypes.c_uint64 * (s.C * 64))()
s._check(s.lib.piadmm_debug_stamps(s._h, buf, s.C * 64))
st = np.array(buf, dtype=np.float64).reshape(s.C, 64)
cc = s.component_counters()
print(f"crossings={n} H={H} steps={steps} natural={natural} pairs={pairs} event_ms={ms:.3f} "
      f"({ms / steps:.3f} ms/step, {1e3 * ms / steps / max(cnt['outer_iters'] / s.C / steps, 1):.1f} us/iter) {cnt}")
tot = st[:, 9].mean()
for i, nm in NAMES.items():
    v = st[:, i].mean()
    print(f"  {nm:14s} mean cycles/comp/step {v / steps:14.0f} ({100 * v / tot:6.1f}%)  max {st[:, i].max() / steps:14.0f}")
for i, nm in COUNTS.items():
    print(f"  {nm:14s} mean /comp/step {st[:, i].mean() / steps:10.1f}  max {st[:, i].max() / steps:10.1f}")
order = np.argsort(-st[:, 9])
print("slowest components (per step): kernel X Z zqp giz_steps zqps | outer x_qps z_qps admm_x pdas_x pdas_z")
for k in order[:8]:
    print(f"  comp {k:4d}: " + " ".join(f"{st[k, j] / steps:10.0f}" for j in (9, 2, 6, 7, 40, 42)) +
          " | " + " ".join(f"{cc[k, j] / steps:7.1f}" for j in (0, 1, 2, 3, 5, 6)))
s.close()
