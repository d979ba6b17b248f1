"""Per-outer-iteration cost of the graph kernel on the crossing workload (bench.py --crossing),
host-stepped (piadmm_outer_iter: one launch per iteration, synchronised): wall time per iteration
next to that iteration's work counters (x / z QPs, ADMM iterations, reduced solves), summed over the
components and for the component with the most ADMM work.  Shows what sets an iteration's time.

    python tools/graph_iter_profile.py [n_crossings] [steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H = 30
cfg = config.matlab_pi(H=H, term_global=1)
scn = scenario.concat([scenario.crossing(4, H, n_steps=steps + 2, seed=k) for k in range(n)])
names = ("outer", "x_qps", "z_qps", "admm_x", "admm_z", "pdas_x", "pdas_z", "inexact")
with PI_ADMM_MI355X(cfg, scn) as s:
    s.mpc_step()                         # page-in, per-scenario caches
    s.set_xt(scn.xt0)
    for t in range(steps):
        prev = s.component_counters().astype(np.int64)
        it = 0
        rows = []
        while True:
            t0 = time.perf_counter()
            stop = s.outer_iter(it, t)
            dt = time.perf_counter() - t0
            cc = s.component_counters().astype(np.int64)
            d = cc - prev
            prev = cc
            k = int(np.argmax(d[:, 3] * 1000 + d[:, 2]))
            rows.append((it, dt * 1e3, d.sum(0), k, d[k]))
            it += 1
            if stop or it == cfg.max_outer:
                break
        t0 = time.perf_counter()
        s.step_finish()
        fin = (time.perf_counter() - t0) * 1e3
        print(f"step {t}: {it} iterations, finish {fin:.2f} ms")
        for (i, ms, tot, k, dk) in rows:
            print(f"  it {i:3d} {ms:8.3f} ms | total " + " ".join(f"{nm}={v}" for nm, v in zip(names[1:7], tot[1:7])) +
                  f" | comp {k}: " + " ".join(f"{nm}={v}" for nm, v in zip(names[1:7], dk[1:7])))
