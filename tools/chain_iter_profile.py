"""Development diagnostic (not shipped): per-outer-iteration cost of the 1024-agent chain
(bench.py --chain: one component split over workgroups), host-stepped for the last steps
(piadmm_outer_iter): wall time per iteration next to that iteration's pair-QP work (z QPs,
reduced solves, ADMM iterations) summed over the blocks and for the block with the most.

    python tools/chain_iter_profile.py [first_profiled_step] [steps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

t0 = int(sys.argv[1]) if len(sys.argv) > 1 else 17
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H, M = 30, 100
cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=M, term_global=1)
scn = scenario.crossing(1024, H, n_steps=t0 + steps + 2, seed=1, pairs="chain")
names = ("outer", "x_qps", "z_qps", "admm_x", "admm_z", "pdas_x", "pdas_z", "inexact")
with PI_ADMM_MI355X(cfg, scn) as s:
    for _ in range(t0):
        s.mpc_step()
    for t in range(t0, t0 + steps):
        rows = []
        for it in range(M):
            prev = s.component_counters().astype(np.int64)
            w0 = time.perf_counter()
            stop = s.outer_iter(it, t)
            dt = (time.perf_counter() - w0) * 1e3
            d = s.component_counters().astype(np.int64) - prev
            k = int(np.argmax(d[:, 6] + 4 * d[:, 2]))
            rows.append((dt, d.sum(0), k, d[k]))
            if stop:
                break
        s.step_finish()
        tot = sum(r[0] for r in rows)
        print(f"step {t}: {len(rows)} iterations, {tot:.1f} ms host-stepped", flush=True)
        for dt, tot_c, k, dk in sorted(rows, key=lambda r: -r[0])[:8]:
            print(f"  {dt:7.3f} ms | z_qps={tot_c[2]} pdas_z={tot_c[6]} admm_z={tot_c[4]} | block {k}: "
                  + " ".join(f"{n}={v}" for n, v in zip(names, dk) if n in ("z_qps", "pdas_z", "admm_z")), flush=True)
