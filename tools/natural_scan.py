"""Where the natural-termination step time goes: ms per MPC step of the bench workload (matlab_pi,
H = 30, seeded tiles) against the number of tiles, for the reference's global stop test
(term_global = 1, in-kernel grid barrier per outer iteration), per-component termination
(term_global = 0: no grid barrier, each component stops on its own residuals) and fixed 100
iterations.  Run on the GPU box from the repo root; prints one JSON line per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]

from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

K, W, H = 20, 5, 30
TILES = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 8, 32, 128, 512]
MODES = sys.argv[2].split(",") if len(sys.argv) > 2 else ["global", "component", "fixed"]
for tiles in TILES:
    for mode in MODES:
        cfg = config.matlab_pi(H=H, max_outer=100, fixed_iters=1 if mode == "fixed" else 0,
                               term_global=0 if mode == "component" else 1)
        scn = scenario.tiled(tiles, H, n_steps=K, perturb=True, seed=0)
        with PI_ADMM_MI355X(cfg, scn, device=0) as s:
            s.steps_async(0, W)
            s.sync()
            s.set_xt(scn.xt0)
            s.reset_counters()
            s.sync()
            t0 = time.perf_counter()
            ev = s.time_steps(0, K)
            s.sync()
            wall = time.perf_counter() - t0
            cnt = s.counters()
        print(json.dumps({"tiles": tiles, "mode": mode, "x_solver": os.environ.get("PIADMM_X_SOLVER", "gi_first"), "ms_per_step": 1e3 * wall / K, "event_ms_per_step": ev / K,
                          "outer_iters_per_comp_step": cnt["outer_iters"] / max(s.C, 1) / K,
                          "z_qps_per_step": cnt["z_qps"] / K, "pdas_x_per_step": cnt["pdas_x"] / K,
                          "inexact": cnt["inexact"]}), flush=True)
