"""Large-N sweep (measurement item 3): the bench workload (matlab_pi preset, H=30,
fixed 100 outer iterations, global residual history) at 256 ... 65 536 agents on one GPU.

Per size: ms per MPC step, outer iterations/s, agent x-step QPs/s and the achieved algorithmic
HBM rate (bench.algorithmic_bytes) against the 8 TB/s peak.  Small sizes leave most of the 256
CUs idle (one workgroup per 2-agent component); from ~512 components on every CU is busy.

  python tools/sweep.py [--tiles 128,512,2048,8192,32768] [--steps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))

import bench  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="128,512,2048,8192,32768")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--H", type=int, default=30)
    args = ap.parse_args()
    H, K = args.H, args.steps
    for tiles in [int(x) for x in args.tiles.split(",")]:
        cfg = config.matlab_pi(H=H, fixed_iters=1, max_outer=bench.MAX_OUTER, term_global=1)
        scn = scenario.tiled(tiles, H, n_steps=2 * K, perturb=True, seed=0)
        with PI_ADMM_MI355X(cfg, scn) as s:
            s.steps_async(0, K)                 # warmup (per-scenario caches)
            s.sync()
            s.set_xt(scn.xt0)
            s.reset_counters()
            ms = s.time_steps(0, K)
            cnt = s.counters()
        step_ms = ms / K
        outer = cnt["outer_iters"] / max(s.C, 1)
        gbs = bench.algorithmic_bytes(cnt, H) / (ms / 1e3) / 1e9
        print(json.dumps({
            "agents": 2 * tiles, "components": tiles, "H": H, "steps": K,
            "ms_per_step": step_ms, "outer_iters_per_s": outer / (ms / 1e3),
            "agent_qps_per_s": cnt["x_qps"] / (ms / 1e3), "pair_qps_per_s": cnt["z_qps"] / (ms / 1e3),
            "achieved_GBps": gbs, "hbm_frac": gbs / bench.PEAK_HBM_GBS, "inexact": cnt["inexact"]}), flush=True)


if __name__ == "__main__":
    main()
