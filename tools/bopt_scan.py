"""B-opt CPU baseline (oracle/piadmm_cpu.cpp) against the job size: ms per MPC step of the bench
workload (matlab_pi, H = 30, seeded tiles, fixed 100 outer iterations and natural global
termination) on min(16, host) threads, for comparison with the GPU's tools/natural_scan.py /
tools/sweep.py lines.  CPU only; prints one JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]

from oracle import cpu_bopt  # noqa: E402
from piadmm import config, scenario  # noqa: E402

H = 30
threads = max(1, min(16, os.cpu_count() or 1))
TILES = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 8, 32, 128, 512, 2048]
for tiles in TILES:
    K = 20 if tiles <= 512 else 5
    scn = scenario.tiled(tiles, H, n_steps=K, perturb=True, seed=0)
    for mode in ("global", "fixed"):
        cfg = config.matlab_pi(H=H, max_outer=100, fixed_iters=1 if mode == "fixed" else 0, term_global=1)
        cpu_bopt.run(cfg, scn, 1, threads, records=False)          # warm-up
        best = min(cpu_bopt.run(cfg, scn, K, threads, records=False)["seconds"] for _ in range(3))
        print(json.dumps({"tiles": tiles, "mode": mode, "threads": threads, "ms_per_step": 1e3 * best / K}), flush=True)
