"""Candidate-pair detection throughput (piadmm_candidate_pairs) at 256k..4M agents: device time of
the detection kernels (inputs resident), pairs found, agents/s.  Run under rocprofv3 for the
per-kernel split (profiles/detect_*)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
import numpy as np  # noqa: E402

from piadmm import candidates, config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

rng = np.random.default_rng(0)
with PI_ADMM_MI355X(config.matlab_pi(H=10), scenario.intersection(10)) as s:
    for n in (1 << 18, 1 << 20, 1 << 22):
        side = np.sqrt(n / 0.1)                       # 0.1 agents per m^2
        xy = rng.uniform(0, side, size=(n, 2))
        r = rng.uniform(1.0, 3.0, n)
        best = None
        for _ in range(3):
            pairs, ms = candidates.candidate_pairs(s, xy, r, with_time=True)
            best = ms if best is None else min(best, ms)
        print(json.dumps({"agents": n, "pairs": int(pairs.shape[0]), "ms": best,
                          "agents_per_s": n / (best * 1e-3), "pairs_per_s": pairs.shape[0] / (best * 1e-3)}), flush=True)
