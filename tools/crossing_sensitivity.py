"""Sensitivity of the reference loop on the crossing workload (bench.py --crossing: 64 four-vehicle
all-pairs crossings, H30, matlab_pi, global natural termination), on the CPU baseline alone: B-opt
(oracle/piadmm_cpu.cpp) against itself started from xt0 (1 + eps).  Writes one JSON with the
per-step deviation, the outer-iteration counts and the near-tie log at a wide tolerance, so the
GPU-vs-CPU parting (tests/test_gpu_configs.py) can be read against the job's own sensitivity.

    python tools/crossing_sensitivity.py [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd")]
from oracle import cpu_bopt  # noqa: E402
from piadmm import config, scenario  # noqa: E402
from piadmm.scenario import Scenario  # noqa: E402


def dev(a, b, k):
    return (float(np.max(np.abs(a["u"][k] - b["u"][k]))),
            float(np.max(np.abs(a["xt"][k] - b["xt"][k]) / (1.0 + np.abs(a["xt"][k])))))


def main(out):
    H, n = 30, 20
    cfg = config.matlab_pi(H=H, term_global=1)
    scn = scenario.concat([scenario.crossing(4, H, n_steps=n + 2, seed=k) for k in range(64)])
    threads = min(16, os.cpu_count() or 1)
    base = cpu_bopt.run(cfg, scn, n, threads=threads, tie_tol=1e-6)
    res = {"workload": "64 four-vehicle all-pairs crossings, H30, matlab_pi, term_global natural, steps 0..19",
           "iters": base["iters"][:, 0].tolist(), "near_ties_tol_1e-6": base["ties"][0], "perturbed": {}}
    for eps in (1e-15, 1e-12):
        s2 = Scenario(spd=scn.spd, xt0=scn.xt0 * (1.0 + eps), ref=scn.ref, edges=scn.edges, n_steps=scn.n_steps)
        p = cpu_bopt.run(cfg, s2, n, threads=threads)
        d = [dev(base, p, k) for k in range(n)]
        res["perturbed"][f"{eps:g}"] = {"max_abs_du": [v[0] for v in d], "max_rel_dxt": [v[1] for v in d],
                                        "iters": p["iters"][:, 0].tolist()}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res)[:600])


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "crossing_sensitivity_r04.json"))
