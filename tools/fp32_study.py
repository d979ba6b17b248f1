"""configs[4] tolerance study: fp64 vs precision 1 (fp32 ADMM matrices, fp64 polish) on the
256-agent H=50 tightening workload.  Prints one JSON object: deviations of u and of the
trajectories, outer-iteration counts, ADMM iterations / reduced solves per QP and step time."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-local-planner-pi-admm_amd"))
import numpy as np  # noqa: E402

from piadmm import config, scenario  # noqa: E402
from piadmm.solver import PI_ADMM_MI355X  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 50
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
natural = len(sys.argv) > 3 and sys.argv[3] == "natural"
out = {"H": H, "steps": steps, "agents": 256, "termination": "natural" if natural else "fixed 100"}
runs = {}
for prec in (0, 1):
    cfg = config.matlab_pi(H=H, tighten=1, precision=prec, fixed_iters=0 if natural else 1, max_outer=100)
    scn = scenario.tiled(128, H, n_steps=steps + 1, seed=0)
    with PI_ADMM_MI355X(cfg, scn) as s:
        s.reset_counters()
        xs, us, its, ms = [], [], [], 0.0
        for t in range(steps):
            ms += s.time_steps(t, 1)
            st = s.state()
            xs.append(st["xt"])
            us.append(st["u"])
            its.append(st["iters"])
        cnt = s.counters()
    runs[prec] = dict(xt=np.array(xs), u=np.array(us), iters=np.array(its), ms=ms / steps, cnt=cnt)
a, b = runs[0], runs[1]
out.update({
    "max_abs_du": float(np.max(np.abs(a["u"] - b["u"]))),
    "max_rel_dxt": float(np.max(np.abs(a["xt"] - b["xt"]) / (1 + np.abs(a["xt"])))),
    "iteration_count_mismatches": int(np.sum(a["iters"] != b["iters"])),
    "ms_per_step": {"fp64": a["ms"], "fp32_admm": b["ms"]},
})
for k, r in (("fp64", a), ("fp32_admm", b)):
    c = r["cnt"]
    out[k] = {"admm_per_zqp": c["admm_z"] / max(c["z_qps"], 1), "solves_per_zqp": c["pdas_z"] / max(c["z_qps"], 1),
              "admm_per_xqp": c["admm_x"] / max(c["x_qps"], 1), "inexact": c["inexact"]}
print(json.dumps(out))
