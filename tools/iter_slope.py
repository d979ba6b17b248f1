"""Cost of one steady-state outer iteration of the fused kernel: the bench job (256 agents x H30,
matlab_pi, fixed iterations, global scope) timed at several fixed iteration counts M; the slope of
ms per MPC step against M is one outer iteration of the slowest component's chain (the per-step
costs -- setup, the first iteration's solves, the z-step -- are the intercept).
    python3 tools/iter_slope.py [lib ...]      (PIADMM_LIB paths; default: the built library)
    PIADMM_SLOPE_JOB=preset,H,tiles selects another job (e.g. casadi_default,20,32: configs[1])."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/distributed-local-planner-pi-admm_amd"]
import os
from piadmm import config, scenario
from piadmm.solver import PI_ADMM_MI355X
preset, H, tiles = (os.environ.get("PIADMM_SLOPE_JOB") or "matlab_pi,30,128").split(",")
H, tiles = int(H), int(tiles)
out = {}
for M in (20, 60, 100, 140):
    cfg = config.PRESETS[preset](H=H, fixed_iters=1, max_outer=M, term_global=1)
    scn = scenario.tiled(tiles, H, n_steps=25, perturb=True, seed=0)
    with PI_ADMM_MI355X(cfg, scn) as s:
        s.time_steps(0, 5)
        s.set_xt(scn.xt0)
        ms = min(s.time_steps(0, 20) for _ in range(2) if s.set_xt(scn.xt0) is None)
    out[M] = ms / 20
print(json.dumps(out))
'''


def main():
    libs = sys.argv[1:] or [""]
    for lib in libs:
        env = dict(os.environ)
        if lib:
            env["PIADMM_LIB"] = os.path.abspath(lib)
        r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(lib, "FAILED", r.stderr[-2000:])
            sys.exit(1)
        d = {int(k): v for k, v in json.loads(r.stdout.strip().splitlines()[-1]).items()}
        Ms = sorted(d)
        n = len(Ms)
        mx, my = sum(Ms) / n, sum(d[m] for m in Ms) / n
        slope = sum((m - mx) * (d[m] - my) for m in Ms) / sum((m - mx) ** 2 for m in Ms)
        print(json.dumps({"lib": os.path.basename(lib) or "libpiadmm.so", "ms_per_step": d,
                          "us_per_outer_iter": slope * 1e3, "cycles_per_outer_iter_at_2.4GHz": slope * 2.4e6,
                          "intercept_ms": my - slope * mx}), flush=True)


if __name__ == "__main__":
    main()
