"""Generate tests/golden/ref_global_pi.npz by executing the global-PI script's OWN statements.

TEST INFRASTRUCTURE (fixture generator; run in the build container, never on the GPU box).

``casadi_old_PI_ADMM/main.py`` imports casadi at module level (an ordinary
ModuleNotFoundError), but its dual update and residuals are plain NumPy.  This script parses
the reference source with ``ast``, takes these statements unchanged (by line number) and runs
them on seeded inputs over several chained outer iterations (sum_err, diff_val and
PI_ADMM.param.rho carry from one iteration to the next, as in the script):

  x_curr_pred / dis_vec / dis_min   casadi_old_PI_ADMM/main.py:128-133
  K_I, K_P, adaptive rho, PI law    :135-142 (trad = 0: the script's setting, :16; and trad = 1,
                                    the plain update with back-calculation, :138-139)
  saturation + back-calculation     :145-151
  residuals                         :154-155

The solver calls (``ca.nlpsol``) are not run or stubbed: the x-step controls ``primal_u`` and
the positions ``pos_old`` / ``hat_pos_old`` these statements consume are seeded inputs.
``PI_ADMM.dynamic_update_edge`` is the reference's own numeric function (identical in
casadi_old_PI_ADMM/PI_ADMM_class.py and casadi/PI_ADMM_class.py, loaded as in
oracle/gen_ref_rollouts.py).  tests/test_oracle.py checks oracle.dual_update_global_pi and
pair_residuals_global_pi bit for bit against the outputs.

Usage: python oracle/gen_ref_global_pi.py [/root/reference]
"""
from __future__ import annotations

import ast
import functools
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_ref_rollouts import load_reference_rollouts  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "ref_global_pi.npz")
BLOCKS = {"dist": (128, 133), "law": (135, 142), "windup": (145, 151), "resid": (154, 155)}


def load_blocks(ref_root: str):
    path = os.path.join(ref_root, "casadi_old_PI_ADMM", "main.py")
    tree = ast.parse(open(path).read(), filename=path)
    stmts = []

    def walk(body):
        for node in body:
            stmts.append(node)
            for field in ("body", "orelse"):
                sub = getattr(node, field, None)
                if isinstance(sub, list):
                    walk(sub)
    walk(tree.body)
    out = {}
    for name, (a, b) in BLOCKS.items():
        sel = [n for n in stmts if a <= n.lineno <= b and n.end_lineno <= b]
        top = [n for n in sel if not any(o is not n and o.lineno <= n.lineno and n.end_lineno <= o.end_lineno
                                         and n in ast.walk(o) for o in sel)]
        assert top, f"no statements for {name}"
        out[name] = compile(ast.Module(body=top, type_ignores=[]), path, "exec")
    return out


def main(ref_root: str = "/root/reference"):
    blocks = load_blocks(ref_root)
    _, due = load_reference_rollouts(ref_root)
    rng = np.random.default_rng(20261016)
    recs = []
    for H, trad in ((5, 0), (8, 0), (15, 0), (30, 0), (5, 1), (15, 1)):
        for rep in range(3):
            param = types.SimpleNamespace(dt=0.1, L=1, num_ho=H, num_veh=2, spd=np.array([4, 8]), rho=1.0,
                                          dis_thres=1.5)
            PI = types.SimpleNamespace(param=param, dynamic_update_edge=functools.partial(
                due, types.SimpleNamespace(param=param)))
            xt = np.array([[-10, 0, 0], [0, 20, -np.pi / 2]], dtype=np.float64) + rng.uniform(-1, 1, (2, 3)) * [6, 6, 0.3]
            ns = {"np": np, "PI_ADMM": PI, "xt": xt, "trad": trad, "windup_sat": 20, "sum_err": 0, "diff_val": 0,
                  "dual_var_old": np.zeros((4, H + 1)), "last_iter_hat_pos": np.zeros((4, H + 1))}
            its = []
            for it in range(6):
                primal_u = np.round(rng.uniform(-np.pi / 6, np.pi / 6, size=(2, H)), 4)
                # positions with errors large enough that the saturation engages in some iterations
                pos_old = rng.normal(0, 3, size=(4, H + 1))
                hat = pos_old + rng.normal(0, 4 if rep == 2 else 1, size=(4, H + 1))
                S_in = np.array(ns["sum_err"], dtype=np.float64) * np.ones((4, H + 1))
                D_in = np.array(ns["diff_val"], dtype=np.float64) * np.ones((4, H + 1))
                rho_in = float(param.rho)
                lam_in = np.array(ns["dual_var_old"], np.float64)
                last = ns["last_iter_hat_pos"]
                ns.update(primal_u=primal_u, pos_old=pos_old, hat_pos_old=hat)
                for b in ("dist", "law", "windup", "resid"):
                    exec(blocks[b], ns)
                its.append(dict(primal_u=primal_u, pos_old=pos_old, hat=hat, last=np.array(last, np.float64),
                                S_in=S_in, D_in=D_in, rho_in=rho_in, lam_in=lam_in,
                                dual_out=np.array(ns["dual_var_old"], np.float64),
                                S_out=np.array(ns["sum_err"], np.float64) * np.ones((4, H + 1)),
                                D_out=np.array(ns["diff_val"], np.float64) * np.ones((4, H + 1)),
                                rho_out=float(param.rho), dis_vec=np.asarray(ns["dis_vec"]),
                                error_rk=float(ns["error_rk"]), error_sk=float(ns["error_sk"])))
                ns["last_iter_hat_pos"] = hat.copy()
            recs.append(dict(H=H, xt=xt, its=its, trad=trad))
    flat = {}
    for k, r in enumerate(recs):
        flat[f"c{k}_H"] = np.array(r["H"])
        flat[f"c{k}_trad"] = np.array(r["trad"])
        flat[f"c{k}_xt"] = r["xt"]
        flat[f"c{k}_n"] = np.array(len(r["its"]))
        for j, it in enumerate(r["its"]):
            for name, v in it.items():
                flat[f"c{k}_i{j}_{name}"] = np.asarray(v)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, n_cases=np.array(len(recs)),
                        source=np.array("casadi_old_PI_ADMM/main.py:128-133,135-142,145-151,154-155 "
                                        "(NumPy statements, executed; trad = 0 and 1, windup_sat = 20)"), **flat)
    print(f"wrote {OUT} ({len(recs)} cases)")


if __name__ == "__main__":
    main(*sys.argv[1:])
