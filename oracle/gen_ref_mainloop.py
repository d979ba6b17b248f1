"""Generate tests/golden/ref_mainloop.npz by executing the reference loop's OWN NumPy statements.

TEST INFRASTRUCTURE (fixture generator; run in the build container, never on the GPU box).

``casadi/main.py`` cannot run here (it imports casadi and the Bunch-based class at module
level; SURVEY.md 8c, an ordinary ModuleNotFoundError), but every statement of its loop that
is not a CasADi solve is plain NumPy.  This script parses the reference source with ``ast``,
takes exactly these statements unchanged (by line number) and executes them on seeded
inputs:

  seeds            casadi/main.py:48-49    x_seed_traj, y_seed_traj
  collision graph  casadi/main.py:110-113  edge_mat (all pairs i < j)
  edge list        casadi/main.py:121      np.where(edge_mat == 1)
  hat positions    casadi/main.py:156-158  dynamic_update_edge of the rounded pair controls
  dual update      casadi/main.py:161-162  plain ADMM, on the reference's object arrays
  residual sums    casadi/main.py:165-173  error_sk, error_rk over the edge list
  propagation      casadi/main.py:185-192  dynamic_update_edge(xt, primal_u) -> xt

The solver calls (``ca.qpsol``) are NOT run or stubbed: the controls these statements
consume (``veh_u`` / ``optimal_u_edge``) are seeded random inputs.  ``PI_ADMM.param`` is a
plain namespace with the reference's parameter values (casadi/PI_ADMM_class.py:15-28), and
``PI_ADMM.dynamic_update_edge`` is the reference's own numeric function (loaded the same way
as in oracle/gen_ref_rollouts.py).  For the pair rollout (:156) that function is handed a
two-vehicle parameter view with the pair's own speeds: the reference sizes it by num_veh and
reads spd[0], spd[1] (PI_ADMM_class.py:84-92), correct only for its two vehicles (quirk B16).  Inputs and outputs are written as data; tests/test_oracle.py
checks the oracle's statements bit for bit against them.

Usage: python oracle/gen_ref_mainloop.py [/root/reference]
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

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "ref_mainloop.npz")

# (name, first line, last line) of the reference statements executed (casadi/main.py)
BLOCKS = {
    "seeds": (48, 49),
    "collide": (110, 113),
    "edges": (121, 121),
    "hat": (156, 158),
    "dual": (161, 162),
    "resid": (165, 173),
    "propagate": (185, 192),
}


def load_blocks(ref_root: str):
    """Compiled code objects of the BLOCKS statements, taken unchanged from casadi/main.py."""
    path = os.path.join(ref_root, "casadi", "main.py")
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
        # top-most statements that start in [a, b] (a statement's children are included with it)
        sel = [n for n in stmts if a <= n.lineno <= b and n.end_lineno <= b]
        top = [n for n in sel if not any(o is not n and o.lineno <= n.lineno and n.end_lineno <= o.end_lineno
                                         and n in ast.walk(o) for o in sel)]
        assert top, f"no statements for {name}"
        out[name] = compile(ast.Module(body=top, type_ignores=[]), path, "exec")
    return out


def main(ref_root: str = "/root/reference"):
    blocks = load_blocks(ref_root)
    _, due = load_reference_rollouts(ref_root)
    rng = np.random.default_rng(20241016)
    recs = []
    for N in (2, 3, 4, 5):
        for H in (8, 15, 30):
            for rep in range(1 if H == 30 else 2):
                param = types.SimpleNamespace(dt=0.1, L=1, num_ho=H, num_veh=N, dis_thres=2.0, rho=2.0,
                                              spd=rng.choice([4.0, 5.0, 6.0, 8.0], size=N))
                obj = types.SimpleNamespace(param=param)
                PI = types.SimpleNamespace(param=param, dynamic_update_edge=functools.partial(due, obj))
                xt = np.column_stack([rng.uniform(-12, 12, N), rng.uniform(-12, 12, N), rng.uniform(-np.pi, np.pi, N)])
                # positions close enough that some pairs collide (the test is d^2 < dis_thres, quirk B2)
                base = rng.uniform(-1.5, 1.5, size=(N, 2, 1))
                pos_old = (base + rng.normal(0, 0.6, size=(N, 2, H + 1)) * np.linspace(0, 1, H + 1)).reshape(2 * N, H + 1)
                ns = {"np": np, "PI_ADMM": PI, "xt": xt.copy(), "pos_old": pos_old.copy(),
                      "edge_mat": np.zeros((N, N))}
                exec(blocks["seeds"], ns)
                exec(blocks["collide"], ns)
                exec(blocks["edges"], ns)
                edge_row, edge_col = ns["edge_row"], ns["edge_col"]
                # per-edge state as the reference's N x N object arrays
                hat = np.empty((N, N), dtype=object)
                dual = np.empty((N, N), dtype=object)
                last = np.empty((N, N), dtype=object)
                for i in range(N):
                    for j in range(N):
                        hat[i, j] = rng.normal(0, 1, size=(2, H + 1))
                        dual[i, j] = rng.normal(0, 1, size=(2, H + 1))
                        last[i, j] = rng.normal(0, 1, size=(2, H + 1))
                hat0 = np.array([[hat[i, j].copy() for j in range(N)] for i in range(N)])
                dual0 = np.array([[dual[i, j].copy() for j in range(N)] for i in range(N)])
                last0 = np.array([[last[i, j].copy() for j in range(N)] for i in range(N)])
                uh = np.round(rng.uniform(-np.pi / 6, np.pi / 6, size=(max(len(edge_row), 1), 2, H)), 4)
                ns.update(hat_pos_old=hat, dual_var_old=dual, last_iter_hat_pos=last)
                for i_edge in range(len(edge_col)):
                    veh1, veh2 = edge_row[i_edge], edge_col[i_edge]
                    # dynamic_update_edge sizes its arrays by param.num_veh and reads param.spd[0..1]
                    # (PI_ADMM_class.py:84-92): the reference only ever calls it on two vehicles, so
                    # the pair call gets a two-vehicle view with the pair's speeds
                    pp = types.SimpleNamespace(**{**vars(param), "num_veh": 2, "spd": param.spd[[veh1, veh2]]})
                    pe = types.SimpleNamespace(param=param, dynamic_update_edge=functools.partial(
                        due, types.SimpleNamespace(param=pp)))
                    ns.update(veh1=veh1, veh2=veh2, optimal_u_edge=uh[i_edge], PI_ADMM=pe,
                              xt_edge=np.vstack((xt[veh1, :], xt[veh2, :])))
                    exec(blocks["hat"], ns)
                    exec(blocks["dual"], ns)
                ns["PI_ADMM"] = PI
                exec(blocks["resid"], ns)
                primal_u = np.round(rng.uniform(-np.pi / 6, np.pi / 6, size=(N, H)), 4)
                ns.update(primal_u=primal_u, xt=xt.copy(), iter_his=np.zeros(1), num_step=0, curr_iter=1)
                exec(blocks["propagate"], ns)
                recs.append(dict(
                    N=N, H=H, spd=param.spd.copy(), xt=xt, pos_old=pos_old, seeds=np.stack([ns["x_seed_traj"], ns["y_seed_traj"]], 1),
                    edge_mat=ns["edge_mat"].copy(), edge_row=np.asarray(edge_row), edge_col=np.asarray(edge_col),
                    hat_in=hat0, dual_in=dual0, last_in=last0, uh=uh,
                    hat_out=np.array([[hat[i, j] for j in range(N)] for i in range(N)]),
                    dual_out=np.array([[dual[i, j] for j in range(N)] for i in range(N)]),
                    error_rk=float(ns["error_rk"]), error_sk=float(ns["error_sk"]),
                    primal_u=primal_u, xt_next=ns["xt"].copy()))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    flat = {}
    for k, r in enumerate(recs):
        for name, v in r.items():
            flat[f"c{k}_{name}"] = np.asarray(v)
    np.savez_compressed(OUT, n_cases=np.array(len(recs)),
                        source=np.array("casadi/main.py:48-49,110-113,121,156-158,161-162,165-173,185-192 "
                                        "(NumPy statements, executed)"), **flat)
    print(f"wrote {OUT} ({len(recs)} cases)")


if __name__ == "__main__":
    main(*sys.argv[1:])
