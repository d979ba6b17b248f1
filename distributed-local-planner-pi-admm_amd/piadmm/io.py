"""Run records: the outputs of the reference's MPC driver as files.

``casadi/main.py`` keeps its results in Python lists and prints one line per MPC step
(``:193-196``): ``x_vec`` (positions, ``:199``), ``theta_vec`` (``:200``), ``u_vec``
(``:201``), ``iter_his`` (``:186``), then scatters the two trajectories (``:206-220``).
Here a run is a :class:`RunRecord`; ``save_run`` writes it as ``.npz`` (arrays) plus a
``.json`` summary, ``plot_run`` draws the reference's figure, ``step_line`` formats the
reference's progress line.
"""
from __future__ import annotations

import dataclasses
import hashlib
import json
import os

import numpy as np


@dataclasses.dataclass
class RunRecord:
    x_vec: np.ndarray        # (steps, N, 2)  positions after each step   (main.py:199)
    theta_vec: np.ndarray    # (steps, N)     headings                    (main.py:200)
    u_vec: np.ndarray        # (steps, N)     applied steering u_0        (main.py:201)
    iter_his: np.ndarray     # (steps, C)     outer iterations per component (main.py:186)
    resid: np.ndarray        # (steps, C, max_outer, 2)  (rk, sk), NaN after the last iteration
    dual_max: np.ndarray     # (steps,)       max of the duals at the end of the step (main.py:194)
    dual_min: np.ndarray     # (steps,)
    meta: dict = dataclasses.field(default_factory=dict)

    @property
    def n_steps(self) -> int:
        return int(self.x_vec.shape[0])


class RunRecorder:
    """Collects the per-step outputs of a solver (``PI_ADMM_MI355X`` or the oracle)."""

    def __init__(self, meta: dict | None = None):
        self.meta = dict(meta or {})
        self._x, self._th, self._u, self._it, self._r, self._dmax, self._dmin = ([] for _ in range(7))

    def add(self, xt, u, iters, resid, lam):
        lam = np.asarray(lam)
        self._x.append(np.asarray(xt)[:, :2].copy())
        self._th.append(np.asarray(xt)[:, 2].copy())
        self._u.append(np.asarray(u)[:, 0].copy())
        self._it.append(np.asarray(iters).copy())
        self._r.append(np.asarray(resid).copy())
        self._dmax.append(float(lam.max()) if lam.size else 0.0)
        self._dmin.append(float(lam.min()) if lam.size else 0.0)

    def record(self) -> RunRecord:
        return RunRecord(x_vec=np.stack(self._x), theta_vec=np.stack(self._th), u_vec=np.stack(self._u),
                         iter_his=np.stack(self._it), resid=np.stack(self._r),
                         dual_max=np.array(self._dmax), dual_min=np.array(self._dmin), meta=dict(self.meta))


def step_line(num_step: int, iters, dual_max: float, dual_min: float, rho: float, xt) -> str:
    """The reference's per-step print (``casadi/main.py:193-196``)."""
    xt = np.asarray(xt)
    it = int(np.max(iters))
    return ("t_step: {}, iter: {}, max dual: {}, min dual: {}, rho: {}, veh_x: {}, veh_y: {}"
            .format(num_step + 1, it, dual_max, dual_min, rho, xt[:, 0], xt[:, 1]))


def save_run(path: str, rec: RunRecord) -> tuple[str, str]:
    """Write ``<path>.npz`` (all arrays) and ``<path>.json`` (summary + meta)."""
    base = path[:-4] if path.endswith(".npz") else path
    npz, js = base + ".npz", base + ".json"
    np.savez_compressed(npz, x_vec=rec.x_vec, theta_vec=rec.theta_vec, u_vec=rec.u_vec,
                        iter_his=rec.iter_his, resid=rec.resid, dual_max=rec.dual_max,
                        dual_min=rec.dual_min)
    summary = {
        "n_steps": rec.n_steps, "n_agents": int(rec.x_vec.shape[1]),
        "iter_his_max_per_step": rec.iter_his.max(axis=1).tolist(),
        "final_xy": rec.x_vec[-1].tolist(), "meta": rec.meta,
    }
    with open(js, "w") as f:
        json.dump(summary, f, indent=1)
    return npz, js


def load_run(path: str) -> RunRecord:
    base = path[:-4] if path.endswith(".npz") else path
    d = np.load(base + ".npz", allow_pickle=False)
    meta = {}
    if os.path.exists(base + ".json"):
        with open(base + ".json") as f:
            meta = json.load(f).get("meta", {})
    return RunRecord(x_vec=d["x_vec"], theta_vec=d["theta_vec"], u_vec=d["u_vec"], iter_his=d["iter_his"],
                     resid=d["resid"], dual_max=d["dual_max"], dual_min=d["dual_min"], meta=meta)


CHECKPOINT_KEYS = ("xt", "hat", "lam", "S", "D", "last_hat", "rho_pi")


def scenario_fingerprint(scn) -> np.ndarray:
    """(N, E, sha256 of the candidate pair list) of a scenario: a checkpoint's pair state (hat /
    lam / S / D, one row per pair) only means something for the same pairs in the same order."""
    edges = np.ascontiguousarray(np.asarray(scn.edges, np.int64).reshape(-1, 2))
    return np.array([str(int(scn.n_agents)), str(int(edges.shape[0])), hashlib.sha256(edges.tobytes()).hexdigest()])


def save_checkpoint(path: str, state: dict, cfg=None, scn=None) -> str:
    """Checkpoint of an MPC run between two steps (the ``.npz`` dump of xt,
    duals, S, D): ``state`` from ``PI_ADMM_MI355X.step_state()`` (or the oracle's edge state) --
    xt, the pair state hat / lam / S / D / last_hat (carried by warm_duals, a12), the global-PI
    pair penalties rho_pi -- and the next reference time index ``t``.  The reference keeps this
    state only in Python variables (``casadi/main.py:52-63,180``)."""
    base = path[:-4] if path.endswith(".npz") else path
    arrs = {k: np.asarray(state[k], np.float64) for k in CHECKPOINT_KEYS if state.get(k) is not None}
    arrs["t"] = np.array(int(state.get("t", 0)), np.int64)
    if cfg is not None:
        arrs["cfg_json"] = np.array(json.dumps(dataclasses.asdict(cfg), sort_keys=True))
    if scn is not None:
        arrs["scenario"] = scenario_fingerprint(scn)
    np.savez_compressed(base + ".npz", **arrs)
    return base + ".npz"


def load_checkpoint(path: str, cfg=None, scn=None) -> dict:
    """The state :func:`save_checkpoint` wrote (NumPy only, no pickles), for
    ``PI_ADMM_MI355X.set_state``.  With ``cfg``: refuses a checkpoint of another configuration;
    with ``scn``: one of another scenario (agent count, pair count or pair list), or one that was
    saved without the scenario's fingerprint.  Non-finite state is refused either way."""
    base = path[:-4] if path.endswith(".npz") else path
    d = np.load(base + ".npz", allow_pickle=False)
    if cfg is not None and "cfg_json" in d.files:
        if json.loads(str(d["cfg_json"])) != json.loads(json.dumps(dataclasses.asdict(cfg), sort_keys=True)):
            raise ValueError("checkpoint was written with another configuration")
    if scn is not None:
        if "scenario" not in d.files:
            raise ValueError("checkpoint carries no scenario fingerprint (save_checkpoint(..., scn=...))")
        if not np.array_equal(d["scenario"], scenario_fingerprint(scn)):
            raise ValueError("checkpoint was written for another scenario (agents, pairs or pair order differ)")
    st = {k: d[k] for k in CHECKPOINT_KEYS if k in d.files}
    for k, v in st.items():
        if not np.all(np.isfinite(v)):
            raise ValueError(f"checkpoint holds non-finite {k}")
    st["t"] = int(d["t"])
    return st


def plot_run(rec: RunRecord, path: str, agents=None) -> str:
    """The reference's figure (``casadi/main.py:206-220``): one scatter per vehicle of its
    positions over the run; more than two agents get one colour each."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    agents = range(rec.x_vec.shape[1]) if agents is None else agents
    fig, ax = plt.subplots()
    colours = ["blue", "red"]
    for k, a in enumerate(agents):
        ax.scatter(rec.x_vec[:, a, 0], rec.x_vec[:, a, 1], color=colours[k] if k < 2 else None, s=12)
    ax.set_title("2D Scatter of Two Lines" if len(list(agents)) == 2 else "Agent trajectories")
    ax.set_xlabel("X Axis")
    ax.set_ylabel("Y Axis")
    fig.savefig(path, dpi=100)
    plt.close(fig)
    return path
