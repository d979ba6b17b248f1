"""Host driver: the MI355X counterpart of ``PI_ADMM_CASADI`` + the ``casadi/main.py`` loop.

The reference builds a ``PI_ADMM_CASADI`` object (``casadi/PI_ADMM_class.py:12-37``),
then runs, in Python, ``for num_step ...: for i_iter ...: for i_veh ...: ca.qpsol(...)``
(``casadi/main.py:43-201``).  Here the object holds a libpiadmm handle and one
``mpc_step`` call runs that whole ``num_step`` body for every agent on the GPU.

Attribute names follow the reference so scripts read the same:
``solver.param.num_ho``, ``solver.param.spd``, ``solver.ref_traj`` (2N x T),
``solver.xt`` (N x 3), ``solver.iter_his``, ``solver.x_vec`` / ``u_vec``.
"""
from __future__ import annotations

import ctypes
import dataclasses
import types

import numpy as np

from . import _lib
from .config import PIADMMConfig
from .scenario import Scenario


@dataclasses.dataclass
class StepResult:
    xt: np.ndarray         # (N,3) state after propagation (casadi/main.py:189-192)
    u: np.ndarray          # (N,H) primal_u used for propagation (:187)
    resid: np.ndarray      # (C, max_outer, 2) (rk, sk) per executed iteration, NaN after
    iters: np.ndarray      # (C,) outer iterations executed (iter_his, :186)
    status: np.ndarray     # (N+E,) PIADMM_QP_* flags per agent then per pair
    global_resid: np.ndarray | None = None   # term_global: (max_outer, 2) summed over all ranks
    global_iters: int | None = None          # term_global: outer iterations of the whole job


class PI_ADMM_MI355X:
    """Batched PI-ADMM planner on one GPU (one handle, one HIP stream)."""

    def __init__(self, cfg: PIADMMConfig, scenario: Scenario | None = None, device: int = 0, shard=None):
        """``shard`` (a :class:`piadmm.dist.Shard`): this rank's part of a job whose candidate
        pairs may cross ranks; ``scenario`` is then ``shard.scn`` (own agents + ghosts)."""
        if shard is not None:
            scenario = shard.scn if scenario is None else scenario
        if scenario is None:
            raise ValueError("a scenario (or a shard) is required")
        self.cfg = cfg
        self.scn = scenario
        self.shard = shard
        self._xfn = None
        self.N = scenario.n_agents
        self.E = scenario.n_edges
        self.lib = _lib.load()
        c = _lib.to_c(cfg, self.N, device)
        h = ctypes.c_void_p()
        _lib.check(self.lib.piadmm_create(ctypes.byref(c), ctypes.byref(h)))
        self._h = h
        self.param = types.SimpleNamespace(
            dt=cfg.dt, L=cfg.L, num_ho=cfg.H, num_veh=self.N, dis_thres=cfg.dis_thres,
            spd=scenario.spd.copy(), beta=cfg.beta, Pnorm=cfg.Pnorm, Pcost=cfg.Pcost,
            iter_num=cfg.max_outer, rho=cfg.rho, eps_pri=cfg.eps_pri, eps_dual=cfg.eps_dual)
        # ref_traj in the reference layout: rows [x_0; y_0; x_1; y_1; ...] (PI_ADMM_class.py:37)
        self.ref_traj = scenario.ref.reshape(2 * self.N, -1)
        spd = np.ascontiguousarray(scenario.spd, np.float64)
        xt0 = np.ascontiguousarray(scenario.xt0, np.float64)
        ref = np.ascontiguousarray(scenario.ref, np.float64)
        edges = np.ascontiguousarray(scenario.edges, np.int32).reshape(-1)
        if shard is None:
            self._check(self.lib.piadmm_set_scenario(self._h, _lib.dptr(spd), _lib.dptr(xt0), _lib.dptr(ref),
                                                     ref.shape[2], _lib.iptr(edges) if edges.size else None,
                                                     self.E))
        else:
            u8 = ctypes.POINTER(ctypes.c_uint8)
            owned = np.ascontiguousarray(shard.owned, np.uint8)
            counted = np.ascontiguousarray(shard.counted, np.uint8)
            slot = np.ascontiguousarray(shard.slot, np.int32)
            self._check(self.lib.piadmm_set_scenario_shard(
                self._h, _lib.dptr(spd), _lib.dptr(xt0), _lib.dptr(ref), ref.shape[2],
                _lib.iptr(edges) if edges.size else None, self.E, owned.ctypes.data_as(u8), _lib.iptr(slot),
                int(shard.n_slots), counted.ctypes.data_as(u8) if counted.size else None))
        self.C = self.lib.piadmm_n_components(self._h)
        self.t = 0
        self.xt = xt0.copy()
        self.iter_his: list[np.ndarray] = []
        self.x_vec: list[np.ndarray] = []
        self.u_vec: list[np.ndarray] = []

    # ------------------------------------------------------------------ core
    def _check(self, rc):
        _lib.check(rc, self._h)

    def mpc_step(self, t: int | None = None) -> StepResult:
        """One ``num_step`` iteration of ``casadi/main.py:43-201`` for all agents."""
        t = self.t if t is None else t
        H = self.cfg.H
        xt = np.empty((self.N, 3))
        u = np.empty((self.N, H))
        resid = np.empty((self.C, self.cfg.max_outer, 2))
        iters = np.empty(self.C, np.int32)
        status = np.empty(self.N + self.E, np.int32)
        self._check(self.lib.piadmm_mpc_step(self._h, t, _lib.dptr(xt), _lib.dptr(u), _lib.dptr(resid),
                                             _lib.iptr(iters), _lib.iptr(status)))
        self.t = t + 1
        self.xt = xt
        self.iter_his.append(iters)
        self.x_vec.append(xt[:, :2].T.copy())
        self.u_vec.append(u[:, 0].copy())
        res = StepResult(xt=xt, u=u, resid=resid, iters=iters, status=status)
        if self.cfg.term_global:
            res.global_resid, res.global_iters = self.global_resid()
        return res

    def global_resid(self):
        """(max_outer, 2) residual history summed over every pair of every rank, and the
        job's outer-iteration count (term_global; casadi/main.py:164-178 over all agents)."""
        out = np.empty((self.cfg.max_outer, 2))
        n = ctypes.c_int32()
        self._check(self.lib.piadmm_global_resid(self._h, _lib.dptr(out), ctypes.byref(n)))
        return out, int(n.value)

    def comm_init(self, unique_id: bytes, nranks: int, rank: int):
        """Join the RCCL communicator of a sharded term_global job (piadmm_comm_init)."""
        if len(unique_id) != 128:
            raise ValueError("an RCCL unique id has 128 bytes")
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        self._check(self.lib.piadmm_comm_init(self._h, buf, int(nranks), int(rank)))

    def set_allreduce(self, fn):
        """Host all-reduce transport (piadmm_set_allreduce): ``fn(buf)`` gets a float64 array view
        and must replace it in place by its sum over the job's ranks (e.g. a gloo all-reduce).
        ``None`` removes it."""
        if fn is None:
            self._xfn = None
            self._check(self.lib.piadmm_set_allreduce(self._h, None, None))
            return

        def cb(ctx, buf, n):
            try:
                fn(np.ctypeslib.as_array(buf, shape=(int(n),)))
                return 0
            except Exception:       # an exception cannot cross the C boundary: fail the step
                return 1
        self._xfn = _lib.ALLREDUCE_FN(cb)      # kept alive as long as the handle
        self._check(self.lib.piadmm_set_allreduce(self._h, ctypes.cast(self._xfn, ctypes.c_void_p), None))

    def set_candidate_graph(self, edges: np.ndarray):
        """Replace the candidate graph between MPC steps (a dynamic graph, e.g. rebuilt from the
        current states by piadmm.candidates): the scenario restarts from the current states with
        the new pairs (per-pair duals and warm starts reset, as at the start of a reference step,
        casadi/main.py:52-63)."""
        if self.shard is not None:
            raise ValueError("a sharded handle keeps its graph")
        if self.cfg.dual_mode == 2:
            # the global-PI law keeps each pair's adaptive penalty across MPC steps
            # (casadi_old_PI_ADMM/main.py:137-139, PI_ADMM.param.rho is never reset); a new
            # scenario would restart every pair from cfg.rho, silently departing from that law
            raise ValueError("set_candidate_graph does not carry the global-PI pair penalties "
                             "(dual_mode 2): keep a static candidate graph for that preset")
        edges = np.ascontiguousarray(edges, np.int32).reshape(-1, 2)
        self.scn = Scenario(spd=self.scn.spd, xt0=np.ascontiguousarray(self.xt, np.float64), ref=self.scn.ref,
                            edges=edges, n_steps=self.scn.n_steps)
        self.E = edges.shape[0]
        flat = edges.reshape(-1)
        self._check(self.lib.piadmm_set_scenario(self._h, _lib.dptr(np.ascontiguousarray(self.scn.spd, np.float64)),
                                                 _lib.dptr(self.scn.xt0),
                                                 _lib.dptr(np.ascontiguousarray(self.scn.ref, np.float64)),
                                                 self.scn.ref.shape[2], _lib.iptr(flat) if flat.size else None,
                                                 self.E))
        self.C = self.lib.piadmm_n_components(self._h)

    def run(self, n_steps: int | None = None) -> list[StepResult]:
        n = self.scn.n_steps if n_steps is None else n_steps
        return [self.mpc_step() for _ in range(n)]

    def steps_async(self, t0: int, n_steps: int):
        """Enqueue MPC steps without host copies (state stays in HBM)."""
        self._check(self.lib.piadmm_mpc_steps_async(self._h, t0, n_steps))

    def sync(self):
        self._check(self.lib.piadmm_sync(self._h))

    def steps_per_launch(self) -> int:
        """MPC steps the library runs per persistent kernel launch."""
        return int(self.lib.piadmm_steps_per_launch(self._h))

    def time_steps(self, t0: int, n_steps: int) -> float:
        """hipEvent time (ms) of n_steps MPC steps on the handle's stream."""
        ms = ctypes.c_float()
        self._check(self.lib.piadmm_time_steps(self._h, t0, n_steps, ctypes.byref(ms)))
        return float(ms.value)

    COUNTER_NAMES = ("outer_iters", "x_qps", "z_qps", "admm_x", "admm_z", "pdas_x", "pdas_z", "inexact")

    def counters(self) -> dict:
        buf = (ctypes.c_uint64 * 8)()
        self._check(self.lib.piadmm_get_counters(self._h, buf))
        return dict(zip(self.COUNTER_NAMES, (int(v) for v in buf)))

    def component_counters(self) -> np.ndarray:
        buf = (ctypes.c_uint64 * (8 * self.C))()
        self._check(self.lib.piadmm_get_component_counters(self._h, buf, 8 * self.C))
        return np.array(buf, dtype=np.int64).reshape(self.C, 8)

    def reset_counters(self):
        """Zero the work counters and the near-tie log."""
        self._check(self.lib.piadmm_reset_counters(self._h))

    def set_tie_tolerance(self, tol: float):
        """Turn the near-tie log on with this tolerance (e.g. 1e-9), or off with 0 (the default:
        the log's kernel instantiation costs 3-10 % of a step; piadmm_set_tie_tolerance)."""
        self._check(self.lib.piadmm_set_tie_tolerance(self._h, float(tol)))

    def near_ties(self):
        """(counts per kind, events) of the near-tie log since the last reset (piadmm_get_near_ties):
        the reference's discrete decisions -- rounding (casadi/main.py:48-49,103,153), the collision
        test (:112-113), the stop test (:174), MATLAB's distance check -- taken within the tolerance
        of their threshold.  events: a NumPy record array (step, iter, kind, id, index, margin)."""
        cnt = (ctypes.c_uint64 * len(_lib.TIE_KINDS))()
        ev = np.zeros(_lib.TIE_CAP * 2, _lib.TIE_DTYPE)
        n = ctypes.c_int32()
        self._check(self.lib.piadmm_get_near_ties(self._h, cnt, ev.ctypes.data, ev.size, ctypes.byref(n)))
        # n = the events written (the C side stops at max_events and at each log's cap); the
        # per-kind counts are the totals
        return dict(zip(_lib.TIE_KINDS, (int(v) for v in cnt))), ev[:max(0, min(int(n.value), ev.size))].copy()

    def step_state(self) -> dict:
        """The state that carries into the next MPC step (piadmm_get_step_state): xt, and hat, lam,
        S, D, last_hat (warm_duals, a12) and the global-PI pair penalties rho_pi -- a checkpoint."""
        H1 = self.cfg.H + 1
        out = dict(xt=np.empty((self.N, 3)), hat=np.empty((self.E, 2, 2, H1)), lam=np.empty((self.E, 2, 2, H1)),
                   S=np.empty((self.E, 2, 2, H1)), D=np.empty((self.E, 2, 2, H1)),
                   last_hat=np.empty((self.E, 2, 2, H1)), rho_pi=np.empty(self.E))
        e = (lambda k: _lib.dptr(out[k]) if self.E else None)
        self._check(self.lib.piadmm_get_step_state(self._h, _lib.dptr(out["xt"]), e("hat"), e("lam"), e("S"),
                                                   e("D"), e("last_hat"), e("rho_pi")))
        out["t"] = self.t
        return out

    def set_state(self, st: dict):
        """Resume from a checkpoint (:meth:`step_state`, or piadmm.io.load_checkpoint): xt and the
        carried pair state; the next :meth:`mpc_step` runs at st["t"] when given."""
        H1 = self.cfg.H + 1
        xt = np.ascontiguousarray(st["xt"], np.float64).reshape(self.N, 3)

        def arr(k, shape):
            v = st.get(k)
            if v is None or not self.E:
                return None
            return np.ascontiguousarray(v, np.float64).reshape(shape)
        parts = [arr(k, (self.E, 2, 2, H1)) for k in ("hat", "lam", "S", "D", "last_hat")]
        rho = arr("rho_pi", (self.E,))
        self._check(self.lib.piadmm_set_state(self._h, _lib.dptr(xt), *[_lib.dptr(p) for p in parts], _lib.dptr(rho)))
        self.xt = xt.copy()
        if st.get("t") is not None:
            self.t = int(st["t"])

    def set_xt(self, xt: np.ndarray):
        xt = np.ascontiguousarray(xt, np.float64)
        self._check(self.lib.piadmm_set_xt(self._h, _lib.dptr(xt)))
        self.xt = xt.copy()

    def state(self) -> dict:
        """xt, u, pos_old, hat, lam and the PI accumulators S, D (ADMM_CVX_..._PI_antiwindup.m:160-188)
        of the last step -- or of the last outer iteration of a host-stepped step."""
        H1 = self.cfg.H + 1
        out = dict(xt=np.empty((self.N, 3)), u=np.empty((self.N, self.cfg.H)),
                   pos_old=np.empty((self.N, 2, H1)), hat=np.empty((self.E, 2, 2, H1)),
                   lam=np.empty((self.E, 2, 2, H1)), S=np.empty((self.E, 2, 2, H1)), D=np.empty((self.E, 2, 2, H1)),
                   edge_active=np.empty(self.E, np.uint8), iters=np.empty(self.C, np.int32))
        ea = out["edge_active"].ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if self.E else None
        e = (lambda k: _lib.dptr(out[k]) if self.E else None)
        self._check(self.lib.piadmm_get_state(
            self._h, _lib.dptr(out["xt"]), _lib.dptr(out["u"]), _lib.dptr(out["pos_old"]),
            e("hat"), e("lam"), e("S"), e("D"), ea, _lib.iptr(out["iters"])))
        return out

    def outer_iter(self, it: int, t: int | None = None) -> bool:
        """ONE outer ADMM iteration of MPC step t (``for i_iter``, casadi/main.py:78-181): it = 0
        starts the step, then 1, 2, ... in order; :meth:`state` shows the iteration's pos_old, hat,
        lam, S, D.  Returns True when the reference's stop rules end the step here.  Finish the
        step with :meth:`step_finish`."""
        t = self.t if t is None else t
        stop = ctypes.c_int32()
        self._check(self.lib.piadmm_outer_iter(self._h, int(t), int(it), ctypes.byref(stop)))
        self._stepping = int(t)
        return bool(stop.value)

    def step_finish(self):
        """Propagate a host-stepped MPC step (casadi/main.py:185-192); returns (xt, u)."""
        xt = np.empty((self.N, 3))
        u = np.empty((self.N, self.cfg.H))
        self._check(self.lib.piadmm_step_finish(self._h, _lib.dptr(xt), _lib.dptr(u)))
        self.t = getattr(self, "_stepping", self.t) + 1
        self.xt = xt
        return xt, u

    def close(self):
        if getattr(self, "_h", None):
            self.lib.piadmm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def device_count() -> int:
    return int(_lib.load().piadmm_device_count())


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 creates it and ships it to the other ranks)."""
    buf = (ctypes.c_uint8 * 128)()
    _lib.check(_lib.load().piadmm_comm_unique_id(buf))
    return bytes(buf)
