"""OBCA local subproblem on the GPU: batched SQP (csrc/piadmm_obca.hip) behind
``piadmm_obca_solve`` (include/piadmm.h).

Mirrors the vehicle side of ``OBCAOptimizer`` (Distributed_planner/decentralized/optimizer.py):
``local_initialize`` + ``local_build_model`` + ``local_generate_constrain`` +
``local_generate_variable`` + ``local_generate_object`` + ``local_solve`` (:40-201) become one
record per (vehicle, ADMM iterate) and one batched call; ``bar_state`` keeps the reference's
arrays (``Z_bar``, ``A``, ``b``, ``lamb_bar``, ``lamb_ij``, ``local_x``, :351-373) and
``iterate_next_state`` (:337-344) shifts them.

Record layout (float64, ``REC`` per problem) -- what the reference's local NLP reads:
  init 5 | ref 8x5 (ref_traj[veh][t_step + k], also the initial X guess) | A_o 7x4x2 | b_o 7x4 |
  lamb_ij_o 7x4 (the other vehicle's bar_state slots) | lamb_bar 7x9 | Z_bar 7x9 |
  rho, min_dis, max_x, max_y, r, q, prob, max_iter | pad
Output (float64, ``OUT`` per problem): X 8x5 | U 7x2 | Lambda 7x4 | y_a 7 | y_b 7x2 | y_n 7 |
  y_x 7x5 | pi 7x5 | y_u 14 | y_l 28 | cost | pad;  status / SQP iterations / QP steps (int32 x 3).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

N_HORZ, NX, NU, NL = 8, 5, 2, 4
NT = N_HORZ - 1
REC = 296
OUT = 224
_O_INIT, _O_REF, _O_AO, _O_BO, _O_LIJ, _O_LB, _O_ZB, _O_PAR = 0, 5, 45, 101, 129, 157, 220, 283

STATUS = {0: "converged", 1: "max_iter", 2: "qp_infeasible", 3: "linesearch_fail", 4: "hessian_fail"}

# VehicleConfig (veh_config.py:7-27)
LENGTH, WIDTH = 3.5, 2.0
DT, T_PERIOD = 0.1, 5.0
AVG_DELAY, VAR_DELAY, DELAY_PROB = 0.05, 0.025, 0.95


def ref_traj_gen():
    """The overtaking scenario's references (veh_config.py:30-47)."""
    n = int(T_PERIOD / DT) + 1
    out = []
    for v, x0 in ((20.0, 0.0), (10.0, 20.0)):
        x = np.linspace(x0, x0 + v * T_PERIOD, n)
        out.append(np.vstack((x, np.zeros_like(x), v * np.ones_like(x), np.zeros_like(x), np.zeros_like(x))).T)
    return out


def halfspaces(state, prob):
    """(A, b) of a vehicle at `state` -- the halfspaces bar_state_update exchanges
    (optimizer.py:205-222 via util.py:12-101)."""
    x, y, v, th = state[0], state[1], state[2], state[3]
    c, s = math.cos(th), math.sin(th)
    e, n = np.array([c, s]), np.array([-s, c])
    if prob:
        A = np.vstack([e, n, -e, -n])
        sig = math.sqrt(DELAY_PROB / (1.0 - DELAY_PROB))
        d = np.array([AVG_DELAY * v * c + sig * (VAR_DELAY * v * c) ** 2,
                      AVG_DELAY * v * s + sig * (VAR_DELAY * v * s) ** 2])
    else:
        A = np.vstack([e, -n, -e, n])
        d = np.zeros(2)
    b0 = np.array([LENGTH / 2, WIDTH / 2, LENGTH / 2, WIDTH / 2])
    return A, b0 + A @ (np.array([x, y]) + d)


def separating_duals(A_o, u, alpha):
    """lamb_ij of the other vehicle with A_o' lamb_ij = alpha * u (u a unit vector pointing from
    the other vehicle towards this one), the smallest such non-negative vector."""
    lam = np.zeros(4)
    # rows come in opposite pairs (0, 2) and (1, 3)
    for r0, r1 in ((0, 2), (1, 3)):
        comp = float(A_o[r0] @ u)
        lam[r0] = alpha * max(comp, 0.0)
        lam[r1] = alpha * max(-comp, 0.0)
    return lam


def pack(init, ref, A_o, b_o, lamb_ij_o, lamb_bar, Z_bar, rho=1.0, min_dis=0.1, max_x=150.0, max_y=20.0,
         r=1e4, q=1e5, prob=1, max_iter=60):
    rec = np.zeros(REC)
    rec[_O_INIT:_O_INIT + 5] = init
    rec[_O_REF:_O_REF + 40] = np.asarray(ref, np.float64).ravel()
    rec[_O_AO:_O_AO + 56] = np.asarray(A_o, np.float64).ravel()
    rec[_O_BO:_O_BO + 28] = np.asarray(b_o, np.float64).ravel()
    rec[_O_LIJ:_O_LIJ + 28] = np.asarray(lamb_ij_o, np.float64).ravel()
    rec[_O_LB:_O_LB + 63] = np.asarray(lamb_bar, np.float64).ravel()
    rec[_O_ZB:_O_ZB + 63] = np.asarray(Z_bar, np.float64).ravel()
    rec[_O_PAR:_O_PAR + 8] = [rho, min_dis, max_x, max_y, r, q, float(prob), float(max_iter)]
    return rec


def unpack(rec):
    """dict of the record's fields (the oracle builds its LocalProblem from this)."""
    rec = np.asarray(rec, np.float64)
    par = rec[_O_PAR:_O_PAR + 8]
    return dict(init=rec[_O_INIT:_O_INIT + 5].copy(), ref=rec[_O_REF:_O_REF + 40].reshape(8, 5).copy(),
                A_o=rec[_O_AO:_O_AO + 56].reshape(7, 4, 2).copy(), b_o=rec[_O_BO:_O_BO + 28].reshape(7, 4).copy(),
                lamb_ij_o=rec[_O_LIJ:_O_LIJ + 28].reshape(7, 4).copy(),
                lamb_bar=rec[_O_LB:_O_LB + 63].reshape(7, 9).copy(), Z_bar=rec[_O_ZB:_O_ZB + 63].reshape(7, 9).copy(),
                rho=par[0], min_dis=par[1], max_x=par[2], max_y=par[3], r=par[4], q=par[5], prob=int(par[6]),
                max_iter=int(par[7]))


def executed_path(veh, tau):
    """Collision-free executed states of the overtaking manoeuvre at time tau (s): vehicle 1 on
    its reference (veh_config.py:41-45); vehicle 0 at 20 m/s changing to y = +lane between
    0.2 s and 0.8 s and back between 3.0 s and 3.6 s (smoothstep profiles, heading = path
    tangent).  The reference's own references run vehicle 0 through vehicle 1; these are the
    states a converged run would exchange."""
    if veh == 1:
        return np.array([20.0 + 10.0 * tau, 0.0, 10.0, 0.0, 0.0])
    lane = 4.0

    def sstep(u):
        u = min(max(u, 0.0), 1.0)
        return u * u * (3 - 2 * u), 6 * u * (1 - u)

    a, da = sstep((tau - 0.2) / 0.6)
    b, db = sstep((tau - 3.0) / 0.6)
    y = lane * (a - b)
    dy = lane * (da - db) / 0.6
    return np.array([20.0 * tau, y, 20.0, math.atan2(dy, 20.0), 0.0])


def overtaking_problem(t_step, veh, variant="initial", prob=1, seed=0, alpha=0.9):
    """One local problem of the two-vehicle overtaking scenario (decentralized_overtaking_ADMM.py:
    22-42: VehicleConfig references, N_horz 8, min_dis 0.1, max_x 150, max_y 20, rho 1).

    ref = the vehicle's reference window ref_traj[veh][t_step:t_step+8] (local_initialize,
    optimizer.py:51-53); init = its executed state (`executed_path`); the other vehicle's
    bar_state slots are the halfspaces of ITS executed states (what bar_state_update exchanges,
    :205-222) and duals lamb_ij separating the two boxes along the centre-to-centre direction.
    variant:
      "initial"   lamb_bar = 1e-3, Z_bar = 0 (the reference's mid_state values, :353-356);
      "consensus" Z_bar = [executed state; 0.5], lamb_bar random (an ADMM iterate's shape);
      "perturbed" like consensus with a perturbed initial state.
    """
    rng = np.random.default_rng(seed * 7919 + t_step * 31 + veh)
    refs = ref_traj_gen()
    o = 1 - veh
    ref = refs[veh][t_step:t_step + N_HORZ].copy()
    init = executed_path(veh, t_step * DT)
    A_o = np.zeros((NT, 4, 2))
    b_o = np.zeros((NT, 4))
    lij = np.zeros((NT, 4))
    mine = np.stack([executed_path(veh, (t_step + t) * DT) for t in range(1, N_HORZ)])
    for t in range(1, N_HORZ):
        so = executed_path(o, (t_step + t) * DT)
        A, b = halfspaces(so, prob)
        A_o[t - 1], b_o[t - 1] = A, b
        dvec = mine[t - 1][:2] - so[:2]
        lij[t - 1] = separating_duals(A, dvec / np.linalg.norm(dvec), alpha)
    if variant == "initial":
        lamb_bar = 1e-3 * np.ones((NT, 9))
        Z_bar = np.zeros((NT, 9))
    else:
        lamb_bar = 0.1 * rng.standard_normal((NT, 9))
        Z_bar = np.concatenate([mine, 0.5 * np.ones((NT, 4))], axis=1)
        Z_bar[:, :5] += 0.05 * rng.standard_normal((NT, 5))
    if variant == "perturbed":
        init = init + np.array([0.2, 0.1, -1.0, 0.02, 0.02]) * rng.uniform(-1, 1, 5)
        init[2] = min(init[2], 20.0 - 0.5)
    return pack(init, ref, A_o, b_o, lij, lamb_bar, Z_bar, prob=prob)


MID_LAMB_IJ = np.stack([
    np.array([[1.49, 0.566, 0.566, 1.49], [1.438, 0.514, 0.514, 1.438], [1.387, 0.462, 0.462, 1.387],
              [1.336, 0.411, 0.411, 1.336], [1.287, 0.361, 0.361, 1.287], [1.238, 0.312, 0.312, 1.238],
              [1.191, 0.263, 0.263, 1.191]]),
    np.repeat(np.array([1.436, 1.325, 1.213, 1.1, 0.986, 0.871, 0.755])[:, None], 4, axis=1)])


def create_bar_state(num_veh=2):
    """The initial bar_state (`mid_state`, optimizer.py:351-373): Z_bar, A, b, local_x zero,
    lamb_bar 1e-3, lamb_ij the hard-coded values of the reference."""
    return dict(Z_bar=np.zeros((num_veh, NT, 9)), A=np.zeros((num_veh, NT, 4, 2)), b=np.zeros((num_veh, NT, 4)),
                lamb_bar=1e-3 * np.ones((num_veh, NT, 9)), lamb_ij=MID_LAMB_IJ[:num_veh].copy(),
                local_x=np.zeros((num_veh, NT, 5)))


def iterate_next_state(bar):
    """Receding-horizon shift (optimizer.py:337-344): every array drops slot 0 and repeats its
    last slot."""
    out = dict(bar)
    for k in ("Z_bar", "A", "b", "lamb_bar", "lamb_ij", "local_x"):
        a = bar[k]
        out[k] = np.concatenate((a[:, 1:], a[:, -1:]), axis=1)
    return out


def bar_state_update(bar, bar_fullx, prob=1):
    """`bar_state_update` (optimizer.py:205-222): each vehicle's halfspaces at its new local
    states (the lamb_ij update stays commented out, as in the reference, :220)."""
    out = {k: v.copy() for k, v in bar.items()}
    for t in range(NT):
        for v in range(len(bar_fullx)):
            st = np.asarray(bar_fullx[v])[t, :5]
            A, b = halfspaces(st, prob)
            out["A"][v, t] = A
            out["b"][v, t] = b
            out["local_x"][v, t] = st
    return out


def local_record(bar, veh, t_step, init_state, ref_traj, rho=1.0, min_dis=0.1, prob=1, max_x=150.0, max_y=20.0,
                 r=1e4, q=1e5, max_iter=60):
    """The record of vehicle `veh`'s local NLP: what local_initialize (:40-58) +
    local_generate_constrain (:84-129, the OTHER vehicle's bar_state slots) +
    local_generate_variable + local_generate_object (:150-168, this vehicle's lamb_bar and Z_bar)
    read, for one batched `OBCABatch.solve`."""
    o = 1 - veh
    ref = np.asarray(ref_traj[veh], np.float64)[t_step:t_step + N_HORZ]
    return pack(np.asarray(init_state, np.float64).ravel(), ref, bar["A"][o], bar["b"][o], bar["lamb_ij"][o],
                bar["lamb_bar"][veh], bar["Z_bar"][veh], rho=rho, min_dis=min_dis, max_x=max_x, max_y=max_y, r=r,
                q=q, prob=prob, max_iter=max_iter)


def as_written_problem(t_step=0, veh=0, prob=1):
    """The reference's first ADMM iterate as written: bar_state = mid_state (A = b = 0, the
    hard-coded lamb_ij, lamb_bar = 1e-3, Z_bar = 0; optimizer.py:351-373).  (5b) then forces
    A(X_t)' Lambda_t = 0, so (5a) reads -b0' Lambda >= 0.1 with Lambda >= 0: infeasible."""
    refs = ref_traj_gen()
    return local_record(create_bar_state(), veh, t_step, refs[veh][t_step], refs, prob=prob)


def scenario_batch(n, prob=1, seed=0):
    """n local problems cycling over (t_step 0..41, vehicle, variant) of the overtaking scenario."""
    recs = []
    variants = ("initial", "consensus", "perturbed")
    k = 0
    while len(recs) < n:
        t_step = k % 42
        veh = (k // 42) % 2
        var = variants[(k // 84) % 3]
        recs.append(overtaking_problem(t_step, veh, var, prob=prob, seed=seed + k // 252))
        k += 1
    return np.ascontiguousarray(np.stack(recs))


class OBCAResult:
    """Decoded output of a batch (fields as in the reference's local_solve, :183-201)."""

    def __init__(self, out, ist):
        self.raw = out
        self.X = out[:, :40].reshape(-1, 8, 5)
        self.U = out[:, 40:54].reshape(-1, 7, 2)
        self.Lam = out[:, 54:82].reshape(-1, 7, 4)
        self.y_a = out[:, 82:89]
        self.y_b = out[:, 89:103].reshape(-1, 7, 2)
        self.y_n = out[:, 103:110]
        self.y_x = out[:, 110:145].reshape(-1, 7, 5)
        self.pi = out[:, 145:180].reshape(-1, 7, 5)
        self.y_u = out[:, 180:194]
        self.y_l = out[:, 194:222]
        self.cost = out[:, 222]
        self.status = ist[:, 0]
        self.iters = ist[:, 1]
        self.qp_steps = ist[:, 2]

    def bar_fullx(self, k):
        """N_horz-1 x 9 [X_t, Lambda_t] of problem k (optimizer.py:201)."""
        return np.concatenate([self.X[k, 1:], self.Lam[k]], axis=1)


class OBCABatch:
    """Device-resident batch of local problems.  ``solve`` runs one launch of the batched SQP
    (one wave per problem) and returns an OBCAResult; there is no CPU path."""

    def __init__(self, device: int = 0):
        from . import _lib
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        rc = self._lib.piadmm_obca_create(int(device), ctypes.byref(self._h))
        if rc != 0:
            raise _lib.PiadmmError(f"piadmm_obca_create failed ({rc})")

    def _check(self, rc):
        from . import _lib
        if rc != 0:
            msg = self._lib.piadmm_obca_last_error(self._h)
            raise _lib.PiadmmError(f"libpiadmm error {rc}: {msg.decode() if msg else ''}")

    def close(self):
        if self._h:
            self._lib.piadmm_obca_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve(self, recs: np.ndarray) -> OBCAResult:
        from . import _lib
        recs = np.ascontiguousarray(recs, np.float64)
        n = recs.shape[0]
        assert recs.shape == (n, REC)
        out = np.zeros((n, OUT))
        ist = np.zeros((n, 3), np.int32)
        self._check(self._lib.piadmm_obca_solve(self._h, _lib.dptr(recs), n, _lib.dptr(out), _lib.iptr(ist)))
        return OBCAResult(out, ist)

    def upload(self, recs: np.ndarray):
        from . import _lib
        recs = np.ascontiguousarray(recs, np.float64)
        self._check(self._lib.piadmm_obca_upload(self._h, _lib.dptr(recs), recs.shape[0]))

    def run_async(self, repeats: int = 1):
        self._check(self._lib.piadmm_obca_run(self._h, int(repeats)))

    def time(self, repeats: int) -> float:
        """ms per launch over `repeats` launches on the resident batch (HIP events)."""
        ms = ctypes.c_float()
        self._check(self._lib.piadmm_obca_time(self._h, int(repeats), ctypes.byref(ms)))
        return ms.value

    def download(self, n: int) -> OBCAResult:
        from . import _lib
        out = np.zeros((n, OUT))
        ist = np.zeros((n, 3), np.int32)
        self._check(self._lib.piadmm_obca_download(self._h, _lib.dptr(out), _lib.iptr(ist), n))
        return OBCAResult(out, ist)
