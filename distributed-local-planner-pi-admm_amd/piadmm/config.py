"""PI-ADMM configuration: the Python mirror of ``piadmm_config_t`` (include/piadmm.h).

The reference keeps its parameters in a ``Bunch`` built in
``casadi/PI_ADMM_class.py:15-28`` plus driver constants (``casadi/main.py:18-27``)
and, for the PI anti-windup variant, the MATLAB block
``matlab_old_files/ADMM_CVX_two_veh_intesection_PI_antiwindup.m:6-25,43``.
Those become one frozen struct with named presets.  Every reference quirk that
changes numbers is an explicit flag here, so a preset
reproduces exactly one reference script.

Field order and types must match ``piadmm_config_t`` byte for byte; the ctypes
mirror lives in ``piadmm/_lib.py`` and ``tests/test_capi.py`` checks the size.
"""
from __future__ import annotations

import dataclasses
import math

# dual-update modes
DUAL_PLAIN = 0      # lam += rho*(p - hat)            casadi/main.py:161-162
DUAL_PI = 1         # per-edge PI + back-calculation   ADMM_CVX_..._PI_antiwindup.m:156-188
DUAL_PI_GLOBAL = 2  # PI with adaptive rho and K_P     casadi_old_PI_ADMM/main.py:133-151

# position model used for pos_old (quirk B15)
POS_LINEAR = 0      # Python dynamic_update_local (heading frozen)   casadi/PI_ADMM_class.py:59-69
POS_NONLINEAR = 1   # MATLAB dynamic_update_local numeric branch      ADMM_CVX_...:312-330


@dataclasses.dataclass(frozen=True)
class PIADMMConfig:
    # --- problem (casadi/PI_ADMM_class.py:15-28) ---
    H: int = 15                 # num_ho
    max_outer: int = 100        # iter_num
    dt: float = 0.1
    L: float = 1.0
    dis_thres: float = 2.0
    beta: float = 10.0
    Pnorm: float = 1.0
    Pcost: float = 1.0
    rho: float = 2.0
    eps_pri: float = 20.0
    eps_dual: float = 1.0
    u_max: float = math.pi / 6      # nonlcon_function :173-174
    du_max: float = math.pi / 9     # nonlcon_function :179-180
    # --- dual update (MATLAB PI anti-windup :20-25,43) ---
    dual_mode: int = DUAL_PLAIN
    windup: int = 0             # 1: saturate + back-calculate (:169-188)
    kP: float = 0.0
    kI: float = 0.0
    theta1: float = 5.0
    theta2: float = 3.0
    windup_sat: float = 30.0
    # --- reference quirks ---
    round_decimals: int = 4     # B6: np.around(.,4) on u, u_hat, seeds; -1 = off
    collide_sq_thres: int = 0   # B2: 0 = Python (d^2 < dis_thres), 1 = MATLAB (d^2 < dis_thres^2)
    alias_dual_residual: int = 1  # B4: Python last_iter_hat_pos aliasing -> s_k == 0 after iter 1
    pos_model: int = POS_LINEAR   # B15: pos_old rollout model
    term_dist_check: int = 0    # MATLAB extra stop condition dis_vec(2) > dis_thres (:202)
    fixed_iters: int = 0        # 1: never terminate early (throughput runs)
    # --- N-agent semantics and hot-path extensions (B9) ---
    term_global: int = 0        # B9: 1 = flag / termination over ALL agents (reference, casadi/main.py:115-118,174);
                                #     0 = per connected component (N-agent generalisation)
    warm_duals: int = 0         # a12: 1 = receding-horizon shift of hat / lam / S / D between MPC steps
                                #      (OBCA iterate_next_state, decentralized/optimizer.py:337-344)
    tighten: int = 0            # a13: 1 = delay-tightened safety distance (decentralized/util.py:70-101)
    tight_p: float = 0.95       # VehicleConfig.prob       (veh_config.py:27)
    avg_delay: float = 0.05     # VehicleConfig.avg_delay  (veh_config.py:25)
    var_delay: float = 0.025    # VehicleConfig.var_delay  (veh_config.py:26)
    precision: int = 0          # 1: ADMM matrices K_s^-1 in fp32 (mixed precision; the polish and its
                                #    certificate stay fp64, so answers do not change) -- configs[4] study
    # --- global PI with adaptive rho and K_P (casadi_old_PI_ADMM/main.py:133-151) ---
    rho_num: float = 4.0        # rho = max(rho_min, min(rho_max, rho_num / dis_min))   (:139)
    rho_min: float = 1.0
    rho_max: float = 5.0
    no_collision_gate: int = 0  # 1: every candidate pair's QP every iteration (the script has no
                                #    collision test: its edge problem is solved unconditionally, :96-115)
    pi_trad: int = 0            # 1: the scripts' `trad == 1` branch: lam += rho e + D (casadi_old_PI_ADMM/main.py:138-139)
    # --- the adaptive-gain global PI (ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m:121-146) ---
    ki_adapt: int = 0           # 1: K_I = kI / dis_min (K_I_coeff / dis_min, :127); 0: K_I = kI (casadi_old :135)
    reserved1: int = 0
    d_gain: float = 2.0         # S += K_I e + d_gain D: 2 (casadi_old_PI_ADMM/main.py:142), 1 (adp :135)
    dual_init: float = 0.0      # hat, lam, last_hat at each step's start: 0 (casadi/main.py:56-63) or 1e-4 (adp :59-61)
    # --- inner QP solver (build's own; not in the reference) ---
    admm_rho: float = 0.05      # ADMM penalty in the Ruiz-scaled space (tools/qp_sim.py sweep)
    admm_sigma: float = 1e-6
    admm_alpha: float = 1.6
    max_inner: int = 4000       # ADMM iteration cap per QP
    polish_every: int = 5       # try an active-set polish every k ADMM iterations
    qp_tol: float = 1e-9        # KKT acceptance tolerance of a polished solution

    def replace(self, **kw) -> "PIADMMConfig":
        return dataclasses.replace(self, **kw)

    @property
    def thr_collide(self) -> float:
        return self.dis_thres ** 2 if self.collide_sq_thres else self.dis_thres

    def collide_thr(self, d_eff: float) -> float:
        """Collision-test threshold for safety distance d_eff (B2: Python compares d^2 with d_eff)."""
        return d_eff * d_eff if self.collide_sq_thres else d_eff


def casadi_default(**kw) -> PIADMMConfig:
    """``casadi/PI_ADMM_class.py:15-28`` + ``casadi/main.py`` (plain dual, rounding, aliasing)."""
    return PIADMMConfig().replace(**kw)


def matlab_pi(**kw) -> PIADMMConfig:
    """``ADMM_CVX_two_veh_intesection_PI_antiwindup.m:6-25,43``: per-edge PI + back-calculation."""
    base = PIADMMConfig(
        H=8, max_outer=100, dt=0.1, L=1.0, dis_thres=2.0, beta=1000.0, Pnorm=5.0,
        Pcost=1.0, rho=3.5, eps_pri=0.1, eps_dual=0.1, dual_mode=DUAL_PI, windup=1,
        kP=0.0, kI=3.5, theta1=5.0, theta2=3.0, windup_sat=30.0, round_decimals=-1,
        collide_sq_thres=1, alias_dual_residual=0, pos_model=POS_NONLINEAR,
        term_dist_check=1)
    if "rho" in kw and "kI" not in kw:
        kw["kI"] = kw["rho"]    # param.kI = param.rho (:21)
    return base.replace(**kw)


def casadi_old_pi(**kw) -> PIADMMConfig:
    """``casadi_old_PI_ADMM/main.py`` + its ``PI_ADMM_class.py:15-28``: the
    global PI law with adaptive rho and K_P (:133-151), the reference's QP costs (the script solves
    them with IPOPT, :78,114 -- convex QPs, so the same minimisers), no collision gate, aliased
    dual residual (:161), stop with dis_vec[1] > dis_thres (:156).  Build decision:
    the edge controls are rounded to 4 decimals like casadi/main.py:153 (the script's
    np.around without decimals, :120, rounds |u| <= pi/6 to 0, which is taken as a typo)."""
    base = PIADMMConfig(
        H=5, max_outer=100, dt=0.1, L=1.0, dis_thres=1.5, beta=1e4, Pnorm=5.0, Pcost=1.0,
        rho=1.0, eps_pri=1.0, eps_dual=1.0, dual_mode=DUAL_PI_GLOBAL, windup=1, kP=0.0, kI=3.0,
        theta1=5.0, theta2=2.5, windup_sat=20.0, round_decimals=4, collide_sq_thres=0,
        alias_dual_residual=1, pos_model=POS_LINEAR, term_dist_check=1, rho_num=4.0, rho_min=1.0,
        rho_max=5.0, no_collision_gate=1)
    return base.replace(**kw)


def matlab_adp_pi(**kw) -> PIADMMConfig:
    """``matlab_old_files/ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m``: the global PI law
    with adaptive gains (:121-147) -- from the minimum distance d of the x-step plans (nonlinear
    rollouts, :121-125), K_I = K_I_coeff / d (:127, K_I_coeff = 3, :51), K_P = min(5 / d, 3)
    (:128), rho = max(1, min(5, 4 / d)) (:129, kept across MPC steps: param.rho is never reset);
    lam = S + K_P e, S += K_I e + D (the back-calculation added once, :134-135), or with ``trad``
    lam += rho e + D (:131-132); saturation +-50 (:40) with back-calculation over the whole dual
    array (:138-147); hat = lam = 1e-4 at each step's start (:59-61); residuals over both sides
    without the factor 2 (:151-152) and the stop test without the distance check (:154, commented
    out); the edge problem solved every iteration (:94-110, no collision test); parameters :3-16
    (H = 5, dis_thres 1.5, beta 1000, Pnorm 5, Pcost 1, rho 1, eps 1 / 1).  CVX solves exactly
    (no rounding); pos_old is the numeric dynamic_update_local (its nargin == 4 branch: the
    nonlinear rollout); the steering box is two-sided as in nonlcon_function (the script's
    one-sided ``veh_u <= pi/6``, :80, is the same typo as in the per-edge PI script)."""
    base = PIADMMConfig(
        H=5, max_outer=100, dt=0.1, L=1.0, dis_thres=1.5, beta=1000.0, Pnorm=5.0, Pcost=1.0,
        rho=1.0, eps_pri=1.0, eps_dual=1.0, dual_mode=DUAL_PI_GLOBAL, windup=1, kP=0.0, kI=3.0,
        theta1=5.0, theta2=3.0, windup_sat=50.0, round_decimals=-1, collide_sq_thres=1,
        alias_dual_residual=0, pos_model=POS_NONLINEAR, term_dist_check=0, rho_num=4.0, rho_min=1.0,
        rho_max=5.0, no_collision_gate=1, pi_trad=0, ki_adapt=1, d_gain=1.0, dual_init=1e-4)
    return base.replace(**kw)


PRESETS = {"casadi_default": casadi_default, "matlab_pi": matlab_pi, "casadi_old_pi": casadi_old_pi,
           "matlab_adp_pi": matlab_adp_pi}
