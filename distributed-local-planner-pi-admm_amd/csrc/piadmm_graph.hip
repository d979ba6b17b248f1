// piadmm_graph.hip -- graph mode of libpiadmm: the PI-ADMM MPC step on ANY static candidate
// graph (MI355X, gfx950).
//
// The reference loop is written for num_veh vehicles (casadi/main.py:43-201): every agent's
// x-step sums the augmented-Lagrangian term over its neighbours (PI_ADMM_class.py:126-129),
// the collision test covers every candidate pair (main.py:110-113) and every colliding pair
// gets its own edge QP and dual update (main.py:121-162).  piadmm_device.hip's fused kernel is
// specialised for components of one or two agents (the tiled benchmark); this kernel takes
// components of any size and agents in any number of pairs (an all-pairs 4-vehicle scene, a
// chain, a grid of crossings).
//
// One workgroup (GW waves) per connected component; one persistent launch = up to 32 MPC steps.
// An outer iteration is three phases separated by workgroup barriers:
//   X  every agent of the component (waves strided over its agents): the x-step QP with the
//      consensus term summed over its candidate neighbours in neighbour order, rounding,
//      rollout -> pos_old, u
//   Z  every candidate pair (waves strided): the collision test; when it collides the pair QP,
//      the nonlinear hat rollouts, the plain / PI anti-windup dual update and the pair's
//      residual contributions
//   T  wave 0: the component's residual sums in pair order and the reference's stop rules
// Each QP's warm state (ADMM iterates, labels, parametric-table signature, penalty) lives in
// HBM between phases -- the matrices already do (the big-mode layout of the fused kernel:
// agent K_s^-1, P^-1, G, X', the pair tables and K_s^-1), so a wave can serve any agent or pair.
// The QP solver itself (pd_qp.h) and the per-step setup (pd_setup.h) are the fused kernel's.
//
// Global termination (term_global) uses the fused kernel's two mechanisms: in-kernel behind a
// grid barrier (cooperative launch, one rank) or one launch per outer iteration with the stop
// decided on the host from all-reduced partials (RCCL).  F_XONLY / F_ZONLY split an iteration
// launch at the position exchange of a sharded job (piadmm_capi.cpp).

#include "pd_setup.h"

namespace pd {

struct GWave {
  double* fac;     // LDS factor / matrix scratch of this wave (x-step and pair, in turn)
  double* vb;      // LDS vectors (512)
  double* xdiag;   // LDS x factor diagonals (128)
  double* zdiag;   // LDS pair factor diagonals (128)
  double* ylds;    // LDS dual active-set columns (H <= HMAX), nullptr: HBM (big mode)
  int *xids, *zids, *xfs, *zfs;
};

struct GCnt {
  int xqp = 0, zqp = 0, admm_x = 0, admm_z = 0, pdas_x = 0, pdas_z = 0, inexact = 0, gi = 0;
};

// -------------------------------------------------------------------- X phase: one agent
template <bool BIG, bool TIES>
__device__ __forceinline__ void g_xstep(const DevArgs& A, int a, int t, int it, const GWave& W, GCnt& n) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, H1 = H + 1, l = lid();
  const bool tl = l <= H;
  const double* xt3 = A.xt + 3 * a;          // the state at the start of the MPC step
  const double s = A.spd[a];
  const Geo gx = make_geo(xt3, s, c);
  double cx, cy;
  affine_c(gx, c.dt, H, cx, cy);
  QP<1> qx;
  qp_common(c, H, A.rho_x[a], qx);
  qx.coefP = 0.0;                            // setup_agent: 2 Pnorm + rho |N(a)|
  qx.K = A.Kx_cache + (size_t)a * H * H;     // HBM / L2 (the big-mode layout at every H)
  qx.Kf = nullptr;
  qx.kf32 = false;
  qx.Pinv = A.Pinv_x + (size_t)a * H * H;
  qx.G = A.Gx_g + (size_t)a * (H * H + H);
  qx.XT = A.XT_g + (size_t)a * H1 * XLDG;
  qx.xld = XLDG;
  qx.gmem = true;
  qx.vb = W.vb;
  qx.fac = W.fac;
  qx.fdiag = W.xdiag;
  qx.ib = W.xids;
  qx.fstate = W.xfs;
  qx.fld = xrows(H) + 1;
  qx.mmax = xrows(H);
  qx.gws = nullptr;
  qx.tstep = t;
  qx.t32 = A.T32_g ? A.T32_g + (size_t)a * (H * H + H * XLDG) : nullptr;
  // the dual active set's columns: LDS when they fit (H <= HMAX), else the agent's HBM buffer
  qx.Y = W.ylds ? W.ylds : A.Yx_g + (size_t)a * WAVE * H;
  qx.ycap = A.x_gi ? (W.ylds ? GYCAP : WAVE) : 0;
  qx.y_in_k = false;
  if (l == 0) W.xfs[0] = -1;                 // the wave's scratch served another QP before
  wsync();
  // global PI: each neighbour term weighted by its pair's adaptive penalty, so P's coefficient of
  // M'M is 2 Pnorm + sum_e rho_e (neighbour order) and the caches are keyed by it
  const bool gpi = c.dual_mode == PIADMM_DUAL_PI_GLOBAL;
  const int k0 = A.nbr_ptr[a], k1 = A.nbr_ptr[a + 1];
  double coef = -1.0;
  if (gpi) {
    double rs = 0.0;
    for (int k = k0; k < k1; ++k) rs = rs + A.rho_pi[A.nbr_edge[k]];
    coef = 2.0 * c.Pnorm + rs;
  }
  unsigned long long t_su = STAMP_T();
  const bool rebuilt = setup_agent(A, a, qx, gx, W.fac, coef);
  STAMP_ADD(ST_SETUP_X, t_su);
  STAMP_CNT(ST_N_XREBUILD, rebuilt ? 1 : 0);
  // warm state of this QP (written by the previous x-step of the agent, or the step init)
  const double* qs = A.qs_x + (size_t)a * 5 * WAVE;
  const signed char* ql = A.ql_x + (size_t)a * 2 * WAVE;
  double xs[1] = {qs[l]}, zs[2] = {qs[WAVE + l], qs[2 * WAVE + l]}, ys[2] = {qs[3 * WAVE + l], qs[4 * WAVE + l]};
  signed char lab[2] = {ql[l], ql[WAVE + l]};
  const bool warm = (A.xflags[a] & 1) != 0;
  qx.csig = rebuilt ? -1 : A.csig_x[(size_t)a * WAVE + l];
  // q of cost_function_primal (PI_ADMM_class.py:114-135): M'(2 Pnorm (c - r) + rho sum_j (c - hat_ij
  // + lam_ij)), the neighbours j in increasing order (the oracle's order)
  double vx = 0.0, vy = 0.0;
  if (tl) {
    const double* rp = A.ref + (size_t)a * 2 * A.T;
    vx = 2.0 * c.Pnorm * (cx - rp[t + l]);
    vy = 2.0 * c.Pnorm * (cy - rp[A.T + t + l]);
  }
  for (int k = k0; k < k1; ++k) {
    const int e = A.nbr_edge[k], d = A.nbr_dir[k];
    const double* hb = A.hat + (size_t)e * 4 * H1 + d * 2 * H1;
    const double* lb = A.lam + (size_t)e * 4 * H1 + d * 2 * H1;
    const double rw = gpi ? A.rho_pi[e] : c.rho;
    if (tl) {
      vx = vx + rw * (cx - hb[l] + lb[l]);
      vy = vy + rw * (cy - hb[H1 + l] + lb[H1 + l]);
    }
  }
  const double wt = tl ? gx.ax * vx + gx.ay * vy : 0.0;
  const double wsh = shdn(wt, 1);
  qx.wq = (l < H) ? wsh : 0.0;
  qx.qvalid = false;
  double ustar[1];
  unsigned long long t_q = STAMP_T();
  const int gi0 = n.gi;
  const int st = qp_solve<1, false, 8, BIG ? RM_S : RM_S | RM_Y>(qx, xs, zs, ys, lab, warm, c.max_inner, c.polish_every, W.fac, qx.fld,
                                             ustar, n.admm_x, n.pdas_x, n.gi);
  STAMP_ADD(ST_XQP, t_q);
  STAMP_CNT(ST_N_GIX, n.gi - gi0);
  ++n.xqp;
  n.inexact += (st & PIADMM_QP_INEXACT) ? 1 : 0;
  // round (casadi/main.py:103), pos_old = dynamic_update_local (:105)
  const double u = around(ustar[0], c.round_decimals);
  if (TIES && c.round_decimals >= 0) round_ties(A, t, it, PIADMM_TIE_ROUND_U, a, 0, ustar[0], l < H);
  double px, py, pth;
  rollout_r(xt3[0], xt3[1], xt3[2], s, s / c.L, (l < H) ? u : 0.0, c, H, c.pos_model != 0, px, py, pth);
  double* po = A.pos_old + (size_t)a * 2 * H1;
  if (tl) {
    po[l] = px;
    po[H1 + l] = py;
  }
  if (l < H) A.u[(size_t)a * H + l] = u;
  // a boundary agent's positions and controls go to the exchange buffer (owner-written slot)
  if (A.xbuf && A.xslot[a] >= 0) {
    double* xb = A.xbuf + (size_t)A.xslot[a] * (3 * H1);
    if (tl) {
      xb[l] = px;
      xb[H1 + l] = py;
    }
    if (l < H) xb[2 * H1 + l] = u;
  }
  // warm state back to HBM (scaled ADMM state, like the fused kernel between launches)
  if (qx.wraw) warm_to_scaled(qx, xs, zs, ys);
  double* qw = A.qs_x + (size_t)a * 5 * WAVE;
  signed char* lw = A.ql_x + (size_t)a * 2 * WAVE;
  qw[l] = xs[0];
  qw[WAVE + l] = zs[0];
  qw[2 * WAVE + l] = zs[1];
  qw[3 * WAVE + l] = ys[0];
  qw[4 * WAVE + l] = ys[1];
  lw[l] = lab[0];
  lw[WAVE + l] = lab[1];
  A.csig_x[(size_t)a * WAVE + l] = qx.csig;
  if (l == 0) {
    A.xflags[a] = 1;
    A.status[a] |= st;
    A.rho_x[a] = qx.rho;
    // an adapted penalty rebuilt K_s^-1 in place (the HBM cache is the matrix itself)
    if (A.xcache_rho[a] != qx.rho) A.xcache_rho[a] = qx.rho;
  }
}

// -------------------------------------------------------------------- Z phase: one pair
// Returns nothing; writes edge_active, and when the pair collides hat, lam, S, D, eres, dischk.
// The collision test of pair e (casadi/main.py:110-113): writes edge_active, returns it.
template <bool TIES>
__device__ __forceinline__ bool g_ztest(const DevArgs& A, int e, int t, int it) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, H1 = H + 1, l = lid();
  const bool tl = l <= H;
  const int v1 = A.edges[2 * e], v2 = A.edges[2 * e + 1];
  const double* p1 = A.pos_old + (size_t)v1 * 2 * H1;
  const double* p2 = A.pos_old + (size_t)v2 * 2 * H1;
  const double deff = A.deff[e];
  const double thr = c.collide_sq_thres ? deff * deff : deff;
  bool hit = false;
  double d2 = 0.0;
  if (tl) {
    const double dx = p1[l] - p2[l], dy = p1[H1 + l] - p2[H1 + l];
    d2 = dx * dx + dy * dy;
    hit = d2 < thr;
  }
  // the global-PI script has no collision test: its edge problem runs every iteration
  if (TIES && !c.no_collision_gate) collide_tie(A, t, it, e, d2, tl, thr);
  const bool act = c.no_collision_gate ? true : wany(hit);
  if (l == 0) A.edge_active[e] = act ? 1 : 0;
  return act;
}

// The z-step of a colliding pair e: the pair QP, the hat rollouts, the dual update and the pair's
// residual terms (casadi/main.py:121-173).
template <bool BIG, bool TIES>
__device__ __forceinline__ void g_zstep(const DevArgs& A, int e, int t, int it, const GWave& W, GCnt& n) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, H1 = H + 1, l = lid();
  const bool tl = l <= H;
  const int v1 = A.edges[2 * e], v2 = A.edges[2 * e + 1];
  const double* p1 = A.pos_old + (size_t)v1 * 2 * H1;
  const double* p2 = A.pos_old + (size_t)v2 * 2 * H1;
  const double deff = A.deff[e];
  double px[2] = {0.0, 0.0}, py[2] = {0.0, 0.0};
  if (tl) {
    px[0] = p1[l];
    py[0] = p1[H1 + l];
    px[1] = p2[l];
    py[1] = p2[H1 + l];
  }
  // pair QP of cost_function_edge (PI_ADMM_class.py:145-169), heading frozen at xt (B3)
  const double* xa = A.xt + 3 * v1;
  const double* xb = A.xt + 3 * v2;
  const Geo ge1 = make_geo(xa, A.spd[v1], c), ge2 = make_geo(xb, A.spd[v2], c);
  double c1x, c1y, c2x, c2y;
  affine_c(ge1, c.dt, H, c1x, c1y);
  affine_c(ge2, c.dt, H, c2x, c2y);
  double* Ke = A.Ke_g + (size_t)e * A.ke_stride;
  QP<2> qe;
  qe.H = H;
  qe.n = 2 * H;
  qe.umax = c.u_max;
  qe.dumax = c.du_max;
  qe.h0 = 0.0;
  qe.Pcost2 = 2.0 * c.Pcost;
  qe.beta = c.beta;
  qe.rho = A.rho_e[e];
  const bool gpi = c.dual_mode == PIADMM_DUAL_PI_GLOBAL;
  const double rw = gpi ? A.rho_pi[e] : c.rho;   // the pair's penalty (global PI: adaptive)
  qe.sigma = c.admm_sigma;
  qe.alpha = c.admm_alpha;
  qe.tol = c.qp_tol;
  qe.K = Ke;
  qe.Kf = nullptr;
  qe.kf32 = false;
  qe.Pinv = A.tab_e + (size_t)e * 8 * H * H;
  qe.vb = W.vb;
  qe.fac = W.fac;
  qe.fdiag = W.zdiag;
  qe.ib = W.zids;
  qe.fstate = W.zfs;
  qe.fld = LD;
  qe.mmax = WAVE;
  qe.gmem = true;
  qe.xld = 0;
  qe.G = nullptr;
  qe.XT = nullptr;
  // the dual active set's columns in LDS (H <= HMAX); big mode: in the pair's K_s^-1 region
  qe.Y = W.ylds ? W.ylds : Ke;
  qe.ycap = A.pair_gi ? (W.ylds ? GYCAP : min(WAVE, A.ke_stride / (2 * H))) : 0;
  qe.y_in_k = W.ylds == nullptr;
  qe.gws = A.gi_ws + (size_t)e * GI_WS;
  qe.gws_warm = A.pair_warm != 0;
  qe.wide = A.gi_wide ? A.gi_wide + ((size_t)blockIdx.x * GW + (threadIdx.x >> 6)) * A.gi_wide_stride : nullptr;
  // the pair's dual active set of its last solve in this step (not under the global-PI law: the
  // pair's penalty, hence P, changes every iteration)
  qe.snap = (A.gi_snap && c.dual_mode != PIADMM_DUAL_PI_GLOBAL)
                ? A.gi_snap + (size_t)e * ((size_t)WAVE * WAVE + (size_t)WAVE * 2 * H + WAVE) : nullptr;
  qe.tstep = t;
  qe.csig = -1;
  if (l == 0) W.zfs[0] = -1;
  wsync();
  const double sd[4] = {A.seed_g[2 * v1], A.seed_g[2 * v1 + 1], A.seed_g[2 * v2], A.seed_g[2 * v2 + 1]};
  unsigned long long t_sz = STAMP_T();
  setup_pair(A, e, qe, ge1, ge2, c1x, c1y, c2x, c2y, sd, W.fac, Ke, deff, gpi ? rw : -1.0);
  STAMP_ADD(ST_SETUP_Z, t_sz);
  const double* qs = A.qs_e + (size_t)e * 12 * WAVE;
  const signed char* ql = A.ql_e + (size_t)e * 5 * WAVE;
  double xs[2] = {qs[l], qs[WAVE + l]}, zs[5], ys[5];
  signed char lab[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    zs[q] = qs[(2 + q) * WAVE + l];
    ys[q] = qs[(7 + q) * WAVE + l];
    lab[q] = ql[q * WAVE + l];
  }
  const bool warm = (A.eflags[e] & 1) != 0;
  double* lam = A.lam + (size_t)e * 4 * H1;
  double* Sa = A.Sacc + (size_t)e * 4 * H1;
  double* Da = A.Dacc + (size_t)e * 4 * H1;
  double* hat = A.hat + (size_t)e * 4 * H1;
  const double* last = A.last + (size_t)e * 4 * H1;
  {
    double bx[2], by[2];
    bx[0] = tl ? px[0] + lam[0 * H1 + l] - c1x : 0.0;
    by[0] = tl ? py[0] + lam[1 * H1 + l] - c1y : 0.0;
    bx[1] = tl ? px[1] + lam[2 * H1 + l] - c2x : 0.0;
    by[1] = tl ? py[1] + lam[3 * H1 + l] - c2y : 0.0;
    const double w1 = tl ? ge1.ax * bx[0] + ge1.ay * by[0] : 0.0;
    const double w2 = tl ? ge2.ax * bx[1] + ge2.ay * by[1] : 0.0;
    const double q1 = Tt_apply(shdn(w1, 1)), q2 = Tt_apply(shdn(w2, 1));
    qe.q[0] = (l < H) ? -rw * q1 : 0.0;
    qe.q[1] = (l < H) ? -rw * q2 : 0.0;
    qe.qvalid = true;
  }
  double uh[2];
  unsigned long long t_zq = STAMP_T();
  const int giz0 = n.gi;
  const int st = qp_solve<2, BIG, XGEMV_U, BIG ? RM_S : RM_S | RM_Y>(qe, xs, zs, ys, lab, warm, c.max_inner, c.polish_every,
                                                 BIG ? Ke : W.fac, BIG ? 2 * H : LD, uh, n.admm_z, n.pdas_z, n.gi);
  STAMP_ADD(ST_ZQP, t_zq);
  STAMP_CNT(ST_N_GIZ, n.gi - giz0);
  STAMP_CNT(ST_N_ZQP, 1);
  STAMP_CNT(ST_N_ZFAIL, (st & PIADMM_QP_INEXACT) ? 1 : 0);
  ++n.zqp;
  n.inexact += (st & PIADMM_QP_INEXACT) ? 1 : 0;
  // hat positions: nonlinear rollout of the rounded pair controls (casadi/main.py:153-158)
  double hx[2], hy[2], hth;
  for (int v = 0; v < 2; ++v) {
    const double uv = (l < H) ? around(uh[v], c.round_decimals) : 0.0;
    if (TIES && c.round_decimals >= 0) round_ties(A, t, it, PIADMM_TIE_ROUND_UHAT, e, v * H, uh[v], l < H);
    rollout(v ? xb : xa, A.spd[v ? v2 : v1], uv, c, H, true, hx[v], hy[v], hth);
  }
  double rr = 0.0, ss = 0.0, dchk;
  if (gpi) {
    // global PI with adaptive rho and K_P (casadi_old_PI_ADMM/main.py:133-151; oracle
    // dual_update_global_pi): distances along the nonlinear rollouts of the x-step plans
    double nx[2], ny[2], nth;
    for (int v = 0; v < 2; ++v) {
      const int av = v ? v2 : v1;
      const double uv = (l < H) ? A.u[(size_t)av * H + l] : 0.0;
      rollout(v ? xb : xa, A.spd[av], uv, c, H, true, nx[v], ny[v], nth);
    }
    double dn;
    {
      const double dx = nx[0] - nx[1], dy = ny[0] - ny[1];
      dn = sqrt(dx * dx + dy * dy);
    }
    const double dmin = wmin(tl ? dn : INFINITY);
    const double kP = fmin(c.theta1 / dmin, c.theta2);
    // K_I: constant (casadi_old :135) or K_I_coeff / d_min (adaptive gains, ADMM_CVX_..._adp_PI_antiwindup1.m:127)
    const double kI = c.ki_adapt ? c.kI / dmin : c.kI;
    const double rnew = fmax(c.rho_min, fmin(c.rho_max, c.rho_num / dmin));
    double lraw[2][2], lsat[2][2];
    bool changed = false;
    for (int v = 0; v < 2; ++v) {
      double* Sv = Sa + v * 2 * H1;
      double* Dv = Da + v * 2 * H1;
      double* hv = hat + v * 2 * H1;
      for (int xy = 0; xy < 2; ++xy) {
        const double p = xy == 0 ? px[v] : py[v];
        const double h = xy == 0 ? hx[v] : hy[v];
        const double err = p - h;
        if (c.pi_trad) {
          // the scripts' trad branch: lam += rho e + D, the updated rho (casadi_old :138-139, adp :131-132)
          const double lo = tl ? lam[v * 2 * H1 + xy * H1 + l] : 0.0;
          const double dv = tl ? Dv[xy * H1 + l] : 0.0;
          lraw[v][xy] = (lo + rnew * err) + dv;
        } else {
          const double so = tl ? Sv[xy * H1 + l] : 0.0;
          lraw[v][xy] = so + kP * err;                        // lam = S + K_P e (casadi_old :141)
          // S += K_I e + d_gain D: d_gain 2 (casadi_old :142), 1 (adp :135)
          if (tl) Sv[xy * H1 + l] = (so + kI * err) + c.d_gain * Dv[xy * H1 + l];
        }
        lsat[v][xy] = c.windup ? fmin(c.windup_sat, fmax(lraw[v][xy], -c.windup_sat)) : lraw[v][xy];
        changed |= tl && (lsat[v][xy] != lraw[v][xy]);
        if (tl) hv[xy * H1 + l] = h;
      }
    }
    const bool anyc = wany(changed);                           // over the whole pair (:148)
    for (int v = 0; v < 2; ++v)
      for (int xy = 0; xy < 2; ++xy)
        if (tl) {
          lam[v * 2 * H1 + xy * H1 + l] = lsat[v][xy];
          if (c.windup) Da[v * 2 * H1 + xy * H1 + l] = anyc ? lsat[v][xy] - lraw[v][xy] : 0.0;
        }
    // residuals (:153-154): both sides, no factor 2, the updated penalty
    if (tl) {
      for (int v = 0; v < 2; ++v) {
        const double ex = px[v] - hx[v], ey = py[v] - hy[v];
        rr += ex * ex + ey * ey;
        const double fx = rnew * (last[v * 2 * H1 + l] - hx[v]);
        const double fy = rnew * (last[v * 2 * H1 + H1 + l] - hy[v]);
        ss += fx * fx + fy * fy;
      }
    }
    rr = wsum(rr);
    ss = wsum(ss);
    dchk = rdl(dn, 1);
    if (l == 0) A.rho_pi[e] = rnew;
  } else {
  // dual update (plain casadi/main.py:161-162 / PI + anti-windup ADMM_CVX_...:156-188)
  double dist;
  {
    const double dx = px[0] - px[1], dy = py[0] - py[1];
    dist = sqrt(dx * dx + dy * dy);
  }
  const double mind = wmin(tl ? dist : INFINITY);
  const double kP = c.theta1 - c.theta2 / (1.0 + exp(-mind));
  const double Wsat = c.windup_sat;
  for (int v = 0; v < 2; ++v) {
    double* lv_ = lam + v * 2 * H1;
    double* Sv = Sa + v * 2 * H1;
    double* Dv = Da + v * 2 * H1;
    double* hv = hat + v * 2 * H1;
    bool changed = false;
    double lraw[2], lsat[2];
    for (int xy = 0; xy < 2; ++xy) {
      const double p = xy == 0 ? px[v] : py[v];
      const double h = xy == 0 ? hx[v] : hy[v];
      double lvv = tl ? lv_[xy * H1 + l] : 0.0;
      const double err = p - h;
      if (c.dual_mode == PIADMM_DUAL_PLAIN) {
        lvv = lvv + c.rho * err;
      } else {
        const double sv = tl ? (Sv[xy * H1 + l] + c.kI * err) + Dv[xy * H1 + l] : 0.0;
        if (tl) Sv[xy * H1 + l] = sv;
        lvv = sv + kP * err;
      }
      lraw[xy] = lvv;
      lsat[xy] = c.windup ? fmin(Wsat, fmax(lvv, -Wsat)) : lvv;
      changed |= tl && (lsat[xy] != lraw[xy]);
      if (tl) hv[xy * H1 + l] = h;
    }
    const bool anyc = wany(changed);
    for (int xy = 0; xy < 2; ++xy) {
      if (tl) {
        lv_[xy * H1 + l] = lsat[xy];
        if (c.windup) Dv[xy * H1 + l] = anyc ? lsat[xy] - lraw[xy] : 0.0;
      }
    }
  }
  // residual contributions of this pair (casadi/main.py:167-173): the v1 side only
  if (tl) {
    const double ex = px[0] - hx[0], ey = py[0] - hy[0];
    rr = ex * ex + ey * ey;
    const double fx = c.rho * (last[0 * H1 + l] - hx[0]);
    const double fy = c.rho * (last[1 * H1 + l] - hy[0]);
    ss = fx * fx + fy * fy;
  }
  rr = wsum(rr);
  ss = wsum(ss);
  dchk = rdl(dist, 1);
  }
  const double rfac = gpi ? 1.0 : 2.0;   // casadi/main.py:170-173 doubles the v1 side (quirk B5)
  // warm state back to HBM (unscaled: the next z-step restarts in identity scaling, setup_pair)
  if (qe.wraw) warm_to_scaled(qe, xs, zs, ys);
  double* qw = A.qs_e + (size_t)e * 12 * WAVE;
  signed char* lw = A.ql_e + (size_t)e * 5 * WAVE;
  qw[l] = qe.D[0] * xs[0];
  qw[WAVE + l] = qe.D[1] * xs[1];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    qw[(2 + q) * WAVE + l] = (qe.E[q] != 0.0) ? zs[q] / qe.E[q] : 0.0;
    qw[(7 + q) * WAVE + l] = qe.E[q] * ys[q];
    lw[q * WAVE + l] = lab[q];
  }
  if (TIES && c.term_dist_check && l == 0) scalar_tie(A, t, it, PIADMM_TIE_DIST, e, 0, dchk, deff);
  if (l == 0) {
    A.eres[2 * e] = rfac * sqrt(rr);
    A.eres[2 * e + 1] = rfac * sqrt(ss);
    A.dischk[e] = dchk;
    A.eflags[e] = 1;
    A.status[A.N + e] |= st;
    A.rho_e[e] = qe.rho;
  }
}

// -------------------------------------------------------------------- step init / final
// Seeds (casadi/main.py:48-49), the per-step reset of hat, lam and the PI accumulators (:52-63;
// shifted one slot with warm_duals, optimizer.py:337-344), the warm labels of the previous step.
template <bool TIES>
__device__ __forceinline__ void g_step_init(const DevArgs& A, int ci, int w, int t) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, H1 = H + 1, l = lid();
  for (int i = A.comp_aptr[ci] + w; i < A.comp_aptr[ci + 1]; i += GW) {
    const int a = A.comp_alist[i];
    const double x = A.xt[3 * a], y = A.xt[3 * a + 1], th = A.xt[3 * a + 2], s = A.spd[a];
    if (l == 0) {
      const double sx = x + c.dt * s * cos(th), sy = y + c.dt * s * sin(th);
      A.seed_g[2 * a] = around(sx, c.round_decimals);
      A.seed_g[2 * a + 1] = around(sy, c.round_decimals);
      double m;
      if (TIES && c.round_decimals >= 0 && round_near(sx, c.round_decimals, A.tie_tol, &m))
        tie_record(A, t, -1, PIADMM_TIE_ROUND_SEED, a, 0, m);
      if (TIES && c.round_decimals >= 0 && round_near(sy, c.round_decimals, A.tie_tol, &m))
        tie_record(A, t, -1, PIADMM_TIE_ROUND_SEED, a, 1, m);
    }
    // the previous step's final labels shifted by one time slot: a guess for the first polish
    const bool wo = A.warm_ok[a] != 0;
    const signed char* lb = A.lab_x + (size_t)a * 2 * HCAP;
    const int src = min(l + 1, H - 1);
    double* qw = A.qs_x + (size_t)a * 5 * WAVE;
    signed char* lw = A.ql_x + (size_t)a * 2 * WAVE;
    for (int q = 0; q < 5; ++q) qw[q * WAVE + l] = 0.0;
    lw[l] = (wo && l < H) ? lb[src] : 0;
    lw[WAVE + l] = (wo && l < H) ? lb[HCAP + src] : 0;
    A.csig_x[(size_t)a * WAVE + l] = -1;
    if (l == 0) {
      A.xflags[a] = wo ? 1 : 0;
      A.status[a] = 0;
    }
  }
  for (int j = A.comp_eptr[ci] + w; j < A.comp_eptr[ci + 1]; j += GW) {
    const int e = A.comp_elist[j];
    const int v1 = A.edges[2 * e], v2 = A.edges[2 * e + 1];
    double* const eh[5] = {A.hat, A.lam, A.Sacc, A.Dacc, A.last};
    for (int k = 0; k < 5; ++k) {
      double* p = eh[k] + (size_t)e * 4 * H1;
      double v[4];
      // (the adaptive-gain script starts hat, lam and last_hat at 1e-4: dual_init, adp :59-61)
      const double v0 = (k == 0 || k == 1 || k == 4) ? c.dual_init : 0.0;
      for (int r = 0; r < 4; ++r) v[r] = (c.warm_duals && l <= H) ? p[r * H1 + min(l + 1, H)] : v0;
      gsync();
      if (l <= H)
        for (int r = 0; r < 4; ++r) p[r * H1 + l] = v[r];
    }
    double* qw = A.qs_e + (size_t)e * 12 * WAVE;
    for (int q = 0; q < 12; ++q) qw[q * WAVE + l] = 0.0;
    signed char* lw = A.ql_e + (size_t)e * 5 * WAVE;
    for (int q = 0; q < 5; ++q) lw[q * WAVE + l] = 0;
    if (l == 0) {
      double d = c.dis_thres;
      if (c.tighten)
        d = c.dis_thres + delay_norm(c, A.xt[3 * v1 + 2], A.spd[v1]) + delay_norm(c, A.xt[3 * v2 + 2], A.spd[v2]);
      A.deff[e] = d;
      A.dischk[e] = NAN;
      A.edge_active[e] = 0;
      A.eflags[e] = 0;
      A.status[A.N + e] = 0;
      A.eres[2 * e] = 0.0;
      A.eres[2 * e + 1] = 0.0;
    }
  }
}

// Propagation (casadi/main.py:185-192) and the next step's warm labels.
__device__ __forceinline__ void g_step_final(const DevArgs& A, int ci, int w) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, l = lid();
  for (int i = A.comp_aptr[ci] + w; i < A.comp_aptr[ci + 1]; i += GW) {
    const int a = A.comp_alist[i];
    const double u = (l < H) ? A.u[(size_t)a * H + l] : 0.0;
    double px, py, pth;
    rollout(A.xt + 3 * a, A.spd[a], u, c, H, true, px, py, pth);
    gsync();                      // every lane has read xt before lane 1 overwrites it
    if (l == 1) {
      A.xt[3 * a + 0] = px;
      A.xt[3 * a + 1] = py;
      A.xt[3 * a + 2] = pth;
    }
    const signed char* lw = A.ql_x + (size_t)a * 2 * WAVE;
    signed char* lb = A.lab_x + (size_t)a * 2 * HCAP;
    lb[l] = lw[l];
    lb[HCAP + l] = lw[WAVE + l];
    if (l == 0) A.warm_ok[a] = 1;
  }
}

// -------------------------------------------------------------------- one MPC step
template <bool BIG, bool TIES>
__device__ __forceinline__ void graph_step_body(const DevArgs& A, int t, int it0, int it1, int flags, int slot,
                                                int& nbar) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int s_int[GW * 272];
  __shared__ double s_sc[8];
  __shared__ int s_cnt[GW][8];
  __shared__ unsigned char s_zact[GZMAX];   // this iteration's collision flags (components of <= GZMAX pairs)
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, H1 = H + 1, M = c.max_outer;
  const int ci = blockIdx.x;
  const int w = threadIdx.x >> 6, l = lid();
  const int e0 = A.comp_eptr[ci], e1 = A.comp_eptr[ci + 1];
  const int a0 = A.comp_aptr[ci], a1 = A.comp_aptr[ci + 1];
  // ---- LDS carve (graph_lds_bytes in piadmm_internal.h)
  const size_t fac_n = graph_fac(H);       // even counts throughout: every region on 16 bytes
  const size_t ylds_n = graph_ylds(H);
  double* wbase = lds + (size_t)w * (fac_n + 512 + 256 + ylds_n);
  GWave W;
  W.fac = wbase;
  W.vb = wbase + fac_n;
  W.xdiag = W.vb + 512;
  W.zdiag = W.xdiag + 128;
  W.ylds = ylds_n ? W.zdiag + 128 : nullptr;
  W.xids = s_int + w * 272;
  W.zids = W.xids + 128;
  W.xfs = W.xids + 256;
  W.zfs = W.xids + 257;

  const bool first = (flags & F_FIRST) != 0;
  const bool last_launch = (flags & F_LAST) != 0;
  const bool global = (flags & F_GLOBAL) != 0;
  const bool coop = (flags & F_COOP) != 0;
  const bool xonly = (flags & F_XONLY) != 0;
  const bool zonly = (flags & F_ZONLY) != 0;
  // both: iteration it0's Z phase, then iteration it0+1's X phase -- one launch between two
  // exchanges (a sharded job's fixed iterations, piadmm_capi.cpp run_steps_phases)
  const bool zx = xonly && zonly;
  bool nanlast = (flags & F_NANLAST) != 0;
  // a component whose step already ended in an earlier launch of this step (per-component stop,
  // host-stepped by piadmm_outer_iter) runs no further iteration
  const bool skip = !first && A.cst[(size_t)ci * 4 + 3] != 0;
  const int it_end = skip ? it0 : it1;
  bool stopped = skip;
  double* resid = A.resid + ((size_t)slot * A.C + ci) * M * 2;

  unsigned long long t_body = STAMP_T();
  if (first) {
    g_step_init<TIES>(A, ci, w, t);
    for (int i = threadIdx.x; i < 2 * M; i += blockDim.x) resid[i] = NAN;   // "not evaluated"
    if (coop && ci == 0)
      for (int i = threadIdx.x; i < 2 * M; i += blockDim.x) A.ghist[(size_t)slot * 2 * M + i] = NAN;
    if (flags & F_INITONLY) {
      __syncthreads();
      if (threadIdx.x == 0) {
        A.cst[(size_t)ci * 4 + 0] = 0;
        A.cst[(size_t)ci * 4 + 1] = 0;
        A.cst[(size_t)ci * 4 + 3] = 0;
        A.iters[ci] = 0;
      }
      return;
    }
  }
  int flag = first ? 0 : A.cst[(size_t)ci * 4 + 0];
  int aliased = first ? 0 : A.cst[(size_t)ci * 4 + 1];
  // host-decided global termination: the previous launch's iteration continued (else there
  // would be no iteration launch now), so its last_iter_hat_pos copy (casadi/main.py:180) is due
  if (!first && it0 < it1 && !zonly && global && !coop && !c.alias_dual_residual && !c.fixed_iters) {
    for (int j = e0 + w; j < e1; j += GW) {
      const int e = A.comp_elist[j];
      if (A.edge_active[e])
        for (int i = l; i < 4 * H1; i += WAVE) A.last[(size_t)e * 4 * H1 + i] = A.hat[(size_t)e * 4 * H1 + i];
    }
  }
  __syncthreads();
  GCnt n;
  int iters = skip ? A.iters[ci] : it0, gflag = 0;
  for (int it = it0; it < it_end; ++it) {
    // -------- X: x-steps of the component's agents (casadi/main.py:81-106)
    if (!(zonly && it == it0)) {
      unsigned long long t_xp = STAMP_T();
      for (int i = a0 + w; i < a1; i += GW) {
        const int a = A.comp_alist[i];
        if (!A.owned || A.owned[a]) g_xstep<BIG, TIES>(A, a, t, it, W, n);
      }
      STAMP_ADD(ST_XSTEP, t_xp);
      unsigned long long t_sa = STAMP_T();
      __syncthreads();
      STAMP_ADD(ST_SYNC_A, t_sa);
    }
    if (xonly && !(zx && it == it0)) break;
    iters = it + 1;
    // -------- ghosts (sharded job): the positions and controls their owner rank computed in this
    // iteration's X phase, from the all-reduced exchange buffer (piadmm_capi.cpp run_steps)
    if (A.xrecv) {
      for (int i = a0 + w; i < a1; i += GW) {
        const int a = A.comp_alist[i];
        if (A.owned[a]) continue;
        const double* xb = A.xrecv + (size_t)A.xslot[a] * (3 * H1);
        double* po = A.pos_old + (size_t)a * 2 * H1;
        for (int k = l; k < 2 * H1; k += WAVE) po[k] = xb[k];
        if (l < H) A.u[(size_t)a * H + l] = xb[2 * H1 + l];
      }
      __syncthreads();
    }
    // -------- Z: collision test + pair QPs + dual updates (casadi/main.py:110-162)
    unsigned long long t_zp = STAMP_T();
    // the collision tests of every pair (waves strided), then the colliding pairs dealt round-robin
    // over the waves in pair order: two colliding pairs never queue on one wave while the other
    // waits at the barrier (pairs are independent within the phase; the residual sums below run in
    // pair order whoever solved them).  Components of more than GZMAX pairs: strided, test + solve.
    const bool deal = e1 - e0 <= GZMAX;
    if (deal) {
      for (int j = e0 + w; j < e1; j += GW) {
        const bool act = g_ztest<TIES>(A, A.comp_elist[j], t, it);
        if (l == 0) s_zact[j - e0] = act ? 1 : 0;
      }
      __syncthreads();
    }
    {
      int k = 0;                                     // colliding pairs before j (pair order)
      for (int j = deal ? e0 : e0 + w; j < e1; j += deal ? 1 : GW) {
        const int e = A.comp_elist[j];
        bool mine;
        if (deal) {
          const bool act = s_zact[j - e0] != 0;
          mine = act && (k % GW == w);
          k += act ? 1 : 0;
        } else {
          mine = g_ztest<TIES>(A, e, t, it);
        }
        if (mine) g_zstep<BIG, TIES>(A, e, t, it, W, n);
      }
    }
    STAMP_ADD(ST_ZSTEP, t_zp);
    unsigned long long t_sb = STAMP_T();
    __syncthreads();
    STAMP_ADD(ST_SYNC_B, t_sb);
    unsigned long long t_tm = STAMP_T();
    // -------- T: the component's residuals in pair order and the stop rules (:164-181)
    double prk = 0.0, psk = 0.0, pact = 0.0, pseen = 0.0, pbad = 0.0;
    if (w == 0) {
      // lane k loads pair e0 + k's terms (one memory latency for up to 64 pairs, not one per pair);
      // the sums then run in pair order through readlanes -- the order of casadi/main.py:165-173
      // and of the oracle, so the residuals are the sequential sums
      for (int j0 = e0; j0 < e1; j0 += WAVE) {
        const int j = j0 + l;
        const bool in = j < e1;
        const int e = in ? A.comp_elist[j] : 0;
        const bool cnt = in && (!A.counted || A.counted[e]);   // a cross-rank pair counts on one rank only
        const double d = cnt ? A.dischk[e] : 0.0;
        const bool seen = cnt && (d == d);
        const bool bad = seen && !(d > A.deff[e]);
        const bool act = cnt && A.edge_active[e] != 0;
        const double r0 = act ? A.eres[2 * e] : 0.0, r1 = act ? A.eres[2 * e + 1] : 0.0;
        // split component: the pair's terms of this iteration's sum, added in the reference's
        // order over the whole original component by k_graph_partials
        if (A.eterm && in) {
          const int sp = A.sum_pos[e];
          A.eterm[sp] = r0;
          A.eterm[A.E + sp] = aliased ? 0.0 : r1;
        }
        const unsigned long long bseen = __ballot(seen), bbad = __ballot(bad), bact = __ballot(act);
        const int npr = min(WAVE, e1 - j0);
        for (int k = 0; k < npr; ++k) {
          if ((bseen >> k) & 1ull) {
            pseen += 1.0;
            pbad += ((bbad >> k) & 1ull) ? 1.0 : 0.0;
          }
          if (!((bact >> k) & 1ull)) continue;
          pact += 1.0;
          if (!aliased) psk += rdl(r1, k);
          prk += rdl(r0, k);
        }
      }
    }
    if (threadIdx.x == 0) {
      const bool anyact = pact > 0.0;
      double* cp = A.cpart + (size_t)ci * 5;
      cp[0] = prk;
      cp[1] = psk;
      cp[2] = pact;
      cp[3] = pseen;
      cp[4] = pbad;
      s_sc[0] = prk;
      s_sc[1] = psk;
      s_sc[2] = anyact ? 1.0 : 0.0;
      s_sc[3] = pseen;
      s_sc[4] = pbad;
    }
    __syncthreads();
    const double rk = s_sc[0], sk = s_sc[1];
    const bool anyact = s_sc[2] != 0.0;
    const bool dist_ok = s_sc[3] > 0.0 && s_sc[4] == 0.0;
    __syncthreads();
    STAMP_ADD(ST_TERM, t_tm);
    if (!anyact && flag == 0 && !c.fixed_iters && !global) {    // no pair collided: stop (:115-116)
      stopped = true;
      break;
    }
    flag = 1;
    if (threadIdx.x == 0) {
      resid[2 * it + 0] = rk;
      resid[2 * it + 1] = sk;
    }
    bool stop = !c.fixed_iters && !global && rk <= c.eps_pri && sk <= c.eps_dual && (!c.term_dist_check || dist_ok);
    if (TIES && !c.fixed_iters && !global && threadIdx.x == 0) {
      scalar_tie(A, t, it, PIADMM_TIE_STOP, ci, 0, rk, c.eps_pri);
      scalar_tie(A, t, it, PIADMM_TIE_STOP, ci, 1, sk, c.eps_dual);
    }
    if (coop && !c.fixed_iters) {
      // global stop in-kernel: per-component partials, one grid barrier, the same fixed-order
      // sum in every workgroup (k_graph_partials sums in this order on the host-decided path)
      __shared__ double s_red[5][GW * WAVE];
      __shared__ double s_tot[5];
      double* part = A.gpart + (size_t)(nbar & 1) * A.C * 5;
      ++nbar;
      if (threadIdx.x == 0) {
        const double* cp = A.cpart + (size_t)ci * 5;
        for (int q = 0; q < 5; ++q)
          __hip_atomic_store(&part[ci * 5 + q], cp[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      grid_flag_barrier(A.gbar, A.C, ci, A.gbar_base + (unsigned long long)nbar);
      double v[5] = {0, 0, 0, 0, 0};
      for (int k = threadIdx.x; k < A.C; k += blockDim.x)
#pragma unroll
        for (int q = 0; q < 5; ++q)
          v[q] += __hip_atomic_load(&part[k * 5 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int q = 0; q < 5; ++q) s_red[q][threadIdx.x] = v[q];
      __syncthreads();
      if (threadIdx.x < 5) {
        double tot = 0.0;
        const int nk = min(A.C, GW * WAVE);            // (the threads beyond hold +0.0)
        for (int k = 0; k < nk; ++k) tot += s_red[threadIdx.x][k];
        s_tot[threadIdx.x] = tot;
      }
      __syncthreads();
      const double trk = s_tot[0], tsk = s_tot[1], tact = s_tot[2], tseen = s_tot[3], tbad = s_tot[4];
      __syncthreads();
      if (tact == 0.0 && gflag == 0) {       // no pair collides anywhere: stop (:115-116)
        nanlast = true;
        stopped = true;
        break;
      }
      gflag = 1;
      if (ci == 0 && threadIdx.x == 0) {
        A.ghist[((size_t)slot * M + it) * 2 + 0] = trk;
        A.ghist[((size_t)slot * M + it) * 2 + 1] = tsk;
      }
      if (TIES && ci == 0 && threadIdx.x == 0) {
        scalar_tie(A, t, it, PIADMM_TIE_STOP, -1, 0, trk, c.eps_pri);
        scalar_tie(A, t, it, PIADMM_TIE_STOP, -1, 1, tsk, c.eps_dual);
      }
      if (trk <= c.eps_pri && tsk <= c.eps_dual && (!c.term_dist_check || (tseen > 0.0 && tbad == 0.0))) stop = true;
    }
    if (stop) {
      stopped = true;
      break;
    }
    // last_iter_hat_pos = hat_pos_old (casadi/main.py:180; MATLAB copies): after the decision
    // (host-decided global termination: at the start of the next launch, once the host has
    // decided to continue)
    if (!c.alias_dual_residual && !(global && !coop && !c.fixed_iters)) {
      for (int j = e0 + w; j < e1; j += GW) {
        const int e = A.comp_elist[j];
        if (A.edge_active[e])
          for (int i = l; i < 4 * H1; i += WAVE) A.last[(size_t)e * 4 * H1 + i] = A.hat[(size_t)e * 4 * H1 + i];
      }
    }
    if (c.alias_dual_residual) aliased = 1;
  }
  __syncthreads();
  // ---- work counters and the launch's component state
  if (l == 0) {
    s_cnt[w][0] = n.xqp; s_cnt[w][1] = n.zqp; s_cnt[w][2] = n.admm_x; s_cnt[w][3] = n.admm_z;
    s_cnt[w][4] = n.pdas_x; s_cnt[w][5] = n.pdas_z; s_cnt[w][6] = n.inexact; s_cnt[w][7] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long* cn = A.counters + (size_t)ci * 8;
    if ((!xonly || zx) && !skip) cn[0] += (unsigned long long)(iters - it0);
    for (int k = 0; k < 7; ++k) {
      unsigned long long sum = 0;
      for (int ww = 0; ww < GW; ++ww) sum += (unsigned long long)s_cnt[ww][k];
      cn[k + 1] += sum;
    }
    if (!xonly || zx) A.iters[ci] = iters;
    A.cst[(size_t)ci * 4 + 0] = flag;
    A.cst[(size_t)ci * 4 + 1] = aliased;
    if (!xonly || zx) A.cst[(size_t)ci * 4 + 3] = stopped ? 1 : 0;
    if (coop && ci == 0) A.giters[slot] = iters;
    if (nanlast && iters > 0 && !skip) {
      resid[2 * (iters - 1) + 0] = NAN;
      resid[2 * (iters - 1) + 1] = NAN;
    }
  }
  if (last_launch) g_step_final(A, ci, w);
  STAMP_ADD(ST_KERNEL, t_body);
}

template <bool BIG, bool TIES>
__global__ void __launch_bounds__(GW * WAVE) k_graph_step(DevArgs A, int t0, int nsteps, int it0, int it1, int flags) {
  if (flags & F_DEVSTOP) {      // device-decided global stop (uniform: every thread reads it)
    if (!(flags & F_LAST)) {
      if (A.gctl[0]) return;
    } else {
      it0 = it1 = A.gctl[2];
      if (A.gctl[1]) flags |= F_NANLAST;
    }
  }
#ifdef PIADMM_STAMPS
  for (int i = threadIdx.x; i < 64 * STAMP_WAVES; i += blockDim.x) s_stamps[i] = 0ull;
  __syncthreads();
#endif
  int nbar = 0;
  for (int k = 0; k < nsteps; ++k) {
    graph_step_body<BIG, TIES>(A, t0 + k, it0, it1, flags, k, nbar);
    __syncthreads();
  }
#ifdef PIADMM_STAMPS
  if (g_stamps)
    for (int i = threadIdx.x; i < 64 * STAMP_WAVES; i += blockDim.x)
      atomicAdd(&g_stamps[(size_t)blockIdx.x * 64 * STAMP_WAVES + i], s_stamps[i]);
#endif
}

}  // namespace pd

namespace pd {

// Termination partials of the last iteration summed over components (host-decided global
// termination in graph mode): the in-kernel (cooperative) order -- thread k accumulates
// components k, k + GW*WAVE, ... in order, then the per-thread sums in thread order.
// Components split over workgroups (A.sum_C > 0): rk and sk are instead the reference's sums over
// the ORIGINAL components -- each component's pairs in increasing pair order, then the components
// in order (casadi/main.py:165-173; the oracle's comp_r sum) -- from the pairs' terms the blocks'
// T phases wrote (A.eterm), wave 0 summing rk and wave 1 sk: bit-identical to the same job on one
// workgroup per component.  (The counts -- active pairs, distance checks -- are integers: any order.)
__global__ void __launch_bounds__(GW * WAVE) k_graph_partials(DevArgs A, double* out, int devstop, int nout) {
  if (devstop && A.gctl[0]) return;
  constexpr int NT = GW * WAVE;
  __shared__ double red[5][NT];
  double v[5] = {0, 0, 0, 0, 0};
  for (int ci = threadIdx.x; ci < A.C; ci += NT)
    for (int q = 0; q < 5; ++q) v[q] += A.cpart[(size_t)ci * 5 + q];
  for (int q = 0; q < 5; ++q) red[q][threadIdx.x] = v[q];
  __syncthreads();
  const bool split = A.sum_C > 0;
  if ((int)threadIdx.x < nout && !(split && threadIdx.x < 2)) {
    double tot = 0.0;
    for (int k = 0; k < NT; ++k) tot += red[threadIdx.x][k];
    out[threadIdx.x] = tot;
  }
  if (split) {
    // Every term is >= 0 and x + 0.0 == x, so the zero terms (inactive pairs: nearly all) and the
    // components without a nonzero term are skipped exactly: the terms are loaded 16 per lane at a
    // time (coalesced: eterm is in sum order), and only the nonzero ones are added, in order.
    const int q = threadIdx.x >> 6;            // wave 0: rk, wave 1: sk
    const int l = lid();
    const double* et = A.eterm + (size_t)q * A.E;
    double tot = 0.0, cs = 0.0;
    int k = 0, kend = A.sum_cptr[1];
    constexpr int PB = 16;
    for (int base = 0; base < A.E; base += PB * WAVE) {
      double r[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int j = base + u * WAVE + l;
        r[u] = j < A.E ? et[j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        unsigned long long nz = __ballot(r[u] != 0.0);
        while (nz) {
          const int i = __ffsll(nz) - 1;
          nz &= nz - 1;
          const int j = base + u * WAVE + i;
          while (j >= kend) {                   // a component boundary: its sum joins the total
            tot += cs;
            cs = 0.0;
            ++k;
            kend = A.sum_cptr[k + 1];
          }
          cs += rdl(r[u], i);
        }
      }
    }
    tot += cs;
    if (l == 0) out[q] = tot;
  }
}

// The kernel instantiation: big-mode layout (BIG) and the near-tie log compiled in or out (TIES).
static const void* graph_fn(bool big, bool ties) {
  if (big) return ties ? (const void*)k_graph_step<true, true> : (const void*)k_graph_step<true, false>;
  return ties ? (const void*)k_graph_step<false, true> : (const void*)k_graph_step<false, false>;
}

int launch_graph_step(const DevArgs& a, int t, int nsteps, int it0, int it1, int flags, hipStream_t s) {
  const size_t sh = graph_lds_bytes(a.cfg.H);
#ifdef PIADMM_STAMPS
  static unsigned long long* last = nullptr;
  if (a.stamps != last) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &a.stamps, sizeof(void*)) != hipSuccess) return -1;
    last = a.stamps;
  }
#endif
  const bool big = a.cfg.H > HMAX;
  const void* fn = graph_fn(big, a.tie_on != 0);
  if (set_dyn_lds(fn, sh) != 0) return -1;
  if (flags & F_COOP) {
    DevArgs aa = a;
    aa.gbar_base = launch_coop_epoch(nsteps, a.cfg.max_outer);
    void* args[] = {&aa, &t, &nsteps, &it0, &it1, &flags};
    (void)hipGetLastError();
    return launch_rc(hipLaunchCooperativeKernel(fn, dim3(a.C), dim3(GW * WAVE), args, (unsigned)sh, s));
  }
  (void)hipGetLastError();   // a stale error of an earlier runtime call is not this launch's
  DevArgs aa = a;
  void* args[] = {&aa, &t, &nsteps, &it0, &it1, &flags};
  return launch_rc(hipLaunchKernel(fn, dim3(a.C), dim3(GW * WAVE), args, sh, s));
}

bool graph_coop_fits(const DevArgs& a, int device) {
  int coopok = 0, ncu = 0, per = 0;
  if (hipDeviceGetAttribute(&coopok, hipDeviceAttributeCooperativeLaunch, device) != hipSuccess || !coopok)
    return false;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return false;
  const size_t sh = graph_lds_bytes(a.cfg.H);
  const void* fn = graph_fn(a.cfg.H > HMAX, a.tie_on != 0);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, GW * WAVE, sh) != hipSuccess) return false;
  return (long long)per * ncu >= (long long)a.C;
}

int launch_graph_partials(const DevArgs& a, double* out, hipStream_t s, int devstop, int nout) {
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_graph_partials, dim3(1), dim3(GW * WAVE), 0, s, a, out, devstop, nout);
  return launch_rc(hipGetLastError());
}

}  // namespace pd
