// piadmm_device.hip -- MI355X (gfx950) kernels of the batched PI-ADMM consensus solver.
//
// One workgroup = one connected component of the candidate-pair graph (two
// agents and their pair in the tiled scenario); one persistent launch = up to 32
// MPC steps of the reference loop (casadi/main.py:43-201) per component: seeds,
// per-step setup of every QP, the outer ADMM loop with device-side termination,
// and propagation.  Components are independent; the only inter-workgroup step is
// the grid barrier of the reference's global stopping test (cooperative launch).
//
// Wave layout: wave w < 2 solves agent w's x-step; wave 2 owns the pair.
// Lane k <-> time/variable index k (H <= 63).  All arithmetic is fp64.
//
// Every QP answer is the exact minimiser, certified by a complete KKT test:
//  * the pair QP and the x-step's working-set changes by a Goldfarb-Idnani dual
//    active set (Schur complement N P^-1 N' as an appended / rank-one-downdated
//    Cholesky factor in LDS), warm-started from the previous active set;
//  * the x-step's steady state by one fused pass over parametric tables of the
//    current working set (x = -G T' w' + g, lam = -X T' w' - beta);
//  * as the fallback, an OSQP-style ADMM in a Ruiz-scaled space feeding a
//    primal-dual active-set (PDAS) polish on the reduced KKT system.
// tools/qp_sim.py and tools/gi_sim.py are the NumPy prototypes of this math.
// Shared device code: pd_common.h (wave primitives, rollouts), pd_qp.h (QP solver), pd_setup.h.
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <tuple>
#include <vector>
#include <algorithm>

#include "pd_setup.h"

static_assert(pd::WPIPE_WORDS == (size_t)pd::WP_DBL + 36, "the warm-row ring: lds_bytes and pd_qp.h WarmPipe agree");

namespace pd {

// The dual active set's S^-1 passes in big mode walk rows (pd_qp.h gi_solve RM_S).  The phase-stamp
// diagnostic build keeps big mode on the lane = column passes: with the stamps compiled in, this
// ROCm's compiler rejects that instantiation ("Operand has incorrect register class" on an LDS
// aperture compare).  The stamps are read for the LDS-mode kernel.
#ifdef PIADMM_STAMPS
constexpr int RM_BIG = 0;
#else
constexpr int RM_BIG = RM_S;
#endif


// ============================================================ the MPC-step kernel
struct CompLds {
  double *pos, *xt, *seed, *u, *hat, *lam, *S, *D, *last, *sc;
};

// What every wave of a component's workgroup knows about the launch (uniform values).
struct StepCtx {
  int H, H1, ci, w, l, a0, na, e, t, it0, it_end, slot;
  bool first, last_launch, global, coop, skip, big, f32;
  double deff, thr;
  CompLds S;
  double* resid;
  double* vec_all;
  WaveMem wm;
  bool spec;        // the speculative loop shape (agent_part)
  bool roll;        // speculative loop with the roller wave (roll_part): agent 1's rollout on wave RW
  bool helper;      // wave RW also builds the pair's warm rows (pd_qp.h WarmPipe): LDS mode, H <= WPIPE_HMAX
  WarmPipe wp;      // its LDS ring (after S.sc)
  int* vd;          // the pair wave's verdict on an iteration (speculative loop): act, stop, flag, aliased
  double* vdd;      // and dis_chk
  int* rflag;       // the roller's progress: it + 1 once agent 1's positions of iteration it are in LDS
};

// The outer loop's control state.  Every wave keeps its own copy and updates it from the same
// LDS values behind the same barriers, so all copies agree (the waves take identical branches).
struct LoopCtl {
  int flag, aliased, iters, gflag;
  bool stopped, nanlast, act;
  double dis_chk;
};

// collision graph (casadi/main.py:110-118), computed by every wave from this iteration's positions
// (the pair wave logs a near tie, piadmm_get_near_ties: every wave runs the test in the plain loop)
template <bool TIES>
__device__ __forceinline__ bool collide(const DevArgs& A, const StepCtx& X, const double* pos, int it) {
  if (X.e < 0 || X.na != 2) return false;
  bool hit = false;
  double d2 = 0.0;
  if (X.l <= X.H) {
    const double dx = pos[0 * X.H1 + X.l] - pos[2 * X.H1 + X.l];
    const double dy = pos[1 * X.H1 + X.l] - pos[3 * X.H1 + X.l];
    d2 = dx * dx + dy * dy;
    hit = d2 < X.thr;
  }
  if constexpr (TIES)
    if (X.w == PW) collide_tie(A, X.t, it, X.e, d2, X.l <= X.H, X.thr);
  return wany(hit);
}

// The end of an outer iteration in every wave (casadi/main.py:164-181; MATLAB :191-210), after
// barrier B when the pair's z-step ran: the residuals in S.sc, the component's stop test, and --
// single rank, natural global termination -- the in-kernel stop test over all components behind
// a grid barrier.  Returns true when the component's step ends here.
template <bool TIES>
__device__ __forceinline__ bool iter_tail(const DevArgs& A, const StepCtx& X, LoopCtl& L, int it, int& nbar) {
  const piadmm_config_t& c = A.cfg;
  const CompLds& S = X.S;
  const double rk = L.act ? S.sc[0] : 0.0;
  const double sk = L.act ? S.sc[1] : 0.0;
  if (L.act) L.dis_chk = S.sc[2];
  if (TIES && !c.fixed_iters && !X.global && X.w == PW && X.l == 0) {   // near ties of the stop test (one wave)
    scalar_tie(A, X.t, it, PIADMM_TIE_STOP, X.ci, 0, rk, c.eps_pri);
    scalar_tie(A, X.t, it, PIADMM_TIE_STOP, X.ci, 1, sk, c.eps_dual);
  }
  if (!c.fixed_iters && !X.global && rk <= c.eps_pri && sk <= c.eps_dual &&
      (!c.term_dist_check || L.dis_chk > X.deff)) {
    L.stopped = true;
    return true;
  }
  if (X.coop && !c.fixed_iters) {
    // global termination over all components, in-kernel (single rank): per-component partials,
    // one grid barrier, every workgroup sums them in the same order and applies the host's stop
    // rules (piadmm_capi.cpp run_steps) identically.  Double-buffered by the parity of the
    // launch's barrier count (iterations and steps), so one barrier per iteration suffices;
    // agent-scope atomic accesses keep the partials out of the non-coherent per-CU cache.
    unsigned long long t_gb = STAMP_T();
    double* part = A.gpart + (size_t)(nbar & 1) * A.C * 5;
    ++nbar;
    const int ci = X.ci;
    if (threadIdx.x == 0) {
      const bool seen = (X.e >= 0) && (L.dis_chk == L.dis_chk);
      const double pv[5] = {rk, sk, (X.e >= 0 && L.act) ? 1.0 : 0.0, seen ? 1.0 : 0.0,
                            (seen && !(L.dis_chk > X.deff)) ? 1.0 : 0.0};
#pragma unroll
      for (int q = 0; q < 5; ++q)
        __hip_atomic_store(&part[ci * 5 + q], pv[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    grid_flag_barrier(A.gbar, A.C, ci, A.gbar_base + (unsigned long long)nbar);
    {
      // the first NT threads load (components tid, tid + NT, ...), then five threads sum the
      // per-thread partials in thread order: a fixed order, identical in every workgroup and equal
      // to k_term_partials' (the host-decided path).  The sum stops at min(C, NT) terms: the
      // threads beyond hold +0.0, which leaves the sum (never -0.0: it starts at +0.0) unchanged
      constexpr int NT = NW * WAVE;
      double v[5] = {0, 0, 0, 0, 0};
      if ((int)threadIdx.x < NT)
        for (int k = threadIdx.x; k < A.C; k += NT)
#pragma unroll
          for (int q = 0; q < 5; ++q)
            v[q] += __hip_atomic_load(&part[k * 5 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      double* red = X.vec_all;         // the waves' vector buffers are free between QP solves
      if ((int)threadIdx.x < NT)
#pragma unroll
        for (int q = 0; q < 5; ++q) red[q * NT + threadIdx.x] = v[q];
      __syncthreads();
      if (threadIdx.x < 5) {
        double tot = 0.0;
#ifndef PIADMM_STAMPS
        const int nk = min(A.C, NT);
#else
        const int nk = NT;   // (the stamps build: ROCm 7.2's backend rejects the variable trip count there,
                             // "Operand has incorrect register class"; the same sum)
#endif
        for (int k = 0; k < nk; ++k) tot += red[threadIdx.x * NT + k];
        S.sc[16 + threadIdx.x] = tot;
      }
    }
    __syncthreads();
    const double trk = S.sc[16], tsk = S.sc[17], tact = S.sc[18], tseen = S.sc[19], tbad = S.sc[20];
    __syncthreads();
    STAMP_ADD(ST_TERM, t_gb);
    if (tact == 0.0 && L.gflag == 0) {       // no pair collides anywhere: stop (:115-116)
      L.nanlast = true;
      L.stopped = true;
      return true;
    }
    L.gflag = 1;
    if (ci == 0 && threadIdx.x == 0) {
      A.ghist[((size_t)X.slot * c.max_outer + it) * 2 + 0] = trk;
      A.ghist[((size_t)X.slot * c.max_outer + it) * 2 + 1] = tsk;
    }
    const bool dist_ok = tseen > 0.0 && tbad == 0.0;
    if (TIES && ci == 0 && threadIdx.x == 0) {
      scalar_tie(A, X.t, it, PIADMM_TIE_STOP, -1, 0, trk, c.eps_pri);
      scalar_tie(A, X.t, it, PIADMM_TIE_STOP, -1, 1, tsk, c.eps_dual);
    }
    if (trk <= c.eps_pri && tsk <= c.eps_dual && (!c.term_dist_check || dist_ok)) {
      L.stopped = true;
      return true;
    }
  }
  if (c.alias_dual_residual) L.aliased = 1;
  return false;
}

// Work counters of one wave (summed over the workgroup's waves in the epilogue).
struct WaveCnt {
  int xqp = 0, zqp = 0, admm_x = 0, admm_z = 0, pdas_x = 0, pdas_z = 0, inexact = 0, gi = 0;
  bool warm = false;
};

// -------------------------------------------------------------------- agent waves (0, 1)
// Wave w < na solves agent a0 + w's x-step every outer iteration (casadi/main.py:81-106); its
// QP state (tables, labels, warm ADMM state) stays in this wave's registers and LDS regions for
// the whole step.  The pair's state never lives here: the pair wave owns it.
template <bool BIG, bool TIES, int SH>
__device__ __forceinline__ void agent_part(const DevArgs& A, const StepCtx& X, LoopCtl& L, int& nbar, WaveCnt& n) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const piadmm_config_t& c = A.cfg;
  const int H = X.H, H1 = X.H1, w = X.w, l = X.l, ci = X.ci, e = X.e, t = X.t;
  const bool big = BIG, f32 = X.f32, first = X.first;
  const CompLds& S = X.S;
  // ---- this wave's LDS regions (lds_bytes() in piadmm_internal.h)
  double *Kx = nullptr, *Gx = nullptr, *xfac, *xt_all = nullptr;
  float* Kxf = nullptr;
  if (!big) {
    double* p = lds;
    if (f32) { Kxf = (float*)p; p += kxf_words(H); }     // 2 x H*H fp32 agent K_s^-1 (even per wave)
    else { Kx = p; p += 2 * H * H; }                     // 2 x H*H   agent K_s^-1
    Gx = p; p += 2 * gt_stride(H);                       // 2 x agent polish G T' | g (transposed)
    p += f32 ? 2 * H * H : 4 * H * H;                    // pair K_s^-1 (the pair wave's)
    p += 64 * (LD + 1);                                  // pair scratch (the pair wave's)
    xfac = p + w * HMAX * (HMAX + 2);                    // NW x HMAX x (HMAX+2)
    xt_all = p + NW * HMAX * (HMAX + 2);                 // NW x HMAX x XLDT (X' T' | beta, transposed)
  } else {
    xfac = lds + 64 * (LD + 1) + w * xreg(H);            // NW x xrows(H) x (xrows+2), even counts
  }
  double* xdiag = X.vec_all + NWT * 512 + w * 128;       // NWT x 128 factor diagonals
  int* xids = X.wm.ib;
  int* xfs = X.wm.ib + 256;
  if (l == 0) xfs[0] = -1;

  QP<1> qx;
  double xs_x[1] = {0.0}, zs_x[2] = {0.0, 0.0}, ys_x[2] = {0.0, 0.0};
  signed char lab_x[2] = {0, 0};
  bool warm_x = false;
  int status_x = 0;
  int nnb = 0;
  Geo gx;
  double cx_own = 0.0, cy_own = 0.0;
  const bool own = w < X.na;
  if (own) {
    unsigned long long t0 = STAMP_T();
    const int a = X.a0 + w;
    gx = make_geo(S.xt + 3 * w, A.spd[a], c);
    affine_c(gx, c.dt, H, cx_own, cy_own);
    qp_common(c, H, A.rho_x[a], qx);
    qx.K = big ? A.Kx_cache + (size_t)a * H * H : (Kx ? Kx + w * H * H : nullptr);
    qx.Kf = (!big && f32) ? Kxf + w * kxf_stride(H) : nullptr;
    qx.kf32 = !big && f32;                        // big mode: the x-step K stays fp64 in HBM
    qx.Pinv = A.Pinv_x + (size_t)a * H * H;    // L2-resident; read only when W changes
    qx.G = big ? A.Gx_g + (size_t)a * (H * H + H) : Gx + w * gt_stride(H);
    qx.vb = X.wm.vb;
    qx.fac = xfac;
    qx.XT = big ? A.XT_g + (size_t)a * H1 * XLDG : xt_all + w * HMAX * XLDT;
    qx.xld = big ? XLDG : XLDT;
    qx.gmem = big;
    qx.fdiag = xdiag;
    qx.ib = xids;
    qx.fstate = xfs;
    qx.fld = big ? xrows(H) + 1 : HMAX + 1;
    qx.mmax = big ? xrows(H) : HMAX;
    // dual active set for the x-step's working-set changes: Y in this wave's K_s^-1 region
    // (LDS mode; K_s^-1 is reloaded from its HBM copy if ADMM runs later)
    qx.gws = nullptr;
    qx.tstep = t;
    qx.t32 = (big && A.T32_g) ? A.T32_g + (size_t)a * (H * H + H * XLDG) : nullptr;
    // (big mode: a per-agent HBM buffer, K_s^-1 stays intact)
    qx.Y = big ? A.Yx_g + (size_t)a * WAVE * H : (f32 ? (double*)(Kxf + w * kxf_stride(H)) : Kx + w * H * H);
    qx.ycap = !A.x_gi ? 0 : (big ? WAVE : (f32 ? (H * H / 2) / H : H));
    qx.y_in_k = !big;
    nnb = A.nbr_cnt[a];
    setup_agent(A, a, qx, gx, xfac);
    // receding-horizon warm start: the previous step's final labels shifted by one time
    // slot (lane k now holds time t+k = lane k+1 of step t-1); only a guess for the polish,
    // the certified minimiser does not depend on it
    if (!first) {
      const double* qs = A.qs_x + (size_t)a * 5 * WAVE;
      const signed char* ql = A.ql_x + (size_t)a * 2 * WAVE;
      xs_x[0] = qs[l];
      zs_x[0] = qs[WAVE + l];
      zs_x[1] = qs[2 * WAVE + l];
      ys_x[0] = qs[3 * WAVE + l];
      ys_x[1] = qs[4 * WAVE + l];
      lab_x[0] = ql[l];
      lab_x[1] = ql[WAVE + l];
      warm_x = (A.cst[(size_t)ci * 4 + 2] >> w) & 1;
      status_x = A.status[a];
    } else if (A.warm_ok[a]) {
      const signed char* lb = A.lab_x + (size_t)a * 2 * HCAP;
      const int src = min(l + 1, H - 1);
#pragma unroll
      for (int s = 0; s < 2; ++s) lab_x[s] = (l < H) ? lb[s * HCAP + src] : 0;
      warm_x = true;
    }
    STAMP_ADD(ST_SETUP_X, t0);
  }
  __syncthreads();

  const bool nonlin_pos = c.pos_model != 0;
  // the own agent's start state and speed in registers for the per-iteration rollout
  double rl_x0 = 0.0, rl_y0 = 0.0, rl_th0 = 0.0, rl_s = 0.0, rl_sl = 0.0;
  if (own) {
    rl_x0 = S.xt[3 * w + 0];
    rl_y0 = S.xt[3 * w + 1];
    rl_th0 = S.xt[3 * w + 2];
    rl_s = A.spd[X.a0 + w];
    rl_sl = rl_s / c.L;
  }
  // reference positions of the own agent at time lanes (fixed for the step)
  double rx_own = 0.0, ry_own = 0.0;
  if (own && l <= H) {
    const double* rp = A.ref + (size_t)(X.a0 + w) * 2 * A.T;
    rx_own = rp[t + l];
    ry_own = rp[A.T + t + l];
  }
  // the x-step's consensus term (cx - hat + lam) of the own direction in registers: hat and lam
  // change only in a z-step, after which it is reloaded (behind the second barrier)
  const bool cpl = own && nnb > 0 && e >= 0 && l <= H;
  double cpx = 0.0, cpy = 0.0;
  auto load_cp = [&]() {
    if (cpl) {
      const int d = w;   // agent local 0 owns hat_{v1 v2} (dir 0), agent 1 dir 1
      cpx = cx_own - S.hat[(d * 2 + 0) * H1 + l] + S.lam[(d * 2 + 0) * H1 + l];
      cpy = cy_own - S.hat[(d * 2 + 1) * H1 + l] + S.lam[(d * 2 + 1) * H1 + l];
    }
  };
  load_cp();
  // Two loop shapes (the same barriers and decisions in every wave):
  //  * speculative (no in-kernel grid barrier): the pair wave rolls the agents' controls out, runs
  //    the collision test, the z-step and the stop decision for iteration it, while the agent waves
  //    already solve iteration it+1's x-step.  That x-step's QP depends only on hat and lam, which
  //    change only in a z-step, so when iteration it had no colliding pair it IS iteration it+1's
  //    x-step and is kept; after a z-step (or a stop) it is discarded and, if the loop goes on,
  //    solved again with the new consensus term.  Barriers per iteration: A (this iteration's
  //    controls are in U) and B (the pair wave's verdict); the rollout and the test leave the
  //    agents' dependent chain.
  //  * in-kernel global termination (coop): every wave takes part in the grid barrier of the stop
  //    test, so the agents roll out their own controls and every wave runs the collision test
  //    (barrier A, then B only after a z-step).
  constexpr bool specm = SH == 1;
  if constexpr (!specm) {
  // rep_ok: the last x-step certified without ADMM, the tables hold its working set and no z-step
  // has changed its consensus term since -- the next x-step is that QP again (the lean repeat)
  bool rep_ok = false, done = false;
  int it = X.it0;
  while (it < X.it_end) {
    // ---- the steady state (r06, plain shape): the compact loop of iterations whose x-step is the
    // lean repeat (agent_part's speculative-shape counterpart below); the general body takes over
    // at the first iteration whose repeat does not certify, and after a z-step
    if (own && rep_ok && !qx.t32) {
      bool lean_fail = false;
      while (true) {
        L.iters = it + 1;
        double* const ps = S.pos + (it & 1) * 4 * H1;
        unsigned long long t_xs = STAMP_T();
        const bool tl = l <= H;
        double vx = 2.0 * c.Pnorm * (cx_own - rx_own), vy = 2.0 * c.Pnorm * (cy_own - ry_own);
        if (cpl) {
          vx = vx + c.rho * cpx;
          vy = vy + c.rho * cpy;
        }
        const double wt = tl ? gx.ax * vx + gx.ay * vy : 0.0;
        const double wsh = shdn(wt, 1);
        qx.wq = (l < H) ? wsh : 0.0;
        qx.qvalid = false;
        double ustar[1];
        if (__builtin_expect(!xhit_repeat<BIG ? 8 : XGEMV_U, !BIG>(qx, lab_x, xs_x, ys_x, ustar, n.pdas_x), 0)) {
          lean_fail = true;                              // iteration it from the top, general body
          break;
        }
        ++n.xqp;
        warm_x = true;
        const double u = around(ustar[0], c.round_decimals);
        if (TIES && c.round_decimals >= 0) round_ties(A, t, it, PIADMM_TIE_ROUND_U, X.a0 + w, 0, ustar[0], l < H);
        double px, py, pth;
        rollout_r(rl_x0, rl_y0, rl_th0, rl_s, rl_sl, (l < H) ? u : 0.0, c, H, nonlin_pos, px, py, pth);
        if (l <= H) {
          ps[(w * 2 + 0) * H1 + l] = px;
          ps[(w * 2 + 1) * H1 + l] = py;
        }
        if (l < H) S.u[(it & 1) * 2 * H + w * H + l] = u;
        STAMP_ADD(ST_XSTEP, t_xs);
        __syncthreads();                                 // A: every agent's positions
        L.act = collide<TIES>(A, X, ps, it);
        if (!L.act && L.flag == 0 && !c.fixed_iters && !X.global) {   // no edge ever: stop (:115-116)
          L.stopped = true;
          done = true;
          break;
        }
        L.flag = 1;
        if (__builtin_expect(L.act, 0)) {
          __syncthreads();                               // B: hat, lam, S, D, last, S.sc
          load_cp();
          rep_ok = false;
        }
        if (iter_tail<TIES>(A, X, L, it, nbar)) {
          done = true;
          break;
        }
        if (++it >= X.it_end || !rep_ok) break;
      }
      if (done) break;
      if (!lean_fail) continue;
      rep_ok = false;
    }
    L.iters = it + 1;
    double* const pos = S.pos + (it & 1) * 4 * H1;
    if (own) {
      unsigned long long t_xs = STAMP_T();
      const bool tl = l <= H;
      double vx = 2.0 * c.Pnorm * (cx_own - rx_own), vy = 2.0 * c.Pnorm * (cy_own - ry_own);
      if (cpl) {
        vx = vx + c.rho * cpx;
        vy = vy + c.rho * cpy;
      }
      const double wt = tl ? gx.ax * vx + gx.ay * vy : 0.0;
      const double wsh = shdn(wt, 1);
      qx.wq = (l < H) ? wsh : 0.0;
      qx.qvalid = false;
      STAMP_ADD(ST_XQ, t_xs);
      double ustar[1];
      unsigned long long t_q = STAMP_T();
      const int admm0 = n.admm_x;
      const int stx = qp_solve<1, false, BIG ? 8 : XGEMV_U, BIG ? RM_BIG : RM_S | RM_T>(qx, xs_x, zs_x, ys_x, lab_x, warm_x, c.max_inner, c.polish_every, xfac,
                               qx.fld, ustar, n.admm_x, n.pdas_x, n.gi, (A.x_gi >= 2 && first && it == X.it0) ? min(A.x_gi - 1, 2) : (A.x_gi == 4 ? 3 : 0));
      STAMP_ADD(ST_XQP, t_q);
      rep_ok = !(stx & PIADMM_QP_INEXACT) && n.admm_x == admm0 && tables_match(qx, lab_x);
      status_x |= stx;
      ++n.xqp;
      n.inexact += (stx & PIADMM_QP_INEXACT) ? 1 : 0;
      warm_x = true;
      const double u = around(ustar[0], c.round_decimals);
      if (TIES && c.round_decimals >= 0) round_ties(A, t, it, PIADMM_TIE_ROUND_U, X.a0 + w, 0, ustar[0], l < H);
      double px, py, pth;
      rollout_r(rl_x0, rl_y0, rl_th0, rl_s, rl_sl, (l < H) ? u : 0.0, c, H, nonlin_pos, px, py, pth);
      if (l <= H) {
        pos[(w * 2 + 0) * H1 + l] = px;
        pos[(w * 2 + 1) * H1 + l] = py;
      }
      if (l < H) S.u[(it & 1) * 2 * H + w * H + l] = u;
      STAMP_ADD(ST_XSTEP, t_xs);
    }
    __syncthreads();                                     // A: every agent's positions
    L.act = collide<TIES>(A, X, pos, it);
    if (!L.act && L.flag == 0 && !c.fixed_iters && !X.global) {   // no edge ever: stop (:115-116)
      L.stopped = true;
      break;
    }
    L.flag = 1;
    if (__builtin_expect(L.act, 0)) {
      __syncthreads();                                   // B: hat, lam, S, D, last, S.sc
      load_cp();
      rep_ok = false;
    }
    if (iter_tail<TIES>(A, X, L, it, nbar)) break;
    ++it;
  }
  } else {
  bool have = false;          // the x-step of iteration `it` is already in U (a kept speculation)
  int spec_st = 0;
  // Determinism: the speculative x-step repeats the QP of the x-step in U (hat, lam unchanged
  // since), so it is only run when that solve was certified without ADMM and left the parametric
  // tables holding its working set: the repeat is then one cached-table hit -- the same reduced
  // solve on the same tables and q, certified identically -- and changes no state (labels, tables,
  // warm iterates, penalty).  A discarded speculation (a z-step or the stop came) gives its one
  // reduced solve back to the counters, and the next x-step starts from exactly the plain loop's
  // state.  An INEXACT x-QP (or one that needed ADMM, or whose tables hold another working set)
  // is never speculated on (tests/test_gpu_modes.py: the two loop shapes are equal).
  bool spec_ok = false;       // the x-step in U may be repeated speculatively
  bool spec_ran = false;      // this iteration's speculative x-step ran
  // (TIES) a speculative x-step's unrounded controls: its round ties are logged once the verdict
  // keeps it (a discarded speculation's rounding never happened in the reference's loop)
  double tie_u = 0.0;
  int it = X.it0, phase = 0;  // phase 0: before barrier A(it); 1: before barrier B(it)
  bool done = false;
  while (it < X.it_end) {
    // ---- the steady state (r06): iterations whose x-step is a kept speculation and whose repeat
    // is the lean table hit run in this compact loop -- barrier A(it), the repeat for it+1, barrier
    // B(it), the verdict -- whose body holds none of the general solver's code, so its few live
    // values stay in registers (the same barriers, statements and counters as the general loop
    // below, which takes over at the first iteration that needs more: a z-step, the stop, the last
    // iteration, a repeat that does not certify)
    if (phase == 0 && have && !qx.t32) {
      while (true) {
        L.iters = it + 1;
        if (own) {                                       // the kept speculation counts now
          status_x |= spec_st;
          ++n.xqp;
          n.inexact += (spec_st & PIADMM_QP_INEXACT) ? 1 : 0;
        }
        unsigned long long t_sa = STAMP_T();
        __syncthreads();                                 // A(it)
        STAMP_ADD(ST_SYNC_A, t_sa);
        const bool dox = own && it + 1 < X.it_end;       // (spec_ok holds: have)
        spec_ran = dox;
        if (dox) {
          unsigned long long t_xs = STAMP_T();
          const bool tl = l <= H;
          double vx = 2.0 * c.Pnorm * (cx_own - rx_own), vy = 2.0 * c.Pnorm * (cy_own - ry_own);
          if (cpl) {
            vx = vx + c.rho * cpx;
            vy = vy + c.rho * cpy;
          }
          const double wt = tl ? gx.ax * vx + gx.ay * vy : 0.0;
          const double wsh = shdn(wt, 1);
          qx.wq = (l < H) ? wsh : 0.0;
          qx.qvalid = false;
          double ustar[1];
          if (__builtin_expect(!xhit_repeat<BIG ? 8 : XGEMV_U, !BIG>(qx, lab_x, xs_x, ys_x, ustar, n.pdas_x), 0)) {
            phase = 1;                                   // the general loop's phase-1 x-step, then B(it)
            break;
          }
#ifdef PIADMM_XREP
          for (int r = 0; r < PIADMM_XREP; ++r) {        // (diagnostic build: the lean repeat again)
            double ud[1];
            int dp = 0;
            (void)xhit_repeat<BIG ? 8 : XGEMV_U, !BIG>(qx, lab_x, xs_x, ys_x, ud, dp);
          }
#endif
          spec_st = 0;
          warm_x = true;
          const double u = around(ustar[0], c.round_decimals);
          if constexpr (TIES) tie_u = ustar[0];
          if (l < H) S.u[((it + 1) & 1) * 2 * H + w * H + l] = u;
          STAMP_ADD(ST_XSTEP, t_xs);
        }
        unsigned long long t_sb = STAMP_T();
        __syncthreads();                                 // B(it): the pair wave's verdict on iteration it
        STAMP_ADD(ST_SYNC_B, t_sb);
        L.act = X.vd[0] != 0;
        L.flag = X.vd[2];
        L.aliased = X.vd[3];
        L.dis_chk = *X.vdd;
        if (X.vd[1]) {
          if (spec_ran && own) n.pdas_x -= 1;           // discarded by the stop: its one table hit
          L.stopped = true;
          done = true;
          break;
        }
        if (__builtin_expect(L.act, 0)) {
          load_cp();                                     // the speculation used the old hat, lam
          if (spec_ran && own) n.pdas_x -= 1;           // discarded: its one table hit
          have = false;
        } else {
          have = spec_ran;
          if (TIES && c.round_decimals >= 0 && spec_ran)
            round_ties(A, t, it + 1, PIADMM_TIE_ROUND_U, X.a0 + w, 0, tie_u, l < H);
        }
        ++it;
        if (!have || it >= X.it_end) break;
      }
      if (done) break;
      continue;
    }
    if (phase == 0) L.iters = it + 1;
    const int tgt = phase == 0 ? it : it + 1;         // the iteration this x-step belongs to
    const bool dox = own && (phase == 0 ? !have : (it + 1 < X.it_end && spec_ok));
    if (phase == 1) spec_ran = dox;
    // -------- x-step (casadi/main.py:81-106)
    if (dox) {
      unsigned long long t_xs = STAMP_T();
      const bool tl = l <= H;
      double vx = 2.0 * c.Pnorm * (cx_own - rx_own), vy = 2.0 * c.Pnorm * (cy_own - ry_own);
      if (cpl) {
        vx = vx + c.rho * cpx;
        vy = vy + c.rho * cpy;
      }
      const double wt = tl ? gx.ax * vx + gx.ay * vy : 0.0;
      const double wsh = shdn(wt, 1);
      qx.wq = (l < H) ? wsh : 0.0;
      qx.qvalid = false;
      STAMP_ADD(ST_XQ, t_xs);
      double ustar[1];
      unsigned long long t_q = STAMP_T();
      const int admm0 = n.admm_x;
      // phase 1 repeats the certified table hit of the x-step in U (spec_ok): the lean repeat on the
      // transposed tables (LDS mode), qp_solve when it does not certify (or in big mode)
      const bool lean = phase == 1 && !qx.t32 && xhit_repeat<BIG ? 8 : XGEMV_U, !BIG>(qx, lab_x, xs_x, ys_x, ustar, n.pdas_x);
      const int stx = lean ? 0 : qp_solve<1, false, BIG ? 8 : XGEMV_U, BIG ? RM_BIG : RM_S | RM_T>(qx, xs_x, zs_x, ys_x, lab_x, warm_x, c.max_inner, c.polish_every, xfac,
                               qx.fld, ustar, n.admm_x, n.pdas_x, n.gi, (A.x_gi >= 2 && first && tgt == X.it0) ? min(A.x_gi - 1, 2) : (A.x_gi == 4 ? 3 : 0));
      STAMP_ADD(ST_XQP, t_q);
#ifdef PIADMM_XREP
      // diagnostic build (libpiadmm_xrep.so, never the measured library): the same x-step solved
      // PIADMM_XREP more times in place -- the step time's increase is the in-kernel cost of the
      // repeated solves (a repeat of a certified solve is a table hit and changes no state)
      for (int r = 0; r < PIADMM_XREP; ++r) {
        int dx = 0, dp = 0, dg = 0;
        double ud[1];
        (void)qp_solve<1, false, BIG ? 8 : XGEMV_U, BIG ? RM_BIG : RM_S | RM_T>(qx, xs_x, zs_x, ys_x, lab_x, true, c.max_inner, c.polish_every, xfac,
                               qx.fld, ud, dx, dp, dg, 0);
      }
#endif
      // a repeat of this solve may be speculated only if it certified without ADMM and its
      // working set's tables are held (the repeat is then one table hit)
      spec_ok = lean || (!(stx & PIADMM_QP_INEXACT) && n.admm_x == admm0 && tables_match(qx, lab_x));
      if (phase == 0) {
        status_x |= stx;
        ++n.xqp;
        n.inexact += (stx & PIADMM_QP_INEXACT) ? 1 : 0;
      } else {
        spec_st = stx;                                 // counted if kept
      }
      warm_x = true;
      unsigned long long t_rd = STAMP_T();
      const double u = around(ustar[0], c.round_decimals);
      if (TIES && c.round_decimals >= 0) {
        if (phase == 0)
          round_ties(A, t, tgt, PIADMM_TIE_ROUND_U, X.a0 + w, 0, ustar[0], l < H);
        else
          tie_u = ustar[0];                              // logged if the verdict keeps it
      }
      STAMP_ADD(ST_ROUND, t_rd);
      if (l < H) S.u[(tgt & 1) * 2 * H + w * H + l] = u;
      STAMP_ADD(ST_XSTEP, t_xs);
    }
    if (phase == 0 && have && own) {                   // the kept speculation counts now
      status_x |= spec_st;
      ++n.xqp;
      n.inexact += (spec_st & PIADMM_QP_INEXACT) ? 1 : 0;
    }
    unsigned long long t_sa = STAMP_T();
    __syncthreads();                                     // A(it) (phase 0) or B(it) (phase 1)
    STAMP_ADD(phase == 0 ? ST_SYNC_A : ST_SYNC_B, t_sa);
    if (phase == 0) {
      phase = 1;
      continue;
    }
    // barrier B(it): the pair wave's verdict on iteration it
    L.act = X.vd[0] != 0;
    L.flag = X.vd[2];
    L.aliased = X.vd[3];
    L.dis_chk = *X.vdd;
    if (X.vd[1]) {
      if (spec_ran && own) n.pdas_x -= 1;   // discarded by the stop: its one table hit
      L.stopped = true;
      break;
    }
    if (__builtin_expect(L.act, 0)) {
      load_cp();                                         // the speculation used the old hat, lam
      if (spec_ran && own) n.pdas_x -= 1;   // discarded: its one table hit
      have = false;
    } else {
      have = spec_ran;
      if (TIES && c.round_decimals >= 0 && spec_ran)
        round_ties(A, t, it + 1, PIADMM_TIE_ROUND_U, X.a0 + w, 0, tie_u, l < H);
    }
    ++it;
    phase = 0;
  }
  }
  n.warm = own && warm_x;
  // ---- the agent's state of this launch and, in the last launch, outputs and propagation
  // (casadi/main.py:185-192)
  if (own) {
    const int a = X.a0 + w;
    // the last executed iteration's buffer (a skipped launch: the buffer its state was restored to)
    const double* posl = S.pos + ((X.skip ? X.it0 - 1 : L.iters - 1) & 1) * 4 * H1;
    for (int i = l; i < 2 * H1; i += WAVE) A.pos_old[(size_t)a * 2 * H1 + i] = posl[w * 2 * H1 + i];
    const double u = (l < H) ? S.u[((X.skip ? X.it0 - 1 : L.iters - 1) & 1) * 2 * H + w * H + l] : 0.0;
    if (l < H) A.u[(size_t)a * H + l] = u;
    if (l == 0) {
      A.status[a] = status_x;
      A.rho_x[a] = qx.rho;
    }
    if (__builtin_expect(A.xcache_rho[a] != qx.rho, 0)) {   // adaptive rho rebuilt K_s^-1: refresh the cache
      double* Kc = A.Kx_cache + (size_t)a * H * H;
      if (qx.kf32) {
        for (int i = l; i < H * H; i += WAVE) Kc[i] = (double)qx.Kf[i];   // the fp32 image
      } else if (qx.K != Kc) {
        for (int i = l; i < H * H; i += WAVE) Kc[i] = qx.K[i];
      }
      if (l == 0) A.xcache_rho[a] = qx.rho;
    }
    if (!X.last_launch) {
      if (qx.wraw) warm_to_scaled(qx, xs_x, zs_x, ys_x);
      double* qs = A.qs_x + (size_t)a * 5 * WAVE;
      signed char* ql = A.ql_x + (size_t)a * 2 * WAVE;
      qs[l] = xs_x[0];
      qs[WAVE + l] = zs_x[0];
      qs[2 * WAVE + l] = zs_x[1];
      qs[3 * WAVE + l] = ys_x[0];
      qs[4 * WAVE + l] = ys_x[1];
      ql[l] = lab_x[0];
      ql[WAVE + l] = lab_x[1];
    } else {
      double px, py, pth;
      rollout(S.xt + 3 * w, A.spd[a], u, c, H, true, px, py, pth);
      if (l == 1) {
        A.xt[3 * a + 0] = px;
        A.xt[3 * a + 1] = py;
        A.xt[3 * a + 2] = pth;
      }
      if (l == 0) A.warm_ok[a] = 1;
      if (l < HCAP) {
        signed char* lb = A.lab_x + (size_t)a * 2 * HCAP;
        lb[l] = lab_x[0];
        lb[HCAP + l] = lab_x[1];
      }
    }
  }
}

// -------------------------------------------------------------------- the pair wave (2)
// Wave PW owns the component's pair (when it has one): the per-step pair setup (concurrent with
// the agents' setups), the z-step QP, the hat rollouts, the dual update and the residuals
// (casadi/main.py:121-181).  Its QP state stays in this wave's registers for the whole step.
template <bool BIG, bool TIES, int SH>
__device__ __forceinline__ void pair_part(const DevArgs& A, const StepCtx& X, LoopCtl& L, int& nbar, WaveCnt& n) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const piadmm_config_t& c = A.cfg;
  const int H = X.H, H1 = X.H1, l = X.l, ci = X.ci, e = X.e, t = X.t;
  const bool big = BIG, f32 = X.f32, first = X.first;
  const CompLds& S = X.S;
  // ---- the pair's LDS regions (lds_bytes() in piadmm_internal.h)
  double *Ke = nullptr, *scr;
  float* Kef = nullptr;
  if (!big) {
    double* p = lds;
    p += f32 ? kxf_words(H) : 2 * H * H;                 // agent K_s^-1 (the agent waves')
    p += 2 * gt_stride(H);                               // agent polish G T' | g (the agent waves')
    if (f32) { Kef = (float*)p; p += 2 * H * H; }        // 4*H*H fp32 pair K_s^-1
    else { Ke = p; p += 4 * H * H; }                     // 4*H*H     pair K_s^-1
    scr = p;                                             // 64 x LD   pair scratch
  } else {
    Ke = (e >= 0) ? A.Ke_g + (size_t)e * 4 * H * H : nullptr;   // HBM / L2 (built in place)
    scr = lds;                                           // 64 x LD   pair scratch
    if (f32) Kef = (float*)(S.sc + 32);                  // big mode: fp32 image of the pair K_s^-1
  }
  double* zdiag = X.vec_all + NWT * 512 + PW * 128;
  int* zids = X.wm.ib + 128;
  int* zfs = X.wm.ib + 257;
  if (l == 0) zfs[0] = -1;

  QP<2> qe;
  double xs_e[2] = {0.0, 0.0}, zs_e[5] = {0, 0, 0, 0, 0}, ys_e[5] = {0, 0, 0, 0, 0};
  signed char lab_e[5] = {0, 0, 0, 0, 0};
  bool warm_e = false;
  int status_e = 0;
  Geo ge1, ge2;
  double c1x = 0.0, c1y = 0.0, c2x = 0.0, c2y = 0.0;
  if (e >= 0) {
    unsigned long long t0 = STAMP_T();
    ge1 = make_geo(S.xt + 0, A.spd[X.a0], c);
    ge2 = make_geo(S.xt + 3, A.spd[X.a0 + 1], c);
    affine_c(ge1, c.dt, H, c1x, c1y);
    affine_c(ge2, c.dt, H, c2x, c2y);
    qe.H = H;
    qe.n = 2 * H;
    qe.umax = c.u_max;
    qe.dumax = c.du_max;
    qe.h0 = 0.0;
    qe.Pcost2 = 2.0 * c.Pcost;
    qe.beta = c.beta;
    qe.rho = A.rho_e[e];
    qe.sigma = c.admm_sigma;
    qe.alpha = c.admm_alpha;
    qe.tol = c.qp_tol;
    qe.K = Ke;
    qe.Kf = Kef;
    qe.kf32 = f32;
    qe.Pinv = A.tab_e + (size_t)e * 8 * H * H;
    qe.vb = X.wm.vb;
    qe.fac = scr;
    qe.fdiag = zdiag;
    qe.ib = zids;
    qe.fstate = zfs;
    qe.fld = LD;
    qe.mmax = WAVE;
    qe.gmem = big;
    qe.xld = 0;
    // dual active-set columns in the K_s^-1 region (4H^2 doubles, or 2H^2 with fp32 images)
    qe.Y = Ke ? Ke : (double*)Kef;
    qe.ycap = A.pair_gi ? ((Ke ? 4 : 2) * H * H) / (2 * H) : 0;
    // LDS mode: the columns transposed (2H rows of stride yld, pd_qp.h gi_solve RM_Y) in the same
    // region -- stride 2H (fp64), H rounded down to even (fp32 images)
    if (!big) {
      qe.yld = Ke ? 2 * H : (H & ~1);
      qe.ycap = min(qe.ycap, qe.yld);
    }
    qe.y_in_k = true;
    qe.gws = A.gi_ws + (size_t)e * GI_WS;
    qe.gws_warm = A.pair_warm != 0;
    qe.wide = A.gi_wide ? A.gi_wide + (size_t)blockIdx.x * A.gi_wide_stride : nullptr;
    qe.tstep = t;
    // Ke doubles as the H x 2H staging of the per-scenario pair tables; with fp32 images in
    // LDS mode the fp32 region (2H^2 doubles of space) takes that role
    setup_pair(A, e, qe, ge1, ge2, c1x, c1y, c2x, c2y, S.seed, scr, Ke ? Ke : (double*)Kef, X.deff);
    if (!first) {
      const double* qs = A.qs_e + (size_t)e * 12 * WAVE;
      const signed char* ql = A.ql_e + (size_t)e * 5 * WAVE;
      xs_e[0] = qs[l];
      xs_e[1] = qs[WAVE + l];
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        zs_e[s] = qs[(2 + s) * WAVE + l];
        ys_e[s] = qs[(7 + s) * WAVE + l];
        lab_e[s] = ql[s * WAVE + l];
      }
      warm_e = (A.cst[(size_t)ci * 4 + 2] >> 2) & 1;
      status_e = A.status[A.N + e];
    }
    // (no receding-horizon label guess for the pair: tools/pair_exp.py found the polish from
    // shifted labels failing on half of the bench's pair QPs, each failure costing PDAS_STEPS
    // reduced solves before the ADMM fallback)
    STAMP_ADD(ST_SETUP_Z, t0);
  }
  const bool prebuild = first && e >= 0 && qe.ycap > 0 && X.it0 < X.it_end;
  if (X.helper) {
    // the warm rows for the helper wave (every step: gm = 0 when there is no warm build)
    int code = -1;
    const int gm = (prebuild && qe.gws && qe.gws_warm) ? warm_codes(qe, code) : 0;
    int* hd = X.wp.hdr;
    if (l == 0) {
      hd[0] = gm;
      hd[1] = 0;
      X.wp.dat[0] = qe.g1;
      X.wp.dat[1] = qe.g2;
      reinterpret_cast<unsigned long long*>(X.wp.dat)[2] = reinterpret_cast<unsigned long long>(qe.Pinv);
    }
    if (l < WP_R) hd[2 + l] = 0;
    hd[8 + l] = code;
  }
  __syncthreads();

  // speculative loop shape (agent_part): this wave also rolls the agents' controls out and
  // publishes the iteration's verdict (X.vd) before barrier B
  constexpr bool specm = SH == 1;
  // the agents' start states and speeds (the per-iteration rollouts of the speculative shape)
  double ra_s[2] = {0.0, 0.0};
  if (specm)
    for (int v = 0; v < X.na; ++v) ra_s[v] = A.spd[X.a0 + v];
  // the pair QP's first solve of the step goes straight to the dual active set from the stored
  // active set (no warm labels yet): append those rows now, while the agents solve their first
  // x-steps (they depend on the step's geometry only; setup_pair built it)
  if (prebuild) {
    double xd[2];
    double yd[5];
    signed char ld[5];
    int nd = 0;
    unsigned long long t_pb = STAMP_T();
    gi_solve<2, BIG ? RM_BIG : RM_S | RM_Y>(qe, nullptr, ld, xd, yd, nd, nullptr, false, true, X.helper ? &X.wp : nullptr);
    STAMP_ADD(ST_ZR_SOLVE, t_pb);
  }
  bool resume = false;   // the compact loop ran barrier A, the rollouts and the test of iteration it
  for (int it = X.it0; it < X.it_end; ++it) {
    if (!specm && !resume) {
      // ---- the steady state (r06, plain shape): iterations in which no pair collides -- barrier
      // A, the collision test, the residual record, the stop test (in-kernel grid barrier included)
      // -- in a compact loop; at the first colliding iteration (or the no-edge-ever stop) the
      // general body below takes over after the test, for the same iteration
      bool stop = false;
      while (true) {
        L.iters = it + 1;
        double* const ps = S.pos + (it & 1) * 4 * H1;
        unsigned long long t_sa = STAMP_T();
        __syncthreads();                                 // A: every agent's positions
        STAMP_ADD(ST_SYNC_A, t_sa);
        L.act = collide<TIES>(A, X, ps, it);
        if (__builtin_expect(L.act || (L.flag == 0 && !c.fixed_iters && !X.global), 0)) {
          resume = true;
          break;
        }
        L.flag = 1;
        unsigned long long t_tw = STAMP_T();
        wsync();
        if (l == 0) {
          X.resid[2 * it + 0] = 0.0;
          X.resid[2 * it + 1] = 0.0;
        }
        STAMP_ADD(ST_TERMW, t_tw);
        stop = iter_tail<TIES>(A, X, L, it, nbar);
        if (stop || ++it >= X.it_end) break;
      }
      if (!resume) break;
    }
    if (specm && X.roll && !resume) {
      // ---- the steady state (r06): iterations in which no pair collides run in this compact loop
      // -- barrier A, the rollouts, the collision test, the residual record, the stop decision, the
      // verdict, barrier B -- whose body holds none of the z-step's code (agent_part's compact loop
      // is its counterpart).  At the first colliding iteration (or the no-edge-ever stop) the
      // general body below takes over after the test, for the same iteration.
      while (true) {
        L.iters = it + 1;
        double* const ps = S.pos + (it & 1) * 4 * H1;
        unsigned long long t_sa = STAMP_T();
        __syncthreads();                                 // A: every agent's controls of iteration it
        STAMP_ADD(ST_SYNC_A, t_sa);
        {
          const bool nonlin_pos = c.pos_model != 0;
          double px, py, pth;
          unsigned long long t_ro = STAMP_T();
          const double u = (l < H) ? S.u[(it & 1) * 2 * H + l] : 0.0;
          rollout_r(S.xt[0], S.xt[1], S.xt[2], ra_s[0], ra_s[0] / c.L, u, c, H, nonlin_pos, px, py, pth);
#ifdef PIADMM_PREP
          for (int r = 0; r < PIADMM_PREP; ++r) {        // (diagnostic build: the rollout again)
            double qx2, qy2, qt2;
            rollout_r(S.xt[0], S.xt[1], S.xt[2], ra_s[0], ra_s[0] / c.L, u + px * 1e-300, c, H, nonlin_pos, qx2, qy2, qt2);
            if (qx2 == -12345.678) S.sc[31] = qy2 + qt2;
          }
#endif
          if (l <= H) {
            ps[0 * H1 + l] = px;
            ps[1 * H1 + l] = py;
          }
          STAMP_ADD(ST_XQ, t_ro);
          unsigned long long t_rw = STAMP_T();
          while (__hip_atomic_load(X.rflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != it + 1)
            __builtin_amdgcn_s_sleep(1);
          STAMP_ADD(ST_XROLL, t_rw);
          wsync();
        }
        L.act = collide<TIES>(A, X, ps, it);
        if (__builtin_expect(L.act || (L.flag == 0 && !c.fixed_iters && !X.global), 0)) {
          resume = true;                                 // the general body, from the test on
          break;
        }
        L.flag = 1;
        // the residual record of an iteration without a z-step (rk = sk = 0; hat unchanged)
        unsigned long long t_tw = STAMP_T();
        wsync();
        if (l == 0) {
          X.resid[2 * it + 0] = 0.0;
          X.resid[2 * it + 1] = 0.0;
        }
        STAMP_ADD(ST_TERMW, t_tw);
        const bool stop = iter_tail<TIES>(A, X, L, it, nbar);
        if (l == 0) {
          X.vd[0] = 0;
          X.vd[1] = stop ? 1 : 0;
          X.vd[2] = L.flag;
          X.vd[3] = L.aliased;
          *X.vdd = L.dis_chk;
        }
        unsigned long long t_sb = STAMP_T();
        __syncthreads();                                 // B: the verdict
        STAMP_ADD(ST_SYNC_B, t_sb);
        if (stop) break;
        if (++it >= X.it_end) break;
      }
      if (!resume) break;                                // stopped, or the last iteration is done
    }
    double* const pos = S.pos + (it & 1) * 4 * H1;
    if (!resume) {
    L.iters = it + 1;
    unsigned long long t_sa = STAMP_T();
    __syncthreads();                                     // A: every agent's positions / controls
    STAMP_ADD(ST_SYNC_A, t_sa);
    if (specm && X.roll) {
      // pos_old = dynamic_update_local of the rounded controls (casadi/main.py:105): agent 0's here,
      // agent 1's on the roller wave at the same time (roll_part); then wait for the roller's flag
      const bool nonlin_pos = c.pos_model != 0;
      double px, py, pth;
      unsigned long long t_ro = STAMP_T();
      const double u = (l < H) ? S.u[(it & 1) * 2 * H + l] : 0.0;
      rollout_r(S.xt[0], S.xt[1], S.xt[2], ra_s[0], ra_s[0] / c.L, u, c, H, nonlin_pos, px, py, pth);
#ifdef PIADMM_PREP
      {
        // diagnostic build (libpiadmm_prep.so, never the measured library): the pair wave's rollout
        // done PIADMM_PREP more times per iteration -- prices the pair wave's chain (is it critical?)
        for (int r = 0; r < PIADMM_PREP; ++r) {
          double qx2, qy2, qt2;
          rollout_r(S.xt[0], S.xt[1], S.xt[2], ra_s[0], ra_s[0] / c.L, u + px * 1e-300, c, H, nonlin_pos, qx2, qy2, qt2);
          if (qx2 == -12345.678) S.sc[31] = qy2 + qt2;
        }
      }
#endif
      if (l <= H) {
        pos[0 * H1 + l] = px;
        pos[1 * H1 + l] = py;
      }
      STAMP_ADD(ST_XQ, t_ro);          // (pair wave: its rollout of agent 0)
      unsigned long long t_rw = STAMP_T();
      while (__hip_atomic_load(X.rflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != it + 1)
        __builtin_amdgcn_s_sleep(1);
      STAMP_ADD(ST_XROLL, t_rw);
      wsync();
    } else if (specm) {
      // pos_old = dynamic_update_local of the rounded controls (casadi/main.py:105), per agent
      // both agents' rollouts side by side (two independent DPP-scan / sincos chains in one block,
      // so their latencies overlap; a single-agent component's second one is discarded)
      const bool nonlin_pos = c.pos_model != 0;
      double px[2], py[2], pth[2];
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const bool va = v < X.na;
        const double u = (l < H && va) ? S.u[(it & 1) * 2 * H + v * H + l] : 0.0;
        rollout_r(va ? S.xt[3 * v + 0] : 0.0, va ? S.xt[3 * v + 1] : 0.0, va ? S.xt[3 * v + 2] : 0.0, ra_s[v],
                  ra_s[v] / c.L, u, c, H, nonlin_pos, px[v], py[v], pth[v]);
      }
      if (l <= H)
        for (int v = 0; v < X.na; ++v) {
          pos[(v * 2 + 0) * H1 + l] = px[v];
          pos[(v * 2 + 1) * H1 + l] = py[v];
        }
      wsync();
    }
    L.act = collide<TIES>(A, X, pos, it);
    }
    resume = false;
    if (!L.act && L.flag == 0 && !c.fixed_iters && !X.global) {   // no edge ever: stop (:115-116)
      L.stopped = true;
      if (specm) {
        if (l == 0) {
          X.vd[0] = 0;
          X.vd[1] = 1;
          X.vd[2] = L.flag;
          X.vd[3] = L.aliased;
          *X.vdd = L.dis_chk;
        }
        __syncthreads();                                 // B: the verdict
      }
      break;
    }
    L.flag = 1;
    // -------- z-step + dual update on the colliding pair (casadi/main.py:121-162)
    if (__builtin_expect(L.act, 0)) {     // cold: about once per MPC step
      unsigned long long t_z = STAMP_T();
      const bool tl = l <= H;
      double bx[2], by[2];
      bx[0] = tl ? pos[0 * H1 + l] + S.lam[0 * H1 + l] - c1x : 0.0;
      by[0] = tl ? pos[1 * H1 + l] + S.lam[1 * H1 + l] - c1y : 0.0;
      bx[1] = tl ? pos[2 * H1 + l] + S.lam[2 * H1 + l] - c2x : 0.0;
      by[1] = tl ? pos[3 * H1 + l] + S.lam[3 * H1 + l] - c2y : 0.0;
      const double w1 = tl ? ge1.ax * bx[0] + ge1.ay * by[0] : 0.0;
      const double w2 = tl ? ge2.ax * bx[1] + ge2.ay * by[1] : 0.0;
      const double q1 = Tt_apply(shdn(w1, 1)), q2 = Tt_apply(shdn(w2, 1));
      qe.q[0] = (l < H) ? -c.rho * q1 : 0.0;
      qe.q[1] = (l < H) ? -c.rho * q2 : 0.0;
      qe.qvalid = true;
      double uh[2];
      unsigned long long t_zq = STAMP_T();
      // K_s^-1 of the pair is built in the LDS scratch and copied (2H <= 64), or in place
      // (big mode, two columns per lane, in HBM)
      const int ste = qp_solve<2, BIG, XGEMV_U, BIG ? RM_BIG : RM_S | RM_Y>(qe, xs_e, zs_e, ys_e, lab_e, warm_e, c.max_inner, c.polish_every,
                               big ? Ke : scr, big ? 2 * H : LD, uh,
                               n.admm_z, n.pdas_z, n.gi);
      STAMP_ADD(ST_ZQP, t_zq);
      status_e |= ste;
      ++n.zqp;
      n.inexact += (ste & PIADMM_QP_INEXACT) ? 1 : 0;
      warm_e = true;
      // hat positions: nonlinear rollout of the rounded pair controls (:153-158)
      double hx[2], hy[2], hth;
      for (int v = 0; v < 2; ++v) {
        const double uv = (l < H) ? around(uh[v], c.round_decimals) : 0.0;
        if (TIES && c.round_decimals >= 0) round_ties(A, t, it, PIADMM_TIE_ROUND_UHAT, e, v * H, uh[v], l < H);
        rollout(S.xt + 3 * v, A.spd[X.a0 + v], uv, c, H, true, hx[v], hy[v], hth);
      }
      // dual update (plain :161-162 / PI + anti-windup MATLAB :156-188)
      double px[2], py[2];
      for (int v = 0; v < 2; ++v) {
        px[v] = tl ? pos[(2 * v + 0) * H1 + l] : 0.0;
        py[v] = tl ? pos[(2 * v + 1) * H1 + l] : 0.0;
      }
      double dist = 0.0;
      {
        const double dx = px[0] - px[1], dy = py[0] - py[1];
        dist = sqrt(dx * dx + dy * dy);
      }
      const double mind = wmin(tl ? dist : INFINITY);
      const double kP = c.theta1 - c.theta2 / (1.0 + exp(-mind));
      const double Wsat = c.windup_sat;
      for (int v = 0; v < 2; ++v) {
        double* lam = S.lam + v * 2 * H1;
        double* Sv = S.S + v * 2 * H1;
        double* Dv = S.D + v * 2 * H1;
        double* hat = S.hat + v * 2 * H1;
        bool changed = false;
        double lraw[2], lsat[2];
        for (int xy = 0; xy < 2; ++xy) {
          const double p = xy == 0 ? px[v] : py[v];
          const double h = xy == 0 ? hx[v] : hy[v];
          double lv = tl ? lam[xy * H1 + l] : 0.0;
          const double err = p - h;
          if (c.dual_mode == PIADMM_DUAL_PLAIN) {
            lv = lv + c.rho * err;
          } else {
            const double sv = tl ? (Sv[xy * H1 + l] + c.kI * err) + Dv[xy * H1 + l] : 0.0;
            if (tl) Sv[xy * H1 + l] = sv;
            lv = sv + kP * err;
          }
          lraw[xy] = lv;
          lsat[xy] = c.windup ? fmin(Wsat, fmax(lv, -Wsat)) : lv;
          changed |= tl && (lsat[xy] != lraw[xy]);
          if (tl) hat[xy * H1 + l] = h;
        }
        const bool anyc = wany(changed);
        for (int xy = 0; xy < 2; ++xy) {
          if (tl) {
            lam[xy * H1 + l] = lsat[xy];
            if (c.windup) Dv[xy * H1 + l] = anyc ? lsat[xy] - lraw[xy] : 0.0;
          }
        }
      }
      // residual contributions of this pair (casadi/main.py:167-173): v1 side only
      double rr = 0.0, ss = 0.0;
      if (tl) {
        const double ex = px[0] - S.hat[0 * H1 + l], ey = py[0] - S.hat[1 * H1 + l];
        rr = ex * ex + ey * ey;
        const double fx = c.rho * (S.last[0 * H1 + l] - S.hat[0 * H1 + l]);
        const double fy = c.rho * (S.last[1 * H1 + l] - S.hat[1 * H1 + l]);
        ss = fx * fx + fy * fy;
      }
      rr = wsum(rr);
      ss = wsum(ss);
      if (l == 0) {
        S.sc[0] = 2.0 * sqrt(rr);
        S.sc[1] = L.aliased ? 0.0 : 2.0 * sqrt(ss);
        S.sc[2] = rdl(dist, 1);
        if (TIES && c.term_dist_check) scalar_tie(A, t, it, PIADMM_TIE_DIST, e, 0, S.sc[2], X.deff);
      }
      STAMP_ADD(ST_ZSTEP, t_z);
    }
    // -------- residual record (casadi/main.py:164-181; MATLAB :191-210): this wave wrote S.sc;
    // it records the residuals and, unless the component stops, last_iter_hat_pos before barrier
    // B.  S.sc is rewritten only after the next iteration's barrier A.
    {
      unsigned long long t_tw = STAMP_T();
      wsync();
      const double rk0 = L.act ? S.sc[0] : 0.0;
      const double sk0 = L.act ? S.sc[1] : 0.0;
      const double dc0 = L.act ? S.sc[2] : L.dis_chk;
      if (l == 0) {
        X.resid[2 * it + 0] = rk0;
        X.resid[2 * it + 1] = sk0;
      }
      const bool stop0 = !c.fixed_iters && !X.global && rk0 <= c.eps_pri && sk0 <= c.eps_dual &&
                         (!c.term_dist_check || dc0 > X.deff);
      // last_iter_hat_pos = hat_pos_old: only a z-step changes hat, so the copy is needed
      // only after one (S.last already equals hat otherwise)
      if (__builtin_expect(L.act && !stop0 && !c.alias_dual_residual, 0))
        for (int i = l; i < 4 * H1; i += WAVE) S.last[i] = S.hat[i];
      STAMP_ADD(ST_TERMW, t_tw);
    }
    if (specm) {
      // the stop decision here (iter_tail without a grid barrier), published with the iteration's
      // flags before barrier B; the agents adopt it from X.vd
      const bool stop = iter_tail<TIES>(A, X, L, it, nbar);
      if (l == 0) {
        X.vd[0] = L.act ? 1 : 0;
        X.vd[1] = stop ? 1 : 0;
        X.vd[2] = L.flag;
        X.vd[3] = L.aliased;
        *X.vdd = L.dis_chk;
      }
      unsigned long long t_sb = STAMP_T();
      __syncthreads();                                   // B: the verdict (and the z-step's state)
      STAMP_ADD(ST_SYNC_B, t_sb);
      if (stop) break;
      continue;
    }
    unsigned long long t_sb = STAMP_T();
    if (__builtin_expect(L.act, 0)) __syncthreads();     // B
    STAMP_ADD(ST_SYNC_B, t_sb);
    if (iter_tail<TIES>(A, X, L, it, nbar)) break;
  }
  n.warm = e >= 0 && warm_e;
  if (e >= 0) {
    if (l == 0) A.rho_e[e] = qe.rho;
    if (!X.last_launch) {
      if (qe.wraw) warm_to_scaled(qe, xs_e, zs_e, ys_e);
      double* qs = A.qs_e + (size_t)e * 12 * WAVE;
      signed char* ql = A.ql_e + (size_t)e * 5 * WAVE;
      // unscaled (the next launch restarts in identity scaling, setup_pair)
      qs[l] = qe.D[0] * xs_e[0];
      qs[WAVE + l] = qe.D[1] * xs_e[1];
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        qs[(2 + s) * WAVE + l] = (qe.E[s] != 0.0) ? zs_e[s] / qe.E[s] : 0.0;
        qs[(7 + s) * WAVE + l] = qe.E[s] * ys_e[s];
        ql[s * WAVE + l] = lab_e[s];
      }
    }
    if (l == 0) A.status[A.N + e] = status_e;
  }
}

// -------------------------------------------------------------------- the roller wave (RW)
// Speculative loop only: agent 1's rollout of each iteration's rounded controls (pos_old =
// dynamic_update_local, casadi/main.py:105), concurrent with the pair wave's rollout of agent 0, so
// the pair wave's chain before the verdict (two rollouts, the collision test) -- which the agent
// waves wait for at barrier B -- holds one rollout, not two.  It takes the same barriers (A, B) and
// stops with the pair wave's verdict.
__device__ __forceinline__ void roll_part(const DevArgs& A, const StepCtx& X) {
  const piadmm_config_t& c = A.cfg;
  const int H = X.H, H1 = X.H1, l = X.l;
  const CompLds& S = X.S;
  const bool has = X.na == 2;
  const double s = has ? A.spd[X.a0 + 1] : 0.0;
  const double x0 = has ? S.xt[3] : 0.0, y0 = has ? S.xt[4] : 0.0, th0 = has ? S.xt[5] : 0.0;
  const bool nonlin_pos = c.pos_model != 0;
  __syncthreads();                                       // the parts' setup barrier
  if (X.helper) warm_help(X.wp, H);                      // the pair's warm rows, before iteration it0's A
  for (int it = X.it0; it < X.it_end; ++it) {
    double* const pos = S.pos + (it & 1) * 4 * H1;
    unsigned long long t_sa = STAMP_T();
    __syncthreads();                                     // A: the agents' controls of iteration it
    STAMP_ADD(ST_SYNC_A, t_sa);
    unsigned long long t_ro = STAMP_T();
    if (has) {
      double px, py, pth;
      const double u = (l < H) ? S.u[(it & 1) * 2 * H + H + l] : 0.0;
      rollout_r(x0, y0, th0, s, s / c.L, u, c, H, nonlin_pos, px, py, pth);
      if (l <= H) {
        pos[2 * H1 + l] = px;
        pos[3 * H1 + l] = py;
      }
    }
    // (release: the wave's position stores complete before the flag)
    if (l == 0) __hip_atomic_store(X.rflag, it + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    STAMP_ADD(ST_XQ, t_ro);
    unsigned long long t_sb = STAMP_T();
    __syncthreads();                                     // B: the pair wave's verdict
    STAMP_ADD(ST_SYNC_B, t_sb);
    if (X.vd[1]) break;
  }
}

// -------------------------------------------------------------------- the helper wave (plain shape)
// The plain loop's fourth wave: the pair's warm rows at the step's start (pd_qp.h warm_help), then
// the loop's barriers and decisions as the agent waves take them -- barrier A, the collision test,
// barrier B after a z-step, the stop test (its grid barrier included) -- with no work of its own.
template <bool TIES>
__device__ __forceinline__ void help_part(const DevArgs& A, const StepCtx& X, LoopCtl& L, int& nbar) {
  const piadmm_config_t& c = A.cfg;
  const CompLds& S = X.S;
  __syncthreads();                                       // the parts' setup barrier
  warm_help(X.wp, X.H);
  for (int it = X.it0; it < X.it_end; ++it) {
    L.iters = it + 1;
    double* const pos = S.pos + (it & 1) * 4 * X.H1;
    __syncthreads();                                     // A
    L.act = collide<TIES>(A, X, pos, it);
    if (!L.act && L.flag == 0 && !c.fixed_iters && !X.global) {   // no edge ever: stop
      L.stopped = true;
      break;
    }
    L.flag = 1;
    if (L.act) __syncthreads();                          // B
    if (iter_tail<TIES>(A, X, L, it, nbar)) break;
  }
}

// One launch runs outer iterations [it0, it1) of MPC step t for every component (one
// workgroup each).  The fused mode is one launch (0, max_outer, FIRST | LAST); the global
// termination mode (term_global, reference quirk B9) runs one launch per outer iteration,
// with the per-step state carried in HBM between launches (restore / save below) and the
// stop decision taken by the host from all-reduced partials, then a LAST launch with no
// iterations for the outputs and the propagation.
// Wave layout: waves 0 and 1 run the agents' x-steps (agent_part), wave 2 the pair
// (pair_part); the two loops take the same barriers and stop decisions.
template <bool BIG, bool TIES, int SH>
__device__ __forceinline__ void mpc_step_body(const DevArgs& A, int t, int it0, int it1, int flags, int slot,
                                              int& nbar) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int s_int[NWT * 272];   // per wave: x ids [128], z ids [128], fstate x, fstate z
  __shared__ int s_vd[4];
  __shared__ double s_vdd;
  __shared__ int s_rflag;
  const piadmm_config_t& c = A.cfg;
  StepCtx X;
  X.vd = s_vd;
  X.vdd = &s_vdd;
  X.rflag = &s_rflag;
  if (threadIdx.x == 0) s_rflag = 0;   // (iterations count from it0 >= 0: the flag waits for it + 1)
  X.H = c.H;
  X.H1 = c.H + 1;
  X.ci = blockIdx.x;
  X.w = threadIdx.x >> 6;
  X.l = lid();
  X.t = t;
  X.slot = slot;
  X.a0 = A.comp_ptr[X.ci];
  X.na = A.comp_ptr[X.ci + 1] - X.a0;
  X.e = A.comp_edge[X.ci];
  X.big = BIG;
  X.f32 = c.precision == 1;
  const int H = X.H, H1 = X.H1, ci = X.ci, e = X.e, na = X.na, a0 = X.a0;

  // ---- LDS carve (lds_bytes() in piadmm_internal.h): the matrix regions are carved by the parts
  double* vec_all;
  if (!BIG) {
    vec_all = lds + (X.f32 ? kxf_words(H) : 2 * H * H) + 2 * gt_stride(H) + (X.f32 ? 2 * H * H : 4 * H * H) +
              64 * (LD + 1) + NW * HMAX * (HMAX + 2) + NW * HMAX * XLDT;   // NWT x 512
  } else {
    vec_all = lds + 64 * (LD + 1) + NW * xreg(H);                          // NWT x 512
  }
  X.vec_all = vec_all;
  double* fdiag_all = vec_all + NWT * 512;               // NWT x 128
  CompLds& S = X.S;
  S.pos = fdiag_all + NWT * 128;
  S.xt = S.pos + 8 * H1;   // pos_old double-buffered by outer-iteration parity
  S.seed = S.xt + 6;
  S.u = S.seed + 4;         // agent controls, double-buffered by outer-iteration parity (2 x 2H)
  S.hat = S.u + 4 * H;
  S.lam = S.hat + 4 * H1;
  S.S = S.lam + 4 * H1;
  S.D = S.S + 4 * H1;
  S.last = S.D + 4 * H1;
  S.sc = S.last + 4 * H1;
  X.wm = WaveMem{vec_all + X.w * 512, s_int + X.w * 272};

  X.first = (flags & F_FIRST) != 0;
  X.last_launch = (flags & F_LAST) != 0;
  X.global = (flags & F_GLOBAL) != 0;
  X.coop = (flags & F_COOP) != 0;   // global stop decided in-kernel (cooperative launch)
  // the speculative loop shape where it pays: no grid barrier in the loop, and the nonlinear
  // position model (MATLAB's dynamic_update_local, a sincos rollout per iteration) whose rollout
  // is worth taking off the agents' chain -- measured: matlab_pi 256 x H30 0.534 -> 0.518 ms per
  // step; the linearised model's cheap rollout does not pay for the second barrier
  // (casadi_default 64 x H20 0.633 -> 0.677 ms)
  X.spec = SH == 1;
  // (launch_mpc_step: SH = 1 iff no in-kernel grid barrier, the nonlinear position model and no F_NOSPEC)
  X.roll = X.spec && blockDim.x == NWA * WAVE;   // launch_mpc_step adds the roller wave to this shape
  // the fourth wave also builds the pair's warm rows where its LDS ring fits (lds_bytes)
  X.helper = !BIG && H <= WPIPE_HMAX && blockDim.x == NWA * WAVE && !(flags & F_NOHELPER);
  X.wp.dat = S.sc + 32;
  X.wp.hdr = reinterpret_cast<int*>(X.wp.dat + WP_DBL);
  X.it0 = it0;
  const bool first = X.first;
  // a component whose step already ended in an earlier launch of this step (per-component stop,
  // host-stepped by piadmm_outer_iter) runs no further iteration: its state is only carried
  X.skip = !first && A.cst[(size_t)ci * 4 + 3] != 0;
  X.it_end = X.skip ? it0 : it1;
  // ---- seeds (casadi/main.py:48-49) and zero per-step state (:52-63)
  if ((int)threadIdx.x < na) {
    const int a = a0 + threadIdx.x;
    const double x = A.xt[3 * a], y = A.xt[3 * a + 1], th = A.xt[3 * a + 2], s = A.spd[a];
    S.xt[3 * threadIdx.x + 0] = x;
    S.xt[3 * threadIdx.x + 1] = y;
    S.xt[3 * threadIdx.x + 2] = th;
    const double sx = x + c.dt * s * cos(th), sy = y + c.dt * s * sin(th);
    S.seed[2 * threadIdx.x + 0] = around(sx, c.round_decimals);
    S.seed[2 * threadIdx.x + 1] = around(sy, c.round_decimals);
    double m;   // near ties of the seeds' rounding, logged once per step (the first launch)
    if (TIES && (flags & F_FIRST) && c.round_decimals >= 0 && round_near(sx, c.round_decimals, A.tie_tol, &m))
      tie_record(A, t, -1, PIADMM_TIE_ROUND_SEED, a, 0, m);
    if (TIES && (flags & F_FIRST) && c.round_decimals >= 0 && round_near(sy, c.round_decimals, A.tie_tol, &m))
      tie_record(A, t, -1, PIADMM_TIE_ROUND_SEED, a, 1, m);
  }
  for (int i = threadIdx.x; i < 32; i += blockDim.x) S.sc[i] = 0.0;
  {
    double* const edge_lds[5] = {S.hat, S.lam, S.S, S.D, S.last};
    double* const edge_hbm[5] = {A.hat, A.lam, A.Sacc, A.Dacc, A.last};
    if (first) {
      for (int i = threadIdx.x; i < 8 * H1; i += blockDim.x) S.pos[i] = 0.0;
      // casadi/main.py:52-63 resets hat, lam (and the PI accumulators) every MPC step; with
      // warm_duals they continue from the previous step shifted by one slot (a12)
      for (int k = 0; k < 5; ++k)
        for (int i = threadIdx.x; i < 4 * H1; i += blockDim.x) {
          double v = 0.0;
          if (e >= 0 && c.warm_duals) {
            const int r = i / H1, tt = i - r * H1;
            v = edge_hbm[k][(size_t)e * 4 * H1 + r * H1 + min(tt + 1, H)];
          }
          edge_lds[k][i] = v;
        }
    } else {
      // state of the previous launch of this step
      for (int i = threadIdx.x; i < 4 * H1; i += blockDim.x)
        S.pos[((it0 - 1) & 1) * 4 * H1 + i] = (i < na * 2 * H1) ? A.pos_old[(size_t)a0 * 2 * H1 + i] : 0.0;
      for (int i = threadIdx.x; i < na * H; i += blockDim.x) S.u[((it0 - 1) & 1) * 2 * H + i] = A.u[(size_t)a0 * H + i];
      for (int k = 0; k < 5; ++k)
        for (int i = threadIdx.x; i < 4 * H1; i += blockDim.x)
          edge_lds[k][i] = (e >= 0) ? edge_hbm[k][(size_t)e * 4 * H1 + i] : 0.0;
    }
  }
  __syncthreads();
  // pair safety distance (a13 tightening from the step's start states, else dis_thres)
  X.deff = c.dis_thres;
  if (e >= 0 && c.tighten && na == 2)
    X.deff = c.dis_thres + delay_norm(c, S.xt[2], A.spd[a0]) + delay_norm(c, S.xt[5], A.spd[a0 + 1]);
  X.thr = c.collide_sq_thres ? X.deff * X.deff : X.deff;
  X.resid = A.resid + ((size_t)slot * A.C + ci) * c.max_outer * 2;   // slot: step of the launch
  if (first)
    for (int i = threadIdx.x; i < 2 * c.max_outer; i += blockDim.x) X.resid[i] = NAN;   // "not evaluated"
  if (X.coop && ci == 0)
    for (int i = threadIdx.x; i < 2 * c.max_outer; i += blockDim.x) A.ghist[(size_t)slot * 2 * c.max_outer + i] = NAN;
  unsigned long long t_k = STAMP_T();

  LoopCtl L;
  L.flag = first ? 0 : A.cst[(size_t)ci * 4 + 0];
  L.aliased = first ? 0 : A.cst[(size_t)ci * 4 + 1];
  L.iters = X.skip ? A.iters[ci] : it0;
  L.gflag = 0;               // coop: some pair ever collided (casadi/main.py:115)
  L.stopped = X.skip;
  L.nanlast = (flags & F_NANLAST) != 0;
  L.act = (!first && e >= 0) ? A.edge_active[e] != 0 : false;
  L.dis_chk = (!first && e >= 0) ? A.dischk[e] : NAN;
  WaveCnt n;
  if (X.w < NW) agent_part<BIG, TIES, SH>(A, X, L, nbar, n);
  else if (X.w == PW) pair_part<BIG, TIES, SH>(A, X, L, nbar, n);
  else if constexpr (SH == 1) roll_part(A, X);
  else help_part<TIES>(A, X, L, nbar);
  __syncthreads();
  STAMP_ADD(ST_KERNEL, t_k);
  unsigned long long t_epi = STAMP_T();

  // ---- work counters (accumulated across launches; one workgroup owns row ci) and the
  // component's state of this launch (every launch)
  {
    __shared__ int s_cnt[NWA][8];
    __shared__ int s_warm;
    if (threadIdx.x == 0) s_warm = 0;
    if (X.l == 0) {
      s_cnt[X.w][0] = n.xqp; s_cnt[X.w][1] = n.zqp; s_cnt[X.w][2] = n.admm_x; s_cnt[X.w][3] = n.admm_z;
      s_cnt[X.w][4] = n.pdas_x; s_cnt[X.w][5] = n.pdas_z; s_cnt[X.w][6] = n.inexact; s_cnt[X.w][7] = 0;
    }
    __syncthreads();
    if (X.l == 0 && n.warm) atomicOr(&s_warm, X.w < NW ? (1 << X.w) : 4);
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long* cn = A.counters + (size_t)ci * 8;
      cn[0] += (unsigned long long)(X.skip ? 0 : L.iters - it0);
      const int nw = (int)(blockDim.x / WAVE);
      for (int k = 0; k < 6; ++k) {
        unsigned long long sum = 0;
        for (int ww = 0; ww < nw; ++ww) sum += (unsigned long long)s_cnt[ww][k];
        cn[k + 1] += sum;
      }
      unsigned long long inex = 0;
      for (int ww = 0; ww < nw; ++ww) inex += (unsigned long long)s_cnt[ww][6];
      cn[7] += inex;
      A.iters[ci] = L.iters;
      if (e >= 0) {
        A.edge_active[e] = L.act ? 1 : 0;
        A.dischk[e] = L.dis_chk;
      }
      A.cst[(size_t)ci * 4 + 0] = L.flag;
      A.cst[(size_t)ci * 4 + 1] = L.aliased;
      A.cst[(size_t)ci * 4 + 2] = s_warm;
      A.cst[(size_t)ci * 4 + 3] = L.stopped ? 1 : 0;
      if (X.coop && ci == 0) A.giters[slot] = L.iters;
      if (L.nanlast && L.iters > 0 && !X.skip) {   // global stop at the collision test of this iteration
        X.resid[2 * (L.iters - 1) + 0] = NAN;
        X.resid[2 * (L.iters - 1) + 1] = NAN;
      }
    }
  }
  if (e >= 0) {
    double* const edge_lds[5] = {S.hat, S.lam, S.S, S.D, S.last};
    double* const edge_hbm[5] = {A.hat, A.lam, A.Sacc, A.Dacc, A.last};
    for (int k = 0; k < 5; ++k)
      for (int i = threadIdx.x; i < 4 * H1; i += blockDim.x) edge_hbm[k][(size_t)e * 4 * H1 + i] = edge_lds[k][i];
  }
  STAMP_ADD(ST_RED_X, t_epi);
}

// Persistent multi-step launch (the reference's `for num_step` loop,
// casadi/main.py:43-201, on the device): each workgroup runs MPC steps t0 .. t0+nsteps-1 of
// its component back to back.  Components are independent whenever no step needs a
// job-wide decision (per-component termination, or fixed iterations), so a component never
// waits for the slowest one of each step: the launch takes max_c sum_t instead of
// sum_t max_c.  The step-to-step state (xt, labels, caches) goes through HBM inside one
// workgroup (same CU: the barrier's workgroup-scope fences order it).
template <bool BIG, bool TIES, int SH>
__global__ void __launch_bounds__(NWA * WAVE) k_mpc_step(DevArgs A, int t0, int nsteps, int it0, int it1, int flags) {
#ifdef PIADMM_STAMPS
  for (int i = threadIdx.x; i < 64 * STAMP_WAVES; i += blockDim.x) s_stamps[i] = 0ull;
  __syncthreads();
#endif
  if (flags & F_DEVSTOP) {      // device-decided global stop (uniform: every thread reads it)
    if (!(flags & F_LAST)) {
      if (A.gctl[0]) return;
    } else {
      it0 = it1 = A.gctl[2];
      if (A.gctl[1]) flags |= F_NANLAST;
    }
  }
  int nbar = 0;   // grid barriers so far (coop): parity of the termination partials
  for (int k = 0; k < nsteps; ++k) {
    mpc_step_body<BIG, TIES, SH>(A, t0 + k, it0, it1, flags, k, nbar);
    __syncthreads();
  }
#ifdef PIADMM_STAMPS
  if (g_stamps)
    for (int i = threadIdx.x; i < 64 * STAMP_WAVES; i += blockDim.x)
      atomicAdd(&g_stamps[(size_t)blockIdx.x * 64 * STAMP_WAVES + i], s_stamps[i]);
#endif
}

#ifndef PIADMM_SPEC_TU
// Global termination partials of outer iteration `it` (one workgroup of NW*WAVE threads):
// rk, sk summed over components, active pairs, pairs with a distance check, pairs failing it.
// The summation order is the in-kernel (cooperative) stop test's: thread k accumulates
// components k, k + NW*WAVE, ... in order, then the per-thread sums are added in thread order,
// so the host-decided / RCCL path and the single-rank in-kernel path take identical decisions.
__global__ void __launch_bounds__(NW * WAVE) k_term_partials(DevArgs A, int it, double* out, int devstop) {
  if (devstop && A.gctl[0]) return;
  constexpr int NT = NW * WAVE;
  __shared__ double red[5][NT];
  double v[5] = {0, 0, 0, 0, 0};
  for (int ci = threadIdx.x; ci < A.C; ci += NT) {
    const double* r = A.resid + ((size_t)ci * A.cfg.max_outer + it) * 2;
    const int e = A.comp_edge[ci];
    const double rk = r[0], sk = r[1];
    v[0] += (rk == rk) ? rk : 0.0;
    v[1] += (sk == sk) ? sk : 0.0;
    if (e >= 0) {
      v[2] += A.edge_active[e] ? 1.0 : 0.0;
      const double d = A.dischk[e];
      if (d == d) {
        v[3] += 1.0;
        v[4] += (d > A.deff[e]) ? 0.0 : 1.0;
      }
    }
  }
  for (int k = 0; k < 5; ++k) red[k][threadIdx.x] = v[k];
  __syncthreads();
  if (threadIdx.x < 5) {
    double tot = 0.0;
    for (int k = 0; k < NT; ++k) tot += red[threadIdx.x][k];
    out[threadIdx.x] = tot;
  }
}

// Residual history of a fixed-iteration step summed over components: out[it] = (rk, sk).
__global__ void __launch_bounds__(256) k_resid_history(DevArgs A, double* out) {
  const int it = blockIdx.x;
  const int slot = blockIdx.y;                 // step of the multi-step launch
  out += (size_t)slot * 2 * A.cfg.max_outer;
  __shared__ double red[2][256];
  double rk = 0.0, sk = 0.0;
  for (int ci = threadIdx.x; ci < A.C; ci += 256) {
    const double* r = A.resid + (((size_t)slot * A.C + ci) * A.cfg.max_outer + it) * 2;
    if (r[0] == r[0]) rk += r[0];
    if (r[1] == r[1]) sk += r[1];
  }
  red[0][threadIdx.x] = rk;
  red[1][threadIdx.x] = sk;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * it + 0] = red[0][0];
    out[2 * it + 1] = red[1][0];
  }
}

// Safety distance per pair for the partials (the kernel recomputes it per launch).
__global__ void k_pair_deff(DevArgs A) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= A.E) return;
  const piadmm_config_t& c = A.cfg;
  const int v1 = A.edges[2 * e], v2 = A.edges[2 * e + 1];
  double d = c.dis_thres;
  if (c.tighten)
    d = c.dis_thres + delay_norm(c, A.xt[3 * v1 + 2], A.spd[v1]) + delay_norm(c, A.xt[3 * v2 + 2], A.spd[v2]);
  A.deff[e] = d;
}

#endif

// The kernel instantiations: matrices in LDS / HBM (BIG); the near-tie log compiled in or out (TIES:
// the log costs 3-10 % of the fused kernel's time, so it is a separate instantiation, on when a handle
// asks for it); and the loop shape (SH: 0 plain, 1 speculative).  The two shapes are separate kernels
// in separate translation units (this file; piadmm_device_spec.hip includes it with PIADMM_SPEC_TU):
// each kernel holds one loop shape, so the register allocation of one shape's hot loops is not shaped
// by the other's code, and the two compile in parallel.
#ifdef PIADMM_SPEC_TU
const void* mpc_fn_spec(bool big, bool ties) {
  if (big) return ties ? (const void*)k_mpc_step<true, true, 1> : (const void*)k_mpc_step<true, false, 1>;
  return ties ? (const void*)k_mpc_step<false, true, 1> : (const void*)k_mpc_step<false, false, 1>;
}
#ifdef PIADMM_STAMPS
int spec_set_stamps(unsigned long long* p) {     // this translation unit's copy of g_stamps
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(void*)) == hipSuccess ? 0 : -1;
}
#endif
#else
const void* mpc_fn_spec(bool big, bool ties);    // piadmm_device_spec.hip
#ifdef PIADMM_STAMPS
int spec_set_stamps(unsigned long long* p);
#endif
static const void* mpc_fn(bool big, bool ties, bool spec) {
  if (spec) return mpc_fn_spec(big, ties);
  if (big) return ties ? (const void*)k_mpc_step<true, true, 0> : (const void*)k_mpc_step<true, false, 0>;
  return ties ? (const void*)k_mpc_step<false, true, 0> : (const void*)k_mpc_step<false, false, 0>;
}

// The speculative loop shape wherever there is no in-kernel grid barrier (F_COOP) and not
// PIADMM_NO_SPEC=1 (DevArgs::no_spec, the plain loop everywhere).  With the compact steady-state
// loops it pays for both position models -- measured (iteration slope, tools/iter_slope.py):
// matlab_pi 256 x H30 (nonlinear sincos rollout) and casadi_default 64 x H20 (linearised rollout)
// 4.6k -> 3.3k cycles per outer iteration, configs[1] fixed 0.469 -> 0.377 ms per step.
static bool spec_shape(const DevArgs& a, int flags) {
  return !(flags & F_COOP) && !(flags & F_NOSPEC) && a.no_spec == 0;
}

int launch_mpc_step(const DevArgs& a, int t, int nsteps, int it0, int it1, int flags, hipStream_t s) {
  const size_t sh = lds_bytes(a.cfg.H, a.cfg.precision);
  const bool big = a.cfg.H > HMAX;
  const bool spec = spec_shape(a, flags);
#ifdef PIADMM_STAMPS
  static unsigned long long* last = nullptr;
  if (a.stamps != last) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &a.stamps, sizeof(void*)) != hipSuccess) return -1;
    if (spec_set_stamps(a.stamps) != 0) return -1;
    last = a.stamps;
  }
#endif
  const void* fn = mpc_fn(big, a.tie_on != 0, spec);
  if (set_dyn_lds(fn, sh) != 0) return -1;
  // the fourth wave: the speculative shape's roller, and in LDS mode up to WPIPE_HMAX the helper
  // that builds the pair's warm rows beside it (both shapes; PIADMM_NO_HELPER=1 leaves it out)
  const char* nh = std::getenv("PIADMM_NO_HELPER");     // (read per launch: the tests' A/B toggles it)
  const bool no_helper = nh && nh[0] == '1';
  if (no_helper) flags |= F_NOHELPER;
  const bool helper = !big && a.cfg.H <= WPIPE_HMAX && !no_helper;
  if (flags & F_COOP) {
    // every workgroup must be resident for the grid barrier: the cooperative launch fails
    // (and the caller falls back to host-decided termination) rather than deadlock
    DevArgs aa = a;
    aa.gbar_base = launch_coop_epoch(nsteps, a.cfg.max_outer);
    void* args[] = {&aa, &t, &nsteps, &it0, &it1, &flags};
    (void)hipGetLastError();
    return launch_rc(hipLaunchCooperativeKernel(fn, dim3(a.C), dim3((helper ? NWA : NWT) * WAVE), args, (unsigned)sh, s));
  }
  (void)hipGetLastError();   // a stale error of an earlier runtime call is not this launch's
  // the speculative loop runs with the roller wave; PIADMM_NO_ROLLER=1 keeps three waves (the pair
  // wave rolls both agents out)
  static const bool no_roller = [] {
    const char* e = std::getenv("PIADMM_NO_ROLLER");
    return e && e[0] == '1';
  }();
  const int nt = ((spec ? !no_roller : helper) ? NWA : NWT) * WAVE;
  DevArgs aa = a;
  void* args[] = {&aa, &t, &nsteps, &it0, &it1, &flags};
  return launch_rc(hipLaunchKernel(fn, dim3(a.C), dim3(nt), args, sh, s));
}

unsigned long long launch_coop_epoch(int nsteps, int max_outer) {
  static std::atomic<unsigned long long> next{0};
  const unsigned long long span = (unsigned long long)std::max(nsteps, 1) * (unsigned long long)(std::max(max_outer, 1) + 2) + 2;
  return next.fetch_add(span);
}

// Can every workgroup of a k_mpc_step launch be resident at once (cooperative launch)?
bool coop_fits(const DevArgs& a, int device) {
  int coopok = 0, ncu = 0, per = 0;
  if (hipDeviceGetAttribute(&coopok, hipDeviceAttributeCooperativeLaunch, device) != hipSuccess || !coopok)
    return false;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return false;
  const size_t sh = lds_bytes(a.cfg.H, a.cfg.precision);
  const bool big = a.cfg.H > HMAX;
  const void* fn = mpc_fn(big, a.tie_on != 0, false);   // (the cooperative launch runs the plain shape)
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, NWA * WAVE, sh) != hipSuccess) return false;
  return (long long)per * ncu >= (long long)a.C;
}

// The dynamic-LDS limit is a per-device function attribute: set once per (kernel, device), and
// again only for a larger size, so handles on several devices of one process each get it.
int set_dyn_lds(const void* fn, size_t bytes) {
  static std::mutex mu;
  static std::vector<std::tuple<const void*, int, size_t>> done;
  int dev = 0;
  if (launch_rc(hipGetDevice(&dev)) != 0) return -1;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& d : done)
    if (std::get<0>(d) == fn && std::get<1>(d) == dev && std::get<2>(d) >= bytes) return 0;
  if (launch_rc(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes)) != 0) return -1;
  done.emplace_back(fn, dev, bytes);
  return 0;
}

__global__ void k_copy(double* __restrict__ dst, const double* __restrict__ src, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int launch_copy(double* dst, const double* src, size_t n, hipStream_t s) {
  if (n == 0 || dst == src) return 0;
  const unsigned nb = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_copy, dim3(nb), dim3(256), 0, s, dst, src, n);
  return launch_rc(hipGetLastError());
}

int launch_term_partials(const DevArgs& a, int it, double* out, hipStream_t s, int devstop) {
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_term_partials, dim3(1), dim3(NW * WAVE), 0, s, a, it, out, devstop);
  return launch_rc(hipGetLastError());
}

// The reference's stop rules over the job (casadi/main.py:115-118,174-178; MATLAB :191-210) on
// the all-reduced partials of outer iteration `it`, decided on the device (F_DEVSTOP): the same
// rules as the host decision in piadmm_capi.cpp global_iteration.  gctl: [0] stop, [1] the stop
// came at the collision test (NANLAST), [2] iterations executed, [3] some pair ever collided.
__global__ void k_decide(DevArgs A, int t, int it, const double* part) {
  int* g = A.gctl;
  if (g[0]) return;
  const piadmm_config_t& c = A.cfg;
  const double rk = part[0], sk = part[1], n_act = part[2], n_seen = part[3], n_bad = part[4];
  g[2] = it + 1;
  if (n_act == 0.0 && g[3] == 0 && !c.fixed_iters) {
    g[1] = 1;
    g[0] = 1;
    return;
  }
  g[3] = 1;
  A.ghist[2 * it + 0] = rk;
  A.ghist[2 * it + 1] = sk;
  if (A.tie_on && !c.fixed_iters) {
    scalar_tie(A, t, it, PIADMM_TIE_STOP, -1, 0, rk, c.eps_pri);
    scalar_tie(A, t, it, PIADMM_TIE_STOP, -1, 1, sk, c.eps_dual);
  }
  if (!c.fixed_iters && rk <= c.eps_pri && sk <= c.eps_dual && (!c.term_dist_check || (n_seen > 0.0 && n_bad == 0.0)))
    g[0] = 1;
}

int launch_decide(const DevArgs& a, int t, int it, const double* part, hipStream_t s) {
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_decide, dim3(1), dim3(1), 0, s, a, t, it, part);
  return launch_rc(hipGetLastError());
}

int launch_resid_history(const DevArgs& a, int nsteps, double* out, hipStream_t s) {
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_resid_history, dim3(a.cfg.max_outer, nsteps), dim3(256), 0, s, a, out);
  return launch_rc(hipGetLastError());
}

int launch_pair_deff(const DevArgs& a, hipStream_t s) {
  if (a.E == 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_pair_deff, dim3((a.E + 255) / 256), dim3(256), 0, s, a);
  return launch_rc(hipGetLastError());
}

#endif  // PIADMM_SPEC_TU

}  // namespace pd
