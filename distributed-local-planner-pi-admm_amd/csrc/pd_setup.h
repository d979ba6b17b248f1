// pd_setup.h -- per-step QP setup of libpiadmm: Ruiz scaling, the x-step QP of an agent
// and the pair (z-step) QP of a candidate pair, and the delay-tightening offset.
#pragma once
#include "pd_qp.h"

namespace pd {

// ============================================================ per-step setup
// Ruiz equilibration of [P A'; A 0] (OSQP-style, RUIZ_ITERS sweeps): fills P.D and P.E.
template <int NV>
__device__ __forceinline__ void ruiz(QP<NV>& P) {
  constexpr int NR = QP<NV>::NR;
  const int l = lid(), H = P.H;
  const bool in = l < H;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    P.D[v] = in ? 1.0 : 0.0;
    P.E[2 * v] = in ? 1.0 : 0.0;
    P.E[2 * v + 1] = (l < H - 1) ? 1.0 : 0.0;
  }
  if constexpr (NV == 2) P.E[4] = P.valid(4) ? 1.0 : 0.0;
  const double ag[2] = {fabs(P.g1), fabs(P.g2)};
  for (int it = 0; it < RUIZ_ITERS; ++it) {
    double cn[NV], rn[NR];
#pragma unroll
    for (int v = 0; v < NV; ++v) cn[v] = 0.0;
    double rh = 0.0;
    for (int i = 0; i < H; ++i) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const double Di = rdl(P.D[v], i);
        if (in) cn[v] = fmax(cn[v], fabs(Di * P_entry(P, v, i, l) * P.D[v]));
        if constexpr (NV == 2) {
          const double Ehi = rdl(P.E[4], i);
          // hinge row i (time i+1): entry g_v (i - j)+ on variable j of vehicle v
          if (in && i > l) cn[v] = fmax(cn[v], Ehi * ag[v] * (double)(i - l) * P.D[v]);
          if (in && i < l) rh = fmax(rh, ag[v] * (double)(l - i) * Di);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const double Eb = P.E[2 * v], Er = P.E[2 * v + 1];
      cn[v] = fmax(cn[v], fmax(Eb * P.D[v], fmax(Er * P.D[v], shup(Er, 1) * P.D[v])));
      rn[2 * v] = Eb * P.D[v];
      rn[2 * v + 1] = Er * fmax(P.D[v], shdn(P.D[v], 1));
    }
    if constexpr (NV == 2) rn[4] = rh * P.E[4];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (in) {
        P.D[v] *= 1.0 / sqrt(clamp_norm(cn[v]));
        P.E[2 * v] *= 1.0 / sqrt(clamp_norm(rn[2 * v]));
      }
      if (l < H - 1) P.E[2 * v + 1] *= 1.0 / sqrt(clamp_norm(rn[2 * v + 1]));
    }
    if constexpr (NV == 2) {
      if (P.valid(4)) P.E[4] *= 1.0 / sqrt(clamp_norm(rn[4]));
    }
  }
}

struct WaveMem {
  double* vb;
  int* ib;
};

__device__ __forceinline__ void qp_common(const piadmm_config_t& c, int H, double rho0, QP<1>& P) {
  P.H = H;
  P.n = H;
  P.umax = c.u_max;
  P.dumax = c.du_max;
  P.h0 = 0.0;
  P.g1 = P.g2 = 0.0;
  P.Pcost2 = 2.0 * c.Pcost;
  P.beta = 0.0;
  P.rho = rho0;
  P.sigma = c.admm_sigma;
  P.alpha = c.admm_alpha;
  P.tol = c.qp_tol;
  P.kready = true;      // setup_agent loads or builds K_s^-1
  P.scaled = true;
  P.wraw = false;
  P.Kcache = nullptr;
  P.csig = -1;
}

// x-step QP of agent a (cost_function_primal, PI_ADMM_class.py:114-135, constraints :172-192):
// scaling, K_s^-1 (LDS) and P^-1 (LDS) for the whole MPC step.
// coef >= 0: the P coefficient of M'M (global PI: 2 Pnorm + sum of the pairs' penalties), part of
// the cache key.  Returns true when the caches were rebuilt (the parametric tables are stale).
__device__ __forceinline__ bool setup_agent(const DevArgs& A, int a, QP<1>& P, const Geo& g, double* xfac,
                                            double coef = -1.0) {
  const piadmm_config_t& c = A.cfg;
  const int H = P.H, l = lid();   // (qp_common set P.H: a constant in the compiled-in horizon kernels)
  const bool in = l < H;
  P.coefP = coef >= 0.0 ? coef : 2.0 * c.Pnorm + c.rho * (double)A.nbr_cnt[a];
  P.mm[0] = g.mm;
  double* Kc = A.Kx_cache + (size_t)a * H * H;
  double* Pc = A.Pinv_x + (size_t)a * H * H;
  double* sc = A.sc_x + (size_t)a * 4 * HCAP;
  const int li = l < HCAP ? l : 0;
  // P depends on the agent's speed only (make_geo): K_s^-1, P^-1 and the scaling are
  // cached in HBM per scenario and rebuilt only when the ADMM penalty differs.
  if (__builtin_expect(A.xcache_rho[a] == P.rho && (!A.xcache_coef || A.xcache_coef[a] == P.coefP), 1)) {
    P.D[0] = in ? sc[li] : 0.0;
    P.E[0] = in ? sc[HCAP + li] : 0.0;
    P.E[1] = (l < H - 1) ? sc[2 * HCAP + li] : 0.0;
    if (P.kf32 || P.K != Kc) {   // LDS image of K_s^-1: loaded by qp_solve when ADMM is needed
      P.Kcache = Kc;
      P.kready = false;
    }
    wsync();
    return false;
  }
  ruiz(P);
  build_K<1, false>(P, xfac, P.fld, Kc);
  P.Kcache = Kc;        // the same matrix: a later reload (after the x-step's dual active set) is a copy
  for (int i = 0; i < H; ++i)
    if (in) xfac[i * P.fld + l] = P_entry(P, 0, i, l);
  wsync();
  gj_invert(xfac, H, P.fld);
  for (int i = 0; i < H; ++i) {
    if (in) {
      Pc[i * H + l] = xfac[i * P.fld + l];
    }
  }
  if (l < HCAP) {
    sc[0 * HCAP + l] = P.D[0];
    sc[1 * HCAP + l] = P.E[0];
    sc[2 * HCAP + l] = P.E[1];
  }
  if (l == 0) {
    A.xcache_rho[a] = P.rho;
    if (A.xcache_coef) A.xcache_coef[a] = P.coefP;
  }
  __threadfence();      // P^-1 (read back through L2 by the polish) is visible to this wave
  wsync();
  return true;
}

// Pair (z-step) QP of cost_function_edge (PI_ADMM_class.py:145-169), heading frozen at
// xt (MATLAB symbolic dynamic_update_edge, ADMM_CVX_..._PI_antiwindup.m:378-397).
// Variables [uh_1; uh_2]; hinge rows G_k = [g1 T(k+1,.), g2 T(k+1,.)],
// h_k = D^2 + |dbar|^2 - 2 dbar'(c2 - c1)_{k+1}.  Builds the polish tables P^-1 (HBM),
// PGt = P^-1 G' (HBM), GPG = G P^-1 G' (HBM) and K_s^-1 (LDS).
__device__ __forceinline__ void setup_pair(const DevArgs& A, int e, QP<2>& P, const Geo& g1, const Geo& g2,
                                           double c1x, double c1y, double c2x, double c2y, const double* seeds,
                                           double* scr, double* Ke_lds, double deff, double rho_pair = -1.0) {
  const piadmm_config_t& c = A.cfg;
  const int H = P.H, n = 2 * H, l = lid();   // (set by the caller)
  const bool in = l < H;
  unsigned long long t_pre = STAMP_T();
  const double dbx = seeds[2] - seeds[0], dby = seeds[3] - seeds[1];
  const double dd = dbx * dbx + dby * dby;
  P.g1 = -2.0 * (dbx * g1.ax + dby * g1.ay);
  P.g2 = 2.0 * (dbx * g2.ax + dby * g2.ay);
  const double Dsq = deff * deff;
  const double h_time = Dsq + dd - 2.0 * (dbx * (c2x - c1x) + dby * (c2y - c1y));
  P.h0 = shdn(h_time, 1);                    // hinge lane k <-> time k+1
  if (!P.valid(4)) P.h0 = 0.0;
  P.coefP = rho_pair >= 0.0 ? rho_pair : c.rho;
  P.mm[0] = g1.mm;
  P.mm[1] = g2.mm;

  // ---- P_v^-1 blocks (HBM), Y = P_v^-1 T' (PGt, unscaled by g) and Z_v = T P_v^-1 T' (GPG):
  // speed-only, so built once per scenario; g1, g2 scale them on the fly (s_gather, x recovery)
  if (__builtin_expect(!A.ecache[e] || (A.ecache_rho && A.ecache_rho[e] != P.coefP), 0)) {
    double* Yl = Ke_lds;             // H x n staging (the Ke region is rebuilt below)
    double* Pi = A.tab_e + (size_t)e * 8 * H * H;
    for (int v = 0; v < 2; ++v) {
      for (int i = 0; i < H; ++i)
        if (in) scr[i * LD + l] = P_entry(P, v, i, l);
      wsync();
      gj_invert(scr, H, LD);
      for (int i = 0; i < H; ++i) {
        if (in) {
          Pi[(v * H + i) * n + v * H + l] = scr[i * LD + l];
          Pi[(v * H + i) * n + (1 - v) * H + l] = 0.0;
        }
      }
      // lane i: Y_k = sum_{j<=k-1} (k-j) Pinv_v[i][j]
      double acc1 = 0.0, Y = 0.0;
      for (int k = 0; k < H; ++k) {
        if (in) Yl[k * n + v * H + l] = Y;
        if (in) acc1 += scr[l * LD + k];
        Y += acc1;
      }
      if (P.gmem) gsync();      // big mode: the staging is in HBM
      else wsync();
    }
    double* Pg = Pi + 4 * H * H;
    double* Zg = Pi + 6 * H * H;
    const int b = in ? l : 0;
    for (int v = 0; v < 2; ++v) {
      double B = 0.0, Z = 0.0;
      for (int a = 0; a < H; ++a) {
        if (in) Zg[v * H * H + a * H + l] = Z;
        B += Yl[b * n + v * H + a];
        Z += B;
      }
    }
    for (int k = 0; k < H; ++k)
      for (int col = l; col < n; col += WAVE) Pg[k * n + col] = Yl[k * n + col];
    if (l == 0) {
      A.ecache[e] = 1;
      if (A.ecache_rho) A.ecache_rho[e] = P.coefP;
    }
    gsync();                    // the tables are read back through L2 by the polish
  }
  STAMP_ADD(ST_SZ_PRE, t_pre);
  // identity scaling: the dual active set and the polish work unscaled; the Ruiz
  // equilibration of the ADMM space is computed by qp_solve only when ADMM is needed
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    P.D[v] = in ? 1.0 : 0.0;
    P.E[2 * v] = in ? 1.0 : 0.0;
    P.E[2 * v + 1] = (l < H - 1) ? 1.0 : 0.0;
  }
  P.E[4] = P.valid(4) ? 1.0 : 0.0;
  P.scaled = false;
  P.wraw = false;
  P.Kcache = nullptr;
  P.kready = false;     // K_s^-1 is built by qp_solve when ADMM is first needed
}

// Delay offset |delta| of compute_square_halfspaces_ca_prob (decentralized/util.py:81-96) for
// an agent with heading th and speed s (oracle delay_offset).
__device__ __forceinline__ double delay_norm(const piadmm_config_t& c, double th, double s) {
#pragma clang fp contract(off)
  const double cs = cos(th), sn = sin(th);
  const double dxa = c.avg_delay * s * cs, dya = c.avg_delay * s * sn;
  const double dxv = (c.var_delay * s * cs) * (c.var_delay * s * cs);
  const double dyv = (c.var_delay * s * sn) * (c.var_delay * s * sn);
  const double kap = sqrt(c.tight_p / (1.0 - c.tight_p));
  return hypot(dxa + kap * dxv, dya + kap * dyv);
}

}  // namespace pd
