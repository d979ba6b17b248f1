// pd_qp.h -- the per-wave QP solver of libpiadmm: generalised QP with box / rate / hinge
// rows, OSQP-style ADMM in a Ruiz-scaled space, PDAS polish on the reduced KKT system,
// parametric x-step tables and the Goldfarb-Idnani dual active set (not part of the ABI).
#pragma once
#include "pd_common.h"

namespace pd {

// ============================================================ QP solver
// Generalised QP  min 1/2 x'Px + q'x + sum_r phi_r(a_r'x)  with box rows
// (indicator of [lo,hi]) and, for the pair, hinge rows beta*max(0, h - a'x).
//   x-step (NV=1): P = coefP*mm*T'T + 2 D2'D2 + 2 Pcost I          (PI_ADMM_class.py:114-135)
//   pair   (NV=2): P = blockdiag(rho*mm_v*T'T + 2 Pcost I)          (PI_ADMM_class.py:145-169)
template <int NV>
struct QP {
  static constexpr int NR = (NV == 1) ? 2 : 5;
  int H, n;
  double q[NV];
  double wq;              // x-step: w' with q = T'-apply(w') (PI_ADMM_class.py:114-135 gradient)
  bool qvalid;            // q holds T'-apply(wq) (the x-step's fused pass needs only wq)
  double D[NV];
  double E[NR];
  double h0;              // hinge lower bound (pair only; 0 on invalid lanes)
  double umax, dumax;     // box / rate bounds (uniform)
  double g1, g2;          // hinge coefficients (pair only)
  double mm[NV];          // |M|^2 factors (ax^2 + ay^2) per vehicle
  double coefP;           // x-step: 2 Pnorm + rho |N| ; pair: rho
  double Pcost2;          // 2 Pcost
  double beta, rho, sigma, alpha, tol;
  double* K;              // LDS  n x n  scaled (P_s + sigma I + rho A_s'A_s)^-1
  float* Kf;              // precision 1: the same matrix in fp32 (what the ADMM iteration reads)
  bool kf32;              // ADMM reads Kf (the polish and its certificate stay fp64)
  const double* Pinv;     // n x n unscaled P^-1 (LDS for the x-step); for the pair the HBM
                          // table block DevArgs::tab_e: P^-1 | PGt (+4H^2) | GPG (+6H^2)
  double* vb;             // per-wave LDS vectors (512 doubles)
  double* XT;             // x-step: per-wave X' (H rows, stride xld) and beta (row H)
  int xld;                // stride of XT (XLD in LDS mode, XLDG in big mode)
  bool gmem;              // big mode: K / G / XT live in HBM (cross-lane reads need a fence)
  double* G;              // x-step: per-wave LDS G = P^-1 - Y X (H x H, stride H), g = Y beta (row H)
  double* fac;            // LDS factor region: L (lower), S (upper), stride fld
  double* fdiag;          // LDS [2*64]: S_aa, 1/L_aa of the cached factor
  int* ib;                // per-wave LDS ints: [0,64) current W ids, [64,128) cached W ids
  int* fstate;            // LDS int: m of the cached factor (-1: none)
  int fld;                // stride of fac
  int mmax;               // capacity of fac (rows)
  bool kready;            // K holds K_s^-1 for the current rho (the pair builds it lazily:
                          // a QP that the warm-label polish certifies never needs it)
  double* Y;              // pair: dual active-set columns P^-1 n_a (shares the K_s^-1 region)
  int ycap;               // pair: columns Y holds
  bool y_in_k;            // Y shares the K_s^-1 region (a GI solve invalidates K_s^-1)
  int yld = GYLD;         // row stride of the transposed Y (gi_solve RM_Y; even, >= ycap)
  bool scaled;            // Ruiz scaling computed (the pair computes it only when ADMM is needed)
  bool wraw;              // the warm ADMM state holds the last certified (x, y) unscaled (zs unset):
                          // converted to the scaled (xs, zs, ys) only when ADMM actually runs
  const double* Kcache;   // x-step: HBM copy of K_s^-1, loaded into K only when ADMM is needed
  mutable int csig;       // x-step: per-lane working-set signature of the cached X', G
  int* gws;               // pair: HBM warm working set of the dual active set (GI_WS ints)
  bool gws_warm = true;   // pair: start from the stored set (false: cold start, the set is still saved)
  int tstep;              // MPC step index (warm-set bookkeeping)
  int pre_m = -1;         // pair: rows of the stored active set already appended (gi_solve prebuild), -1: none
  int pre_wbits = 0;
  bool pre_lin = false;   // pair, restored active set (gi_snap_restore): this lane's hinge regime (linear)
  double* wide = nullptr; // pair: HBM scratch of the wide dual active set (gi_solve_wide), nullptr: none
  double* snap = nullptr; // pair (graph kernel): HBM snapshot of the last dual active set's S^-1 and Y
                          // columns, written with gws (gi_snap_restore), nullptr: none
  bool gi_full = false;   // pair: the last gi_solve stopped at its working-set capacity
  float* t32 = nullptr;   // x-step, precision 2 (tables in HBM): fp32 copies of the UNFOLDED G (H x H) and
                          // X' (H rows, stride XLDG) -- the hit path's tables, refined once in fp64

  __device__ __forceinline__ bool hinge(int s) const { return NV == 2 && s == 4; }
  // Row s of vehicle v = s / 2: even = box (lanes < H), odd = rate (lanes < H-1), 4 = hinge
  // (lanes 1..H-1 when the pair's geometry couples them).  Bounds are recomputed, not stored,
  // to keep the per-lane register state of the two live QPs small.
  __device__ __forceinline__ bool valid(int s) const {
    const int l = lid();
    if (hinge(s)) return l >= 1 && l < H && (g1 != 0.0 || g2 != 0.0);
    return (s & 1) ? l < H - 1 : l < H;
  }
  __device__ __forceinline__ double lo(int s) const { return hinge(s) ? h0 : ((s & 1) ? -dumax : -umax); }
  __device__ __forceinline__ double hi(int s) const { return hinge(s) ? INFINITY : ((s & 1) ? dumax : umax); }
};

template <int NV>
__device__ constexpr int NR_HINGE() { return NV == 2 ? 4 : 0; }

// Hinge rows sit at their kink at most optima (beta = 1000 makes them near-equalities);
// like OSQP's larger rho on equality rows they get HINGE_RHO x rho (tools/qp_sim.py sweep:
// pair-QP ADMM iterations mean 29.6 -> 20.3, max 880 -> 295).
constexpr double HINGE_RHO = 3.0;
template <int NV>
__device__ __forceinline__ double rrow(const QP<NV>& P, int s) { return P.hinge(s) ? P.rho * HINGE_RHO : P.rho; }

// Unscaled P x (var lanes), matrix-free: T'T via two double scans, D2'D2 via neighbours.
template <int NV>
__device__ __forceinline__ void P_mul(const QP<NV>& P, const double* x, double* px) {
  const bool in = lid() < P.H;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double tx = T_apply(x[v]);
    const double tt = Tt_apply(in ? tx : 0.0);       // T rows live on hinge lanes < H only
    double r = P.coefP * P.mm[v] * tt + P.Pcost2 * x[v];
    if constexpr (NV == 1) {
      // (D2 x)_r = x_r - 2 x_{r+1} + x_{r+2}, r <= H-3 ; (D2' w)_j = w_j - 2 w_{j-1} + w_{j-2}
      const double d2 = (lid() <= P.H - 3) ? x[v] - 2.0 * shdn(x[v], 1) + shdn(x[v], 2) : 0.0;
      r += 2.0 * (d2 - 2.0 * shup(d2, 1) + shup(d2, 2));
    }
    px[v] = in ? r : 0.0;
  }
}

// Build K_s = D P D + sigma I + rho A_s'A_s in LDS scratch m (stride ld, lane = column),
// invert it in place and copy it to P.K (stride n).
template <int NV>
__device__ __forceinline__ double P_entry(const QP<NV>& P, int v, int i, int j) {
  const double mmv = (NV == 2 && v) ? P.mm[NV - 1] : P.mm[0];
  double e = P.coefP * mmv * TT(i, j, P.H) + (i == j ? P.Pcost2 : 0.0);
  if constexpr (NV == 1) e += 2.0 * D2D2(i, j, P.H);
  return e;
}

// TWO: the pair beyond H = 32 (n > 64), lane l owning columns l and l + 64 (big mode only,
// a separate instantiation so the LDS-mode kernel carries none of it).
template <int NV, bool TWO>
__device__ __forceinline__ void build_K(QP<NV>& P, double* m, int ld, double* kcache = nullptr) {
  unsigned long long t_km = STAMP_T();
  const int l = lid();
  const int H = P.H, n = P.n;
  constexpr int ncol = TWO ? 2 : 1;
  int vc[ncol], jc[ncol];
  double Dc[ncol], gc[ncol];
#pragma unroll
  for (int cc = 0; cc < ncol; ++cc) {
    const int col = l + WAVE * cc;
    vc[cc] = (NV == 2 && col >= H) ? 1 : 0;
    jc[cc] = col - vc[cc] * H;
    const int src = (jc[cc] >= 0 && jc[cc] < H) ? jc[cc] : 0;
    double Dsh[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) Dsh[v] = __shfl(P.D[v], src);
    Dc[cc] = (NV == 2 && vc[cc] == 1) ? Dsh[NV - 1] : Dsh[0];
    gc[cc] = (vc[cc] == 0) ? P.g1 : P.g2;
  }
  // hinge block of A_s'A_s: sum_{k > max(i,j)} e2_k (k-i)(k-j) = S2 - (i+j) S1 + i j S0 with
  // suffix sums S0..S2 of e2_k k^0..2 taken at lane max(i,j)+1 (one bpermute each per row)
  double hS0 = 0.0, hS1 = 0.0, hS2 = 0.0;
  if constexpr (NV == 2) {
    const double Eh2 = P.valid(NR_HINGE<NV>()) ? P.E[NR_HINGE<NV>()] * P.E[NR_HINGE<NV>()] : 0.0;
    const double kd = (double)l;
    hS0 = scan_incl_rev(Eh2);
    hS1 = scan_incl_rev(Eh2 * kd);
    hS2 = scan_incl_rev(Eh2 * kd * kd);
  }
  for (int r = 0; r < n; ++r) {
    const int vr = (NV == 2 && r >= H) ? 1 : 0;
    const int ir = r - vr * H;
    double Dr, Ebr, Err, Errm;
    if (NV == 2 && vr) {
      Dr = rdl(P.D[NV - 1], ir);
      Ebr = rdl(P.E[(2 * NV - 2) % QP<NV>::NR], ir);
      Err = rdl(P.E[(2 * NV - 1) % QP<NV>::NR], ir);
      Errm = (ir >= 1) ? rdl(P.E[(2 * NV - 1) % QP<NV>::NR], ir - 1) : 0.0;
    } else {
      Dr = rdl(P.D[0], ir);
      Ebr = rdl(P.E[0], ir);
      Err = rdl(P.E[1], ir);
      Errm = (ir >= 1) ? rdl(P.E[1], ir - 1) : 0.0;
    }
    for (int cc = 0; cc < ncol; ++cc) {
      const int col = l + WAVE * cc;
      double hs = 0.0;
      if constexpr (NV == 2) {
        const double gr = (vr == 0) ? P.g1 : P.g2;
        const int M = max(ir, jc[cc]) + 1;
        const int ms = (M < H) ? M : 0;
        const double s0 = __shfl(hS0, ms), s1 = __shfl(hS1, ms), s2 = __shfl(hS2, ms);
        if (M < H) hs = s2 - (double)(ir + jc[cc]) * s1 + (double)ir * (double)jc[cc] * s0;
        hs *= gr * gc[cc] * HINGE_RHO;
      }
      if (col < n) {
        double ata = hs, v = 0.0;
        if (vr == vc[cc]) {
          v = Dr * P_entry(P, vr, ir, jc[cc]) * Dc[cc];
          if (ir == jc[cc]) ata += Ebr * Ebr + Err * Err + Errm * Errm;
          else if (jc[cc] == ir + 1) ata += -Err * Err;
          else if (jc[cc] == ir - 1) ata += -Errm * Errm;
        }
        v += P.rho * Dr * Dc[cc] * ata + (r == col ? P.sigma : 0.0);
        m[r * ld + col] = v;
      }
    }
  }
  wsync();
  if (NV == 2) STAMP_ADD(ST_SZ_KMAT, t_km);
  unsigned long long t_gj = STAMP_T();
  if (P.gmem && m == P.K) gsync();
  if constexpr (TWO) gj_invert2(m, n, ld, P.gmem && m == P.K);
  else gj_invert(m, n, ld);
  if (NV == 2) STAMP_ADD(ST_SZ_GJ, t_gj);
  // copies: the fp64 matrix (unless built in place), its fp32 image (precision 1) and the
  // per-scenario HBM cache (x-step); lane = column, up to two columns per lane
  for (int col = l; col < n; col += WAVE) {
    for (int r = 0; r < n; ++r) {
      const double v = m[r * ld + col];
      if (P.kf32) P.Kf[r * n + col] = (float)v;
      else if (m != P.K) P.K[r * n + col] = v;
      if (kcache) kcache[r * n + col] = v;
    }
  }
  if (P.gmem || kcache) gsync();
  else wsync();
}
template <int NV>
__device__ __forceinline__ void A_mul(const QP<NV>& P, const double* x, double* ax) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double xn = shdn(x[v], 1);
    ax[2 * v] = P.valid(2 * v) ? x[v] : 0.0;
    ax[2 * v + 1] = P.valid(2 * v + 1) ? xn - x[v] : 0.0;
  }
  if constexpr (NV == 2) {
    const double th = T_apply(P.g1 * x[0] + P.g2 * x[1]);
    ax[4] = P.valid(4) ? th : 0.0;
  }
}

template <int NV>
__device__ __forceinline__ void At_mul(const QP<NV>& P, const double* w, double* out) {
  const bool in = lid() < P.H;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double wr = P.valid(2 * v + 1) ? w[2 * v + 1] : 0.0;
    const double wb = P.valid(2 * v) ? w[2 * v] : 0.0;
    out[v] = wb - wr + shup(wr, 1);
  }
  if constexpr (NV == 2) {
    const double tt = Tt_apply(P.valid(4) ? w[4] : 0.0);
    out[0] += P.g1 * tt;
    out[1] += P.g2 * tt;
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
    if (!in) out[v] = 0.0;
}

// y = M r with M (n x n, symmetric) at row-major base (LDS or HBM), r at var lanes.
// BD: M is block-diagonal in the NV vehicle blocks (the pair's P^-1), only those are read.
// Loads are issued GEMV_U deep before their first use so that the pair's L2-resident
// tables cost one latency per batch, not one per column.
constexpr int GEMV_U = 8;
#ifndef PIADMM_XGEMV_U
#define PIADMM_XGEMV_U 15
#endif
constexpr int XGEMV_U = PIADMM_XGEMV_U;   // x-step fused pass batch, LDS mode (big mode: 8; tools/xcost.py)
template <bool BD, int NV, typename Ptr>
__device__ __forceinline__ void gemv_sym(const QP<NV>& P, Ptr M, const double* r, double* y) {
  const int l = lid();
  const int H = P.H, n = P.n;
  if (l < H) {
#pragma unroll
    for (int v = 0; v < NV; ++v) P.vb[v * H + l] = r[v];
  }
  wsync();
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
  const int lc = (l < H) ? l : 0;
  if constexpr (BD) {
    for (int j0 = 0; j0 < H; j0 += GEMV_U) {
      double mv[NV][GEMV_U], rv[NV][GEMV_U];
#pragma unroll
      for (int u = 0; u < GEMV_U; ++u) {
        const int j = min(j0 + u, H - 1);
        const bool ok = j0 + u < H;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          mv[v][u] = M[(v * H + j) * n + v * H + lc];
          rv[v][u] = ok ? P.vb[v * H + j] : 0.0;
        }
      }
#pragma unroll
      for (int u = 0; u < GEMV_U; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += mv[v][u] * rv[v][u];
    }
  } else {
    for (int j0 = 0; j0 < n; j0 += GEMV_U) {
      double mv[NV][GEMV_U], rv[GEMV_U];
#pragma unroll
      for (int u = 0; u < GEMV_U; ++u) {
        const int j = min(j0 + u, n - 1);
        rv[u] = (j0 + u < n) ? P.vb[j] : 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) mv[v][u] = M[j * n + v * H + lc];
      }
#pragma unroll
      for (int u = 0; u < GEMV_U; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[v] += mv[v][u] * rv[u];
    }
  }
  wsync();
#pragma unroll
  for (int v = 0; v < NV; ++v) y[v] = (l < H) ? acc[v] : 0.0;
}

// prox of phi/rho at v in scaled units for row slot s
template <int NV>
__device__ __forceinline__ double prox_s(const QP<NV>& P, int s, double v) {
  const double e = P.E[s];
  if (P.hinge(s)) {
    const double hs = e * P.lo(s);
    const double thr = (P.beta / e) / rrow(P, s);
    return v >= hs ? v : (v <= hs - thr ? v + thr : hs);
  }
  return fmin(fmax(v, e * P.lo(s)), e * P.hi(s));
}

// label from a prox input in scaled units (ADMM state)
template <int NV>
__device__ __forceinline__ signed char label_scaled(const QP<NV>& P, int s, double v) {
  const double e = P.E[s];
  if (!P.valid(s)) return 0;
  if (P.hinge(s)) {
    const double hs = e * P.lo(s);
    const double thr = (P.beta / e) / rrow(P, s);
    return v >= hs ? HZERO : (v <= hs - thr ? HLINEAR : HKINK);
  }
  return v <= e * P.lo(s) ? LOWER : (v >= e * P.hi(s) ? UPPER : FREE);
}

template <int NV>
__device__ __forceinline__ void admm_iter(const QP<NV>& P, double* xs, double* zs, double* ys) {
  constexpr int NR = QP<NV>::NR;
  double w[NR], t[NV], rhs[NV], xt[NV], xu[NV], a[NR];
#pragma unroll
  for (int s = 0; s < NR; ++s) w[s] = P.valid(s) ? P.E[s] * (rrow(P, s) * zs[s] - ys[s]) : 0.0;
  At_mul(P, w, t);
#pragma unroll
  for (int v = 0; v < NV; ++v) rhs[v] = P.sigma * xs[v] - P.D[v] * P.q[v] + P.D[v] * t[v];
  if (P.kf32) gemv_sym<false>(P, P.Kf, rhs, xt);     // fp32 storage, fp64 accumulation
  else gemv_sym<false>(P, P.K, rhs, xt);
#pragma unroll
  for (int v = 0; v < NV; ++v) xu[v] = P.D[v] * xt[v];
  A_mul(P, xu, a);
#pragma unroll
  for (int v = 0; v < NV; ++v) xs[v] = P.alpha * xt[v] + (1.0 - P.alpha) * xs[v];
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    if (!P.valid(s)) {
      zs[s] = ys[s] = 0.0;
      continue;
    }
    const double rs = rrow(P, s);
    const double zr = P.alpha * (P.E[s] * a[s]) + (1.0 - P.alpha) * zs[s];
    const double vin = zr + ys[s] / rs;
    const double zn = prox_s(P, s, vin);
    ys[s] += rs * (zr - zn);
    zs[s] = zn;
  }
}

// ---- Schur-complement entry a' P^-1 b for rows given by ids (slot*H + lane).
// A box/rate row is c0 e_{i0} + c1 e_{i1} (c1 = 0 for a box row); hinge rows use PGt/GPG.
struct RowT {
  int i0, i1, hk;
  double c0, c1;
};
template <int NV>
__device__ __forceinline__ RowT row_terms(const QP<NV>& P, int id) {
  const int s = id / P.H, k = id - s * P.H;
  RowT r;
  if (NV == 2 && s == 4) {
    r.hk = k;
    r.i0 = r.i1 = 0;
    r.c0 = r.c1 = 0.0;
    return r;
  }
  const int base = (s >> 1) * P.H + k;
  r.hk = -1;
  if ((s & 1) == 0) {
    r.i0 = base; r.c0 = 1.0; r.i1 = base; r.c1 = 0.0;
  } else {
    r.i0 = base + 1; r.c0 = 1.0; r.i1 = base; r.c1 = -1.0;
  }
  return r;
}

// hinge coefficient of variable i (vehicle 1: g1, vehicle 2: g2); PGt/GPG hold unscaled tables
template <int NV>
__device__ __forceinline__ double gvar(const QP<NV>& P, int i) { return i < P.H ? P.g1 : P.g2; }

// Gather form: an entry of S = A_W P^-1 A_W' is sum_t c[t] P.Pinv[o[t]] over at most four
// terms (the pair's PGt / GPG follow P^-1 in the same per-edge block at +4H^2 / +6H^2),
// so a batch of entries issues all its loads before the first use.
struct Gather4 {
  int o[4];
  double c[4];
};
template <int NV>
__device__ __forceinline__ Gather4 s_gather(const QP<NV>& P, int ia, int ibd) {
  const RowT a = row_terms(P, ia), b = row_terms(P, ibd);
  const int n = P.n, HH = P.H * P.H;
  Gather4 g;
  if (a.hk < 0 && b.hk < 0) {
    g.o[0] = a.i0 * n + b.i0; g.c[0] = a.c0 * b.c0;
    g.o[1] = a.i0 * n + b.i1; g.c[1] = a.c0 * b.c1;
    g.o[2] = a.i1 * n + b.i0; g.c[2] = a.c1 * b.c0;
    g.o[3] = a.i1 * n + b.i1; g.c[3] = a.c1 * b.c1;
    return g;
  }
  g.o[2] = g.o[3] = 0;
  g.c[2] = g.c[3] = 0.0;
  if (a.hk < 0 || b.hk < 0) {
    const RowT& bx = (a.hk < 0) ? a : b;
    const int hk = (a.hk < 0) ? b.hk : a.hk;
    const int base = 4 * HH + hk * n;
    g.o[0] = base + bx.i0; g.c[0] = bx.c0 * gvar(P, bx.i0);
    g.o[1] = base + bx.i1; g.c[1] = bx.c1 * gvar(P, bx.i1);
    return g;
  }
  const int base = 6 * HH + a.hk * P.H + b.hk;
  g.o[0] = base; g.c[0] = P.g1 * P.g1;
  g.o[1] = base + HH; g.c[1] = P.g2 * P.g2;
  return g;
}

// Solve L L' x = b (lane a holds b_a, a < m).  L lower in fac (stride ld), linv = 1/L_aa.
__device__ __forceinline__ double chol_solve(const double* L_, int ld, double linv, double b, int m) {
  const ldsd* L = lds_ptr(L_);      // the factor lives in the wave's LDS scratch
  const int l = lid();
  for (int k = 0; k < m; ++k) {       // forward, column-oriented
    const double Llk = (l > k && l < m) ? L[l * ld + k] : 0.0;
    const double zk = rdl(b * linv, k);
    if (l == k) b = zk;
    b -= Llk * zk;
  }
  for (int k = m - 1; k >= 0; --k) {  // backward with L'
    const double Lkl = (l < k) ? L[k * ld + l] : 0.0;
    const double xk = rdl(b * linv, k);
    if (l == k) b = xk;
    b -= Lkl * xk;
  }
  return (l < m) ? b : 0.0;
}

// Left-looking Cholesky of S + delta I.  S is stored in the upper triangle of fac
// (row a, columns b >= a) with its diagonal in sdiag (lane a); L goes to the strict
// lower triangle and the diagonal.  A row whose pivot collapses below DEP_TOL * S_kk is
// linearly dependent on the earlier working-set rows (degenerate vertices of the box/rate
// polytope, e.g. u_k = -umax, u_{k+3} = +umax and the three rates between them at +dumax):
// it is dropped (zero column of L, linv = 0, so its multiplier solves to 0), as the
// oracle's active-set solver does.  Returns false only on a non-finite pivot.
constexpr double DEP_TOL = 1e-10;
__device__ __forceinline__ bool chol_factor(double* fac_, int ld, double sdiag, double delta, int m, double& linv) {
  ldsd* fac = lds_ptr(fac_);        // the wave's LDS scratch
  const int l = lid();
  for (int k = 0; k < m; ++k) {
    double acc = 0.0;
    if (l >= k && l < m) {
      const ldsd* ri = fac + l * ld;
      const ldsd* rk = fac + k * ld;
      int j = 0;
      for (; j + 4 <= k; j += 4)
        acc += ri[j] * rk[j] + ri[j + 1] * rk[j + 1] + ri[j + 2] * rk[j + 2] + ri[j + 3] * rk[j + 3];
      for (; j < k; ++j) acc += ri[j] * rk[j];
    }
    const double sik = (l == k) ? sdiag + delta : ((l > k && l < m) ? fac[k * ld + l] : 0.0);
    const double d = sik - acc;
    const double piv = rdl(d, k);
    if (!isfinite(piv)) return false;
    const bool dep = !(piv > DEP_TOL * rdl(sdiag, k));
    const double lkk = dep ? 1.0 : sqrt(piv);
    const double inv = dep ? 0.0 : 1.0 / lkk;
    wsync();
    if (l == k) {
      fac[k * ld + k] = lkk;
      linv = inv;
    }
    if (l > k && l < m) fac[l * ld + k] = d * inv;
    wsync();
  }
  return true;
}

// One PDAS reduced solve for labels lab; returns false on numerical failure.
// The Cholesky factor of S = A_W P^-1 A_W' is cached per wave and reused when the
// working set W is unchanged (P is fixed for the whole MPC step).
template <int NV>
__device__ __forceinline__ bool reduced_solve(const QP<NV>& P, const signed char* lab, double* x, double* y) {
  constexpr int NR = QP<NV>::NR;
  const int l = lid();
  const int H = P.H;
  const int ld = P.fld;
  double* vb_b = P.vb + 64;        // [64,128) rhs b of W rows
  double* vb_lam = P.vb + 128;     // [128,192)
  double* vb_ax = P.vb + 192;      // [192,512) A x0 by row id (<= 5*32 = 160)
  int* ids = P.ib;                 // current W
  int* cids = P.ib + 64;           // W of the cached factor
  // q~ = q - beta G'(1_linear)
  double qt[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) qt[v] = P.q[v];
  if constexpr (NV == 2) {
    const double lin = (P.valid(4) && lab[4] == HLINEAR) ? 1.0 : 0.0;
    const double tt = Tt_apply(lin);
    if (l < H) {
      qt[0] -= P.beta * P.g1 * tt;
      qt[1] -= P.beta * P.g2 * tt;
    }
  }
  double x0[NV];
  unsigned long long t_rs = STAMP_T();
  gemv_sym<true>(P, P.Pinv, qt, x0);
  STAMP_ADD(NV == 1 ? ST_RED_GEMV : ST_ZR_GEMV, t_rs);
#pragma unroll
  for (int v = 0; v < NV; ++v) x0[v] = -x0[v];
  // working set, compacted in slot-major order
  bool inW[NR];
  int pos[NR];
  int m = 0;
  const unsigned long long ltmask = (l == 0) ? 0ull : (~0ull >> (64 - l));
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    inW[s] = P.valid(s) && (P.hinge(s) ? (lab[s] == HKINK) : (lab[s] != FREE));
    const unsigned long long bm = __ballot(inW[s]);
    pos[s] = m + __popcll(bm & ltmask);
    m += __popcll(bm);
  }
  double ax0[NR];
  A_mul(P, x0, ax0);
  if (__builtin_expect(m > P.mmax, 0)) return false;
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    if (l < H) vb_ax[s * H + l] = ax0[s];
    if (inW[s]) {
      ids[pos[s]] = s * H + l;
      vb_b[pos[s]] = P.hinge(s) ? P.lo(s) : (lab[s] == LOWER ? P.lo(s) : P.hi(s));
    }
  }
  wsync();
  if (m == 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) x[v] = x0[v];
#pragma unroll
    for (int s = 0; s < NR; ++s) y[s] = (P.hinge(s) && P.valid(s) && lab[s] == HLINEAR) ? -P.beta : 0.0;
    return true;
  }
  const int myid = (l < m) ? ids[l] : 0;
  const double rhs = (l < m) ? (vb_ax[myid] - vb_b[l]) : 0.0;
  const bool cached = (P.fstate[0] == m) && wall(l >= m || cids[l] == myid);
  double sdiag, linv;
  if (cached) {
    sdiag = (l < m) ? P.fdiag[l] : 0.0;
    linv = (l < m) ? P.fdiag[64 + l] : 0.0;
  } else {
    // S (upper triangle) into fac: lane a = row a, columns b >= a
    unsigned long long t_s = STAMP_T();
    sdiag = 0.0;
    constexpr int SB = 4;
    for (int b0 = 0; b0 < m; b0 += SB) {
      Gather4 gg[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) gg[u] = s_gather(P, myid, rdli(myid, min(b0 + u, m - 1)));
      double tv[SB][4];
#pragma unroll
      for (int u = 0; u < SB; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) tv[u][k] = P.Pinv[gg[u].o[k]];
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int b = b0 + u;
        const double sv = gg[u].c[0] * tv[u][0] + gg[u].c[1] * tv[u][1] + gg[u].c[2] * tv[u][2] + gg[u].c[3] * tv[u][3];
        if (b < m && l <= b && l < m) {
          if (b == l) sdiag = sv;
          else lds_ptr(P.fac)[l * ld + b] = sv;
        }
      }
    }
    STAMP_ADD(NV == 1 ? ST_RED_S : ST_ZR_S, t_s);
    unsigned long long t_c = STAMP_T();
    // no diagonal shift: a dependent working-set row is dropped by its collapsed pivot
    // (chol_factor); a shift would hide the collapse of rows with a small S_kk
    const double delta = 0.0;
    wsync();
    linv = 0.0;
    const bool fok = chol_factor(P.fac, ld, sdiag, delta, m, linv);
    STAMP_ADD(NV == 1 ? ST_RED_CHOL : ST_ZR_CHOL, t_c);
    if (!fok) {
      if (l == 0) P.fstate[0] = -1;
      wsync();
      return false;
    }
    if (l < m) {
      P.fdiag[l] = sdiag;
      P.fdiag[64 + l] = linv;
      cids[l] = myid;
    }
    if (l == 0) P.fstate[0] = m;
    wsync();
  }
  unsigned long long t_sv = STAMP_T();
  double lamv = chol_solve(P.fac, ld, linv, rhs, m);
  // one step of iterative refinement against the unregularised S
  {
    double sl = 0.0;
    for (int b = 0; b < m; ++b) {
      const double lb = rdl(lamv, b);
      if (l < m) {
        const ldsd* F = lds_ptr(P.fac);
        const double sab = (b == l) ? sdiag : (b > l ? F[l * ld + b] : F[b * ld + l]);
        sl += sab * lb;
      }
    }
    const double r = (l < m) ? rhs - sl : 0.0;
    lamv += chol_solve(P.fac, ld, linv, r, m);
  }
  STAMP_ADD(NV == 1 ? ST_XR_SOLVE : ST_ZR_SOLVE, t_sv);
  if (!isfinite(lamv)) return false;
  unsigned long long t_x = STAMP_T();
  // x = x0 - sum_a (P^-1 a_a) lam_a
  double xv[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) xv[v] = x0[v];
  auto sub_Y = [&](double lamv) {
    constexpr int XB = 4;
    const int lc = (l < H) ? l : 0;
    for (int a0 = 0; a0 < m; a0 += XB) {
      int o[XB][NV][2];
      double cf[XB][NV][2], la[XB];
#pragma unroll
      for (int u = 0; u < XB; ++u) {
        const int a = min(a0 + u, m - 1);
        const RowT r = row_terms(P, rdli(myid, a));
        la[u] = (a0 + u < m) ? rdl(lamv, a) : 0.0;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const int i = v * H + lc;
          if (NV == 2 && r.hk >= 0) {        // (P^-1 G_k')_i, unscaled table times g_v
            o[u][v][0] = o[u][v][1] = 4 * H * H + r.hk * P.n + i;
            cf[u][v][0] = v ? P.g2 : P.g1;
            cf[u][v][1] = 0.0;
          } else {
            o[u][v][0] = r.i0 * P.n + i; cf[u][v][0] = r.c0;
            o[u][v][1] = r.i1 * P.n + i; cf[u][v][1] = r.c1;
          }
        }
      }
      double tv[XB][NV][2];
#pragma unroll
      for (int u = 0; u < XB; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
          for (int k = 0; k < 2; ++k) tv[u][v][k] = P.Pinv[o[u][v][k]];
#pragma unroll
      for (int u = 0; u < XB; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) xv[v] -= (cf[u][v][0] * tv[u][v][0] + cf[u][v][1] * tv[u][v][1]) * la[u];
    }
  };
  sub_Y(lamv);
  // one step of primal refinement: at a vertex held by large multipliers (a saturated pair
  // pushed by linear hinge rows: |lam| ~ 1e6 at beta = 1000) x0 - Y lam cancels to ~1e-9, above
  // the certificate's feasibility tolerance; the correction of the active rows' residual
  // e = A_W x - b is small, so its own cancellation is not
  {
    double axr[NR];
    A_mul(P, xv, axr);
    wsync();
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = axr[s];
    }
    wsync();
    const double e = (l < m) ? vb_ax[myid] - vb_b[l] : 0.0;
    const double dl = chol_solve(P.fac, ld, linv, e, m);
    if (!isfinite(dl)) return false;
    lamv += dl;
    sub_Y(dl);
  }
  STAMP_ADD(NV == 1 ? ST_RED_X : ST_ZR_X, t_x);
  if (l < m) vb_lam[l] = lamv;
  wsync();
#pragma unroll
  for (int v = 0; v < NV; ++v) x[v] = (l < H) ? xv[v] : 0.0;
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    if (inW[s]) y[s] = vb_lam[pos[s]];
    else if (P.hinge(s) && P.valid(s) && lab[s] == HLINEAR) y[s] = -P.beta;
    else y[s] = 0.0;
  }
  wsync();
  return true;
}

// x-step (NV = 1) polish in parametric form.  P and A are fixed for the whole MPC step and
// only q changes between outer iterations, so for a working set W with bounds b
//   lam = S^-1 (A_W x0 - b) = -X q - beta,   x = x0 - Y lam,   x0 = -P^-1 q,
// with Y = P^-1 A_W', S = A_W Y, X = S^-1 Y', beta = S^-1 b.  X' (rows = variables) and
// beta (row H) are rebuilt in LDS only when W or the bound side of one of its rows changes;
// a hit costs one fused pass over P^-1 and X' plus the x recovery.
// TT (fused kernel, LDS mode): the tables transposed -- X T' as rows a of stride xld (beta at
// column H), G T' as rows of stride gt_ld(H) (g after the H rows) -- so the hit pass reads a
// lane's own row two doubles at a time (reduced_solve_x).
template <bool TT = false>
__device__ __forceinline__ bool param_build_x(const QP<1>& P, int m, int myid, const int* ids, const double* vb_b) {
  const int l = lid(), H = P.H, ld = P.fld;
  ldsd* fac = lds_ptr(P.fac);       // the wave's LDS scratch
  double* XT = P.XT;
  // S (upper triangle, lane a = row a) from the LDS P^-1
  unsigned long long t_s = STAMP_T();
  double sdiag = 0.0;
  constexpr int SB = 4;
  for (int b0 = 0; b0 < m; b0 += SB) {
    Gather4 gg[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) gg[u] = s_gather(P, myid, ids[min(b0 + u, m - 1)]);
    double tv[SB][4];
#pragma unroll
    for (int u = 0; u < SB; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) tv[u][k] = P.Pinv[gg[u].o[k]];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int b = b0 + u;
      const double sv = gg[u].c[0] * tv[u][0] + gg[u].c[1] * tv[u][1] + gg[u].c[2] * tv[u][2] + gg[u].c[3] * tv[u][3];
      if (b < m && l <= b && l < m) {
        if (b == l) sdiag = sv;
        else fac[l * ld + b] = sv;
      }
    }
  }
  STAMP_ADD(ST_RED_S, t_s);
  unsigned long long t_c = STAMP_T();
  wsync();
  double linv = 0.0;
  // unshifted: a dependent working-set row (degenerate vertex) is dropped by chol_factor
  if (!chol_factor(P.fac, ld, sdiag, 0.0, m, linv)) return false;
  if (l < m) P.fdiag[64 + l] = linv;
  STAMP_ADD(ST_RED_CHOL, t_c);
  unsigned long long t_x = STAMP_T();
  // right-hand sides, one per lane: lane i < H -> row i of Y = P^-1 A_W', lane H -> b
  // X', G, g: LDS (LDS mode) or HBM (big / graph mode) -- the same space for both tables
  auto tables = [&](auto XTp, auto Gp) {
  const int li = (l <= H) ? l : H;
  const bool own = l <= H;
  const int gld = gt_ld(H);
  // element (li, a) of X' (lane li = time index, or H: the right-hand side b / beta)
  auto xr = [&](int a) -> auto& { return TT ? XTp[a * P.xld + li] : XTp[li * P.xld + a]; };
  constexpr int XB = 4;
  for (int a0 = 0; a0 < m; a0 += XB) {
    int o[XB][2];
    double cf[XB][2];
#pragma unroll
    for (int u = 0; u < XB; ++u) {
      const RowT r = row_terms(P, ids[min(a0 + u, m - 1)]);
      const int i = (l < H) ? l : 0;
      o[u][0] = r.i0 * H + i; cf[u][0] = r.c0;
      o[u][1] = r.i1 * H + i; cf[u][1] = r.c1;
    }
    double tv[XB][2];
#pragma unroll
    for (int u = 0; u < XB; ++u) {
      tv[u][0] = P.Pinv[o[u][0]];
      tv[u][1] = P.Pinv[o[u][1]];
    }
#pragma unroll
    for (int u = 0; u < XB; ++u) {
      const int a = a0 + u;
      if (a < m) {
        const double v = (l < H) ? cf[u][0] * tv[u][0] + cf[u][1] * tv[u][1] : vb_b[a];
        if (own) xr(a) = v;
      }
    }
  }
  wsync();
  // L L' sol = rhs for every lane's right-hand side (L broadcast from fac, lane-own sol)
  constexpr int TB = 8;
  for (int a = 0; a < m; ++a) {
    double acc = xr(a);
    for (int b0 = 0; b0 < a; b0 += TB) {
      double Lv[TB], sv[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        const int b = min(b0 + u, a - 1);
        Lv[u] = (b0 + u < a) ? fac[a * ld + b] : 0.0;
        sv[u] = xr(b);
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) acc -= Lv[u] * sv[u];
    }
    acc *= P.fdiag[64 + a];
    if (own) xr(a) = acc;
  }
  for (int a = m - 1; a >= 0; --a) {
    double acc = xr(a);
    for (int b0 = a + 1; b0 < m; b0 += TB) {
      double Lv[TB], sv[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        const int b = min(b0 + u, m - 1);
        Lv[u] = (b0 + u < m) ? fac[b * ld + a] : 0.0;
        sv[u] = xr(b);
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) acc -= Lv[u] * sv[u];
    }
    acc *= P.fdiag[64 + a];
    if (own) xr(a) = acc;
  }
  if (P.gmem) gsync();
  else wsync();
  STAMP_ADD(ST_XR_SOLVE, t_x);
  // G = P^-1 - Y X and g = Y beta (lane j = column j): Y is re-gathered column by column
  // into the factor scratch (the factor is not needed once X' is known), then every lane
  // accumulates its column of Y X from LDS broadcasts of Y and its own row of X'.
  {
    const int lc = (l < H) ? l : 0;
    for (int a0 = 0; a0 < m; a0 += XB) {
      double tv[XB][2], cf[XB][2];
#pragma unroll
      for (int u = 0; u < XB; ++u) {
        const RowT r = row_terms(P, ids[min(a0 + u, m - 1)]);
        cf[u][0] = r.c0;
        cf[u][1] = r.c1;
        tv[u][0] = P.Pinv[r.i0 * H + lc];
        tv[u][1] = P.Pinv[r.i1 * H + lc];
      }
#pragma unroll
      for (int u = 0; u < XB; ++u)
        if (a0 + u < m && l < H) fac[(a0 + u) * ld + l] = cf[u][0] * tv[u][0] + cf[u][1] * tv[u][1];
    }
    wsync();
    // X'[lc][a]: lane lc's time row of X'
    auto xj = [&](int a) -> double { return TT ? XTp[a * P.xld + lc] : XTp[lc * P.xld + a]; };
    constexpr int GB = 8;
    for (int i0 = 0; i0 < H; i0 += GB) {
      double acc[GB], pv[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        acc[u] = 0.0;
        pv[u] = P.Pinv[min(i0 + u, H - 1) * H + lc];
      }
      for (int a = 0; a < m; ++a) {
        const double xja = xj(a);
        const ldsd* ya = fac + a * ld + i0;
#pragma unroll
        for (int u = 0; u < GB; ++u) acc[u] += ya[u] * xja;     // rows past H are never stored
      }
#pragma unroll
      for (int u = 0; u < GB; ++u)   // (G is symmetric: TT stores lane l's column as its row)
        if (l < H && i0 + u < H) Gp[TT ? l * gld + i0 + u : (i0 + u) * H + l] = pv[u] - acc[u];
    }
    double gacc = 0.0;
    for (int a = 0; a < m; ++a) gacc += fac[a * ld + lc] * XTp[TT ? a * P.xld + H : H * P.xld + a];
    if (l < H) Gp[TT ? H * gld + l : H * H + l] = gacc;
    if (TT && gld > H && l < H) Gp[l * gld + H] = 0.0;   // the row's pad: read (times q = 0) by the pass
    if (P.gmem) gsync();
    else wsync();
    if (!TT && P.t32) {
      // precision 2: fp32 images of the unfolded G and X' (the fp64 tables stay: the fallback)
      float* G32 = P.t32;
      float* X32 = P.t32 + H * H;
      for (int k = 0; k < H; ++k) {
        if (l < H) G32[k * H + l] = (float)Gp[k * H + l];
        if (l < m) X32[k * XLDG + l] = (float)XTp[k * P.xld + l];
      }
      gsync();
    }
  }
  // fold q = T'-apply(w') into the tables: row k of G T' (and X T') is
  // sum_{j<k} (k - j) row j -- two running sums per lane, in place (read before write)
  {
    double s1 = 0.0, s2 = 0.0, t1 = 0.0, t2 = 0.0;
    const int la = (l < m) ? l : 0;
    const int lg = (l < H) ? l : 0;
    for (int k = 0; k < H; ++k) {
      const double gk = Gp[TT ? lg * gld + k : k * H + lg];
      const double xk = XTp[TT ? la * P.xld + k : k * P.xld + la];
      if (l < H) Gp[TT ? l * gld + k : k * H + l] = s2;
      if (l < m) XTp[TT ? l * P.xld + k : k * P.xld + l] = t2;
      s1 += gk;
      s2 += s1;
      t1 += xk;
      t2 += t1;
    }
    if (P.gmem) gsync();
    else wsync();
  }
  };
  if (in_lds(XT)) tables(lds_ptr(XT), lds_ptr(P.G));
  else tables(gbl_ptr(XT), gbl_ptr(P.G));
  return true;
}

// ---- precision 2: the parametric hit from fp32 tables, refined once in fp64 (configs[4] study).
// s_g = sum_j G32[j][lane] a_j (lane < H), s_x = sum_j X32[j][lane] b_j (lane < m): fp32 table entries,
// fp64 products and sums; a, b broadcast from LDS (zero-padded to 64).
template <int XU>
__device__ __forceinline__ void pass32(const QP<1>& P, int m, const ldsd* va, const ldsd* vbv, double& sg, double& sx) {
  const int l = lid(), H = P.H;
  const int lc = (l < H) ? l : 0, la = (l < m) ? l : 0;
  const float* gp = P.t32 + lc;
  const float* xp = P.t32 + H * H + la;
  double ag = 0.0, ax = 0.0;
  for (int j0 = 0; j0 < H; j0 += XU) {
    float gv[XU], xv[XU];
    double av[XU], bv[XU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      const int j = min(j0 + u, H - 1);
      gv[u] = gp[j * H];
      xv[u] = xp[j * XLDG];
      av[u] = va[j0 + u];
      bv[u] = vbv[j0 + u];
    }
#pragma unroll
    for (int u = 0; u < XU; ++u) {
      ag += (double)gv[u] * av[u];
      ax += (double)xv[u] * bv[u];
    }
  }
  sg = ag;
  sx = ax;
}

// The hit with fp32 G, X' (unfolded) and ONE step of iterative refinement in fp64 against the exact
// KKT residual of the working set: x0 = g - G32 q, lam0 = -X32 q - beta; r1 = P x0 + q + A_W' lam0,
// r2 = A_W x0 - b (matrix-free P, stencil A); d = X32' r2; dx = -G32 r1 - d,
// dlam = -X32 (r1 - P d) (S^-1 = X P X', so S^-1 r2 = X P d).  g and beta stay fp64.  The answer goes
// to the same KKT certificate as every other solve (a failure falls back to the fp64 paths).
template <int XU>
__device__ __forceinline__ void hit32(const QP<1>& P, int m, const bool* inW, const int* pos, const signed char* lab,
                                      double* x, double* y) {
  const int l = lid(), H = P.H;
  const int lc = (l < H) ? l : 0, la = (l < m) ? l : 0;
  ldsd* va = lds_ptr(P.vb + 256);
  ldsd* vbv = lds_ptr(P.vb + 320);
  ldsd* vr2 = lds_ptr(P.vb + 384);
  const double gfix = P.G[H * H + lc];                         // g (fp64, row H of the table)
  const double bfix = P.XT[H * P.xld + la];                    // beta (fp64, row H of X')
  const double q = Tt_apply(P.wq);
  const double qv = (l < H) ? q : 0.0;
  va[l] = qv;
  vbv[l] = qv;
  wsync();
  double sg, sx;
  pass32<XU>(P, m, va, vbv, sg, sx);
  double x0[1] = {(l < H) ? gfix - sg : 0.0};
  const double lam0 = (l < m) ? -sx - bfix : 0.0;
  wsync();
  vr2[l] = lam0;                                               // (W-row multipliers, lane a)
  wsync();
  double y0[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) y0[s] = inW[s] ? vr2[pos[s]] : 0.0;
  // r1 = P x0 + q + A_W' lam0 (var lanes), r2 = A_W x0 - b (W rows)
  double px[1], aty[1], ax[2];
  P_mul(P, x0, px);
  At_mul(P, y0, aty);
  A_mul(P, x0, ax);
  const double r1 = (l < H) ? px[0] + qv + aty[0] : 0.0;
  wsync();
  vr2[l] = 0.0;
  wsync();
#pragma unroll
  for (int s = 0; s < 2; ++s)
    if (inW[s]) vr2[pos[s]] = ax[s] - ((lab[s] == LOWER) ? P.lo(s) : P.hi(s));
  wsync();
  // d = X32' r2 (lane j = variable: its own row of X')
  double dd = 0.0;
  {
    const int mu = unif(m);
    const float* xr = P.t32 + H * H + lc * XLDG;
    for (int a0 = 0; a0 < mu; a0 += XU) {
      float xv[XU];
      double rv[XU];
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        xv[u] = xr[min(a0 + u, mu - 1)];
        rv[u] = (a0 + u < mu) ? vr2[a0 + u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < XU; ++u) dd += (double)xv[u] * rv[u];
    }
    if (l >= H) dd = 0.0;
  }
  double dv[1] = {dd}, pd[1];
  P_mul(P, dv, pd);
  wsync();
  va[l] = r1;
  vbv[l] = (l < H) ? r1 - pd[0] : 0.0;
  wsync();
  pass32<XU>(P, m, va, vbv, sg, sx);
  x[0] = (l < H) ? x0[0] - sg - dd : 0.0;
  const double lam = (l < m) ? lam0 - sx : 0.0;
  wsync();
  vr2[l] = lam;
  wsync();
#pragma unroll
  for (int s = 0; s < 2; ++s) y[s] = inW[s] ? vr2[pos[s]] : 0.0;
  wsync();
}

// The x-step hit's fused pass over the transposed tables (reduced_solve_x TT): lane rows gr (G T') and
// xr2 (X T') against q2 = w', hp pairs of time indices in batches of 8 pairs, two accumulators per table
// (even / odd time index), the last batch's pairs beyond hp clamped to pair hp - 1 against the
// zero-padded q.  HPC > 0: hp compiled in (every load an immediate offset from the row bases, no loop
// control, no clamp arithmetic); 0: hp at run time.  Both perform the same products and sums in the
// same order, so their results are bit-identical.
template <int HPC>
__device__ __forceinline__ void hit_pass(const ldsd2* gr, const ldsd2* xr2, const ldsd2* q2, int hp_rt, double& ag,
                                         double& ag1, double& ax, double& ax1) {
  constexpr int U = 8;
  if constexpr (HPC > 0) {
    constexpr int HF = HPC - HPC % U;
#pragma unroll
    for (int p0 = 0; p0 < HF; p0 += U) {
      dv2 qv[U], gv[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        qv[u] = q2[p0 + u];
        gv[u] = gr[p0 + u];
        xv[u] = xr2[p0 + u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ag += gv[u].x * qv[u].x;
        ag1 += gv[u].y * qv[u].y;
        ax += xv[u].x * qv[u].x;
        ax1 += xv[u].y * qv[u].y;
      }
    }
    if constexpr (HF < HPC) {
      dv2 qv[U], gv[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        constexpr int last = HPC - 1;
        const int pi = (HF + u < last) ? HF + u : last;
        qv[u] = q2[HF + u];            // zero beyond H (vb_q is zero-padded to 64)
        gv[u] = gr[pi];
        xv[u] = xr2[pi];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ag += gv[u].x * qv[u].x;
        ag1 += gv[u].y * qv[u].y;
        ax += xv[u].x * qv[u].x;
        ax1 += xv[u].y * qv[u].y;
      }
    }
  } else {
    const int hp = hp_rt;
    const int hf = hp - hp % U;
    for (int p0 = 0; p0 < hf; p0 += U) {
      dv2 qv[U], gv[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        qv[u] = q2[p0 + u];
        gv[u] = gr[p0 + u];
        xv[u] = xr2[p0 + u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ag += gv[u].x * qv[u].x;
        ag1 += gv[u].y * qv[u].y;
        ax += xv[u].x * qv[u].x;
        ax1 += xv[u].y * qv[u].y;
      }
    }
    if (hf < hp) {
      dv2 qv[U], gv[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pi = min(hf + u, hp - 1);
        qv[u] = q2[hf + u];            // zero beyond H (vb_q is zero-padded to 64)
        gv[u] = gr[pi];
        xv[u] = xr2[pi];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ag += gv[u].x * qv[u].x;
        ag1 += gv[u].y * qv[u].y;
        ax += xv[u].x * qv[u].x;
        ax1 += xv[u].y * qv[u].y;
      }
    }
  }
}

template <int XU, bool TT = false>
__device__ __forceinline__ bool reduced_solve_x(const QP<1>& P, const signed char* lab, double* x, double* y) {
  const int l = lid(), H = P.H;
  unsigned long long t_pre = STAMP_T();
  double* vb_q = P.vb;             // [0,64) q
  double* vb_b = P.vb + 64;        // [64,128) rhs b of W rows
  double* vb_lam = P.vb + 128;     // [128,192)
  int* ids = P.ib;                 // current W
  int* cids = P.ib + 64;           // W (with bound sides) of the cached X', beta
  const double* XT = P.XT;
  bool inW[2];
  int pos[2];
  int m = 0;
  const unsigned long long ltmask = (l == 0) ? 0ull : (~0ull >> (64 - l));
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    inW[s] = P.valid(s) && lab[s] != FREE;
    const unsigned long long bm = __ballot(inW[s]);
    pos[s] = m + __popcll(bm & ltmask);
    m += __popcll(bm);
  }
  if (__builtin_expect(m > P.mmax, 0)) return false;
  // w' (q = T'-apply(w'), folded into the tables: G T', X T'), zero-padded to 64 so that the
  // fused pass loads it unconditionally
  vb_q[l] = (l < H) ? P.wq : 0.0;
  // the working set with its bound sides as a per-lane signature (this lane's box and rate
  // rows) in a register: a hit on the cached X', G is one ballot, no LDS round trip
  const int sig = (inW[0] ? (int)lab[0] : 0) | ((inW[1] ? (int)lab[1] : 0) << 2);
  if (__builtin_expect(!wall(sig == P.csig), 0)) {   // csig = -1 whenever the tables are not valid
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (inW[s]) {
        ids[pos[s]] = s * H + l;
        vb_b[pos[s]] = (lab[s] == LOWER) ? P.lo(s) : P.hi(s);
      }
    }
    wsync();
    const int myid = (l < m) ? ids[l] : 0;
    if (!param_build_x<TT>(P, m, myid, ids, vb_b)) {
      if (l == 0) P.fstate[0] = -1;
      P.csig = -1;
      wsync();
      return false;
    }
    P.csig = sig;
    if (l == 0) P.fstate[0] = m;
  }
  (void)cids;
  wsync();
  STAMP_ADD(ST_RSX_PRE, t_pre);
  if (!TT && P.t32) {                // precision 2: fp32 tables + one fp64 refinement step
    hit32<XU>(P, m, inW, pos, lab, x, y);
    return true;
  }
  unsigned long long t_rs = STAMP_T();
  // one fused pass: x = -G q + g (lane = variable), lam = -X q - beta (lane = W row)
  double ag = 0.0, ax = 0.0;
  if constexpr (TT) {
    // transposed tables: lane lc walks its row of G T', lane la its row of X T' (16-byte loads;
    // pairs of time indices, the last one padded: q is zero there)
    const int lc = (l < H) ? l : 0, la = (l < m) ? l : 0;
    const int gld = unif(gt_ld(H)), xs = unif(P.xld);
    const ldsd2* gr = (const ldsd2*)(lds_ptr(P.G) + lc * gld);
    const ldsd2* xr2 = (const ldsd2*)(lds_ptr(XT) + la * xs);
    const ldsd2* q2 = (const ldsd2*)lds_ptr(vb_q);
    const int hp = unif((H + 1) >> 1);
    double ag1 = 0.0, ax1 = 0.0;
    // BASELINE's horizons (10, 20, 30) with the pair count compiled in: immediate offsets, no loop
    switch (hp) {
      case 15: hit_pass<15>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
      case 10: hit_pass<10>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
      case 5: hit_pass<5>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
      default: hit_pass<0>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
    }
    ag += ag1;
    ax += ax1;
    if (l < m) vb_lam[l] = -ax - XT[l * xs + H];
    ag = P.G[H * gld + lc] - ag;
  } else {
    const int lc = (l < H) ? l : 0, la = (l < m) ? l : 0;
    const double* G = P.G;
    // full batches: row pointers advance by a stride, no clamp
    const int Hf = H - H % XU;
    const double* gp = G + lc;
    const double* xp = XT + la;
    const int xs = P.xld;
    for (int j0 = 0; j0 < Hf; j0 += XU) {
      double qv[XU], gv[XU], xv[XU];
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        qv[u] = vb_q[j0 + u];
        gv[u] = gp[u * H];
        xv[u] = xp[u * xs];
      }
      gp += XU * H;
      xp += XU * xs;
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        ag += gv[u] * qv[u];
        ax += xv[u] * qv[u];
      }
    }
    if (Hf < H) {                       // tail: rows clamped to H - 1, q is 0 beyond H
      double qv[XU], gv[XU], xv[XU];
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        const int j = min(Hf + u, H - 1);
        qv[u] = vb_q[Hf + u];
        gv[u] = G[j * H + lc];
        xv[u] = XT[j * xs + la];
      }
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        ag += gv[u] * qv[u];
        ax += xv[u] * qv[u];
      }
    }
    if (l < m) vb_lam[l] = -ax - XT[H * P.xld + l];
    ag = G[H * H + lc] - ag;
  }
  wsync();
  STAMP_ADD(ST_RED_GEMV, t_rs);
  x[0] = (l < H) ? ag : 0.0;
#pragma unroll
  for (int s = 0; s < 2; ++s) y[s] = inW[s] ? vb_lam[pos[s]] : 0.0;
  wsync();
  return true;
}

// KKT test of (x, y) for labels lab at multiplier tolerance ty; on failure fills new labels (PDAS
// update).  yfail: some multiplier test of this lane failed at ty.
template <int NV>
__device__ __forceinline__ bool kkt_eval(const QP<NV>& P, const signed char* lab, const double* x, const double* y,
                                         const double* ax, double ty, signed char* nlab, bool& yfail) {
  constexpr int NR = QP<NV>::NR;
  bool ok = true;
  yfail = false;
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    if (!P.valid(s)) {
      nlab[s] = 0;
      continue;
    }
    const double tp = P.tol * (1.0 + fabs(P.lo(s)));
    // Label update: a violated row changes state by one step only -- an active row whose
    // multiplier has the wrong sign is released (never flipped to the opposite bound), a
    // free row becomes active only when its bound is violated beyond the tolerance.  At a
    // degenerate vertex (dependent rows, zero multipliers) this releases the row that
    // received the wrong-signed multiplier instead of cycling between the two bounds.
    if (P.hinge(s)) {
      const double h = P.lo(s);
      if (lab[s] == HZERO) {
        const bool v = ax[s] < h - tp;
        ok &= !v;
        nlab[s] = v ? HKINK : HZERO;
      } else if (lab[s] == HLINEAR) {
        const bool v = ax[s] > h + tp;
        ok &= !v;
        nlab[s] = v ? HKINK : HLINEAR;
      } else {
        // a kink row must sit at h: the reduced solve drops a dependent row, which is only
        // right when the dropped equation is implied by the others (consistent labels)
        const bool yok = (y[s] <= ty) && (y[s] >= -P.beta - ty);
        yfail |= !yok;
        ok &= yok && fabs(ax[s] - h) <= tp;
        nlab[s] = (y[s] > ty) ? HZERO : ((y[s] < -P.beta - ty) ? HLINEAR : HKINK);
      }
    } else {
      if (lab[s] == FREE) {
        const bool vl = ax[s] < P.lo(s) - tp, vu = ax[s] > P.hi(s) + tp;
        ok &= !vl && !vu;
        nlab[s] = vl ? LOWER : (vu ? UPPER : FREE);
      } else if (lab[s] == LOWER) {
        const bool yok = y[s] <= ty;
        yfail |= !yok;
        ok &= yok && fabs(ax[s] - P.lo(s)) <= tp;   // equality too (dropped rows)
        nlab[s] = (y[s] > ty) ? FREE : LOWER;
      } else {
        const bool yok = y[s] >= -ty;
        yfail |= !yok;
        ok &= yok && fabs(ax[s] - P.hi(s)) <= tp;
        nlab[s] = (y[s] < -ty) ? FREE : UPPER;
      }
    }
    ok &= isfinite(x[0]) && isfinite(y[s]);
  }
  return ok;
}

// KKT test of (x, y) for labels lab; on failure fills new labels (PDAS update).  The multiplier
// tolerance is tol (1 + max |y|); the tests are first evaluated at its lower bound tol, and only
// when one of them fails there is the wave max formed and the test repeated: a multiplier test that
// passes at tol passes at any larger tolerance with the same label decision, so the outcome and
// the labels are exactly those of the test at tol (1 + max |y|), without the wave reduction in the
// common case (every multiplier inside its sign band).
template <int NV>
__device__ __forceinline__ bool kkt_check(const QP<NV>& P, const signed char* lab, const double* x, const double* y,
                          signed char* nlab) {
  constexpr int NR = QP<NV>::NR;
  double ax[NR];
  A_mul(P, x, ax);
  bool yfail;
  bool ok = kkt_eval(P, lab, x, y, ax, P.tol, nlab, yfail);
  if (__builtin_expect(wany(yfail), 0)) {
    double ym = 0.0;
#pragma unroll
    for (int s = 0; s < NR; ++s) ym = fmax(ym, fabs(y[s]));
    ym = wmax(ym);
    ok = kkt_eval(P, lab, x, y, ax, P.tol * (1.0 + ym), nlab, yfail);
  }
  return wall(ok);
}

// the x-step's parametric tables hold labels lab's working set (the signature reduced_solve_x
// compares): a reduced solve on lab is one fused pass, not a rebuild
template <int NV>
__device__ __forceinline__ bool tables_match(const QP<NV>& P, const signed char* lab) {
  if constexpr (NV != 1) return true;
  int sig = 0;
#pragma unroll
  for (int s = 0; s < 2; ++s) sig |= ((P.valid(s) && lab[s] != FREE) ? (int)lab[s] : 0) << (2 * s);
  return wall(sig == P.csig);
}

// The repeat of a certified x-step table hit: the speculative x-step of piadmm_device.hip agent_part,
// run only when the x-step in U certified without ADMM and the parametric tables hold its working
// set (spec_ok), so this QP is that one again (q changes only in a z-step).  It is the same solve as
// qp_solve's first branch on transposed tables (tables_match -> pdas, one step -> reduced_solve_x<XU,
// true> -> kkt_check) -- the same pass, products, sums, certificate and counters -- without the
// general solver's scaffolding: the signature is known to match, and the working-set multipliers
// reach their rows through lane permutes instead of an LDS store, sync and gather.  Results are
// bit-identical; on a failed certificate (not expected: the same QP certified before) it gives its
// solve back to the counter and returns false, and the caller runs qp_solve.
// TT: the transposed LDS tables (LDS mode, reduced_solve_x<XU, true>); false: the big mode's tables in
// HBM / L2, lane = column (reduced_solve_x<XU, false>, the same batches of XU rows).
template <int XU, bool TT = true>
__device__ __forceinline__ bool xhit_repeat(QP<1>& P, const signed char* lab, double* xs, double* ys, double* x_out,
                                            int& n_pdas) {
  const int l = lid(), H = P.H;
  bool inW[2];
  int pos[2];
  int m = 0;
  const unsigned long long ltmask = (l == 0) ? 0ull : (~0ull >> (64 - l));
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    inW[s] = P.valid(s) && lab[s] != FREE;
    const unsigned long long bm = __ballot(inW[s]);
    pos[s] = m + __popcll(bm & ltmask);
    m += __popcll(bm);
  }
  double* vb_q = P.vb;
  vb_q[l] = (l < H) ? P.wq : 0.0;
  wsync();
  const int lc = (l < H) ? l : 0, la = (l < m) ? l : 0;
  double ag = 0.0, ax = 0.0, lam;
  if constexpr (TT) {
    const int gld = unif(gt_ld(H)), xsd = unif(P.xld);
    const ldsd2* gr = (const ldsd2*)(lds_ptr(P.G) + lc * gld);
    const ldsd2* xr2 = (const ldsd2*)(lds_ptr(P.XT) + la * xsd);
    const ldsd2* q2 = (const ldsd2*)lds_ptr(vb_q);
    const int hp = unif((H + 1) >> 1);
    double ag1 = 0.0, ax1 = 0.0;
    switch (hp) {
      case 15: hit_pass<15>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
      case 10: hit_pass<10>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
      case 5: hit_pass<5>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
      default: hit_pass<0>(gr, xr2, q2, hp, ag, ag1, ax, ax1); break;
    }
    ag += ag1;
    ax += ax1;
    const ldsd* XT = lds_ptr(P.XT);
    lam = (l < m) ? -ax - XT[l * xsd + H] : 0.0;                    // lane a: multiplier of W row a
    ag = lds_ptr(P.G)[H * gld + lc] - ag;
  } else {
    // (reduced_solve_x<XU, false>'s pass, statement for statement)
    const double* G = P.G;
    const double* XT = P.XT;
    const int Hf = H - H % XU;
    const double* gp = G + lc;
    const double* xp = XT + la;
    const int xsd = P.xld;
    for (int j0 = 0; j0 < Hf; j0 += XU) {
      double qv[XU], gv[XU], xv[XU];
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        qv[u] = vb_q[j0 + u];
        gv[u] = gp[u * H];
        xv[u] = xp[u * xsd];
      }
      gp += XU * H;
      xp += XU * xsd;
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        ag += gv[u] * qv[u];
        ax += xv[u] * qv[u];
      }
    }
    if (Hf < H) {
      double qv[XU], gv[XU], xv[XU];
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        const int j = min(Hf + u, H - 1);
        qv[u] = vb_q[Hf + u];
        gv[u] = G[j * H + lc];
        xv[u] = XT[j * xsd + la];
      }
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        ag += gv[u] * qv[u];
        ax += xv[u] * qv[u];
      }
    }
    lam = (l < m) ? -ax - XT[H * P.xld + l] : 0.0;
    ag = G[H * H + lc] - ag;
  }
  double x[1] = {(l < H) ? ag : 0.0}, y[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const double ys_ = __shfl(lam, pos[s]);
    y[s] = inW[s] ? ys_ : 0.0;
  }
  ++n_pdas;
  signed char nl[2];
  if (__builtin_expect(!kkt_check(P, lab, x, y, nl), 0)) {
    --n_pdas;
    return false;
  }
  xs[0] = x[0];
#pragma unroll
  for (int s = 0; s < 2; ++s) ys[s] = P.valid(s) ? y[s] : 0.0;
  P.wraw = true;
  x_out[0] = x[0];
  return true;
}

template <int NV, int XU = XGEMV_U, bool TT = false>
__device__ __forceinline__ bool pdas(const QP<NV>& P, signed char* lab, double* x, double* y, int& nsolve,
                                     int steps = PDAS_STEPS) {
  constexpr int NR = QP<NV>::NR;
  signed char nl[NR];
  for (int it = 0; it < steps; ++it) {
    ++nsolve;
    unsigned long long t_r = STAMP_T();
    bool rs_ok;
    if constexpr (NV == 1) rs_ok = reduced_solve_x<XU, TT>(P, lab, x, y);
    else rs_ok = reduced_solve(P, lab, x, y);
    STAMP_ADD(NV == 1 ? ST_XRED : ST_ZRED, t_r);
    if (__builtin_expect(!rs_ok, 0)) return false;
    unsigned long long t_k = STAMP_T();
    const bool kok = kkt_check(P, lab, x, y, nl);
    STAMP_ADD(NV == 1 ? ST_XKKT : ST_ZKKT, t_k);
    if (__builtin_expect(kok, 1)) return true;
    bool same = true;
#pragma unroll
    for (int s = 0; s < NR; ++s) same &= (nl[s] == lab[s]);
    if (wall(same)) return false;
#pragma unroll
    for (int s = 0; s < NR; ++s) lab[s] = nl[s];
  }
  return false;
}


// ============================================================ dual active set (pair QP)
// Goldfarb-Idnani dual active-set method on the pair QP in hinge form, in Schur-complement
// form.  From the unconstrained minimiser x0 = -P^-1 q it adds the most violated one-sided
// constraint n_p'x >= b_p at a time (box/rate row r: side 0 = a_r'x >= lo, side 1 =
// -a_r'x >= -hi; hinge row: a_r'x >= h with multiplier cap beta), taking partial (dual)
// steps that drop a constraint whose multiplier reaches 0.  The active set's Schur complement
// S = N P^-1 N' is kept as its EXPLICIT INVERSE (LDS, lane = column, symmetric, any order of the
// active constraints): an add borders it (r = S^-1 v, delta = s_pp - v'r: S^-1 += r r'/delta plus
// one row and column), a drop downdates it (S^-1 - c c'/d over the other rows) and moves the last
// active constraint into the freed slot.  Every piece is an m-term lane-parallel pass over LDS
// (one broadcast operand per term, batched loads) -- no sequential triangular solve: on a
// wave the m-step readlane chains of a Cholesky factor cost ~170 cycles per step (r03 stamps,
// tools/graph_stamps.py), the parallel passes a few cycles per term.  Y holds the columns
// P^-1 n_a.  The final answer is the equality-constrained minimiser on the final active set with
// three steps of iterative refinement against the exact residual A_W x - b (x from Y, so S is
// never needed explicitly); the KKT certificate judges it either way.  On the recorded bench
// pair QPs (tools/gi_sim.py) the method certifies every one in 28 steps on average (max 51)
// where ADMM + PDAS took ~45 ADMM iterations and ~6 full reduced solves.  A hinge multiplier
// reaching the cap, a full set or the step limit return false and the caller falls back to
// ADMM + PDAS; the result is certified by the same KKT test either way.

// (LDS-typed views ldsd / lds_ptr / in_lds: pd_common.h)

// The broadcast operand of an m-term pass: vbuf[a] = v (lanes a < m), 0 up to lane 63, so the
// batched loads of a pass (never beyond lane 63: m <= 63, batches of 8 from multiples of 8) need
// no bounds test and use immediate offsets.
__device__ __forceinline__ void put_bcast(ldsd* vb, double v, int m) {
  const int l = lid();
  vb[l] = (l < m) ? v : 0.0;
  wsync();
}

// r = S^-1 v over the m active constraints (v, r at lanes a < m): lane = column of the symmetric
// inverse (LDS, stride ld), v broadcast from LDS (vbuf: 64 doubles of the wave's vector buffer).
constexpr int SINV_U = 8;
__device__ __forceinline__ double sinv_gemv(double* Si_, int ld_, double* vbuf_, double v, int m_) {
  const int l = lid();
  const int m = unif(m_), ld = unif(ld_);
  ldsd* vb = lds_ptr(vbuf_);
  const ldsd* col = lds_ptr(Si_) + ((l < m) ? l : 0);
  put_bcast(vb, v, m);
  double a0 = 0.0, a1 = 0.0;
  for (int j0 = 0; j0 < m; j0 += SINV_U) {
    double sv[SINV_U], vv[SINV_U];
#pragma unroll
    for (int u = 0; u < SINV_U; ++u) {
      sv[u] = col[unif(min(j0 + u, m - 1) * ld)];
      vv[u] = vb[j0 + u];
    }
#pragma unroll
    for (int u = 0; u < SINV_U; u += 2) {
      a0 += sv[u] * vv[u];
      a1 += sv[u + 1] * vv[u + 1];
    }
  }
  wsync();
  return (l < m) ? a0 + a1 : 0.0;
}

// z[v] -= sum_{a < m} coef_a Y[a][v] (lane = variable; coef at lanes a < m, broadcast from LDS).
template <int NV, typename YP>
__device__ __forceinline__ void y_axpy_t(YP Y, int H_, ldsd* vb, int m_, double* z) {
  const int l = lid(), H = unif(H_), m = unif(m_), H2 = NV * H;
  const int lc = (l < H) ? l : 0;
  const auto Yl = Y + lc;
  for (int a0 = 0; a0 < m; a0 += SINV_U) {
    double yv[SINV_U][NV], cv[SINV_U];
#pragma unroll
    for (int u = 0; u < SINV_U; ++u) {
      const int a = unif(min(a0 + u, m - 1));
      cv[u] = vb[a0 + u];
#pragma unroll
      for (int v = 0; v < NV; ++v) yv[u][v] = Yl[unif(a * H2 + v * H)];
    }
#pragma unroll
    for (int u = 0; u < SINV_U; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) z[v] -= cv[u] * yv[u][v];
  }
}
template <int NV>
__device__ __forceinline__ void y_axpy(double* Y, int H, double* vbuf_, double coef, int m, double* z) {
  ldsd* vb = lds_ptr(vbuf_);
  put_bcast(vb, coef, m);
  if (in_lds(Y)) y_axpy_t<NV>((const ldsd*)lds_ptr(Y), H, vb, m, z);
  else y_axpy_t<NV>(gbl_ptr((const double*)Y), H, vb, m, z);   // big mode: the columns in HBM / L2
  wsync();
}

// ---- Row-access passes (graph kernel, LDS mode: gi_solve<NV, RM_S | RM_Y>).  Lane a walks ROW a of the
// symmetric S^-1 (the same matrix and storage; stride ld rounded up to even, so each row starts
// on 16 bytes) and of the transposed columns Yt[v*H + l][a] (stride P.yld), two doubles per LDS
// access (ds_read_b128 / ds_write_b128) instead of one: tools/gi_ubench.hip measured the m = 50
// passes at 1312 / 1836 / 3336 cycles (S^-1 v / Y axpy / bordering) against 2212 / 2920 / 5252
// for the lane = column passes.  Row entries beyond m hold other data (the region also serves
// the PDAS factor), so the last partial batch masks them.
constexpr int RM_S = 1, RM_Y = 2;   // gi_solve's row-access modes
constexpr int RM_T = 4;             // the x-step's parametric tables transposed (param_build_x TT)
__device__ __forceinline__ int rows_ld(int fld) { return (fld + 1) & ~1; }

// row[j] += coef * vb[j] over j < m (one lane's row of S^-1; the last batch's entries beyond m
// are written back unchanged: vb is zero there)
__device__ __forceinline__ void rank1_row(ldsd* row_, const ldsd* vb, double coef, int m_) {
  const int m = unif(m_);
  ldsd2* row = (ldsd2*)row_;
  const ldsd2* v2 = (const ldsd2*)vb;
  for (int j0 = 0; j0 < m; j0 += 8) {
    dv2 sv[4], wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sv[u] = row[(j0 >> 1) + u];
      wv[u] = v2[(j0 >> 1) + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sv[u].x += wv[u].x * coef;
      sv[u].y += wv[u].y * coef;
      row[(j0 >> 1) + u] = sv[u];
    }
  }
}

__device__ __forceinline__ double sinv_rows(double* Si_, int ld_, double* vbuf_, double v, int m_) {
  const int l = lid();
  const int m = unif(m_), ld = unif(ld_);
  ldsd* vb = lds_ptr(vbuf_);
  put_bcast(vb, v, m);
  const ldsd2* row = (const ldsd2*)(lds_ptr(Si_) + ((l < m) ? l : 0) * ld);
  const ldsd2* v2 = (const ldsd2*)vb;
  double a0 = 0.0, a1 = 0.0;
  const int mf = m & ~7;
  for (int j0 = 0; j0 < mf; j0 += 8) {
    dv2 sv[4], wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sv[u] = row[(j0 >> 1) + u];
      wv[u] = v2[(j0 >> 1) + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0 += sv[u].x * wv[u].x;
      a1 += sv[u].y * wv[u].y;
    }
  }
  if (mf < m) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (mf + 2 * u < m) {
        const dv2 sv = row[(mf >> 1) + u], wv = v2[(mf >> 1) + u];
        a0 += sv.x * wv.x;
        if (mf + 2 * u + 1 < m) a1 += sv.y * wv.y;
      }
    }
  }
  wsync();
  return (l < m) ? a0 + a1 : 0.0;
}

// z[v] -= sum_{a < m} coef_a Yt[v*H + l][a] (lane = variable)
template <int NV>
__device__ __forceinline__ void y_axpy_rows(double* Y_, int H_, int yld_, double* vbuf_, double coef, int m_,
                                            double* z) {
  const int l = lid(), H = unif(H_), m = unif(m_), yld = unif(yld_);
  ldsd* vb = lds_ptr(vbuf_);
  put_bcast(vb, coef, m);
  const int lc = (l < H) ? l : 0;
  const ldsd2* yr[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) yr[v] = (const ldsd2*)(lds_ptr(Y_) + (v * H + lc) * yld);
  const ldsd2* c2 = (const ldsd2*)vb;
  const int mf = m & ~7;
  for (int a0 = 0; a0 < mf; a0 += 8) {
    dv2 cv[4], yv[4][NV];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      cv[u] = c2[(a0 >> 1) + u];
#pragma unroll
      for (int v = 0; v < NV; ++v) yv[u][v] = yr[v][(a0 >> 1) + u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) z[v] -= cv[u].x * yv[u][v].x + cv[u].y * yv[u][v].y;
  }
  if (mf < m) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (mf + 2 * u < m) {
        const dv2 cv = c2[(mf >> 1) + u];
        const bool two = mf + 2 * u + 1 < m;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const dv2 yv = yr[v][(mf >> 1) + u];
          z[v] -= two ? cv.x * yv.x + cv.y * yv.y : cv.x * yv.x;
        }
      }
    }
  }
  wsync();
}

template <bool ROWS>
__device__ __forceinline__ double sinv_any(double* Si, int ld, double* vbuf, double v, int m) {
  if constexpr (ROWS) return sinv_rows(Si, ld, vbuf, v, m);
  else return sinv_gemv(Si, ld, vbuf, v, m);
}
template <int NV, bool ROWS>
__device__ __forceinline__ void y_axpy_any(double* Y, int H, int yld, double* vbuf, double coef, int m, double* z) {
  if constexpr (ROWS) y_axpy_rows<NV>(Y, H, yld, vbuf, coef, m, z);
  else y_axpy<NV>(Y, H, vbuf, coef, m, z);
}
// P^-1 n for the one-sided constraint (row id, sign sg): lane = variable (one value per vehicle)
template <int NV>
__device__ __forceinline__ void pinv_row(const QP<NV>& P, int row, double sg, double* out) {
  const int l = lid(), H = P.H;
  const int lc = (l < H) ? l : 0;
  const RowT r = row_terms(P, row);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int i = v * H + lc;
    double val;
    if (NV == 2 && r.hk >= 0) {
      val = (v ? P.g2 : P.g1) * P.Pinv[4 * H * H + r.hk * P.n + i];
    } else {
      val = r.c0 * P.Pinv[r.i0 * P.n + i] + r.c1 * P.Pinv[r.i1 * P.n + i];
    }
    out[v] = (l < H) ? sg * val : 0.0;
  }
}

// The pair's warm build split over two waves (r06): a helper wave computes each stored row's
// P^-1 n (the Y column), A y and so the row's entries n_j' y against every earlier warm row, and
// hands them over through a small LDS ring; the pair wave keeps only the S^-1 pass, the pivot and
// the bordering.  The values are those the pair wave would compute itself (the same pinv_row and
// A_mul, read through shuffles instead of the vb_ax buffer), so the build is bit-identical.
// (LDS mode only, H <= WPIPE_HMAX: piadmm_internal.h; the ring follows S.sc)
constexpr int WP_R = 3;                 // ring slots
constexpr int WP_SLOT = 2 * 32 + 64 + 2;  // per slot: y (2 vehicles x H <= 32 lanes), n_j' y (64 rows), n_p' y_p, pad
constexpr int WP_DBL = 4 + WP_R * WP_SLOT;  // g1, g2, the P^-1 pointer, pad, then the slots
struct WarmPipe {
  double* dat;     // LDS: WP_DBL doubles
  int* hdr;        // LDS, after dat: [0] rows gm (0: no pipelined build this step), [1] rows
                   // consumed, [2 .. 2 + WP_R) slot ready (row index + 1), [8 .. 72) the rows' codes
};
// The pair's stored active set as this step's warm rows: lane i gets the code of row i (-1: not
// used) -- this step's set as stored, or the previous step's shifted one time slot.  Returns the
// row count, 0 when there is no usable set.
template <int NV>
__device__ __forceinline__ int warm_codes(const QP<NV>& P, int& code) {
  const int l = lid(), H = P.H;
  code = -1;
  const int gm = P.gws[0], gt = P.gws[1];
  const bool same = gt == P.tstep, prev = gt == P.tstep - 1;
  if (!((same || prev) && gm > 0 && gm <= WAVE)) return 0;
  code = (l < gm) ? P.gws[2 + l] : -1;
  if (prev && code >= 0) {
    const int row = code >> 1, s0 = row / H, k = row - s0 * H;
    const bool keep = P.hinge(s0) ? (k >= 2) : (k >= 1);
    code = keep ? 2 * (row - 1) + (code & 1) : -1;
  }
  // a kink held from its upper side (a linear row) restarts as the lower side (regimes
  // start at zero; both sides are the same equality a'x = h)
  if (code >= 0 && P.hinge((code >> 1) / H)) code &= ~1;
  if (NV == 2 && P.g1 == 0.0 && P.g2 == 0.0 && code >= 0 && P.hinge((code >> 1) / H)) code = -1;
  return gm;
}

// The helper wave's half of the pipelined warm build: rows 0 .. gm-1 of the codes the pair wave
// published before the setup barrier, each into ring slot i % WP_R once the pair has taken row
// i - WP_R out of it.  Every row is handed over (a row that is not appended just carries no data),
// so both loops run exactly gm times.
__device__ __forceinline__ void warm_help(const WarmPipe& wp, int H) {
  const int gm = wp.hdr[0];
  if (gm <= 0) return;
  const int l = lid();
  QP<2> Q;                          // the fields pinv_row and A_mul read
  Q.H = H;
  Q.n = 2 * H;
  Q.g1 = wp.dat[0];
  Q.g2 = wp.dat[1];
  Q.Pinv = reinterpret_cast<const double*>(reinterpret_cast<const unsigned long long*>(wp.dat)[2]);
  const int code = (l < gm) ? wp.hdr[8 + l] : -1;
  const int rowj = code >= 0 ? code >> 1 : 0, sj = rowj / H, kj = rowj - sj * H;
  const double sgj = (code & 1) ? -1.0 : 1.0;
  for (int i = 0; i < gm; ++i) {
    const int pc = rdli(code, i);
    const int sl = i % WP_R;
    if (i >= WP_R)
      while (__hip_atomic_load(&wp.hdr[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < i + 1 - WP_R)
        __builtin_amdgcn_s_sleep(1);
    double* sd = wp.dat + 4 + sl * WP_SLOT;
    if (pc >= 0) {
      const int prow = pc >> 1;
      const double sgp = (pc & 1) ? -1.0 : 1.0;
      double yp[2], ay[QP<2>::NR];
      pinv_row(Q, prow, sgp, yp);
      A_mul(Q, yp, ay);
      // (A y)[s H + k] is lane k's ay[s]: row j's entry n_j' y = sg_j (A y)[row_j], and the pivot's
      // n_p' y_p = sg_p (A y)[row_p] -- the products prep and nvec form from the vb_ax buffer
      double at[QP<2>::NR];
#pragma unroll
      for (int s = 0; s < QP<2>::NR; ++s) at[s] = __shfl(ay[s], kj);
      double aj = at[0];
#pragma unroll
      for (int s = 1; s < QP<2>::NR; ++s)
        if (sj == s) aj = at[s];
      const int sp = prow / H, kp = prow - sp * H;
      double ap = 0.0;
#pragma unroll
      for (int s = 0; s < QP<2>::NR; ++s)
        if (sp == s) ap = __shfl(ay[s], kp);
      if (l < 32)
#pragma unroll
        for (int v = 0; v < 2; ++v) sd[v * 32 + l] = yp[v];   // (lanes >= H hold 0: H <= 32)
      sd[64 + l] = sgj * aj;
      if (l == 0) sd[128] = sgp * ap;
    }
    // (release: the slot's stores complete before the flag)
    if (l == 0) __hip_atomic_store(&wp.hdr[2 + sl], i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

constexpr int GI_MAX_STEPS = 1024;   // a cold pair QP at H = 30 with most rows active takes ~300 adds + drops
constexpr int GI_WS = 2 + WAVE;   // per-pair warm working set in HBM: m, step t, codes
// Warm start (receding horizon): the previous MPC step's final active set, shifted one time
// slot (tools/gi_sim.py + the warm-start prototype: 28 -> 3.6 GI steps per bench pair QP),
// is appended row by row (dependent rows skipped), its equality-constrained minimiser formed
// and constraints with negative (or beyond-cap) multipliers dropped until the start is dual
// feasible -- the state GI requires -- before the usual adds.  Any starting set is only a
// guess: the minimiser and its certificate do not depend on it.
#ifdef PIADMM_GI_DEBUG
#define GI_DBG(...) do { if (lid() == 0) printf(__VA_ARGS__); } while (0)
#else
#define GI_DBG(...) ((void)0)
#endif
// RM: row-access passes (bit RM_S: S^-1; bit RM_Y: the transposed Y columns); 0 = lane = column
template <int NV, int RM = 0>
__device__ __forceinline__ bool gi_solve(QP<NV>& P, const signed char* wlab, signed char* lab, double* x, double* y,
                                         int& nsteps, signed char* flab = nullptr, bool use_wlab = true,
                                         bool prebuild = false, const WarmPipe* wp = nullptr) {
  // (prebuild: only append the pair's stored active set -- S^-1, the Y columns and the codes
  // depend on the step's geometry, not on q -- and return; the next solve of this QP starts from
  // it.  The pair wave does it while the agents' first x-steps run.)
  // (use_wlab = false: a cold start although wlab points at labels -- a flag, not a null
  // pointer selected at the call site, so that the caller's label array stays in registers)
  constexpr int NR = QP<NV>::NR;
  constexpr bool RS = (RM & RM_S) != 0, RY = (RM & RM_Y) != 0;
  const int l = lid(), H = P.H, ld = RS ? rows_ld(P.fld) : P.fld, H2 = NV * H;
  double* vb_ax = P.vb + 192;      // [192, 192 + NR*H): (A v) by row id
  double* vbuf = P.vb + 128;       // [128, 192): broadcast operand of the LDS passes
  int* wc = P.ib;                  // active constraint codes 2*row + side
  double* Si = P.fac;              // S^-1 (m x m, lane = column, stride ld; LDS in every mode)
  ldsd* Sil = lds_ptr(Si);
  ldsd* vbl = lds_ptr(vbuf);
  double* Y = P.Y;
  // element (a, v, l) of the dual active-set columns: column a (lane = variable), or row v*H + l
  // of the transposed layout (RY)
  const int yld = RY ? unif(P.yld) : 0;
  auto yi = [&](int a, int v, int ll) -> int { return RY ? (v * H + ll) * yld + a : a * H2 + v * H + ll; };
  const int cap = min(P.mmax - 1, P.ycap);
  P.gi_full = false;
  if (P.y_in_k) P.kready = false;  // Y overwrites the K_s^-1 region
  if (l == 0) P.fstate[0] = -1;    // and S^-1 the cached PDAS factor
  P.csig = -1;                     // (x-step: the factor scratch the parametric tables were built in)
  double x0[NV], xc[NV];
  int m = 0, wbits = 0;
  double ua = 0.0;                 // lane a < m: multiplier of active constraint a
  // Pair: hinge rows in their linear regime (this lane's hinge row).  A hinge row's multiplier
  // is bounded, u in [0, beta] (dual of beta max(0, h - a'x)): when a step takes it to beta the
  // row turns linear -- its term beta (h - a'x) moves into q, i.e. x0 += beta P^-1 n, and the
  // row leaves the active set -- and the search then watches the other side of the kink
  // (a'x <= h, normal -a, multiplier v = beta - u): an active upper side whose v reaches beta
  // turns the row back to its zero regime (x0 += beta P^-1 n again).  Both events keep the
  // iterate stationary and dual feasible, so the dual active set continues in place (a bounded
  // dual method): no restart, no cycling between the regimes.
  // (a restored active set of this step comes with its hinge regimes: gi_snap_restore)
  bool lin = (!prebuild && P.pre_m >= 0) ? P.pre_lin : false;
  auto start = [&]() {
    double qt[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) qt[v] = P.q[v];
    if constexpr (NV == 2) {
      const double tt = Tt_apply((P.valid(4) && lin) ? 1.0 : 0.0);
      if (l < H) {
        qt[0] -= P.beta * P.g1 * tt;
        qt[1] -= P.beta * P.g2 * tt;
      }
    }
    gemv_sym<true>(P, P.Pinv, qt, x0);
#pragma unroll
    for (int v = 0; v < NV; ++v) xc[v] = x0[v] = -x0[v];
    m = 0;
    wbits = 0;
    ua = 0.0;
  };

  // y_p = P^-1 n_p (lane = variable), A y_p to vb_ax; returns n_p' P^-1 n_p
  auto prep = [&](int pc, double* yp) -> double {
    const int prow = pc >> 1;
    const double sgp = (pc & 1) ? -1.0 : 1.0;
    pinv_row(P, prow, sgp, yp);
    double ay[NR];
    A_mul(P, yp, ay);
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = ay[s];
    }
    wsync();
    return sgp * vb_ax[prow];
  };
  // v = N y_p for the current active set (lane a < m)
  auto nvec = [&]() -> double {
    const int myc = (l < m) ? wc[l] : 0;
    return (l < m) ? ((myc & 1) ? -1.0 : 1.0) * vb_ax[myc >> 1] : 0.0;   // n_a' y_p
  };
  // append constraint pc: border S^-1 with r = S^-1 v and delta = n_p'y_p - v'r; Y column m = y_p
  auto append = [&](int pc, const double* yp, double r, double delta, double u0) {
    const int prow = pc >> 1, ps = prow / H, pk = prow - ps * H;
    const double id = 1.0 / delta;
    put_bcast(vbl, r, m);
    if (l < m) {
      const double rl = r * id;
      if constexpr (RS) {
        rank1_row(Sil + l * ld, vbl, rl, m);
      } else {
        ldsd* col = Sil + l;
        const int mu = unif(m), ldu = unif(ld);
        for (int j0 = 0; j0 < mu; j0 += SINV_U) {
          double sv[SINV_U], rv[SINV_U];
#pragma unroll
          for (int u = 0; u < SINV_U; ++u) {
            sv[u] = col[unif(min(j0 + u, mu - 1) * ldu)];
            rv[u] = vbl[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < SINV_U; ++u)
            if (j0 + u < mu) col[unif((j0 + u) * ldu)] = sv[u] + rv[u] * rl;
        }
      }
      Sil[m * ld + l] = -rl;      // row m, column l
      Sil[l * ld + m] = -rl;      // row l, column m
    }
    if (l == m) {
      Sil[m * ld + m] = id;
      ua = u0;
      wc[m] = pc;
    }
    if (l < H) {
#pragma unroll
      for (int v = 0; v < NV; ++v) Y[yi(m, v, l)] = yp[v];
    }
    if (l == pk) wbits |= 1 << (2 * ps + (pc & 1));
    ++m;
    if (P.gmem) gsync();
    else wsync();
  };
  // drop active constraint k: S^-1 of the others = S^-1 - c c'/d (c = column k, d = its diagonal),
  // then the last active constraint moves into slot k (row, column, code, multiplier, Y column)
  auto drop = [&](int k) {
    unsigned long long t_dr = STAMP_T();
    if (NV == 2) STAMP_CNT(ST_N_DROP, 1);
    const int kc = rdli((l < m) ? wc[l] : 0, k);
    if (l == (kc >> 1) % H) wbits &= ~(1 << (2 * ((kc >> 1) / H) + (kc & 1)));
    const double c = (l < m) ? Sil[k * ld + l] : 0.0;
    const double d = rdl(c, k);
    put_bcast(vbl, c, m);
    if (l < m && l != k) {
      const double cl = c / d;
      if constexpr (RS) {
        rank1_row(Sil + l * ld, vbl, -cl, m);
      } else {
        ldsd* col = Sil + l;
        const int mu = unif(m), ldu = unif(ld);
        for (int j0 = 0; j0 < mu; j0 += SINV_U) {
          double sv[SINV_U], cv[SINV_U];
#pragma unroll
          for (int u = 0; u < SINV_U; ++u) {
            sv[u] = col[unif(min(j0 + u, mu - 1) * ldu)];
            cv[u] = vbl[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < SINV_U; ++u)
            if (j0 + u < mu) col[unif((j0 + u) * ldu)] = sv[u] - cv[u] * cl;
        }
      }
    }
    wsync();
    const int last = m - 1;
    if (k != last) {
      // row last -> row k (lane b = column b < last; column k takes the diagonal of last)
      if (l < last) {
        const double v = Sil[last * ld + (l == k ? last : l)];
        Sil[k * ld + l] = v;
      }
      wsync();
      // column last -> column k (lane a = row a < last, a != k)
      if (l < last && l != k) {
        const double v = Sil[l * ld + last];
        Sil[l * ld + k] = v;
      }
      const int clast = wc[last];
      const double ulast = rdl(ua, last);
      if (l < H) {
#pragma unroll
        for (int v = 0; v < NV; ++v) Y[yi(k, v, l)] = Y[yi(last, v, l)];
      }
      wsync();
      if (l == k) {
        wc[k] = clast;
        ua = ulast;
      }
    }
    if (l >= last) ua = 0.0;
    --m;
    if (P.gmem) gsync();
    else wsync();
    if (NV == 2) STAMP_ADD(ST_GI_DROP, t_dr);
  };
  // multipliers of the equality-constrained minimiser on the active set (signed normals):
  // lam = S^-1 (N x0 - b); kernel multiplier of row a = sign_a * lam_a, GI multiplier -lam_a
  auto eqp_lam = [&](const double* xv) -> double {
    double ax0[NR];
    A_mul(P, xv, ax0);
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = ax0[s] - P.lo(s);   // lower-side residual
    }
    wsync();
    double rhs = 0.0;
    if (l < m) {
      const int myc = wc[l], rw = myc >> 1, rs = rw / H;
      // upper side (box / rate rows only, uniform bounds): -(a'x0 - hi)
      const double blo = P.hinge(rs) ? 0.0 : ((rs & 1) ? -P.dumax : -P.umax);   // hinge: hi = lo = h
      rhs = (myc & 1) ? -(vb_ax[rw] + blo + blo) : vb_ax[rw];
    }
    return sinv_any<RS>(Si, ld, vbuf, rhs, m);
  };
  auto x_of = [&](double lam) {
#pragma unroll
    for (int v = 0; v < NV; ++v) xc[v] = x0[v];
    y_axpy_any<NV, RY>(Y, H, yld, vbuf, lam, m, xc);
  };

  // On failure (flab != nullptr): the current working set as PDAS labels -- a start for the
  // polish instead of ADMM (a linear hinge row: HLINEAR, or HKINK with its upper side active).
  auto fail_labels = [&]() {
    if (!flab) return;
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      const bool lo_in = (wbits >> (2 * s)) & 1, hi_in = (wbits >> (2 * s + 1)) & 1;
      if (P.hinge(s)) flab[s] = (lo_in || hi_in) ? HKINK : (lin ? HLINEAR : HZERO);
      else flab[s] = lo_in ? LOWER : (hi_in ? UPPER : FREE);
      if (!P.valid(s)) flab[s] = 0;
    }
  };

  // warm row: append unless linearly dependent on the rows already in (multiplier set later)
  auto warm_add = [&](int pc) {
    if (m >= cap) return;
    double yp[NV];
    unsigned long long t_p = STAMP_T();
    const double spp = prep(pc, yp);
    const double va = nvec();
    if (NV == 2) STAMP_ADD(ST_WARM_PREP, t_p);
    unsigned long long t_s = STAMP_T();
    const double r = sinv_any<RS>(Si, ld, vbuf, va, m);
    const double delta = spp - wsum(va * r);
    if (NV == 2) STAMP_ADD(ST_WARM_SINV, t_s);
    unsigned long long t_a = STAMP_T();
    if (delta > DEP_TOL * spp) append(pc, yp, r, delta, 0.0);
    if (NV == 2) STAMP_ADD(ST_WARM_APPEND, t_a);
    if (NV == 2) STAMP_CNT(ST_N_WARMROW, 1);
  };
  if (prebuild) {
    m = 0;
    wbits = 0;
    ua = 0.0;
  } else {
    start();
  }
  bool warm = false;
  unsigned long long t_wb = STAMP_T();
  if (!prebuild && P.pre_m >= 0) {
    // the stored active set was appended before q was known (a prebuild): x0 is this call's
    m = P.pre_m;
    wbits = P.pre_wbits;
    P.pre_m = -1;
    warm = true;
  } else if (P.gws && P.gws_warm) {
    // ---- pair: the stored active set (this step's, or the previous step's shifted)
    int code;
    const int gm = warm_codes(P, code);
    if (gm > 0) {
      if (NV == 2 && wp && prebuild) {
        // the helper wave's rows (WarmPipe): the same values warm_add's prep and nvec compute
        int wj = 0;                                    // lane a < m: warm row index of active slot a
        for (int i = 0; i < gm; ++i) {
          const int pc = rdli(code, i);
          const int sl = i % WP_R;
          while (__hip_atomic_load(&wp->hdr[2 + sl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != i + 1)
            __builtin_amdgcn_s_sleep(1);
          const double* sd = wp->dat + 4 + sl * WP_SLOT;
          double yp[NV];
#pragma unroll
          for (int v = 0; v < NV; ++v) yp[v] = (l < 32) ? sd[v * 32 + l] : 0.0;
          const double gl = sd[64 + l];
          const double spp = sd[128];
          const double gs = __shfl(gl, wj);
          const double va = (l < m) ? gs : 0.0;          // n_a' y_p, a in the active set
          // (release: the slot's loads are done before it is handed back)
          if (l == 0) __hip_atomic_store(&wp->hdr[1], i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (pc < 0 || m >= cap) continue;
          unsigned long long t_s = STAMP_T();
          const double r = sinv_any<RS>(Si, ld, vbuf, va, m);
          const double delta = spp - wsum(va * r);
          STAMP_ADD(ST_WARM_SINV, t_s);
          unsigned long long t_a = STAMP_T();
          if (delta > DEP_TOL * spp) {
            if (l == m) wj = i;
            append(pc, yp, r, delta, 0.0);
          }
          STAMP_ADD(ST_WARM_APPEND, t_a);
          STAMP_CNT(ST_N_WARMROW, 1);
        }
      } else {
        for (int i = 0; i < gm; ++i) {
          const int pc = rdli(code, i);
          if (pc >= 0) warm_add(pc);
        }
      }
      warm = true;
    }
  } else if (wlab && use_wlab) {
    // ---- x-step: the rows the current labels hold at a bound
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      const bool in = P.valid(s) && wlab[s] != 0;
      unsigned long long bm = __ballot(in);
      const int side = (!P.hinge(s) && wlab[s] == UPPER) ? 1 : 0;
      while (bm) {
        const int k = __ffsll(bm) - 1;
        bm &= bm - 1;
        warm_add(2 * (s * H + k) + rdli(side, k));
      }
    }
    warm = true;
  }
  STAMP_ADD(NV == 2 ? ST_ZR_GEMV : ST_ZR_X, t_wb);
  if (prebuild) {
    P.pre_m = warm ? m : -1;
    P.pre_wbits = wbits;
    wsync();
    return true;
  }
  unsigned long long t_wf = STAMP_T();
  if (warm) {
    {
      // dual feasibility: drop the most negative (or beyond-cap hinge) multiplier until none
      double lam = 0.0;
      while (m > 0) {
        lam = eqp_lam(x0);
        const int myc = (l < m) ? wc[l] : 0;
        const double u = -lam;
        double sc = 0.0;
        if (l < m) {
          if (u < 0.0) sc = u;
          else if (P.hinge((myc >> 1) / H) && u > P.beta) sc = P.beta - u;
        }
        const double smin = wmin(sc);
        if (!(smin < 0.0)) break;
        const int k = __ffsll((unsigned long long)__ballot(l < m && sc == smin)) - 1;
        drop(k);
      }
      ua = (l < m) ? -lam : 0.0;
      x_of(lam);
    }
  }
  STAMP_ADD(NV == 2 ? ST_ZR_S : ST_ZR_CHOL, t_wf);

  while (true) {
    unsigned long long t_gs = STAMP_T();
    // ---- most violated constraint outside the active set
    double ax[NR];
    A_mul(P, xc, ax);
    double best = 0.0;
    int code = -1;
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      if (!P.valid(s)) continue;
      const bool hl = P.hinge(s) && lin;        // linear hinge row: only its upper side a'x <= h
      const double tp = P.tol * (1.0 + fabs(P.lo(s)));
      if (!hl && !((wbits >> (2 * s)) & 1)) {
        const double sv = ax[s] - P.lo(s);
        if (sv < -tp && sv < best) { best = sv; code = 2 * (s * H + l); }
      }
      if ((hl || !P.hinge(s)) && !((wbits >> (2 * s + 1)) & 1)) {
        const double sv = (hl ? P.lo(s) : P.hi(s)) - ax[s];
        if (sv < -tp && sv < best) { best = sv; code = 2 * (s * H + l) + 1; }
      }
    }
    const double bmin = wmin(best);
    if (!(bmin < 0.0)) break;
    const int pl = __ffsll((unsigned long long)__ballot(code >= 0 && best == bmin)) - 1;
    const int pc = rdli(code, pl);
    const int prow = pc >> 1, pside = pc & 1, ps = prow / H, pk = prow - ps * H;
    const bool phinge = P.hinge(ps);
    double sp = rdl(pside ? (phinge ? P.lo(ps) : P.hi(ps)) - ax[ps] : ax[ps] - P.lo(ps), pk);   // slack of p (< 0)
    double yp[NV];
    const double spp = prep(pc, yp);       // n_p' P^-1 n_p
    double up = 0.0;
    STAMP_ADD(ST_GI_SEARCH, t_gs);
    while (true) {
      if (++nsteps > GI_MAX_STEPS) {
        GI_DBG("GI fail: step limit m=%d\n", m);
        fail_labels();
        return false;
      }
      unsigned long long t_gv = STAMP_T();
      if (NV == 2) STAMP_CNT(ST_SUM_M, m);
      const double va = nvec();
      const double r = sinv_any<RS>(Si, ld, vbuf, va, m);     // S^-1 N y_p
      if (NV == 2) STAMP_ADD(ST_GI_FWD, t_gv);
      unsigned long long t_yp = STAMP_T();
      // z = y_p - Y r
      double z[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) z[v] = yp[v];
      y_axpy_any<NV, RY>(Y, H, yld, vbuf, r, m, z);
      const double lpp2 = spp - wsum(va * r);                  // n_p' z
      if (NV == 2) STAMP_ADD(ST_GI_YPASS, t_yp);
      STAMP_ADD(ST_GI_SOLVE, t_gv);
      unsigned long long t_gu = STAMP_T();
      const double t2 = (lpp2 > DEP_TOL * spp) ? -sp / lpp2 : INFINITY;
      // dual step limits: an active multiplier reaching 0 (drop) or a hinge one reaching beta
      const int myc = (l < m) ? wc[l] : 0;
      const bool hin_a = (l < m) && P.hinge((myc >> 1) / H);
      const double tdrop = (l < m && r > 0.0) ? ua / r : INFINITY;
      const double tcap = (hin_a && r < 0.0) ? (P.beta - ua) / (-r) : INFINITY;
      const double t1 = wmin(tdrop);
      const double tc = fmin(wmin(tcap), phinge ? P.beta - up : INFINITY);
      const double t = fmin(t1, t2);
      if (tc <= t) {
        // a hinge multiplier reaches its bound beta: step there, then the row changes regime
        // (lower side -> linear, upper side -> zero) and its constraint leaves the active set
        const double tca = wmin(tcap);
        const bool entering = phinge && P.beta - up <= tca;
        if (t2 < INFINITY) {
#pragma unroll
          for (int v = 0; v < NV; ++v) xc[v] += tc * z[v];
          sp += tc * lpp2;
        }
        if (l < m) ua -= tc * r;
        up += tc;
        if (entering) {
          if (l == pk) lin = pside == 0;
#pragma unroll
          for (int v = 0; v < NV; ++v) x0[v] += P.beta * yp[v];
          STAMP_ADD(ST_GI_UPD, t_gu);
          break;                                     // p never enters: next search
        }
        const int k = __ffsll((unsigned long long)__ballot(l < m && hin_a && tcap == tca)) - 1;
        const int kc = rdli(myc, k), krow = kc >> 1;
        if (l == krow - (NV == 2 ? 4 : 0) * H) lin = (kc & 1) == 0;
        {
          const int lc = (l < H) ? l : 0;
#pragma unroll
          for (int v = 0; v < NV; ++v) x0[v] += P.beta * Y[yi(k, v, lc)];
        }
        drop(k);
        STAMP_ADD(ST_GI_UPD, t_gu);
        continue;                                    // the same p, a new step direction
      }
      if (!(t < INFINITY)) {                         // unbounded dual step
        GI_DBG("GI fail: unbounded dual step m=%d lpp2=%g spp=%g sp=%g\n", m, lpp2, spp, sp);
        fail_labels();
        return false;
      }
      if (t2 < INFINITY) {
#pragma unroll
        for (int v = 0; v < NV; ++v) xc[v] += t * z[v];
        sp += t * lpp2;
      }
      if (l < m) ua -= t * r;
      up += t;
      if (t2 <= t1) {
        if (m >= cap) {
          GI_DBG("GI fail: full m=%d cap=%d\n", m, cap);
          P.gi_full = true;
          fail_labels();
          return false;
        }
        append(pc, yp, r, lpp2, up);
        if (NV == 2) STAMP_CNT(ST_N_APPEND, 1);
        STAMP_ADD(ST_GI_UPD, t_gu);
        break;
      }
      drop(__ffsll((unsigned long long)__ballot(l < m && tdrop == t1)) - 1);
      STAMP_ADD(ST_GI_UPD, t_gu);
    }
  }
  // ---- exact solution of the final active set: lam = S^-1 (N x0 - b), x = x0 - Y lam, then three
  // steps of iterative refinement on the active rows' exact residual A_W x - b (the inverse
  // carries the rounding of its updates; the residual is formed from Y and A, not from S^-1);
  // kernel multipliers y_a = sign_a * lam_a
  {
    double lam = eqp_lam(x0);
    x_of(lam);
#pragma unroll 1
    for (int rf = 0; rf < 3; ++rf) {
      const double dl = eqp_lam(xc);
      y_axpy_any<NV, RY>(Y, H, yld, vbuf, dl, m, xc);
      lam += dl;
    }
    const int myc = (l < m) ? wc[l] : 0;
    const int rw = myc >> 1;
    wsync();
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = 0.0;
    }
    wsync();
    if (l < m) vb_ax[rw] = (myc & 1) ? -lam : lam;
    wsync();
#pragma unroll
    for (int v = 0; v < NV; ++v) x[v] = (l < H) ? xc[v] : 0.0;
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      const bool lo_in = (wbits >> (2 * s)) & 1, hi_in = (wbits >> (2 * s + 1)) & 1;
      y[s] = (P.valid(s) && l < H && (lo_in || hi_in)) ? vb_ax[s * H + l] : 0.0;
      // linear hinge row: multiplier -beta, or -(beta - v) at a kink held from the upper side
      if (P.hinge(s) && lin && P.valid(s)) y[s] = hi_in ? y[s] - P.beta : -P.beta;
      if (P.hinge(s)) lab[s] = (lo_in || hi_in) ? HKINK : (lin ? HLINEAR : HZERO);
      else lab[s] = lo_in ? LOWER : (hi_in ? UPPER : FREE);
      if (!P.valid(s)) lab[s] = 0;
    }
    if (NV == 2) STAMP_CNT(ST_SUM_MEND, m);
    if (NV == 2) STAMP_CNT(ST_N_GICALL, 1);
    // this step's active set: the next solve's warm start
    if (P.gws) {
      if (l < m) P.gws[2 + l] = myc;
      if (l == 0) {
        P.gws[0] = m;
        P.gws[1] = P.tstep;
      }
      // and its S^-1 and Y columns (they depend on the step's geometry only, not on q): the pair's
      // next solve in this step restores them instead of appending the rows again
      if (P.snap) {
        double* sS = P.snap;
        double* sY = P.snap + WAVE * WAVE;
        for (int j = 0; j < m; ++j)
          if (l < m) sS[j * WAVE + l] = Sil[j * ld + l];
        if (l < H)
          for (int a = 0; a < m; ++a)
#pragma unroll
            for (int v = 0; v < NV; ++v) sY[a * H2 + v * H + l] = Y[yi(a, v, l)];
        sY[WAVE * H2 + l] = lin ? 1.0 : 0.0;   // the hinge regimes of the final state
      }
    }
    wsync();
  }
  return true;
}

// ---- Restore of a pair's dual active set within an MPC step (graph kernel).  The active set a
// pair's last solve ended with (P.gws: m, step, codes) comes with its S^-1 and Y columns
// (P.snap, written by gi_solve): in the same MPC step the pair's QP has the same P and rows --
// only q changed -- so the next solve starts from them (gi_solve's pre_m path: x0 from the new q,
// then the dual-feasibility drops) instead of appending the m rows again (one P^-1 column, one
// bordering pass each).  The hinge rows' regimes (linear or zero) of that final state come with
// it, so the solve resumes from exactly the state it ended in.  Not under the global-PI law (the
// pair's penalty changes every iteration).
template <int RM = 0>
__device__ __forceinline__ void gi_snap_restore(QP<2>& P) {
  constexpr int NV = 2;
  constexpr bool RS = (RM & RM_S) != 0, RY = (RM & RM_Y) != 0;
  const int l = lid(), H = P.H, H2 = NV * H, ld = RS ? rows_ld(P.fld) : P.fld;
  if (!P.snap || !P.gws || !P.gws_warm) return;
  const int gm = P.gws[0], gt = P.gws[1];
  if (gt != P.tstep || gm <= 0 || gm > min(P.mmax - 1, P.ycap)) return;
  const int code = (l < gm) ? P.gws[2 + l] : 0;
  const bool kill = (l < gm) && (code < 0 || (P.g1 == 0.0 && P.g2 == 0.0 && P.hinge((code >> 1) / H)));
  if (wany(kill)) return;
  ldsd* Sil = lds_ptr(P.fac);
  const double* sS = P.snap;
  const double* sY = P.snap + WAVE * WAVE;
  for (int j0 = 0; j0 < gm; j0 += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (l < gm && j0 + u < gm) ? sS[(j0 + u) * WAVE + l] : 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (l < gm && j0 + u < gm) Sil[(j0 + u) * ld + l] = v[u];
  }
  if (l < H) {
    for (int a0 = 0; a0 < gm; a0 += 4) {
      double v[4][NV];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w = 0; w < NV; ++w) v[u][w] = (a0 + u < gm) ? sY[(a0 + u) * H2 + w * H + l] : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int w = 0; w < NV; ++w)
          if (a0 + u < gm) P.Y[RY ? (w * H + l) * P.yld + a0 + u : (a0 + u) * H2 + w * H + l] = v[u][w];
    }
  }
  if (l < gm) P.ib[l] = code;
  P.pre_lin = sY[WAVE * H2 + l] != 0.0;
  int wb = 0;
  for (int a = 0; a < gm; ++a) {
    const int c = rdli(code, a), row = c >> 1, sl = row / H, k = row - sl * H;
    if (k == l) wb |= 1 << (2 * sl + (c & 1));
  }
  P.pre_m = gm;
  P.pre_wbits = wb;
  if (P.gmem) gsync();
  else wsync();
}

// ---- Wide dual active set: pair QPs whose working set outgrows one row per lane (saturated
// coupled pairs at H > 31: both vehicles' controls and rates at their bounds plus the hinge
// kinks, 78-79 active rows at H = 40-50 on the 4-vehicle crossings).  The same Goldfarb-Idnani
// method as gi_solve, cold-started, with two active rows per lane (rows a and a + 64 on lane
// a & 63): the multipliers and codes in registers, S^-1 (up to 126 x 126, symmetric, stored
// full) and the Y columns P^-1 n_a in the pair's HBM scratch (L2-resident), the broadcast
// operands in the wave's LDS factor region (free: S^-1 is in HBM).  Certified by kkt_check.
// (GIW_LD, GIW_CAP, giw_stride: piadmm_internal.h -- the host sizes the scratch)
constexpr int GIW_MAX_STEPS = 4096;
__device__ __forceinline__ bool gi_solve_wide(QP<2>& P, signed char* lab, double* x, double* y, int& nsteps) {
  constexpr int NV = 2, NR = QP<2>::NR;
  const int l = lid(), H = P.H, H2 = NV * H;
  gbld* S = gbl_ptr(P.wide);
  gbld* Yg = gbl_ptr(P.wide + (size_t)GIW_LD * GIW_LD);
  ldsd* B = lds_ptr(P.fac);                  // 128-double broadcast operand
  double* vb_ax = P.vb + 192;                // (A v) by row id, as gi_solve
  const int cap = min(GIW_CAP, H2);          // at most n independent rows
  if (l == 0) P.fstate[0] = -1;              // the LDS factor region is overwritten
  P.csig = -1;
  double x0[NV], xc[NV];
  int m = 0, wbits = 0;
  double ua[2] = {0.0, 0.0};                 // multipliers of active rows l, l + 64
  int wc[2] = {0, 0};                        // their codes 2*row + side
  bool lin = false;                          // this lane's hinge row in its linear regime
  auto start = [&]() {
    double qt[NV] = {P.q[0], P.q[1]};
    const double tt = Tt_apply((P.valid(4) && lin) ? 1.0 : 0.0);
    if (l < H) {
      qt[0] -= P.beta * P.g1 * tt;
      qt[1] -= P.beta * P.g2 * tt;
    }
    gemv_sym<true>(P, P.Pinv, qt, x0);
#pragma unroll
    for (int v = 0; v < NV; ++v) xc[v] = x0[v] = -x0[v];
  };
  // B[a] = v_a over the active rows (0 beyond m, up to 127)
  auto put2 = [&](double v0, double v1) {
    B[l] = (l < m) ? v0 : 0.0;
    B[WAVE + l] = (WAVE + l < m) ? v1 : 0.0;
    wsync();
  };
  // r = S^-1 v: lane owns columns l and l + 64
  auto sinv2 = [&](double v0, double v1, double* r) {
    put2(v0, v1);
    const int mu = unif(m);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cl = l + h * WAVE;
      const gbld* col = S + ((cl < mu) ? cl : 0);
      double a0 = 0.0, a1 = 0.0;
      if (h * WAVE < mu) {
        for (int j0 = 0; j0 < mu; j0 += SINV_U) {
          double sv[SINV_U], bv[SINV_U];
#pragma unroll
          for (int u = 0; u < SINV_U; ++u) {
            sv[u] = col[unif(min(j0 + u, mu - 1) * GIW_LD)];
            bv[u] = B[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < SINV_U; u += 2) {
            a0 += sv[u] * bv[u];
            a1 += sv[u + 1] * bv[u + 1];
          }
        }
      }
      r[h] = (cl < mu) ? a0 + a1 : 0.0;
    }
    wsync();
  };
  // z[v] -= sum_a c_a Y[a][v]
  auto yaxpy2 = [&](double c0, double c1, double* z) {
    put2(c0, c1);
    const int mu = unif(m);
    const int lc = (l < H) ? l : 0;
    for (int a0 = 0; a0 < mu; a0 += SINV_U) {
      double yv[SINV_U][NV], cv[SINV_U];
#pragma unroll
      for (int u = 0; u < SINV_U; ++u) {
        const int a = unif(min(a0 + u, mu - 1));
        cv[u] = B[a0 + u];
#pragma unroll
        for (int v = 0; v < NV; ++v) yv[u][v] = Yg[unif(a * H2 + v * H) + lc];
      }
#pragma unroll
      for (int u = 0; u < SINV_U; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) z[v] -= cv[u] * yv[u][v];
    }
    wsync();
  };
  auto prep = [&](int pc, double* yp) -> double {
    const int prow = pc >> 1;
    const double sgp = (pc & 1) ? -1.0 : 1.0;
    pinv_row(P, prow, sgp, yp);
    double ay[NR];
    A_mul(P, yp, ay);
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = ay[s];
    }
    wsync();
    return sgp * vb_ax[prow];
  };
  auto nvec = [&](double* va) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool in = l + h * WAVE < m;
      const int c = in ? wc[h] : 0;
      va[h] = in ? ((c & 1) ? -1.0 : 1.0) * vb_ax[c >> 1] : 0.0;
    }
  };
  auto append = [&](int pc, const double* yp, const double* r, double delta, double u0) {
    const int prow = pc >> 1, ps = prow / H, pk = prow - ps * H;
    const double id = 1.0 / delta;
    put2(r[0], r[1]);
    const int mu = unif(m);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cl = l + h * WAVE;
      if (cl < mu) {
        const double rl = r[h] * id;
        gbld* col = S + cl;
        for (int j0 = 0; j0 < mu; j0 += SINV_U) {
          double sv[SINV_U], rv[SINV_U];
#pragma unroll
          for (int u = 0; u < SINV_U; ++u) {
            sv[u] = col[unif(min(j0 + u, mu - 1) * GIW_LD)];
            rv[u] = B[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < SINV_U; ++u)
            if (j0 + u < mu) col[unif((j0 + u) * GIW_LD)] = sv[u] + rv[u] * rl;
        }
        S[mu * GIW_LD + cl] = -rl;      // row m, column cl
        S[cl * GIW_LD + mu] = -rl;      // row cl, column m
      }
    }
    if (l == (mu & (WAVE - 1))) {
      S[mu * GIW_LD + mu] = id;
      if (mu < WAVE) { ua[0] = u0; wc[0] = pc; }
      else { ua[1] = u0; wc[1] = pc; }
    }
    if (l < H) {
#pragma unroll
      for (int v = 0; v < NV; ++v) Yg[mu * H2 + v * H + l] = yp[v];
    }
    if (l == pk) wbits |= 1 << (2 * ps + (pc & 1));
    ++m;
    gsync();
  };
  auto drop = [&](int k) {
    const int kh = k >> 6, kl = k & (WAVE - 1);
    const int kc = rdli(kh ? wc[1] : wc[0], kl);
    if (l == (kc >> 1) % H) wbits &= ~(1 << (2 * ((kc >> 1) / H) + (kc & 1)));
    const int mu = unif(m);
    double c[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cl = l + h * WAVE;
      c[h] = (cl < mu) ? S[k * GIW_LD + cl] : 0.0;   // column k (symmetric)
    }
    const double d = rdl(kh ? c[1] : c[0], kl);
    put2(c[0], c[1]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cl = l + h * WAVE;
      if (cl < mu && cl != k) {
        const double cf = c[h] / d;
        gbld* col = S + cl;
        for (int j0 = 0; j0 < mu; j0 += SINV_U) {
          double sv[SINV_U], bv[SINV_U];
#pragma unroll
          for (int u = 0; u < SINV_U; ++u) {
            sv[u] = col[unif(min(j0 + u, mu - 1) * GIW_LD)];
            bv[u] = B[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < SINV_U; ++u)
            if (j0 + u < mu) col[unif((j0 + u) * GIW_LD)] = sv[u] - bv[u] * cf;
        }
      }
    }
    gsync();
    const int last = mu - 1;
    if (k != last) {
      // row last -> row k (column k takes the diagonal of last), then column last -> column k
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int cl = l + h * WAVE;
        if (cl < last) S[k * GIW_LD + cl] = S[last * GIW_LD + (cl == k ? last : cl)];
      }
      gsync();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int cl = l + h * WAVE;
        if (cl < last && cl != k) S[cl * GIW_LD + k] = S[cl * GIW_LD + last];
      }
      const int lh = last >> 6, ll = last & (WAVE - 1);
      const int clast = rdli(lh ? wc[1] : wc[0], ll);
      const double ulast = rdl(lh ? ua[1] : ua[0], ll);
      if (l < H) {
#pragma unroll
        for (int v = 0; v < NV; ++v) Yg[k * H2 + v * H + l] = Yg[last * H2 + v * H + l];
      }
      if (l == kl) {
        if (kh) { wc[1] = clast; ua[1] = ulast; }
        else { wc[0] = clast; ua[0] = ulast; }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (l + h * WAVE >= last) ua[h] = 0.0;
    --m;
    gsync();
  };
  // multipliers of the equality-constrained minimiser on the active set: lam = S^-1 (N xv - b)
  auto eqp_lam = [&](const double* xv, double* lam) {
    double ax0[NR];
    A_mul(P, xv, ax0);
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = ax0[s] - P.lo(s);
    }
    wsync();
    double rhs[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      rhs[h] = 0.0;
      if (l + h * WAVE < m) {
        const int myc = wc[h], rw = myc >> 1, rs = rw / H;
        const double blo = P.hinge(rs) ? 0.0 : ((rs & 1) ? -P.dumax : -P.umax);
        rhs[h] = (myc & 1) ? -(vb_ax[rw] + blo + blo) : vb_ax[rw];
      }
    }
    sinv2(rhs[0], rhs[1], lam);
  };
  auto x_of = [&](const double* lam) {
#pragma unroll
    for (int v = 0; v < NV; ++v) xc[v] = x0[v];
    yaxpy2(lam[0], lam[1], xc);
  };
  // first active row (by index) among lanes where pred holds for row l (h = 0) or l + 64 (h = 1)
  auto first_of = [&](bool p0, bool p1) -> int {
    const unsigned long long b0 = __ballot(p0);
    if (b0) return __ffsll(b0) - 1;
    return WAVE + __ffsll(__ballot(p1)) - 1;
  };

  start();
  while (true) {
    // ---- most violated constraint outside the active set
    double ax[NR];
    A_mul(P, xc, ax);
    double best = 0.0;
    int code = -1;
#pragma unroll
    for (int s = 0; s < NR; ++s) {
      if (!P.valid(s)) continue;
      const bool hl = P.hinge(s) && lin;
      const double tp = P.tol * (1.0 + fabs(P.lo(s)));
      if (!hl && !((wbits >> (2 * s)) & 1)) {
        const double sv = ax[s] - P.lo(s);
        if (sv < -tp && sv < best) { best = sv; code = 2 * (s * H + l); }
      }
      if ((hl || !P.hinge(s)) && !((wbits >> (2 * s + 1)) & 1)) {
        const double sv = (hl ? P.lo(s) : P.hi(s)) - ax[s];
        if (sv < -tp && sv < best) { best = sv; code = 2 * (s * H + l) + 1; }
      }
    }
    const double bmin = wmin(best);
    if (!(bmin < 0.0)) break;
    const int pl = __ffsll((unsigned long long)__ballot(code >= 0 && best == bmin)) - 1;
    const int pc = rdli(code, pl);
    const int prow = pc >> 1, pside = pc & 1, ps = prow / H, pk = prow - ps * H;
    const bool phinge = P.hinge(ps);
    double sp = rdl(pside ? (phinge ? P.lo(ps) : P.hi(ps)) - ax[ps] : ax[ps] - P.lo(ps), pk);
    double yp[NV];
    const double spp = prep(pc, yp);
    double up = 0.0;
    while (true) {
      if (++nsteps > GIW_MAX_STEPS) return false;
      double va[2], r[2];
      nvec(va);
      sinv2(va[0], va[1], r);
      double z[NV] = {yp[0], yp[1]};
      yaxpy2(r[0], r[1], z);
      const double lpp2 = spp - wsum(va[0] * r[0] + va[1] * r[1]);
      const double t2 = (lpp2 > DEP_TOL * spp) ? -sp / lpp2 : INFINITY;
      double tdrop[2], tcap[2];
      bool hin[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool in = l + h * WAVE < m;
        hin[h] = in && P.hinge((wc[h] >> 1) / H);
        tdrop[h] = (in && r[h] > 0.0) ? ua[h] / r[h] : INFINITY;
        tcap[h] = (hin[h] && r[h] < 0.0) ? (P.beta - ua[h]) / (-r[h]) : INFINITY;
      }
      const double t1 = wmin(fmin(tdrop[0], tdrop[1]));
      const double tca = wmin(fmin(tcap[0], tcap[1]));
      const double tc = fmin(tca, phinge ? P.beta - up : INFINITY);
      const double t = fmin(t1, t2);
      if (tc <= t) {
        const bool entering = phinge && P.beta - up <= tca;
        if (t2 < INFINITY) {
#pragma unroll
          for (int v = 0; v < NV; ++v) xc[v] += tc * z[v];
          sp += tc * lpp2;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (l + h * WAVE < m) ua[h] -= tc * r[h];
        up += tc;
        if (entering) {
          if (l == pk) lin = pside == 0;
#pragma unroll
          for (int v = 0; v < NV; ++v) x0[v] += P.beta * yp[v];
          break;
        }
        const int k = first_of(hin[0] && tcap[0] == tca, hin[1] && tcap[1] == tca);
        const int kc = rdli((k >> 6) ? wc[1] : wc[0], k & (WAVE - 1)), krow = kc >> 1;
        if (l == krow - 4 * H) lin = (kc & 1) == 0;
        {
          const int lc = (l < H) ? l : 0;
#pragma unroll
          for (int v = 0; v < NV; ++v) x0[v] += P.beta * Yg[k * H2 + v * H + lc];
        }
        drop(k);
        continue;
      }
      if (!(t < INFINITY)) return false;
      if (t2 < INFINITY) {
#pragma unroll
        for (int v = 0; v < NV; ++v) xc[v] += t * z[v];
        sp += t * lpp2;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (l + h * WAVE < m) ua[h] -= t * r[h];
      up += t;
      if (t2 <= t1) {
        if (m >= cap) return false;
        append(pc, yp, r, lpp2, up);
        break;
      }
      drop(first_of(l < m && tdrop[0] == t1, l + WAVE < m && tdrop[1] == t1));
    }
  }
  // ---- the final active set's exact solution, three refinement steps, kernel multipliers
  double lam[2];
  eqp_lam(x0, lam);
  x_of(lam);
#pragma unroll 1
  for (int rf = 0; rf < 3; ++rf) {
    double dl[2];
    eqp_lam(xc, dl);
    yaxpy2(dl[0], dl[1], xc);
    lam[0] += dl[0];
    lam[1] += dl[1];
  }
  wsync();
  if (l < H) {
#pragma unroll
    for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = 0.0;
  }
  wsync();
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (l + h * WAVE < m) vb_ax[wc[h] >> 1] = (wc[h] & 1) ? -lam[h] : lam[h];
  wsync();
#pragma unroll
  for (int v = 0; v < NV; ++v) x[v] = (l < H) ? xc[v] : 0.0;
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    const bool lo_in = (wbits >> (2 * s)) & 1, hi_in = (wbits >> (2 * s + 1)) & 1;
    y[s] = (P.valid(s) && l < H && (lo_in || hi_in)) ? vb_ax[s * H + l] : 0.0;
    if (P.hinge(s) && lin && P.valid(s)) y[s] = hi_in ? y[s] - P.beta : -P.beta;
    if (P.hinge(s)) lab[s] = (lo_in || hi_in) ? HKINK : (lin ? HLINEAR : HZERO);
    else lab[s] = lo_in ? LOWER : (hi_in ? UPPER : FREE);
    if (!P.valid(s)) lab[s] = 0;
  }
  wsync();
  return true;
}

// OSQP-style adaptive rho (in the scaled space): rho *= sqrt((|r_prim|/|Ax,z|) / (|r_dual|/|Px,A'y,q|)).
// Returns the proposed factor (1 when inside [0.2, 5]).
template <int NV>
__device__ __forceinline__ double rho_ratio(const QP<NV>& P, const double* xs, const double* zs, const double* ys) {
  constexpr int NR = QP<NV>::NR;
  double xu[NV], ax[NR], px[NV], w[NR], aty[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) xu[v] = P.D[v] * xs[v];
  A_mul(P, xu, ax);
  P_mul(P, xu, px);
#pragma unroll
  for (int s = 0; s < NR; ++s) w[s] = P.valid(s) ? P.E[s] * ys[s] : 0.0;
  At_mul(P, w, aty);
  double rp = 0.0, na = 0.0, rd = 0.0, nd = 0.0;
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    if (!P.valid(s)) continue;
    const double a = P.E[s] * ax[s];
    rp = fmax(rp, fabs(a - zs[s]));
    na = fmax(na, fmax(fabs(a), fabs(zs[s])));
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if (lid() >= P.H) continue;
    const double ps = P.D[v] * px[v], qs = P.D[v] * P.q[v], as = P.D[v] * aty[v];
    rd = fmax(rd, fabs(ps + qs + as));
    nd = fmax(nd, fmax(fabs(ps), fmax(fabs(qs), fabs(as))));
  }
  rp = wmax(rp);
  na = wmax(na);
  rd = wmax(rd);
  nd = wmax(nd);
  const double num = rp / fmax(na, 1e-30), den = rd / fmax(nd, 1e-30);
  const double ratio = sqrt(num / fmax(den, 1e-30));
  return (ratio > 5.0 || ratio < 0.2) ? ratio : 1.0;
}

// x-step: the linear term q = T'-apply(w') is formed only when a path other than the fused
// parametric pass needs it (dual active set, ADMM)
template <int NV>
__device__ __forceinline__ void ensure_q(QP<NV>& P) {
  if constexpr (NV == 1) {
    if (!P.qvalid) {
      const double qv = Tt_apply(P.wq);
      P.q[0] = (lid() < P.H) ? qv : 0.0;
      P.qvalid = true;
    }
  }
}

// Raw warm state (x, y of the last certified solve, unscaled) -> scaled ADMM state.
template <int NV>
__device__ __forceinline__ void warm_to_scaled(QP<NV>& P, double* xs, double* zs, double* ys) {
  constexpr int NR = QP<NV>::NR;
  double ax[NR];
  A_mul(P, xs, ax);
#pragma unroll
  for (int v = 0; v < NV; ++v) xs[v] = (P.D[v] != 0.0) ? xs[v] / P.D[v] : 0.0;
#pragma unroll
  for (int s = 0; s < NR; ++s) {
    zs[s] = P.valid(s) ? P.E[s] * ax[s] : 0.0;
    ys[s] = P.valid(s) ? ys[s] / P.E[s] : 0.0;
  }
  P.wraw = false;
}

// Solve one QP.  (xs, zs, ys) is the warm ADMM state (scaled), lab the warm labels.
// P.rho may be adapted (K^-1 rebuilt in the scratch kscr, stride kld) and persists.
// Returns PIADMM_QP_* flags; x_out = unscaled minimiser.
#ifndef PIADMM_ADAPT_EVERY
#define PIADMM_ADAPT_EVERY 25
#endif
constexpr int ADAPT_EVERY = PIADMM_ADAPT_EVERY;
template <int NV, bool TWO, int XU = XGEMV_U, int RM = 0>
__device__ __forceinline__ int qp_solve(QP<NV>& P, double* xs, double* zs, double* ys, signed char* lab,
                                        bool warm_lab, int max_inner, int polish_every, double* kscr, int kld,
                                        double* x_out, int& n_admm, int& n_pdas, int& n_gi,
                                        int gi_first = 0) {
  constexpr int NR = QP<NV>::NR;
  double x[NV], y[NR];
  bool ok = false;
  signed char flab[NR];   // labels a PDAS attempt already failed from
#pragma unroll
  for (int s = 0; s < NR; ++s) flab[s] = -1;
  if (warm_lab) {
#pragma unroll
    for (int s = 0; s < NR; ++s) flab[s] = lab[s];
    if (NV == 1 && P.ycap > 0) {
      // x-step: the warm labels' reduced solve (a cached-table hit in the steady state); when
      // its certificate fails, the dual active set warm-started from those labels finds the
      // new working set in a few steps, and one reduced solve on it certifies (instead of a
      // table rebuild per one-step PDAS label move, then ADMM)
      // Only when the parametric tables hold the warm labels' working set (a hit pass): a
      // reduced solve on other labels costs a table rebuild (~20 us) and after a dual update or
      // at a step's first x-QP (gi_first: the previous step's labels shifted) rarely certifies,
      // so the dual active set starts from those labels directly
      if ((gi_first == 0 || gi_first == 3) && tables_match(P, lab)) ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas, 1);
      if (__builtin_expect(!ok, 0)) {
        int ngi = 0;
        signed char glab[NR];
        ensure_q(P);
        if (gi_solve<NV, RM>(P, flab, glab, x, y, ngi, nullptr, gi_first < 2)) {
#pragma unroll
          for (int s = 0; s < NR; ++s) lab[s] = glab[s];
          // the dual active set's own answer (exact solve of its final working set + one step
          // of refinement), certified by the KKT test: no table rebuild here -- the parametric
          // tables of the new working set are built when a later x-QP tries these labels (in a
          // natural-termination step the last x-QP's tables are never used)
          bool stable = true;
#pragma unroll
          for (int s = 0; s < NR; ++s) stable &= !P.valid(s) || glab[s] == flab[s];
          if (wall(stable)) {
            // the working set held: build its tables now for the cheap hits that follow
            ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas);
          } else {
            signed char nl[NR];
            ok = kkt_check(P, lab, x, y, nl);
            if (!ok) ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas);
          }
        }
        n_gi += ngi;
        if (!ok) {
#pragma unroll
          for (int s = 0; s < NR; ++s) lab[s] = flab[s];
          ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas);
        }
      }
    } else {
      // pair: one reduced solve on the previous solve's labels (a hit when the pair QP barely
      // moved since); label moves are left to the dual active set, warm-started from the same
      // active set -- each further PDAS step is a full Schur build + factorization (r03 stamps:
      // 3.25 of them per step on a crossing, nearly all followed by the dual active set anyway)
      ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas, NV == 2 ? 1 : PDAS_STEPS);
    }
  }
  if constexpr (NV == 2) {
    // pair QP: dual active set first (no K_s^-1, no ADMM); certified by the KKT test, and
    // when that fails, polished from its labels before the ADMM fallback
    if (!ok && P.ycap > 0) {
      int ngi = 0;
      signed char glab[NR];
      signed char clab[NR];
      if constexpr (NV == 2) gi_snap_restore<RM>(P);
      if (gi_solve<NV, RM>(P, nullptr, glab, x, y, ngi, clab)) {
        signed char nl[NR];
        ok = kkt_check(P, glab, x, y, nl);
#ifdef PIADMM_GI_DEBUG
        GI_DBG("GI done steps=%d kkt=%d\n", ngi, (int)ok);
        if (!ok) {
          double axd[NR];
          A_mul(P, x, axd);
#pragma unroll
          for (int s = 0; s < NR; ++s)
            if (P.valid(s)) {
              const double bd = (glab[s] == UPPER && !P.hinge(s)) ? P.hi(s) : P.lo(s);
              const bool act = P.hinge(s) ? glab[s] == HKINK : glab[s] != FREE;
              const double tp = P.tol * (1.0 + fabs(P.lo(s)));
              if (nl[s] != glab[s] || (act && fabs(axd[s] - bd) > tp) || !isfinite(y[s]))
                printf("  kkt viol slot %d lane %d lab %d -> %d ax %.12g bd %.12g y %.12g\n", s, lid(),
                       (int)glab[s], (int)nl[s], axd[s], bd, y[s]);
            }
        }
#endif
#pragma unroll
        for (int s = 0; s < NR; ++s) lab[s] = glab[s];
        if (!ok) ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas);
        GI_DBG("  after pdas ok=%d\n", (int)ok);
      } else if (TWO && P.gi_full && P.wide) {
        // the working set outgrew one row per lane: the wide dual active set (two per lane;
        // big mode only -- H > 32, where a pair QP's 2H variables can hold more than 63 rows)
        if constexpr (NV == 2 && TWO) {
          if (gi_solve_wide(P, glab, x, y, ngi)) {
            signed char nl[NR];
            ok = kkt_check(P, glab, x, y, nl);
          }
        }
#pragma unroll
        for (int s = 0; s < NR; ++s) lab[s] = ok ? glab[s] : clab[s];
        if (!ok) ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas, 4 * PDAS_STEPS);
      } else {
        // GI stopped (typically a hinge multiplier at its cap beta: that hinge is linear at the
        // optimum, which the dual active set does not model): polish from its working set with
        // the saturated row linear before falling back to ADMM
#pragma unroll
        for (int s = 0; s < NR; ++s) lab[s] = clab[s];
        ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas, 4 * PDAS_STEPS);
      }
      n_gi += ngi;
    }
  }
  signed char plab[NR];
#pragma unroll
  for (int s = 0; s < NR; ++s) plab[s] = -1;
  if (__builtin_expect(!ok && !P.kready, 0)) {
    if (!P.scaled) {
      // the warm ADMM state is in identity scaling (x, A x, y): move it to the Ruiz space
      if (P.wraw) warm_to_scaled(P, xs, zs, ys);     // identity D, E: (x, A x, y)
      unsigned long long t_r = STAMP_T();
      ruiz(P);
      STAMP_ADD(ST_SZ_RUIZ, t_r);
#pragma unroll
      for (int v = 0; v < NV; ++v) xs[v] = (P.D[v] != 0.0) ? xs[v] / P.D[v] : 0.0;
#pragma unroll
      for (int s = 0; s < NR; ++s) {
        zs[s] = P.valid(s) ? P.E[s] * zs[s] : 0.0;
        ys[s] = P.valid(s) ? ys[s] / P.E[s] : 0.0;
      }
      P.scaled = true;
    }
    if (NV == 1 && P.Kcache) {
      // the per-scenario HBM copy (same penalty): batched loads, then the LDS stores
      const int l = lid(), n = P.n;
      for (int i0 = 0; i0 < n; i0 += 8) {
        double kv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) kv[u] = (l < n) ? P.Kcache[min(i0 + u, n - 1) * n + l] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (l < n && i0 + u < n) {
            if (P.kf32) P.Kf[(i0 + u) * n + l] = (float)kv[u];
            else P.K[(i0 + u) * n + l] = kv[u];
          }
        }
      }
    } else {
      build_K<NV, TWO>(P, kscr, kld);
    }
    P.kready = true;
    if (NV == 2 && lid() == 0) P.fstate[0] = -1;   // the scratch held the pair's cached factor
    wsync();
  }
  if (__builtin_expect(!ok, 0)) ensure_q(P);
  if (!ok && P.wraw) warm_to_scaled(P, xs, zs, ys);
  for (int it = 1; __builtin_expect(!ok, 0) && it <= max_inner; ++it) {
    unsigned long long t_a = STAMP_T();
    admm_iter(P, xs, zs, ys);
    STAMP_ADD(ST_ADMM, t_a);
    ++n_admm;
    // adaptive rho for the x-step only: on the pair QPs with long runs of hinge kinks the
    // OSQP rule stalls ADMM (tools/pair_policy.py: 3 of 15 hard pair QPs uncertified after
    // 4000 iterations with it, all 15 certified within 530 without it)
    if (NV == 1 && it % ADAPT_EVERY == 0) {
      const double f = rho_ratio(P, xs, zs, ys);
      if (f != 1.0) {
        P.rho = fmin(fmax(P.rho * f, 1e-6), 1e6);
        build_K<NV, TWO>(P, kscr, kld);
        P.Kcache = nullptr;      // the cached copy is for the old penalty
        if (NV == 2 && lid() == 0) P.fstate[0] = -1;   // the scratch held the pair's cached factor
        wsync();
      }
    }
    if (it % polish_every == 0) {
      // polish when the ADMM active-set estimate has not moved since the last check
      // (or every 8 periods), and never twice from the same labels
      bool same = true, tried = true;
#pragma unroll
      for (int s = 0; s < NR; ++s) {
        lab[s] = label_scaled(P, s, zs[s] + ys[s] / rrow(P, s));
        same &= (lab[s] == plab[s]);
        tried &= (lab[s] == flab[s]);
        plab[s] = lab[s];
      }
      if ((wall(same) || it % (8 * polish_every) == 0) && !wall(tried)) {
#pragma unroll
        for (int s = 0; s < NR; ++s) flab[s] = lab[s];
        ok = pdas<NV, XU, (RM & RM_T) != 0>(P, lab, x, y, n_pdas);
      }
    }
  }
  unsigned long long t_ep = STAMP_T();
  int st = PIADMM_QP_OK;
  if (ok) {
    // warm ADMM state at the exact optimum, kept raw until an ADMM iteration needs it
#pragma unroll
    for (int v = 0; v < NV; ++v) xs[v] = x[v];
#pragma unroll
    for (int s = 0; s < NR; ++s) ys[s] = P.valid(s) ? y[s] : 0.0;
    P.wraw = true;
  } else {
    st |= PIADMM_QP_INEXACT;
#pragma unroll
    for (int v = 0; v < NV; ++v) x[v] = P.D[v] * xs[v];
#pragma unroll
    for (int s = 0; s < NR; ++s) lab[s] = label_scaled(P, s, zs[s] + ys[s] / rrow(P, s));
  }
  bool fin = true;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    x_out[v] = (lid() < P.H) ? x[v] : 0.0;
    fin &= isfinite(x_out[v]);
  }
  if (!wall(fin)) st |= PIADMM_QP_NAN;
  if (NV == 1) STAMP_ADD(ST_QEPI, t_ep);
  return st;
}

}  // namespace pd
