// piadmm_device.hip -- MI355X (gfx950) kernels of the batched PI-ADMM consensus solver.
//
// One workgroup = one connected component of the candidate-pair graph (two
// agents and their pair in the tiled scenario); one persistent launch = up to 32
// MPC steps of the reference loop (casadi/main.py:43-201) per component: seeds,
// per-step setup of every QP, the outer ADMM loop with device-side termination,
// and propagation.  Components are independent; the only inter-workgroup step is
// the grid barrier of the reference's global stopping test (cooperative launch).
//
// Wave layout: wave w solves agent w's x-step; wave 0 also owns the pair.
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
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "piadmm_internal.h"

namespace pd {

// Diagnostic phase stamps (separate build, never in the measured library).
#ifdef PIADMM_STAMPS
// cycles accumulate in LDS (one ds_add_u64 per stamp, lane 0) and are flushed to g_stamps
// once per launch, so that a stamp costs an LDS atomic, not a global one
__device__ unsigned long long* g_stamps;
__shared__ unsigned long long s_stamps[64];
#define STAMP_T() __builtin_amdgcn_s_memtime()
#define STAMP_ADD(slot, t0)                                                                   \
  do {                                                                                        \
    const unsigned long long _d = __builtin_amdgcn_s_memtime() - (t0);                       \
    if (__lane_id() == 0) atomicAdd(&s_stamps[(slot)], _d);                                  \
  } while (0)
#else
#define STAMP_T() 0ull
#define STAMP_ADD(slot, t0) ((void)(t0))
#endif
enum StampSlot { ST_SETUP_X = 0, ST_SETUP_Z, ST_XSTEP, ST_XQP, ST_XRED, ST_XROLL, ST_ZSTEP, ST_ZQP, ST_ZRED,
                 ST_KERNEL, ST_RED_GEMV, ST_RED_S, ST_RED_CHOL, ST_RED_X, ST_ADMM, ST_XQ, ST_TERM,
                 ST_SZ_RUIZ, ST_SZ_KMAT, ST_SZ_GJ, ST_SZ_PRE, ST_ZR_GEMV, ST_ZR_S, ST_ZR_CHOL, ST_ZR_X,
                 ST_ZR_SOLVE, ST_XR_SOLVE, ST_ZKKT, ST_XKKT, ST_GI_SEARCH, ST_GI_SOLVE, ST_GI_UPD,
                 ST_SYNC_A, ST_TERMW, ST_SYNC_B, ST_RSX_PRE, ST_QEPI, ST_ROUND, NSTAMP = 64 };

// ============================================================ wave primitives
__device__ __forceinline__ int lid() { return (int)__lane_id(); }

// Intra-wave LDS hand-off: LDS ops of one wave execute in order, so only the
// compiler must be kept from moving memory operations across this point.
__device__ __forceinline__ void wsync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Global-memory hand-off between lanes of one wave (big mode): wait for the stores, then
// the wave barrier; all waves of the workgroup share the CU's vector L1.
__device__ __forceinline__ void gsync() {
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
}

// Broadcast lane k's value (k wave-uniform) through SGPRs.
__device__ __forceinline__ double rdl(double v, int k) {
  unsigned long long b = (unsigned long long)__double_as_longlong(v);
  int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffull), k);
  int hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), k);
  unsigned long long r = ((unsigned long long)(unsigned)hi << 32) | (unsigned long long)(unsigned)lo;
  return __longlong_as_double((long long)r);
}
__device__ __forceinline__ int rdli(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

// DPP move of a double (two 32-bit halves); lanes whose source is outside the row/wave read 0.
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b & 0xffffffffull), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
constexpr int DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138;

__device__ __forceinline__ double shup(double v, int o) {
  if (o == 1) return dppd<DPP_WAVE_SHR1>(v);          // lane l <- lane l-1, lane 0 <- 0
  double t = __shfl_up(v, (unsigned)o);
  return lid() >= o ? t : 0.0;
}
__device__ __forceinline__ double shdn(double v, int o) {
  if (o == 1) return dppd<DPP_WAVE_SHL1>(v);          // lane l <- lane l+1, lane 63 <- 0
  double t = __shfl_down(v, (unsigned)o);
  return lid() + o < WAVE ? t : 0.0;
}
__device__ __forceinline__ bool wany(bool p) { return __ballot(p) != 0ull; }
__device__ __forceinline__ bool wall(bool p) { return __ballot(!p) == 0ull; }

// DPP move restricted to the 16-lane rows in ROWS (other rows read 0).
template <int CTRL, int ROWS>
__device__ __forceinline__ double dppd_rows(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b & 0xffffffffull), CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// DPP move in which lanes without a valid source (or outside ROWS) keep their own value:
// the identity for min / max.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dppd_keep(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int l0 = (int)(unsigned)(b & 0xffffffffull), h0 = (int)(unsigned)(b >> 32);
  const int lo = __builtin_amdgcn_update_dpp(l0, l0, CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(h0, h0, CTRL, ROWS, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// Wave-wide min / max / sum of a double, broadcast to every lane: the same DPP scan as
// scan_incl (row_shr 1,2,4,8, then row_bcast:15 / row_bcast:31) ending in lane 63, read back
// through SGPRs -- a few VALU cycles per stage instead of the LDS round trip of a
// ds_bpermute per stage (__shfl_xor).
template <bool MAX>
__device__ __forceinline__ double wext(double v) {
  auto op = [](double a, double b) { return MAX ? fmax(a, b) : fmin(a, b); };
  v = op(v, dppd_keep<0x111, 0xf>(v));
  v = op(v, dppd_keep<0x112, 0xf>(v));
  v = op(v, dppd_keep<0x114, 0xf>(v));
  v = op(v, dppd_keep<0x118, 0xf>(v));
  v = op(v, dppd_keep<0x142, 0xa>(v));
  v = op(v, dppd_keep<0x143, 0xc>(v));
  return rdl(v, 63);
}
__device__ __forceinline__ double wmax(double v) { return wext<true>(v); }
__device__ __forceinline__ double wmin(double v) { return wext<false>(v); }

// Inclusive prefix / suffix sums over the 64 lanes (time lanes 0..H, H <= 63).  Four DPP
// row shifts inside each 16-lane row; the prefix carries across rows with the GFX9
// row_bcast:15 / row_bcast:31 DPP broadcasts, the suffix with three readlanes.
__device__ __forceinline__ double scan_incl(double v) {
  v += dppd<0x111>(v);   // row_shr:1
  v += dppd<0x112>(v);   // row_shr:2
  v += dppd<0x114>(v);   // row_shr:4
  v += dppd<0x118>(v);   // row_shr:8
  v += dppd_rows<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
  v += dppd_rows<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ double scan_incl_rev(double v) {
  v += dppd<0x101>(v);   // row_shl:1
  v += dppd<0x102>(v);   // row_shl:2
  v += dppd<0x104>(v);   // row_shl:4
  v += dppd<0x108>(v);   // row_shl:8
  const double r1 = rdl(v, 16), r2 = rdl(v, 32), r3 = rdl(v, 48);
  const int l = lid();
  const double c = (l < 16) ? r1 + (r2 + r3) : ((l < 32) ? r2 + r3 : ((l < 48) ? r3 : 0.0));
  return v + c;
}
__device__ __forceinline__ double wsum(double v) { return rdl(scan_incl(v), 63); }

// T(t, j) = (t-1-j)+ is the rollout's double integrator (casadi/PI_ADMM_class.py:59-69:
// theta accumulates u, x/y accumulate theta).  "hinge lane" k holds time t = k+1.
// T_apply : var lanes u_j        -> hinge lanes (T u)_{k+1} = sum_{j<=k-1} (k-j) u_j
// Tt_apply: hinge lanes w_k      -> var lanes   sum_{k>=j+1} (k-j) w_k
__device__ __forceinline__ double T_apply(double u) {
  return shup(scan_incl(scan_incl(u)), 1);
}
__device__ __forceinline__ double Tt_apply(double w) {
  return shdn(scan_incl_rev(scan_incl_rev(w)), 1);
}

// ============================================================ reference arithmetic
__device__ __forceinline__ double pow10i(int d) {
  double f = 1.0;
  for (int i = 0; i < d; ++i) f *= 10.0;
  return f;
}
// np.around(x, d) = rint(x * 10^d) / 10^d   (casadi/main.py:48-49,103,153)
__device__ __forceinline__ double around(double x, int d) {
  if (d < 0) return x;
  const double f = pow10i(d);
  return rint(x * f) / f;
}

// sum_{k=0}^{H} (k-1-i)+ (k-1-j)+ = (T'T)_{ij}, exact in integers.
__device__ __forceinline__ double TT(int i, int j, int H) {
  const int a = max(i, j), b = min(i, j);
  const int n = H - 1 - a;
  if (n < 0) return 0.0;
  const int d = a - b;
  const int s = n * (n + 1) * (2 * n + 1) / 6 + d * (n * (n + 1) / 2);   // < 2^31 for H <= 64
  return (double)s;
}
// (D2'D2)_{ij}, D2 = second difference (H-2) x H  (cost_smooth, PI_ADMM_class.py:123)
__device__ __forceinline__ double d2c(int d) { return d == 1 ? -2.0 : ((d == 0 || d == 2) ? 1.0 : 0.0); }
__device__ __forceinline__ double D2D2(int i, int j, int H) {
  if (abs(i - j) > 2) return 0.0;
  double s = 0.0;
  const int r0 = max(max(i, j) - 2, 0), r1 = min(min(i, j), H - 3);
  for (int r = r0; r <= r1; ++r) s += d2c(i - r) * d2c(j - r);
  return s;
}

struct Geo {
  double x0, y0, th0, s, sn, cs, ax, ay, mm, xdot0, ydot0;
};
// Linearised rollout at theta0 (PI_ADMM_class.py:56-69): p = c + M u with
// M = [ax T; ay T], c_{t+1} = c_t + xdot0*dt.
__device__ __forceinline__ Geo make_geo(const double* xt3, double s, const piadmm_config_t& c) {
#pragma clang fp contract(off)
  Geo g;
  g.x0 = xt3[0];
  g.y0 = xt3[1];
  g.th0 = xt3[2];
  g.s = s;
  g.sn = sin(g.th0);
  g.cs = cos(g.th0);
  g.ax = (-s * g.sn * c.dt) * (s / c.L * c.dt);
  g.ay = (s * g.cs * c.dt) * (s / c.L * c.dt);
  // |M_x|^2 + |M_y|^2 = (dt s a)^2 (sin^2 + cos^2): written without the trig so that the
  // x-step P (and the pair P blocks) depend on the speed only and can be cached per scenario
  const double msc = s * c.dt * (s / c.L * c.dt);
  g.mm = msc * msc;
  g.xdot0 = -s * g.sn * g.th0 + (s * g.cs + s * g.th0 * g.sn);
  g.ydot0 = s * g.cs * g.th0 + (s * g.sn - s * g.th0 * g.cs);
  return g;
}
// c at time lanes t = 0..H (literal sequential accumulation).
__device__ __forceinline__ void affine_c(const Geo& g, double dt, int H, double& cx, double& cy) {
#pragma clang fp contract(off)
  const int l = lid();
  double ax = g.x0, ay = g.y0;
  cx = (l == 0) ? ax : 0.0;
  cy = (l == 0) ? ay : 0.0;
  for (int t = 0; t < H; ++t) {
    ax = ax + g.xdot0 * dt;
    ay = ay + g.ydot0 * dt;
    if (l == t + 1) {
      cx = ax;
      cy = ay;
    }
  }
}

// Numeric rollouts at time lanes (u at var lanes).  Linear: dynamic_update_local
// numeric branch (PI_ADMM_class.py:56-70).  Nonlinear: dynamic_update_edge
// numeric branch (:88-105) = MATLAB numeric dynamic_update_local (:312-330).
// (x0, y0, theta0, s, s/L) in registers: the per-iteration x-step rollout reads no memory
__device__ __forceinline__ void rollout_r(double x0, double y0, double th0, double s, double sl, double u,
                                          const piadmm_config_t& c, int H, bool nonlinear, double& px, double& py,
                                          double& pth) {
#pragma clang fp contract(off)
  const int l = lid();
  // theta_k = theta_0 + sum_{j<k} (s/L u_j) dt  (wave prefix scan)
  const double inc = (l < H) ? (sl * u) * c.dt : 0.0;
  const double my_th = th0 + shup(scan_incl(inc), 1);
  // per-lane rates at time k = lane
  double xd, yd;
  if (nonlinear) {
    double sk, ck;
    sincos(my_th, &sk, &ck);
    xd = -s * sk * my_th + (s * ck + s * my_th * sk);
    yd = s * ck * my_th + (s * sk - s * my_th * ck);
  } else {
    const double sn0 = sin(th0), cs0 = cos(th0);
    xd = -s * sn0 * my_th + (s * cs0 + s * th0 * sn0);
    yd = s * cs0 * my_th + (s * sn0 - s * th0 * cs0);
  }
  const double xi = (l < H) ? xd * c.dt : 0.0, yi = (l < H) ? yd * c.dt : 0.0;
  px = x0 + shup(scan_incl(xi), 1);
  py = y0 + shup(scan_incl(yi), 1);
  pth = my_th;
  if (l > H) px = py = pth = 0.0;
}
__device__ __forceinline__ void rollout(const double* xt3, double s, double u, const piadmm_config_t& c, int H,
                        bool nonlinear, double& px, double& py, double& pth) {
  rollout_r(xt3[0], xt3[1], xt3[2], s, s / c.L, u, c, H, nonlinear, px, py, pth);
}

// ============================================================ in-wave dense kernels
// In-place Gauss-Jordan inverse of an SPD matrix held in LDS (stride ld), lane = column.
__device__ __forceinline__ void gj_invert(double* m, int n, int ld) {
  const int l = lid();
  const int lc = (l < n) ? l : n - 1;     // lanes >= n mirror column n-1 and never store
  constexpr int U = 8;
  for (int p = 0; p < n; ++p) {
    const double ip = 1.0 / m[p * ld + p];                 // uniform address: LDS broadcast
    const double rpj = (l == p) ? ip : m[p * ld + lc] * ip;
    // every row i (row p included: it is overwritten below) -= a_ip * new row p;
    // column p becomes -a_ip / a_pp.  a_ip is read as an LDS broadcast: within a group all
    // reads come before lane p's writes of the same rows, and later groups touch later rows.
    int i = 0;
    for (; i + U <= n; i += U) {
      double v[U], a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u] = m[(i + u) * ld + p];
        v[u] = m[(i + u) * ld + lc];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double nv = (l == p) ? -a[u] * ip : v[u] - a[u] * rpj;
        if (l < n) m[(i + u) * ld + l] = nv;
      }
    }
    for (; i < n; ++i) {
      const double a = m[i * ld + p];
      const double v = m[i * ld + lc];
      const double nv = (l == p) ? -a * ip : v - a * rpj;
      if (l < n) m[i * ld + l] = nv;
    }
    if (l < n) m[p * ld + l] = rpj;
    wsync();
  }
}

// Gauss-Jordan inverse of an SPD n x n matrix (64 < n <= 128), lane l owning columns l and
// l + 64 (the pair's K beyond H = 32, in HBM in big mode: each pivot ends with a fence).
// Same read-before-write ordering as gj_invert.
__device__ __forceinline__ void gj_invert2(double* m, int n, int ld, bool global_mem) {
  const int l = lid();
  const int c1 = l + WAVE;
  const bool own1 = c1 < n;
  const int lc1 = own1 ? c1 : n - 1;
  constexpr int U = 4;
  for (int p = 0; p < n; ++p) {
    const double ip = 1.0 / m[p * ld + p];
    const double r0 = (l == p) ? ip : m[p * ld + l] * ip;
    const double r1 = (c1 == p) ? ip : m[p * ld + lc1] * ip;
    int i = 0;
    for (; i + U <= n; i += U) {
      double a[U], v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u] = m[(i + u) * ld + p];
        v0[u] = m[(i + u) * ld + l];
        v1[u] = m[(i + u) * ld + lc1];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        m[(i + u) * ld + l] = (l == p) ? -a[u] * ip : v0[u] - a[u] * r0;
        if (own1) m[(i + u) * ld + c1] = (c1 == p) ? -a[u] * ip : v1[u] - a[u] * r1;
      }
    }
    for (; i < n; ++i) {
      const double a = m[i * ld + p];
      const double v0 = m[i * ld + l], v1 = m[i * ld + lc1];
      m[i * ld + l] = (l == p) ? -a * ip : v0 - a * r0;
      if (own1) m[i * ld + c1] = (c1 == p) ? -a * ip : v1 - a * r1;
    }
    m[p * ld + l] = r0;
    if (own1) m[p * ld + c1] = r1;
    if (global_mem) gsync();
    else wsync();
  }
}

__device__ __forceinline__ double clamp_norm(double v) {
  if (!(v > 1e-6)) return 1.0;
  return v > 1e6 ? 1e6 : v;
}

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
  bool scaled;            // Ruiz scaling computed (the pair computes it only when ADMM is needed)
  bool wraw;              // the warm ADMM state holds the last certified (x, y) unscaled (zs unset):
                          // converted to the scaled (xs, zs, ys) only when ADMM actually runs
  const double* Kcache;   // x-step: HBM copy of K_s^-1, loaded into K only when ADMM is needed
  mutable int csig;       // x-step: per-lane working-set signature of the cached X', G
  int* gws;               // pair: HBM warm working set of the dual active set (GI_WS ints)
  int tstep;              // MPC step index (warm-set bookkeeping)

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
__device__ __forceinline__ double chol_solve(const double* L, int ld, double linv, double b, int m) {
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
__device__ __forceinline__ bool chol_factor(double* fac, int ld, double sdiag, double delta, int m, double& linv) {
  const int l = lid();
  for (int k = 0; k < m; ++k) {
    double acc = 0.0;
    if (l >= k && l < m) {
      const double* ri = fac + l * ld;
      const double* rk = fac + k * ld;
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
          else P.fac[l * ld + b] = sv;
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
        const double sab = (b == l) ? sdiag : (b > l ? P.fac[l * ld + b] : P.fac[b * ld + l]);
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
  {
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
__device__ __forceinline__ bool param_build_x(const QP<1>& P, int m, int myid, const int* ids, const double* vb_b) {
  const int l = lid(), H = P.H, ld = P.fld;
  double* fac = P.fac;
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
  if (!chol_factor(fac, ld, sdiag, 0.0, m, linv)) return false;
  if (l < m) P.fdiag[64 + l] = linv;
  STAMP_ADD(ST_RED_CHOL, t_c);
  unsigned long long t_x = STAMP_T();
  // right-hand sides, one per lane: lane i < H -> row i of Y = P^-1 A_W', lane H -> b
  const int li = (l <= H) ? l : H;
  const bool own = l <= H;
  double* xr = XT + li * P.xld;
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
        if (own) xr[a] = v;
      }
    }
  }
  wsync();
  // L L' sol = rhs for every lane's right-hand side (L broadcast from fac, lane-own sol)
  constexpr int TB = 8;
  for (int a = 0; a < m; ++a) {
    double acc = xr[a];
    for (int b0 = 0; b0 < a; b0 += TB) {
      double Lv[TB], sv[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        const int b = min(b0 + u, a - 1);
        Lv[u] = (b0 + u < a) ? fac[a * ld + b] : 0.0;
        sv[u] = xr[b];
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) acc -= Lv[u] * sv[u];
    }
    acc *= P.fdiag[64 + a];
    if (own) xr[a] = acc;
  }
  for (int a = m - 1; a >= 0; --a) {
    double acc = xr[a];
    for (int b0 = a + 1; b0 < m; b0 += TB) {
      double Lv[TB], sv[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        const int b = min(b0 + u, m - 1);
        Lv[u] = (b0 + u < m) ? fac[b * ld + a] : 0.0;
        sv[u] = xr[b];
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) acc -= Lv[u] * sv[u];
    }
    acc *= P.fdiag[64 + a];
    if (own) xr[a] = acc;
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
    const double* xj = XT + lc * P.xld;
    constexpr int GB = 8;
    for (int i0 = 0; i0 < H; i0 += GB) {
      double acc[GB], pv[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) {
        acc[u] = 0.0;
        pv[u] = P.Pinv[min(i0 + u, H - 1) * H + lc];
      }
      for (int a = 0; a < m; ++a) {
        const double xja = xj[a];
        const double* ya = fac + a * ld + i0;
#pragma unroll
        for (int u = 0; u < GB; ++u) acc[u] += ya[u] * xja;     // rows past H are never stored
      }
#pragma unroll
      for (int u = 0; u < GB; ++u)
        if (l < H && i0 + u < H) P.G[(i0 + u) * H + l] = pv[u] - acc[u];
    }
    double gacc = 0.0;
    for (int a = 0; a < m; ++a) gacc += fac[a * ld + lc] * XT[H * P.xld + a];
    if (l < H) P.G[H * H + l] = gacc;
    if (P.gmem) gsync();
    else wsync();
  }
  // fold q = T'-apply(w') into the tables: row k of G T' (and X T') is
  // sum_{j<k} (k - j) row j -- two running sums per lane, in place (read before write)
  {
    double s1 = 0.0, s2 = 0.0, t1 = 0.0, t2 = 0.0;
    const int la = (l < m) ? l : 0;
    for (int k = 0; k < H; ++k) {
      const double gk = P.G[k * H + (l < H ? l : 0)];
      const double xk = XT[k * P.xld + la];
      if (l < H) P.G[k * H + l] = s2;
      if (l < m) XT[k * P.xld + l] = t2;
      s1 += gk;
      s2 += s1;
      t1 += xk;
      t2 += t1;
    }
    if (P.gmem) gsync();
    else wsync();
  }
  return true;
}

template <int XU>
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
    if (!param_build_x(P, m, myid, ids, vb_b)) {
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
  unsigned long long t_rs = STAMP_T();
  // one fused pass: x = -G q + g (lane = variable), lam = -X q - beta (lane = W row)
  double ag = 0.0, ax = 0.0;
  {
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

// KKT test of (x, y) for labels lab; on failure fills new labels (PDAS update).
template <int NV>
__device__ __forceinline__ bool kkt_check(const QP<NV>& P, const signed char* lab, const double* x, const double* y,
                          signed char* nlab) {
  constexpr int NR = QP<NV>::NR;
  double ax[NR];
  A_mul(P, x, ax);
  double ym = 0.0;
#pragma unroll
  for (int s = 0; s < NR; ++s) ym = fmax(ym, fabs(y[s]));
  ym = wmax(ym);
  const double ty = P.tol * (1.0 + ym);
  bool ok = true;
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
        ok &= (y[s] <= ty) && (y[s] >= -P.beta - ty) && fabs(ax[s] - h) <= tp;
        nlab[s] = (y[s] > ty) ? HZERO : ((y[s] < -P.beta - ty) ? HLINEAR : HKINK);
      }
    } else {
      if (lab[s] == FREE) {
        const bool vl = ax[s] < P.lo(s) - tp, vu = ax[s] > P.hi(s) + tp;
        ok &= !vl && !vu;
        nlab[s] = vl ? LOWER : (vu ? UPPER : FREE);
      } else if (lab[s] == LOWER) {
        ok &= (y[s] <= ty) && fabs(ax[s] - P.lo(s)) <= tp;   // equality too (dropped rows)
        nlab[s] = (y[s] > ty) ? FREE : LOWER;
      } else {
        ok &= (y[s] >= -ty) && fabs(ax[s] - P.hi(s)) <= tp;
        nlab[s] = (y[s] < -ty) ? FREE : UPPER;
      }
    }
    ok &= isfinite(x[0]) && isfinite(y[s]);
  }
  return wall(ok);
}

template <int NV, int XU = XGEMV_U>
__device__ __forceinline__ bool pdas(const QP<NV>& P, signed char* lab, double* x, double* y, int& nsolve,
                                     int steps = PDAS_STEPS) {
  constexpr int NR = QP<NV>::NR;
  signed char nl[NR];
  for (int it = 0; it < steps; ++it) {
    ++nsolve;
    unsigned long long t_r = STAMP_T();
    bool rs_ok;
    if constexpr (NV == 1) rs_ok = reduced_solve_x<XU>(P, lab, x, y);
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
// steps that drop a constraint whose multiplier reaches 0.  The active set's Schur
// complement S = N P^-1 N' is kept as a Cholesky factor L (LDS, insertion order): an add
// appends one row (its forward-solve vector w and sqrt(S_pp - w'w)), a drop deletes row k and
// restores the trailing block by a rank-one update.  Y holds the columns P^-1 n_a.  Each step
// costs two m-step triangular solves, one m-column pass over Y and a few wave reductions --
// no K_s^-1 and no ADMM.  On the recorded bench pair QPs (tools/gi_sim.py) it certifies every
// one in 28 steps on average (max 51) where ADMM + PDAS took ~45 ADMM iterations and ~6
// full reduced solves.  A hinge multiplier reaching the cap, a full factor or the step limit
// return false and the caller falls back to ADMM + PDAS; the result is certified by the same
// KKT test either way.
// Triangular solves with lane = row, the factor's column (fwd) / row (bwd) entries of a batch
// of TRI_U steps loaded before the batch's dependent chain: one LDS latency per batch
// instead of one per step.
constexpr int TRI_U = 8;
__device__ __forceinline__ double tri_fwd(const double* L, int ld, double linv, double b, int m) {
  const int l = lid();
  const int lr = (l < m) ? l : 0;
  for (int k0 = 0; k0 < m; k0 += TRI_U) {
    double Lv[TRI_U];
#pragma unroll
    for (int u = 0; u < TRI_U; ++u) Lv[u] = L[lr * ld + min(k0 + u, 63)];
#pragma unroll
    for (int u = 0; u < TRI_U; ++u) {
      const int k = k0 + u;
      if (k < m) {
        const double zk = rdl(b * linv, k);
        if (l == k) b = zk;
        if (l > k && l < m) b -= Lv[u] * zk;
      }
    }
  }
  return (l < m) ? b : 0.0;
}
__device__ __forceinline__ double tri_bwd(const double* L, int ld, double linv, double b, int m) {
  const int l = lid();
  const int lc = (l < m) ? l : 0;
  for (int k0 = m - 1; k0 >= 0; k0 -= TRI_U) {
    double Lv[TRI_U];
#pragma unroll
    for (int u = 0; u < TRI_U; ++u) Lv[u] = L[max(k0 - u, 0) * ld + lc];
#pragma unroll
    for (int u = 0; u < TRI_U; ++u) {
      const int k = k0 - u;
      if (k >= 0) {
        const double xk = rdl(b * linv, k);
        if (l == k) b = xk;
        if (l < k) b -= Lv[u] * xk;
      }
    }
  }
  return (l < m) ? b : 0.0;
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

constexpr int GI_MAX_STEPS = 256;
constexpr int GI_WS = 2 + WAVE;   // per-pair warm working set in HBM: m, step t, codes
// Warm start (receding horizon): the previous MPC step's final active set, shifted one time
// slot (tools/gi_sim.py + the warm-start prototype: 28 -> 3.6 GI steps per bench pair QP),
// is appended row by row (dependent rows skipped), its equality-constrained minimiser formed
// and constraints with negative (or beyond-cap) multipliers dropped until the start is dual
// feasible -- the state GI requires -- before the usual adds.  Any starting set is only a
// guess: the minimiser and its certificate do not depend on it.
template <int NV>
__device__ __forceinline__ bool gi_solve(QP<NV>& P, const signed char* wlab, signed char* lab, double* x, double* y,
                                         int& nsteps) {
  constexpr int NR = QP<NV>::NR;
  const int l = lid(), H = P.H, ld = P.fld, H2 = NV * H;
  double* vb_ax = P.vb + 192;      // [192, 192 + NR*H): (A v) by row id
  int* wc = P.ib;                  // active constraint codes 2*row + side, insertion order
  double* L = P.fac;
  double* Y = P.Y;
  const int cap = min(P.mmax - 1, P.ycap);
  if (P.y_in_k) P.kready = false;  // Y overwrites the K_s^-1 region
  if (l == 0) P.fstate[0] = -1;    // and L the cached PDAS factor
  P.csig = -1;                     // (x-step: the factor scratch the parametric tables were built in)
  double x0[NV], xc[NV];
  gemv_sym<true>(P, P.Pinv, P.q, x0);
#pragma unroll
  for (int v = 0; v < NV; ++v) xc[v] = x0[v] = -x0[v];
  int m = 0, wbits = 0;
  double ua = 0.0, linv = 0.0;     // lane a < m: multiplier and 1/L_aa of active constraint a

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
  // w = L^-1 (N y_p) for the current active set (lane a < m)
  auto fwd = [&]() -> double {
    const int myc = (l < m) ? wc[l] : 0;
    const double va = (l < m) ? ((myc & 1) ? -1.0 : 1.0) * vb_ax[myc >> 1] : 0.0;   // n_a' y_p
    return tri_fwd(L, ld, linv, va, m);
  };
  // append constraint pc: L row m = (w', sqrt(lpp2)), Y column m = y_p
  auto append = [&](int pc, const double* yp, double w, double lpp2, double u0) {
    const int prow = pc >> 1, ps = prow / H, pk = prow - ps * H;
    const double lmm = sqrt(lpp2);
    if (l < m) L[m * ld + l] = w;
    if (l == m) {
      L[m * ld + m] = lmm;
      linv = 1.0 / lmm;
      ua = u0;
      wc[m] = pc;
    }
    if (l < H) {
#pragma unroll
      for (int v = 0; v < NV; ++v) Y[m * H2 + v * H + l] = yp[v];
    }
    if (l == pk) wbits |= 1 << (2 * ps + (pc & 1));
    ++m;
    if (P.gmem) gsync();
    else wsync();
  };
  // drop active constraint k: delete row/column k of L, rank-one update of the trailing block
  // with the deleted column, compact L, Y, codes and multipliers
  auto drop = [&](int k) {
    const int kc = rdli((l < m) ? wc[l] : 0, k);
    if (l == (kc >> 1) % H) wbits &= ~(1 << (2 * ((kc >> 1) / H) + (kc & 1)));
    double xv = (l > k && l < m) ? L[l * ld + k] : 0.0;
    for (int j = k + 1; j < m; ++j) {
      const double Ljj = L[j * ld + j];
      const double xj = rdl(xv, j);
      const double rr = sqrt(Ljj * Ljj + xj * xj);
      const double cc = rr / Ljj, sn = xj / Ljj;
      if (l == j) L[j * ld + j] = rr;
      if (l > j && l < m) {
        const double Lij = (L[l * ld + j] + sn * xv) / cc;
        xv = cc * xv - sn * Lij;
        L[l * ld + j] = Lij;
      }
    }
    wsync();
    // compact: row i <- row i+1 (i >= k), column j <- column j+1 (j >= k); lane = column
    for (int i = k; i < m - 1; ++i) {
      const double v = (l < m - 1) ? L[(i + 1) * ld + l + (l >= k ? 1 : 0)] : 0.0;
      wsync();
      if (l <= i) L[i * ld + l] = v;
      wsync();
    }
    const int cnext = (l + 1 < m) ? wc[l + 1] : 0;
    wsync();
    if (l >= k && l < m - 1) wc[l] = cnext;
    const double un = shdn(ua, 1);
    if (l >= k) ua = (l < m - 1) ? un : 0.0;
    for (int a = k; a < m - 1; ++a) {
      if (l < H) {
#pragma unroll
        for (int v = 0; v < NV; ++v) Y[a * H2 + v * H + l] = Y[(a + 1) * H2 + v * H + l];
      }
    }
    --m;
    if (P.gmem) gsync();
    else wsync();
    linv = (l < m) ? 1.0 / L[l * ld + l] : 0.0;
  };
  // multipliers of the equality-constrained minimiser on the active set (signed normals):
  // lam = S^-1 (N x0 - b); kernel multiplier of row a = sign_a * lam_a, GI multiplier -lam_a
  auto eqp_lam = [&]() -> double {
    double ax0[NR];
    A_mul(P, x0, ax0);
    if (l < H) {
#pragma unroll
      for (int s = 0; s < NR; ++s) vb_ax[s * H + l] = ax0[s] - P.lo(s);   // lower-side residual
    }
    wsync();
    double rhs = 0.0;
    if (l < m) {
      const int myc = wc[l], rw = myc >> 1, rs = rw / H;
      // upper side (box / rate rows only, uniform bounds): -(a'x0 - hi)
      const double blo = (rs & 1) ? -P.dumax : -P.umax;
      rhs = (myc & 1) ? -(vb_ax[rw] + blo + blo) : vb_ax[rw];
    }
    return tri_bwd(L, ld, linv, tri_fwd(L, ld, linv, rhs, m), m);
  };
  auto x_of = [&](double lam) {
    const int lc = (l < H) ? l : 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) xc[v] = x0[v];
    for (int a = 0; a < m; ++a) {
      const double la = rdl(lam, a);
#pragma unroll
      for (int v = 0; v < NV; ++v) xc[v] -= la * Y[a * H2 + v * H + lc];
    }
  };

  // warm row: append unless linearly dependent on the rows already in (multiplier set later)
  auto warm_add = [&](int pc) {
    if (m >= cap) return;
    double yp[NV];
    const double spp = prep(pc, yp);
    const double w = fwd();
    const double lpp2 = spp - wsum(w * w);
    if (lpp2 > DEP_TOL * spp) append(pc, yp, w, lpp2, 0.0);
  };
  bool warm = false;
  unsigned long long t_wb = STAMP_T();
  if (P.gws) {
    // ---- pair: the stored active set (this step's, or the previous step's shifted)
    const int gm = P.gws[0], gt = P.gws[1];
    const bool same = gt == P.tstep, prev = gt == P.tstep - 1;
    if ((same || prev) && gm > 0 && gm <= WAVE) {
      int code = (l < gm) ? P.gws[2 + l] : -1;
      if (prev && code >= 0) {
        const int row = code >> 1, s0 = row / H, k = row - s0 * H;
        const bool keep = P.hinge(s0) ? (k >= 2) : (k >= 1);
        code = keep ? 2 * (row - 1) + (code & 1) : -1;
      }
      if (NV == 2 && P.g1 == 0.0 && P.g2 == 0.0 && code >= 0 && P.hinge((code >> 1) / H)) code = -1;
      for (int i = 0; i < gm; ++i) {
        const int pc = rdli(code, i);
        if (pc >= 0) warm_add(pc);
      }
      warm = true;
    }
  } else if (wlab) {
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
  unsigned long long t_wf = STAMP_T();
  if (warm) {
    {
      // dual feasibility: drop the most negative (or beyond-cap hinge) multiplier until none
      double lam = 0.0;
      while (m > 0) {
        lam = eqp_lam();
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
      const double tp = P.tol * (1.0 + fabs(P.lo(s)));
      if (!((wbits >> (2 * s)) & 1)) {
        const double sv = ax[s] - P.lo(s);
        if (sv < -tp && sv < best) { best = sv; code = 2 * (s * H + l); }
      }
      if (!P.hinge(s) && !((wbits >> (2 * s + 1)) & 1)) {
        const double sv = P.hi(s) - ax[s];
        if (sv < -tp && sv < best) { best = sv; code = 2 * (s * H + l) + 1; }
      }
    }
    const double bmin = wmin(best);
    if (!(bmin < 0.0)) break;
    const int pl = __ffsll((unsigned long long)__ballot(code >= 0 && best == bmin)) - 1;
    const int pc = rdli(code, pl);
    const int prow = pc >> 1, pside = pc & 1, ps = prow / H, pk = prow - ps * H;
    const bool phinge = P.hinge(ps);
    double sp = rdl(pside ? P.hi(ps) - ax[ps] : ax[ps] - P.lo(ps), pk);   // slack of p (< 0)
    double yp[NV];
    const double spp = prep(pc, yp);       // n_p' P^-1 n_p
    double up = 0.0;
    STAMP_ADD(ST_GI_SEARCH, t_gs);
    while (true) {
      if (++nsteps > GI_MAX_STEPS) return false;
      unsigned long long t_gv = STAMP_T();
      const double w = fwd();
      const double r = tri_bwd(L, ld, linv, w, m);
      // z = y_p - Y r
      double z[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) z[v] = yp[v];
      {
        const int lc = (l < H) ? l : 0;
        for (int a0 = 0; a0 < m; a0 += GEMV_U) {
          double yv[GEMV_U][NV], rv[GEMV_U];
#pragma unroll
          for (int u = 0; u < GEMV_U; ++u) {
            const int a = min(a0 + u, m - 1);
            rv[u] = (a0 + u < m) ? rdl(r, a) : 0.0;
#pragma unroll
            for (int v = 0; v < NV; ++v) yv[u][v] = Y[a * H2 + v * H + lc];
          }
#pragma unroll
          for (int u = 0; u < GEMV_U; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v) z[v] -= rv[u] * yv[u][v];
        }
      }
      const double lpp2 = spp - wsum(w * w);                   // n_p' z
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
      if (!(t < INFINITY) || tc <= t) return false;   // unbounded dual step / hinge saturates
      if (t2 < INFINITY) {
#pragma unroll
        for (int v = 0; v < NV; ++v) xc[v] += t * z[v];
        sp += t * lpp2;
      }
      if (l < m) ua -= t * r;
      up += t;
      if (t2 <= t1) {
        if (m >= cap) return false;
        append(pc, yp, w, lpp2, up);
        STAMP_ADD(ST_GI_UPD, t_gu);
        break;
      }
      drop(__ffsll((unsigned long long)__ballot(l < m && tdrop == t1)) - 1);
      STAMP_ADD(ST_GI_UPD, t_gu);
    }
  }
  // ---- exact solution of the final active set (the reduced solve with this factor):
  // lam = S^-1 (N x0 - b), x = x0 - Y lam;  kernel multipliers y_a = sign_a * lam_a
  {
    const double lam = eqp_lam();
    x_of(lam);
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
      if (P.hinge(s)) lab[s] = lo_in ? HKINK : HZERO;
      else lab[s] = lo_in ? LOWER : (hi_in ? UPPER : FREE);
      if (!P.valid(s)) lab[s] = 0;
    }
    // this step's active set: the next solve's warm start
    if (P.gws) {
      if (l < m) P.gws[2 + l] = myc;
      if (l == 0) {
        P.gws[0] = m;
        P.gws[1] = P.tstep;
      }
    }
    wsync();
  }
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
template <int NV, bool TWO, int XU = XGEMV_U>
__device__ __forceinline__ int qp_solve(QP<NV>& P, double* xs, double* zs, double* ys, signed char* lab,
                                        bool warm_lab, int max_inner, int polish_every, double* kscr, int kld,
                                        double* x_out, int& n_admm, int& n_pdas, int& n_gi) {
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
      ok = pdas<NV, XU>(P, lab, x, y, n_pdas, 1);
      if (__builtin_expect(!ok, 0)) {
        int ngi = 0;
        signed char glab[NR];
        ensure_q(P);
        if (gi_solve(P, flab, glab, x, y, ngi)) {
#pragma unroll
          for (int s = 0; s < NR; ++s) lab[s] = glab[s];
          ok = pdas<NV, XU>(P, lab, x, y, n_pdas);
        }
        n_gi += ngi;
        if (!ok) {
#pragma unroll
          for (int s = 0; s < NR; ++s) lab[s] = flab[s];
          ok = pdas<NV, XU>(P, lab, x, y, n_pdas);
        }
      }
    } else {
      ok = pdas<NV, XU>(P, lab, x, y, n_pdas);
    }
  }
  if constexpr (NV == 2) {
    // pair QP: dual active set first (no K_s^-1, no ADMM); certified by the KKT test, and
    // when that fails, polished from its labels before the ADMM fallback
    if (!ok && P.ycap > 0) {
      int ngi = 0;
      signed char glab[NR];
      if (gi_solve(P, nullptr, glab, x, y, ngi)) {
        signed char nl[NR];
        ok = kkt_check(P, glab, x, y, nl);
#pragma unroll
        for (int s = 0; s < NR; ++s) lab[s] = glab[s];
        if (!ok) ok = pdas<NV, XU>(P, lab, x, y, n_pdas);
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
        ok = pdas<NV, XU>(P, lab, x, y, n_pdas);
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
__device__ __forceinline__ void setup_agent(const DevArgs& A, int a, QP<1>& P, const Geo& g, double* xfac) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, l = lid();
  const bool in = l < H;
  P.coefP = 2.0 * c.Pnorm + c.rho * (double)A.nbr_cnt[a];
  P.mm[0] = g.mm;
  double* Kc = A.Kx_cache + (size_t)a * H * H;
  double* Pc = A.Pinv_x + (size_t)a * H * H;
  double* sc = A.sc_x + (size_t)a * 4 * HCAP;
  const int li = l < HCAP ? l : 0;
  // P depends on the agent's speed only (make_geo): K_s^-1, P^-1 and the scaling are
  // cached in HBM per scenario and rebuilt only when the ADMM penalty differs.
  if (__builtin_expect(A.xcache_rho[a] == P.rho, 1)) {
    P.D[0] = in ? sc[li] : 0.0;
    P.E[0] = in ? sc[HCAP + li] : 0.0;
    P.E[1] = (l < H - 1) ? sc[2 * HCAP + li] : 0.0;
    if (P.kf32 || P.K != Kc) {   // LDS image of K_s^-1: loaded by qp_solve when ADMM is needed
      P.Kcache = Kc;
      P.kready = false;
    }
    wsync();
    return;
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
  if (l == 0) A.xcache_rho[a] = P.rho;
  __threadfence();      // P^-1 (read back through L2 by the polish) is visible to this wave
  wsync();
}

// Pair (z-step) QP of cost_function_edge (PI_ADMM_class.py:145-169), heading frozen at
// xt (MATLAB symbolic dynamic_update_edge, ADMM_CVX_..._PI_antiwindup.m:378-397).
// Variables [uh_1; uh_2]; hinge rows G_k = [g1 T(k+1,.), g2 T(k+1,.)],
// h_k = D^2 + |dbar|^2 - 2 dbar'(c2 - c1)_{k+1}.  Builds the polish tables P^-1 (HBM),
// PGt = P^-1 G' (HBM), GPG = G P^-1 G' (HBM) and K_s^-1 (LDS).
__device__ __forceinline__ void setup_pair(const DevArgs& A, int e, QP<2>& P, const Geo& g1, const Geo& g2,
                                           double c1x, double c1y, double c2x, double c2y, const double* seeds,
                                           double* scr, double* Ke_lds, double deff) {
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, n = 2 * H, l = lid();
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
  P.coefP = c.rho;
  P.mm[0] = g1.mm;
  P.mm[1] = g2.mm;

  // ---- P_v^-1 blocks (HBM), Y = P_v^-1 T' (PGt, unscaled by g) and Z_v = T P_v^-1 T' (GPG):
  // speed-only, so built once per scenario; g1, g2 scale them on the fly (s_gather, x recovery)
  if (__builtin_expect(!A.ecache[e], 0)) {
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
    if (l == 0) A.ecache[e] = 1;
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
// ============================================================ the MPC-step kernel
struct CompLds {
  double *pos, *xt, *seed, *u, *hat, *lam, *S, *D, *last, *sc;
};

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

// One launch runs outer iterations [it0, it1) of MPC step t for every component (one
// workgroup each).  The fused mode is one launch (0, max_outer, FIRST | LAST); the global
// termination mode (term_global, reference quirk B9) runs one launch per outer iteration,
// with the per-step state carried in HBM between launches (restore / save below) and the
// stop decision taken by the host from all-reduced partials, then a LAST launch with no
// iterations for the outputs and the propagation.
template <bool BIG>
__device__ __forceinline__ void mpc_step_body(const DevArgs& A, int t, int it0, int it1, int flags, int slot,
                                              int& nbar) {
  extern __shared__ double lds[];
  __shared__ int s_int[NW * 272];   // per wave: x ids [128], z ids [128], fstate x, fstate z
  const piadmm_config_t& c = A.cfg;
  const int H = c.H, H1 = H + 1;
  const int ci = blockIdx.x;
  const int w = threadIdx.x >> 6, l = lid();
  const int a0 = A.comp_ptr[ci];
  const int na = A.comp_ptr[ci + 1] - a0;
  const int e = A.comp_edge[ci];

  // ---- LDS carve (lds_bytes() in piadmm_internal.h)
  constexpr bool big = BIG;      // H > HMAX (launch_mpc_step picks the instantiation)
  const bool f32 = c.precision == 1;   // ADMM matrices in fp32 (lds_bytes: half the space)
  double *Kx = nullptr, *Gx = nullptr, *Ke = nullptr, *scr, *xfac_all, *xt_all = nullptr, *vec_all;
  float* Kef = nullptr;
  float* Kxf = nullptr;
  if (!big) {
    double* p = lds;
    if (f32) { Kxf = (float*)p; p += H * H; }            // 2 x H*H fp32 agent K_s^-1
    else { Kx = p; p += 2 * H * H; }                     // 2 x H*H   agent K_s^-1
    Gx = p; p += 2 * (H * H + H);                        // 2 x (H*H+H) agent polish G | g
    if (f32) { Kef = (float*)p; p += 2 * H * H; }        // 4*H*H fp32 pair K_s^-1
    else { Ke = p; p += 4 * H * H; }                     // 4*H*H     pair K_s^-1
    scr = p;                                             // 64 x LD   pair scratch (wave 0)
    xfac_all = scr + 64 * LD;                            // NW x HMAX x (HMAX+1)
    xt_all = xfac_all + NW * HMAX * (HMAX + 1);          // NW x (HMAX+1) x XLD
    vec_all = xt_all + NW * (HMAX + 1) * XLD;            // NW x 512
  } else {
    Ke = (e >= 0) ? A.Ke_g + (size_t)e * 4 * H * H : nullptr;   // HBM / L2 (built in place)
    scr = lds;                                           // 64 x LD   pair scratch (wave 0)
    xfac_all = scr + 64 * LD;                            // NW x xrows(H) x (xrows+1)
    vec_all = xfac_all + NW * xrows(H) * (xrows(H) + 1); // NW x 512
  }
  double* fdiag_all = vec_all + NW * 512;                // NW x 256
  CompLds S;
  S.pos = fdiag_all + NW * 256;
  S.xt = S.pos + 8 * H1;   // pos_old double-buffered by outer-iteration parity
  S.seed = S.xt + 6;
  S.u = S.seed + 4;
  S.hat = S.u + 2 * H;
  S.lam = S.hat + 4 * H1;
  S.S = S.lam + 4 * H1;
  S.D = S.S + 4 * H1;
  S.last = S.D + 4 * H1;
  S.sc = S.last + 4 * H1;
  if (big && f32) Kef = (float*)(S.sc + 32);             // big mode: fp32 image of the pair K_s^-1
  WaveMem wm{vec_all + w * 512, s_int + w * 272};
  double* xfac = big ? xfac_all + w * xrows(H) * (xrows(H) + 1) : xfac_all + w * HMAX * (HMAX + 1);
  double* xdiag = fdiag_all + w * 256;
  double* zdiag = xdiag + 128;
  int* xids = wm.ib;
  int* zids = wm.ib + 128;
  int* xfs = wm.ib + 256;
  int* zfs = wm.ib + 257;
  if (l == 0) {
    xfs[0] = -1;
    zfs[0] = -1;
  }

  const bool first = (flags & F_FIRST) != 0;
  const bool last_launch = (flags & F_LAST) != 0;
  const bool global = (flags & F_GLOBAL) != 0;
  const bool coop = (flags & F_COOP) != 0;   // global stop decided in-kernel (cooperative launch)
  int gflag = 0;                             // coop: some pair ever collided (casadi/main.py:115)
  bool nanlast = (flags & F_NANLAST) != 0;
  // ---- seeds (casadi/main.py:48-49) and zero per-step state (:52-63)
  if ((int)threadIdx.x < na) {
    const int a = a0 + threadIdx.x;
    const double x = A.xt[3 * a], y = A.xt[3 * a + 1], th = A.xt[3 * a + 2], s = A.spd[a];
    S.xt[3 * threadIdx.x + 0] = x;
    S.xt[3 * threadIdx.x + 1] = y;
    S.xt[3 * threadIdx.x + 2] = th;
    S.seed[2 * threadIdx.x + 0] = around(x + c.dt * s * cos(th), c.round_decimals);
    S.seed[2 * threadIdx.x + 1] = around(y + c.dt * s * sin(th), c.round_decimals);
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
      for (int i = threadIdx.x; i < na * H; i += blockDim.x) S.u[i] = A.u[(size_t)a0 * H + i];
      for (int k = 0; k < 5; ++k)
        for (int i = threadIdx.x; i < 4 * H1; i += blockDim.x)
          edge_lds[k][i] = (e >= 0) ? edge_hbm[k][(size_t)e * 4 * H1 + i] : 0.0;
    }
  }
  __syncthreads();
  // pair safety distance (a13 tightening from the step's start states, else dis_thres)
  double deff = c.dis_thres;
  if (e >= 0 && c.tighten && na == 2)
    deff = c.dis_thres + delay_norm(c, S.xt[2], A.spd[a0]) + delay_norm(c, S.xt[5], A.spd[a0 + 1]);
  unsigned long long t_k = STAMP_T();

  // ---- per-step QP setup (registers of the owning wave stay live for the whole step)
  QP<1> qx;
  double xs_x[1] = {0.0}, zs_x[2] = {0.0, 0.0}, ys_x[2] = {0.0, 0.0};
  signed char lab_x[2] = {0, 0};
  bool warm_x = false;
  int status_x = 0;
  int nnb = 0;
  Geo gx;
  double cx_own = 0.0, cy_own = 0.0;
  if (w < na) {
    unsigned long long t0 = STAMP_T();
    const int a = a0 + w;
    gx = make_geo(S.xt + 3 * w, A.spd[a], c);
    affine_c(gx, c.dt, H, cx_own, cy_own);
    qp_common(c, H, A.rho_x[a], qx);
    qx.K = big ? A.Kx_cache + (size_t)a * H * H : (Kx ? Kx + w * H * H : nullptr);
    qx.Kf = (!big && f32) ? Kxf + w * H * H : nullptr;
    qx.kf32 = !big && f32;                        // big mode: the x-step K stays fp64 in HBM
    qx.Pinv = A.Pinv_x + (size_t)a * H * H;    // L2-resident; read only when W changes
    qx.G = big ? A.Gx_g + (size_t)a * (H * H + H) : Gx + w * (H * H + H);
    qx.vb = wm.vb;
    qx.fac = xfac;
    qx.XT = big ? A.XT_g + (size_t)a * H1 * XLDG : xt_all + w * (HMAX + 1) * XLD;
    qx.xld = big ? XLDG : XLD;
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
    // (big mode: a per-agent HBM buffer, K_s^-1 stays intact)
    qx.Y = big ? A.Yx_g + (size_t)a * WAVE * H : (f32 ? (double*)(Kxf + w * H * H) : Kx + w * H * H);
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
  QP<2> qe;
  double xs_e[2] = {0.0, 0.0}, zs_e[5] = {0, 0, 0, 0, 0}, ys_e[5] = {0, 0, 0, 0, 0};
  signed char lab_e[5] = {0, 0, 0, 0, 0};
  bool warm_e = false;
  int status_e = 0;
  Geo ge1, ge2;
  double c1x = 0.0, c1y = 0.0, c2x = 0.0, c2y = 0.0;
#ifdef PIADMM_DIAG_NO_PAIR   // diagnostic timing build only: no pair QP code at all
  if (false) {
#else
  if (w == 0 && e >= 0) {
#endif
    unsigned long long t0 = STAMP_T();
    ge1 = make_geo(S.xt + 0, A.spd[a0], c);
    ge2 = make_geo(S.xt + 3, A.spd[a0 + 1], c);
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
    qe.vb = wm.vb;
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
    qe.y_in_k = true;
    qe.gws = A.gi_ws + (size_t)e * GI_WS;
    qe.tstep = t;
    // Ke doubles as the H x 2H staging of the per-scenario pair tables; with fp32 images in
    // LDS mode the fp32 region (2H^2 doubles of space) takes that role
    setup_pair(A, e, qe, ge1, ge2, c1x, c1y, c2x, c2y, S.seed, scr, Ke ? Ke : (double*)Kef, deff);
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
  __syncthreads();

  const bool nonlin_pos = c.pos_model != 0;
  const double thr = c.collide_sq_thres ? deff * deff : deff;
  int flag = first ? 0 : A.cst[(size_t)ci * 4 + 0];
  int aliased = first ? 0 : A.cst[(size_t)ci * 4 + 1];
  int iters = it0;
  int n_xqp = 0, n_zqp = 0, n_admm_x = 0, n_admm_z = 0, n_pdas_x = 0, n_pdas_z = 0, n_inexact = 0, n_gi = 0;
  bool act = (!first && e >= 0) ? A.edge_active[e] != 0 : false;
  double dis_chk = (!first && e >= 0) ? A.dischk[e] : NAN;
  double* resid = A.resid + ((size_t)slot * A.C + ci) * c.max_outer * 2;   // slot: step of the launch
  if (first)
    for (int i = threadIdx.x; i < 2 * c.max_outer; i += blockDim.x) resid[i] = NAN;   // "not evaluated"
  if (coop && ci == 0)
    for (int i = threadIdx.x; i < 2 * c.max_outer; i += blockDim.x) A.ghist[(size_t)slot * 2 * c.max_outer + i] = NAN;
  // the own agent's start state and speed in registers for the per-iteration rollout
  double rl_x0 = 0.0, rl_y0 = 0.0, rl_th0 = 0.0, rl_s = 0.0, rl_sl = 0.0;
  if (w < na) {
    rl_x0 = S.xt[3 * w + 0];
    rl_y0 = S.xt[3 * w + 1];
    rl_th0 = S.xt[3 * w + 2];
    rl_s = A.spd[a0 + w];
    rl_sl = rl_s / c.L;
  }
  // reference positions of the own agent at time lanes (fixed for the step)
  double rx_own = 0.0, ry_own = 0.0;
  if (w < na && l <= H) {
    const double* rp = A.ref + (size_t)(a0 + w) * 2 * A.T;
    rx_own = rp[t + l];
    ry_own = rp[A.T + t + l];
  }

  // the x-step's consensus term (cx - hat + lam) of the own direction in registers: hat and lam
  // change only in a z-step, after which it is reloaded (behind the second barrier)
  const bool cpl = w < na && nnb > 0 && e >= 0 && l <= H;
  double cpx = 0.0, cpy = 0.0;
  auto load_cp = [&]() {
    if (cpl) {
      const int d = w;   // agent local 0 owns hat_{v1 v2} (dir 0), agent 1 dir 1
      cpx = cx_own - S.hat[(d * 2 + 0) * H1 + l] + S.lam[(d * 2 + 0) * H1 + l];
      cpy = cy_own - S.hat[(d * 2 + 1) * H1 + l] + S.lam[(d * 2 + 1) * H1 + l];
    }
  };
  load_cp();
  for (int it = it0; it < it1; ++it) {
    iters = it + 1;
    // this iteration's pos_old buffer: a wave may start the next iteration's x-step while
    // the other still reads this one's positions (no second barrier without a z-step)
    double* const pos = S.pos + (it & 1) * 4 * H1;
    // -------- x-step: every agent of the component (casadi/main.py:81-106)
    if (w < na) {
      unsigned long long t_xs = STAMP_T();
      const int a = a0 + w;
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
#ifdef PIADMM_DIAG_NO_XQP   // diagnostic timing build only: skip the x-step QP
      const int stx = 0;
      ustar[0] = 1e-3 * qx.wq;
#else
      const int stx = qp_solve<1, false, BIG ? 8 : XGEMV_U>(qx, xs_x, zs_x, ys_x, lab_x, warm_x, c.max_inner, c.polish_every, xfac,
                               qx.fld, ustar, n_admm_x, n_pdas_x, n_gi);
#endif
      STAMP_ADD(ST_XQP, t_q);
      status_x |= stx;
      ++n_xqp;
      n_inexact += (stx & PIADMM_QP_INEXACT) ? 1 : 0;
      warm_x = true;
      unsigned long long t_rd = STAMP_T();
      const double u = around(ustar[0], c.round_decimals);
      STAMP_ADD(ST_ROUND, t_rd);
      double px, py, pth;
      unsigned long long t_r = STAMP_T();
#ifdef PIADMM_DIAG_NO_ROLL  // diagnostic timing build only: skip the rollout
      px = py = pth = u;
#else
      rollout_r(rl_x0, rl_y0, rl_th0, rl_s, rl_sl, (l < H) ? u : 0.0, c, H, nonlin_pos, px, py, pth);
#ifdef PIADMM_DIAG_ROLL2     // diagnostic timing build only: the rollout twice (same result)
      {
        double u2 = (l < H) ? u : 0.0, qx2, qy2, qt2;
        asm volatile("" : "+v"(u2));
        rollout(S.xt + 3 * w, A.spd[a], u2, c, H, nonlin_pos, qx2, qy2, qt2);
        asm volatile("" : "+v"(qx2), "+v"(qy2), "+v"(qt2));
        asm volatile("" : : "v"(px), "v"(py), "v"(pth));
        px = qx2; py = qy2; pth = qt2;
      }
#endif
#endif
      STAMP_ADD(ST_XROLL, t_r);
      if (l <= H) {
        pos[(w * 2 + 0) * H1 + l] = px;
        pos[(w * 2 + 1) * H1 + l] = py;
      }
      if (l < H) S.u[w * H + l] = u;
      STAMP_ADD(ST_XSTEP, t_xs);
    }
    unsigned long long t_sa = STAMP_T();
    __syncthreads();
    STAMP_ADD(ST_SYNC_A, t_sa);
    // -------- collision graph (casadi/main.py:110-118), computed by every wave
    act = false;
    if (e >= 0 && na == 2) {
      bool hit = false;
      if (l <= H) {
        const double dx = pos[0 * H1 + l] - pos[2 * H1 + l];
        const double dy = pos[1 * H1 + l] - pos[3 * H1 + l];
        hit = (dx * dx + dy * dy) < thr;
      }
      act = wany(hit);
    }
    if (!act && flag == 0 && !c.fixed_iters && !global) break;   // no edge ever: stop (:115-116)
    flag = 1;
    // -------- z-step + dual update on the colliding pair (casadi/main.py:121-162)
#ifdef PIADMM_DIAG_NO_PAIR
    if (false) {
#else
    if (__builtin_expect(act && w == 0, 0)) {     // cold: about once per MPC step
#endif
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
      const int ste = qp_solve<2, BIG>(qe, xs_e, zs_e, ys_e, lab_e, warm_e, c.max_inner, c.polish_every,
                               big ? Ke : scr, big ? 2 * H : LD, uh,
                               n_admm_z, n_pdas_z, n_gi);
      STAMP_ADD(ST_ZQP, t_zq);
      status_e |= ste;
      ++n_zqp;
      n_inexact += (ste & PIADMM_QP_INEXACT) ? 1 : 0;
      warm_e = true;
      // hat positions: nonlinear rollout of the rounded pair controls (:153-158)
      double hx[2], hy[2], hth;
      for (int v = 0; v < 2; ++v) {
        const double uv = (l < H) ? around(uh[v], c.round_decimals) : 0.0;
        rollout(S.xt + 3 * v, A.spd[a0 + v], uv, c, H, true, hx[v], hy[v], hth);
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
        S.sc[1] = aliased ? 0.0 : 2.0 * sqrt(ss);
        S.sc[2] = rdl(dist, 1);
      }
      STAMP_ADD(ST_ZSTEP, t_z);
    }
    // -------- termination (casadi/main.py:164-181; MATLAB :191-210).  Wave 0 (which wrote
    // S.sc) records the residuals and, unless the component stops, last_iter_hat_pos before
    // the barrier; after it every wave takes the same stop decision from S.sc.  One barrier per
    // half-iteration: S.sc is rewritten only after the next iteration's first barrier.
    if (w == 0) {
      unsigned long long t_tw = STAMP_T();
      wsync();
      const double rk0 = act ? S.sc[0] : 0.0;
      const double sk0 = act ? S.sc[1] : 0.0;
      const double dc0 = act ? S.sc[2] : dis_chk;
      if (l == 0) {
        resid[2 * it + 0] = rk0;
        resid[2 * it + 1] = sk0;
      }
      const bool stop0 = !c.fixed_iters && !global && rk0 <= c.eps_pri && sk0 <= c.eps_dual &&
                         (!c.term_dist_check || dc0 > deff);
      // last_iter_hat_pos = hat_pos_old: only a z-step changes hat, so the copy is needed
      // only after one (S.last already equals hat otherwise)
      if (__builtin_expect(act && !stop0 && !c.alias_dual_residual, 0))
        for (int i = l; i < 4 * H1; i += WAVE) S.last[i] = S.hat[i];
      STAMP_ADD(ST_TERMW, t_tw);
    }
    // second barrier only after a z-step (it wrote hat, lam, S, D, last and S.sc); without
    // one every wave takes the stop decision from its registers (rk = sk = 0)
    unsigned long long t_sb = STAMP_T();
    if (__builtin_expect(act, 0)) {
      __syncthreads();
      load_cp();
    }
    STAMP_ADD(ST_SYNC_B, t_sb);
    const double rk = act ? S.sc[0] : 0.0;
    const double sk = act ? S.sc[1] : 0.0;
    if (act) dis_chk = S.sc[2];
    if (!c.fixed_iters && !global && rk <= c.eps_pri && sk <= c.eps_dual &&
        (!c.term_dist_check || dis_chk > deff))
      break;
    if (coop && !c.fixed_iters) {
      // -------- global termination over all components, in-kernel (single rank): the
      // partials of k_term_partials, one grid barrier, every workgroup sums them in the same
      // order and applies the host's stop rules (piadmm_capi.cpp run_steps) identically.
      // Double-buffered by the parity of the launch's barrier count (iterations and steps),
      // so one barrier per iteration suffices; agent-scope atomic accesses keep the
      // partials out of the non-coherent per-CU cache.
      unsigned long long t_gb = STAMP_T();
      double* part = A.gpart + (size_t)(nbar & 1) * A.C * 5;
      ++nbar;
      if (threadIdx.x == 0) {
        const bool seen = (e >= 0) && (dis_chk == dis_chk);
        const double pv[5] = {rk, sk, (e >= 0 && act) ? 1.0 : 0.0, seen ? 1.0 : 0.0,
                              (seen && !(dis_chk > deff)) ? 1.0 : 0.0};
#pragma unroll
        for (int q = 0; q < 5; ++q)
          __hip_atomic_store(&part[ci * 5 + q], pv[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      cooperative_groups::this_grid().sync();
      {
        // all threads load (components tid, tid + 128, ...), then five threads sum the
        // per-thread partials in thread order: a fixed order, identical in every workgroup
        double v[5] = {0, 0, 0, 0, 0};
        for (int k = threadIdx.x; k < A.C; k += blockDim.x)
#pragma unroll
          for (int q = 0; q < 5; ++q)
            v[q] += __hip_atomic_load(&part[k * 5 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        double* red = vec_all;           // the waves' vector buffers are free between QP solves
#pragma unroll
        for (int q = 0; q < 5; ++q) red[q * NW * WAVE + threadIdx.x] = v[q];
        __syncthreads();
        if (threadIdx.x < 5) {
          double tot = 0.0;
          for (int k = 0; k < NW * WAVE; ++k) tot += red[threadIdx.x * NW * WAVE + k];
          S.sc[16 + threadIdx.x] = tot;
        }
      }
      __syncthreads();
      const double trk = S.sc[16], tsk = S.sc[17], tact = S.sc[18], tseen = S.sc[19], tbad = S.sc[20];
      __syncthreads();
      STAMP_ADD(ST_TERM, t_gb);
      if (tact == 0.0 && gflag == 0) {       // no pair collides anywhere: stop (:115-116)
        nanlast = true;
        break;
      }
      gflag = 1;
      if (ci == 0 && threadIdx.x == 0) {
        A.ghist[((size_t)slot * c.max_outer + it) * 2 + 0] = trk;
        A.ghist[((size_t)slot * c.max_outer + it) * 2 + 1] = tsk;
      }
      const bool dist_ok = tseen > 0.0 && tbad == 0.0;
      if (trk <= c.eps_pri && tsk <= c.eps_dual && (!c.term_dist_check || dist_ok)) break;
    }
    if (c.alias_dual_residual) aliased = 1;
  }
  __syncthreads();
  STAMP_ADD(ST_KERNEL, t_k);
  unsigned long long t_epi = STAMP_T();

  // ---- work counters (accumulated across launches; one workgroup owns row ci)
  {
    __shared__ int s_cnt[NW][8];
    if (l == 0) {
      s_cnt[w][0] = n_xqp; s_cnt[w][1] = n_zqp; s_cnt[w][2] = n_admm_x; s_cnt[w][3] = n_admm_z;
      s_cnt[w][4] = n_pdas_x; s_cnt[w][5] = n_pdas_z; s_cnt[w][6] = n_inexact; s_cnt[w][7] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long* cn = A.counters + (size_t)ci * 8;
      cn[0] += (unsigned long long)(iters - it0);
      for (int k = 0; k < 6; ++k) {
        unsigned long long sum = 0;
        for (int ww = 0; ww < NW; ++ww) sum += (unsigned long long)s_cnt[ww][k];
        cn[k + 1] += sum;
      }
      unsigned long long inex = 0;
      for (int ww = 0; ww < NW; ++ww) inex += (unsigned long long)s_cnt[ww][6];
      cn[7] += inex;
    }
  }
  // ---- state of this launch (every launch) and outputs / propagation (LAST, casadi/main.py:185-192)
  if (threadIdx.x == 0) {
    A.iters[ci] = iters;
    if (e >= 0) {
      A.edge_active[e] = act ? 1 : 0;
      A.dischk[e] = dis_chk;
    }
    A.cst[(size_t)ci * 4 + 0] = flag;
    A.cst[(size_t)ci * 4 + 1] = aliased;
    if (coop && ci == 0) A.giters[slot] = iters;
    if (nanlast && iters > 0) {      // global stop at the collision test of this iteration
      resid[2 * (iters - 1) + 0] = NAN;
      resid[2 * (iters - 1) + 1] = NAN;
    }
  }
  {
    __shared__ int s_warm;
    if (threadIdx.x == 0) s_warm = 0;
    __syncthreads();
    if (l == 0 && w < na && warm_x) atomicOr(&s_warm, 1 << w);
    if (l == 0 && w == 0 && e >= 0 && warm_e) atomicOr(&s_warm, 4);
    __syncthreads();
    if (threadIdx.x == 0) A.cst[(size_t)ci * 4 + 2] = s_warm;
  }
  if (w < na) {
    const int a = a0 + w;
    const double* posl = S.pos + ((iters - 1) & 1) * 4 * H1;   // the last executed iteration's buffer
    for (int i = l; i < 2 * H1; i += WAVE) A.pos_old[(size_t)a * 2 * H1 + i] = posl[w * 2 * H1 + i];
    const double u = (l < H) ? S.u[w * H + l] : 0.0;
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
    if (!last_launch) {
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
  if (w == 0 && e >= 0) {
    if (l == 0) A.rho_e[e] = qe.rho;
    if (!last_launch) {
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
  }
  if (e >= 0) {
    double* const edge_lds[5] = {S.hat, S.lam, S.S, S.D, S.last};
    double* const edge_hbm[5] = {A.hat, A.lam, A.Sacc, A.Dacc, A.last};
    for (int k = 0; k < 5; ++k)
      for (int i = threadIdx.x; i < 4 * H1; i += blockDim.x) edge_hbm[k][(size_t)e * 4 * H1 + i] = edge_lds[k][i];
    if (threadIdx.x == 0) A.status[A.N + e] = status_e;
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
template <bool BIG>
__global__ void __launch_bounds__(NW * WAVE) k_mpc_step(DevArgs A, int t0, int nsteps, int it0, int it1, int flags) {
#ifdef PIADMM_STAMPS
  if (threadIdx.x < 64) s_stamps[threadIdx.x] = 0ull;
  __syncthreads();
#endif
  int nbar = 0;   // grid barriers so far (coop): parity of the termination partials
  for (int k = 0; k < nsteps; ++k) {
    mpc_step_body<BIG>(A, t0 + k, it0, it1, flags, k, nbar);
    __syncthreads();
  }
#ifdef PIADMM_STAMPS
  if (threadIdx.x < 64 && g_stamps) atomicAdd(&g_stamps[blockIdx.x * 64 + threadIdx.x], s_stamps[threadIdx.x]);
#endif
}

// Global termination partials of outer iteration `it` (one workgroup): rk, sk summed over
// components, active pairs, pairs with a distance check, pairs failing it.
__global__ void __launch_bounds__(256) k_term_partials(DevArgs A, int it, double* out) {
  __shared__ double red[5][256];
  double v[5] = {0, 0, 0, 0, 0};
  for (int ci = threadIdx.x; ci < A.C; ci += 256) {
    const double* r = A.resid + ((size_t)ci * A.cfg.max_outer + it) * 2;
    if (r[0] == r[0]) v[0] += r[0];
    if (r[1] == r[1]) v[1] += r[1];
  }
  for (int e = threadIdx.x; e < A.E; e += 256) {
    v[2] += A.edge_active[e] ? 1.0 : 0.0;
    const double d = A.dischk[e];
    if (d == d) {
      v[3] += 1.0;
      v[4] += (d > A.deff[e]) ? 0.0 : 1.0;
    }
  }
  for (int k = 0; k < 5; ++k) red[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int k = 0; k < 5; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 5) out[threadIdx.x] = red[threadIdx.x][0];
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

int launch_mpc_step(const DevArgs& a, int t, int nsteps, int it0, int it1, int flags, hipStream_t s) {
  const size_t sh = lds_bytes(a.cfg.H, a.cfg.precision);
  const bool big = a.cfg.H > HMAX;
  static size_t attr[2] = {0, 0};     // dynamic LDS limit set so far per instantiation
#ifdef PIADMM_STAMPS
  static unsigned long long* last = nullptr;
  if (a.stamps != last) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &a.stamps, sizeof(void*)) != hipSuccess) return -1;
    last = a.stamps;
  }
#endif
  const void* fn = big ? (const void*)k_mpc_step<true> : (const void*)k_mpc_step<false>;
  if (sh > attr[big]) {
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess) return -1;
    attr[big] = sh;
  }
  if (flags & F_COOP) {
    // every workgroup must be resident for the grid barrier: the cooperative launch fails
    // (and the caller falls back to host-decided termination) rather than deadlock
    DevArgs aa = a;
    void* args[] = {&aa, &t, &nsteps, &it0, &it1, &flags};
    return hipLaunchCooperativeKernel(fn, dim3(a.C), dim3(NW * WAVE), args, (unsigned)sh, s) == hipSuccess ? 0 : -1;
  }
  if (big)
    hipLaunchKernelGGL(k_mpc_step<true>, dim3(a.C), dim3(NW * WAVE), sh, s, a, t, nsteps, it0, it1, flags);
  else
    hipLaunchKernelGGL(k_mpc_step<false>, dim3(a.C), dim3(NW * WAVE), sh, s, a, t, nsteps, it0, it1, flags);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Can every workgroup of a k_mpc_step launch be resident at once (cooperative launch)?
bool coop_fits(const DevArgs& a, int device) {
  int coopok = 0, ncu = 0, per = 0;
  if (hipDeviceGetAttribute(&coopok, hipDeviceAttributeCooperativeLaunch, device) != hipSuccess || !coopok)
    return false;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return false;
  const size_t sh = lds_bytes(a.cfg.H, a.cfg.precision);
  const bool big = a.cfg.H > HMAX;
  const void* fn = big ? (const void*)k_mpc_step<true> : (const void*)k_mpc_step<false>;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, NW * WAVE, sh) != hipSuccess) return false;
  return (long long)per * ncu >= (long long)a.C;
}

int launch_term_partials(const DevArgs& a, int it, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_term_partials, dim3(1), dim3(256), 0, s, a, it, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_resid_history(const DevArgs& a, int nsteps, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_resid_history, dim3(a.cfg.max_outer, nsteps), dim3(256), 0, s, a, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_pair_deff(const DevArgs& a, hipStream_t s) {
  if (a.E == 0) return 0;
  hipLaunchKernelGGL(k_pair_deff, dim3((a.E + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pd
