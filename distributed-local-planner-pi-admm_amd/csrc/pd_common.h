// pd_common.h -- wave primitives, the reference's arithmetic (rollouts, rounding) and the
// in-wave dense kernels shared by the MI355X kernels of libpiadmm (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "piadmm_internal.h"

namespace pd {

// Diagnostic phase stamps (separate build, never in the measured library).
#ifdef PIADMM_STAMPS
// cycles accumulate in LDS per wave (one ds_add_u64 per stamp, lane 0; slot + 64 x wave, waves
// 0..3) and are flushed to g_stamps (C x 4 x 64) once per launch, so that a stamp costs an LDS
// atomic, not a global one
constexpr int STAMP_WAVES = 4;
__device__ unsigned long long* g_stamps;
__shared__ unsigned long long s_stamps[64 * STAMP_WAVES];
#define STAMP_T() __builtin_amdgcn_s_memtime()
#define STAMP_W() (((int)threadIdx.x >> 6) & (STAMP_WAVES - 1))
#define STAMP_ADD(slot, t0)                                                                   \
  do {                                                                                        \
    const unsigned long long _d = __builtin_amdgcn_s_memtime() - (t0);                       \
    if (__lane_id() == 0) atomicAdd(&s_stamps[(slot) + 64 * STAMP_W()], _d);                 \
  } while (0)
#define STAMP_CNT(slot, n)                                                                    \
  do {                                                                                        \
    if (__lane_id() == 0) atomicAdd(&s_stamps[(slot) + 64 * STAMP_W()], (unsigned long long)(n)); \
  } while (0)
#else
#define STAMP_CNT(slot, n) ((void)(n))
#define STAMP_T() 0ull
#define STAMP_ADD(slot, t0) ((void)(t0))
#endif
enum StampSlot { ST_SETUP_X = 0, ST_SETUP_Z, ST_XSTEP, ST_XQP, ST_XRED, ST_XROLL, ST_ZSTEP, ST_ZQP, ST_ZRED,
                 ST_KERNEL, ST_RED_GEMV, ST_RED_S, ST_RED_CHOL, ST_RED_X, ST_ADMM, ST_XQ, ST_TERM,
                 ST_SZ_RUIZ, ST_SZ_KMAT, ST_SZ_GJ, ST_SZ_PRE, ST_ZR_GEMV, ST_ZR_S, ST_ZR_CHOL, ST_ZR_X,
                 ST_ZR_SOLVE, ST_XR_SOLVE, ST_ZKKT, ST_XKKT, ST_GI_SEARCH, ST_GI_SOLVE, ST_GI_UPD,
                 ST_SYNC_A, ST_TERMW, ST_SYNC_B, ST_RSX_PRE, ST_QEPI, ST_ROUND,
                 // graph kernel: event counts (not cycles) in the same buffer
                 ST_N_GIZ = 40, ST_N_GIX, ST_N_ZQP, ST_N_ZFAIL, ST_N_XREBUILD,
                 // dual active set detail (pair QPs only): cycles of fwd / bwd / Y pass / drop, and counts
                 ST_GI_FWD = 45, ST_GI_BWD, ST_GI_YPASS, ST_GI_DROP, ST_N_DROP, ST_N_APPEND, ST_N_WARMROW,
                 ST_SUM_M, ST_SUM_MEND, ST_N_GICALL,
                 // the pair's warm build per appended row: P^-1 n + A y (prep), S^-1 v + pivot, the bordering
                 ST_WARM_PREP = 56, ST_WARM_SINV, ST_WARM_APPEND, NSTAMP = 64 };

// ============================================================ address spaces
// The kernels' scratch pointers travel through structs that also carry HBM pointers, so the
// compiler sees generic pointers and emits flat loads (TA path; waits on vmcnt AND lgkmcnt) for
// what is LDS.  Code that knows a pointer is the wave's LDS scratch addresses it through an
// address_space(3) view (ds_read / ds_write); in_lds() tells the two apart at run time where a
// pointer is LDS in one mode and HBM in another (a uniform branch).
typedef __attribute__((address_space(3))) double ldsd;
typedef double dv2 __attribute__((ext_vector_type(2)));     // two doubles: 16-byte LDS accesses
typedef __attribute__((address_space(3))) dv2 ldsd2;
__device__ __forceinline__ ldsd* lds_ptr(double* p) { return (ldsd*)p; }
__device__ __forceinline__ const ldsd* lds_ptr(const double* p) { return (const ldsd*)p; }
typedef __attribute__((address_space(1))) double gbld;      // HBM (global) view
__device__ __forceinline__ gbld* gbl_ptr(double* p) { return (gbld*)p; }
__device__ __forceinline__ const gbld* gbl_ptr(const double* p) { return (const gbld*)p; }
// generic pointer into LDS? (device pass only; the host pass never runs device code)
__device__ __forceinline__ bool in_lds(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p);
#else
  (void)p;
  return false;
#endif
}

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
// A wave-uniform int the compiler cannot prove uniform (an active-set size carried in a VGPR) into
// an SGPR: loop bounds, clamps and row offsets derived from it become scalar ops, and an LDS
// address is one v_add instead of a min / mul_lo (quarter rate) / shift-add chain per element.
__device__ __forceinline__ int unif(int v) { return __builtin_amdgcn_readfirstlane(v); }

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

// The in-kernel grid barrier of the natural global stop test (one rank, cooperative launch: every
// workgroup resident, every one calls it the same number of times).  Each workgroup release-stores
// the barrier's epoch into its own word -- no read-modify-write on one shared counter to serialise
// the arrivals -- and its first wave polls every word until all hold the epoch (or a later one).
// Measured per barrier with the partials' reduction (tools/gbar_ubench.hip): 128 workgroups
// 14.3 us with cooperative_groups' grid sync -> 6.0 us; 32 workgroups 6.8 -> 3.0 us.  Epochs grow
// across launches (DevArgs::gbar_base), so the words are never reset.  The caller's thread 0
// stores its partials before the call: its release store orders them.
__device__ __forceinline__ void grid_flag_barrier(unsigned long long* words, int n, int me, unsigned long long epoch) {
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&words[me], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < WAVE) {
    while (true) {
      bool ok = true;
      for (int k = threadIdx.x; k < n; k += WAVE)
        ok = ok && __hip_atomic_load(&words[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (wall(ok)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

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

// ============================================================ near-tie log (piadmm_get_near_ties)
#ifndef PIADMM_NO_TIES   // (-DPIADMM_NO_TIES: a diagnostic build without the log, to price it)
// One event of a discrete decision taken within A.tie_tol of its threshold.  Called by ONE lane,
// in a cold branch (ties are rare: the hot path pays a compare and a ballot).
__device__ __forceinline__ void tie_record(const DevArgs& A, int t, int it, int kind, int id, int idx, double margin) {
  atomicAdd(A.tie_cnt + kind, 1ull);
  // 64-bit event counter: it cannot wrap to a negative slot however many decisions a wide
  // tolerance logs; only the first tie_cap events are stored
  const unsigned long long k = atomicAdd(A.tie_n, 1ull);
  if (k < (unsigned long long)A.tie_cap) {
    int* ev = A.tie_ev + 6 * k;
    ev[0] = t;
    ev[1] = it;
    ev[2] = kind;
    ev[3] = id;
    ev[4] = idx;
    ev[5] = 0;
    A.tie_mg[k] = margin;
  }
}
// around(x, d) near its rounding boundary: x 10^d within tol 10^d of k + 1/2 (per lane; the
// caller ballots).  Returns the signed absolute margin x - (k + 1/2) 10^-d in *m.
__device__ __forceinline__ bool round_near(double x, int d, double tol, double* m) {
  const double f = pow10i(d);
  const double y = x * f;
  const double b = floor(y) + 0.5;
  *m = (y - b) / f;
  return fabs(y - b) <= tol * f;
}
// Every lane flagged in `near` logs its round tie (one event per lane; ties are rare).
__device__ __forceinline__ void round_ties(const DevArgs& A, int t, int it, int kind, int id, int idx0, double x,
                                           bool valid) {
  double m;
  const bool nr = valid && round_near(x, A.cfg.round_decimals, A.tie_tol, &m);
  if (__builtin_expect(wany(nr), 0))
    if (nr) tie_record(A, t, it, kind, id, idx0 + lid(), m);
}
// The collision test any_k(d_k^2 < thr) == (min_k d_k^2 < thr): a tie when min_k d_k^2 lies within
// tol thr of thr.  d2 per time lane (valid lanes only); decided by two ballots, the minimum (a wave
// reduction) only in the cold branch.
__device__ __forceinline__ void collide_tie(const DevArgs& A, int t, int it, int e, double d2, bool valid, double thr) {
  const double tol = A.tie_tol;
  const bool lo = valid && d2 < thr * (1.0 - tol);
  const bool near = valid && d2 <= thr * (1.0 + tol);
  if (__builtin_expect(!wany(lo) && wany(near), 0)) {
    const double mn = wmin(valid ? d2 : INFINITY);
    const unsigned long long at = __ballot(valid && d2 == mn);
    if (lid() == 0) tie_record(A, t, it, PIADMM_TIE_COLLIDE, e, (int)__builtin_ctzll(at), (mn - thr) / thr);
  }
}
// A scalar threshold test v <= thr (the stop test) or v > thr (the distance check) taken within
// tol |thr| of thr: logged by the calling lane.
__device__ __forceinline__ void scalar_tie(const DevArgs& A, int t, int it, int kind, int id, int idx, double v,
                                           double thr) {
  if (__builtin_expect(fabs(v - thr) <= A.tie_tol * fabs(thr), 0)) tie_record(A, t, it, kind, id, idx, (v - thr) / thr);
}

#else
__device__ __forceinline__ void tie_record(const DevArgs&, int, int, int, int, int, double) {}
__device__ __forceinline__ bool round_near(double, int, double, double*) { return false; }
__device__ __forceinline__ void round_ties(const DevArgs&, int, int, int, int, int, double, bool) {}
__device__ __forceinline__ void collide_tie(const DevArgs&, int, int, int, double, bool, double) {}
__device__ __forceinline__ void scalar_tie(const DevArgs&, int, int, int, int, int, double, double) {}
#endif

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
__device__ __forceinline__ void gj_invert(double* m_, int n, int ld) {
  ldsd* m = lds_ptr(m_);            // every caller passes the wave's LDS scratch
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


}  // namespace pd
