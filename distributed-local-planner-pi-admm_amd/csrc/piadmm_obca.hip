// piadmm_obca.hip -- OBCA local subproblem: batched SQP, one wavefront per local NLP (gfx950).
//
// The NLP is OBCAOptimizer's vehicle-side problem as written
// (Distributed_planner/decentralized/optimizer.py:61-168): kinematic-bicycle multiple shooting
// over N_horz = 8 (:75-100), OBCA dual-distance constraints (5a)/(5b) against the other
// vehicle's exchanged halfspaces (:105-124), ||A' Lambda||^2 <= 1 (:126-129), bounds (:131-148),
// objective (:150-168).  The reference hands it to IPOPT (:170-180); this kernel runs an SQP:
//   * exact Lagrangian Hessian (dynamics curvature weighted by the shooting multipliers pi,
//     (5a)/(5b) curvature weighted by their multipliers);
//   * the dynamics condensed (dX_t = T_t dU + s_t) and (5b) eliminated on its null space
//     (dLam_t = -P m_theta dtheta_t + P r_t + N zeta_t, M P = I, M N = 0), leaving a dense
//     28-variable QP in (dU, zeta) with 175 inequality rows;
//   * Hessian modification: sigma * sum a a' over the rows active in the previous QP, then
//     tau diag(|H_ii|), until the Cholesky factorisation succeeds;
//   * the QP by the Goldfarb-Idnani dual active set method (J = L^-T Q, R factor, Givens
//     updates), most violated row first;
//   * l1-merit Armijo backtracking; multipliers blended by the step length.
// oracle/obca_oracle.py (solve_local, gi_qp) is the same algorithm statement by statement;
// tests/test_gpu_obca.py holds the two to each other and certifies the answers as KKT points.
//
// Layout: one workgroup = one wavefront (64 lanes) = one problem; the SQP state (~39 KB)
// lives in LDS; lanes split stage-wise work (7 stages) and matrix work (28 x 28) among them.
// HBM traffic per problem: 296 doubles in, 224 doubles + 3 ints out -- the kernel is latency
// bound (barrier chains of the factorisations and the active-set updates), not HBM bound.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "piadmm.h"

namespace obca {

constexpr int NH = 8, NX = 5, NU = 2, NL = 4, NT = 7;
constexpr int NUV = NU * NT;          // 14
constexpr int NZ = NUV + 2 * NT;      // 28
constexpr int ROWS_T = 21;            // per stage: state lo/hi x5, (5a) lo/hi, norm, Lambda lo/hi x4
constexpr int NROW = ROWS_T * NT + 2 * NUV;   // 175
constexpr int REC = PIADMM_OBCA_REC, OUT = PIADMM_OBCA_OUT;
constexpr int MAXACT = NZ;
constexpr int NZP = NZ + 1;         // padded LDS row stride of the 28 x 28 matrices (odd: no bank conflicts
                                     // when each lane walks its own row)

// VehicleConfig (veh_config.py:7-27), OBCAOptimizer (optimizer.py:10-37)
constexpr double LENGTH = 3.5, WIDTH = 2.0, LF = 1.5, LR = 1.0;
constexpr double MAX_STEER = 0.6, MAX_V = 20.0, MAX_ACC = 5.0, MAX_STEER_RATE = 20.0;
constexpr double DT = 0.1, AVG_DELAY = 0.05, VAR_DELAY = 0.025;
constexpr double LAM_MAX = 100000.0, GA_MAX = 1000.0;
constexpr double KB = LR / (LR + LF);
constexpr double TWO_PI = 6.283185307179586;

struct Ws;
struct Ws {
  // problem
  double init[NX], ref[NH][NX], w[NT][2], c[NT], lb[NT][9], zb[NT][9];
  double rho, min_dis, max_x, max_y, rr, qq, sig_delay;
  int prob, max_iter;
  // iterate, trial point, multipliers (current / QP)
  double X[NH][NX], U[NT][NU], L[NT][NL];
  double Xn[NH][NX], Un[NT][NU], Ln[NT][NL];
  double ya[NT], yb[NT][2], yn[NT], yx[NT][NX], pi[NT][NX], yu[NUV], yl[NT][NL];
  double nya[NT], nyb[NT][2], nyn[NT], nyx[NT][NX], npi[NT][NX], nyu[NUV], nyl[NT][NL];
  // linearisation (the blocks read in the condensing / assembly and the multiplier recovery
  // only live in HBM: WsG)
  double ga_v[NT], gb_v[NT][2], gn_v[NT], gn_g[NT][NL];
  // [dX_t; dLam_t] = K_t z + k0_t with z = (dU, zeta) and K_t = [[T_t, 0], [-pmv_t (x) T_t[3], N_t]]
  // (N_t = the null space of dm/dLam at zeta block t): K is never stored
  double T[NT][NX][NUV];      // dX_t = T_t dU + s_t  (stage t = index + 1)
  double pmv[NT][NL];         // P m_theta
  double k0[NT][9];
  double Pm[NT][NL][2];
  double gq[NZ];
  double Hm[NZ][NZP];         // modified Hessian, then its Cholesky factor; warm-solve scratch
  double J[NZ][NZP];          // the condensed Hessian Hq until the QP, then J = L^-T
  double R[NZ][NZP];          // W_t G_t during the assembly, Ga during the modification, then R
  double garow[NT][NZ], gnrow[NT][NZ];
  double din[NROW], uin[NROW];
  double x[NZ], d[NZ], npv[NZ], u[MAXACT + 1], dd[NZ];
  double dX[NH][NX], dU[NT][NU], dL[NT][NL];
  int act[MAXACT + 1], pact[NROW];
  int nact, npact;
  int flag;
};

// The linearisation blocks of one problem, in HBM (L2 / L1-resident): read by the condensing, the
// Hessian assembly and the multiplier recovery of each SQP iteration, never inside the QP's
// active-set loop.  Off the LDS workspace they take it from ~48 KB to ~39 KB per problem, so four
// problems (one wave each) share a CU's 160 KB -- one per SIMD -- instead of three.
struct WsG {
  double A[NT][NX][NX], F[NT][NX], Wd[NT][NX][NX];
  double Wxx[NH][NX][NX], Wxl[NH][NX][NL], Wll[NH][NL][NL];
  double gX[NH][NX], gL[NT][NL];
  double ga_g[NT][9], gb_J[NT][2][9];
  double sv[NH][NX];
};

static_assert(sizeof(Ws) <= 160 * 1024 / 4, "OBCA workspace: four problems per CU");

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
// min value, lowest index on ties (idx < 0 = none)
__device__ __forceinline__ void wargmin(double& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double v2 = __shfl_xor(v, o, 64);
    int i2 = __shfl_xor(i, o, 64);
    bool take = (i2 >= 0) && (i < 0 || v2 < v || (v2 == v && i2 < i));
    if (take) { v = v2; i = i2; }
  }
}

#define SYNC() __syncthreads()

// diagnostic build (-DPIADMM_STAMPS, libpiadmm_stamps.so): per-problem cycle sums of the SQP phases
// and event counts, lane 0's clock; never the measured library
constexpr int NSTAMP = 16;
enum { ST_LIN, ST_COND, ST_HESS, ST_ROWS, ST_MOD, ST_GI, ST_REC, ST_LS, ST_INIT, ST_OUT,
       ST_N_CHOL, ST_N_ADD, ST_N_DROP, ST_N_TRIAL, ST_N_SQP, ST_TOTAL };
#ifdef PIADMM_STAMPS
#define OST_DECL unsigned long long st_acc[NSTAMP] = {}; unsigned long long st_last = clock64(), st_t0 = st_last;
#define OST(slot) do { if (threadIdx.x == 0) { unsigned long long _n = clock64(); st_acc[slot] += _n - st_last; st_last = _n; } } while (0)
#define OCNT(slot, v) do { if (threadIdx.x == 0) st_acc[slot] += (v); } while (0)
#else
#define OST_DECL
#define OST(slot) do { } while (0)
#define OCNT(slot, v) do { } while (0)
#endif

// ---------------------------------------------------------------------------------------------
// geometry and dynamics (util.py:12-101, optimizer.py:75-100); same closed forms as the oracle
// ---------------------------------------------------------------------------------------------
struct Geo {
  double e[2], n[2], m[2], mt[2], mL[2][4], mtL[2][4], d[2], dv[2], dvv[2], dt[2], dtt[2], dvt[2], q[2];
};

__device__ void geo(const double* Xt, const double* Lt, int prob, double sigd, Geo& G) {
  double v = Xt[2], th = Xt[3];
  double c = cos(th), s = sin(th);
  G.e[0] = c; G.e[1] = s; G.n[0] = -s; G.n[1] = c;
  double sg = prob ? 1.0 : -1.0;
  double a1 = Lt[0] - Lt[2], a2 = sg * (Lt[1] - Lt[3]);
  for (int i = 0; i < 2; ++i) {
    G.m[i] = a1 * G.e[i] + a2 * G.n[i];
    G.mt[i] = a1 * G.n[i] - a2 * G.e[i];
    G.mL[i][0] = G.e[i]; G.mL[i][1] = sg * G.n[i]; G.mL[i][2] = -G.e[i]; G.mL[i][3] = -sg * G.n[i];
    G.mtL[i][0] = G.n[i]; G.mtL[i][1] = -sg * G.e[i]; G.mtL[i][2] = -G.n[i]; G.mtL[i][3] = sg * G.e[i];
  }
  if (prob) {
    double k = sigd * VAR_DELAY * VAR_DELAY, da = AVG_DELAY;
    G.d[0] = da * v * c + k * v * v * c * c;           G.d[1] = da * v * s + k * v * v * s * s;
    G.dv[0] = da * c + 2 * k * v * c * c;              G.dv[1] = da * s + 2 * k * v * s * s;
    G.dvv[0] = 2 * k * c * c;                          G.dvv[1] = 2 * k * s * s;
    G.dt[0] = -da * v * s - 2 * k * v * v * c * s;     G.dt[1] = da * v * c + 2 * k * v * v * s * c;
    G.dtt[0] = -da * v * c - 2 * k * v * v * (c * c - s * s);
    G.dtt[1] = -da * v * s + 2 * k * v * v * (c * c - s * s);
    G.dvt[0] = -da * s - 4 * k * v * c * s;            G.dvt[1] = da * c + 4 * k * v * s * c;
  } else {
    for (int i = 0; i < 2; ++i) G.d[i] = G.dv[i] = G.dvv[i] = G.dt[i] = G.dtt[i] = G.dvt[i] = 0.0;
  }
  G.q[0] = Xt[0] + G.d[0];
  G.q[1] = Xt[1] + G.d[1];
}

__device__ __forceinline__ double dot2(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1]; }

// (5a) value and gradient (9); optionally its Hessian (9 x 9, full)
__device__ double ga_val_grad(const Geo& G, const double* Lt, double ct, double* g) {
  const double B0[4] = {LENGTH / 2, WIDTH / 2, LENGTH / 2, WIDTH / 2};
  double val = -(B0[0] * Lt[0] + B0[1] * Lt[1] + B0[2] * Lt[2] + B0[3] * Lt[3]) - dot2(G.q, G.m) - ct;
  if (g) {
    g[0] = -G.m[0]; g[1] = -G.m[1];
    g[2] = -dot2(G.dv, G.m);
    g[3] = -dot2(G.dt, G.m) - dot2(G.q, G.mt);
    g[4] = 0.0;
    for (int j = 0; j < 4; ++j) g[5 + j] = -B0[j] - (G.q[0] * G.mL[0][j] + G.q[1] * G.mL[1][j]);
  }
  return val;
}

__device__ void ga_hess(const Geo& G, double H[9][9]) {
  for (int i = 0; i < 9; ++i)
    for (int j = 0; j < 9; ++j) H[i][j] = 0.0;
  H[0][3] = H[3][0] = -G.mt[0];
  H[1][3] = H[3][1] = -G.mt[1];
  for (int j = 0; j < 4; ++j) {
    H[0][5 + j] = H[5 + j][0] = -G.mL[0][j];
    H[1][5 + j] = H[5 + j][1] = -G.mL[1][j];
    H[2][5 + j] = H[5 + j][2] = -(G.dv[0] * G.mL[0][j] + G.dv[1] * G.mL[1][j]);
    H[3][5 + j] = H[5 + j][3] = -(G.dt[0] * G.mL[0][j] + G.dt[1] * G.mL[1][j])
                                - (G.q[0] * G.mtL[0][j] + G.q[1] * G.mtL[1][j]);
  }
  H[2][2] = -dot2(G.dvv, G.m);
  H[2][3] = H[3][2] = -dot2(G.dvt, G.m) - dot2(G.dv, G.mt);
  // m_tt = -m
  H[3][3] = -dot2(G.dtt, G.m) - 2 * dot2(G.dt, G.mt) + dot2(G.q, G.m);
}

struct Dyn {
  double F[5], A[5][5], Hf[3][3][3];   // Hessians of f0, f1, f3 in (v, theta, steer)
};

__device__ void dyn_eval(const double* Xk, const double* Uk, Dyn& D) {
  double v = Xk[2], th = Xk[3], st = Xk[4];
  double tn = tan(st);
  double beta = atan(KB * tn);
  double sec2 = 1.0 + tn * tn;
  double den = 1.0 + KB * KB * tn * tn;
  double bp = KB * sec2 / den;
  double bpp = 2.0 * KB * tn * sec2 * (1.0 - KB * KB) / (den * den);
  double ph = th + beta;
  double cp = cos(ph), sp = sin(ph), cb = cos(beta), sb = sin(beta);
  double f[5] = {v * cp, v * sp, Uk[0], v / LR * sb, Uk[1]};
  for (int i = 0; i < 5; ++i) D.F[i] = Xk[i] + DT * f[i];
  double Jx[5][5] = {};
  Jx[0][2] = cp; Jx[0][3] = -v * sp; Jx[0][4] = -v * sp * bp;
  Jx[1][2] = sp; Jx[1][3] = v * cp;  Jx[1][4] = v * cp * bp;
  Jx[3][2] = sb / LR; Jx[3][4] = v * cb * bp / LR;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) D.A[i][j] = (i == j ? 1.0 : 0.0) + DT * Jx[i][j];
  // index 0 = v, 1 = theta, 2 = steer
  double (*H0)[3] = D.Hf[0];
  double (*H1)[3] = D.Hf[1];
  double (*H3)[3] = D.Hf[2];
  H0[0][0] = 0.0; H0[0][1] = H0[1][0] = -sp; H0[0][2] = H0[2][0] = -sp * bp;
  H0[1][1] = -v * cp; H0[1][2] = H0[2][1] = -v * cp * bp; H0[2][2] = -v * cp * bp * bp - v * sp * bpp;
  H1[0][0] = 0.0; H1[0][1] = H1[1][0] = cp; H1[0][2] = H1[2][0] = cp * bp;
  H1[1][1] = -v * sp; H1[1][2] = H1[2][1] = -v * sp * bp; H1[2][2] = -v * sp * bp * bp + v * cp * bpp;
  H3[0][0] = 0.0; H3[0][1] = H3[1][0] = 0.0; H3[0][2] = H3[2][0] = cb * bp / LR;
  H3[1][1] = 0.0; H3[1][2] = H3[2][1] = 0.0; H3[2][2] = v * (-sb * bp * bp + cb * bpp) / LR;
}

// ---------------------------------------------------------------------------------------------
// cost and l1 violation at (X, U, L) (oracle _cost / _viol), lane-parallel + wave sums
// ---------------------------------------------------------------------------------------------
__device__ void cost_viol(Ws& S, const double (*X)[NX], const double (*U)[NU], const double (*L)[NL],
                          double& cost, double& viol) {
  int lane = threadIdx.x;
  double f = 0.0, v = 0.0;
  if (lane < NT) {
    int t = lane + 1;
    const double* Xt = X[t];
    const double* Lt = L[t - 1];
    double s9[9];
    for (int i = 0; i < 5; ++i) s9[i] = Xt[i];
    for (int i = 0; i < 4; ++i) s9[5 + i] = Lt[i];
    double uu = U[t - 1][0] * U[t - 1][0] + U[t - 1][1] * U[t - 1][1];
    double ee = 0.0, lbs = 0.0, zz = 0.0;
    for (int i = 0; i < 5; ++i) { double e = Xt[i] - S.ref[t][i]; ee += e * e; }
    for (int i = 0; i < 9; ++i) { lbs += S.lb[t - 1][i] * s9[i]; double z = s9[i] - S.zb[t - 1][i]; zz += z * z; }
    f = S.rr * uu + S.qq * ee + lbs + 0.5 * S.rho * zz;
    Geo G;
    geo(Xt, Lt, S.prob, S.sig_delay, G);
    double ga = ga_val_grad(G, Lt, S.c[t - 1], nullptr);
    v += fmax(0.0, S.min_dis - ga) + fmax(0.0, ga - GA_MAX);
    v += fabs(G.m[0] + S.w[t - 1][0]) + fabs(G.m[1] + S.w[t - 1][1]);
    double a1 = Lt[0] - Lt[2], a2 = Lt[1] - Lt[3];
    v += fmax(0.0, a1 * a1 + a2 * a2 - 1.0);
    const double lo[5] = {0.0, -S.max_y, -MAX_V, -TWO_PI, -MAX_STEER};
    const double hi[5] = {S.max_x, S.max_y, MAX_V, TWO_PI, MAX_STEER};
    for (int j = 0; j < 5; ++j) v += fmax(0.0, lo[j] - Xt[j]) + fmax(0.0, Xt[j] - hi[j]);
  } else if (lane >= 8 && lane < 8 + NT) {
    int k = lane - 8;
    Dyn D;
    dyn_eval(X[k], U[k], D);
    for (int i = 0; i < 5; ++i) v += fabs(X[k + 1][i] - D.F[i]);
  } else if (lane == 16) {
    for (int i = 0; i < 5; ++i) v += fabs(X[0][i] - S.init[i]);
  }
  cost = wsum(f);
  viol = wsum(v);
}

// ---------------------------------------------------------------------------------------------
// dense Cholesky (lower, in place) of the leading n x n block of M, lane i owning row i: per
// column a pivot read, the column scaled by its owners, then each owner updates its own row
// (the same operation order per entry as the right-looking form); false if a pivot is <= thr^2
// (thr = 0: not positive).
__device__ bool chol_n(double (*M)[NZP], int n, double thr) {
  int lane = threadIdx.x;
  for (int j = 0; j < n; ++j) {
    SYNC();
    double piv = M[j][j];
    if (!(piv > 0.0)) { SYNC(); return false; }
    double l = sqrt(piv);
    if (!(l > thr)) { SYNC(); return false; }
    double lij = 0.0;
    if (lane > j && lane < n) { lij = M[lane][j] / l; M[lane][j] = lij; }
    if (lane == j) M[j][j] = l;
    SYNC();
    if (lane > j && lane < n)
      for (int k = j + 1; k <= lane; ++k) M[lane][k] -= lij * M[k][j];
  }
  SYNC();
  return true;
}
__device__ __forceinline__ bool chol(Ws& S) { return chol_n(S.Hm, NZ, 0.0); }

// row c of the constraint matrix (C z >= din) dotted with v (28)
__device__ double row_dot(const Ws& S, int c, const double* v) {
  if (c >= ROWS_T * NT) {
    int j = (c - ROWS_T * NT) >> 1;
    return (c & 1) ? -v[j] : v[j];
  }
  int ti = c / ROWS_T, r = c % ROWS_T;
  if (r < 10) {                       // state rows: T_t only
    const double* a = S.T[ti][r >> 1];
    double s = 0.0;
    for (int k = 0; k < NUV; ++k) s += a[k] * v[k];
    return (r & 1) ? -s : s;
  }
  if (r >= 13) {                      // Lambda rows: -pmv T_t[3] dU + N zeta_t
    int q = r - 13, j = q >> 1;
    const double* a = S.T[ti][3];
    double s = 0.0;
    for (int k = 0; k < NUV; ++k) s += a[k] * v[k];
    s = -S.pmv[ti][j] * s + v[NUV + 2 * ti + (j & 1)];
    return (q & 1) ? -s : s;
  }
  const double* a = (r == 12) ? S.gnrow[ti] : S.garow[ti];
  double s = 0.0;
  for (int k = 0; k < NZ; ++k) s += a[k] * v[k];
  return (r == 10) ? s : -s;
}
__device__ double row_elem(const Ws& S, int c, int k) {
  if (c >= ROWS_T * NT) {
    int j = (c - ROWS_T * NT) >> 1;
    return (k == j) ? ((c & 1) ? -1.0 : 1.0) : 0.0;
  }
  int ti = c / ROWS_T, r = c % ROWS_T;
  if (r < 10) return (k < NUV) ? ((r & 1) ? -1.0 : 1.0) * S.T[ti][r >> 1][k] : 0.0;
  if (r == 10) return S.garow[ti][k];
  if (r == 11) return -S.garow[ti][k];
  if (r == 12) return -S.gnrow[ti][k];
  int q = r - 13, j = q >> 1;
  double e = (k < NUV) ? -S.pmv[ti][j] * S.T[ti][3][k] : ((k == NUV + 2 * ti + (j & 1)) ? 1.0 : 0.0);
  return (q & 1) ? -e : e;
}

// the dU part of K_t, row i (i < 9), column a < NUV
__device__ __forceinline__ double gval(const Ws& S, int ti, int i, int a) {
  return (i < 5) ? S.T[ti][i][a] : -S.pmv[ti][i - 5] * S.T[ti][3][a];
}
__device__ __forceinline__ double wval(const WsG& Q, int t, int i, int j) {
  return (i < 5) ? (j < 5 ? Q.Wxx[t][i][j] : Q.Wxl[t][i][j - 5]) : (j < 5 ? Q.Wxl[t][j][i - 5] : Q.Wll[t][i - 5][j - 5]);
}

// ---------------------------------------------------------------------------------------------
// Goldfarb-Idnani on min 1/2 z'Hz + gq'z, C z >= din (no equalities); H = L L' in S.Hm.
// Returns 0 ok, 2 infeasible, 1 step limit; S.x = solution, S.uin = multipliers (dense).
// ---------------------------------------------------------------------------------------------
// Lane ownership inside the active-set updates: lane i owns row i of J (every Givens rotation of a
// J column pair is row-local), lane c owns column c of R during a drop's rotations; rotation
// parameters are uniform (computed by every lane from LDS / a shuffle), so the rotation chains run
// without barriers.
__device__ void gi_drop(Ws& S, int k) {
  int lane = threadIdx.x;
  SYNC();
  int q = S.nact;
  // remove column k of R (row-owned shift)
  if (lane < NZ) {
    for (int j = k; j < q - 1; ++j) S.R[lane][j] = S.R[lane][j + 1];
    S.R[lane][q - 1] = 0.0;
  }
  SYNC();
  for (int j = k; j < q - 1; ++j) {
    // column j is lane j's: its (R[j][j], R[j+1][j]) after the previous rotations
    double aj = (lane < NZ) ? S.R[j][lane] : 0.0;
    double bj = (lane < NZ) ? S.R[j + 1][lane] : 0.0;
    double a = __shfl(aj, j, 64), b = __shfl(bj, j, 64);
    double h = hypot(a, b);
    if (h != 0.0) {
      double cs = a / h, sn = b / h;
      if (lane >= j && lane < q - 1) {
        S.R[j][lane] = cs * aj + sn * bj;
        S.R[j + 1][lane] = -sn * aj + cs * bj;
      }
      if (lane < NZ) {
        double Jj = S.J[lane][j], Jj1 = S.J[lane][j + 1];
        S.J[lane][j] = cs * Jj + sn * Jj1;
        S.J[lane][j + 1] = -sn * Jj + cs * Jj1;
      }
    }
  }
  SYNC();
  if (lane == 0) {
    for (int j = k; j < q - 1; ++j) { S.act[j] = S.act[j + 1]; S.u[j] = S.u[j + 1]; }
    S.nact = q - 1;
  }
  SYNC();
}

// returns 1 added, 0 infeasible, -1 step limit
__device__ int gi_add(Ws& S, int p, int& steps) {
  int lane = threadIdx.x;
  double up = 0.0;
  const double bp = S.din[p];
  SYNC();
  if (lane < NZ) S.npv[lane] = row_elem(S, p, lane);
  SYNC();
  const double npl = (lane < NZ) ? S.npv[lane] : 0.0;
  while (true) {
    if (++steps > 500) return -1;
    const int q = S.nact;
    // d = J' n_p (lane j)
    double dj = 0.0;
    if (lane < NZ)
      for (int i = 0; i < NZ; ++i) dj += S.J[i][lane] * S.npv[i];
    if (lane < NZ) S.d[lane] = dj;
    SYNC();
    // z = J[:, q:] d[q:] (lane i)
    double zi = 0.0;
    if (lane < NZ)
      for (int j = q; j < NZ; ++j) zi += S.J[lane][j] * S.d[j];
    // r = R^-1 d[:q]: back substitution on the lanes' registers (lane k ends with r_k)
    double ddk = (lane < q) ? dj : 0.0, rk = 0.0;
    for (int j = q - 1; j >= 0; --j) {
      double rj = __shfl(ddk, j, 64) / S.R[j][j];
      if (lane == j) rk = rj;
      if (lane < j) ddk -= S.R[lane][j] * rj;
    }
    // partial step t1 over active rows with r_k > 1e-13 max(1, max|r|)
    const double rmax = fmax(1.0, wmax(lane < q ? fabs(rk) : 0.0));
    double t1v = INFINITY;
    int l = -1;
    if (lane < q && rk > 1e-13 * rmax) { t1v = S.u[lane] / rk; l = lane; }
    wargmin(t1v, l);
    const double t1 = (l >= 0) ? t1v : INFINITY;
    // full step t2
    const double xl = (lane < NZ) ? S.x[lane] : 0.0;
    const double zn = wsum(zi * npl);
    const double dd2 = wsum(dj * dj);
    const double sx = wsum(npl * xl) - bp;
    const double t2 = (zn > 1e-12 * dd2) ? -sx / zn : INFINITY;
    const double t = fmin(t1, t2);
    if (t == INFINITY) return 0;
    if (t2 == INFINITY) {
      if (lane < q) S.u[lane] -= t * rk;
      up += t;
      gi_drop(S, l);
      continue;
    }
    if (lane < NZ) S.x[lane] = xl + t * zi;
    if (lane < q) S.u[lane] -= t * rk;
    up += t;
    if (t == t2) {
      // one Householder reflection of J[:, q:] zeroing d[q+1..] (uniform v, each lane its own row)
      double alpha = S.d[q];
      if (q < NZ - 1) {
        double ss = 0.0;
        for (int j = q + 1; j < NZ; ++j) ss += S.d[j] * S.d[j];
        if (ss > 0.0) {
          const double a0 = S.d[q];
          const double sig = sqrt(a0 * a0 + ss);
          alpha = (a0 > 0.0) ? -sig : sig;
          const double v0 = a0 - alpha;
          const double beta = 1.0 / (sig * (sig + fabs(a0)));     // 2 / v'v
          if (lane < NZ) {
            double sv = S.J[lane][q] * v0;
            for (int j = q + 1; j < NZ; ++j) sv += S.J[lane][j] * S.d[j];
            sv *= beta;
            S.J[lane][q] -= sv * v0;
            for (int j = q + 1; j < NZ; ++j) S.J[lane][j] -= sv * S.d[j];
          }
        }
      }
      if (lane < q) S.R[lane][q] = S.d[lane];
      if (lane == q) S.R[q][q] = alpha;
      SYNC();
      if (lane == 0) { S.act[q] = p; S.u[q] = up; S.nact = q + 1; }
      SYNC();
      return 1;
    }
    gi_drop(S, l);
  }
}

// ---------------------------------------------------------------------------------------------
// warm equality solve (oracle warm_eqp): the previous SQP iteration's active rows W as the QP's
// active set.  Y = L^-1 A_W' (= J' A_W'), S = Y'Y, lam = S^-1 (d_W + Y'y0), z = L^-T (Y lam - y0),
// two refinement steps on d_W - A_W z; certified iff lam >= 0 and every row holds -- then z is
// THE minimiser of the strictly convex QP.  Scratch: A_W and then S in Hm (the factor of H is
// no longer needed once J is formed), Y in R (zeroed again before a fallback).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double s_solve(Ws& S, int m, double v) {
  // S.Hm holds Ls (m x m lower); lane k < m carries component k of the right-hand side
  int lane = threadIdx.x;
  for (int j = 0; j < m; ++j) {
    double yj = __shfl(v, j, 64) / S.Hm[j][j];
    if (lane == j) v = yj;
    if (lane > j && lane < m) v -= S.Hm[lane][j] * yj;
  }
  for (int j = m - 1; j >= 0; --j) {
    double xj = __shfl(v, j, 64) / S.Hm[j][j];
    if (lane == j) v = xj;
    if (lane < j) v -= S.Hm[j][lane] * xj;
  }
  return v;
}

__device__ bool warm_eqp(Ws& S) {
  const int lane = threadIdx.x;
  const int m = S.npact;
  for (int e = lane; e < m * NZ; e += 64) S.Hm[e / NZ][e % NZ] = row_elem(S, S.pact[e / NZ], e % NZ);
  SYNC();
  for (int e = lane; e < NZ * m; e += 64) {
    int i = e / m, k = e % m;
    double s = 0.0;
    for (int j = 0; j < NZ; ++j) s += S.J[j][i] * S.Hm[k][j];
    S.R[i][k] = s;
  }
  SYNC();
  for (int e = lane; e < m * m; e += 64) {
    int k = e / m, l = e % m;
    double s = 0.0;
    for (int i = 0; i < NZ; ++i) s += S.R[i][k] * S.R[i][l];
    S.Hm[k][l] = s;
  }
  SYNC();
  const double dmax = wmax(lane < m ? S.Hm[lane][lane] : 0.0);
  if (!chol_n(S.Hm, m, 1e-7 * sqrt(dmax))) return false;
  // lam
  double lam = 0.0;
  if (lane < m) {
    lam = S.din[S.pact[lane]];
    for (int i = 0; i < NZ; ++i) lam += S.R[i][lane] * S.dd[i];
  }
  lam = s_solve(S, m, lam);
  // w = Y lam - y0  (lane i), kept in S.d
  double wi = 0.0;
  for (int k = 0; k < m; ++k) {
    double lk = __shfl(lam, k, 64);
    if (lane < NZ) wi += S.R[lane][k] * lk;
  }
  if (lane < NZ) { wi -= S.dd[lane]; S.d[lane] = wi; }
  for (int rep = 0; rep < 2; ++rep) {
    SYNC();
    if (lane < NZ) {
      double z = 0.0;
      for (int j = 0; j < NZ; ++j) z += S.J[lane][j] * S.d[j];
      S.x[lane] = z;
    }
    SYNC();
    double r = (lane < m) ? S.din[S.pact[lane]] - row_dot(S, S.pact[lane], S.x) : 0.0;
    double dl = s_solve(S, m, r);
    if (lane < m) lam += dl;
    for (int k = 0; k < m; ++k) {
      double dk = __shfl(dl, k, 64);
      if (lane < NZ) wi += S.R[lane][k] * dk;
    }
    SYNC();
    if (lane < NZ) S.d[lane] = wi;
  }
  const double lmax = fmax(1.0, wmax(lane < m ? fabs(lam) : 0.0));
  const int neg = __any(lane < m && lam < -1e-12 * lmax);
  if (neg) { SYNC(); return false; }
  SYNC();
  if (lane < NZ) {
    double z = 0.0;
    for (int j = 0; j < NZ; ++j) z += S.J[lane][j] * S.d[j];
    S.x[lane] = z;
  }
  SYNC();
  int bad = 0;
  for (int c = lane; c < NROW; c += 64) {
    double sc = row_dot(S, c, S.x) - S.din[c];
    bad |= (sc < -1e-11 * (1.0 + fabs(S.din[c])));
  }
  if (__any(bad)) { SYNC(); return false; }
  if (lane < m) { S.act[lane] = S.pact[lane]; S.u[lane] = fmax(lam, 0.0); }
  if (lane == 0) S.nact = m;
  SYNC();
  return true;
}

__device__ int gi_solve(Ws& S, int& steps) {
  int lane = threadIdx.x;
  // J = L^-T: lane j solves L y = e_j, J[:, j]... J = (L^-1)'  =>  J[i][j] = (L^-1)[j][i]
  if (lane < NZ) {
    // column j of L^-1 (forward substitution of L y = e_j) is row j of J; each lane owns its row
    int j = lane;
    double* y = S.J[j];
    for (int i = 0; i < NZ; ++i) {
      if (i < j) { y[i] = 0.0; continue; }
      double s = (i == j) ? 1.0 : 0.0;
      for (int k = j; k < i; ++k) s -= S.Hm[i][k] * y[k];
      y[i] = s / S.Hm[i][i];
    }
  }
  SYNC();
  // x = -J J' g
  if (lane < NZ) {
    double s = 0.0;
    for (int i = 0; i < NZ; ++i) s += S.J[i][lane] * S.gq[i];
    S.dd[lane] = s;
  }
  SYNC();
  if (S.npact > 0 && warm_eqp(S)) {
    steps = 0;
  } else {
  if (lane < NZ) {
    double s = 0.0;
    for (int j = 0; j < NZ; ++j) s += S.J[lane][j] * S.dd[j];
    S.x[lane] = -s;
  }
  for (int e = lane; e < NZ * NZ; e += 64) S.R[e / NZ][e % NZ] = 0.0;
  if (lane == 0) S.nact = 0;
  SYNC();
  while (true) {
    double best = INFINITY;
    int bi = -1;
    for (int c = lane; c < NROW; c += 64) {
      double s = row_dot(S, c, S.x) - S.din[c];
      if (bi < 0 || s < best) { best = s; bi = c; }
    }
    wargmin(best, bi);
    if (!(best < -1e-11 * (1.0 + fabs(S.din[bi])))) break;
    int ok = gi_add(S, bi, steps);
    if (ok < 0) return 1;
    if (ok == 0) return 2;
  }
  }
  SYNC();
  for (int c = lane; c < NROW; c += 64) S.uin[c] = 0.0;
  SYNC();
  if (lane == 0)
    for (int k = 0; k < S.nact; ++k) S.uin[S.act[k]] = S.u[k];
  SYNC();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// the SQP
// ---------------------------------------------------------------------------------------------
// One local NLP (record pb) on this wave; S is the workgroup's LDS state (reinitialised here).
__device__ __forceinline__ void sqp_one(Ws& S, int pb, const double* __restrict__ recs, double* __restrict__ out,
                                        int* __restrict__ ist, unsigned long long* __restrict__ stamps,
                                        WsG* __restrict__ qg) {
  OST_DECL
  const int lane = threadIdx.x;
  WsG& Q = qg[pb];
  const double* rec = recs + (size_t)pb * REC;

  // ---- load the record, derive w_t = A_o' lamb_ij, c_t = b_o' lamb_ij ----
  if (lane < NX) S.init[lane] = rec[lane];
  for (int e = lane; e < NH * NX; e += 64) (&S.ref[0][0])[e] = rec[5 + e];
  for (int e = lane; e < NT * 9; e += 64) {
    (&S.lb[0][0])[e] = rec[157 + e];
    (&S.zb[0][0])[e] = rec[220 + e];
  }
  if (lane < NT) {
    int t = lane;
    const double* Ao = rec + 45 + t * 8;
    const double* bo = rec + 101 + t * 4;
    const double* lij = rec + 129 + t * 4;
    double w0 = 0.0, w1 = 0.0, cc = 0.0;
    for (int i = 0; i < 4; ++i) { w0 += Ao[i * 2 + 0] * lij[i]; w1 += Ao[i * 2 + 1] * lij[i]; cc += bo[i] * lij[i]; }
    S.w[t][0] = w0; S.w[t][1] = w1; S.c[t] = cc;
  }
  if (lane == 0) {
    const double* par = rec + 283;
    S.rho = par[0]; S.min_dis = par[1]; S.max_x = par[2]; S.max_y = par[3];
    S.rr = par[4]; S.qq = par[5]; S.prob = (int)par[6]; S.max_iter = (int)par[7];
    S.sig_delay = sqrt(0.95 / (1.0 - 0.95));
    S.npact = -1;    // "no previous QP"
  }
  SYNC();
  // ---- initial iterate: X = ref, U = 0, Lambda = smallest non-negative (5b) solution at ref ----
  for (int e = lane; e < NH * NX; e += 64) (&S.X[0][0])[e] = (&S.ref[0][0])[e];
  if (lane < NUV) (&S.U[0][0])[lane] = 0.0;
  if (lane < NT) {
    int t = lane + 1;
    double th = S.ref[t][3], c = cos(th), s = sin(th);
    double e0[2] = {c, s}, n0[2] = {-s, c};
    double sg = S.prob ? 1.0 : -1.0;
    double u0 = -S.w[lane][0], u1 = -S.w[lane][1];
    double ce = e0[0] * u0 + e0[1] * u1;            // row 0 = e
    double cn = sg * (n0[0] * u0 + n0[1] * u1);     // row 1 = sg n
    S.L[lane][0] = fmax(ce, 0.0); S.L[lane][2] = fmax(-ce, 0.0);
    S.L[lane][1] = fmax(cn, 0.0); S.L[lane][3] = fmax(-cn, 0.0);
  }
  for (int e = lane; e < NT * NX; e += 64) { (&S.yx[0][0])[e] = 0.0; (&S.pi[0][0])[e] = 0.0; }
  for (int e = lane; e < NT * NL; e += 64) (&S.yl[0][0])[e] = 0.0;
  if (lane < NT) { S.ya[lane] = 0.0; S.yn[lane] = 0.0; S.yb[lane][0] = S.yb[lane][1] = 0.0; }
  if (lane < NUV) S.yu[lane] = 0.0;
  SYNC();

  OST(ST_INIT);
  double mu = 0.0;
  int qp_total = 0;
  int status = PIADMM_OBCA_MAX_ITER;
  int it = 0;
  const int max_iter = S.max_iter;
  for (it = 0; it < max_iter; ++it) {
    // ---- linearise: dynamics per k (lanes 0..6) ----
    if (lane < NT) {
      int k = lane;
      Dyn D;
      dyn_eval(S.X[k], S.U[k], D);
      for (int i = 0; i < 5; ++i) {
        Q.F[k][i] = D.F[i];
        for (int j = 0; j < 5; ++j) { Q.A[k][i][j] = D.A[i][j]; Q.Wd[k][i][j] = 0.0; }
      }
      const int fi[3] = {0, 1, 3};
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
          for (int f = 0; f < 3; ++f) s += S.pi[k][fi[f]] * D.Hf[f][a][b];
          Q.Wd[k][2 + a][2 + b] = DT * s;
        }
    }
    SYNC();
    // ---- stages t = 1..7 (lanes 0..6): cost gradient, (5a)/(5b)/norm, Hessian blocks ----
    if (lane < NT) {
      int t = lane + 1;
      const double* Xt = S.X[t];
      const double* Lt = S.L[t - 1];
      for (int i = 0; i < 5; ++i)
        Q.gX[t][i] = 2 * S.qq * (Xt[i] - S.ref[t][i]) + S.lb[t - 1][i] + S.rho * (Xt[i] - S.zb[t - 1][i]);
      for (int i = 0; i < 4; ++i) Q.gL[t - 1][i] = S.lb[t - 1][5 + i] + S.rho * (Lt[i] - S.zb[t - 1][5 + i]);
      Geo G;
      geo(Xt, Lt, S.prob, S.sig_delay, G);
      double ga[9];
      S.ga_v[t - 1] = ga_val_grad(G, Lt, S.c[t - 1], ga);
      for (int i = 0; i < 9; ++i) Q.ga_g[t - 1][i] = ga[i];
      for (int r = 0; r < 2; ++r) {
        S.gb_v[t - 1][r] = G.m[r] + S.w[t - 1][r];
        for (int i = 0; i < 9; ++i) Q.gb_J[t - 1][r][i] = 0.0;
        Q.gb_J[t - 1][r][3] = G.mt[r];
        for (int j = 0; j < 4; ++j) Q.gb_J[t - 1][r][5 + j] = G.mL[r][j];
      }
      double a1 = Lt[0] - Lt[2], a2 = Lt[1] - Lt[3];
      S.gn_v[t - 1] = a1 * a1 + a2 * a2;
      S.gn_g[t - 1][0] = 2 * a1; S.gn_g[t - 1][1] = 2 * a2; S.gn_g[t - 1][2] = -2 * a1; S.gn_g[t - 1][3] = -2 * a2;
      double H[9][9];
      ga_hess(G, H);
      double ya = S.ya[t - 1], yb0 = S.yb[t - 1][0], yb1 = S.yb[t - 1][1], yn = S.yn[t - 1];
      for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) H[i][j] *= -ya;
      // (5b) Hessians: (theta, theta) = m_tt = -m, (theta, Lam_j) = mtL
      H[3][3] -= yb0 * (-G.m[0]) + yb1 * (-G.m[1]);
      for (int j = 0; j < 4; ++j) {
        double hv = yb0 * G.mtL[0][j] + yb1 * G.mtL[1][j];
        H[3][5 + j] -= hv;
        H[5 + j][3] -= hv;
      }
      const double Hn[4][4] = {{2, 0, -2, 0}, {0, 2, 0, -2}, {-2, 0, 2, 0}, {0, -2, 0, 2}};
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j)
          Q.Wxx[t][i][j] = (t < NH - 1 ? Q.Wd[t][i][j] : 0.0) + (i == j ? 2 * S.qq + S.rho : 0.0) + H[i][j];
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 4; ++j) Q.Wxl[t][i][j] = H[i][5 + j];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Q.Wll[t][i][j] = (i == j ? S.rho : 0.0) + H[5 + i][5 + j] - yn * Hn[i][j];
    }
    OST(ST_LIN);
    // ---- condense: T_t, s_t ----
    if (lane < NX) Q.sv[0][lane] = S.init[lane] - S.X[0][lane];
    SYNC();
    for (int k = 0; k < NT; ++k) {
      // T_{k+1} = A_k T_k + B_k E_k  (T_0 = 0); index k holds T_{k+1}
      for (int e = lane; e < NX * NUV; e += 64) {
        int i = e / NUV, j = e % NUV;
        double s = 0.0;
        if (k > 0)
          for (int m = 0; m < NX; ++m) s += Q.A[k][i][m] * S.T[k - 1][m][j];
        if (j == 2 * k && i == 2) s += DT;
        if (j == 2 * k + 1 && i == 4) s += DT;
        S.T[k][i][j] = s;
      }
      if (lane < NX) {
        double s = 0.0;
        for (int m = 0; m < NX; ++m) s += Q.A[k][lane][m] * Q.sv[k][m];
        Q.sv[k + 1][lane] = s + Q.F[k][lane] - S.X[k + 1][lane];
      }
      SYNC();
    }
    // ---- (5b) elimination: P m_theta and k0 ----
    if (lane < NT) {
      int ti = lane;
      double P[4][2], pm[4], pr[4];
      double mth0 = Q.gb_J[ti][0][3], mth1 = Q.gb_J[ti][1][3];
      double r0 = -S.gb_v[ti][0], r1 = -S.gb_v[ti][1];
      double s3 = Q.sv[ti + 1][3];
      for (int i = 0; i < 4; ++i) {
        P[i][0] = 0.5 * Q.gb_J[ti][0][5 + i];
        P[i][1] = 0.5 * Q.gb_J[ti][1][5 + i];
        S.Pm[ti][i][0] = P[i][0];
        S.Pm[ti][i][1] = P[i][1];
        pm[i] = P[i][0] * mth0 + P[i][1] * mth1;
        pr[i] = P[i][0] * (r0 - mth0 * s3) + P[i][1] * (r1 - mth1 * s3);
      }
      for (int i = 0; i < 5; ++i) S.k0[ti][i] = Q.sv[ti + 1][i];
      for (int i = 0; i < 4; ++i) S.k0[ti][5 + i] = pr[i];
      for (int i = 0; i < 4; ++i) S.pmv[ti][i] = pm[i];
    }
    SYNC();
    OST(ST_COND);
    // ---- condensed Hessian and gradient by blocks: UU += G_t' W_t G_t, U zeta_t += G_t' W_t N,
    //      zeta_t zeta_t += N' W_ll N; gq += K_t' (W_t k0_t + g_t) ----
    for (int e = lane; e < NZ * NZ; e += 64) {
      int a = e / NZ, b = e % NZ;
      S.J[a][b] = (a == b && a < NUV) ? 2 * S.rr : 0.0;
    }
    if (lane < NZ) S.gq[lane] = lane < NUV ? 2 * S.rr * (&S.U[0][0])[lane] : 0.0;
    SYNC();
    for (int ti = 0; ti < NT; ++ti) {
      const int t = ti + 1;
      // R[i][0..13] = (W_t G_t)[i][:], R[i][14 + c] = (W_t N)[i][c]; dd[i] = (W_t k0_t + g_t)[i]
      for (int e = lane; e < 9 * 16; e += 64) {
        int i = e >> 4, a = e & 15;
        double v = 0.0;
        if (a < NUV) {
          for (int j = 0; j < 9; ++j) v += wval(Q, t, i, j) * gval(S, ti, j, a);
        } else {
          int c = a - NUV;
          v = wval(Q, t, i, 5 + c) + wval(Q, t, i, 7 + c);
        }
        S.R[i][a] = v;
      }
      if (lane >= 48 && lane < 57) {
        int i = lane - 48;
        double v = (i < 5) ? Q.gX[t][i] : Q.gL[ti][i - 5];
        for (int j = 0; j < 9; ++j) v += wval(Q, t, i, j) * S.k0[ti][j];
        S.dd[i] = v;
      }
      SYNC();
      for (int e = lane; e < NUV * NUV; e += 64) {
        int a = e / NUV, b = e % NUV;
        double v = 0.0;
        for (int i = 0; i < 9; ++i) v += gval(S, ti, i, a) * S.R[i][b];
        S.J[a][b] += v;
      }
      if (lane < 2 * NUV) {
        int a = lane >> 1, c = lane & 1;
        double v = 0.0;
        for (int i = 0; i < 9; ++i) v += gval(S, ti, i, a) * S.R[i][NUV + c];
        S.J[a][NUV + 2 * ti + c] += v;
        S.J[NUV + 2 * ti + c][a] += v;
      } else if (lane < 2 * NUV + 4) {
        int c1 = (lane - 2 * NUV) >> 1, c2 = (lane - 2 * NUV) & 1;
        S.J[NUV + 2 * ti + c1][NUV + 2 * ti + c2] += S.R[5 + c1][NUV + c2] + S.R[7 + c1][NUV + c2];
      }
      if (lane >= 32 && lane < 32 + NUV) {
        int a = lane - 32;
        double v = 0.0;
        for (int i = 0; i < 9; ++i) v += gval(S, ti, i, a) * S.dd[i];
        S.gq[a] += v;
      } else if (lane >= 48 && lane < 50) {
        int c = lane - 48;
        S.gq[NUV + 2 * ti + c] += S.dd[5 + c] + S.dd[7 + c];
      }
      SYNC();
    }
    // symmetrise
    for (int e = lane; e < NZ * NZ; e += 64) {
      int a = e / NZ, b = e % NZ;
      if (a < b) {
        double v = 0.5 * (S.J[a][b] + S.J[b][a]);
        S.J[a][b] = v;
        S.J[b][a] = v;
      }
    }
    OST(ST_HESS);
    // ---- constraint rows ----
    for (int e = lane; e < NT * NZ; e += 64) {
      int ti = e / NZ, a = e % NZ;
      double sa = 0.0, sn = 0.0;
      if (a < NUV) {
        for (int i = 0; i < 9; ++i) sa += Q.ga_g[ti][i] * gval(S, ti, i, a);
        for (int j = 0; j < 4; ++j) sn += S.gn_g[ti][j] * gval(S, ti, 5 + j, a);
      } else if (((a - NUV) >> 1) == ti) {
        int c = (a - NUV) & 1;
        sa = Q.ga_g[ti][5 + c] + Q.ga_g[ti][7 + c];
        sn = S.gn_g[ti][c] + S.gn_g[ti][2 + c];
      }
      S.garow[ti][a] = sa;
      S.gnrow[ti][a] = sn;
    }
    for (int c = lane; c < NROW; c += 64) {
      double dv;
      if (c >= ROWS_T * NT) {
        int j = (c - ROWS_T * NT) >> 1;
        double lo = (j & 1) ? -MAX_STEER_RATE : -MAX_ACC;
        double uj = (&S.U[0][0])[j];
        dv = (c & 1) ? (uj + lo) : (lo - uj);      // lo - u  |  u - hi  (hi = -lo)
      } else {
        int ti = c / ROWS_T, r = c % ROWS_T, t = ti + 1;
        if (r < 10) {
          int j = r >> 1;
          const double lo[5] = {0.0, -S.max_y, -MAX_V, -TWO_PI, -MAX_STEER};
          const double hi[5] = {S.max_x, S.max_y, MAX_V, TWO_PI, MAX_STEER};
          double base = S.X[t][j] + S.k0[ti][j];
          dv = (r & 1) ? base - hi[j] : lo[j] - base;
        } else if (r <= 11) {
          double base = S.ga_v[ti];
          for (int i = 0; i < 9; ++i) base += Q.ga_g[ti][i] * S.k0[ti][i];
          dv = (r == 10) ? S.min_dis - base : base - GA_MAX;
        } else if (r == 12) {
          double base = S.gn_v[ti];
          for (int j = 0; j < 4; ++j) base += S.gn_g[ti][j] * S.k0[ti][5 + j];
          dv = base - 1.0;
        } else {
          int q = r - 13, j = q >> 1;
          double base = S.L[ti][j] + S.k0[ti][5 + j];
          dv = (q & 1) ? base - LAM_MAX : -base;
        }
      }
      S.din[c] = dv;
    }
    SYNC();
    OST(ST_ROWS);
    // ---- Hessian modification ----
    for (int e = lane; e < NZ * NZ; e += 64) S.Hm[e / NZ][e % NZ] = S.J[e / NZ][e % NZ];
    bool pd = chol(S);
    OCNT(ST_N_CHOL, 1);
    if (!pd && S.npact > 0) {
      // sigma/2 sum_k (a_k'z - d_k)^2 over the previous QP's active rows, normalised (zero and
      // stationary on their face: a QP solution keeping them active is unchanged):
      // Ga = sum a a' (in R, free until the QP), gav = sum d a (in npv)
      for (int e = lane; e < NZ * NZ; e += 64) S.R[e / NZ][e % NZ] = 0.0;
      if (lane < NZ) S.npv[lane] = 0.0;
      SYNC();
      for (int k = 0; k < S.npact; ++k) {
        int c = S.pact[k];
        double a = (lane < NZ) ? row_elem(S, c, lane) : 0.0;
        double nn = wsum(a * a);
        double inv = 1.0 / fmax(sqrt(nn), 1e-300);
        if (lane < NZ) { S.dd[lane] = a * inv; S.npv[lane] += (S.din[c] * inv) * (a * inv); }
        SYNC();
        for (int e = lane; e < NZ * NZ; e += 64) {
          int i = e / NZ, j = e % NZ;
          S.R[i][j] += S.dd[i] * S.dd[j];
        }
        SYNC();
      }
      double hm = wmax(lane < NZ ? fabs(S.J[lane][lane]) : 0.0);
      double sig = 1e-4 * hm;
      for (int a = 0; a < 8; ++a) {
        for (int e = lane; e < NZ * NZ; e += 64) S.Hm[e / NZ][e % NZ] = S.J[e / NZ][e % NZ] + sig * S.R[e / NZ][e % NZ];
        pd = chol(S);
        OCNT(ST_N_CHOL, 1);
        if (pd) break;
        sig *= 10.0;
      }
      if (!pd) {
        // H0 = Hq + sig_last Ga (sig was multiplied once more after the last try)
        sig /= 10.0;
        for (int e = lane; e < NZ * NZ; e += 64) S.R[e / NZ][e % NZ] = S.J[e / NZ][e % NZ] + sig * S.R[e / NZ][e % NZ];
      }
      if (lane < NZ) S.gq[lane] -= sig * S.npv[lane];
      SYNC();
    } else if (!pd) {
      for (int e = lane; e < NZ * NZ; e += 64) S.R[e / NZ][e % NZ] = S.J[e / NZ][e % NZ];
      SYNC();
    }
    if (!pd) {
      // H0 in R: H0 + tau diag(max(|H0_ii|, 1e-12)), tau = 1e-6, 1e-5, ...
      double tau = 0.0;
      for (int a = 0; a < 16; ++a) {
        tau = (tau == 0.0) ? 1e-6 : tau * 10.0;
        for (int e = lane; e < NZ * NZ; e += 64) {
          int i = e / NZ, j = e % NZ;
          double h = S.R[i][j];
          S.Hm[i][j] = (i == j) ? h + tau * fmax(fabs(h), 1e-12) : h;
        }
        pd = chol(S);
        OCNT(ST_N_CHOL, 1);
        if (pd) break;
      }
      if (!pd) { status = PIADMM_OBCA_HESSIAN_FAIL; break; }
    }
    OST(ST_MOD);
    // ---- QP ----
    int steps = 0;
    int qst = gi_solve(S, steps);
    qp_total += steps;
    OCNT(ST_N_ADD, S.nact);
    OST(ST_GI);
    OCNT(ST_N_SQP, 1);
    if (qst != 0) { status = (qst == 2) ? PIADMM_OBCA_QP_INFEASIBLE : PIADMM_OBCA_MAX_ITER; break; }
    if (lane == 0) {
      int m = 0;
      for (int c = 0; c < NROW; ++c)
        if (S.uin[c] > 0.0) S.pact[m++] = c;
      S.npact = m;
    }
    // ---- step in the full space ----
    if (lane < NUV) (&S.dU[0][0])[lane] = S.x[lane];
    if (lane < NX) S.dX[0][lane] = Q.sv[0][lane];
    for (int e = lane; e < NT * 9; e += 64) {
      int ti = e / 9, i = e % 9;
      int ir = (i < 5) ? i : 3;
      double s = 0.0;
      for (int a = 0; a < NUV; ++a) s += S.T[ti][ir][a] * S.x[a];
      if (i < 5) S.dX[ti + 1][i] = S.k0[ti][i] + s;
      else S.dL[ti][i - 5] = S.k0[ti][i] - S.pmv[ti][i - 5] * s + S.x[NUV + 2 * ti + ((i - 5) & 1)];
    }
    // ---- QP multipliers -> NLP multipliers ----
    if (lane < NT) {
      int ti = lane;
      const double* ui = S.uin + ti * ROWS_T;
      for (int j = 0; j < NX; ++j) S.nyx[ti][j] = ui[2 * j] - ui[2 * j + 1];
      S.nya[ti] = ui[10] - ui[11];
      S.nyn[ti] = -ui[12];
      for (int j = 0; j < NL; ++j) S.nyl[ti][j] = ui[13 + 2 * j] - ui[14 + 2 * j];
    }
    if (lane < NUV) S.nyu[lane] = S.uin[ROWS_T * NT + 2 * lane] - S.uin[ROWS_T * NT + 2 * lane + 1];
    SYNC();
    if (lane < NT) {
      int ti = lane, t = ti + 1;
      double resL[4];
      for (int i = 0; i < 4; ++i) {
        double s = Q.gL[ti][i];
        for (int j = 0; j < 5; ++j) s += Q.Wxl[t][j][i] * S.dX[t][j];
        for (int j = 0; j < 4; ++j) s += Q.Wll[t][i][j] * S.dL[ti][j];
        s -= S.nya[ti] * Q.ga_g[ti][5 + i] + S.nyn[ti] * S.gn_g[ti][i] + S.nyl[ti][i];
        resL[i] = s;
      }
      for (int r = 0; r < 2; ++r) {
        double s = 0.0;
        for (int i = 0; i < 4; ++i) s += S.Pm[ti][i][r] * resL[i];
        S.nyb[ti][r] = s;
      }
    }
    SYNC();
    // shooting multipliers, backward: pi_{t-1} = q_t + A_t' pi_t
    for (int t = NH - 1; t >= 1; --t) {
      if (lane < NX) {
        int i = lane, ti = t - 1;
        double s = Q.gX[t][i];
        for (int j = 0; j < 5; ++j) s += Q.Wxx[t][i][j] * S.dX[t][j];
        for (int j = 0; j < 4; ++j) s += Q.Wxl[t][i][j] * S.dL[ti][j];
        s -= S.nya[ti] * Q.ga_g[ti][i] + S.nyb[ti][0] * Q.gb_J[ti][0][i] + S.nyb[ti][1] * Q.gb_J[ti][1][i];
        s -= S.nyx[ti][i];
        if (t < NH - 1)
          for (int j = 0; j < 5; ++j) s += Q.A[t][j][i] * S.npi[t][j];
        S.npi[ti][i] = s;
      }
      SYNC();
    }
    OST(ST_REC);
    // ---- convergence test ----
    double f0, viol;
    cost_viol(S, S.X, S.U, S.L, f0, viol);
    double stp = 0.0;
    for (int e = lane; e < NH * NX; e += 64) stp = fmax(stp, fabs((&S.dX[0][0])[e]));
    if (lane < NUV) stp = fmax(stp, fabs((&S.dU[0][0])[lane]));
    if (lane < NT * NL) stp = fmax(stp, fabs((&S.dL[0][0])[lane]));
    stp = wmax(stp);
    if (stp <= 1e-9 && viol <= 1e-9) {
      for (int e = lane; e < NH * NX; e += 64) (&S.X[0][0])[e] += (&S.dX[0][0])[e];
      if (lane < NUV) (&S.U[0][0])[lane] += (&S.dU[0][0])[lane];
      if (lane < NT * NL) (&S.L[0][0])[lane] += (&S.dL[0][0])[lane];
      for (int e = lane; e < NT * NX; e += 64) {
        (&S.yx[0][0])[e] = (&S.nyx[0][0])[e];
        (&S.pi[0][0])[e] = (&S.npi[0][0])[e];
      }
      if (lane < NT * NL) (&S.yl[0][0])[lane] = (&S.nyl[0][0])[lane];
      if (lane < NUV) S.yu[lane] = S.nyu[lane];
      if (lane < NT) { S.ya[lane] = S.nya[lane]; S.yn[lane] = S.nyn[lane]; S.yb[lane][0] = S.nyb[lane][0]; S.yb[lane][1] = S.nyb[lane][1]; }
      SYNC();
      status = PIADMM_OBCA_CONVERGED;
      break;
    }
    // ---- l1 merit line search ----
    double mm = 0.0;
    if (lane < NT) mm = fmax(fmax(fabs(S.nya[lane]), fabs(S.nyn[lane])), fmax(fabs(S.nyb[lane][0]), fabs(S.nyb[lane][1])));
    for (int e = lane; e < NT * NX; e += 64) mm = fmax(mm, fmax(fabs((&S.nyx[0][0])[e]), fabs((&S.npi[0][0])[e])));
    mm = wmax(mm);
    mu = fmax(mu, 1.01 * mm + 1e-6);
    double phi0 = f0 + mu * viol;
    double gd = 0.0;
    for (int e = lane; e < NT * NX; e += 64) gd += (&Q.gX[1][0])[e] * (&S.dX[1][0])[e];
    if (lane < NUV) gd += 2 * S.rr * (&S.U[0][0])[lane] * (&S.dU[0][0])[lane];
    if (lane < NT * NL) gd += (&Q.gL[0][0])[lane] * (&S.dL[0][0])[lane];
    gd = wsum(gd);
    double D = gd - mu * viol;
    double alpha = 1.0;
    bool ok = false;
    for (int a = 0; a <= 30; ++a) {
      for (int e = lane; e < NH * NX; e += 64) (&S.Xn[0][0])[e] = (&S.X[0][0])[e] + alpha * (&S.dX[0][0])[e];
      if (lane < NUV) (&S.Un[0][0])[lane] = (&S.U[0][0])[lane] + alpha * (&S.dU[0][0])[lane];
      if (lane < NT * NL) (&S.Ln[0][0])[lane] = (&S.L[0][0])[lane] + alpha * (&S.dL[0][0])[lane];
      SYNC();
      double fn, vn;
      cost_viol(S, S.Xn, S.Un, S.Ln, fn, vn);
      OCNT(ST_N_TRIAL, 1);
      if (fn + mu * vn <= phi0 + 1e-4 * alpha * D) { ok = true; break; }
      alpha *= 0.5;
      SYNC();
    }
    if (!ok) { status = PIADMM_OBCA_LINESEARCH_FAIL; break; }
    SYNC();
    for (int e = lane; e < NH * NX; e += 64) (&S.X[0][0])[e] = (&S.Xn[0][0])[e];
    if (lane < NUV) (&S.U[0][0])[lane] = (&S.Un[0][0])[lane];
    if (lane < NT * NL) (&S.L[0][0])[lane] = (&S.Ln[0][0])[lane];
    for (int e = lane; e < NT * NX; e += 64) {
      (&S.yx[0][0])[e] += alpha * ((&S.nyx[0][0])[e] - (&S.yx[0][0])[e]);
      (&S.pi[0][0])[e] += alpha * ((&S.npi[0][0])[e] - (&S.pi[0][0])[e]);
    }
    if (lane < NT * NL) (&S.yl[0][0])[lane] += alpha * ((&S.nyl[0][0])[lane] - (&S.yl[0][0])[lane]);
    if (lane < NUV) S.yu[lane] += alpha * (S.nyu[lane] - S.yu[lane]);
    OST(ST_LS);
    if (lane < NT) {
      S.ya[lane] += alpha * (S.nya[lane] - S.ya[lane]);
      S.yn[lane] += alpha * (S.nyn[lane] - S.yn[lane]);
      S.yb[lane][0] += alpha * (S.nyb[lane][0] - S.yb[lane][0]);
      S.yb[lane][1] += alpha * (S.nyb[lane][1] - S.yb[lane][1]);
    }
    SYNC();
  }
  SYNC();
  double fc, vc;
  cost_viol(S, S.X, S.U, S.L, fc, vc);
  // ---- write out ----
  double* o = out + (size_t)pb * OUT;
  for (int e = lane; e < NH * NX; e += 64) o[e] = (&S.X[0][0])[e];
  if (lane < NUV) o[40 + lane] = (&S.U[0][0])[lane];
  if (lane < NT * NL) o[54 + lane] = (&S.L[0][0])[lane];
  if (lane < NT) { o[82 + lane] = S.ya[lane]; o[89 + 2 * lane] = S.yb[lane][0]; o[90 + 2 * lane] = S.yb[lane][1]; o[103 + lane] = S.yn[lane]; }
  for (int e = lane; e < NT * NX; e += 64) { o[110 + e] = (&S.yx[0][0])[e]; o[145 + e] = (&S.pi[0][0])[e]; }
  if (lane < NUV) o[180 + lane] = S.yu[lane];
  if (lane < NT * NL) o[194 + lane] = (&S.yl[0][0])[lane];
  if (lane == 0) {
    o[222] = fc;
    o[223] = 0.0;
    ist[(size_t)pb * 3 + 0] = status;
    ist[(size_t)pb * 3 + 1] = (it < max_iter) ? it + 1 : max_iter;
    ist[(size_t)pb * 3 + 2] = qp_total;
  }
#ifdef PIADMM_STAMPS
  OST(ST_OUT);
  if (lane == 0 && stamps) {
    st_acc[ST_N_DROP] = (unsigned long long)qp_total;
    st_acc[ST_TOTAL] = clock64() - st_t0;
    for (int k = 0; k < NSTAMP; ++k) stamps[(size_t)pb * NSTAMP + k] = st_acc[k];
  }
#endif
}

// Workgroup b (one wave) solves problem order[b]: the workgroup dispatcher starts workgroups in
// index order as the CUs' slots free up, so `order` -- the host's longest-first schedule from the
// last solve's work (piadmm_obca_run) -- makes the launch a longest-processing-time-first list
// schedule: the long problems start while the CUs are full and the short ones fill in behind
// them, instead of a long problem placed last setting the launch's end.
__global__ void __launch_bounds__(64) k_obca_sqp(const double* __restrict__ recs, int n,
                                                 double* __restrict__ out, int* __restrict__ ist,
                                                 unsigned long long* __restrict__ stamps, WsG* __restrict__ qg,
                                                 const int* __restrict__ order) {
  __shared__ Ws S;
  if ((int)blockIdx.x >= n) return;
  const int pb = order[blockIdx.x];
  sqp_one(S, pb, recs, out, ist, stamps, qg);
}

}  // namespace obca

// ---------------------------------------------------------------------------------------------
// C-ABI (include/piadmm.h)
// ---------------------------------------------------------------------------------------------
struct piadmm_obca_s {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double* d_rec = nullptr;
  double* d_out = nullptr;
  int* d_ist = nullptr;
  obca::WsG* d_qg = nullptr;   // per-problem linearisation blocks (HBM)
  unsigned long long* d_stamps = nullptr;
  int* d_order = nullptr;       // the launch's problem order (longest first; cap ints)
  std::vector<int> order;       // host copy of the order
  std::vector<int> cost;        // the last solve's status / SQP iterations / QP steps per problem
  int cost_n = 0;               // batch size of the last solve (0: none yet)
  int cap = 0, n = 0;
  std::string err;
};

namespace {
int fail(piadmm_obca_t h, int code, const std::string& msg) {
  if (h) h->err = msg;
  return code;
}
#define OHIP(h, call)                                                                 \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess) return fail(h, PIADMM_E_HIP, std::string(#call ": ") + hipGetErrorString(_e)); \
  } while (0)

int ensure(piadmm_obca_t h, int n) {
  if (n <= h->cap) return 0;
  if (h->d_rec) { (void)hipFree(h->d_rec); (void)hipFree(h->d_out); (void)hipFree(h->d_ist); (void)hipFree(h->d_qg); }
  if (h->d_stamps) (void)hipFree(h->d_stamps);
  h->d_rec = nullptr; h->d_out = nullptr; h->d_ist = nullptr; h->d_qg = nullptr; h->d_stamps = nullptr; h->cap = 0;
#ifdef PIADMM_STAMPS
  OHIP(h, hipMalloc(&h->d_stamps, (size_t)n * obca::NSTAMP * sizeof(unsigned long long)));
  OHIP(h, hipMemset(h->d_stamps, 0, (size_t)n * obca::NSTAMP * sizeof(unsigned long long)));
#endif
  OHIP(h, hipMalloc(&h->d_rec, (size_t)n * obca::REC * sizeof(double)));
  OHIP(h, hipMalloc(&h->d_out, (size_t)n * obca::OUT * sizeof(double)));
  OHIP(h, hipMalloc(&h->d_ist, (size_t)n * 3 * sizeof(int)));
  OHIP(h, hipMalloc(&h->d_qg, (size_t)n * sizeof(obca::WsG)));
  if (h->d_order) (void)hipFree(h->d_order);
  h->d_order = nullptr;
  h->cost_n = 0;
  OHIP(h, hipMalloc(&h->d_order, (size_t)n * sizeof(int)));
  h->cap = n;
  return 0;
}

int check_recs(piadmm_obca_t h, const double* recs, int n) {
  // host-side shape checks before any launch: parameters the kernel's bounds assume
  for (int i = 0; i < n; ++i) {
    const double* par = recs + (size_t)i * obca::REC + 283;
    if (!(par[0] > 0.0) || !(par[4] > 0.0) || !(par[5] > 0.0) || (par[6] != 0.0 && par[6] != 1.0) ||
        !(par[7] >= 1.0 && par[7] <= 1000.0) || !(par[2] > 0.0) || !(par[3] > 0.0))
      return fail(h, PIADMM_E_ARG, "obca record " + std::to_string(i) + ": bad parameters (rho, r, q > 0; prob 0/1; 1 <= max_iter <= 1000)");
  }
  return 0;
}

// The schedule of the next launches: problems by decreasing work of the last solve of this batch
// size (QP steps, then SQP iterations; the index breaks ties), or in index order when none ran
// yet.  The work each problem does does not depend on the order (tests/test_gpu_obca.py).
int schedule(piadmm_obca_t h) {
  const int n = h->n;
  h->order.resize(n);
  for (int i = 0; i < n; ++i) h->order[i] = i;
  if (h->cost_n == n) {
    // the last solve's work (waits for its launches: the batch is rescheduled between runs)
    h->cost.resize((size_t)3 * n);
    OHIP(h, hipMemcpyAsync(h->cost.data(), h->d_ist, (size_t)n * 3 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    OHIP(h, hipStreamSynchronize(h->stream));
    const int* c = h->cost.data();
    std::stable_sort(h->order.begin(), h->order.end(), [&](int a, int b) {
      if (c[3 * a + 2] != c[3 * b + 2]) return c[3 * a + 2] > c[3 * b + 2];
      return c[3 * a + 1] > c[3 * b + 1];
    });
  }
  OHIP(h, hipStreamSynchronize(h->stream));    // no earlier launch still reads the order
  OHIP(h, hipMemcpy(h->d_order, h->order.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice));
  return 0;
}

int launch(piadmm_obca_t h) {
  hipLaunchKernelGGL(obca::k_obca_sqp, dim3(h->n), dim3(64), 0, h->stream, h->d_rec, h->n, h->d_out, h->d_ist,
                     h->d_stamps, h->d_qg, h->d_order);
  OHIP(h, hipGetLastError());
  return 0;
}

// After the launches of a run: their work becomes the next run's schedule.
int record_cost(piadmm_obca_t h) {
  h->cost_n = h->n;
  return 0;
}
}  // namespace

extern "C" {

int32_t piadmm_obca_create(int32_t device, piadmm_obca_t* out) {
  if (!out) return PIADMM_E_ARG;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return PIADMM_E_NODEV;
  if (device < 0 || device >= nd) return PIADMM_E_ARG;
  auto* h = new piadmm_obca_s();
  h->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->e0) != hipSuccess || hipEventCreate(&h->e1) != hipSuccess) {
    delete h;
    return PIADMM_E_HIP;
  }
  *out = h;
  return 0;
}

int32_t piadmm_obca_destroy(piadmm_obca_t h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->d_rec) { (void)hipFree(h->d_rec); (void)hipFree(h->d_out); (void)hipFree(h->d_ist); (void)hipFree(h->d_qg); }
  if (h->d_stamps) (void)hipFree(h->d_stamps);
  if (h->d_order) (void)hipFree(h->d_order);
  if (h->e0) (void)hipEventDestroy(h->e0);
  if (h->e1) (void)hipEventDestroy(h->e1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

const char* piadmm_obca_last_error(piadmm_obca_t h) { return h ? h->err.c_str() : "null handle"; }

int32_t piadmm_obca_upload(piadmm_obca_t h, const double* recs, int32_t n) {
  if (!h) return PIADMM_E_ARG;
  if (!recs || n <= 0) return fail(h, PIADMM_E_ARG, "obca_upload: recs / n");
  if (int rc = check_recs(h, recs, n)) return rc;
  OHIP(h, hipSetDevice(h->device));
  // no batch until this upload succeeds: a failed reallocation or copy must not leave a batch size
  // that a later obca_run would launch on freed (null) buffers
  h->n = 0;
  // a new batch: the longest-first order of the last run belongs to other problems (even when the
  // size is the same), so the next run goes in index order and records this batch's work
  h->cost_n = 0;
  if (int rc = ensure(h, n)) return rc;
  OHIP(h, hipMemcpyAsync(h->d_rec, recs, (size_t)n * obca::REC * sizeof(double), hipMemcpyHostToDevice, h->stream));
  OHIP(h, hipStreamSynchronize(h->stream));
  h->n = n;
  return 0;
}

int32_t piadmm_obca_run(piadmm_obca_t h, int32_t repeats) {
  if (!h) return PIADMM_E_ARG;
  if (h->n <= 0) return fail(h, PIADMM_E_STATE, "obca_run before obca_upload");
  OHIP(h, hipSetDevice(h->device));
  if (int rc = schedule(h)) return rc;
  for (int r = 0; r < repeats; ++r)
    if (int rc = launch(h)) return rc;
  return record_cost(h);
}

int32_t piadmm_obca_time(piadmm_obca_t h, int32_t repeats, float* ms) {
  if (!h || !ms || repeats <= 0) return PIADMM_E_ARG;
  if (h->n <= 0) return fail(h, PIADMM_E_STATE, "obca_time before obca_upload");
  OHIP(h, hipSetDevice(h->device));
  if (int rc = schedule(h)) return rc;
  OHIP(h, hipEventRecord(h->e0, h->stream));
  for (int r = 0; r < repeats; ++r)
    if (int rc = launch(h)) return rc;
  OHIP(h, hipEventRecord(h->e1, h->stream));
  OHIP(h, hipEventSynchronize(h->e1));
  float t = 0.f;
  OHIP(h, hipEventElapsedTime(&t, h->e0, h->e1));
  *ms = t / (float)repeats;
  return record_cost(h);
}

int32_t piadmm_obca_download(piadmm_obca_t h, double* out, int32_t* status3, int32_t n) {
  if (!h) return PIADMM_E_ARG;
  if (n != h->n || !out || !status3) return fail(h, PIADMM_E_ARG, "obca_download: n must equal the uploaded batch");
  OHIP(h, hipSetDevice(h->device));
  OHIP(h, hipMemcpyAsync(out, h->d_out, (size_t)n * obca::OUT * sizeof(double), hipMemcpyDeviceToHost, h->stream));
  OHIP(h, hipMemcpyAsync(status3, h->d_ist, (size_t)n * 3 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
  OHIP(h, hipStreamSynchronize(h->stream));
  return 0;
}

int32_t piadmm_obca_debug_stamps(piadmm_obca_t h, uint64_t* out, int32_t n) {
  if (!h) return PIADMM_E_ARG;
  if (!h->d_stamps) return fail(h, PIADMM_E_STATE, "not a stamps build (make stamps)");
  if (n != h->n * obca::NSTAMP) return fail(h, PIADMM_E_ARG, "obca_debug_stamps: n must be 16 x the batch");
  OHIP(h, hipSetDevice(h->device));
  OHIP(h, hipMemcpyAsync(out, h->d_stamps, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
  OHIP(h, hipStreamSynchronize(h->stream));
  return 0;
}

int32_t piadmm_obca_solve(piadmm_obca_t h, const double* recs, int32_t n, double* out, int32_t* status3) {
  if (int rc = piadmm_obca_upload(h, recs, n)) return rc;
  if (int rc = piadmm_obca_run(h, 1)) return rc;
  return piadmm_obca_download(h, out, status3, n);
}

}  // extern "C"
