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
// Layout: one workgroup = one wavefront (64 lanes) = one problem; the whole SQP state (~62 KB)
// lives in LDS; lanes split stage-wise work (7 stages) and matrix work (28 x 28) among them.
// HBM traffic per problem: 296 doubles in, 224 doubles + 3 ints out -- the kernel is latency
// bound (barrier chains of the factorisations and the active-set updates), not HBM bound.

#include <hip/hip_runtime.h>

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
  // linearisation
  double A[NT][NX][NX], F[NT][NX], Wd[NT][NX][NX];
  double Wxx[NH][NX][NX], Wxl[NH][NX][NL], Wll[NH][NL][NL];
  double gX[NH][NX], gL[NT][NL];
  double ga_v[NT], ga_g[NT][9], gb_v[NT][2], gb_J[NT][2][9], gn_v[NT], gn_g[NT][NL];
  double sv[NH][NX];
  double K[NT][9][NZ];        // [dX_t; dLam_t] = K_t z + k0_t  (stage t = index + 1)
  double k0[NT][9];
  double Pm[NT][NL][2];
  double WK[9][NZ];
  double Hq[NZ][NZ], gq[NZ];
  double Hm[NZ][NZ];          // modified Hessian, then its Cholesky factor
  double J[NZ][NZ], R[NZ][NZ];
  double garow[NT][NZ], gnrow[NT][NZ];
  double din[NROW], uin[NROW];
  double x[NZ], d[NZ], zd[NZ], rd[NZ], u[MAXACT + 1], dd[NZ];
  double dX[NH][NX], dU[NT][NU], dL[NT][NL];
  double red[64];
  int act[MAXACT + 1], pact[NROW];
  int nact, npact;
  int flag;
};

static_assert(sizeof(Ws) <= 160 * 1024, "OBCA workspace exceeds the LDS of one CU");

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
// dense Cholesky of Hm in place (lower); returns true if positive definite
// ---------------------------------------------------------------------------------------------
__device__ bool chol(Ws& S) {
  int lane = threadIdx.x;
  for (int j = 0; j < NZ; ++j) {
    SYNC();
    double piv = S.Hm[j][j];
    if (!(piv > 0.0)) { SYNC(); return false; }
    double l = sqrt(piv);
    SYNC();
    if (lane == 0) S.Hm[j][j] = l;
    if (lane > j && lane < NZ) S.Hm[lane][j] /= l;
    SYNC();
    // trailing update: rows i > j, cols k in (j, i]
    for (int e = lane; e < NZ * NZ; e += 64) {
      int i = e / NZ, k = e % NZ;
      if (i > j && k > j && k <= i) S.Hm[i][k] -= S.Hm[i][j] * S.Hm[k][j];
    }
  }
  SYNC();
  return true;
}

// row c of the constraint matrix (C z >= din) dotted with v (28)
__device__ double row_dot(const Ws& S, int c, const double* v) {
  if (c >= ROWS_T * NT) {
    int j = (c - ROWS_T * NT) >> 1;
    return (c & 1) ? -v[j] : v[j];
  }
  int ti = c / ROWS_T, r = c % ROWS_T;
  const double* a;
  double sgn = 1.0;
  if (r < 10) { a = S.K[ti][r >> 1]; sgn = (r & 1) ? -1.0 : 1.0; }
  else if (r == 10) a = S.garow[ti];
  else if (r == 11) { a = S.garow[ti]; sgn = -1.0; }
  else if (r == 12) { a = S.gnrow[ti]; sgn = -1.0; }
  else { int q = r - 13; a = S.K[ti][5 + (q >> 1)]; sgn = (q & 1) ? -1.0 : 1.0; }
  double s = 0.0;
  for (int k = 0; k < NZ; ++k) s += a[k] * v[k];
  return sgn * s;
}
__device__ double row_elem(const Ws& S, int c, int k) {
  if (c >= ROWS_T * NT) {
    int j = (c - ROWS_T * NT) >> 1;
    return (k == j) ? ((c & 1) ? -1.0 : 1.0) : 0.0;
  }
  int ti = c / ROWS_T, r = c % ROWS_T;
  if (r < 10) return ((r & 1) ? -1.0 : 1.0) * S.K[ti][r >> 1][k];
  if (r == 10) return S.garow[ti][k];
  if (r == 11) return -S.garow[ti][k];
  if (r == 12) return -S.gnrow[ti][k];
  int q = r - 13;
  return ((q & 1) ? -1.0 : 1.0) * S.K[ti][5 + (q >> 1)][k];
}

// ---------------------------------------------------------------------------------------------
// Goldfarb-Idnani on min 1/2 z'Hz + gq'z, C z >= din (no equalities); H = L L' in S.Hm.
// Returns 0 ok, 2 infeasible, 1 step limit; S.x = solution, S.uin = multipliers (dense).
// ---------------------------------------------------------------------------------------------
__device__ void gi_drop(Ws& S, int k) {
  int lane = threadIdx.x;
  int q = S.nact;
  SYNC();
  // remove column k of R (shift left)
  if (lane < NZ) {
    for (int j = k; j < q - 1; ++j) S.R[lane][j] = S.R[lane][j + 1];
    S.R[lane][q - 1] = 0.0;
  }
  SYNC();
  for (int j = k; j < q - 1; ++j) {
    double a = S.R[j][j], b = S.R[j + 1][j];
    double h = hypot(a, b);
    SYNC();
    if (h != 0.0) {
      double cs = a / h, sn = b / h;
      if (lane >= j && lane < q - 1) {
        double rj = S.R[j][lane], rj1 = S.R[j + 1][lane];
        S.R[j][lane] = cs * rj + sn * rj1;
        S.R[j + 1][lane] = -sn * rj + cs * rj1;
      }
      if (lane < NZ) {
        double Jj = S.J[lane][j], Jj1 = S.J[lane][j + 1];
        S.J[lane][j] = cs * Jj + sn * Jj1;
        S.J[lane][j + 1] = -sn * Jj + cs * Jj1;
      }
    }
    SYNC();
  }
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
  double bp = S.din[p];
  while (true) {
    if (++steps > 500) return -1;
    int q = S.nact;
    SYNC();
    // d = J' n_p
    if (lane < NZ) {
      double s = 0.0;
      for (int i = 0; i < NZ; ++i) s += S.J[i][lane] * row_elem(S, p, i);
      S.d[lane] = s;
      S.dd[lane] = s;
    }
    SYNC();
    // z = J[:, q:] d[q:]
    if (lane < NZ) {
      double s = 0.0;
      for (int j = q; j < NZ; ++j) s += S.J[lane][j] * S.d[j];
      S.zd[lane] = s;
    }
    // r = R^-1 d[:q] (back substitution)
    for (int j = q - 1; j >= 0; --j) {
      SYNC();
      double rj = S.dd[j] / S.R[j][j];
      SYNC();
      if (lane == 0) S.rd[j] = rj;
      if (lane < j) S.dd[lane] -= S.R[lane][j] * rj;
    }
    SYNC();
    // partial step t1 over active rows with r_k > 1e-13 max(1, max|r|)
    double rmax = 1.0;
    {
      double v = (lane < q) ? fabs(S.rd[lane]) : 0.0;
      rmax = fmax(1.0, wmax(v));
    }
    double t1v = INFINITY;
    int l = -1;
    if (lane < q && S.rd[lane] > 1e-13 * rmax) { t1v = S.u[lane] / S.rd[lane]; l = lane; }
    wargmin(t1v, l);
    double t1 = (l >= 0) ? t1v : INFINITY;
    // full step t2
    double zn = wsum(lane < NZ ? S.zd[lane] * row_elem(S, p, lane) : 0.0);
    double dd2 = wsum(lane < NZ ? S.d[lane] * S.d[lane] : 0.0);
    double sx = row_dot(S, p, S.x) - bp;
    double t2 = (zn > 1e-12 * dd2) ? -sx / zn : INFINITY;
    double t = fmin(t1, t2);
    if (t == INFINITY) return 0;
    if (t2 == INFINITY) {
      SYNC();
      if (lane < q) S.u[lane] -= t * S.rd[lane];
      up += t;
      SYNC();
      gi_drop(S, l);
      continue;
    }
    SYNC();
    if (lane < NZ) S.x[lane] += t * S.zd[lane];
    if (lane < q) S.u[lane] -= t * S.rd[lane];
    up += t;
    SYNC();
    if (t == t2) {
      for (int j = NZ - 1; j > q; --j) {
        double a = S.d[j - 1], b = S.d[j];
        SYNC();
        if (b != 0.0) {
          double h = hypot(a, b);
          double cs = a / h, sn = b / h;
          if (lane < NZ) {
            double Jj = S.J[lane][j - 1], Jj1 = S.J[lane][j];
            S.J[lane][j - 1] = cs * Jj + sn * Jj1;
            S.J[lane][j] = -sn * Jj + cs * Jj1;
          }
          if (lane == 0) { S.d[j - 1] = h; S.d[j] = 0.0; }
        }
        SYNC();
      }
      if (lane <= q) S.R[lane][q] = S.d[lane];
      if (lane == 0) { S.act[q] = p; S.u[q] = up; S.nact = q + 1; }
      SYNC();
      return 1;
    }
    gi_drop(S, l);
  }
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
  if (lane < NZ) {
    double s = 0.0;
    for (int j = 0; j < NZ; ++j) s += S.J[lane][j] * S.dd[j];
    S.x[lane] = -s;
  }
  for (int e = lane; e < NZ * NZ; e += 64) (&S.R[0][0])[e] = 0.0;
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
__global__ void __launch_bounds__(64) k_obca_sqp(const double* __restrict__ recs, int n,
                                                 double* __restrict__ out, int* __restrict__ ist) {
  __shared__ Ws S;
  const int lane = threadIdx.x;
  const int pb = blockIdx.x;
  if (pb >= n) return;
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
  // constant parts of K: X rows' zeta columns 0; Lambda rows' zeta columns = N at block t-1
  for (int e = lane; e < NT * 9 * NZ; e += 64) (&S.K[0][0][0])[e] = 0.0;
  SYNC();
  if (lane < NT) {
    int ti = lane;
    const double NN[4][2] = {{1, 0}, {0, 1}, {1, 0}, {0, 1}};
    for (int i = 0; i < 4; ++i)
      for (int cc = 0; cc < 2; ++cc) S.K[ti][5 + i][NUV + 2 * ti + cc] = NN[i][cc];
  }
  SYNC();

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
        S.F[k][i] = D.F[i];
        for (int j = 0; j < 5; ++j) { S.A[k][i][j] = D.A[i][j]; S.Wd[k][i][j] = 0.0; }
      }
      const int fi[3] = {0, 1, 3};
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
          double s = 0.0;
          for (int f = 0; f < 3; ++f) s += S.pi[k][fi[f]] * D.Hf[f][a][b];
          S.Wd[k][2 + a][2 + b] = DT * s;
        }
    }
    SYNC();
    // ---- stages t = 1..7 (lanes 0..6): cost gradient, (5a)/(5b)/norm, Hessian blocks ----
    if (lane < NT) {
      int t = lane + 1;
      const double* Xt = S.X[t];
      const double* Lt = S.L[t - 1];
      for (int i = 0; i < 5; ++i)
        S.gX[t][i] = 2 * S.qq * (Xt[i] - S.ref[t][i]) + S.lb[t - 1][i] + S.rho * (Xt[i] - S.zb[t - 1][i]);
      for (int i = 0; i < 4; ++i) S.gL[t - 1][i] = S.lb[t - 1][5 + i] + S.rho * (Lt[i] - S.zb[t - 1][5 + i]);
      Geo G;
      geo(Xt, Lt, S.prob, S.sig_delay, G);
      double ga[9];
      S.ga_v[t - 1] = ga_val_grad(G, Lt, S.c[t - 1], ga);
      for (int i = 0; i < 9; ++i) S.ga_g[t - 1][i] = ga[i];
      for (int r = 0; r < 2; ++r) {
        S.gb_v[t - 1][r] = G.m[r] + S.w[t - 1][r];
        for (int i = 0; i < 9; ++i) S.gb_J[t - 1][r][i] = 0.0;
        S.gb_J[t - 1][r][3] = G.mt[r];
        for (int j = 0; j < 4; ++j) S.gb_J[t - 1][r][5 + j] = G.mL[r][j];
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
          S.Wxx[t][i][j] = (t < NH - 1 ? S.Wd[t][i][j] : 0.0) + (i == j ? 2 * S.qq + S.rho : 0.0) + H[i][j];
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 4; ++j) S.Wxl[t][i][j] = H[i][5 + j];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) S.Wll[t][i][j] = (i == j ? S.rho : 0.0) + H[5 + i][5 + j] - yn * Hn[i][j];
    }
    // ---- condense: K_t[0:5][0:14] = T_t, s_t ----
    if (lane < NX) S.sv[0][lane] = S.init[lane] - S.X[0][lane];
    SYNC();
    for (int k = 0; k < NT; ++k) {
      // T_{k+1} = A_k T_k + B_k E_k  (T_0 = 0); K index k holds T_{k+1}
      for (int e = lane; e < NX * NUV; e += 64) {
        int i = e / NUV, j = e % NUV;
        double s = 0.0;
        if (k > 0)
          for (int m = 0; m < NX; ++m) s += S.A[k][i][m] * S.K[k - 1][m][j];
        if (j == 2 * k && i == 2) s += DT;
        if (j == 2 * k + 1 && i == 4) s += DT;
        S.K[k][i][j] = s;
      }
      if (lane < NX) {
        double s = 0.0;
        for (int m = 0; m < NX; ++m) s += S.A[k][lane][m] * S.sv[k][m];
        S.sv[k + 1][lane] = s + S.F[k][lane] - S.X[k + 1][lane];
      }
      SYNC();
    }
    // ---- (5b) elimination: Lambda rows of K and k0 ----
    if (lane < NT) {
      int ti = lane;
      double P[4][2], pm[4], pr[4];
      double mth0 = S.gb_J[ti][0][3], mth1 = S.gb_J[ti][1][3];
      double r0 = -S.gb_v[ti][0], r1 = -S.gb_v[ti][1];
      double s3 = S.sv[ti + 1][3];
      for (int i = 0; i < 4; ++i) {
        P[i][0] = 0.5 * S.gb_J[ti][0][5 + i];
        P[i][1] = 0.5 * S.gb_J[ti][1][5 + i];
        S.Pm[ti][i][0] = P[i][0];
        S.Pm[ti][i][1] = P[i][1];
        pm[i] = P[i][0] * mth0 + P[i][1] * mth1;
        pr[i] = P[i][0] * (r0 - mth0 * s3) + P[i][1] * (r1 - mth1 * s3);
      }
      for (int i = 0; i < 5; ++i) S.k0[ti][i] = S.sv[ti + 1][i];
      for (int i = 0; i < 4; ++i) S.k0[ti][5 + i] = pr[i];
      for (int i = 0; i < 4; ++i) S.red[ti * 4 + i] = pm[i];   // P m_theta, used below
    }
    SYNC();
    for (int e = lane; e < NT * 4 * NUV; e += 64) {
      int ti = e / (4 * NUV), rem = e % (4 * NUV), i = rem / NUV, j = rem % NUV;
      S.K[ti][5 + i][j] = -S.red[ti * 4 + i] * S.K[ti][3][j];
    }
    // ---- condensed Hessian and gradient ----
    for (int e = lane; e < NZ * NZ; e += 64) {
      int a = e / NZ, b = e % NZ;
      (&S.Hq[0][0])[e] = (a == b && a < NUV) ? 2 * S.rr : 0.0;
    }
    if (lane < NZ) S.gq[lane] = lane < NUV ? 2 * S.rr * (&S.U[0][0])[lane] : 0.0;
    SYNC();
    for (int ti = 0; ti < NT; ++ti) {
      int t = ti + 1;
      // WK = W_t K_t (9 x 28)
      for (int e = lane; e < 9 * NZ; e += 64) {
        int i = e / NZ, a = e % NZ;
        double s = 0.0;
        for (int j = 0; j < 9; ++j) {
          double wij = (i < 5) ? (j < 5 ? S.Wxx[t][i][j] : S.Wxl[t][i][j - 5])
                               : (j < 5 ? S.Wxl[t][j][i - 5] : S.Wll[t][i - 5][j - 5]);
          s += wij * S.K[ti][j][a];
        }
        S.WK[i][a] = s;
      }
      SYNC();
      for (int e = lane; e < NZ * NZ; e += 64) {
        int a = e / NZ, b = e % NZ;
        double s = 0.0;
        for (int i = 0; i < 9; ++i) s += S.K[ti][i][a] * S.WK[i][b];
        S.Hq[a][b] += s;
      }
      if (lane < NZ) {
        // gq += K_t' (W_t k0_t + g_t)
        double s = 0.0;
        for (int i = 0; i < 9; ++i) {
          double v = (i < 5) ? S.gX[t][i] : S.gL[ti][i - 5];
          for (int j = 0; j < 9; ++j) {
            double wij = (i < 5) ? (j < 5 ? S.Wxx[t][i][j] : S.Wxl[t][i][j - 5])
                                 : (j < 5 ? S.Wxl[t][j][i - 5] : S.Wll[t][i - 5][j - 5]);
            v += wij * S.k0[ti][j];
          }
          s += S.K[ti][i][lane] * v;
        }
        S.gq[lane] += s;
      }
      SYNC();
    }
    // symmetrise
    for (int e = lane; e < NZ * NZ; e += 64) {
      int a = e / NZ, b = e % NZ;
      if (a < b) {
        double v = 0.5 * (S.Hq[a][b] + S.Hq[b][a]);
        S.Hq[a][b] = v;
        S.Hq[b][a] = v;
      }
    }
    // ---- constraint rows ----
    for (int e = lane; e < NT * NZ; e += 64) {
      int ti = e / NZ, a = e % NZ;
      double s = 0.0;
      for (int i = 0; i < 9; ++i) s += S.ga_g[ti][i] * S.K[ti][i][a];
      S.garow[ti][a] = s;
      double g = 0.0;
      for (int j = 0; j < 4; ++j) g += S.gn_g[ti][j] * S.K[ti][5 + j][a];
      S.gnrow[ti][a] = g;
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
          for (int i = 0; i < 9; ++i) base += S.ga_g[ti][i] * S.k0[ti][i];
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
    // ---- Hessian modification ----
    for (int e = lane; e < NZ * NZ; e += 64) (&S.Hm[0][0])[e] = (&S.Hq[0][0])[e];
    bool pd = chol(S);
    if (!pd && S.npact > 0) {
      // Ga = sum over previous active rows of a a' / |a|^2  (in R, free until the QP)
      for (int e = lane; e < NZ * NZ; e += 64) (&S.R[0][0])[e] = 0.0;
      SYNC();
      for (int k = 0; k < S.npact; ++k) {
        int c = S.pact[k];
        double a = (lane < NZ) ? row_elem(S, c, lane) : 0.0;
        double nn = wsum(a * a);
        double inv = 1.0 / fmax(sqrt(nn), 1e-300);
        if (lane < NZ) S.dd[lane] = a * inv;
        SYNC();
        for (int e = lane; e < NZ * NZ; e += 64) {
          int i = e / NZ, j = e % NZ;
          S.R[i][j] += S.dd[i] * S.dd[j];
        }
        SYNC();
      }
      double hm = wmax(lane < NZ ? fabs(S.Hq[lane][lane]) : 0.0);
      double sig = 1e-4 * hm;
      for (int a = 0; a < 8; ++a) {
        for (int e = lane; e < NZ * NZ; e += 64) (&S.Hm[0][0])[e] = (&S.Hq[0][0])[e] + sig * (&S.R[0][0])[e];
        pd = chol(S);
        if (pd) break;
        sig *= 10.0;
      }
      if (!pd) {
        // H0 = Hq + sig_last Ga (sig was multiplied once more after the last try)
        sig /= 10.0;
        for (int e = lane; e < NZ * NZ; e += 64) (&S.R[0][0])[e] = (&S.Hq[0][0])[e] + sig * (&S.R[0][0])[e];
        SYNC();
      }
    } else if (!pd) {
      for (int e = lane; e < NZ * NZ; e += 64) (&S.R[0][0])[e] = (&S.Hq[0][0])[e];
      SYNC();
    }
    if (!pd) {
      // H0 in R: H0 + tau diag(max(|H0_ii|, 1e-12)), tau = 1e-6, 1e-5, ...
      double tau = 0.0;
      for (int a = 0; a < 16; ++a) {
        tau = (tau == 0.0) ? 1e-6 : tau * 10.0;
        for (int e = lane; e < NZ * NZ; e += 64) {
          int i = e / NZ, j = e % NZ;
          double h = (&S.R[0][0])[e];
          (&S.Hm[0][0])[e] = (i == j) ? h + tau * fmax(fabs(h), 1e-12) : h;
        }
        pd = chol(S);
        if (pd) break;
      }
      if (!pd) { status = PIADMM_OBCA_HESSIAN_FAIL; break; }
    }
    // ---- QP ----
    int steps = 0;
    int qst = gi_solve(S, steps);
    qp_total += steps;
    if (qst != 0) { status = (qst == 2) ? PIADMM_OBCA_QP_INFEASIBLE : PIADMM_OBCA_MAX_ITER; break; }
    if (lane == 0) {
      int m = 0;
      for (int c = 0; c < NROW; ++c)
        if (S.uin[c] > 0.0) S.pact[m++] = c;
      S.npact = m;
    }
    // ---- step in the full space ----
    if (lane < NUV) (&S.dU[0][0])[lane] = S.x[lane];
    if (lane < NX) S.dX[0][lane] = S.sv[0][lane];
    for (int e = lane; e < NT * 9; e += 64) {
      int ti = e / 9, i = e % 9;
      double s = S.k0[ti][i];
      for (int a = 0; a < NZ; ++a) s += S.K[ti][i][a] * S.x[a];
      if (i < 5) S.dX[ti + 1][i] = s;
      else S.dL[ti][i - 5] = s;
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
        double s = S.gL[ti][i];
        for (int j = 0; j < 5; ++j) s += S.Wxl[t][j][i] * S.dX[t][j];
        for (int j = 0; j < 4; ++j) s += S.Wll[t][i][j] * S.dL[ti][j];
        s -= S.nya[ti] * S.ga_g[ti][5 + i] + S.nyn[ti] * S.gn_g[ti][i] + S.nyl[ti][i];
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
        double s = S.gX[t][i];
        for (int j = 0; j < 5; ++j) s += S.Wxx[t][i][j] * S.dX[t][j];
        for (int j = 0; j < 4; ++j) s += S.Wxl[t][i][j] * S.dL[ti][j];
        s -= S.nya[ti] * S.ga_g[ti][i] + S.nyb[ti][0] * S.gb_J[ti][0][i] + S.nyb[ti][1] * S.gb_J[ti][1][i];
        s -= S.nyx[ti][i];
        if (t < NH - 1)
          for (int j = 0; j < 5; ++j) s += S.A[t][j][i] * S.npi[t][j];
        S.npi[ti][i] = s;
      }
      SYNC();
    }
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
    for (int e = lane; e < NT * NX; e += 64) gd += (&S.gX[1][0])[e] * (&S.dX[1][0])[e];
    if (lane < NUV) gd += 2 * S.rr * (&S.U[0][0])[lane] * (&S.dU[0][0])[lane];
    if (lane < NT * NL) gd += (&S.gL[0][0])[lane] * (&S.dL[0][0])[lane];
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
  if (h->d_rec) { (void)hipFree(h->d_rec); (void)hipFree(h->d_out); (void)hipFree(h->d_ist); }
  h->d_rec = nullptr; h->d_out = nullptr; h->d_ist = nullptr; h->cap = 0;
  OHIP(h, hipMalloc(&h->d_rec, (size_t)n * obca::REC * sizeof(double)));
  OHIP(h, hipMalloc(&h->d_out, (size_t)n * obca::OUT * sizeof(double)));
  OHIP(h, hipMalloc(&h->d_ist, (size_t)n * 3 * sizeof(int)));
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

int launch(piadmm_obca_t h) {
  hipLaunchKernelGGL(obca::k_obca_sqp, dim3(h->n), dim3(64), 0, h->stream, h->d_rec, h->n, h->d_out, h->d_ist);
  OHIP(h, hipGetLastError());
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
  if (h->d_rec) { (void)hipFree(h->d_rec); (void)hipFree(h->d_out); (void)hipFree(h->d_ist); }
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
  for (int r = 0; r < repeats; ++r)
    if (int rc = launch(h)) return rc;
  return 0;
}

int32_t piadmm_obca_time(piadmm_obca_t h, int32_t repeats, float* ms) {
  if (!h || !ms || repeats <= 0) return PIADMM_E_ARG;
  if (h->n <= 0) return fail(h, PIADMM_E_STATE, "obca_time before obca_upload");
  OHIP(h, hipSetDevice(h->device));
  OHIP(h, hipEventRecord(h->e0, h->stream));
  for (int r = 0; r < repeats; ++r)
    if (int rc = launch(h)) return rc;
  OHIP(h, hipEventRecord(h->e1, h->stream));
  OHIP(h, hipEventSynchronize(h->e1));
  float t = 0.f;
  OHIP(h, hipEventElapsedTime(&t, h->e0, h->e1));
  *ms = t / (float)repeats;
  return 0;
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

int32_t piadmm_obca_solve(piadmm_obca_t h, const double* recs, int32_t n, double* out, int32_t* status3) {
  if (int rc = piadmm_obca_upload(h, recs, n)) return rc;
  if (int rc = piadmm_obca_run(h, 1)) return rc;
  return piadmm_obca_download(h, out, status3, n);
}

}  // extern "C"
