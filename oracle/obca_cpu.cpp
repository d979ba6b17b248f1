// obca_cpu.cpp -- CPU baseline of the OBCA local subproblem (MEASUREMENT / TEST INFRASTRUCTURE).
//
// The SQP of oracle/obca_oracle.py (solve_local, gi_qp) in C++ -O3, sequential per problem,
// OpenMP over the problems of a batch: the "B-opt" analogue for the OBCA path (bench.py --obca
// cpu_baseline).  Same record / output layout as the GPU path (include/piadmm.h PIADMM_OBCA_*).
// tests/test_obca_cpu.py holds it to the NumPy oracle.  It restates the reference's NLP
// (Distributed_planner/decentralized/optimizer.py:61-168); the reference solves it with IPOPT
// (:170-180), absent here.
#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstring>

namespace {

constexpr int NH = 8, NX = 5, NU = 2, NL = 4, NT = 7;
constexpr int NUV = NU * NT, NZ = NUV + 2 * NT, ROWS_T = 21, NROW = ROWS_T * NT + 2 * NUV;
constexpr int REC = 296, OUT = 224;
constexpr double LENGTH = 3.5, WIDTH = 2.0, LF = 1.5, LR = 1.0;
constexpr double MAX_STEER = 0.6, MAX_V = 20.0, MAX_ACC = 5.0, MAX_STEER_RATE = 20.0;
constexpr double DT = 0.1, AVG_DELAY = 0.05, VAR_DELAY = 0.025;
constexpr double LAM_MAX = 100000.0, GA_MAX = 1000.0, KB = LR / (LR + LF), TWO_PI = 6.283185307179586;

struct Geo {
  double e[2], n[2], m[2], mt[2], mL[2][4], mtL[2][4], d[2], dv[2], dvv[2], dt[2], dtt[2], dvt[2], q[2];
};

void geo(const double* Xt, const double* Lt, int prob, Geo& G) {
  double v = Xt[2], th = Xt[3], c = std::cos(th), s = std::sin(th);
  G.e[0] = c; G.e[1] = s; G.n[0] = -s; G.n[1] = c;
  double sg = prob ? 1.0 : -1.0, a1 = Lt[0] - Lt[2], a2 = sg * (Lt[1] - Lt[3]);
  for (int i = 0; i < 2; ++i) {
    G.m[i] = a1 * G.e[i] + a2 * G.n[i];
    G.mt[i] = a1 * G.n[i] - a2 * G.e[i];
    G.mL[i][0] = G.e[i]; G.mL[i][1] = sg * G.n[i]; G.mL[i][2] = -G.e[i]; G.mL[i][3] = -sg * G.n[i];
    G.mtL[i][0] = G.n[i]; G.mtL[i][1] = -sg * G.e[i]; G.mtL[i][2] = -G.n[i]; G.mtL[i][3] = sg * G.e[i];
  }
  if (prob) {
    double k = std::sqrt(0.95 / 0.05) * VAR_DELAY * VAR_DELAY, da = AVG_DELAY;
    G.d[0] = da * v * c + k * v * v * c * c;        G.d[1] = da * v * s + k * v * v * s * s;
    G.dv[0] = da * c + 2 * k * v * c * c;           G.dv[1] = da * s + 2 * k * v * s * s;
    G.dvv[0] = 2 * k * c * c;                       G.dvv[1] = 2 * k * s * s;
    G.dt[0] = -da * v * s - 2 * k * v * v * c * s;  G.dt[1] = da * v * c + 2 * k * v * v * s * c;
    G.dtt[0] = -da * v * c - 2 * k * v * v * (c * c - s * s);
    G.dtt[1] = -da * v * s + 2 * k * v * v * (c * c - s * s);
    G.dvt[0] = -da * s - 4 * k * v * c * s;         G.dvt[1] = da * c + 4 * k * v * s * c;
  } else {
    for (int i = 0; i < 2; ++i) G.d[i] = G.dv[i] = G.dvv[i] = G.dt[i] = G.dtt[i] = G.dvt[i] = 0.0;
  }
  G.q[0] = Xt[0] + G.d[0];
  G.q[1] = Xt[1] + G.d[1];
}

inline double dot2(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1]; }

double ga_val(const Geo& G, const double* Lt, double ct, double* g) {
  const double B0[4] = {LENGTH / 2, WIDTH / 2, LENGTH / 2, WIDTH / 2};
  double val = -(B0[0] * Lt[0] + B0[1] * Lt[1] + B0[2] * Lt[2] + B0[3] * Lt[3]) - dot2(G.q, G.m) - ct;
  if (g) {
    g[0] = -G.m[0]; g[1] = -G.m[1]; g[2] = -dot2(G.dv, G.m); g[3] = -dot2(G.dt, G.m) - dot2(G.q, G.mt); g[4] = 0.0;
    for (int j = 0; j < 4; ++j) g[5 + j] = -B0[j] - (G.q[0] * G.mL[0][j] + G.q[1] * G.mL[1][j]);
  }
  return val;
}

void ga_hess(const Geo& G, double H[9][9]) {
  std::memset(H, 0, sizeof(double) * 81);
  H[0][3] = H[3][0] = -G.mt[0];
  H[1][3] = H[3][1] = -G.mt[1];
  for (int j = 0; j < 4; ++j) {
    H[0][5 + j] = H[5 + j][0] = -G.mL[0][j];
    H[1][5 + j] = H[5 + j][1] = -G.mL[1][j];
    H[2][5 + j] = H[5 + j][2] = -(G.dv[0] * G.mL[0][j] + G.dv[1] * G.mL[1][j]);
    H[3][5 + j] = H[5 + j][3] = -(G.dt[0] * G.mL[0][j] + G.dt[1] * G.mL[1][j]) - (G.q[0] * G.mtL[0][j] + G.q[1] * G.mtL[1][j]);
  }
  H[2][2] = -dot2(G.dvv, G.m);
  H[2][3] = H[3][2] = -dot2(G.dvt, G.m) - dot2(G.dv, G.mt);
  H[3][3] = -dot2(G.dtt, G.m) - 2 * dot2(G.dt, G.mt) + dot2(G.q, G.m);
}

struct Dyn { double F[5], A[5][5], Hf[3][3][3]; };

void dyn_eval(const double* Xk, const double* Uk, Dyn& D) {
  double v = Xk[2], th = Xk[3], st = Xk[4], tn = std::tan(st), beta = std::atan(KB * tn);
  double sec2 = 1.0 + tn * tn, den = 1.0 + KB * KB * tn * tn, bp = KB * sec2 / den;
  double bpp = 2.0 * KB * tn * sec2 * (1.0 - KB * KB) / (den * den);
  double ph = th + beta, cp = std::cos(ph), sp = std::sin(ph), cb = std::cos(beta), sb = std::sin(beta);
  double f[5] = {v * cp, v * sp, Uk[0], v / LR * sb, Uk[1]};
  for (int i = 0; i < 5; ++i) D.F[i] = Xk[i] + DT * f[i];
  double Jx[5][5] = {};
  Jx[0][2] = cp; Jx[0][3] = -v * sp; Jx[0][4] = -v * sp * bp;
  Jx[1][2] = sp; Jx[1][3] = v * cp; Jx[1][4] = v * cp * bp;
  Jx[3][2] = sb / LR; Jx[3][4] = v * cb * bp / LR;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) D.A[i][j] = (i == j ? 1.0 : 0.0) + DT * Jx[i][j];
  double(*H0)[3] = D.Hf[0];
  double(*H1)[3] = D.Hf[1];
  double(*H3)[3] = D.Hf[2];
  H0[0][0] = 0; H0[0][1] = H0[1][0] = -sp; H0[0][2] = H0[2][0] = -sp * bp;
  H0[1][1] = -v * cp; H0[1][2] = H0[2][1] = -v * cp * bp; H0[2][2] = -v * cp * bp * bp - v * sp * bpp;
  H1[0][0] = 0; H1[0][1] = H1[1][0] = cp; H1[0][2] = H1[2][0] = cp * bp;
  H1[1][1] = -v * sp; H1[1][2] = H1[2][1] = -v * sp * bp; H1[2][2] = -v * sp * bp * bp + v * cp * bpp;
  H3[0][0] = 0; H3[0][1] = H3[1][0] = 0; H3[0][2] = H3[2][0] = cb * bp / LR;
  H3[1][1] = 0; H3[1][2] = H3[2][1] = 0; H3[2][2] = v * (-sb * bp * bp + cb * bpp) / LR;
}

struct P {
  double init[NX], ref[NH][NX], w[NT][2], c[NT], lb[NT][9], zb[NT][9];
  double rho, min_dis, max_x, max_y, rr, qq;
  int prob, max_iter;
};

void cost_viol(const P& p, const double (*X)[NX], const double (*U)[NU], const double (*L)[NL], double& f, double& v) {
  f = 0.0; v = 0.0;
  for (int i = 0; i < 5; ++i) v += std::fabs(X[0][i] - p.init[i]);
  for (int k = 0; k < NT; ++k) {
    Dyn D;
    dyn_eval(X[k], U[k], D);
    for (int i = 0; i < 5; ++i) v += std::fabs(X[k + 1][i] - D.F[i]);
  }
  const double lo[5] = {0.0, -p.max_y, -MAX_V, -TWO_PI, -MAX_STEER};
  const double hi[5] = {p.max_x, p.max_y, MAX_V, TWO_PI, MAX_STEER};
  for (int t = 1; t < NH; ++t) {
    const double* Xt = X[t];
    const double* Lt = L[t - 1];
    double s9[9];
    for (int i = 0; i < 5; ++i) s9[i] = Xt[i];
    for (int i = 0; i < 4; ++i) s9[5 + i] = Lt[i];
    double ee = 0, lbs = 0, zz = 0;
    for (int i = 0; i < 5; ++i) { double e = Xt[i] - p.ref[t][i]; ee += e * e; }
    for (int i = 0; i < 9; ++i) { lbs += p.lb[t - 1][i] * s9[i]; double z = s9[i] - p.zb[t - 1][i]; zz += z * z; }
    f += p.rr * (U[t - 1][0] * U[t - 1][0] + U[t - 1][1] * U[t - 1][1]) + p.qq * ee + lbs + 0.5 * p.rho * zz;
    Geo G;
    geo(Xt, Lt, p.prob, G);
    double ga = ga_val(G, Lt, p.c[t - 1], nullptr);
    v += std::fmax(0.0, p.min_dis - ga) + std::fmax(0.0, ga - GA_MAX);
    v += std::fabs(G.m[0] + p.w[t - 1][0]) + std::fabs(G.m[1] + p.w[t - 1][1]);
    double a1 = Lt[0] - Lt[2], a2 = Lt[1] - Lt[3];
    v += std::fmax(0.0, a1 * a1 + a2 * a2 - 1.0);
    for (int j = 0; j < 5; ++j) v += std::fmax(0.0, lo[j] - Xt[j]) + std::fmax(0.0, Xt[j] - hi[j]);
  }
}

bool chol(double H[NZ][NZ]) {
  for (int j = 0; j < NZ; ++j) {
    double piv = H[j][j];
    if (!(piv > 0.0)) return false;
    double l = std::sqrt(piv);
    H[j][j] = l;
    for (int i = j + 1; i < NZ; ++i) H[i][j] /= l;
    for (int i = j + 1; i < NZ; ++i)
      for (int k = j + 1; k <= i; ++k) H[i][k] -= H[i][j] * H[k][j];
  }
  return true;
}

// warm equality solve on the rows `warm` (oracle warm_eqp): J = L^-T, y0 = L^-1 g
bool warm_eqp(const double J[NZ][NZ], const double* y0, const double C[NROW][NZ], const double* din, const int* warm,
              int m, double* x, double* uin) {
  static thread_local double Y[NZ][NZ], S[NZ][NZ];
  for (int k = 0; k < m; ++k)
    for (int i = 0; i < NZ; ++i) { double s = 0; for (int j = 0; j < NZ; ++j) s += J[j][i] * C[warm[k]][j]; Y[i][k] = s; }
  double dmax = 0;
  for (int k = 0; k < m; ++k)
    for (int l = 0; l < m; ++l) { double s = 0; for (int i = 0; i < NZ; ++i) s += Y[i][k] * Y[i][l]; S[k][l] = s; }
  for (int k = 0; k < m; ++k) dmax = std::fmax(dmax, S[k][k]);
  for (int j = 0; j < m; ++j) {          // Cholesky of S in place (lower)
    double piv = S[j][j];
    for (int k = 0; k < j; ++k) piv -= S[j][k] * S[j][k];
    if (!(piv > 0.0)) return false;
    double l = std::sqrt(piv);
    if (l <= 1e-7 * std::sqrt(dmax)) return false;
    S[j][j] = l;
    for (int i = j + 1; i < m; ++i) {
      double v = S[i][j];
      for (int k = 0; k < j; ++k) v -= S[i][k] * S[j][k];
      S[i][j] = v / l;
    }
  }
  auto ssolve = [&](double* v) {
    for (int j = 0; j < m; ++j) { for (int k = 0; k < j; ++k) v[j] -= S[j][k] * v[k]; v[j] /= S[j][j]; }
    for (int j = m - 1; j >= 0; --j) { for (int k = j + 1; k < m; ++k) v[j] -= S[k][j] * v[k]; v[j] /= S[j][j]; }
  };
  double lam[NZ], w[NZ], z[NZ], dl[NZ];
  for (int k = 0; k < m; ++k) { double s = din[warm[k]]; for (int i = 0; i < NZ; ++i) s += Y[i][k] * y0[i]; lam[k] = s; }
  ssolve(lam);
  for (int i = 0; i < NZ; ++i) { double s = -y0[i]; for (int k = 0; k < m; ++k) s += Y[i][k] * lam[k]; w[i] = s; }
  for (int rep = 0; rep < 2; ++rep) {
    for (int i = 0; i < NZ; ++i) { double s = 0; for (int j = 0; j < NZ; ++j) s += J[i][j] * w[j]; z[i] = s; }
    for (int k = 0; k < m; ++k) { double s = din[warm[k]]; for (int j = 0; j < NZ; ++j) s -= C[warm[k]][j] * z[j]; dl[k] = s; }
    ssolve(dl);
    for (int k = 0; k < m; ++k) lam[k] += dl[k];
    for (int i = 0; i < NZ; ++i) { double s = 0; for (int k = 0; k < m; ++k) s += Y[i][k] * dl[k]; w[i] += s; }
  }
  double lmax = 1.0;
  for (int k = 0; k < m; ++k) lmax = std::fmax(lmax, std::fabs(lam[k]));
  for (int k = 0; k < m; ++k) if (lam[k] < -1e-12 * lmax) return false;
  for (int i = 0; i < NZ; ++i) { double s = 0; for (int j = 0; j < NZ; ++j) s += J[i][j] * w[j]; z[i] = s; }
  for (int c = 0; c < NROW; ++c) {
    double s = -din[c];
    for (int k = 0; k < NZ; ++k) s += C[c][k] * z[k];
    if (s < -1e-11 * (1.0 + std::fabs(din[c]))) return false;
  }
  for (int i = 0; i < NZ; ++i) x[i] = z[i];
  for (int c = 0; c < NROW; ++c) uin[c] = 0.0;
  for (int k = 0; k < m; ++k) uin[warm[k]] = std::fmax(lam[k], 0.0);
  return true;
}

// Goldfarb-Idnani (oracle gi_qp without equalities); Lf = Cholesky factor (lower) of H.
int gi(const double Lf[NZ][NZ], const double* g, const double C[NROW][NZ], const double* din, double* x, double* uin,
       int& steps, const int* warm, int nwarm, int& hit) {
  static thread_local double J[NZ][NZ], R[NZ][NZ];
  double u[NZ + 1], d[NZ], z[NZ], r[NZ];
  int act[NZ + 1], q = 0;
  for (int j = 0; j < NZ; ++j) {
    double y[NZ];
    for (int i = 0; i < NZ; ++i) {
      if (i < j) { y[i] = 0; continue; }
      double s = (i == j) ? 1.0 : 0.0;
      for (int k = j; k < i; ++k) s -= Lf[i][k] * y[k];
      y[i] = s / Lf[i][i];
    }
    for (int i = 0; i < NZ; ++i) J[j][i] = y[i];
  }
  for (int j = 0; j < NZ; ++j) { double s = 0; for (int i = 0; i < NZ; ++i) s += J[i][j] * g[i]; d[j] = s; }
  hit = 0;
  if (nwarm > 0 && warm_eqp(J, d, C, din, warm, nwarm, x, uin)) { hit = 1; return 0; }
  for (int i = 0; i < NZ; ++i) { double s = 0; for (int j = 0; j < NZ; ++j) s += J[i][j] * d[j]; x[i] = -s; }
  std::memset(R, 0, sizeof(R));
  auto drop = [&](int k) {
    for (int i = 0; i < NZ; ++i) { for (int j = k; j < q - 1; ++j) R[i][j] = R[i][j + 1]; R[i][q - 1] = 0.0; }
    for (int j = k; j < q - 1; ++j) {
      double a = R[j][j], b = R[j + 1][j], h = std::hypot(a, b);
      if (h == 0.0) continue;
      double cs = a / h, sn = b / h;
      for (int col = j; col < q - 1; ++col) {
        double rj = R[j][col], rj1 = R[j + 1][col];
        R[j][col] = cs * rj + sn * rj1;
        R[j + 1][col] = -sn * rj + cs * rj1;
      }
      for (int i = 0; i < NZ; ++i) {
        double Jj = J[i][j], Jj1 = J[i][j + 1];
        J[i][j] = cs * Jj + sn * Jj1;
        J[i][j + 1] = -sn * Jj + cs * Jj1;
      }
    }
    for (int j = k; j < q - 1; ++j) { act[j] = act[j + 1]; u[j] = u[j + 1]; }
    --q;
  };
  while (true) {
    int p = -1;
    double best = 0.0;
    for (int cI = 0; cI < NROW; ++cI) {
      double s = -din[cI];
      for (int k = 0; k < NZ; ++k) s += C[cI][k] * x[k];
      if (p < 0 || s < best) { best = s; p = cI; }
    }
    if (!(best < -1e-11 * (1.0 + std::fabs(din[p])))) break;
    const double* np_ = C[p];
    double bp = din[p], up = 0.0;
    while (true) {
      if (++steps > 500) return 1;
      for (int j = 0; j < NZ; ++j) { double s = 0; for (int i = 0; i < NZ; ++i) s += J[i][j] * np_[i]; d[j] = s; }
      for (int i = 0; i < NZ; ++i) { double s = 0; for (int j = q; j < NZ; ++j) s += J[i][j] * d[j]; z[i] = s; }
      double dd[NZ];
      for (int j = 0; j < q; ++j) dd[j] = d[j];
      for (int j = q - 1; j >= 0; --j) { r[j] = dd[j] / R[j][j]; for (int i = 0; i < j; ++i) dd[i] -= R[i][j] * r[j]; }
      double rmax = 1.0;
      for (int k = 0; k < q; ++k) rmax = std::fmax(rmax, std::fabs(r[k]));
      double t1 = INFINITY;
      int l = -1;
      for (int k = 0; k < q; ++k)
        if (r[k] > 1e-13 * rmax) { double ratio = u[k] / r[k]; if (ratio < t1) { t1 = ratio; l = k; } }
      double zn = 0, d2 = 0, sx = -bp;
      for (int i = 0; i < NZ; ++i) { zn += z[i] * np_[i]; d2 += d[i] * d[i]; sx += np_[i] * x[i]; }
      double t2 = (zn > 1e-12 * d2) ? -sx / zn : INFINITY;
      double t = std::fmin(t1, t2);
      if (t == INFINITY) return 2;
      if (t2 == INFINITY) {
        for (int k = 0; k < q; ++k) u[k] -= t * r[k];
        up += t;
        drop(l);
        continue;
      }
      for (int i = 0; i < NZ; ++i) x[i] += t * z[i];
      for (int k = 0; k < q; ++k) u[k] -= t * r[k];
      up += t;
      if (t == t2) {
        double alpha = d[q];
        if (q < NZ - 1) {
          double ss = 0.0;
          for (int j = q + 1; j < NZ; ++j) ss += d[j] * d[j];
          if (ss > 0.0) {
            double a0 = d[q], sig = std::sqrt(a0 * a0 + ss);
            alpha = (a0 > 0.0) ? -sig : sig;
            double v0 = a0 - alpha, beta = 1.0 / (sig * (sig + std::fabs(a0)));
            for (int i = 0; i < NZ; ++i) {
              double sv = J[i][q] * v0;
              for (int j = q + 1; j < NZ; ++j) sv += J[i][j] * d[j];
              sv *= beta;
              J[i][q] -= sv * v0;
              for (int j = q + 1; j < NZ; ++j) J[i][j] -= sv * d[j];
            }
          }
        }
        for (int i = 0; i < q; ++i) R[i][q] = d[i];
        R[q][q] = alpha;
        act[q] = p; u[q] = up; ++q;
        break;
      }
      drop(l);
    }
  }
  for (int cI = 0; cI < NROW; ++cI) uin[cI] = 0.0;
  for (int k = 0; k < q; ++k) uin[act[k]] = u[k];
  return 0;
}

void solve_one(const double* rec, double* o, int* ist) {
  P p;
  std::memcpy(p.init, rec, 5 * sizeof(double));
  std::memcpy(p.ref, rec + 5, 40 * sizeof(double));
  for (int t = 0; t < NT; ++t) {
    const double* Ao = rec + 45 + t * 8;
    const double* bo = rec + 101 + t * 4;
    const double* lij = rec + 129 + t * 4;
    double w0 = 0, w1 = 0, cc = 0;
    for (int i = 0; i < 4; ++i) { w0 += Ao[i * 2] * lij[i]; w1 += Ao[i * 2 + 1] * lij[i]; cc += bo[i] * lij[i]; }
    p.w[t][0] = w0; p.w[t][1] = w1; p.c[t] = cc;
  }
  std::memcpy(p.lb, rec + 157, 63 * sizeof(double));
  std::memcpy(p.zb, rec + 220, 63 * sizeof(double));
  const double* par = rec + 283;
  p.rho = par[0]; p.min_dis = par[1]; p.max_x = par[2]; p.max_y = par[3]; p.rr = par[4]; p.qq = par[5];
  p.prob = (int)par[6]; p.max_iter = (int)par[7];

  double X[NH][NX], U[NT][NU] = {}, L[NT][NL];
  std::memcpy(X, p.ref, sizeof(X));
  for (int ti = 0; ti < NT; ++ti) {
    double th = p.ref[ti + 1][3], c = std::cos(th), s = std::sin(th), sg = p.prob ? 1.0 : -1.0;
    double u0 = -p.w[ti][0], u1 = -p.w[ti][1];
    double ce = c * u0 + s * u1, cn = sg * (-s * u0 + c * u1);
    L[ti][0] = std::fmax(ce, 0.0); L[ti][2] = std::fmax(-ce, 0.0);
    L[ti][1] = std::fmax(cn, 0.0); L[ti][3] = std::fmax(-cn, 0.0);
  }
  double ya[NT] = {}, yb[NT][2] = {}, yn[NT] = {}, yx[NT][NX] = {}, pi[NT][NX] = {}, yu[NUV] = {}, yl[NT][NL] = {};
  double nya[NT], nyb[NT][2], nyn[NT], nyx[NT][NX], npi[NT][NX], nyu[NUV], nyl[NT][NL];
  static thread_local double K[NT][9][NZ], Hq[NZ][NZ], Hm[NZ][NZ], H0[NZ][NZ], Ga[NZ][NZ], C[NROW][NZ];
  double k0[NT][9], Pm[NT][4][2], gq[NZ], din[NROW], uin[NROW], zq[NZ];
  std::memset(K, 0, sizeof(K));
  for (int ti = 0; ti < NT; ++ti) {
    const double NN[4][2] = {{1, 0}, {0, 1}, {1, 0}, {0, 1}};
    for (int i = 0; i < 4; ++i)
      for (int c2 = 0; c2 < 2; ++c2) K[ti][5 + i][NUV + 2 * ti + c2] = NN[i][c2];
  }
  int pact[NROW], npact = -1;
  double mu = 0.0;
  int qp_total = 0, status = 1, it;
  for (it = 0; it < p.max_iter; ++it) {
    Dyn dyn[NT];
    for (int k = 0; k < NT; ++k) dyn_eval(X[k], U[k], dyn[k]);
    double Wxx[NH][NX][NX], Wxl[NH][NX][NL], Wll[NH][NL][NL], gX[NH][NX], gL[NT][NL];
    double ga_v[NT], ga_g[NT][9], gb_v[NT][2], gb_J[NT][2][9], gn_v[NT], gn_g[NT][4];
    for (int t = 1; t < NH; ++t) {
      const double* Xt = X[t];
      const double* Lt = L[t - 1];
      for (int i = 0; i < 5; ++i) gX[t][i] = 2 * p.qq * (Xt[i] - p.ref[t][i]) + p.lb[t - 1][i] + p.rho * (Xt[i] - p.zb[t - 1][i]);
      for (int i = 0; i < 4; ++i) gL[t - 1][i] = p.lb[t - 1][5 + i] + p.rho * (Lt[i] - p.zb[t - 1][5 + i]);
      Geo G;
      geo(Xt, Lt, p.prob, G);
      ga_v[t - 1] = ga_val(G, Lt, p.c[t - 1], ga_g[t - 1]);
      for (int r = 0; r < 2; ++r) {
        gb_v[t - 1][r] = G.m[r] + p.w[t - 1][r];
        for (int i = 0; i < 9; ++i) gb_J[t - 1][r][i] = 0.0;
        gb_J[t - 1][r][3] = G.mt[r];
        for (int j = 0; j < 4; ++j) gb_J[t - 1][r][5 + j] = G.mL[r][j];
      }
      double a1 = Lt[0] - Lt[2], a2 = Lt[1] - Lt[3];
      gn_v[t - 1] = a1 * a1 + a2 * a2;
      gn_g[t - 1][0] = 2 * a1; gn_g[t - 1][1] = 2 * a2; gn_g[t - 1][2] = -2 * a1; gn_g[t - 1][3] = -2 * a2;
      double H[9][9];
      ga_hess(G, H);
      for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j) H[i][j] *= -ya[t - 1];
      H[3][3] -= yb[t - 1][0] * (-G.m[0]) + yb[t - 1][1] * (-G.m[1]);
      for (int j = 0; j < 4; ++j) {
        double hv = yb[t - 1][0] * G.mtL[0][j] + yb[t - 1][1] * G.mtL[1][j];
        H[3][5 + j] -= hv;
        H[5 + j][3] -= hv;
      }
      const double Hn[4][4] = {{2, 0, -2, 0}, {0, 2, 0, -2}, {-2, 0, 2, 0}, {0, -2, 0, 2}};
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) {
          double wd = 0.0;
          if (t < NH - 1 && i >= 2 && j >= 2) {
            const int fi[3] = {0, 1, 3};
            for (int f = 0; f < 3; ++f) wd += pi[t][fi[f]] * dyn[t].Hf[f][i - 2][j - 2];
            wd *= DT;
          }
          Wxx[t][i][j] = wd + (i == j ? 2 * p.qq + p.rho : 0.0) + H[i][j];
        }
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 4; ++j) Wxl[t][i][j] = H[i][5 + j];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Wll[t][i][j] = (i == j ? p.rho : 0.0) + H[5 + i][5 + j] - yn[t - 1] * Hn[i][j];
    }
    // condense
    double sv[NH][NX];
    for (int i = 0; i < 5; ++i) sv[0][i] = p.init[i] - X[0][i];
    for (int k = 0; k < NT; ++k) {
      for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NUV; ++j) {
          double s = 0.0;
          if (k > 0) for (int m = 0; m < NX; ++m) s += dyn[k].A[i][m] * K[k - 1][m][j];
          if (j == 2 * k && i == 2) s += DT;
          if (j == 2 * k + 1 && i == 4) s += DT;
          K[k][i][j] = s;
        }
      for (int i = 0; i < NX; ++i) {
        double s = 0.0;
        for (int m = 0; m < NX; ++m) s += dyn[k].A[i][m] * sv[k][m];
        sv[k + 1][i] = s + dyn[k].F[i] - X[k + 1][i];
      }
    }
    for (int ti = 0; ti < NT; ++ti) {
      double mth0 = gb_J[ti][0][3], mth1 = gb_J[ti][1][3], r0 = -gb_v[ti][0], r1 = -gb_v[ti][1], s3 = sv[ti + 1][3];
      for (int i = 0; i < 4; ++i) {
        Pm[ti][i][0] = 0.5 * gb_J[ti][0][5 + i];
        Pm[ti][i][1] = 0.5 * gb_J[ti][1][5 + i];
        double pm = Pm[ti][i][0] * mth0 + Pm[ti][i][1] * mth1;
        k0[ti][5 + i] = Pm[ti][i][0] * (r0 - mth0 * s3) + Pm[ti][i][1] * (r1 - mth1 * s3);
        for (int j = 0; j < NUV; ++j) K[ti][5 + i][j] = -pm * K[ti][3][j];
      }
      for (int i = 0; i < 5; ++i) k0[ti][i] = sv[ti + 1][i];
    }
    for (int a = 0; a < NZ; ++a) {
      for (int b = 0; b < NZ; ++b) Hq[a][b] = (a == b && a < NUV) ? 2 * p.rr : 0.0;
      gq[a] = a < NUV ? 2 * p.rr * (&U[0][0])[a] : 0.0;
    }
    for (int ti = 0; ti < NT; ++ti) {
      int t = ti + 1;
      double W[9][9], WK[9][NZ], v9[9];
      for (int i = 0; i < 9; ++i)
        for (int j = 0; j < 9; ++j)
          W[i][j] = (i < 5) ? (j < 5 ? Wxx[t][i][j] : Wxl[t][i][j - 5]) : (j < 5 ? Wxl[t][j][i - 5] : Wll[t][i - 5][j - 5]);
      for (int i = 0; i < 9; ++i) {
        for (int a = 0; a < NZ; ++a) { double s = 0; for (int j = 0; j < 9; ++j) s += W[i][j] * K[ti][j][a]; WK[i][a] = s; }
        double v = (i < 5) ? gX[t][i] : gL[ti][i - 5];
        for (int j = 0; j < 9; ++j) v += W[i][j] * k0[ti][j];
        v9[i] = v;
      }
      for (int a = 0; a < NZ; ++a) {
        for (int b = 0; b < NZ; ++b) { double s = 0; for (int i = 0; i < 9; ++i) s += K[ti][i][a] * WK[i][b]; Hq[a][b] += s; }
        double s = 0;
        for (int i = 0; i < 9; ++i) s += K[ti][i][a] * v9[i];
        gq[a] += s;
      }
    }
    for (int a = 0; a < NZ; ++a)
      for (int b = a + 1; b < NZ; ++b) { double v = 0.5 * (Hq[a][b] + Hq[b][a]); Hq[a][b] = Hq[b][a] = v; }
    // rows
    const double lo[5] = {0.0, -p.max_y, -MAX_V, -TWO_PI, -MAX_STEER};
    const double hi[5] = {p.max_x, p.max_y, MAX_V, TWO_PI, MAX_STEER};
    for (int ti = 0; ti < NT; ++ti) {
      int t = ti + 1;
      double* base = &C[ti * ROWS_T][0];
      double garow[NZ], gnrow[NZ];
      for (int a = 0; a < NZ; ++a) {
        double s = 0, g = 0;
        for (int i = 0; i < 9; ++i) s += ga_g[ti][i] * K[ti][i][a];
        for (int j = 0; j < 4; ++j) g += gn_g[ti][j] * K[ti][5 + j][a];
        garow[a] = s; gnrow[a] = g;
      }
      for (int j = 0; j < 5; ++j) {
        for (int a = 0; a < NZ; ++a) { base[(2 * j) * NZ + a] = K[ti][j][a]; base[(2 * j + 1) * NZ + a] = -K[ti][j][a]; }
        double b0 = X[t][j] + k0[ti][j];
        din[ti * ROWS_T + 2 * j] = lo[j] - b0;
        din[ti * ROWS_T + 2 * j + 1] = b0 - hi[j];
      }
      double gb0 = ga_v[ti], gn0 = gn_v[ti];
      for (int i = 0; i < 9; ++i) gb0 += ga_g[ti][i] * k0[ti][i];
      for (int j = 0; j < 4; ++j) gn0 += gn_g[ti][j] * k0[ti][5 + j];
      for (int a = 0; a < NZ; ++a) { base[10 * NZ + a] = garow[a]; base[11 * NZ + a] = -garow[a]; base[12 * NZ + a] = -gnrow[a]; }
      din[ti * ROWS_T + 10] = p.min_dis - gb0;
      din[ti * ROWS_T + 11] = gb0 - GA_MAX;
      din[ti * ROWS_T + 12] = gn0 - 1.0;
      for (int j = 0; j < 4; ++j) {
        for (int a = 0; a < NZ; ++a) { base[(13 + 2 * j) * NZ + a] = K[ti][5 + j][a]; base[(14 + 2 * j) * NZ + a] = -K[ti][5 + j][a]; }
        double b0 = L[ti][j] + k0[ti][5 + j];
        din[ti * ROWS_T + 13 + 2 * j] = -b0;
        din[ti * ROWS_T + 14 + 2 * j] = b0 - LAM_MAX;
      }
    }
    for (int j = 0; j < NUV; ++j) {
      int cI = ROWS_T * NT + 2 * j;
      for (int a = 0; a < NZ; ++a) { C[cI][a] = (a == j) ? 1.0 : 0.0; C[cI + 1][a] = (a == j) ? -1.0 : 0.0; }
      double lo_u = (j & 1) ? -MAX_STEER_RATE : -MAX_ACC, uj = (&U[0][0])[j];
      din[cI] = lo_u - uj;
      din[cI + 1] = uj + lo_u;
    }
    // Hessian modification
    std::memcpy(Hm, Hq, sizeof(Hm));
    bool pd = chol(Hm);
    if (!pd) {
      std::memcpy(H0, Hq, sizeof(H0));
      if (npact > 0) {
        std::memset(Ga, 0, sizeof(Ga));
        double gav[NZ] = {};
        for (int k = 0; k < npact; ++k) {
          const double* a = C[pact[k]];
          double nn = 0;
          for (int i = 0; i < NZ; ++i) nn += a[i] * a[i];
          double inv = 1.0 / std::fmax(std::sqrt(nn), 1e-300);
          for (int i = 0; i < NZ; ++i) gav[i] += (din[pact[k]] * inv) * (a[i] * inv);
          for (int i = 0; i < NZ; ++i)
            for (int j = 0; j < NZ; ++j) Ga[i][j] += (a[i] * inv) * (a[j] * inv);
        }
        double hmax = 0;
        for (int i = 0; i < NZ; ++i) hmax = std::fmax(hmax, std::fabs(Hq[i][i]));
        double sig = 1e-4 * hmax;
        for (int at = 0; at < 8; ++at) {
          for (int i = 0; i < NZ; ++i)
            for (int j = 0; j < NZ; ++j) H0[i][j] = Hq[i][j] + sig * Ga[i][j];
          std::memcpy(Hm, H0, sizeof(Hm));
          pd = chol(Hm);
          if (pd) break;
          sig *= 10.0;
        }
        if (!pd) sig /= 10.0;
        for (int i = 0; i < NZ; ++i) gq[i] -= sig * gav[i];
      }
      if (!pd) {
        double tau = 0.0;
        for (int at = 0; at < 16; ++at) {
          tau = (tau == 0.0) ? 1e-6 : tau * 10.0;
          std::memcpy(Hm, H0, sizeof(Hm));
          for (int i = 0; i < NZ; ++i) Hm[i][i] += tau * std::fmax(std::fabs(H0[i][i]), 1e-12);
          pd = chol(Hm);
          if (pd) break;
        }
        if (!pd) { status = 4; break; }
      }
    }
    int steps = 0, hit = 0;
    int qst = gi(Hm, gq, C, din, zq, uin, steps, pact, npact, hit);
    qp_total += steps;
    if (qst != 0) { status = (qst == 2) ? 2 : 1; break; }
    npact = 0;
    for (int cI = 0; cI < NROW; ++cI)
      if (uin[cI] > 0.0) pact[npact++] = cI;
    double dX[NH][NX], dU[NT][NU], dL[NT][NL];
    for (int j = 0; j < NUV; ++j) (&dU[0][0])[j] = zq[j];
    for (int i = 0; i < 5; ++i) dX[0][i] = sv[0][i];
    for (int ti = 0; ti < NT; ++ti)
      for (int i = 0; i < 9; ++i) {
        double s = k0[ti][i];
        for (int a = 0; a < NZ; ++a) s += K[ti][i][a] * zq[a];
        if (i < 5) dX[ti + 1][i] = s; else dL[ti][i - 5] = s;
      }
    for (int ti = 0; ti < NT; ++ti) {
      const double* ui = uin + ti * ROWS_T;
      for (int j = 0; j < NX; ++j) nyx[ti][j] = ui[2 * j] - ui[2 * j + 1];
      nya[ti] = ui[10] - ui[11];
      nyn[ti] = -ui[12];
      for (int j = 0; j < NL; ++j) nyl[ti][j] = ui[13 + 2 * j] - ui[14 + 2 * j];
    }
    for (int j = 0; j < NUV; ++j) nyu[j] = uin[ROWS_T * NT + 2 * j] - uin[ROWS_T * NT + 2 * j + 1];
    for (int ti = 0; ti < NT; ++ti) {
      int t = ti + 1;
      double resL[4];
      for (int i = 0; i < 4; ++i) {
        double s = gL[ti][i];
        for (int j = 0; j < 5; ++j) s += Wxl[t][j][i] * dX[t][j];
        for (int j = 0; j < 4; ++j) s += Wll[t][i][j] * dL[ti][j];
        s -= nya[ti] * ga_g[ti][5 + i] + nyn[ti] * gn_g[ti][i] + nyl[ti][i];
        resL[i] = s;
      }
      for (int r = 0; r < 2; ++r) { double s = 0; for (int i = 0; i < 4; ++i) s += Pm[ti][i][r] * resL[i]; nyb[ti][r] = s; }
    }
    for (int t = NH - 1; t >= 1; --t) {
      int ti = t - 1;
      for (int i = 0; i < 5; ++i) {
        double s = gX[t][i];
        for (int j = 0; j < 5; ++j) s += Wxx[t][i][j] * dX[t][j];
        for (int j = 0; j < 4; ++j) s += Wxl[t][i][j] * dL[ti][j];
        s -= nya[ti] * ga_g[ti][i] + nyb[ti][0] * gb_J[ti][0][i] + nyb[ti][1] * gb_J[ti][1][i] + nyx[ti][i];
        if (t < NH - 1) for (int j = 0; j < 5; ++j) s += dyn[t].A[j][i] * npi[t][j];
        npi[ti][i] = s;
      }
    }
    double f0, viol;
    cost_viol(p, X, U, L, f0, viol);
    double stp = 0.0;
    for (int e = 0; e < NH * NX; ++e) stp = std::fmax(stp, std::fabs((&dX[0][0])[e]));
    for (int e = 0; e < NUV; ++e) stp = std::fmax(stp, std::fabs((&dU[0][0])[e]));
    for (int e = 0; e < NT * NL; ++e) stp = std::fmax(stp, std::fabs((&dL[0][0])[e]));
    if (stp <= 1e-9 && viol <= 1e-9) {
      for (int e = 0; e < NH * NX; ++e) (&X[0][0])[e] += (&dX[0][0])[e];
      for (int e = 0; e < NUV; ++e) (&U[0][0])[e] += (&dU[0][0])[e];
      for (int e = 0; e < NT * NL; ++e) (&L[0][0])[e] += (&dL[0][0])[e];
      std::memcpy(ya, nya, sizeof(ya)); std::memcpy(yb, nyb, sizeof(yb)); std::memcpy(yn, nyn, sizeof(yn));
      std::memcpy(yx, nyx, sizeof(yx)); std::memcpy(pi, npi, sizeof(pi)); std::memcpy(yu, nyu, sizeof(yu));
      std::memcpy(yl, nyl, sizeof(yl));
      status = 0;
      break;
    }
    double mm = 0.0;
    for (int ti = 0; ti < NT; ++ti) {
      mm = std::fmax(mm, std::fmax(std::fmax(std::fabs(nya[ti]), std::fabs(nyn[ti])), std::fmax(std::fabs(nyb[ti][0]), std::fabs(nyb[ti][1]))));
      for (int j = 0; j < NX; ++j) mm = std::fmax(mm, std::fmax(std::fabs(nyx[ti][j]), std::fabs(npi[ti][j])));
    }
    mu = std::fmax(mu, 1.01 * mm + 1e-6);
    double phi0 = f0 + mu * viol, gd = 0.0;
    for (int t = 1; t < NH; ++t) for (int i = 0; i < 5; ++i) gd += gX[t][i] * dX[t][i];
    for (int j = 0; j < NUV; ++j) gd += 2 * p.rr * (&U[0][0])[j] * (&dU[0][0])[j];
    for (int e = 0; e < NT * NL; ++e) gd += (&gL[0][0])[e] * (&dL[0][0])[e];
    double D = gd - mu * viol, alpha = 1.0;
    bool ok = false;
    double Xn[NH][NX], Un[NT][NU], Ln[NT][NL];
    for (int at = 0; at <= 30; ++at) {
      for (int e = 0; e < NH * NX; ++e) (&Xn[0][0])[e] = (&X[0][0])[e] + alpha * (&dX[0][0])[e];
      for (int e = 0; e < NUV; ++e) (&Un[0][0])[e] = (&U[0][0])[e] + alpha * (&dU[0][0])[e];
      for (int e = 0; e < NT * NL; ++e) (&Ln[0][0])[e] = (&L[0][0])[e] + alpha * (&dL[0][0])[e];
      double fn, vn;
      cost_viol(p, Xn, Un, Ln, fn, vn);
      if (fn + mu * vn <= phi0 + 1e-4 * alpha * D) { ok = true; break; }
      alpha *= 0.5;
    }
    if (!ok) { status = 3; break; }
    std::memcpy(X, Xn, sizeof(X)); std::memcpy(U, Un, sizeof(U)); std::memcpy(L, Ln, sizeof(L));
    for (int ti = 0; ti < NT; ++ti) {
      ya[ti] += alpha * (nya[ti] - ya[ti]);
      yn[ti] += alpha * (nyn[ti] - yn[ti]);
      for (int r = 0; r < 2; ++r) yb[ti][r] += alpha * (nyb[ti][r] - yb[ti][r]);
      for (int j = 0; j < NX; ++j) { yx[ti][j] += alpha * (nyx[ti][j] - yx[ti][j]); pi[ti][j] += alpha * (npi[ti][j] - pi[ti][j]); }
      for (int j = 0; j < NL; ++j) yl[ti][j] += alpha * (nyl[ti][j] - yl[ti][j]);
    }
    for (int j = 0; j < NUV; ++j) yu[j] += alpha * (nyu[j] - yu[j]);
  }
  double fc, vc;
  cost_viol(p, X, U, L, fc, vc);
  std::memcpy(o, X, 40 * sizeof(double));
  std::memcpy(o + 40, U, 14 * sizeof(double));
  std::memcpy(o + 54, L, 28 * sizeof(double));
  for (int ti = 0; ti < NT; ++ti) { o[82 + ti] = ya[ti]; o[89 + 2 * ti] = yb[ti][0]; o[90 + 2 * ti] = yb[ti][1]; o[103 + ti] = yn[ti]; }
  std::memcpy(o + 110, yx, 35 * sizeof(double));
  std::memcpy(o + 145, pi, 35 * sizeof(double));
  std::memcpy(o + 180, yu, 14 * sizeof(double));
  std::memcpy(o + 194, yl, 28 * sizeof(double));
  o[222] = fc;
  o[223] = 0.0;
  ist[0] = status;
  ist[1] = (it < p.max_iter) ? it + 1 : p.max_iter;
  ist[2] = qp_total;
}

}  // namespace

extern "C" int obca_cpu_solve(const double* recs, int n, double* out, int* ist, int threads) {
  if (n <= 0) return 0;
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads > 0 ? threads : 1)
  for (int i = 0; i < n; ++i) solve_one(recs + (size_t)i * REC, out + (size_t)i * OUT, ist + (size_t)i * 3);
  return 0;
}
