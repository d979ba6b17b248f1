// B-opt CPU baseline of the PI-ADMM hot path -- C++, OpenMP over connected components.
//
// MEASUREMENT / TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/ load it (through
// oracle/cpu_bopt.py); the product path (libpiadmm.so, include/piadmm.h) never does.
//
// What it computes: the loop of oracle/piadmm_oracle.py (the NumPy restatement of
// casadi/main.py:43-201 with the MATLAB PI anti-windup law, ADMM_CVX_..._PI_antiwindup.m:152-188)
// on any static candidate graph -- the tiled intersection of the benchmark (components of two
// agents), the 4-vehicle all-pairs crossings, chains -- with the same semantics flags (dual mode
// plain / PI, windup, rounding, B2 threshold, B4 aliasing, B15 position model, MATLAB distance
// stop, fixed iterations, delay tightening, warm duals (a12), no collision gate, per-component or
// global termination).  Every QP answer is the exact minimiser, so the results equal the
// oracle's (tests/test_cpu_bopt.py, 1e-8).  Not covered: the global-PI law (dual mode 2).
//
// How (SURVEY.md 8d "B-opt": same algorithm as the GPU kernel, -O3, OpenMP, all cores given):
//   * x-step QP (casadi/PI_ADMM_class.py:114-135,172-192): P depends on the speed only, so each
//     agent keeps P^-1 and the Cholesky factor of its last working set's Schur complement
//     S = N P^-1 N' with Y = P^-1 N'.  A solve first tries that working set (x0 = -P^-1 q,
//     u = S^-1 (b - N x0), x = x0 + Y u, certified by primal feasibility and dual signs: the
//     GPU's parametric "hit"), else runs the Goldfarb-Idnani dual active set warm-started from
//     it (the GPU's x-step GI).
//   * pair QP (PI_ADMM_class.py:145-169, heading frozen, quirk B3): the same dual active set
//     with the safety hinge beta*max(0, h - a'x) as a row with a bounded multiplier u in
//     [0, beta] (a row whose multiplier reaches beta turns linear and is watched from the
//     other side of its kink), warm-started from the pair's previous active set shifted one slot.
//   * rollouts, collision test, dual update, residuals, propagation in the oracle's operation
//     order (the functions of oracle/piadmm_oracle.py it follows are named at each one).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

#include <omp.h>
#ifdef BOPT_DEBUG
#include <cstdio>
#define DBG(...) std::fprintf(stderr, __VA_ARGS__)
#else
#define DBG(...) ((void)0)
#endif

namespace {

struct CpuCfg {          // mirror: oracle/cpu_bopt.py _Cfg
  int H, max_outer, dual_mode, windup, round_decimals, collide_sq_thres, alias_dual_residual,
      pos_model, term_dist_check, fixed_iters, term_global, tighten, warm_duals, no_collision_gate;
  double dt, L, dis_thres, beta, Pnorm, Pcost, rho, eps_pri, eps_dual, u_max, du_max, kI,
      theta1, theta2, windup_sat, tight_p, avg_delay, var_delay, qp_tol;
};

constexpr double DEP_TOL = 1e-10;     // linear dependence of an entering row (as pd_qp.h)
constexpr int GI_MAX_STEPS = 4096;

double around(double x, int dec) {    // np.around(x, dec): rint(x * 10^dec) / 10^dec
  if (dec < 0) return x;
  const double s = std::pow(10.0, dec);
  return std::nearbyint(x * s) / s;
}

// ---------------------------------------------------------------- rollouts (piadmm_oracle.py)
void rollout_linear(const double* xt, const double* u, double s, double dt, double L, int H, double* x, double* y) {
  double th = xt[2];
  x[0] = xt[0];
  y[0] = xt[1];
  const double s0 = std::sin(xt[2]), c0 = std::cos(xt[2]);
  for (int k = 0; k < H; ++k) {
    const double xd = -s * s0 * th + (s * c0 + s * xt[2] * s0);
    x[k + 1] = x[k] + xd * dt;
    const double yd = s * c0 * th + (s * s0 - s * xt[2] * c0);
    y[k + 1] = y[k] + yd * dt;
    th = th + (s / L * u[k]) * dt;
  }
}

void rollout_nonlinear(const double* xt, const double* u, double s, double dt, double L, int H, double* x,
                       double* y, double* thout = nullptr) {
  double th = xt[2];
  x[0] = xt[0];
  y[0] = xt[1];
  for (int k = 0; k < H; ++k) {
    const double sk = std::sin(th), ck = std::cos(th);
    const double xd = -s * sk * th + (s * ck + s * th * sk);
    x[k + 1] = x[k] + xd * dt;
    const double yd = s * ck * th + (s * sk - s * th * ck);
    y[k + 1] = y[k] + yd * dt;
    th = th + (s / L * u[k]) * dt;
    if (thout && k == 0) *thout = th;
  }
}

// rollout_affine: p = c + M u of the linearised rollout; c (2, H+1), M (2, H+1, H) row-major
void rollout_affine(const double* xt, double s, double dt, double L, int H, double* c, double* M) {
  const int R = H + 1;
  std::fill(M, M + 2 * R * H, 0.0);
  c[0] = xt[0];
  c[R] = xt[1];
  const double s0 = std::sin(xt[2]), c0 = std::cos(xt[2]), thc = xt[2];
  const double kx = -s * s0 * dt, ky = s * c0 * dt, tm = s / L * dt;
  for (int k = 0; k < H; ++k) {
    c[k + 1] = c[k] + (-s * s0 * thc + (s * c0 + s * xt[2] * s0)) * dt;
    c[R + k + 1] = c[R + k] + (s * c0 * thc + (s * s0 - s * xt[2] * c0)) * dt;
    for (int j = 0; j < H; ++j) {
      const double thm = (j < k) ? tm : 0.0;
      M[(k + 1) * H + j] = M[k * H + j] + kx * thm;
      M[(R + k + 1) * H + j] = M[(R + k) * H + j] + ky * thm;
    }
  }
}

// symmetric positive definite inverse by Cholesky (n <= 128)
bool spd_inverse(const double* A, int n, double* Ainv) {
  std::vector<double> Lc(n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    double d = A[j * n + j];
    for (int k = 0; k < j; ++k) d -= Lc[j * n + k] * Lc[j * n + k];
    if (!(d > 0.0)) return false;
    const double ljj = std::sqrt(d);
    Lc[j * n + j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double v = A[i * n + j];
      for (int k = 0; k < j; ++k) v -= Lc[i * n + k] * Lc[j * n + k];
      Lc[i * n + j] = v / ljj;
    }
  }
  // L^-1 (lower), then A^-1 = L^-T L^-1
  std::vector<double> Li(n * n, 0.0);
  for (int j = 0; j < n; ++j) {
    Li[j * n + j] = 1.0 / Lc[j * n + j];
    for (int i = j + 1; i < n; ++i) {
      double v = 0.0;
      for (int k = j; k < i; ++k) v -= Lc[i * n + k] * Li[k * n + j];
      Li[i * n + j] = v / Lc[i * n + i];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double v = 0.0;
      for (int k = i; k < n; ++k) v += Li[k * n + i] * Li[k * n + j];
      Ainv[i * n + j] = Ainv[j * n + i] = v;
    }
  return true;
}

// ---------------------------------------------------------------- QP with box / rate / hinge rows
// min 1/2 x'Px + q'x + beta sum_k max(0, h_k - G_k x)  s.t.  |x_vk| <= umax, |x_v(k+1) - x_vk| <= dumax
// Rows: vehicle v < NV: box k (H), rate k (H-1); then hinge k (H, NV == 2 only).
// One-sided constraint code c = 2 row + side: side 0 a'x >= lo, side 1 -a'x >= -hi
// (for a hinge row, side 1 is the linear regime's a'x <= h).
struct QPDef {
  int n = 0, H = 0, NV = 1;
  const double* Pinv = nullptr;    // n x n
  const double* q = nullptr;       // n
  const double* G = nullptr;       // H x n hinge normals
  const double* h = nullptr;       // H hinge thresholds
  double umax = 0, dumax = 0, beta = 0, tol = 1e-9;
  int nbr() const { return 2 * H - 1; }
  int nrows() const { return NV * nbr() + (NV == 2 ? H : 0); }
  bool hinge(int r) const { return r >= NV * nbr(); }
  double lo(int r) const {
    if (hinge(r)) return h[r - NV * nbr()];
    return (r % nbr() < H) ? -umax : -dumax;
  }
  double hi(int r) const {
    if (hinge(r)) return h[r - NV * nbr()];
    return (r % nbr() < H) ? umax : dumax;
  }
  double adot(int r, const double* x) const {
    if (hinge(r)) {
      const double* g = G + (size_t)(r - NV * nbr()) * n;
      double v = 0.0;
      for (int i = 0; i < n; ++i) v += g[i] * x[i];
      return v;
    }
    const int v = r / nbr(), j = r % nbr();
    if (j < H) return x[v * H + j];
    const int k = j - H;
    return x[v * H + k + 1] - x[v * H + k];
  }
  // out = sg * P^-1 a_r
  void pinv_col(int r, double sg, double* out) const {
    if (hinge(r)) {
      const double* g = G + (size_t)(r - NV * nbr()) * n;
      for (int i = 0; i < n; ++i) {
        double v = 0.0;
        const double* pr = Pinv + (size_t)i * n;
        for (int j = 0; j < n; ++j) v += pr[j] * g[j];
        out[i] = sg * v;
      }
      return;
    }
    const int v = r / nbr(), j = r % nbr();
    if (j < H) {
      const double* pc = Pinv + (size_t)(v * H + j) * n;
      for (int i = 0; i < n; ++i) out[i] = sg * pc[i];
      return;
    }
    const int k = j - H;
    const double* p1 = Pinv + (size_t)(v * H + k + 1) * n;
    const double* p0 = Pinv + (size_t)(v * H + k) * n;
    for (int i = 0; i < n; ++i) out[i] = sg * (p1[i] - p0[i]);
  }
  double ndot(int c, const double* x) const { return (c & 1) ? -adot(c >> 1, x) : adot(c >> 1, x); }
  double bnd(int c) const { return (c & 1) ? -hi(c >> 1) : lo(c >> 1); }
};

// Dual active set state: Cholesky factor L of S = N P^-1 N' (insertion order), Y = P^-1 N'.
struct ActiveSet {
  int n = 0, cap = 0, m = 0;
  std::vector<double> L, Y, u;
  std::vector<int> codes;
  void init(int n_, int cap_) {
    n = n_;
    cap = cap_;
    m = 0;
    L.assign((size_t)cap * cap, 0.0);
    Y.assign((size_t)cap * n, 0.0);
    u.assign(cap, 0.0);
    codes.assign(cap, -1);
  }
  void fwd(const double* b, double* w) const {      // L w = b
    for (int i = 0; i < m; ++i) {
      double v = b[i];
      const double* li = &L[(size_t)i * cap];
      for (int k = 0; k < i; ++k) v -= li[k] * w[k];
      w[i] = v / li[i];
    }
  }
  void bwd(const double* w, double* r) const {      // L' r = w
    for (int i = m - 1; i >= 0; --i) {
      double v = w[i];
      for (int k = i + 1; k < m; ++k) v -= L[(size_t)k * cap + i] * r[k];
      r[i] = v / L[(size_t)i * cap + i];
    }
  }
  void append(int pc, const double* yp, const double* w, double lpp2, double u0) {
    double* lm = &L[(size_t)m * cap];
    for (int k = 0; k < m; ++k) lm[k] = w[k];
    lm[m] = std::sqrt(lpp2);
    std::memcpy(&Y[(size_t)m * n], yp, sizeof(double) * n);
    codes[m] = pc;
    u[m] = u0;
    ++m;
  }
  void drop(int k) {
    // rank-one update of the trailing block with the deleted column, then compact
    std::vector<double> xv(m, 0.0);
    for (int i = k + 1; i < m; ++i) xv[i] = L[(size_t)i * cap + k];
    for (int j = k + 1; j < m; ++j) {
      const double Ljj = L[(size_t)j * cap + j], xj = xv[j];
      const double rr = std::sqrt(Ljj * Ljj + xj * xj);
      const double cc = rr / Ljj, sn = xj / Ljj;
      L[(size_t)j * cap + j] = rr;
      for (int i = j + 1; i < m; ++i) {
        const double Lij = (L[(size_t)i * cap + j] + sn * xv[i]) / cc;
        xv[i] = cc * xv[i] - sn * Lij;
        L[(size_t)i * cap + j] = Lij;
      }
    }
    for (int i = k; i < m - 1; ++i) {
      double* dst = &L[(size_t)i * cap];
      const double* src = &L[(size_t)(i + 1) * cap];
      for (int j = 0; j < k; ++j) dst[j] = src[j];
      for (int j = k; j <= i; ++j) dst[j] = src[j + 1];
      std::memcpy(&Y[(size_t)i * n], &Y[(size_t)(i + 1) * n], sizeof(double) * n);
      codes[i] = codes[i + 1];
      u[i] = u[i + 1];
    }
    --m;
  }
};

struct Work {             // per-thread scratch
  std::vector<double> x0, x, yp, z, na, w, r, tmp, lin_dummy;
  void ensure(int n) {
    if ((int)x0.size() >= 2 * n + 8) return;
    const int s = 2 * n + 8;
    for (auto* v : {&x0, &x, &yp, &z, &na, &w, &r, &tmp}) v->assign(s, 0.0);
  }
};

// u = S^-1 (b - N xb) on the active set
void eqp_u(const QPDef& Q, const ActiveSet& A, const double* xb, Work& W, double* uo) {
  for (int a = 0; a < A.m; ++a) W.na[a] = Q.bnd(A.codes[a]) - Q.ndot(A.codes[a], xb);
  A.fwd(W.na.data(), W.w.data());
  A.bwd(W.w.data(), uo);
}

// x = x0 + Y u, then one step of primal refinement on the active rows' residual
void final_x(const QPDef& Q, ActiveSet& A, Work& W, double* x) {
  const int n = Q.n;
  std::vector<double>& uu = W.r;
  eqp_u(Q, A, W.x0.data(), W, uu.data());
  for (int i = 0; i < n; ++i) x[i] = W.x0[i];
  for (int a = 0; a < A.m; ++a) {
    const double* ya = &A.Y[(size_t)a * n];
    for (int i = 0; i < n; ++i) x[i] += uu[a] * ya[i];
  }
  for (int a = 0; a < A.m; ++a) A.u[a] = uu[a];
  eqp_u(Q, A, x, W, W.tmp.data());
  for (int a = 0; a < A.m; ++a) {
    const double d = W.tmp[a];
    const double* ya = &A.Y[(size_t)a * n];
    for (int i = 0; i < n; ++i) x[i] += d * ya[i];
    A.u[a] += d;
  }
}

// KKT certificate of x with the active set's multipliers (signs, caps, primal feasibility)
bool certify(const QPDef& Q, const ActiveSet& A, const double* x, const char* lin) {
  const int R = Q.nrows();
  double umax = 0.0;
  for (int a = 0; a < A.m; ++a) umax = std::max(umax, std::fabs(A.u[a]));
  const double dtol = 1e-9 * (1.0 + umax);
  for (int a = 0; a < A.m; ++a) {
    if (A.u[a] < -dtol) return false;
    if (Q.hinge(A.codes[a] >> 1) && A.u[a] > Q.beta + dtol) return false;
  }
  for (int r = 0; r < R; ++r) {
    const double ax = Q.adot(r, x);
    const double tp = 1e-8 * (1.0 + std::fabs(Q.lo(r)));
    if (Q.hinge(r)) {
      const int k = r - Q.NV * Q.nbr();
      bool held = false;
      for (int a = 0; a < A.m; ++a) held |= (A.codes[a] >> 1) == r;
      if (held) continue;
      if (lin[k] ? (ax > Q.h[k] + tp) : (ax < Q.h[k] - tp)) return false;
    } else if (ax < Q.lo(r) - tp || ax > Q.hi(r) + tp) {
      return false;
    }
  }
  return true;
}

// Goldfarb-Idnani dual active set with bounded hinge multipliers (pd_qp.h gi_solve).
// The active set A holds the warm rows on entry (codes only; rebuilt here).  lin[k]: hinge row k
// in its linear regime (in/out).  Returns false on failure (step limit, unbounded dual step).
bool gi_solve(const QPDef& Q, ActiveSet& A, const int* warm, int nwarm, char* lin, Work& W, double* xout,
              long long& steps) {
  const int n = Q.n, R = Q.nrows(), nb = Q.NV * Q.nbr();
  W.ensure(n);
  double* x0 = W.x0.data();
  double* x = W.x.data();
  double* yp = W.yp.data();
  double* z = W.z.data();
  double* w = W.w.data();
  double* r = W.r.data();
  int nsteps = 0;
  // x0 = -P^-1 (q - beta sum_{linear hinge} G_k)
  {
    std::vector<double>& qt = W.tmp;
    for (int i = 0; i < n; ++i) qt[i] = Q.q[i];
    if (Q.NV == 2)
      for (int k = 0; k < Q.H; ++k)
        if (lin[k])
          for (int i = 0; i < n; ++i) qt[i] -= Q.beta * Q.G[(size_t)k * n + i];
    for (int i = 0; i < n; ++i) {
      double v = 0.0;
      const double* pr = Q.Pinv + (size_t)i * n;
      for (int j = 0; j < n; ++j) v += pr[j] * qt[j];
      x0[i] = -v;
    }
  }
  A.m = 0;
  thread_local std::vector<char> inA;
  inA.assign(2 * R, 0);
  auto prep = [&](int pc) -> double {
    Q.pinv_col(pc >> 1, (pc & 1) ? -1.0 : 1.0, yp);
    return Q.ndot(pc, yp);
  };
  auto fwd_np = [&]() {
    for (int a = 0; a < A.m; ++a) W.na[a] = Q.ndot(A.codes[a], yp);
    A.fwd(W.na.data(), w);
  };
  auto drop = [&](int k) {
    inA[A.codes[k]] = 0;
    A.drop(k);
  };
  // warm rows: appended unless dependent, then dropped until dual feasible
  for (int i = 0; i < nwarm; ++i) {
    const int pc = warm[i];
    if (A.m >= A.cap || pc < 0 || inA[pc] || inA[pc ^ 1]) continue;
    const double spp = prep(pc);
    if (!(spp > 0.0)) continue;
    fwd_np();
    double ww = 0.0;
    for (int a = 0; a < A.m; ++a) ww += w[a] * w[a];
    const double lpp2 = spp - ww;
    if (lpp2 > DEP_TOL * spp) {
      A.append(pc, yp, w, lpp2, 0.0);
      inA[pc] = 1;
    }
  }
  while (A.m > 0) {
    eqp_u(Q, A, x0, W, r);
    double smin = 0.0;
    int k = -1;
    for (int a = 0; a < A.m; ++a) {
      double sc = 0.0;
      if (r[a] < 0.0) sc = r[a];
      else if (Q.hinge(A.codes[a] >> 1) && r[a] > Q.beta) sc = Q.beta - r[a];
      if (sc < smin) { smin = sc; k = a; }
    }
    if (k < 0) break;
    drop(k);
  }
  if (A.m > 0) eqp_u(Q, A, x0, W, r);
  for (int i = 0; i < n; ++i) x[i] = x0[i];
  for (int a = 0; a < A.m; ++a) {
    A.u[a] = r[a];
    const double* ya = &A.Y[(size_t)a * n];
    for (int i = 0; i < n; ++i) x[i] += r[a] * ya[i];
  }

  while (true) {
    // most violated constraint outside the active set
    double best = 0.0;
    int pc = -1;
    for (int row = 0; row < R; ++row) {
      const bool hg = row >= nb;
      const double ax = Q.adot(row, x);
      const double lo = Q.lo(row);
      const double tp = Q.tol * (1.0 + std::fabs(lo));
      const bool hl = hg && lin[row - nb];
      if (!hl && !inA[2 * row]) {
        const double sv = ax - lo;
        if (sv < -tp && sv < best) { best = sv; pc = 2 * row; }
      }
      if ((hl || !hg) && !inA[2 * row + 1]) {
        const double sv = (hl ? lo : Q.hi(row)) - ax;
        if (sv < -tp && sv < best) { best = sv; pc = 2 * row + 1; }
      }
    }
    if (pc < 0) break;
    const int prow = pc >> 1, pside = pc & 1;
    const bool phinge = prow >= nb;
    double sp = best;
    const double spp = prep(pc);
    double up = 0.0;
    while (true) {
      ++steps;
      if (++nsteps > GI_MAX_STEPS) { DBG("step limit m=%d\n", A.m); return false; }
      fwd_np();
      A.bwd(w, r);
      double ww = 0.0;
      for (int a = 0; a < A.m; ++a) ww += w[a] * w[a];
      for (int i = 0; i < n; ++i) z[i] = yp[i];
      for (int a = 0; a < A.m; ++a) {
        const double* ya = &A.Y[(size_t)a * n];
        for (int i = 0; i < n; ++i) z[i] -= r[a] * ya[i];
      }
      const double lpp2 = spp - ww;
      const double t2 = (lpp2 > DEP_TOL * spp) ? -sp / lpp2 : INFINITY;
      double t1 = INFINITY, tca = INFINITY;
      int k1 = -1, kc = -1;
      for (int a = 0; a < A.m; ++a) {
        if (r[a] > 0.0) {
          const double t = A.u[a] / r[a];
          if (t < t1) { t1 = t; k1 = a; }
        } else if (r[a] < 0.0 && Q.hinge(A.codes[a] >> 1)) {
          const double t = (Q.beta - A.u[a]) / (-r[a]);
          if (t < tca) { tca = t; kc = a; }
        }
      }
      const double tc = std::min(tca, phinge ? Q.beta - up : INFINITY);
      const double t = std::min(t1, t2);
      if (tc <= t) {
        const bool entering = phinge && Q.beta - up <= tca;
        if (t2 < INFINITY) {
          for (int i = 0; i < n; ++i) x[i] += tc * z[i];
          sp += tc * lpp2;
        }
        for (int a = 0; a < A.m; ++a) A.u[a] -= tc * r[a];
        up += tc;
        if (entering) {
          lin[prow - nb] = pside == 0;
          for (int i = 0; i < n; ++i) x0[i] += Q.beta * yp[i];
          break;
        }
        const int kcode = A.codes[kc];
        lin[(kcode >> 1) - nb] = (kcode & 1) == 0;
        const double* yk = &A.Y[(size_t)kc * n];
        for (int i = 0; i < n; ++i) x0[i] += Q.beta * yk[i];
        drop(kc);
        continue;
      }
      if (!(t < INFINITY)) { DBG("unbounded m=%d lpp2=%g spp=%g\n", A.m, lpp2, spp); return false; }
      if (t2 < INFINITY) {
        for (int i = 0; i < n; ++i) x[i] += t * z[i];
        sp += t * lpp2;
      }
      for (int a = 0; a < A.m; ++a) A.u[a] -= t * r[a];
      up += t;
      if (t2 <= t1) {
        if (A.m >= A.cap) { DBG("full m=%d\n", A.m); return false; }
        A.append(pc, yp, w, lpp2, up);
        inA[pc] = 1;
        break;
      }
      drop(k1);
    }
  }
  final_x(Q, A, W, xout);
  return true;
}

// ---------------------------------------------------------------- agents, pairs, components
// Any static candidate graph (the reference's num_veh loop, casadi/main.py:81,110-162): an agent's
// x-step sums the consensus term over its candidate neighbours in neighbour order
// (PI_ADMM_class.py:126-129; oracle xstep_qp), every candidate pair is collision-tested and, when
// it collides, gets its pair QP, hat rollouts and dual update in pair order; a connected component
// is one termination group (or the whole job under term_global) -- the oracle's Oracle.mpc_step.
struct Agent {
  double spd;
  double xt[3], seeds[2];
  std::vector<double> Pinv;       // H x H (speed and neighbour count only: fixed for the run)
  ActiveSet ws;                   // cached working set + factor (valid: P and rows are fixed)
  bool factor_ok = false;
  std::vector<double> u, px, py;  // primal_u, pos_old
  std::vector<std::pair<int, int>> nbr;   // (pair, direction), sorted by neighbour id
};

struct Pair {
  int v[2];
  std::vector<double> hat, lam, S, D, last;     // [d][2][H+1]
  double d_eff;
  std::vector<double> Ppinv;      // 2H x 2H block diagonal P^-1
  std::vector<int> pws;           // pair's last active set (codes)
  int pws_t = -1000;
  bool active, seen;
  double dis_chk, rk, sk;
};

struct Comp {
  std::vector<int> agents, pairs;
  bool flag, alias, done;
  int iters;
  double part[5];
  std::vector<double> resid;      // per iteration (rk, sk) of this step
};

struct World {
  std::vector<Agent> ag;
  std::vector<Pair> pr;
  std::vector<Comp> comps;
};

struct Run {
  CpuCfg c;
  int H;
  long long x_qps = 0, z_qps = 0, x_hits = 0, gi_steps = 0, inexact = 0;
};

void agent_P(const CpuCfg& c, double s, int nN, std::vector<double>& Pinv) {
  const int H = c.H, R2 = 2 * (H + 1);
  std::vector<double> cc(R2), M(R2 * H), P(H * H, 0.0);
  const double xt[3] = {0.0, 0.0, 0.0};
  rollout_affine(xt, s, c.dt, c.L, H, cc.data(), M.data());   // M'M is heading-independent
  const double coef = 2.0 * c.Pnorm + c.rho * nN;
  for (int i = 0; i < H; ++i)
    for (int j = 0; j < H; ++j) {
      double v = 0.0;
      for (int r = 0; r < R2; ++r) v += M[r * H + i] * M[r * H + j];
      P[i * H + j] = coef * v;
    }
  for (int k = 0; k < H - 2; ++k) {      // 2 D2'D2
    const int idx[3] = {k, k + 1, k + 2};
    const double cf[3] = {1.0, -2.0, 1.0};
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) P[idx[a] * H + idx[b]] += 2.0 * cf[a] * cf[b];
  }
  for (int i = 0; i < H; ++i) P[i * H + i] += 2.0 * c.Pcost;
  Pinv.assign(H * H, 0.0);
  spd_inverse(P.data(), H, Pinv.data());
}

void pair_P(const CpuCfg& c, double s1, double s2, std::vector<double>& Pinv) {
  const int H = c.H, n = 2 * H, R2 = 2 * (H + 1);
  Pinv.assign(n * n, 0.0);
  for (int v = 0; v < 2; ++v) {
    std::vector<double> cc(R2), M(R2 * H), P(H * H), Pi(H * H);
    const double xt[3] = {0.0, 0.0, 0.0};
    rollout_affine(xt, v ? s2 : s1, c.dt, c.L, H, cc.data(), M.data());
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < H; ++j) {
        double a = 0.0;
        for (int r = 0; r < R2; ++r) a += M[r * H + i] * M[r * H + j];
        P[i * H + j] = c.rho * a + (i == j ? 2.0 * c.Pcost : 0.0);
      }
    spd_inverse(P.data(), H, Pi.data());
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < H; ++j) Pinv[(v * H + i) * n + v * H + j] = Pi[i * H + j];
  }
}

double delay_norm(const CpuCfg& c, const double* xt, double s) {
  const double th = xt[2];
  const double dxa = c.avg_delay * s * std::cos(th), dya = c.avg_delay * s * std::sin(th);
  const double dxv = (c.var_delay * s * std::cos(th)) * (c.var_delay * s * std::cos(th));
  const double dyv = (c.var_delay * s * std::sin(th)) * (c.var_delay * s * std::sin(th));
  const double kap = std::sqrt(c.tight_p / (1.0 - c.tight_p));
  return std::hypot(dxa + kap * dxv, dya + kap * dyv);
}

struct Ctx {
  const CpuCfg& c;
  const double* ref;     // (N, 2, T)
  int T;
  Run& run;
  int t;                 // MPC step (reference slice t .. t+H)
  int it = 0;            // outer iteration (near-tie log)
};

// ---------------------------------------------------------------- near-tie log
// The mirror of piadmm_get_near_ties (include/piadmm.h, oracle TieLog): the reference's discrete
// decisions taken within g_tie_tol of their threshold.  Rare: one critical section per event.
enum { TIE_ROUND_U = 0, TIE_ROUND_UHAT, TIE_ROUND_SEED, TIE_COLLIDE, TIE_STOP, TIE_DIST, TIE_KINDS };
double g_tie_tol = 1e-9;
std::vector<int> g_tie_ev;          // 6 ints per event: step, iter, kind, id, index, 0
std::vector<double> g_tie_mg;
long long g_tie_cnt[TIE_KINDS] = {};

void tie_add(int t, int it, int kind, int id, int idx, double m) {
#pragma omp critical(piadmm_ties)
  {
    ++g_tie_cnt[kind];
    if (g_tie_mg.size() < 4096) {
      const int e[6] = {t, it, kind, id, idx, 0};
      g_tie_ev.insert(g_tie_ev.end(), e, e + 6);
      g_tie_mg.push_back(m);
    }
  }
}
void tie_round(const CpuCfg& c, int t, int it, int kind, int id, int idx, double x) {
  if (c.round_decimals < 0) return;
  double f = 1.0;
  for (int i = 0; i < c.round_decimals; ++i) f *= 10.0;
  const double y = x * f, b = std::floor(y) + 0.5;
  if (std::fabs(y - b) <= g_tie_tol * f) tie_add(t, it, kind, id, idx, (y - b) / f);
}
void tie_scalar(int t, int it, int kind, int id, int idx, double v, double thr) {
  if (std::fabs(v - thr) <= g_tie_tol * std::fabs(thr)) tie_add(t, it, kind, id, idx, (v - thr) / thr);
}

// x-step of agent a (casadi/main.py:81-106; oracle xstep_qp / solve_xstep)
void x_step(Ctx& X, World& Wd, int a, Work& W) {
  const CpuCfg& c = X.c;
  const int H = c.H, R = H + 1;
  Agent& A = Wd.ag[a];
  W.ensure(2 * H);
  // constant part c of the linearised rollout (rollout_affine) and q = M'v through the rollout
  // matrix's structure M_a(t, j) = k_a tm (t-1-j)_+ (two reverse running sums, as the kernel's
  // prefix scans) instead of the dense M
  thread_local std::vector<double> buf;
  buf.resize(6 * R + 2 * H);
  double* cc = buf.data();            // 2R
  double* vv = cc + 2 * R;            // 2R
  double* q = vv + 2 * R;             // H
  double* x = q + H;                  // H
  const double* xt = A.xt;
  const double s = A.spd, s0 = std::sin(xt[2]), c0 = std::cos(xt[2]);
  const double kx = -s * s0 * c.dt, ky = s * c0 * c.dt, tm = s / c.L * c.dt;
  cc[0] = xt[0];
  cc[R] = xt[1];
  for (int k = 0; k < H; ++k) {
    cc[k + 1] = cc[k] + (-s * s0 * xt[2] + (s * c0 + s * xt[2] * s0)) * c.dt;
    cc[R + k + 1] = cc[R + k] + (s * c0 * xt[2] + (s * s0 - s * xt[2] * c0)) * c.dt;
  }
  const double* ref = X.ref + (size_t)a * 2 * X.T;
  for (int ax = 0; ax < 2; ++ax)
    for (int k = 0; k < R; ++k) {
      const int i = ax * R + k;
      vv[i] = 2.0 * c.Pnorm * (cc[i] - ref[(size_t)ax * X.T + X.t + k]);
    }
  for (const auto& nd : A.nbr) {         // neighbour order (oracle: v = v + rho (c - hat + lam))
    const Pair& p = Wd.pr[nd.first];
    const double* hat = &p.hat[(size_t)nd.second * 2 * R];
    const double* lam = &p.lam[(size_t)nd.second * 2 * R];
    for (int i = 0; i < 2 * R; ++i) vv[i] = vv[i] + c.rho * (cc[i] - hat[i] + lam[i]);
  }
  {
    double ax = 0.0, ay = 0.0, bx = 0.0, by = 0.0;   // sums over t >= j + 2
    for (int j = H - 1; j >= 0; --j) {
      if (j + 2 <= H) {
        ax += vv[j + 2];
        ay += vv[R + j + 2];
      }
      bx += ax;
      by += ay;
      q[j] = tm * (kx * bx + ky * by);
    }
  }
  QPDef Q;
  Q.n = H;
  Q.H = H;
  Q.NV = 1;
  Q.Pinv = A.Pinv.data();
  Q.q = q;
  Q.umax = c.u_max;
  Q.dumax = c.du_max;
  Q.tol = c.qp_tol;
  ++X.run.x_qps;
  bool ok = false;
  char lin_none[1] = {0};
  if (A.factor_ok) {                     // the cached working set (the GPU's parametric hit)
    for (int i = 0; i < H; ++i) {
      double sm = 0.0;
      const double* pr = &A.Pinv[(size_t)i * H];
      for (int j = 0; j < H; ++j) sm += pr[j] * q[j];
      W.x0[i] = -sm;
    }
    final_x(Q, A.ws, W, x);
    ok = certify(Q, A.ws, x, lin_none);
    if (ok) ++X.run.x_hits;
  }
  if (!ok) {
    int warm[64];
    const int nw = A.factor_ok ? A.ws.m : 0;
    for (int i = 0; i < nw; ++i) warm[i] = A.ws.codes[i];
    ok = gi_solve(Q, A.ws, warm, nw, lin_none, W, x, X.run.gi_steps);
    A.factor_ok = ok;
    if (ok) ok = certify(Q, A.ws, x, lin_none);
    if (!ok) ++X.run.inexact;
  }
  for (int k = 0; k < H; ++k) {
    A.u[k] = around(x[k], c.round_decimals);
    tie_round(c, X.t, X.it, TIE_ROUND_U, a, k, x[k]);
  }
  if (c.pos_model == 0) rollout_linear(A.xt, A.u.data(), A.spd, c.dt, c.L, H, A.px.data(), A.py.data());
  else rollout_nonlinear(A.xt, A.u.data(), A.spd, c.dt, c.L, H, A.px.data(), A.py.data());
}

// pair z-step + hat rollouts (casadi/main.py:121-158, edge_qp / hinge_rows of the oracle)
void z_step(Ctx& X, World& Wd, int e, int t, Work& W) {
  const CpuCfg& c = X.c;
  const int H = c.H, R = H + 1, n = 2 * H;
  Pair& P = Wd.pr[e];
  const Agent* ag[2] = {&Wd.ag[P.v[0]], &Wd.ag[P.v[1]]};
  W.ensure(n);
  std::vector<double> cv[2], Mv[2];
  for (int v = 0; v < 2; ++v) {
    cv[v].resize(2 * R);
    Mv[v].resize(2 * R * H);
    rollout_affine(ag[v]->xt, ag[v]->spd, c.dt, c.L, H, cv[v].data(), Mv[v].data());
  }
  std::vector<double> q(n, 0.0), G((size_t)H * n, 0.0), h(H);
  for (int v = 0; v < 2; ++v) {
    const double* p[2] = {ag[v]->px.data(), ag[v]->py.data()};
    const double* lam = &P.lam[(size_t)v * 2 * R];
    for (int j = 0; j < H; ++j) {
      double s = 0.0;
      for (int a = 0; a < 2; ++a)
        for (int k = 0; k < R; ++k) {
          const int i = a * R + k;
          const double b = p[a][k] + lam[i] - cv[v][i];
          s += Mv[v][i * H + j] * b;
        }
      q[v * H + j] = -c.rho * s;
    }
  }
  const double db0 = ag[1]->seeds[0] - ag[0]->seeds[0], db1 = ag[1]->seeds[1] - ag[0]->seeds[1];
  const double dd = db0 * db0 + db1 * db1;
  const double D2 = P.d_eff * P.d_eff;
  for (int k = 1; k <= H; ++k) {
    h[k - 1] = D2 + dd - 2.0 * (db0 * (cv[1][k] - cv[0][k]) + db1 * (cv[1][R + k] - cv[0][R + k]));
    for (int j = 0; j < H; ++j) {
      G[(size_t)(k - 1) * n + j] = -2.0 * (db0 * Mv[0][k * H + j] + db1 * Mv[0][(R + k) * H + j]);
      G[(size_t)(k - 1) * n + H + j] = 2.0 * (db0 * Mv[1][k * H + j] + db1 * Mv[1][(R + k) * H + j]);
    }
  }
  QPDef Q;
  Q.n = n;
  Q.H = H;
  Q.NV = 2;
  Q.Pinv = P.Ppinv.data();
  Q.q = q.data();
  Q.G = G.data();
  Q.h = h.data();
  Q.umax = c.u_max;
  Q.dumax = c.du_max;
  Q.beta = c.beta;
  Q.tol = c.qp_tol;
  // warm start: this step's last active set, or the previous step's shifted one slot
  std::vector<int> warm;
  if (P.pws_t == t) {
    warm = P.pws;
  } else if (P.pws_t == t - 1) {
    const int nb = 2 * H - 1;
    for (int code : P.pws) {
      const int row = code >> 1;
      int k, base;
      if (row >= 2 * nb) { k = row - 2 * nb; base = 2 * nb; }
      else { k = (row % nb < H) ? row % nb : row % nb - H; base = row - k; }
      if (k < 1) continue;
      int nc = 2 * (base + k - 1) + (code & 1);
      if (row >= 2 * nb) nc &= ~1;
      warm.push_back(nc);
    }
  }
  thread_local ActiveSet As;
  if (As.n != n) As.init(n, n);
  std::vector<char> lin(H, 0);
  std::vector<double> x(n);
  ++X.run.z_qps;
  bool ok = gi_solve(Q, As, warm.data(), (int)warm.size(), lin.data(), W, x.data(), X.run.gi_steps);
  if (!ok) DBG("pair gi fail t=%d\n", t);
  if (ok) { ok = certify(Q, As, x.data(), lin.data()); if (!ok) DBG("pair cert fail t=%d m=%d\n", t, As.m); }
  if (!ok) ++X.run.inexact;
  P.pws.assign(As.codes.begin(), As.codes.begin() + As.m);
  P.pws_t = t;
  std::vector<double> uh(H), hx(R), hy(R);
  for (int d = 0; d < 2; ++d) {
    for (int k = 0; k < H; ++k) {
      uh[k] = around(x[d * H + k], c.round_decimals);
      tie_round(c, t, X.it, TIE_ROUND_UHAT, e, d * H + k, x[d * H + k]);
    }
    rollout_nonlinear(ag[d]->xt, uh.data(), ag[d]->spd, c.dt, c.L, H, hx.data(), hy.data());
    double* ht = &P.hat[(size_t)d * 2 * R];
    for (int k = 0; k < R; ++k) {
      ht[k] = hx[k];
      ht[R + k] = hy[k];
    }
  }
}

// dual update of a pair (oracle dual_update): plain casadi/main.py:161-162, PI :156-188
void dual_update(const CpuCfg& c, World& Wd, Pair& P, const double* dist) {
  const int R = c.H + 1;
  const Agent &a0 = Wd.ag[P.v[0]], &a1 = Wd.ag[P.v[1]];
  const double* ps[2][2] = {{a0.px.data(), a0.py.data()}, {a1.px.data(), a1.py.data()}};
  double kP = 0.0;
  if (c.dual_mode != 0) {
    double dmin = dist[0];
    for (int k = 1; k < R; ++k) dmin = std::min(dmin, dist[k]);
    kP = c.theta1 - c.theta2 / (1 + std::exp(-dmin));
  }
  for (int d = 0; d < 2; ++d) {
    double* lam = &P.lam[(size_t)d * 2 * R];
    double* S = &P.S[(size_t)d * 2 * R];
    double* D = &P.D[(size_t)d * 2 * R];
    const double* hat = &P.hat[(size_t)d * 2 * R];
    for (int a = 0; a < 2; ++a)
      for (int k = 0; k < R; ++k) {
        const int i = a * R + k;
        const double err = ps[d][a][k] - hat[i];
        if (c.dual_mode == 0) {
          lam[i] += c.rho * err;
        } else {
          S[i] = S[i] + c.kI * err + D[i];
          lam[i] = S[i] + kP * err;
        }
      }
    if (c.windup) {
      const double Wc = c.windup_sat;
      double orig[2 * 64 + 2];
      bool any = false;
      for (int i = 0; i < 2 * R; ++i) {
        orig[i] = lam[i];
        lam[i] = std::min(Wc, std::max(lam[i], -Wc));
        any |= orig[i] != lam[i];
      }
      for (int i = 0; i < 2 * R; ++i) D[i] = any ? lam[i] - orig[i] : 0.0;
    }
  }
}

// seeds (casadi/main.py:48-49), the per-step reset of the pair state (:52-63; with warm_duals the
// previous step's shifted one slot, optimizer.py:337-344 / oracle shift_horizon), safety distance
void begin_step(const CpuCfg& c, World& Wd, Comp& C, bool first_step, int t) {
  const int R = c.H + 1;
  for (int a : C.agents) {
    Agent& A = Wd.ag[a];
    const double sx = A.xt[0] + c.dt * A.spd * std::cos(A.xt[2]), sy = A.xt[1] + c.dt * A.spd * std::sin(A.xt[2]);
    A.seeds[0] = around(sx, c.round_decimals);
    A.seeds[1] = around(sy, c.round_decimals);
    tie_round(c, t, -1, TIE_ROUND_SEED, a, 0, sx);
    tie_round(c, t, -1, TIE_ROUND_SEED, a, 1, sy);
  }
  for (int e : C.pairs) {
    Pair& P = Wd.pr[e];
    for (auto* arr : {&P.hat, &P.lam, &P.S, &P.D, &P.last}) {
      if (c.warm_duals && !first_step) {
        for (int r = 0; r < 4; ++r) {
          double* row = arr->data() + (size_t)r * R;
          for (int k = 0; k < R - 1; ++k) row[k] = row[k + 1];     // drop slot 0, duplicate the last
        }
      } else {
        arr->assign((size_t)2 * 2 * R, 0.0);
      }
    }
    const Agent &a0 = Wd.ag[P.v[0]], &a1 = Wd.ag[P.v[1]];
    P.d_eff = c.tighten ? c.dis_thres + delay_norm(c, a0.xt, a0.spd) + delay_norm(c, a1.xt, a1.spd) : c.dis_thres;
    P.active = P.seen = false;
    P.dis_chk = NAN;
    P.rk = P.sk = 0.0;
  }
  C.flag = C.alias = C.done = false;
  C.iters = 0;
  C.resid.clear();
}

// one outer iteration of a component up to its partials: x-steps, collision tests, pair QPs, dual
// updates, residual terms (pair order), and [rk, sk, active pairs, checked pairs, failed checks]
void iterate(Ctx& X, World& Wd, Comp& C, int t, int it, Work& W) {
  const CpuCfg& c = X.c;
  const int R = c.H + 1;
  C.iters = it + 1;
  X.it = it;
  for (int a : C.agents) x_step(X, Wd, a, W);
  double rk = 0.0, sk = 0.0, nact = 0.0, nseen = 0.0, nbad = 0.0;
  for (int e : C.pairs) {
    Pair& P = Wd.pr[e];
    const Agent &a0 = Wd.ag[P.v[0]], &a1 = Wd.ag[P.v[1]];
    const double thr = c.collide_sq_thres ? P.d_eff * P.d_eff : P.d_eff;
    bool col = c.no_collision_gate != 0;
    double dmin2 = INFINITY;
    int kmin = 0;
    for (int k = 0; k < R && !col; ++k) {
      const double dx = a0.px[k] - a1.px[k], dy = a0.py[k] - a1.py[k];
      const double d2 = dx * dx + dy * dy;
      col = d2 < thr;
      if (d2 < dmin2) { dmin2 = d2; kmin = k; }
    }
    // near tie of the test (oracle TieLog.collide): no slot decisively below, the minimum within tol
    // (a colliding pair's scan stops at its first hit, below thr (1 - tol) unless that hit is a tie)
    if (!c.no_collision_gate && (!col || dmin2 >= thr * (1.0 - g_tie_tol)) && dmin2 <= thr * (1.0 + g_tie_tol)) {
      bool lo = false;
      for (int k = 0; k < R; ++k) {
        const double dx = a0.px[k] - a1.px[k], dy = a0.py[k] - a1.py[k];
        const double d2 = dx * dx + dy * dy;
        lo |= d2 < thr * (1.0 - g_tie_tol);
        if (d2 < dmin2) { dmin2 = d2; kmin = k; }
      }
      if (!lo) tie_add(t, it, TIE_COLLIDE, e, kmin, (dmin2 - thr) / thr);
    }
    P.active = col;
    if (col) {
      z_step(X, Wd, e, t, W);
      double dist[64 + 1];
      for (int k = 0; k < R; ++k) {
        const double dx = a0.px[k] - a1.px[k], dy = a0.py[k] - a1.py[k];
        dist[k] = std::sqrt(dx * dx + dy * dy);
      }
      dual_update(c, Wd, P, dist);
      P.dis_chk = dist[1];
      if (c.term_dist_check) tie_scalar(t, it, TIE_DIST, e, 0, P.dis_chk, P.d_eff);
      P.seen = true;
      // residuals (oracle pair_residuals): v1 side only, times 2
      const double* hat0 = &P.hat[0];
      const double* last0 = &P.last[0];
      double r2 = 0.0, s2 = 0.0;
      for (int k = 0; k < R; ++k) {
        const double e1 = a0.px[k] - hat0[k], e2 = a0.py[k] - hat0[R + k];
        r2 += e1 * e1 + e2 * e2;
      }
      for (int i = 0; i < 2 * R; ++i) {
        const double ev = c.rho * (last0[i] - hat0[i]);
        s2 += ev * ev;
      }
      P.rk = 2 * std::sqrt(r2);
      P.sk = 2 * std::sqrt(s2);
    }
    if (P.seen) {
      nseen += 1.0;
      nbad += (P.dis_chk > P.d_eff) ? 0.0 : 1.0;
    }
    if (!P.active) continue;
    nact += 1.0;
    if (!C.alias) sk += P.sk;
    rk += P.rk;
  }
  C.part[0] = rk;
  C.part[1] = sk;
  C.part[2] = nact;
  C.part[3] = nseen;
  C.part[4] = nbad;
}

// stop rules of one termination group (casadi/main.py:115-118,174-181); part = summed partials
void decide(const CpuCfg& c, const double* part, bool& g_flag, bool& g_alias, bool& g_done, int t, int it, int gid) {
  const double rk = part[0], sk = part[1], n_act = part[2], n_seen = part[3], n_bad = part[4];
  if (n_act == 0 && !g_flag && !c.fixed_iters) {
    g_done = true;
    return;
  }
  g_flag = true;
  if (!c.fixed_iters) {
    tie_scalar(t, it, TIE_STOP, gid, 0, rk, c.eps_pri);
    tie_scalar(t, it, TIE_STOP, gid, 1, sk, c.eps_dual);
  }
  const bool dist_ok = n_seen > 0 && n_bad == 0;
  if (!c.fixed_iters && rk <= c.eps_pri && sk <= c.eps_dual && (!c.term_dist_check || dist_ok)) {
    g_done = true;
    return;
  }
  if (c.alias_dual_residual) g_alias = true;
}

void after_decide(const CpuCfg& c, World& Wd, Comp& C, bool recorded, bool g_alias) {
  const int R = c.H + 1;
  if (recorded) {
    C.resid.push_back(C.part[0]);
    C.resid.push_back(C.part[1]);
  }
  if (C.done) return;
  if (c.alias_dual_residual) {
    C.alias = g_alias;
  } else {
    for (int e : C.pairs) std::memcpy(Wd.pr[e].last.data(), Wd.pr[e].hat.data(), sizeof(double) * 2 * 2 * R);
  }
}

// propagation (oracle propagate, casadi/main.py:185-192): slot 1 of rollout_nonlinear
void end_step(const CpuCfg& c, World& Wd, const Comp& C) {
  for (int a : C.agents) {
    Agent& A = Wd.ag[a];
    double* xt = A.xt;
    const double s = A.spd, th = xt[2];
    const double sk = std::sin(th), ck = std::cos(th);
    const double x1 = xt[0] + (-s * sk * th + (s * ck + s * th * sk)) * c.dt;
    const double y1 = xt[1] + (s * ck * th + (s * sk - s * th * ck)) * c.dt;
    xt[2] = th + (s / c.L * A.u[0]) * c.dt;
    xt[0] = x1;
    xt[1] = y1;
  }
}

}  // namespace

extern "C" {

int piadmm_cpu_cfg_size() { return (int)sizeof(CpuCfg); }

// Near-tie log of the last run (the mirror of piadmm_get_near_ties): tolerance, counts per kind,
// events (6 ints + margin each, at most cap).  Returns the number of events kept.
void piadmm_cpu_set_tie_tol(double tol) { g_tie_tol = tol; }
int piadmm_cpu_get_ties(long long* counts, int* ev, double* mg, int cap) {
  if (counts) std::memcpy(counts, g_tie_cnt, sizeof(g_tie_cnt));
  const int n = std::min<int>((int)g_tie_mg.size(), cap);
  if (ev) std::memcpy(ev, g_tie_ev.data(), sizeof(int) * 6 * (size_t)n);
  if (mg) std::memcpy(mg, g_tie_mg.data(), sizeof(double) * (size_t)n);
  return n;
}

// Runs n_steps MPC steps (t = t0 ...) of N agents with the E candidate pairs `edges` (E x 2,
// v1 < v2) on `threads` OpenMP threads, OpenMP over connected components (labelled in order of
// their first agent, the oracle's Scenario.components(); agents and pairs of a component in
// increasing index).  ref is (N, 2, T).  Outputs (any may be null): xt_out (n_steps, N, 3), u_out
// (n_steps, N, H), iters_out (n_steps, C), resid_out (n_steps, C, max_outer, 2; unused slots NaN),
// counters [x_qps, z_qps, x_hits, gi_steps, inexact].  seconds_out = wall time of the steps.
// Returns the number of components C (>= 1), or -1 on bad arguments.
int piadmm_cpu_run_graph(const CpuCfg* cfg, int N, const double* spd, const double* xt0, const double* ref, int T,
                         int E, const int* edges, int t0, int n_steps, int threads, double* xt_out, double* u_out,
                         int* iters_out, double* resid_out, double* seconds_out, long long* counters) {
  const CpuCfg& c = *cfg;
  const int H = c.H, MO = c.max_outer;
  if (H < 3 || H > 63 || N < 1 || E < 0 || t0 + n_steps + H > T || MO < 1) return -1;
  if (c.dual_mode != 0 && c.dual_mode != 1) return -1;
  if (threads < 1) threads = 1;
  g_tie_ev.clear();
  g_tie_mg.clear();
  for (auto& v : g_tie_cnt) v = 0;
  World Wd;
  Wd.ag.resize(N);
  Wd.pr.resize(E);
  std::vector<int> parent(N);
  for (int a = 0; a < N; ++a) parent[a] = a;
  auto find = [&](int a) {
    while (parent[a] != a) a = parent[a] = parent[parent[a]];
    return a;
  };
  std::vector<std::vector<std::pair<int, std::pair<int, int>>>> adj(N);   // (neighbour, (pair, dir))
  for (int e = 0; e < E; ++e) {
    const int v1 = edges[2 * e], v2 = edges[2 * e + 1];
    if (v1 < 0 || v2 >= N || v1 >= v2) return -1;
    Wd.pr[e].v[0] = v1;
    Wd.pr[e].v[1] = v2;
    adj[v1].push_back({v2, {e, 0}});
    adj[v2].push_back({v1, {e, 1}});
    const int ra = find(v1), rb = find(v2);
    if (ra != rb) parent[std::max(ra, rb)] = std::min(ra, rb);
  }
  std::vector<int> cid(N, -1), root_id(N, -1);
  for (int a = 0; a < N; ++a) {
    const int r = find(a);
    if (root_id[r] < 0) {
      root_id[r] = (int)Wd.comps.size();
      Wd.comps.emplace_back();
    }
    cid[a] = root_id[r];
    Wd.comps[cid[a]].agents.push_back(a);
  }
  for (int e = 0; e < E; ++e) Wd.comps[cid[edges[2 * e]]].pairs.push_back(e);
  const int C = (int)Wd.comps.size();
  for (int a = 0; a < N; ++a) {
    Agent& A = Wd.ag[a];
    A.spd = spd[a];
    std::sort(adj[a].begin(), adj[a].end());
    for (const auto& x : adj[a]) A.nbr.push_back(x.second);
    agent_P(c, A.spd, (int)A.nbr.size(), A.Pinv);
    A.ws.init(H, H);
    A.u.assign(H, 0.0);
    A.px.assign(H + 1, 0.0);
    A.py.assign(H + 1, 0.0);
    for (int j = 0; j < 3; ++j) A.xt[j] = xt0[a * 3 + j];
  }
  for (int e = 0; e < E; ++e) {
    Pair& P = Wd.pr[e];
    pair_P(c, Wd.ag[P.v[0]].spd, Wd.ag[P.v[1]].spd, P.Ppinv);
    for (auto* arr : {&P.hat, &P.lam, &P.S, &P.D, &P.last}) arr->assign((size_t)2 * 2 * (H + 1), 0.0);
  }
  std::vector<Run> runs(threads);
  for (auto& r : runs) r.c = c, r.H = H;
  const auto tstart = std::chrono::steady_clock::now();
  for (int st = 0; st < n_steps; ++st) {
    const int t = t0 + st;
    if (!c.term_global || c.fixed_iters) {
      // per-component termination (or fixed iterations): every component runs its own loop
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
      for (int k = 0; k < C; ++k) {
        Run& run = runs[omp_get_thread_num()];
        Ctx X{c, ref, T, run, t};
        thread_local Work W;
        Comp& Cm = Wd.comps[k];
        begin_step(c, Wd, Cm, st == 0, t);
        bool gf = false, ga = false;
        for (int it = 0; it < MO && !Cm.done; ++it) {
          iterate(X, Wd, Cm, t, it, W);
          bool gd = false;
          decide(c, Cm.part, gf, ga, gd, t, it, k);
          Cm.done = gd;
          after_decide(c, Wd, Cm, gf, ga);
        }
        end_step(c, Wd, Cm);
      }
    } else {
      // the reference's global scope: one stop decision per outer iteration over all components
      for (int k = 0; k < C; ++k) begin_step(c, Wd, Wd.comps[k], st == 0, t);
      bool gf = false, ga = false, gd = false;
      for (int it = 0; it < MO && !gd; ++it) {
#pragma omp parallel for schedule(dynamic, 4) num_threads(threads)
        for (int k = 0; k < C; ++k) {
          Run& run = runs[omp_get_thread_num()];
          Ctx X{c, ref, T, run, t};
          thread_local Work W;
          iterate(X, Wd, Wd.comps[k], t, it, W);
        }
        double part[5] = {0, 0, 0, 0, 0};
        for (int k = 0; k < C; ++k)                 // component order (the oracle's sum)
          for (int j = 0; j < 5; ++j) part[j] += Wd.comps[k].part[j];
        decide(c, part, gf, ga, gd, t, it, -1);
        for (int k = 0; k < C; ++k) {
          Wd.comps[k].done = gd;
          after_decide(c, Wd, Wd.comps[k], gf, ga);   // recorded unless no pair ever collided (gf)
        }
      }
#pragma omp parallel for schedule(static) num_threads(threads)
      for (int k = 0; k < C; ++k) end_step(c, Wd, Wd.comps[k]);
    }
    if (xt_out || u_out) {
      for (int a = 0; a < N; ++a) {
        if (xt_out)
          for (int j = 0; j < 3; ++j) xt_out[((size_t)st * N + a) * 3 + j] = Wd.ag[a].xt[j];
        if (u_out)
          for (int j = 0; j < H; ++j) u_out[((size_t)st * N + a) * H + j] = Wd.ag[a].u[j];
      }
    }
    for (int k = 0; k < C; ++k) {
      const Comp& Cm = Wd.comps[k];
      if (iters_out) iters_out[(size_t)st * C + k] = Cm.iters;
      if (resid_out) {
        double* ro = resid_out + ((size_t)st * C + k) * MO * 2;
        for (int i = 0; i < 2 * MO; ++i) ro[i] = (i < (int)Cm.resid.size()) ? Cm.resid[i] : NAN;
      }
    }
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - tstart).count();
  if (seconds_out) *seconds_out = secs;
  if (counters) {
    long long s[5] = {0, 0, 0, 0, 0};
    for (auto& r : runs) {
      s[0] += r.x_qps;
      s[1] += r.z_qps;
      s[2] += r.x_hits;
      s[3] += r.gi_steps;
      s[4] += r.inexact;
    }
    std::memcpy(counters, s, sizeof(s));
  }
  return C;
}

// The tiled workload (agents 2k, 2k+1 and candidate pair (2k, 2k+1) = tile k; ref (2 n_tiles, 2, T)):
// piadmm_cpu_run_graph on that graph.  Returns 0 or -1.
int piadmm_cpu_run(const CpuCfg* cfg, int n_tiles, const double* spd, const double* xt0, const double* ref, int T,
                   int t0, int n_steps, int threads, double* xt_out, double* u_out, int* iters_out, double* resid_out,
                   double* seconds_out, long long* counters) {
  if (n_tiles < 1) return -1;
  std::vector<int> edges(2 * (size_t)n_tiles);
  for (int k = 0; k < n_tiles; ++k) {
    edges[2 * k] = 2 * k;
    edges[2 * k + 1] = 2 * k + 1;
  }
  const int C = piadmm_cpu_run_graph(cfg, 2 * n_tiles, spd, xt0, ref, T, n_tiles, edges.data(), t0, n_steps, threads,
                                     xt_out, u_out, iters_out, resid_out, seconds_out, counters);
  return C == n_tiles ? 0 : -1;
}

}  // extern "C"
