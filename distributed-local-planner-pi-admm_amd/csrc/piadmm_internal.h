// Internal device/host shared definitions for libpiadmm (not part of the ABI).
#pragma once
#include "piadmm.h"

namespace pd {

// The HIP error of the last kernel launch (launchers return launch_rc(...); the C-ABI's error
// message reports it -- hipGetLastError() is consumed by the launcher itself).
extern thread_local hipError_t g_launch_err;
inline int launch_rc(hipError_t e) {
  g_launch_err = e;
  return e == hipSuccess ? 0 : -1;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, size, device) rather than on
// every launch: the split / exchange paths launch several kernels per outer iteration.
int set_dyn_lds(const void* fn, size_t bytes);

// dst[0:n) = src[0:n) on stream s, as a kernel on the compute queue (the single-rank stand-in of
// an all-reduce: no DMA-engine hand-off between two compute launches).
int launch_copy(double* dst, const double* src, size_t n, hipStream_t s);


constexpr int WAVE = 64;
constexpr int NW = 2;        // agent waves per workgroup of k_mpc_step = agents per component (max)
constexpr int PW = NW;       // the pair's wave (k_mpc_step): its own loop, registers and LDS vectors
constexpr int NWT = NW + 1;  // waves per workgroup of k_mpc_step that solve QPs
constexpr int RW = NW + 1;   // speculative loop only: the roller wave -- agent 1's per-iteration rollout,
                             // concurrent with the pair wave's rollout of agent 0
constexpr int NWA = NW + 2;  // waves per workgroup of k_mpc_step in the speculative loop
constexpr int HCAP = 64;     // storage stride of per-lane state: lane k <-> time index k, H <= 63
constexpr int HMAX = 32;     // largest H of the all-in-LDS layout ("LDS mode")
constexpr int HBIG = 63;     // largest H supported (matrices in HBM / L2 beyond HMAX: "big mode")
constexpr int LD = 65;       // odd LDS stride of the per-wave matrix scratch
constexpr int XLDT = HMAX + 2; // LDS mode: stride of the transposed X' T' rows (a < HMAX; beta at column H)
// LDS mode: the transposed G T' (H rows of even stride gt_ld, then g), per agent
__host__ __device__ constexpr int gt_ld(int H) { return H + (H & 1); }
__host__ __device__ constexpr int gt_stride(int H) { return H * gt_ld(H) + gt_ld(H); }
constexpr int XLDG = 65;       // stride of X' in HBM (big mode: up to 64 working-set rows)
constexpr int RUIZ_ITERS = 10;
constexpr int PDAS_STEPS = 4;

// Row slots per lane.  x-step: 0 box, 1 rate.  pair (z-step): 0 box v1, 1 rate v1,
// 2 box v2, 3 rate v2, 4 hinge (time k+1).  Global row id = slot*H + lane.
enum RowLab : signed char { FREE = 0, LOWER = 1, UPPER = 2 };        // box / rate rows
enum HingeLab : signed char { HZERO = 0, HKINK = 1, HLINEAR = 2 };   // hinge rows

struct DevArgs {
  piadmm_config_t cfg;
  int N, E, C, T;
  int pair_gi;              // 1: pair QPs try the dual active set first (env PIADMM_PAIR_SOLVER)
  int pair_warm;            // 1: the pair's dual active set starts from its last active set (PIADMM_PAIR_WARM=0: cold)
  int x_gi;                 // x-step working-set changes by the dual active set (1); the step's first x-QP
                            // without the labels' reduced solve (2), started cold (3); all cold (4); PIADMM_X_SOLVER
  int no_spec;              // 1: k_mpc_step keeps the plain loop shape (PIADMM_NO_SPEC=1, read at set_scenario)
  // scenario (read-only during a step)
  const double* spd;        // N
  const double* ref;        // N*2*T
  const int* comp_ptr;      // C+1 : agents of component c are [comp_ptr[c], comp_ptr[c+1])
  const int* comp_edge;     // C   : the component's pair index or -1
  const int* edges;         // E*2
  const int* nbr_cnt;       // N   : candidate neighbours per agent (|N(i)| in the AL sum)
  // state
  double* xt;               // N*3
  double* u;                // N*H   primal_u
  double* pos_old;          // N*2*(H+1)
  double* hat;              // E*2*2*(H+1)
  double* lam;              // E*2*2*(H+1)
  unsigned char* edge_active;  // E
  int* iters;               // C
  double* resid;            // step_cap*C*max_outer*2 (slot k: step k of a multi-step launch)
  int* status;              // N+E
  // per-step solver workspace
  double* Pinv_x;           // N*H*H
  double* sc_x;             // N*4*HCAP   (D, Ebox, Erate, spare)
  signed char* lab_x;       // N*2*HCAP   final x-step labels of the last step (next step's warm guess)
  // big mode (H > HMAX): the matrices the LDS layout keeps per workgroup live in HBM / L2
  double* Gx_g;             // N*(H*H+H)   x-step polish G | g
  double* XT_g;             // N*(H+1)*XLDG  x-step X' | beta
  double* Ke_g;             // E*4*H*H     pair K_s^-1
  double* Yx_g;             // N*64*H      x-step dual active-set columns P^-1 n_a (big mode)
  float* T32_g;             // precision 2: N*(H*H + H*XLDG) fp32 images of the x-step G | X' (unfolded)
  double* tab_e;            // E * 8H^2 polish tables per edge, one block each:
                            //   [0, 4H^2) P^-1 (2H x 2H, block-diagonal), [4H^2, 6H^2) PGt (H x 2H,
                            //   row k = P_v^-1 T(k+1,.)'), [6H^2, 8H^2) GPG (Z_v = T P_v^-1 T')
  int* warm_ok;             // N          1: lab_x holds the labels of the previous MPC step
  // per-step state carried between the launches of one step (term_global) and, for the
  // PI accumulators, between steps (warm_duals)
  double* Sacc;             // E*2*2*(H+1) PI integral S
  double* Dacc;             // E*2*2*(H+1) back-calculation D
  double* last;             // E*2*2*(H+1) last_iter_hat_pos (dual residual)
  double* dischk;           // E   dis_vec(2) of the pair's last dual update (NaN: none yet)
  double* deff;             // E   safety distance of the pair for the current step
  double* qs_x;             // N*5*WAVE  ADMM state (xs, zs0, zs1, ys0, ys1) of the x-step QP
  signed char* ql_x;        // N*2*WAVE  labels of the x-step QP
  double* qs_e;             // E*12*WAVE ADMM state (xs0, xs1, zs0..4, ys0..4) of the pair QP
  signed char* ql_e;        // E*5*WAVE  labels of the pair QP
  int* cst;                 // C*4       flag, aliased, warm bits (x0, x1, pair), spare
  unsigned long long* counters;  // C*8  accumulated work counters (see piadmm_get_counters)
  unsigned long long* stamps;    // C x 4 waves x 64 phase cycle sums (diagnostic build -DPIADMM_STAMPS only)
  double* rho_x;            // N   ADMM penalty per agent QP (adapted, persists across steps)
  double* rho_e;            // E   ADMM penalty per pair QP
  double* Kx_cache;         // N*H*H agent K_s^-1 for the penalty xcache_rho[a] (per scenario)
  double* xcache_rho;       // N   penalty of the cached agent setup (NaN: none)
  int* ecache;              // E   1 when the pair's speed-only tables are built
  int* gi_ws;               // E*(2+64) the pair's last dual active set: m, step t, codes
  double* gi_wide;          // H >= 32: C * (GW | 1) * giw_stride(H) wide dual active-set scratch
  size_t gi_wide_stride;    // giw_stride(H)
  double* gi_snap;          // graph mode: E * (64*64 + 64*2H + 64) the pair's last dual active set: S^-1 | Y | hinge regimes
  double* gpart;            // 2*C*5 coop: per-component termination partials (iteration parity)
  unsigned long long* gbar;  // C coop: the grid barrier's arrival epochs, one word per workgroup (pd_common.h
                            //   grid_flag_barrier); zeroed once, epochs only grow
  unsigned long long gbar_base;  // coop: epoch base of this launch (set per cooperative launch, launch_coop_epoch)
  double* ghist;            // step_cap*max_outer*2 coop: global (rk, sk) history per step
  int* giters;              // step_cap coop: global outer iterations per step
  int* gctl;                // 4: device-decided global stop (F_DEVSTOP): stop, nanlast, iterations, flag
  // ---- graph mode (k_graph_step): any static candidate graph (components of any size, agents
  // in several pairs).  All per-QP state lives in HBM between the phases of an outer iteration.
  int graph;                // 1: the scenario runs on k_graph_step
  const int* nbr_ptr;       // N+1 CSR: incident candidate pairs of agent a, sorted by neighbour id
  const int* nbr_edge;      // 2E  pair index
  const int* nbr_dir;       // 2E  0: a is v1 of the pair (owns hat_{v1 v2}), 1: a is v2
  const int* comp_aptr;     // C+1 agents of component c: comp_alist[comp_aptr[c] .. comp_aptr[c+1])
  const int* comp_alist;    // N   (increasing agent index)
  const int* comp_eptr;     // C+1 pairs of component c: comp_elist[comp_eptr[c] .. comp_eptr[c+1])
  const int* comp_elist;    // E   (increasing pair index: the residual sum order, casadi/main.py:165-173)
  const unsigned char* owned;   // N   1: this rank solves the agent's x-step (0: ghost of another rank)
  const unsigned char* counted; // E   1: this rank counts the pair's residual (cross-rank pairs: one rank)
  const int* xslot;         // N   slot of a boundary agent in the exchange buffer (-1: none)
  double* xbuf;             // n_slots * 3(H+1): send buffer, px | py | u of the rank's own boundary
                            //   agents (other slots stay 0, so the all-reduce sum is an all-gather)
  const double* xrecv;      // n_slots * 3(H+1): the all-reduced buffer (ghost agents read theirs)
  int n_slots;
  double* seed_g;           // N*2 seeds of the current MPC step (casadi/main.py:48-49)
  double* eres;             // E*2 (rk_e, sk_e) of the pair's last z-step
  double* cpart;            // C*5 termination partials of the component's last iteration
  int* csig_x;              // N*WAVE per-lane signature of the agent's cached x-step tables (-1: none)
  int* xflags;              // N   bit 0: the x-step QP holds a warm state
  int* eflags;              // E   bit 0: the pair QP holds a warm state
  int ke_stride;            // doubles per pair in Ke_g (graph mode: room for 64 dual active-set columns)
  // global PI (PIADMM_DUAL_PI_GLOBAL, graph mode): the pair's adaptive penalty (kept across MPC
  // steps) and the penalty-dependent caches' keys
  double* rho_pi;           // E   rho of the pair (casadi_old_PI_ADMM/main.py:139)
  double* xcache_coef;      // N   x-step P coefficient 2 Pnorm + sum_e rho_e the caches were built for
  double* ecache_rho;       // E   pair penalty the pair's polish tables were built for
  // ---- components split over workgroups (graph mode, term_global): the job's residual sums in the
  // reference's order -- per ORIGINAL connected component its pairs in increasing pair order, then
  // the components in order (casadi/main.py:165-173; the oracle's comp_r sum) -- instead of the
  // blocks' partial sums.  The T phase writes each pair's effective terms, k_graph_partials sums them.
  double* eterm;            // 2*E: rk terms | sk terms of this iteration, in the sum order (0: inactive /
                            //   not counted / aliased)
  const int* sum_cptr;      // sum_C+1 original component k = sum positions [sum_cptr[k], sum_cptr[k+1])
  const int* sum_pos;       // E   the pair's position in the sum order
  int sum_C;                // 0: no split (the blocks ARE the components)
  // ---- near-tie log (piadmm_get_near_ties): the reference's discrete decisions taken within
  // tie_tol of their threshold -- rounding (casadi/main.py:48-49,103,153), the collision test
  // (:112-113), the stop test (:174) and MATLAB's distance check -- where two exact
  // implementations may resolve them differently
  unsigned long long* tie_cnt;   // PIADMM_TIE_KINDS counts
  unsigned long long* tie_n;     // events so far (may exceed tie_cap)
  int* tie_ev;                   // tie_cap x 6 ints: step, iter, kind, id, index, 0
  double* tie_mg;                // tie_cap margins
  int tie_cap;
  int tie_on;                    // the log is on (tie_tol > 0): the kernels' TIES instantiation
  double tie_tol;
};

// Big mode: rows of the per-wave x-step factor scratch (working sets of up to H + 2 rows:
// a degenerate vertex can hold one or two dependent rows beyond the H variables).
constexpr int xrows(int H) { return H + 2 < 64 ? H + 2 : 64; }
// Big mode: doubles of one agent wave's x-step region (xrows x (xrows + 2)), rounded up to an even
// count so that the next wave's region -- whose S^-1 rows the dual active set reads and writes with
// 16-byte LDS accesses (pd_qp.h gi_solve RM_S) -- starts on 16 bytes for odd H as well.
constexpr int xreg(int H) { return xrows(H) * (xrows(H) + 2) + ((xrows(H) * (xrows(H) + 2)) & 1); }
// LDS the kernel declares statically (s_int, s_cnt, s_warm) on top of lds_bytes().
constexpr size_t STATIC_LDS = NWT * 272 * 4 + NWA * 8 * 4 + 16 + 4 * 4 + 8 + 8;
constexpr size_t MAX_LDS = 160 * 1024;

// fp32 agent K_s^-1 images in LDS mode: per wave H*H floats rounded up to an even count, so
// that the next wave's region (which also holds its fp64 dual active-set columns) is 8-byte
// aligned for odd H; kxf_words = the two waves' regions in doubles.
constexpr size_t kxf_stride(int H) { return ((size_t)H * H + 1) & ~(size_t)1; }
constexpr size_t kxf_words(int H) { return kxf_stride(H); }

// The pair's warm build on two waves (pd_qp.h WarmPipe): its LDS ring (4 + 3 x 130 doubles, then
// 72 ints) after the scalars, in LDS mode up to H = 30 (at H = 31, 32 the workgroup would exceed
// 160 KB; there the pair wave builds alone).
constexpr int WPIPE_HMAX = 30;
constexpr size_t WPIPE_WORDS = 4 + 3 * 130 + 36;
// LDS bytes needed by one workgroup for horizon H (must match the carve in k_mpc_step).
// LDS mode (H <= HMAX): every matrix of the component in LDS.  Big mode: agent K_s^-1, G and
// X' and the pair K_s^-1 in HBM / L2; LDS keeps the factor scratches and the vectors.
inline size_t lds_bytes(int H, int precision = 0) {
  size_t d = 0;
  const bool f32 = precision == 1;
  if (H <= HMAX) {
    d += f32 ? kxf_words(H) : 2 * (size_t)H * H;   // agent K_s^-1 (2 agents; fp32: half)
    d += 2 * (size_t)gt_stride(H);   // agent polish G T' | g (2 agents, transposed)
    d += (f32 ? 2 : 4) * (size_t)H * H;   // pair K_s^-1 (2H x 2H)
    d += 64 * (LD + 1);              // pair matrix scratch (PDAS factor, or the dual active set's
                                     // S^-1 in rows of even stride: pd_qp.h gi_solve RM_S)
    d += NW * HMAX * (HMAX + 2);     // per-wave x-step scratch / Cholesky factor / S^-1 rows
    d += NW * HMAX * XLDT;           // per-wave x-step parametric table X' T' | beta (transposed)
  } else {
    d += 64 * (LD + 1);              // pair matrix scratch (wave 0; S^-1 rows of even stride)
    d += NW * (size_t)xreg(H);       // per-wave x-step scratch / Cholesky factor / S^-1 rows (even counts)
  }
  d += NWT * 512;                  // per-wave vector buffers (agents, pair)
  d += NWT * 128;                  // per-wave factor diagonals (x-step or pair)
  size_t H1 = H + 1;
  d += 2 * 2 * 2 * H1;             // pos_old (two buffers: outer-iteration parity)
  d += 2 * 3 + 2 * 2 + 4 * H;      // xt, seeds, u (two buffers: outer-iteration parity)
  d += 5 * 2 * 2 * H1;             // hat, lam, S, D, last_hat
  d += 32;                         // scalars
  if (H <= WPIPE_HMAX) d += WPIPE_WORDS;   // the helper wave's warm-row ring (pd_qp.h WarmPipe)
  if (H > HMAX && f32) d += 2 * (size_t)H * H + 2;   // big mode: fp32 image of the pair K_s^-1
  return d * sizeof(double);
}

// launch flags of k_mpc_step
constexpr int F_FIRST = 1;    // first launch of the step: seeds, zero / warm per-step state
constexpr int F_LAST = 2;     // last launch: outputs, propagation, cross-step warm labels
constexpr int F_GLOBAL = 4;   // termination decided outside (term_global): no per-component stop
constexpr int F_NANLAST = 8;  // the global loop stopped at the collision test of iteration it0-1
constexpr int F_COOP = 16;    // global termination decided in-kernel (cooperative launch, one rank)

// Graph mode: LDS per workgroup of k_graph_step (GW waves, one component per workgroup).
constexpr int GW = 2;
// The wide dual active set of pair QPs (pd_qp.h gi_solve_wide): working sets up to 126 rows
// (two per lane), S^-1 (stride GIW_LD) and the Y columns (2H doubles each) in HBM scratch, one
// region per solving wave (graph kernel: GW per workgroup; fused kernel: its pair wave).  Only
// H >= 32 can outgrow the 63-row capacity (a pair QP has 2H variables).
constexpr int GIW_LD = 2 * WAVE;
constexpr int GIW_CAP = 2 * WAVE - 2;
inline __host__ __device__ constexpr size_t giw_stride(int H) {
  return (size_t)GIW_LD * GIW_LD + (size_t)GIW_LD * 2 * H;
}
constexpr int GZMAX = 1024;   // pairs per component whose colliding pairs are balanced over the waves
// Dual active-set columns P^-1 n_a in LDS per wave (H <= HMAX; beyond, in HBM): the pair's
// 2H-long columns (63 of them) or the x-step's H-long ones, in turn.
// LDS mode stores them transposed (row v*H + l holds the m coefficients of variable l, stride
// GYLD: pd_qp.h gi_solve<NV, true>), so a lane reads its row two doubles at a time.
constexpr int GYCAP = 63;
constexpr int GYLD = 66;
constexpr size_t graph_ylds(int H) { return H <= HMAX ? (size_t)2 * H * GYLD : 0; }
// The per-wave factor scratch: the pair's PDAS factor (64 x LD) or its dual active set's S^-1
// (rows of even stride LD + 1), the x-step's factor or S^-1 (xrows x (xrows + 2) covers both).
inline __host__ __device__ size_t graph_fac(int H) {
  size_t fac = 64 * (LD + 1);
  const size_t xr = (size_t)xrows(H) * (xrows(H) + 2);
  return xr > fac ? xr : fac;
}
inline size_t graph_lds_bytes(int H) {
  return (GW * (graph_fac(H) + 512 + 256 + graph_ylds(H)) + 64) * sizeof(double);  // + vectors, diagonals, Y
}
// Graph launches also use these flags: F_XPHASE / F_ZPHASE restrict an iteration launch to
// its x-step or its z-step + termination half (the exchange of a sharded job sits between).
constexpr int F_XONLY = 32;
constexpr int F_ZONLY = 64;
// Device-decided global termination (term_global across ranks, RCCL or host transport): iteration
// launches return at once when A.gctl[0] (stop) is set -- a chunk of iterations is enqueued ahead
// with the all-reduce and k_decide between them, and the host reads the stop state once per
// chunk; the LAST launch takes its iteration count and NANLAST from A.gctl.
constexpr int F_DEVSTOP = 128;
// With F_FIRST: only the step init (seeds, per-step pair reset), no iteration -- a component split
// over workgroups resets the pairs its blocks own before ANY block's first x-step reads them.
constexpr int F_INITONLY = 256;
// k_mpc_step: the plain loop shape even where the speculative one would run (PIADMM_NO_SPEC=1; the
// equality test of the two shapes, tests/test_gpu_modes.py)
constexpr int F_NOSPEC = 512;
// k_mpc_step: the pair wave builds its warm rows alone (PIADMM_NO_HELPER=1: the helper wave's A/B)
constexpr int F_NOHELPER = 1024;

int launch_graph_step(const DevArgs& a, int t, int nsteps, int it0, int it1, int flags, hipStream_t s);
// The epoch base of a cooperative launch of nsteps MPC steps: larger than every epoch an earlier
// launch of the process used (a launch's barriers take base + 1 .. base + nsteps * max_outer)
unsigned long long launch_coop_epoch(int nsteps, int max_outer);
// candidate-pair detection (piadmm_detect.hip)
int launch_detect_count(const double* xy, const double* r, int n, double inv_cs, unsigned T, unsigned* key, int* cnt,
                        int* start, int* fill, int* order, int* pcnt, int* off, long long* total, long long* bsum,
                        double* xs, double* rs, hipStream_t s);
constexpr int DETECT_SCAN_B = 1024;   // ints per workgroup of the detection's scans (bsum sizing, 64-bit sums)
int launch_detect_emit(const double* xs, const double* rs, int n, double inv_cs, unsigned T, const int* start,
                       const int* order, const int* off, int* out, hipStream_t s);
bool graph_coop_fits(const DevArgs& a, int device);
int launch_graph_partials(const DevArgs& a, double* out, hipStream_t s, int devstop = 0, int nout = 5);
int launch_decide(const DevArgs& a, int t, int it, const double* part, hipStream_t s);
int launch_mpc_step(const DevArgs& a, int t, int nsteps, int it0, int it1, int flags, hipStream_t s);
int launch_term_partials(const DevArgs& a, int it, double* out, hipStream_t s, int devstop = 0);
int launch_resid_history(const DevArgs& a, int nsteps, double* out, hipStream_t s);
int launch_pair_deff(const DevArgs& a, hipStream_t s);
bool coop_fits(const DevArgs& a, int device);

}  // namespace pd
