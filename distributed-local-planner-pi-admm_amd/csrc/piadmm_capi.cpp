// piadmm_capi.cpp -- C-ABI of libpiadmm (include/piadmm.h): handle, device
// buffers, scenario upload, step launches and state download.
//
// Replaces the reference's per-call CasADi/OSQP instantiation
// (casadi/main.py:96,146) and its Python loop state (casadi/main.py:52-72).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "piadmm_internal.h"

namespace pd {
thread_local hipError_t g_launch_err = hipSuccess;
}

struct piadmm_ctx {
  piadmm_config_t cfg{};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool have_scn = false;
  int N = 0, E = 0, C = 0, T = 0;
  std::vector<int> comp_ptr, comp_edge;
  std::vector<void*> allocs;
  pd::DevArgs a{};
  std::string err;
  // term_global: RCCL communicator (null = single rank), device partials, pinned host copy
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  double* d_part = nullptr;      // max_outer x 5 partials, or max_outer x 2 residual history
  double* h_part = nullptr;      // pinned
  std::vector<double> ghist;     // global (rk, sk) history of the last step
  int giters = 0;
  int step_cap = 1;              // MPC steps per persistent launch (resid slots)
  bool coop = false;             // term_global natural termination decided in-kernel (one rank)
  std::vector<double> rho_init;  // host staging of the initial ADMM penalties (outlives the async copy)
  std::vector<double> rho_pi_init;   // host staging of the global-PI pair penalties
  std::vector<std::vector<int>> graph_host;   // graph-mode index arrays (host staging)
  std::vector<unsigned char> shard_host;      // owned | counted (host staging)
  // sharded graph (piadmm_set_scenario_shard): ghost agents fed by one all-reduce of the
  // boundary exchange buffer per outer iteration
  bool xchg = false;
  int n_slots = 0;
  // a connected component larger than the workgroup block (term_global) split over several
  // workgroups: the graph kernel's X and Z phases as separate launches (like a sharded job's,
  // without the exchange: every agent's positions are in this handle's memory)
  bool split = false;
  double* d_xrecv = nullptr;
  // host all-reduce transport (piadmm_set_allreduce): used when there is no RCCL communicator
  piadmm_allreduce_fn xfn = nullptr;
  void* xctx = nullptr;
  double* h_x = nullptr;         // pinned staging of the host transport
  size_t h_x_n = 0;
  // host-stepped MPC step (piadmm_outer_iter / piadmm_step_finish): the open step, the next
  // outer iteration, and the host-decided stop state of the global scope
  bool step_open = false;
  // the MPC step the receding-horizon sequence continues with (-1: a fresh sequence, any t).  A
  // step run at any other t (the same t again, a jump) must not resume a pair's stored dual active
  // set: its S^-1 and Y columns were built for another step's geometry (pd_qp.h gi_snap_restore)
  int t_next = -1;
  int step_t = -1, step_it = 0, step_flag = 0, step_nanlast = 0, step_stop = 0;
  // device-decided global termination (F_DEVSTOP): pinned copy of the stop state, iterations
  // enqueued per chunk (the last step's count), PIADMM_HOST_DECIDE=1 keeps one host decision
  // per outer iteration
  int* h_ctl = nullptr;
  int chunk_guess = 2;
  bool host_decide = false;
  // near-tie log (piadmm_get_near_ties): tolerance, and the ties of stop decisions the host takes
  double tie_tol = 0.0;         // 0: the log is off (piadmm_set_tie_tolerance turns it on)
  std::vector<piadmm_near_tie_t> host_ties;
  unsigned long long host_tie_cnt[PIADMM_TIE_KINDS] = {};
  // MPC steps per persistent launch agreed over the job's ranks (the fixed-iteration residual
  // history is all-reduced once per launch: every rank must cut the steps into the same launches)
  bool cap_synced = false;
};

namespace {

thread_local std::string g_err;

int fail(piadmm_ctx* h, int code, const std::string& msg) {
  if (h) h->err = msg;
  g_err = msg;
  return code;
}

// A stop / distance decision the host takes within tie_tol of its threshold (the device kernels
// log their own, pd::scalar_tie).
void host_tie(piadmm_ctx* h, int t, int it, int kind, int id, int idx, double v, double thr) {
  if (!(h->tie_tol > 0.0) || !(std::fabs(v - thr) <= h->tie_tol * std::fabs(thr))) return;
  ++h->host_tie_cnt[kind];
  piadmm_near_tie_t ev{};
  ev.step = t;
  ev.iter = it;
  ev.kind = kind;
  ev.id = id;
  ev.index = idx;
  ev.margin = (v - thr) / thr;
  if (h->host_ties.size() < PIADMM_TIE_CAP) h->host_ties.push_back(ev);
}

#define HIPCHK(h, expr)                                                              \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      return fail((h), PIADMM_E_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

template <typename T>
int dalloc(piadmm_ctx* h, T** p, size_t n) {
  void* q = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc(&q, n * sizeof(T));
  if (e != hipSuccess) return fail(h, PIADMM_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
  e = hipMemsetAsync(q, 0, n * sizeof(T), h->stream);
  if (e != hipSuccess) return fail(h, PIADMM_E_HIP, std::string("hipMemset: ") + hipGetErrorString(e));
  h->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return 0;
}

void free_all(piadmm_ctx* h) {
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  h->d_part = nullptr;
  h->have_scn = false;
}

int check_cfg(piadmm_ctx* h, const piadmm_config_t& c) {
  if (c.n_agents <= 0) return fail(h, PIADMM_E_ARG, "n_agents must be > 0");
  if (c.H < 3 || c.H > pd::HBIG) return fail(h, PIADMM_E_ARG, "H must be in [3, 63] in this version");
  if (c.max_outer <= 0) return fail(h, PIADMM_E_ARG, "max_outer must be > 0");
  if (c.dual_mode != PIADMM_DUAL_PLAIN && c.dual_mode != PIADMM_DUAL_PI && c.dual_mode != PIADMM_DUAL_PI_GLOBAL)
    return fail(h, PIADMM_E_ARG, "dual_mode must be 0 (plain), 1 (PI) or 2 (global PI)");
  if (c.dual_mode == PIADMM_DUAL_PI_GLOBAL && !(c.rho_min > 0 && c.rho_max >= c.rho_min && c.rho_num > 0))
    return fail(h, PIADMM_E_ARG, "global PI needs 0 < rho_min <= rho_max and rho_num > 0");
  if ((c.pi_trad != 0 && c.pi_trad != 1) || (c.ki_adapt != 0 && c.ki_adapt != 1))
    return fail(h, PIADMM_E_ARG, "pi_trad and ki_adapt must be 0 or 1");
  if ((c.pi_trad || c.ki_adapt) && c.dual_mode != PIADMM_DUAL_PI_GLOBAL)
    return fail(h, PIADMM_E_ARG, "pi_trad / ki_adapt select variants of the global PI law (dual_mode 2)");
  if (!std::isfinite(c.d_gain) || !std::isfinite(c.dual_init))
    return fail(h, PIADMM_E_ARG, "d_gain and dual_init must be finite");
  // ABI 7 made the back-calculation gain of the global PI law a field: a zero-initialised config
  // would silently drop the term of casadi_old_PI_ADMM/main.py:142 (d_gain 2) and of the adaptive
  // script (1), so 0 is refused rather than taken as a variant
  if (c.dual_mode == PIADMM_DUAL_PI_GLOBAL && c.d_gain == 0.0)
    return fail(h, PIADMM_E_ARG, "global PI needs d_gain != 0 (2.0: casadi_old_PI_ADMM, 1.0: the adaptive-gain script)");
  // warm_duals carries the previous step's shifted duals; dual_init sets every step's start
  // values -- the reference's scripts never combine the two (the first step would be ambiguous)
  if (c.warm_duals && c.dual_init != 0.0)
    return fail(h, PIADMM_E_ARG, "warm_duals and a nonzero dual_init are exclusive");
  if (!(c.dt > 0) || !(c.L > 0) || !(c.rho > 0) || !(c.Pcost > 0) || c.Pnorm < 0 || c.beta < 0)
    return fail(h, PIADMM_E_ARG, "dt, L, rho, Pcost must be > 0; Pnorm, beta >= 0");
  if (c.max_inner <= 0 || c.polish_every <= 0) return fail(h, PIADMM_E_ARG, "max_inner, polish_every must be > 0");
  if (c.round_decimals > 12) return fail(h, PIADMM_E_ARG, "round_decimals must be <= 12");
  if (c.tighten && !(c.tight_p > 0 && c.tight_p < 1)) return fail(h, PIADMM_E_ARG, "tight_p must be in (0, 1)");
  if (c.precision < 0 || c.precision > 2)
    return fail(h, PIADMM_E_ARG, "precision must be 0 (fp64), 1 (fp32 ADMM matrices) or 2 (fp32 x-step tables)");
  if (pd::lds_bytes(c.H, c.precision) + pd::STATIC_LDS > pd::MAX_LDS)
    return fail(h, PIADMM_E_ARG, "the workgroup's LDS exceeds 160 KB (precision 1 keeps the pair's fp32 "
                                  "K_s^-1 in LDS: H <= 55 in big mode)");
  return 0;
}

// Initial ADMM penalties (x-step: adapted by the OSQP rule and carried across steps; pair QPs
// keep this penalty: no adaptation, and on the GPU smaller fixed penalties cost more ADMM
// iterations on the bench's pair QPs -- 0.5x: +0%, 0.2x: +39%, 0.1x: +114% time).
int reset_penalties(piadmm_ctx* h) {
  const size_t N = h->N, E = h->E;
  h->rho_init.assign(std::max<size_t>(N, E) + 1, h->cfg.admm_rho);
  h->rho_pi_init.assign(E + 1, h->cfg.rho);
  HIPCHK(h, hipMemcpyAsync(h->a.rho_x, h->rho_init.data(), N * sizeof(double), hipMemcpyHostToDevice, h->stream));
  if (E) HIPCHK(h, hipMemcpyAsync(h->a.rho_e, h->rho_init.data(), E * sizeof(double), hipMemcpyHostToDevice, h->stream));
  // global PI: every pair starts from the configured penalty (PI_ADMM_class.py:26, rho = 1)
  if (E && h->a.rho_pi)
    HIPCHK(h, hipMemcpyAsync(h->a.rho_pi, h->rho_pi_init.data(), E * sizeof(double), hipMemcpyHostToDevice, h->stream));
  return 0;
}

// Sum over the job's ranks of n doubles at send into recv (may alias), on the handle's stream:
// ncclAllReduce over the RCCL communicator, else the host transport callback (through pinned
// memory; the callback returns when every rank has contributed), else one rank: a copy.
int allreduce(piadmm_ctx* h, const double* send, double* recv, size_t n) {
  if (n == 0) return 0;
  if (h->comm) {
    ncclResult_t r = ncclAllReduce(send, recv, n, ncclDouble, ncclSum, h->comm, h->stream);
    if (r != ncclSuccess) return fail(h, PIADMM_E_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return 0;
  }
  if (h->xfn) {
    if (n > h->h_x_n) {
      if (h->h_x) (void)hipHostFree(h->h_x);
      h->h_x = nullptr;
      h->h_x_n = 0;
      HIPCHK(h, hipHostMalloc((void**)&h->h_x, n * sizeof(double)));
      h->h_x_n = n;
    }
    HIPCHK(h, hipMemcpyAsync(h->h_x, send, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (int rc = h->xfn(h->xctx, h->h_x, (int64_t)n))
      return fail(h, PIADMM_E_STATE, "all-reduce callback failed with " + std::to_string(rc));
    HIPCHK(h, hipMemcpyAsync(recv, h->h_x, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
    return 0;
  }
  if (send != recv && pd::launch_copy(recv, send, n, h->stream) != 0)
    return fail(h, PIADMM_E_HIP, std::string("copy kernel: ") + hipGetErrorString(pd::g_launch_err));
  return 0;
}

}  // namespace

extern "C" {

int32_t piadmm_abi_version(void) { return PIADMM_ABI_VERSION; }

const char* piadmm_build_info(void) {
  static char buf[160];
  std::snprintf(buf, sizeof(buf), "libpiadmm abi=%d arch=gfx950 hip=%d.%d waves/wg=%d hmax=%d (lds layout <= %d)",
                PIADMM_ABI_VERSION, HIP_VERSION_MAJOR, HIP_VERSION_MINOR, pd::NW, pd::HBIG, pd::HMAX);
  return buf;
}

int32_t piadmm_config_size(void) { return (int32_t)sizeof(piadmm_config_t); }

int32_t piadmm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* piadmm_last_error(piadmm_handle_t h) { return h ? h->err.c_str() : g_err.c_str(); }

int32_t piadmm_create(const piadmm_config_t* cfg, piadmm_handle_t* out) {
  if (!cfg || !out) return fail(nullptr, PIADMM_E_ARG, "null argument");
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return fail(nullptr, PIADMM_E_NODEV, "no HIP device");
  if (cfg->device < 0 || cfg->device >= nd) return fail(nullptr, PIADMM_E_ARG, "device ordinal out of range");
  piadmm_ctx* h = new piadmm_ctx();
  h->cfg = *cfg;
  if (h->cfg.admm_rho <= 0) h->cfg.admm_rho = 0.05;
  if (h->cfg.admm_sigma <= 0) h->cfg.admm_sigma = 1e-6;
  if (h->cfg.admm_alpha <= 0 || h->cfg.admm_alpha >= 2) h->cfg.admm_alpha = 1.6;
  if (h->cfg.qp_tol <= 0) h->cfg.qp_tol = 1e-9;
  if (int rc = check_cfg(h, h->cfg)) {
    g_err = h->err;
    delete h;
    return rc;
  }
  hipError_t e = hipSetDevice(cfg->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&h->ev0);
  if (e == hipSuccess) e = hipEventCreate(&h->ev1);
  if (e == hipSuccess) e = hipHostMalloc((void**)&h->h_part, (size_t)std::max(cfg->max_outer, 1) * 5 * sizeof(double));
  if (e == hipSuccess) e = hipHostMalloc((void**)&h->h_ctl, 4 * sizeof(int));
  {
    const char* hd = std::getenv("PIADMM_HOST_DECIDE");
    h->host_decide = hd && hd[0] == '1';
  }
  if (e != hipSuccess) {
    g_err = std::string("HIP init: ") + hipGetErrorString(e);
    delete h;
    return PIADMM_E_HIP;
  }
  *out = h;
  return PIADMM_OK;
}

int32_t piadmm_destroy(piadmm_handle_t h) {
  if (!h) return PIADMM_OK;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_all(h);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  if (h->h_part) (void)hipHostFree(h->h_part);
  if (h->h_ctl) (void)hipHostFree(h->h_ctl);
  if (h->h_x) (void)hipHostFree(h->h_x);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return PIADMM_OK;
}

static int32_t set_scenario_impl(piadmm_handle_t h, const double* spd, const double* xt0, const double* ref,
                                 int32_t T, const int32_t* edges, int32_t n_edges, const uint8_t* owned,
                                 const int32_t* slot, int32_t n_slots, const uint8_t* counted) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!spd || !xt0 || !ref || (n_edges > 0 && !edges)) return fail(h, PIADMM_E_ARG, "null array");
  const int N = h->cfg.n_agents, H = h->cfg.H;
  if (T < H + 1) return fail(h, PIADMM_E_ARG, "reference too short: T < H+1");
  if (n_edges < 0) return fail(h, PIADMM_E_ARG, "n_edges < 0");
  for (int e = 0; e < n_edges; ++e) {
    const int v1 = edges[2 * e], v2 = edges[2 * e + 1];
    if (v1 < 0 || v2 >= N || v1 >= v2) return fail(h, PIADMM_E_ARG, "edge must satisfy 0 <= v1 < v2 < N");
  }
  {
    // a pair listed twice would add its AL term twice to both x-steps and solve its QP twice
    std::vector<long long> key((size_t)n_edges);
    for (int e = 0; e < n_edges; ++e) key[e] = (long long)edges[2 * e] * N + edges[2 * e + 1];
    std::sort(key.begin(), key.end());
    if (std::adjacent_find(key.begin(), key.end()) != key.end())
      return fail(h, PIADMM_E_ARG, "duplicate candidate pair (the same (v1, v2) twice)");
  }
  // The fused kernel (piadmm_device.hip) takes components of one agent or one pair (v, v+1);
  // any other candidate graph -- components of more agents, agents in several pairs -- runs
  // on the graph kernel (piadmm_graph.hip).  PIADMM_GRAPH=1 forces graph mode (tests).
  std::vector<int> pair_of(N, -1);
  bool simple = true;
  for (int e = 0; e < n_edges && simple; ++e) {
    const int v1 = edges[2 * e], v2 = edges[2 * e + 1];
    if (v2 != v1 + 1 || pair_of[v1] >= 0 || pair_of[v2] >= 0) simple = false;
    else pair_of[v1] = pair_of[v2] = e;
  }
  {
    const char* g = std::getenv("PIADMM_GRAPH");
    if (g && g[0] == '1') simple = false;
  }
  // the global PI law (adaptive per-pair penalties) runs on the graph kernel
  // (and a nonzero initial pair state, dual_init: the adaptive-gain script's 1e-4)
  if (h->cfg.dual_mode == PIADMM_DUAL_PI_GLOBAL || h->cfg.no_collision_gate || h->cfg.dual_init != 0.0) simple = false;
  // a sharded job with a boundary exchange runs on the graph kernel (its X / Z phases are
  // split launches around the all-reduce)
  const bool sharded = owned != nullptr;
  if (sharded) {
    if (!slot || !counted || n_slots < 0) return fail(h, PIADMM_E_ARG, "shard: null array or n_slots < 0");
    bool ghosts = false;
    for (int i = 0; i < N; ++i) {
      if (owned[i] > 1 || slot[i] < -1 || slot[i] >= n_slots)
        return fail(h, PIADMM_E_ARG, "shard: owned must be 0/1 and slot in [-1, n_slots)");
      if (!owned[i] && slot[i] < 0) return fail(h, PIADMM_E_ARG, "shard: a ghost agent needs an exchange slot");
      ghosts |= !owned[i];
    }
    for (int e = 0; e < n_edges; ++e) {
      if (counted[e] > 1) return fail(h, PIADMM_E_ARG, "shard: counted must be 0/1");
      if (!owned[edges[2 * e]] && !owned[edges[2 * e + 1]])
        return fail(h, PIADMM_E_ARG, "shard: a pair of two ghost agents (it belongs to another rank)");
    }
    if (ghosts && n_slots == 0) return fail(h, PIADMM_E_ARG, "shard: ghost agents without an exchange buffer");
    if (n_slots > 0 && !h->cfg.term_global)
      return fail(h, PIADMM_E_ARG, "shard: pairs across ranks need term_global (one stop for the whole job)");
    if (n_slots > 0) simple = false;
  }
  for (int i = 0; i < N; ++i)
    if (!std::isfinite(spd[i]) || !std::isfinite(xt0[3 * i]) || !std::isfinite(xt0[3 * i + 1]) ||
        !std::isfinite(xt0[3 * i + 2]))
      return fail(h, PIADMM_E_ARG, "non-finite speed or state");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  free_all(h);
  h->step_open = false;
  h->split = false;
  h->cap_synced = false;
  h->comp_ptr.assign(1, 0);
  h->comp_edge.clear();
  std::vector<int> nbr(N, 0);
  // graph mode: connected components labelled in order of their first agent (the oracle's
  // Scenario.components()), agent / pair lists per component, neighbour CSR sorted by
  // neighbour id (the order of the x-step's consensus sum)
  std::vector<int> g_aptr, g_alist, g_eptr, g_elist, g_nptr, g_nedge, g_ndir;
  std::vector<int> s_cptr, s_elist;     // split: pairs per original component (the residual-sum order)
  std::vector<int> pair_block;          // split: the block (workgroup) that owns each pair
  if (simple) {
    for (int a = 0; a < N;) {
      const int e = pair_of[a];
      if (e >= 0) {
        h->comp_edge.push_back(e);
        nbr[a] = nbr[a + 1] = 1;
        a += 2;
      } else {
        h->comp_edge.push_back(-1);
        a += 1;
      }
      h->comp_ptr.push_back(a);
    }
  } else {
    std::vector<int> parent(N);
    for (int a = 0; a < N; ++a) parent[a] = a;
    auto find = [&](int a) {
      while (parent[a] != a) a = parent[a] = parent[parent[a]];
      return a;
    };
    for (int e = 0; e < n_edges; ++e) {
      const int ra = find(edges[2 * e]), rb = find(edges[2 * e + 1]);
      if (ra != rb) parent[std::max(ra, rb)] = std::min(ra, rb);
    }
    std::vector<int> comp(N), id_of(N, -1);
    int C = 0;
    for (int a = 0; a < N; ++a) {
      const int r = find(a);
      if (id_of[r] < 0) id_of[r] = C++;
      comp[a] = id_of[r];
    }
    // Components of more than `block` agents (PIADMM_GRAPH_BLOCK, default 4; 0: never) span
    // several workgroups under the global scope: blocks of `block` consecutive agents (in index
    // order, numbered by first agent), the component's pairs dealt round-robin over its blocks.  The x-step
    // of an agent reads the hat / lam of pairs other blocks own and a pair reads positions of
    // agents other blocks own, so the X and Z phases run as separate launches (the kernel boundary
    // orders them); the stop test sums the blocks' partials (one job-wide decision).
    h->split = false;
    if (h->cfg.term_global && !sharded) {
      int block = 4;
      if (const char* gb = std::getenv("PIADMM_GRAPH_BLOCK")) block = std::atoi(gb);
      if (block > 0) {
        std::vector<int> csize(C, 0);
        for (int a = 0; a < N; ++a) ++csize[comp[a]];
        bool any = false;
        for (int k = 0; k < C; ++k) any |= csize[k] > block;
        if (any) {
          // the original components' pair lists (pairs in increasing index): k_graph_partials sums
          // the residual terms in this order, the reference's (casadi/main.py:165-173)
          s_cptr.assign(C + 1, 0);
          for (int e = 0; e < n_edges; ++e) ++s_cptr[comp[edges[2 * e]] + 1];
          for (int k = 0; k < C; ++k) s_cptr[k + 1] += s_cptr[k];
          s_elist.resize(n_edges);      // (here: the pair's position in the sum order)
          {
            std::vector<int> fill(s_cptr.begin(), s_cptr.end() - 1);
            for (int e = 0; e < n_edges; ++e) s_elist[e] = fill[comp[edges[2 * e]]]++;
          }
          const std::vector<int> ocomp = comp;      // original component of each agent
          std::vector<int> seen(C, 0), cur(C, -1);
          std::vector<std::vector<int>> blocks_of(C);
          int NB = 0;
          for (int a = 0; a < N; ++a) {
            const int k = comp[a];
            if (seen[k] % block == 0) {                  // a new block of component k
              cur[k] = NB++;
              blocks_of[k].push_back(cur[k]);
            }
            ++seen[k];
            comp[a] = cur[k];
          }
          // pairs dealt round-robin over the component's blocks (in pair order), so the pair QPs of
          // a densely coupled component -- an all-pairs crossing: 6 pairs of 4 agents -- run on
          // several workgroups at once instead of queueing on the first agents' blocks
          pair_block.assign(n_edges, 0);
          {
            std::vector<int> dealt(C, 0);
            for (int e = 0; e < n_edges; ++e) {
              const int k = ocomp[edges[2 * e]];
              pair_block[e] = blocks_of[k][dealt[k]++ % blocks_of[k].size()];
            }
          }
          C = NB;
          h->split = true;
        }
      }
    }
    g_aptr.assign(C + 1, 0);
    g_eptr.assign(C + 1, 0);
    for (int a = 0; a < N; ++a) ++g_aptr[comp[a] + 1];
    auto owner = [&](int e) { return h->split ? pair_block[e] : comp[edges[2 * e]]; };
    for (int e = 0; e < n_edges; ++e) ++g_eptr[owner(e) + 1];
    for (int k = 0; k < C; ++k) {
      g_aptr[k + 1] += g_aptr[k];
      g_eptr[k + 1] += g_eptr[k];
    }
    g_alist.resize(N);
    g_elist.resize(n_edges);
    {
      std::vector<int> fa(g_aptr.begin(), g_aptr.end() - 1), fe(g_eptr.begin(), g_eptr.end() - 1);
      for (int a = 0; a < N; ++a) g_alist[fa[comp[a]]++] = a;
      for (int e = 0; e < n_edges; ++e) g_elist[fe[owner(e)]++] = e;
    }
    std::vector<std::vector<std::array<int, 3>>> adj(N);
    for (int e = 0; e < n_edges; ++e) {
      const int v1 = edges[2 * e], v2 = edges[2 * e + 1];
      adj[v1].push_back({v2, e, 0});
      adj[v2].push_back({v1, e, 1});
    }
    g_nptr.assign(N + 1, 0);
    for (int a = 0; a < N; ++a) {
      std::sort(adj[a].begin(), adj[a].end());
      nbr[a] = (int)adj[a].size();
      g_nptr[a + 1] = g_nptr[a] + nbr[a];
      for (const auto& x : adj[a]) {
        g_nedge.push_back(x[1]);
        g_ndir.push_back(x[2]);
      }
    }
    h->comp_ptr = g_aptr;                  // (sizes only: agents of a component need not be contiguous)
    h->comp_edge.assign(C, -1);
  }
  h->N = N;
  h->E = n_edges;
  h->C = (int)h->comp_edge.size();
  h->T = T;
  pd::DevArgs& A = h->a;
  A = pd::DevArgs{};
  A.cfg = h->cfg;
  // PIADMM_PAIR_SOLVER=admm: pair QPs skip the dual active set and take the ADMM + PDAS path
  // (the fallback), so that tests can check both solvers against each other and the oracle
  {
    const char* ps = std::getenv("PIADMM_PAIR_SOLVER");
    A.pair_gi = (ps && std::strcmp(ps, "admm") == 0) ? 0 : 1;
    const char* pw = std::getenv("PIADMM_PAIR_WARM");
    A.pair_warm = (pw && pw[0] == '0') ? 0 : 1;
    // PIADMM_X_SOLVER: "pdas" = one-step label moves + ADMM only; "gi" = the dual active set
    // warm-started from the labels after a failed reduced solve of them; "gi_warm" = the same,
    // except that an MPC step's first x-QP skips that reduced solve (a table rebuild, ~20 us,
    // that rarely certifies); default ("gi_cold") = that first x-QP's dual active set starts
    // cold (from the unconstrained minimiser: cheaper on a wave than appending and dropping the
    // previous step's shifted rows); "gi_cold_all" = every x-step dual active set starts cold
    const char* xs = std::getenv("PIADMM_X_SOLVER");
    A.x_gi = (xs && std::strcmp(xs, "pdas") == 0) ? 0 : (xs && std::strcmp(xs, "gi") == 0) ? 1
           : (xs && std::strcmp(xs, "gi_warm") == 0) ? 2 : (xs && std::strcmp(xs, "gi_cold_all") == 0) ? 4 : 3;
    // PIADMM_NO_SPEC=1: the fused kernel's plain loop shape instead of the speculative one (the
    // two shapes' equality test)
    const char* ns = std::getenv("PIADMM_NO_SPEC");
    A.no_spec = (ns && ns[0] == '1') ? 1 : 0;
  }
  A.N = N;
  A.E = n_edges;
  A.C = h->C;
  A.T = T;
  const size_t H1 = H + 1, E = n_edges, C = h->C;
  double *d_spd, *d_ref;
  int *d_cp, *d_ce, *d_ed, *d_nb;
  int rc = 0;
  rc |= dalloc(h, &d_spd, N);
  rc |= dalloc(h, &d_ref, (size_t)N * 2 * T);
  rc |= dalloc(h, &d_cp, C + 1);
  rc |= dalloc(h, &d_ce, C);
  rc |= dalloc(h, &d_ed, 2 * E);
  rc |= dalloc(h, &d_nb, N);
  rc |= dalloc(h, &A.xt, (size_t)N * 3);
  rc |= dalloc(h, &A.u, (size_t)N * H);
  rc |= dalloc(h, &A.pos_old, (size_t)N * 2 * H1);
  rc |= dalloc(h, &A.hat, E * 4 * H1);
  rc |= dalloc(h, &A.lam, E * 4 * H1);
  rc |= dalloc(h, &A.edge_active, E);
  rc |= dalloc(h, &A.iters, C);
  // one residual-history slot per step of a persistent multi-step launch (<= 32 steps,
  // <= 64 MB of history per launch)
  {
    const size_t per_step = (size_t)C * std::max(h->cfg.max_outer, 1) * 2 * sizeof(double);
    h->step_cap = (int)std::max<size_t>(1, std::min<size_t>(32, ((size_t)64 << 20) / per_step));
  }
  rc |= dalloc(h, &A.resid, (size_t)h->step_cap * C * h->cfg.max_outer * 2);
  rc |= dalloc(h, &A.status, (size_t)N + E);
  rc |= dalloc(h, &A.Pinv_x, (size_t)N * H * H);
  rc |= dalloc(h, &A.sc_x, (size_t)N * 4 * pd::HCAP);
  rc |= dalloc(h, &A.lab_x, (size_t)N * 2 * pd::HCAP);
  A.graph = simple ? 0 : 1;
  const bool big = H > pd::HMAX || A.graph;   // graph mode: the big-mode HBM layout at every H
  rc |= dalloc(h, &A.Gx_g, big ? (size_t)N * (H * H + H) : 1);
  rc |= dalloc(h, &A.XT_g, big ? (size_t)N * H1 * pd::XLDG : 1);
  A.ke_stride = A.graph ? std::max(4 * H * H, 2 * H * pd::WAVE) : 4 * H * H;
  rc |= dalloc(h, &A.Ke_g, big ? E * A.ke_stride : 1);
  rc |= dalloc(h, &A.Yx_g, big ? (size_t)N * pd::WAVE * H : 1);
  if (h->cfg.precision == 2 && big)
    rc |= dalloc(h, &A.T32_g, (size_t)N * (H * H + H * pd::XLDG));
  rc |= dalloc(h, &A.tab_e, E * 8 * H * H);
  rc |= dalloc(h, &A.warm_ok, (size_t)N);
  rc |= dalloc(h, &A.Sacc, E * 4 * H1);
  rc |= dalloc(h, &A.Dacc, E * 4 * H1);
  rc |= dalloc(h, &A.last, E * 4 * H1);
  rc |= dalloc(h, &A.dischk, E);
  rc |= dalloc(h, &A.deff, E);
  rc |= dalloc(h, &A.qs_x, (size_t)N * 5 * pd::WAVE);
  rc |= dalloc(h, &A.ql_x, (size_t)N * 2 * pd::WAVE);
  rc |= dalloc(h, &A.qs_e, E * 12 * pd::WAVE);
  rc |= dalloc(h, &A.ql_e, E * 5 * pd::WAVE);
  rc |= dalloc(h, &A.cst, C * 4);
  rc |= dalloc(h, &h->d_part, std::max<size_t>(33, (size_t)h->cfg.max_outer * std::max(5, 2 * h->step_cap)));
  rc |= dalloc(h, &A.counters, C * 8);
  rc |= dalloc(h, &A.rho_x, (size_t)N);
  rc |= dalloc(h, &A.rho_e, E);
  rc |= dalloc(h, &A.Kx_cache, (size_t)N * H * H);
  rc |= dalloc(h, &A.xcache_rho, (size_t)N);
  rc |= dalloc(h, &A.ecache, E);
  rc |= dalloc(h, &A.gi_ws, E * (2 + pd::WAVE));
  // the wide dual active set's scratch (pair working sets beyond 63 rows, H >= 32): one region
  // per wave that solves pair QPs -- the graph kernel's GW waves, the fused kernel's pair wave
  A.gi_wide_stride = pd::giw_stride(H);
  // (over 8 GB -- hundreds of thousands of components at H >= 32 -- the wide path is off: such
  // saturated pair QPs are then reported PIADMM_QP_INEXACT, as before it existed)
  if (E > 0 && A.pair_gi && 2 * H > pd::WAVE - 1) {
    const size_t wide_n = C * (A.graph ? pd::GW : 1) * A.gi_wide_stride;
    if (wide_n * sizeof(double) <= ((size_t)8 << 30)) rc |= dalloc(h, &A.gi_wide, wide_n);
  }
  // graph mode: each pair's last dual active set (S^-1 and Y columns) for its next solve in the
  // same MPC step (pd_qp.h gi_snap_restore); PIADMM_PAIR_SNAP=0 appends the rows again instead
  {
    const char* sn = std::getenv("PIADMM_PAIR_SNAP");
    const size_t snap_n = E * ((size_t)pd::WAVE * pd::WAVE + (size_t)pd::WAVE * 2 * H + pd::WAVE);
    if (A.graph && E > 0 && A.pair_gi && !(sn && sn[0] == '0') && snap_n * sizeof(double) <= ((size_t)8 << 30))
      rc |= dalloc(h, &A.gi_snap, snap_n);
  }
  rc |= dalloc(h, &A.gpart, (size_t)2 * C * 5);
  rc |= dalloc(h, &A.gbar, (size_t)C);
  rc |= dalloc(h, &A.ghist, (size_t)h->step_cap * std::max(h->cfg.max_outer, 1) * 2);
  rc |= dalloc(h, &A.giters, (size_t)h->step_cap);
  rc |= dalloc(h, &A.gctl, 4);
  rc |= dalloc(h, &A.tie_cnt, PIADMM_TIE_KINDS);
  rc |= dalloc(h, &A.tie_n, 1);
  rc |= dalloc(h, &A.tie_ev, (size_t)PIADMM_TIE_CAP * 6);
  rc |= dalloc(h, &A.tie_mg, (size_t)PIADMM_TIE_CAP);
  A.tie_cap = PIADMM_TIE_CAP;
  A.tie_tol = h->tie_tol;
  A.tie_on = h->tie_tol > 0.0 ? 1 : 0;
  int *d_scp = nullptr, *d_sel = nullptr;
  if (h->split) {
    rc |= dalloc(h, &A.eterm, E * 2);
    rc |= dalloc(h, &d_scp, s_cptr.size());
    rc |= dalloc(h, &d_sel, E);
  }
  int *d_gap = nullptr, *d_gal = nullptr, *d_gep = nullptr, *d_gel = nullptr, *d_gnp = nullptr, *d_gne = nullptr,
      *d_gnd = nullptr;
  if (A.graph) {
    rc |= dalloc(h, &d_gap, C + 1);
    rc |= dalloc(h, &d_gal, (size_t)N);
    rc |= dalloc(h, &d_gep, C + 1);
    rc |= dalloc(h, &d_gel, E);
    rc |= dalloc(h, &d_gnp, (size_t)N + 1);
    rc |= dalloc(h, &d_gne, 2 * E);
    rc |= dalloc(h, &d_gnd, 2 * E);
    rc |= dalloc(h, &A.seed_g, (size_t)N * 2);
    rc |= dalloc(h, &A.eres, E * 2);
    rc |= dalloc(h, &A.cpart, C * 5);
    rc |= dalloc(h, &A.csig_x, (size_t)N * pd::WAVE);
    rc |= dalloc(h, &A.xflags, (size_t)N);
    rc |= dalloc(h, &A.eflags, E);
    if (h->cfg.dual_mode == PIADMM_DUAL_PI_GLOBAL) {
      rc |= dalloc(h, &A.rho_pi, E);
      rc |= dalloc(h, &A.xcache_coef, (size_t)N);
      rc |= dalloc(h, &A.ecache_rho, E);
    }
  }
  unsigned char *d_owned = nullptr, *d_counted = nullptr;
  int* d_xslot = nullptr;
  h->xchg = sharded && n_slots > 0;
  h->n_slots = h->xchg ? n_slots : 0;
  h->d_xrecv = nullptr;
  if (sharded) {
    rc |= dalloc(h, &d_owned, (size_t)N);
    rc |= dalloc(h, &d_counted, E);
    rc |= dalloc(h, &d_xslot, (size_t)N);
  }
  if (h->xchg) {
    rc |= dalloc(h, &A.xbuf, (size_t)n_slots * 3 * H1);
    rc |= dalloc(h, &h->d_xrecv, (size_t)n_slots * 3 * H1);
  }
#ifdef PIADMM_STAMPS
  rc |= dalloc(h, &A.stamps, C * 64 * 4);     // per component and wave (pd_common.h STAMP_WAVES)
#endif
  if (rc) return PIADMM_E_HIP;
  HIPCHK(h, hipMemcpyAsync(d_spd, spd, N * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(d_ref, ref, (size_t)N * 2 * T * sizeof(double), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(d_cp, h->comp_ptr.data(), (C + 1) * sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(d_ce, h->comp_edge.data(), C * sizeof(int), hipMemcpyHostToDevice, h->stream));
  if (E) HIPCHK(h, hipMemcpyAsync(d_ed, edges, 2 * E * sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(d_nb, nbr.data(), N * sizeof(int), hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipMemcpyAsync(A.xt, xt0, (size_t)N * 3 * sizeof(double), hipMemcpyHostToDevice, h->stream));
  if (A.graph) {
    h->graph_host = {g_aptr, g_alist, g_eptr, g_elist, g_nptr, g_nedge, g_ndir};   // outlive the copies
    int* dst[7] = {d_gap, d_gal, d_gep, d_gel, d_gnp, d_gne, d_gnd};
    for (int k = 0; k < 7; ++k)
      if (!h->graph_host[k].empty())
        HIPCHK(h, hipMemcpyAsync(dst[k], h->graph_host[k].data(), h->graph_host[k].size() * sizeof(int),
                                 hipMemcpyHostToDevice, h->stream));
    A.comp_aptr = d_gap;
    A.comp_alist = d_gal;
    A.comp_eptr = d_gep;
    A.comp_elist = d_gel;
    A.nbr_ptr = d_gnp;
    A.nbr_edge = d_gne;
    A.nbr_dir = d_gnd;
  }
  if (h->split) {
    h->graph_host.push_back(s_cptr);
    h->graph_host.push_back(s_elist);
    const auto& hc = h->graph_host[h->graph_host.size() - 2];
    const auto& he = h->graph_host.back();
    HIPCHK(h, hipMemcpyAsync(d_scp, hc.data(), hc.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
    if (E) HIPCHK(h, hipMemcpyAsync(d_sel, he.data(), he.size() * sizeof(int), hipMemcpyHostToDevice, h->stream));
    A.sum_cptr = d_scp;
    A.sum_pos = d_sel;
    A.sum_C = (int)hc.size() - 1;
  }
  if (sharded) {
    h->shard_host.assign(owned, owned + N);
    h->shard_host.insert(h->shard_host.end(), counted, counted + E);
    h->graph_host.push_back(std::vector<int>(slot, slot + N));
    HIPCHK(h, hipMemcpyAsync(d_owned, h->shard_host.data(), N, hipMemcpyHostToDevice, h->stream));
    if (E) HIPCHK(h, hipMemcpyAsync(d_counted, h->shard_host.data() + N, E, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(d_xslot, h->graph_host.back().data(), (size_t)N * sizeof(int), hipMemcpyHostToDevice,
                             h->stream));
    A.owned = d_owned;
    A.counted = d_counted;
    A.xslot = d_xslot;
    A.xrecv = h->d_xrecv;
    A.n_slots = h->n_slots;
  }
  if (int rc2 = reset_penalties(h)) return rc2;
  HIPCHK(h, hipMemsetAsync(A.xcache_rho, 0xff, (size_t)N * sizeof(double), h->stream));   // NaN: no cache
  if (A.xcache_coef) HIPCHK(h, hipMemsetAsync(A.xcache_coef, 0xff, (size_t)N * sizeof(double), h->stream));
  if (A.ecache_rho && E) HIPCHK(h, hipMemsetAsync(A.ecache_rho, 0xff, E * sizeof(double), h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  A.spd = d_spd;
  A.ref = d_ref;
  A.comp_ptr = d_cp;
  A.comp_edge = d_ce;
  A.edges = d_ed;
  A.nbr_cnt = d_nb;
  // natural global termination without a communicator (one rank): the stop test in-kernel
  // behind a grid barrier, when every workgroup can be resident (cooperative launch);
  // PIADMM_NO_COOP=1 keeps the host-decided path (one launch per outer iteration, the path
  // every rank of a sharded job takes, with the RCCL all-reduce) for tests and comparisons
  {
    const char* nc = std::getenv("PIADMM_NO_COOP");
    h->coop = h->cfg.term_global && !h->cfg.fixed_iters && !(nc && nc[0] == '1') && !h->xchg &&
              !h->split && (A.graph ? pd::graph_coop_fits(A, h->cfg.device) : pd::coop_fits(A, h->cfg.device));
    (void)hipGetLastError();   // a refused query must not surface as the next launch's error
  }
  h->have_scn = true;
  h->t_next = -1;
  return PIADMM_OK;
}

int32_t piadmm_set_scenario(piadmm_handle_t h, const double* spd, const double* xt0, const double* ref,
                            int32_t T, const int32_t* edges, int32_t n_edges) {
  return set_scenario_impl(h, spd, xt0, ref, T, edges, n_edges, nullptr, nullptr, 0, nullptr);
}

int32_t piadmm_set_scenario_shard(piadmm_handle_t h, const double* spd, const double* xt0, const double* ref,
                                  int32_t T, const int32_t* edges, int32_t n_edges, const uint8_t* owned,
                                  const int32_t* slot, int32_t n_slots, const uint8_t* counted) {
  if (!owned) return fail(h, PIADMM_E_ARG, "shard: null owned");
  return set_scenario_impl(h, spd, xt0, ref, T, edges, n_edges, owned, slot, n_slots, counted);
}

int32_t piadmm_set_allreduce(piadmm_handle_t h, piadmm_allreduce_fn fn, void* ctx) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (h->comm && fn) return fail(h, PIADMM_E_STATE, "the handle already has an RCCL communicator");
  h->xfn = fn;
  h->xctx = ctx;
  h->cap_synced = false;
  return PIADMM_OK;
}

int32_t piadmm_set_xt(piadmm_handle_t h, const double* xt) {
  if (!h || !xt) return fail(h, PIADMM_E_ARG, "null argument");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  h->step_open = false;
  HIPCHK(h, hipSetDevice(h->cfg.device));
  HIPCHK(h, hipMemcpyAsync(h->a.xt, xt, (size_t)h->N * 3 * sizeof(double), hipMemcpyHostToDevice, h->stream));
  // a new state breaks the receding-horizon sequence: no label warm start for the next step
  HIPCHK(h, hipMemsetAsync(h->a.warm_ok, 0, (size_t)h->N * sizeof(int), h->stream));
  if (h->E) HIPCHK(h, hipMemsetAsync(h->a.gi_ws, 0, (size_t)h->E * (2 + pd::WAVE) * sizeof(int), h->stream));
  h->t_next = -1;
  // and no carried ADMM penalties: a run from a new state starts from the configured penalty
  // (the per-scenario caches stay: they are keyed by the penalty they were built for)
  if (int rc = reset_penalties(h)) return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PIADMM_OK;
}

#define LAUNCH(h, expr)                                                                       \
  do {                                                                                        \
    if ((expr) != 0)                                                                          \
      return fail((h), PIADMM_E_HIP, std::string("kernel launch " #expr ": ") + hipGetErrorString(pd::g_launch_err)); \
  } while (0)
#define NCCLCHK(h, expr)                                                                      \
  do {                                                                                        \
    ncclResult_t _r = (expr);                                                                 \
    if (_r != ncclSuccess) return fail((h), PIADMM_E_HIP, std::string(#expr ": ") + ncclGetErrorString(_r)); \
  } while (0)

// One launch of the step kernel of the scenario's mode (fused components / general graph).
static int launch_step(const pd::DevArgs& a, int t, int n, int it0, int it1, int flags, hipStream_t s) {
  return a.graph ? pd::launch_graph_step(a, t, n, it0, it1, flags, s) : pd::launch_mpc_step(a, t, n, it0, it1, flags, s);
}

// The launches of ONE outer iteration `it` of MPC step tk under the global scope (term_global,
// the stop decided outside the kernel): one launch; or -- a sharded graph with pairs across ranks
// (SURVEY.md 8e), or a connected component split over workgroups -- an X launch (the x-steps;
// boundary agents write px | py | u to their exchange slot), ONE all-reduce of the exchange buffer
// (sharded: the ranks' slots are disjoint and zero elsewhere, so the sum is an all-gather), and a Z
// launch (ghost agents read their owner's values; every local pair -- a cross-rank pair on both of
// its ranks, bit-identically -- runs its collision test, pair QP, dual update and residual terms).
// A split component's blocks reset their pairs in a step-init launch before any block's first
// x-step reads them (casadi/main.py:52-63).
static int32_t iteration_launches(piadmm_handle_t h, int32_t tk, int it, int extra) {
  hipStream_t s = h->stream;
  int f = (it == 0 ? pd::F_FIRST : 0) | pd::F_GLOBAL | extra;
  if (h->xchg || h->split) {
    if (it == 0 && h->split) {
      LAUNCH(h, launch_step(h->a, tk, 1, 0, 0, pd::F_FIRST | pd::F_GLOBAL | pd::F_INITONLY, s));
      f &= ~pd::F_FIRST;
    }
    LAUNCH(h, launch_step(h->a, tk, 1, it, it + 1, f | pd::F_XONLY, s));
    const size_t nx = h->xchg ? (size_t)h->n_slots * 3 * (h->cfg.H + 1) : 0;
    if (int rc = allreduce(h, h->a.xbuf, h->d_xrecv, nx)) return rc;
    LAUNCH(h, launch_step(h->a, tk, 1, it, it + 1, pd::F_GLOBAL | pd::F_ZONLY | extra, s));
  } else {
    LAUNCH(h, launch_step(h->a, tk, 1, it, it + 1, f, s));
  }
  return PIADMM_OK;
}

// One MPC step under device-decided global termination (term_global with natural termination
// across ranks -- RCCL or the host transport --, a split component, or PIADMM_NO_COOP on one rank).
// Chunks of outer iterations are enqueued ahead: per iteration its launches (iteration_launches),
// the termination partials, their all-reduce and k_decide, which applies the reference's stop rules
// (casadi/main.py:115-118,174-178) on the device and sets the stop flag; launches after the stop
// return at once.  The host reads the stop state once per chunk (chunk = the previous step's
// iteration count, doubled while the step runs on), instead of one host round trip per outer
// iteration; the LAST launch takes the iteration count and the NANLAST case from the device.
static int32_t devstop_step(piadmm_handle_t h, int32_t tk, bool sync_outputs) {
  const piadmm_config_t& c = h->cfg;
  hipStream_t s = h->stream;
  const int M = c.max_outer;
  HIPCHK(h, hipMemsetAsync(h->a.gctl, 0, 4 * sizeof(int), s));
  if (!h->a.graph) LAUNCH(h, pd::launch_pair_deff(h->a, s));
  int it = 0, K = std::max(1, std::min(h->chunk_guess, M));
  while (true) {
    const int n = std::min(K, M - it);
    for (int j = 0; j < n; ++j, ++it) {
      if (int rc = iteration_launches(h, tk, it, pd::F_DEVSTOP)) return rc;
      double* part = h->d_part + (size_t)5 * it;
      LAUNCH(h, h->a.graph ? pd::launch_graph_partials(h->a, part, s, 1) : pd::launch_term_partials(h->a, it, part, s, 1));
      if (int rc = allreduce(h, part, part, 5)) return rc;
      LAUNCH(h, pd::launch_decide(h->a, tk, it, part, s));
    }
    HIPCHK(h, hipMemcpyAsync(h->h_ctl, h->a.gctl, 4 * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    if (h->h_ctl[0] || it >= M) break;
    K *= 2;
  }
  const int nit = h->h_ctl[2], nanlast = h->h_ctl[1];
  h->chunk_guess = std::max(1, nit);
  h->giters = nit;
  LAUNCH(h, launch_step(h->a, tk, 1, nit, nit, pd::F_LAST | pd::F_GLOBAL | pd::F_DEVSTOP, s));
  if (sync_outputs) {
    const int nrec = nanlast ? nit - 1 : nit;
    h->ghist.assign((size_t)2 * M, NAN);
    if (nrec > 0) {
      HIPCHK(h, hipMemcpyAsync(h->h_part, h->a.ghist, (size_t)2 * nrec * sizeof(double), hipMemcpyDeviceToHost, s));
      HIPCHK(h, hipStreamSynchronize(s));
      std::copy(h->h_part, h->h_part + 2 * nrec, h->ghist.begin());
    }
  }
  return PIADMM_OK;
}

// One outer iteration `it` of MPC step t under host-decided global termination (term_global
// without the in-kernel stop test: PIADMM_HOST_DECIDE, or host stepping): the iteration's launches,
// the job's termination partials (all-reduced), and the reference's stop rules over all agents
// (casadi/main.py:115-118,174-178; MATLAB :191-210).  flag / nanlast carry the step's state;
// *stop = 1 when the step ends at this iteration.
static int32_t global_iteration(piadmm_handle_t h, int32_t tk, int it, int& flag, int& nanlast, int* stop) {
  const piadmm_config_t& c = h->cfg;
  hipStream_t s = h->stream;
  *stop = 0;
  if (int rc = iteration_launches(h, tk, it, 0)) return rc;
  double* part = h->d_part + (size_t)5 * it;
  LAUNCH(h, h->a.graph ? pd::launch_graph_partials(h->a, part, s) : pd::launch_term_partials(h->a, it, part, s));
  if (int rc = allreduce(h, part, part, 5)) return rc;
  HIPCHK(h, hipMemcpyAsync(h->h_part, part, 5 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  const double rk = h->h_part[0], sk = h->h_part[1], n_act = h->h_part[2];
  const double n_seen = h->h_part[3], n_bad = h->h_part[4];
  if (n_act == 0.0 && flag == 0 && !c.fixed_iters) {   // no pair collides anywhere: stop (casadi/main.py:115-116)
    nanlast = 1;
    *stop = 1;
    return PIADMM_OK;
  }
  flag = 1;
  h->ghist[2 * it + 0] = rk;
  h->ghist[2 * it + 1] = sk;
  if (c.fixed_iters) return PIADMM_OK;   // throughput mode: the history only, never a stop
  host_tie(h, tk, it, PIADMM_TIE_STOP, -1, 0, rk, c.eps_pri);
  host_tie(h, tk, it, PIADMM_TIE_STOP, -1, 1, sk, c.eps_dual);
  const bool dist_ok = n_seen > 0.0 && n_bad == 0.0;
  if (rk <= c.eps_pri && sk <= c.eps_dual && (!c.term_dist_check || dist_ok)) *stop = 1;
  return PIADMM_OK;
}

// PIADMM_NO_ZX=1: a sharded job's fixed iterations as separate X and Z launches (A/B check)
static bool no_zx() {
  static const bool v = [] {
    const char* e = std::getenv("PIADMM_NO_ZX");
    return e && e[0] == '1';
  }();
  return v;
}

// MPC steps of a job whose iterations are split into X and Z launches (a sharded graph with pairs
// across ranks, or a component split over workgroups), one step at a time.  Fixed iterations: the
// steps' residual histories are all-reduced ONCE for the n steps (n x 2 x max_outer doubles), the
// same collective as run_steps' persistent launch, so ranks of one job that take different paths
// (a split component on one rank only) still issue matching collectives.
static int32_t run_steps_phases(piadmm_handle_t h, int32_t t, int32_t n, bool sync_outputs) {
  const piadmm_config_t& c = h->cfg;
  hipStream_t s = h->stream;
  const int M = c.max_outer;
  for (int k = 0; k < n; ++k) {
    const int tk = t + k;
    if (!c.fixed_iters && !h->host_decide) {
      if (int rc = devstop_step(h, tk, sync_outputs && k == n - 1)) return rc;
      continue;
    }
    h->ghist.assign((size_t)2 * M, NAN);
    int flag = 0, nit = 0, nanlast = 0;
    if (c.fixed_iters && h->xchg && !h->split && M > 1 && !no_zx()) {
      // a sharded job's fixed iterations, one launch between two exchanges: X(0), then per
      // iteration it the Z phase of it and the X phase of it+1 in ONE launch (a component is one
      // workgroup: its x-steps read only its own pairs' hat / lam), then Z(M-1) -- M + 1 launches
      // and M all-reduces per step instead of 2M launches
      const size_t nx = (size_t)h->n_slots * 3 * (c.H + 1);
      LAUNCH(h, launch_step(h->a, tk, 1, 0, 1, pd::F_FIRST | pd::F_GLOBAL | pd::F_XONLY, s));
      if (int rc = allreduce(h, h->a.xbuf, h->d_xrecv, nx)) return rc;
      for (int it = 0; it + 1 < M; ++it) {
        LAUNCH(h, launch_step(h->a, tk, 1, it, it + 2, pd::F_GLOBAL | pd::F_ZONLY | pd::F_XONLY, s));
        if (int rc = allreduce(h, h->a.xbuf, h->d_xrecv, nx)) return rc;
      }
      LAUNCH(h, launch_step(h->a, tk, 1, M - 1, M, pd::F_GLOBAL | pd::F_ZONLY, s));
      nit = M;
    } else
    for (int it = 0; it < M; ++it) {
      nit = it + 1;
      if (c.fixed_iters) {
        if (int rc = iteration_launches(h, tk, it, 0)) return rc;
        // the iteration's (rk, sk): a split component's sums in the reference's pair order
        // (k_graph_partials), a sharded graph's the blocks' partials -- the history of the step
        if (h->split) LAUNCH(h, pd::launch_graph_partials(h->a, h->d_part + (size_t)k * 2 * M + 2 * it, s, 0, 2));
        continue;
      }
      int stop = 0;
      if (int rc = global_iteration(h, tk, it, flag, nanlast, &stop)) return rc;
      if (stop) break;
    }
    h->giters = nit;
    LAUNCH(h, launch_step(h->a, tk, 1, nit, nit, pd::F_LAST | pd::F_GLOBAL | (nanlast ? pd::F_NANLAST : 0), s));
    if (c.fixed_iters && !h->split) LAUNCH(h, pd::launch_resid_history(h->a, 1, h->d_part + (size_t)k * 2 * M, s));
  }
  if (c.fixed_iters) {
    if (int rc = allreduce(h, h->d_part, h->d_part, (size_t)n * 2 * M)) return rc;
    h->giters = M;
    if (sync_outputs) {
      HIPCHK(h, hipMemcpyAsync(h->h_part, h->d_part + (size_t)(n - 1) * 2 * M, (size_t)2 * M * sizeof(double),
                               hipMemcpyDeviceToHost, s));
      HIPCHK(h, hipStreamSynchronize(s));
      h->ghist.assign(h->h_part, h->h_part + 2 * M);
    }
  }
  return PIADMM_OK;
}

// MPC steps t .. t+n-1 (n <= step_cap).  Per-component termination, or fixed iterations under
// term_global: ONE persistent launch for all n steps (each workgroup runs its component's steps
// back to back), plus, under term_global, the component-summed residual history of every step,
// all-reduced once (n x 2 x max_outer doubles).  Natural global termination: in-kernel behind a
// grid barrier (one rank, cooperative launch), else one step at a time with the stop decided on
// the device (devstop_step) or, PIADMM_HOST_DECIDE=1, on the host after every outer iteration.
static int32_t run_steps(piadmm_handle_t h, int32_t t, int32_t n, bool sync_outputs) {
  const piadmm_config_t& c = h->cfg;
  hipStream_t s = h->stream;
  const int M = c.max_outer;
  if (h->xchg || h->split) return run_steps_phases(h, t, n, sync_outputs);
  if (!c.term_global) {
    LAUNCH(h, launch_step(h->a, t, n, 0, M, pd::F_FIRST | pd::F_LAST, s));
    return PIADMM_OK;
  }
  if (c.fixed_iters) {
    LAUNCH(h, launch_step(h->a, t, n, 0, M, pd::F_FIRST | pd::F_LAST | pd::F_GLOBAL, s));
    LAUNCH(h, pd::launch_resid_history(h->a, n, h->d_part, s));
    if (int rc = allreduce(h, h->d_part, h->d_part, (size_t)n * 2 * M)) return rc;
    h->giters = M;
    if (sync_outputs) {
      const double* last = h->d_part + (size_t)(n - 1) * 2 * M;
      HIPCHK(h, hipMemcpyAsync(h->h_part, last, (size_t)2 * M * sizeof(double), hipMemcpyDeviceToHost, s));
      HIPCHK(h, hipStreamSynchronize(s));
      h->ghist.assign(h->h_part, h->h_part + 2 * M);
    }
    return PIADMM_OK;
  }
  if (h->coop && !h->comm && !h->xfn &&
      launch_step(h->a, t, n, 0, M, pd::F_FIRST | pd::F_LAST | pd::F_GLOBAL | pd::F_COOP, s) != 0) {
    (void)hipGetLastError();       // the cooperative launch was refused: host-decided path from now on
    h->coop = false;
  }
  if (h->coop && !h->comm && !h->xfn) {
    if (sync_outputs) {
      int gi = 0;
      HIPCHK(h, hipMemcpyAsync(h->h_part, h->a.ghist + (size_t)(n - 1) * 2 * M, (size_t)2 * M * sizeof(double),
                               hipMemcpyDeviceToHost, s));
      HIPCHK(h, hipMemcpyAsync(&gi, h->a.giters + (n - 1), sizeof(int), hipMemcpyDeviceToHost, s));
      HIPCHK(h, hipStreamSynchronize(s));
      h->ghist.assign(h->h_part, h->h_part + 2 * M);
      h->giters = gi;
    }
    return PIADMM_OK;
  }
  for (int k = 0; k < n; ++k) {
    const int tk = t + k;
    if (!h->host_decide) {
      if (int rc = devstop_step(h, tk, sync_outputs && k == n - 1)) return rc;
      continue;
    }
    LAUNCH(h, pd::launch_pair_deff(h->a, s));
    h->ghist.assign((size_t)2 * M, NAN);
    int flag = 0, nit = 0, nanlast = 0;
    for (int it = 0; it < M; ++it) {
      int stop = 0;
      if (int rc = global_iteration(h, tk, it, flag, nanlast, &stop)) return rc;
      nit = it + 1;
      if (stop) break;
    }
    h->giters = nit;
    LAUNCH(h, launch_step(h->a, tk, 1, nit, nit, pd::F_LAST | pd::F_GLOBAL | (nanlast ? pd::F_NANLAST : 0), s));
  }
  return PIADMM_OK;
}

// The job's ranks agree on the MPC steps per launch (the smallest): the fixed-iteration residual
// history is all-reduced once per launch, so every rank must cut a run into the same launches
// (step_cap depends on the rank's component count).  An all-gather through the sum: slot k of a
// 33-double buffer counts the ranks whose cap is k.
static int32_t sync_step_cap(piadmm_handle_t h) {
  double v[33] = {};
  v[std::min(32, std::max(1, h->step_cap))] = 1.0;
  hipStream_t s = h->stream;
  HIPCHK(h, hipMemcpyAsync(h->d_part, v, sizeof(v), hipMemcpyHostToDevice, s));   // (d_part: >= 33 doubles)
  if (int rc = allreduce(h, h->d_part, h->d_part, 33)) return rc;
  HIPCHK(h, hipMemcpyAsync(v, h->d_part, sizeof(v), hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  int cap = h->step_cap;
  for (int k = 1; k <= 32; ++k)
    if (v[k] > 0.0) {
      cap = std::min(cap, k);
      break;
    }
  h->step_cap = cap;
  h->cap_synced = true;
  return PIADMM_OK;
}

// A step at t0 that does not continue the receding-horizon sequence forgets the pairs' stored
// active sets (codes, step index, the snapshot's validity: pd_qp.h gi_solve / gi_snap_restore).
// t_next: -1 = no step yet (nothing stored), -2 = the last run failed part-way (whatever is stored
// may belong to any step: always forget it), else the step the last completed run leads to.
static int32_t continue_sequence(piadmm_handle_t h, int32_t t0) {
  if (h->t_next != -1 && t0 != h->t_next && h->E)
    HIPCHK(h, hipMemsetAsync(h->a.gi_ws, 0, (size_t)h->E * (2 + pd::WAVE) * sizeof(int), h->stream));
  return PIADMM_OK;
}

static int32_t enqueue_steps(piadmm_handle_t h, int32_t t0, int32_t n) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  if (h->step_open) return fail(h, PIADMM_E_STATE, "a host-stepped MPC step is open: piadmm_step_finish first");
  if (n < 0 || t0 < 0 || t0 + (n > 0 ? n - 1 : 0) + h->cfg.H + 1 > h->T)
    return fail(h, PIADMM_E_ARG, "time index out of the reference trajectory");
  if (n == 0) return PIADMM_OK;    // nothing runs: the stored active sets and t_next stay as they are
  HIPCHK(h, hipSetDevice(h->cfg.device));
  if (int rc = continue_sequence(h, t0)) return rc;
  if ((h->comm || h->xfn) && !h->cap_synced)
    if (int rc = sync_step_cap(h)) return rc;
  for (int i = 0; i < n;) {
    const int k = std::min(h->step_cap, n - i);
    if (int rc = run_steps(h, t0 + i, k, i + k == n)) {
      h->t_next = -2;              // part of the sequence may have run: the next step forgets the sets
      return rc;
    }
    i += k;
  }
  h->t_next = t0 + n;              // only a sequence enqueued in full continues at t0 + n
  return PIADMM_OK;
}

int32_t piadmm_mpc_steps_async(piadmm_handle_t h, int32_t t0, int32_t n_steps) {
  return enqueue_steps(h, t0, n_steps);
}

int32_t piadmm_sync(piadmm_handle_t h) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PIADMM_OK;
}

int32_t piadmm_get_state(piadmm_handle_t h, double* xt, double* u, double* pos_old, double* hat, double* lam,
                         double* S, double* D, uint8_t* edge_active, int32_t* iters) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  const int N = h->N, E = h->E, C = h->C, H = h->cfg.H, H1 = H + 1;
  HIPCHK(h, hipSetDevice(h->cfg.device));
  hipStream_t s = h->stream;
  if (xt) HIPCHK(h, hipMemcpyAsync(xt, h->a.xt, (size_t)N * 3 * 8, hipMemcpyDeviceToHost, s));
  if (u) HIPCHK(h, hipMemcpyAsync(u, h->a.u, (size_t)N * H * 8, hipMemcpyDeviceToHost, s));
  if (pos_old) HIPCHK(h, hipMemcpyAsync(pos_old, h->a.pos_old, (size_t)N * 2 * H1 * 8, hipMemcpyDeviceToHost, s));
  if (hat && E) HIPCHK(h, hipMemcpyAsync(hat, h->a.hat, (size_t)E * 4 * H1 * 8, hipMemcpyDeviceToHost, s));
  if (lam && E) HIPCHK(h, hipMemcpyAsync(lam, h->a.lam, (size_t)E * 4 * H1 * 8, hipMemcpyDeviceToHost, s));
  if (S && E) HIPCHK(h, hipMemcpyAsync(S, h->a.Sacc, (size_t)E * 4 * H1 * 8, hipMemcpyDeviceToHost, s));
  if (D && E) HIPCHK(h, hipMemcpyAsync(D, h->a.Dacc, (size_t)E * 4 * H1 * 8, hipMemcpyDeviceToHost, s));
  if (edge_active && E) HIPCHK(h, hipMemcpyAsync(edge_active, h->a.edge_active, E, hipMemcpyDeviceToHost, s));
  if (iters) HIPCHK(h, hipMemcpyAsync(iters, h->a.iters, (size_t)C * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  return PIADMM_OK;
}

// Host stepping of one MPC step, one outer iteration per call (SURVEY.md 8b piadmm_outer_iter):
// the state of casadi/main.py:78-181 after each iteration (pos_old, hat, lam and the PI
// accumulators S, D of ADMM_CVX_..._PI_antiwindup.m:160-188) is read with piadmm_get_state.
int32_t piadmm_outer_iter(piadmm_handle_t h, int32_t t, int32_t it, int32_t* stop_out) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  const piadmm_config_t& c = h->cfg;
  if (it < 0 || it >= c.max_outer) return fail(h, PIADMM_E_ARG, "it must be in [0, max_outer)");
  if (t < 0 || t + c.H + 1 > h->T) return fail(h, PIADMM_E_ARG, "time index out of the reference trajectory");
  if (it == 0) {
    HIPCHK(h, hipSetDevice(c.device));
    if (int rc = continue_sequence(h, t)) return rc;
    h->t_next = t + 1;
    h->step_open = true;
    h->step_t = t;
    h->step_flag = h->step_nanlast = h->step_stop = 0;
    h->ghist.assign((size_t)2 * c.max_outer, NAN);
  } else if (!h->step_open || t != h->step_t || it != h->step_it) {
    return fail(h, PIADMM_E_STATE, "outer_iter out of order: iterations of a step run 0, 1, 2, ...");
  } else if (h->step_stop) {
    return fail(h, PIADMM_E_STATE, "the step's stop rule already fired: piadmm_step_finish");
  }
  HIPCHK(h, hipSetDevice(c.device));
  hipStream_t s = h->stream;
  int stop = 0;
  if (c.term_global) {
    if (it == 0 && !h->a.graph) LAUNCH(h, pd::launch_pair_deff(h->a, s));
    if (int rc = global_iteration(h, t, it, h->step_flag, h->step_nanlast, &stop)) return rc;
    h->giters = it + 1;
  } else {
    // per-component stop: a component whose stop rule fired keeps its state (the kernels skip it)
    LAUNCH(h, launch_step(h->a, t, 1, it, it + 1, it == 0 ? pd::F_FIRST : 0, s));
    std::vector<int> cst((size_t)h->C * 4);
    HIPCHK(h, hipMemcpyAsync(cst.data(), h->a.cst, cst.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    stop = 1;
    for (int ci = 0; ci < h->C; ++ci) stop &= cst[(size_t)ci * 4 + 3] != 0;
  }
  h->step_it = it + 1;
  h->step_stop = stop;
  if (stop_out) *stop_out = stop;
  return PIADMM_OK;
}

int32_t piadmm_step_finish(piadmm_handle_t h, double* xt_out, double* u_out) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->step_open) return fail(h, PIADMM_E_STATE, "no host-stepped MPC step is open");
  const piadmm_config_t& c = h->cfg;
  HIPCHK(h, hipSetDevice(c.device));
  hipStream_t s = h->stream;
  const int nit = h->step_it;
  int flags = pd::F_LAST;
  if (c.term_global) flags |= pd::F_GLOBAL | (h->step_nanlast ? pd::F_NANLAST : 0);
  LAUNCH(h, launch_step(h->a, h->step_t, 1, nit, nit, flags, s));
  h->step_open = false;
  const int N = h->N, H = c.H;
  if (xt_out) HIPCHK(h, hipMemcpyAsync(xt_out, h->a.xt, (size_t)N * 3 * 8, hipMemcpyDeviceToHost, s));
  if (u_out) HIPCHK(h, hipMemcpyAsync(u_out, h->a.u, (size_t)N * H * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  return PIADMM_OK;
}

int32_t piadmm_mpc_step(piadmm_handle_t h, int32_t t, double* xt_out, double* u_out, double* resid_out,
                        int32_t* iters_out, int32_t* status_out) {
  if (int rc = enqueue_steps(h, t, 1)) return rc;
  hipStream_t s = h->stream;
  const int N = h->N, E = h->E, C = h->C, H = h->cfg.H;
  if (xt_out) HIPCHK(h, hipMemcpyAsync(xt_out, h->a.xt, (size_t)N * 3 * 8, hipMemcpyDeviceToHost, s));
  if (u_out) HIPCHK(h, hipMemcpyAsync(u_out, h->a.u, (size_t)N * H * 8, hipMemcpyDeviceToHost, s));
  if (resid_out)
    HIPCHK(h, hipMemcpyAsync(resid_out, h->a.resid, (size_t)C * h->cfg.max_outer * 2 * 8, hipMemcpyDeviceToHost, s));
  if (iters_out) HIPCHK(h, hipMemcpyAsync(iters_out, h->a.iters, (size_t)C * 4, hipMemcpyDeviceToHost, s));
  if (status_out) HIPCHK(h, hipMemcpyAsync(status_out, h->a.status, (size_t)(N + E) * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  return PIADMM_OK;
}

int32_t piadmm_time_steps(piadmm_handle_t h, int32_t t0, int32_t n_steps, float* ms_out) {
  if (!h || !ms_out) return fail(h, PIADMM_E_ARG, "null argument");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  if (int rc = enqueue_steps(h, t0, n_steps)) return rc;
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  HIPCHK(h, hipEventElapsedTime(ms_out, h->ev0, h->ev1));
  return PIADMM_OK;
}

int32_t piadmm_n_components(piadmm_handle_t h) { return h && h->have_scn ? h->C : 0; }

int32_t piadmm_steps_per_launch(piadmm_handle_t h) {
  if (!h || !h->have_scn) return 0;
  if (h->xchg || h->split) return 1;
  if (h->cfg.term_global && !h->cfg.fixed_iters) return (h->coop && !h->comm && !h->xfn) ? h->step_cap : 1;
  return h->step_cap;
}

int32_t piadmm_get_counters(piadmm_handle_t h, uint64_t* out) {
  if (!h || !out) return fail(h, PIADMM_E_ARG, "null argument");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  std::vector<unsigned long long> buf((size_t)h->C * 8);
  HIPCHK(h, hipSetDevice(h->cfg.device));
  HIPCHK(h, hipMemcpyAsync(buf.data(), h->a.counters, buf.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (int k = 0; k < 8; ++k) out[k] = 0;
  for (int c = 0; c < h->C; ++c)
    for (int k = 0; k < 8; ++k) out[k] += buf[(size_t)c * 8 + k];
  return PIADMM_OK;
}

int32_t piadmm_get_component_counters(piadmm_handle_t h, uint64_t* out, int32_t n) {
  if (!h || !out) return fail(h, PIADMM_E_ARG, "null argument");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  if (n < h->C * 8) return fail(h, PIADMM_E_ARG, "buffer too small");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  HIPCHK(h, hipMemcpyAsync(out, h->a.counters, (size_t)h->C * 8 * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PIADMM_OK;
}

int32_t piadmm_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return fail(nullptr, PIADMM_E_ARG, "null argument");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(nullptr, PIADMM_E_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return PIADMM_OK;
}

int32_t piadmm_comm_init(piadmm_handle_t h, const uint8_t* id_in, int32_t nranks, int32_t rank) {
  if (!h || !id_in) return fail(h, PIADMM_E_ARG, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(h, PIADMM_E_ARG, "bad rank / nranks");
  if (h->comm) return fail(h, PIADMM_E_STATE, "communicator already initialised");
  if (h->xfn) return fail(h, PIADMM_E_STATE, "the handle already has a host all-reduce transport");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  ncclUniqueId id;
  std::memcpy(id.internal, id_in, NCCL_UNIQUE_ID_BYTES);
  NCCLCHK(h, ncclCommInitRank(&h->comm, nranks, id, rank));
  h->nranks = nranks;
  h->rank = rank;
  h->cap_synced = false;
  return PIADMM_OK;
}

int32_t piadmm_global_resid(piadmm_handle_t h, double* resid_out, int32_t* iters_out) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->cfg.term_global) return fail(h, PIADMM_E_STATE, "term_global is off: residuals are per component");
  const int M = h->cfg.max_outer;
  if (resid_out) {
    for (int i = 0; i < 2 * M; ++i) resid_out[i] = NAN;
    for (int i = 0; i < 2 * h->giters && i < (int)h->ghist.size(); ++i) resid_out[i] = h->ghist[i];
  }
  if (iters_out) *iters_out = h->giters;
  return PIADMM_OK;
}

// Candidate pairs on a uniform grid hash (piadmm_detect.hip; casadi/main.py:110-113 at O(N)).
int32_t piadmm_candidate_pairs(piadmm_handle_t h, const double* xy, const double* radius, int32_t n,
                               int32_t* pairs_out, int32_t max_pairs, int32_t* n_pairs_out, float* ms_out) {
  if (!h || !n_pairs_out || (n > 0 && (!xy || !radius))) return fail(h, PIADMM_E_ARG, "null argument");
  if (n < 0 || n > (1 << 25)) return fail(h, PIADMM_E_ARG, "n must be in [0, 2^25]");
  if (max_pairs < 0 || (max_pairs > 0 && !pairs_out)) return fail(h, PIADMM_E_ARG, "bad pairs_out / max_pairs");
  *n_pairs_out = 0;
  if (ms_out) *ms_out = 0.0f;
  if (n == 0) return PIADMM_OK;
  (void)hipGetLastError();   // a stale error of an earlier runtime call is not this call's
  double rmax = 0.0;
  for (int i = 0; i < n; ++i) {
    if (!std::isfinite(xy[2 * i]) || !std::isfinite(xy[2 * i + 1]) || !std::isfinite(radius[i]) || radius[i] < 0)
      return fail(h, PIADMM_E_ARG, "positions and radii must be finite, radii >= 0");
    rmax = std::max(rmax, radius[i]);
  }
  // cell size >= 2 max r (a candidate pair is in the same or an adjacent cell), with margin for
  // the rounding of x / cs; buckets: a power of two >= 2n
  const double cs = rmax > 0 ? 2.0 * rmax * (1.0 + 1e-9) : 1.0;
  unsigned T = 1024;
  while (T < 2u * (unsigned)n) T <<= 1;
  HIPCHK(h, hipSetDevice(h->cfg.device));
  hipStream_t s = h->stream;
  std::vector<void*> tmp;
  auto get = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
    tmp.push_back(p);
    return p;
  };
  auto release = [&]() {
    (void)hipStreamSynchronize(s);
    for (void* p : tmp) (void)hipFree(p);
    tmp.clear();
  };
  double* d_xy = (double*)get((size_t)n * 2 * sizeof(double));
  double* d_r = (double*)get((size_t)n * sizeof(double));
  unsigned* d_key = (unsigned*)get((size_t)n * sizeof(unsigned));
  int* d_cnt = (int*)get((size_t)T * sizeof(int));
  int* d_fill = (int*)get((size_t)T * sizeof(int));
  int* d_start = (int*)get(((size_t)T + 1) * sizeof(int));
  int* d_order = (int*)get((size_t)n * sizeof(int));
  int* d_pcnt = (int*)get((size_t)n * sizeof(int));
  int* d_off = (int*)get(((size_t)n + 1) * sizeof(int));
  long long* d_total = (long long*)get(sizeof(long long));
  long long* d_bsum = (long long*)get(((size_t)T / pd::DETECT_SCAN_B + 2) * sizeof(long long));   // T >= n: the larger scan
  double* d_xs = (double*)get((size_t)n * 2 * sizeof(double));                     // bucket-ordered copies
  double* d_rs = (double*)get((size_t)n * sizeof(double));
  if (tmp.size() != 13) {
    release();
    return fail(h, PIADMM_E_HIP, "hipMalloc failed (candidate pairs)");
  }
  hipEvent_t e[4];
  for (auto& ev : e) (void)hipEventCreate(&ev);
  auto cleanup = [&]() {
    release();
    for (auto& ev : e) (void)hipEventDestroy(ev);
  };
  int rc = 0;
  long long total = 0;
  rc |= hipMemcpyAsync(d_xy, xy, (size_t)n * 2 * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess;
  rc |= hipMemcpyAsync(d_r, radius, (size_t)n * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess;
  rc |= hipEventRecord(e[0], s) != hipSuccess;
  rc |= pd::launch_detect_count(d_xy, d_r, n, 1.0 / cs, T, d_key, d_cnt, d_start, d_fill, d_order, d_pcnt, d_off,
                                d_total, d_bsum, d_xs, d_rs, s) != 0;
  rc |= hipEventRecord(e[1], s) != hipSuccess;
  rc |= hipMemcpyAsync(&total, d_total, sizeof(long long), hipMemcpyDeviceToHost, s) != hipSuccess;
  rc |= hipStreamSynchronize(s) != hipSuccess;
  if (rc) {
    cleanup();
    return fail(h, PIADMM_E_HIP, "candidate pairs: count phase failed");
  }
  if (total > 0x7fffffffll / 2) {
    cleanup();
    return fail(h, PIADMM_E_ARG, "candidate pairs: more than 2^30 pairs");
  }
  int* d_out = (int*)get((size_t)total * 2 * sizeof(int));
  if (!d_out) {
    cleanup();
    return fail(h, PIADMM_E_HIP, "hipMalloc failed (candidate pairs output)");
  }
  rc |= hipEventRecord(e[2], s) != hipSuccess;
  rc |= pd::launch_detect_emit(d_xs, d_rs, n, 1.0 / cs, T, d_start, d_order, d_off, d_out, s) != 0;
  rc |= hipEventRecord(e[3], s) != hipSuccess;
  const long long ncopy = std::min<long long>(total, max_pairs);
  if (ncopy > 0)
    rc |= hipMemcpyAsync(pairs_out, d_out, (size_t)ncopy * 2 * sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess;
  rc |= hipStreamSynchronize(s) != hipSuccess;
  float m1 = 0.0f, m2 = 0.0f;
  if (!rc && ms_out && hipEventElapsedTime(&m1, e[0], e[1]) == hipSuccess &&
      hipEventElapsedTime(&m2, e[2], e[3]) == hipSuccess)
    *ms_out = m1 + m2;
  cleanup();
  if (rc) return fail(h, PIADMM_E_HIP, "candidate pairs: emit phase failed");
  *n_pairs_out = (int32_t)total;
  return PIADMM_OK;
}

// Diagnostic builds only: per-component phase cycle sums, reset with the counters: C x 64 summed
// over the workgroup's waves, or (n >= C x 256) C x 4 x 64 per wave.
int32_t piadmm_debug_stamps(piadmm_handle_t h, uint64_t* out, int32_t n) {
  if (!h || !out) return fail(h, PIADMM_E_ARG, "null argument");
  if (!h->a.stamps) return fail(h, PIADMM_E_STATE, "library built without PIADMM_STAMPS");
  if (n < h->C * 64) return fail(h, PIADMM_E_ARG, "buffer too small");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  std::vector<uint64_t> raw((size_t)h->C * 64 * 4);
  HIPCHK(h, hipMemcpyAsync(raw.data(), h->a.stamps, raw.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (n >= h->C * 64 * 4) {
    std::copy(raw.begin(), raw.end(), out);
  } else {
    for (int ci = 0; ci < h->C; ++ci)
      for (int k = 0; k < 64; ++k) {
        uint64_t v = 0;
        for (int w = 0; w < 4; ++w) v += raw[((size_t)ci * 4 + w) * 64 + k];
        out[(size_t)ci * 64 + k] = v;
      }
  }
  return PIADMM_OK;
}

int32_t piadmm_set_tie_tolerance(piadmm_handle_t h, double tol) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!(tol >= 0.0) || !std::isfinite(tol)) return fail(h, PIADMM_E_ARG, "tie tolerance must be finite and >= 0");
  h->tie_tol = tol;
  h->a.tie_tol = tol;          // (the kernels take DevArgs by value: from the next launch on)
  h->a.tie_on = tol > 0.0 ? 1 : 0;
  return PIADMM_OK;
}

int32_t piadmm_get_near_ties(piadmm_handle_t h, uint64_t* counts, piadmm_near_tie_t* events, int32_t max_events,
                             int32_t* n_events) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  if (max_events < 0 || (max_events > 0 && !events)) return fail(h, PIADMM_E_ARG, "bad events / max_events");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  hipStream_t s = h->stream;
  unsigned long long cnt[PIADMM_TIE_KINDS];
  unsigned long long nd = 0;
  HIPCHK(h, hipMemcpyAsync(cnt, h->a.tie_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipMemcpyAsync(&nd, h->a.tie_n, sizeof(nd), hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  const int kept = (int)std::min<unsigned long long>(nd, (unsigned long long)PIADMM_TIE_CAP);
  std::vector<int> ev((size_t)kept * 6);
  std::vector<double> mg((size_t)kept);
  if (kept > 0) {
    HIPCHK(h, hipMemcpyAsync(ev.data(), h->a.tie_ev, ev.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipMemcpyAsync(mg.data(), h->a.tie_mg, mg.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
  }
  if (counts)
    for (int k = 0; k < PIADMM_TIE_KINDS; ++k) counts[k] = cnt[k] + h->host_tie_cnt[k];
  int w = 0;
  for (int i = 0; i < kept && w < max_events; ++i, ++w) {
    piadmm_near_tie_t& o = events[w];
    o.step = ev[6 * i];
    o.iter = ev[6 * i + 1];
    o.kind = ev[6 * i + 2];
    o.id = ev[6 * i + 3];
    o.index = ev[6 * i + 4];
    o.reserved = 0;
    o.margin = mg[i];
  }
  for (size_t i = 0; i < h->host_ties.size() && w < max_events; ++i, ++w) events[w] = h->host_ties[i];
  if (n_events) *n_events = w;   // events written; the totals are the per-kind counts
  return PIADMM_OK;
}

int32_t piadmm_get_step_state(piadmm_handle_t h, double* xt, double* hat, double* lam, double* S, double* D,
                              double* last_hat, double* rho_pi) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  if (h->step_open) return fail(h, PIADMM_E_STATE, "a host-stepped MPC step is open: piadmm_step_finish first");
  const size_t N = h->N, E = h->E, H1 = h->cfg.H + 1;
  HIPCHK(h, hipSetDevice(h->cfg.device));
  hipStream_t s = h->stream;
  if (xt) HIPCHK(h, hipMemcpyAsync(xt, h->a.xt, N * 3 * 8, hipMemcpyDeviceToHost, s));
  double* src[5] = {h->a.hat, h->a.lam, h->a.Sacc, h->a.Dacc, h->a.last};
  double* dst[5] = {hat, lam, S, D, last_hat};
  for (int k = 0; k < 5; ++k)
    if (dst[k] && E) HIPCHK(h, hipMemcpyAsync(dst[k], src[k], E * 4 * H1 * 8, hipMemcpyDeviceToHost, s));
  if (rho_pi && E) {
    if (h->a.rho_pi) HIPCHK(h, hipMemcpyAsync(rho_pi, h->a.rho_pi, E * 8, hipMemcpyDeviceToHost, s));
    else
      for (size_t e = 0; e < E; ++e) rho_pi[e] = h->cfg.rho;
  }
  HIPCHK(h, hipStreamSynchronize(s));
  return PIADMM_OK;
}

int32_t piadmm_set_state(piadmm_handle_t h, const double* xt, const double* hat, const double* lam, const double* S,
                         const double* D, const double* last_hat, const double* rho_pi) {
  if (!h || !xt) return fail(h, PIADMM_E_ARG, "null argument (xt is required)");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  const size_t N = h->N, E = h->E, H1 = h->cfg.H + 1;
  for (size_t i = 0; i < 3 * N; ++i)
    if (!std::isfinite(xt[i])) return fail(h, PIADMM_E_ARG, "non-finite state");
  if (rho_pi)
    for (size_t e = 0; e < E; ++e)
      if (!(rho_pi[e] > 0.0) || !std::isfinite(rho_pi[e])) return fail(h, PIADMM_E_ARG, "rho_pi must be finite and > 0");
  {
    const double* pst[5] = {hat, lam, S, D, last_hat};
    for (int k = 0; k < 5; ++k)
      if (pst[k])
        for (size_t i = 0; i < E * 4 * H1; ++i)
          if (!std::isfinite(pst[k][i])) return fail(h, PIADMM_E_ARG, "non-finite pair state");
  }
  // xt, and a fresh receding-horizon sequence (labels, warm active sets, ADMM penalties)
  if (int rc = piadmm_set_xt(h, xt)) return rc;
  HIPCHK(h, hipSetDevice(h->cfg.device));
  hipStream_t s = h->stream;
  double* dst[5] = {h->a.hat, h->a.lam, h->a.Sacc, h->a.Dacc, h->a.last};
  const double* src[5] = {hat, lam, S, D, last_hat};
  for (int k = 0; k < 5 && E; ++k) {
    if (src[k]) HIPCHK(h, hipMemcpyAsync(dst[k], src[k], E * 4 * H1 * 8, hipMemcpyHostToDevice, s));
    else HIPCHK(h, hipMemsetAsync(dst[k], 0, E * 4 * H1 * 8, s));
  }
  if (h->a.rho_pi && E) {
    std::vector<double> r(rho_pi ? rho_pi : h->rho_pi_init.data(), (rho_pi ? rho_pi : h->rho_pi_init.data()) + E);
    HIPCHK(h, hipMemcpyAsync(h->a.rho_pi, r.data(), E * 8, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipStreamSynchronize(s));
  }
  HIPCHK(h, hipStreamSynchronize(s));
  return PIADMM_OK;
}

int32_t piadmm_reset_counters(piadmm_handle_t h) {
  if (!h) return fail(nullptr, PIADMM_E_ARG, "null handle");
  if (!h->have_scn) return fail(h, PIADMM_E_STATE, "set_scenario first");
  HIPCHK(h, hipSetDevice(h->cfg.device));
  HIPCHK(h, hipMemsetAsync(h->a.counters, 0, (size_t)h->C * 8 * 8, h->stream));
  HIPCHK(h, hipMemsetAsync(h->a.tie_cnt, 0, PIADMM_TIE_KINDS * sizeof(unsigned long long), h->stream));
  HIPCHK(h, hipMemsetAsync(h->a.tie_n, 0, sizeof(unsigned long long), h->stream));
  h->host_ties.clear();
  for (auto& v : h->host_tie_cnt) v = 0;
  if (h->a.stamps) HIPCHK(h, hipMemsetAsync(h->a.stamps, 0, (size_t)h->C * 64 * 4 * 8, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return PIADMM_OK;
}

}  // extern "C"
