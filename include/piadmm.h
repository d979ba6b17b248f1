/*
 * piadmm.h -- C-ABI of the MI355X PI-ADMM consensus solver (libpiadmm.so).
 *
 * Drop-in boundary for the reference's per-MPC-step inner loop
 * (casadi/main.py:43-201 with the PI anti-windup dual update of
 * matlab_old_files/ADMM_CVX_two_veh_intesection_PI_antiwindup.m:152-188).
 *
 * The reference has no plugin API: its only solver seam is CasADi,
 *   F = ca.qpsol("solver", "osqp", {"x": u, "f": J(u), "g": g(u)}, opts); sol = F(lbg=0)
 * called once per agent per outer iteration (casadi/main.py:96,101) and once
 * per colliding pair (casadi/main.py:146,151), with the loop, collision test,
 * dual update, residuals and propagation in Python around it.  This library
 * replaces that whole loop for all agents at once: one call = one MPC step
 * (every outer ADMM iteration of every agent and pair), so the per-call
 * CasADi graph build + OSQP setup of the reference disappears.
 *
 * Conventions
 *   - return value: 0 on success, a negative PIADMM_E* code on failure;
 *     piadmm_last_error() gives the message.  Per-agent / per-pair QP status
 *     comes back in status_out (never silent, unlike the reference's
 *     error_on_fail=False at casadi/main.py:145).
 *   - all arrays are row-major fp64 (int32 for indices); the caller owns host
 *     arrays, the library copies them; the library owns all device memory.
 *   - a handle is bound to one HIP device and is not thread-safe.
 *   - multi-GPU = one process per GPU, each with its own handle over its shard of
 *     agents.  Whole components per rank need no data-path collective (global
 *     termination all-reduces 5 scalars per outer iteration); pairs across ranks add
 *     one all-reduce of the boundary exchange buffer per outer iteration
 *     (piadmm_set_scenario_shard).
 */
#ifndef PIADMM_H
#define PIADMM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PIADMM_ABI_VERSION 7

enum {
  PIADMM_OK = 0,
  PIADMM_E_ARG = -1,       /* bad argument / unsupported size */
  PIADMM_E_HIP = -2,       /* HIP runtime error */
  PIADMM_E_STATE = -3,     /* call out of order (e.g. step before set_scenario) */
  PIADMM_E_NODEV = -4      /* no HIP device */
};

/* dual_mode */
#define PIADMM_DUAL_PLAIN 0  /* lam += rho (p - hat)            casadi/main.py:161-162 */
#define PIADMM_DUAL_PI 1     /* per-edge PI + back-calculation  ADMM_CVX_..._PI_antiwindup.m:156-188 */
#define PIADMM_DUAL_PI_GLOBAL 2  /* PI with adaptive rho and K_P   casadi_old_PI_ADMM/main.py:133-151;
                                    with ki_adapt / d_gain / dual_init (ABI 7) the adaptive-gain
                                    variant ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m:121-147 */

/* status_out codes per agent / pair (bit flags accumulated over one MPC step) */
#define PIADMM_QP_OK 0
#define PIADMM_QP_INEXACT 1  /* a QP hit max_inner without a certified polish */
#define PIADMM_QP_NAN 2      /* a non-finite value was produced */

/* Mirror of the reference parameters: casadi/PI_ADMM_class.py:15-28 (Bunch),
 * casadi/main.py:26-27, ADMM_CVX_..._PI_antiwindup.m:6-25,43.  Field order is
 * ABI: the Python dataclass piadmm.config.PIADMMConfig has the same fields. */
typedef struct piadmm_config {
  int32_t n_agents;
  int32_t H;                 /* num_ho, 3 <= H <= 63 (H > 32: matrices in HBM / L2) */
  int32_t max_outer;         /* iter_num */
  int32_t dual_mode;
  double dt, L, dis_thres, beta, Pnorm, Pcost, rho, eps_pri, eps_dual, u_max, du_max;
  double kP, kI, theta1, theta2, windup_sat;
  int32_t windup;            /* 1: saturation + back-calculation */
  int32_t round_decimals;    /* 4 (reference np.around) or -1 */
  int32_t collide_sq_thres;  /* 0: d^2 < dis_thres (Python), 1: d^2 < dis_thres^2 (MATLAB) */
  int32_t alias_dual_residual; /* 1: Python last_iter_hat_pos aliasing (quirk B4) */
  int32_t pos_model;         /* 0: linearised pos_old (Python), 1: nonlinear (MATLAB numeric) */
  int32_t term_dist_check;   /* 1: MATLAB extra stop condition dis_vec(2) > dis_thres */
  int32_t fixed_iters;       /* 1: run exactly max_outer iterations (throughput runs) */
  int32_t max_inner;         /* ADMM iteration cap per QP */
  double admm_rho, admm_sigma, admm_alpha, qp_tol;
  int32_t polish_every;      /* PDAS polish attempt period (ADMM iterations) */
  int32_t device;            /* HIP device ordinal */
  /* ABI 2: N-agent semantics and the hot path's remaining rows */
  int32_t term_global;       /* 1: flag / termination over ALL agents of all ranks (casadi/main.py:
                                115-118,174; one RCCL all-reduce per outer iteration when sharded);
                                0: per connected component */
  int32_t warm_duals;        /* 1: hat, lam, S, D shifted one slot into the next MPC step
                                (iterate_next_state, Distributed_planner/decentralized/optimizer.py:337-344) */
  int32_t tighten;           /* 1: delay-tightened safety distance d_eff = dis_thres + |delta_i| + |delta_j|
                                (compute_square_halfspaces_ca_prob, decentralized/util.py:70-101) */
  int32_t precision;         /* 0: fp64; 1: ADMM iteration matrices K_s^-1 stored fp32 (half the LDS),
                                polish and certificate fp64 -- answers unchanged; 2 (ABI 6): the x-step's
                                parametric tables G, X' read in fp32 where they live in HBM (H > 32, or
                                the graph kernel), fp64 accumulation and ONE fp64 refinement step
                                against the exact KKT residual, then the same certificate -- answers
                                move at the 1e-7..1e-9 level (configs[4] fp32 tolerance study) */
  double tight_p, avg_delay, var_delay;   /* VehicleConfig prob / avg_delay / var_delay (veh_config.py:25-27) */
  /* ABI 3: PIADMM_DUAL_PI_GLOBAL (casadi_old_PI_ADMM/main.py:133-151), per pair from the minimum
   * distance d of the x-step plans (nonlinear rollouts): rho = clamp(rho_num / d, rho_min, rho_max)
   * (penalty of the next x-steps and pair QPs, kept across MPC steps), K_P = min(theta1 / d,
   * theta2), lam = S + K_P e, S += kI e + 2 D, saturation +-windup_sat with back-calculation D */
  double rho_num, rho_min, rho_max;
  int32_t no_collision_gate; /* 1: every candidate pair runs its pair QP every iteration (the
                                global-PI script solves the edge problem unconditionally) */
  int32_t pi_trad;           /* ABI 7 (was reserved0), PIADMM_DUAL_PI_GLOBAL: the scripts' `trad == 1`
                                branch, lam += rho e + D then the same saturation / back-calculation
                                (casadi_old_PI_ADMM/main.py:138-139, ADMM_CVX_..._adp_PI_antiwindup1.m:131-132) */
  /* ABI 7: the adaptive-gain global PI (ADMM_CVX_two_veh_intesection_adp_PI_antiwindup1.m:121-147) */
  int32_t ki_adapt;          /* 1: K_I = kI / d_min (K_I_coeff / dis_min, :127); 0: K_I = kI (casadi_old :135) */
  int32_t reserved1;
  double d_gain;             /* S += K_I e + d_gain D: 2 (casadi_old_PI_ADMM/main.py:142), 1 (adp :135).
                                Set it to 2.0 to keep ABI 6's dual_mode 2 behaviour; with dual_mode 2 a
                                zero (e.g. a zero-initialised struct) is refused with PIADMM_E_ARG */
  double dual_init;          /* hat, lam and last_hat at every MPC step's start: 0 (casadi/main.py:56-63,
                                casadi_old :49-51) or 1e-4 (adp :59-61); nonzero excludes warm_duals */
} piadmm_config_t;

typedef struct piadmm_ctx* piadmm_handle_t;

/* Library / device queries (no handle). */
int32_t piadmm_abi_version(void);
const char* piadmm_build_info(void);           /* e.g. "gfx950 hip 7.2 ..." */
int32_t piadmm_device_count(void);
int32_t piadmm_config_size(void);              /* sizeof(piadmm_config_t), for binding checks */

/* Create / destroy.  Replaces PI_ADMM_CASADI.__init__ (casadi/PI_ADMM_class.py:13-37). */
int32_t piadmm_create(const piadmm_config_t* cfg, piadmm_handle_t* out);
int32_t piadmm_destroy(piadmm_handle_t h);
const char* piadmm_last_error(piadmm_handle_t h);

/* Scenario: speeds (N), initial states (N x 3: x, y, theta), reference positions
 * (N x 2 x T, ref[i][0][t] = x, ref[i][1][t] = y; casadi/PI_ADMM_class.py:33-37)
 * and candidate pairs (E x 2, v1 < v2; any static graph: an agent's x-step sums the
 * consensus term over all its candidate neighbours, PI_ADMM_class.py:126-129, and every
 * candidate pair is collision-tested, casadi/main.py:110-113).  Resets xt to xt0. */
int32_t piadmm_set_scenario(piadmm_handle_t h, const double* spd, const double* xt0,
                            const double* ref, int32_t T, const int32_t* edges, int32_t n_edges);

/* One rank's part of a sharded job whose candidate pairs may cross ranks.
 * The arrays describe the rank's LOCAL scenario: its own agents plus a ghost copy of every
 * neighbour owned by another rank, and every pair with at least one own agent (the host
 * side, piadmm.dist.shard_graph, builds it).
 *   owned   N   1: this rank solves the agent's x-step; 0: ghost (another rank's agent)
 *   slot    N   the agent's slot in the job-wide boundary exchange buffer, -1 if none; every
 *               ghost has one, and so has every own agent with a neighbour on another rank
 *   n_slots     slots in the job (the same on every rank; 0: nothing crosses ranks)
 *   counted E   1: this rank counts the pair's residuals and termination terms (a cross-rank
 *               pair on exactly one of its ranks, e.g. the owner of v1)
 * With n_slots > 0 every outer iteration all-reduces n_slots x 3(H+1) doubles (positions and
 * controls of the boundary agents, each slot written by its owner and 0 elsewhere) between
 * the x-steps and the pair step; a cross-rank pair is solved on both of its ranks, bit-
 * identically.  Requires term_global (the job stops as one).  Transport: the RCCL
 * communicator (piadmm_comm_init) or the host callback (piadmm_set_allreduce). */
int32_t piadmm_set_scenario_shard(piadmm_handle_t h, const double* spd, const double* xt0,
                                  const double* ref, int32_t T, const int32_t* edges, int32_t n_edges,
                                  const uint8_t* owned, const int32_t* slot, int32_t n_slots,
                                  const uint8_t* counted);

/* Host all-reduce transport for jobs without RCCL (e.g. ranks sharing one GPU, or a gloo /
 * MPI host fabric): fn(ctx, buf, n) must replace buf[0..n) by its sum over all ranks of the
 * job and return 0 (non-zero aborts the step).  Used for the exchange buffer, termination
 * partials and residual histories; fn = NULL removes it. */
typedef int32_t (*piadmm_allreduce_fn)(void* ctx, double* buf, int64_t n);
int32_t piadmm_set_allreduce(piadmm_handle_t h, piadmm_allreduce_fn fn, void* ctx);

/* Overwrite the current agent states (N x 3). */
int32_t piadmm_set_xt(piadmm_handle_t h, const double* xt);

/* One MPC step at reference time index t (casadi/main.py:43-201): seeds,
 * outer ADMM loop (x-step QPs, collision graph, z-step QPs, dual update,
 * residuals, termination) and propagation of xt.  Outputs may be NULL:
 *   xt_out     N x 3        state after propagation
 *   u_out      N x H        primal_u used for propagation
 *   resid_out  C x max_outer x 2   (rk, sk) per executed iteration, NaN after
 *   iters_out  C            outer iterations executed per component
 *   status_out N + E        PIADMM_QP_* flags per agent then per pair
 * Blocking: returns after the step and the copies have finished. */
int32_t piadmm_mpc_step(piadmm_handle_t h, int32_t t, double* xt_out, double* u_out,
                        double* resid_out, int32_t* iters_out, int32_t* status_out);

/* Enqueue n_steps consecutive MPC steps starting at t0 on the handle's stream
 * without host copies or synchronisation (device-resident MPC loop: the reference's
 * `for num_step` loop, casadi/main.py:43-201).  Unless global termination with the
 * stopping test is on, up to piadmm_steps_per_launch() steps run in ONE persistent
 * launch, each component stepping through them on its own. */
int32_t piadmm_mpc_steps_async(piadmm_handle_t h, int32_t t0, int32_t n_steps);
int32_t piadmm_sync(piadmm_handle_t h);

/* Device time (ms, hipEvent on the handle's stream) of n_steps MPC steps from t0. */
int32_t piadmm_time_steps(piadmm_handle_t h, int32_t t0, int32_t n_steps, float* ms_out);

/* State of the last step, or of the last outer iteration of a host-stepped step (any pointer
 * may be NULL):
 *   xt N x 3, u N x H, pos_old N x 2 x (H+1), hat / lam / S / D E x 2 x 2 x (H+1)
 *   (direction 0 = hat_{v1 v2}, 1 = hat_{v2 v1}; S, D: the PI integral and back-calculation
 *   term of ADMM_CVX_..._PI_antiwindup.m:160-188), edge_active E, iters C.  (ABI 4: S, D added.) */
int32_t piadmm_get_state(piadmm_handle_t h, double* xt, double* u, double* pos_old,
                         double* hat, double* lam, double* S, double* D, uint8_t* edge_active, int32_t* iters);

/* Host stepping of ONE outer ADMM iteration of MPC step t (the body of
 * `for i_iter in range(iter_num)`, casadi/main.py:78-181): it = 0 starts the step (seeds, the
 * per-step reset of :52-63), it = 1, 2, ... continue it in order.  After each call
 * piadmm_get_state shows pos_old, hat, lam, S, D of that iteration.  *stop_out (may be NULL) = 1
 * when the reference's stop rules end the step at this iteration (casadi/main.py:115-118,174-178:
 * over all agents with term_global, else once every component has stopped -- a stopped
 * component keeps its state while the others continue).  Calling on after a stop, or out of
 * order, is PIADMM_E_STATE.  piadmm_step_finish then propagates (casadi/main.py:185-192); no
 * other step call is accepted while a host-stepped step is open.  (ABI 6: also a sharded graph --
 * every rank steps, the exchange all-reduce inside each call -- and a component split over
 * workgroups.) */
int32_t piadmm_outer_iter(piadmm_handle_t h, int32_t t, int32_t it, int32_t* stop_out);
int32_t piadmm_step_finish(piadmm_handle_t h, double* xt_out /* N x 3 */, double* u_out /* N x H */);

int32_t piadmm_n_components(piadmm_handle_t h);
/* MPC steps per persistent launch (after set_scenario; 1 under global natural termination). */
int32_t piadmm_steps_per_launch(piadmm_handle_t h);

/* Work counters accumulated over all steps since the last reset, summed over
 * components: [0] outer iterations executed (per component), [1] x-step QPs,
 * [2] z-step (pair) QPs, [3] ADMM iterations in x-step QPs, [4] ADMM iterations
 * in pair QPs, [5] PDAS reduced KKT solves (x), [6] PDAS reduced solves (pair),
 * [7] QPs that ended without a certified polish (PIADMM_QP_INEXACT). */
int32_t piadmm_get_counters(piadmm_handle_t h, uint64_t* out8);
int32_t piadmm_reset_counters(piadmm_handle_t h);
/* The same counters per component (C x 8 uint64, n >= 8*C). */
int32_t piadmm_get_component_counters(piadmm_handle_t h, uint64_t* out, int32_t n);

/* ABI 6: near-tie log.  The reference's loop takes discrete decisions --
 * rounding to round_decimals (casadi/main.py:48-49,103,153), the collision test d^2 < thr
 * (:112-113), the stop test rk <= eps_pri, sk <= eps_dual (:174) and MATLAB's distance check
 * dis_vec(2) > dis_thres (ADMM_CVX_..._PI_antiwindup.m:202).  Two exact implementations (this
 * library, a CPU port, the reference) agree on every continuous value to rounding, so their
 * trajectories can part only where such a decision falls within rounding of its threshold.  The
 * library records, once piadmm_set_tie_tolerance(h, tol > 0) has turned the log on, every decision
 * taken within `tol` of its threshold (1e-9 is a good choice; tol = 0, the default, turns it off:
 * the kernels then run an instantiation without the checks -- the log costs 3-10 % of a step):
 *   PIADMM_TIE_ROUND_U     an x-step control        id = agent, index = horizon slot k
 *   PIADMM_TIE_ROUND_UHAT  a pair (edge) control    id = pair,  index = side * H + k
 *   PIADMM_TIE_ROUND_SEED  a seed                   id = agent, index = 0 (x) / 1 (y)
 *     margin = value - nearest rounding boundary (k + 1/2) 10^-d, absolute, |margin| <= tol
 *   PIADMM_TIE_COLLIDE     the collision test       id = pair, index = closest slot k,
 *     margin = (min_k d_k^2 - thr) / thr (relative)
 *   PIADMM_TIE_STOP        the stop test            id = component (-1: the job under term_global),
 *     index 0: rk vs eps_pri, 1: sk vs eps_dual, margin = (r - eps) / eps (relative)
 *   PIADMM_TIE_DIST        the distance check       id = pair (-1: unknown), margin = (d - d_eff) / d_eff
 * Each event carries the reference time index of the MPC step and the outer iteration (-1: the
 * step's seeds).  Counts and events accumulate until piadmm_reset_counters; the counts are the
 * totals, and at most PIADMM_TIE_CAP device events (the kernels' decisions) plus PIADMM_TIE_CAP host
 * events (the host's stop decisions) are kept.  *n_events = the number of events written to
 * `events` (<= max_events). */
#define PIADMM_TIE_ROUND_U 0
#define PIADMM_TIE_ROUND_UHAT 1
#define PIADMM_TIE_ROUND_SEED 2
#define PIADMM_TIE_COLLIDE 3
#define PIADMM_TIE_STOP 4
#define PIADMM_TIE_DIST 5
#define PIADMM_TIE_KINDS 6
#define PIADMM_TIE_CAP 4096
typedef struct piadmm_near_tie {
  int32_t step, iter, kind, id, index, reserved;
  double margin;
} piadmm_near_tie_t;
int32_t piadmm_set_tie_tolerance(piadmm_handle_t h, double tol);
int32_t piadmm_get_near_ties(piadmm_handle_t h, uint64_t* counts /* PIADMM_TIE_KINDS, may be NULL */,
                             piadmm_near_tie_t* events /* may be NULL */, int32_t max_events, int32_t* n_events);

/* ABI 6: checkpoint / resume.  The state that carries from one MPC step to the
 * next: xt (N x 3) and, for warm_duals (a12) and the global-PI law, hat / lam / S / D / last_hat
 * (E x 2 x 2 x (H+1), the layout of piadmm_get_state; last_hat = last_iter_hat_pos,
 * casadi/main.py:180) and the global-PI pair penalties rho_pi (E).  piadmm_get_step_state reads it
 * after a step; piadmm_set_state writes it before the next (any pointer but xt may be NULL: that
 * part is zeroed, as at the reference's per-step reset, casadi/main.py:52-63; rho_pi NULL: the
 * configured rho).  A run resumed from a checkpoint continues like the uninterrupted one, to
 * rounding: the QP solvers' warm starts (active sets, labels) are not part of the checkpoint, and
 * they are guesses only -- every answer is the certified minimiser of the same QP. */
int32_t piadmm_get_step_state(piadmm_handle_t h, double* xt, double* hat, double* lam, double* S, double* D,
                              double* last_hat, double* rho_pi);
int32_t piadmm_set_state(piadmm_handle_t h, const double* xt, const double* hat, const double* lam,
                         const double* S, const double* D, const double* last_hat, const double* rho_pi);

/* Multi-GPU (term_global): one process per GPU, one handle each, joined by an RCCL
 * communicator over xGMI.  Rank 0 calls piadmm_comm_unique_id and ships the 128 bytes to
 * the other ranks (any out-of-band channel); every rank then calls piadmm_comm_init.
 * mpc_step then all-reduces the termination partials (rk, sk, active pairs, distance
 * checks) once per outer iteration, or, with fixed_iters, the residual history once per
 * MPC step, and, for a sharded graph (piadmm_set_scenario_shard), the boundary exchange
 * buffer once per outer iteration.  Without a communicator (or host transport) the
 * handle is a single-rank job. */
int32_t piadmm_comm_unique_id(uint8_t* id_out /* 128 bytes */);
int32_t piadmm_comm_init(piadmm_handle_t h, const uint8_t* id /* 128 bytes */, int32_t nranks, int32_t rank);

/* Global residual history of the last step (term_global): max_outer x 2 (rk, sk summed over
 * every active pair of every rank, NaN after the last executed iteration) and the number of
 * executed outer iterations (equal on every rank). */
int32_t piadmm_global_resid(piadmm_handle_t h, double* resid_out, int32_t* iters_out);

/* Candidate pairs for large N: all pairs i < j of the n points
 * xy (n x 2) with |xy_i - xy_j| <= radius_i + radius_j, in increasing (i, j) order, found on a
 * uniform grid hash in O(n) on the handle's device (replaces the O(N^2) pair loop of
 * casadi/main.py:110-113 as the source of the candidate graph).  With radius_i the reach bound
 * of piadmm.candidates.reach_radii no other pair can collide within the horizon: for the
 * linearised position model (pos_model 0) it is sum_k dt s sqrt(1 + (k dt s u_max / L)^2) plus half
 * the collision distance (and the delay offset with tighten) -- NOT the constant-speed s H dt,
 * which the linearised rollout can exceed.
 * Writes min(total, max_pairs) pairs to pairs_out (max_pairs x 2) and the total to
 * *n_pairs_out (call again with a larger buffer when total > max_pairs); ms_out (may be NULL):
 * device time of the detection kernels, inputs resident. */
int32_t piadmm_candidate_pairs(piadmm_handle_t h, const double* xy, const double* radius, int32_t n,
                               int32_t* pairs_out, int32_t max_pairs, int32_t* n_pairs_out, float* ms_out);

/* Diagnostic builds (-DPIADMM_STAMPS, libpiadmm_stamps.so) only: per-component
 * cycle sums of the kernel phases (C x 32 uint64); PIADMM_E_STATE otherwise. */
int32_t piadmm_debug_stamps(piadmm_handle_t h, uint64_t* out, int32_t n);

/* ---- OBCA local subproblem ------------------------------------------
 * Replaces the vehicle side of the OBCA-ADMM planner: OBCAOptimizer.local_initialize,
 * local_build_model, local_generate_constrain, local_generate_variable, local_generate_object and
 * local_solve (Distributed_planner/decentralized/optimizer.py:40-201) -- one CasADi/IPOPT NLP per
 * vehicle per ADMM iterate (decentralized_overtaking_ADMM.py:49-63) -- with a batched SQP on the
 * device: n independent local NLPs (kinematic bicycle, N_horz 8, OBCA dual-distance constraints
 * against the other vehicle's exchanged halfspaces), one wavefront each, one launch.
 *
 * recs: n x PIADMM_OBCA_REC fp64 records, each
 *   init[5] | ref[8][5] (ref_traj[veh][t_step + k]) | A_o[7][4][2] | b_o[7][4] | lamb_ij_o[7][4]
 *   (bar_state.A/b/lamb_ij of the OTHER vehicle) | lamb_bar[7][9] | Z_bar[7][9] (this vehicle's) |
 *   rho, min_dis, max_x, max_y, r, q, prob (0/1: util.py:48-68 or :70-101 halfspaces),
 *   max_sqp_iters | pad.
 * out: n x PIADMM_OBCA_OUT fp64: X[8][5] | U[7][2] | Lambda[7][4] (local_solve's x_opt..steer_opt,
 *   a_opt, steerate_opt, lambda_loc, :183-201) | multipliers y_a[7] y_b[7][2] y_n[7] y_x[7][5]
 *   pi[7][5] y_u[14] y_l[28] | cost | pad.
 * status3: n x 3 int32: PIADMM_OBCA_* status, SQP iterations, QP active-set steps.
 * The NLP is the reference's as written; the solver is not IPOPT. */
#define PIADMM_OBCA_REC 296
#define PIADMM_OBCA_OUT 224
#define PIADMM_OBCA_CONVERGED 0
#define PIADMM_OBCA_MAX_ITER 1
#define PIADMM_OBCA_QP_INFEASIBLE 2
#define PIADMM_OBCA_LINESEARCH_FAIL 3
#define PIADMM_OBCA_HESSIAN_FAIL 4

typedef struct piadmm_obca_s* piadmm_obca_t;
int32_t piadmm_obca_create(int32_t device, piadmm_obca_t* out);
int32_t piadmm_obca_destroy(piadmm_obca_t h);
const char* piadmm_obca_last_error(piadmm_obca_t h);
/* upload + one launch + download (synchronous) */
int32_t piadmm_obca_solve(piadmm_obca_t h, const double* recs, int32_t n, double* out, int32_t* status3);
/* resident batch: upload once, launch, time, download.  Block b of a launch solves problem
 * order[b]: longest first by the QP steps each problem took in the previous run of the SAME upload
 * (index order on the first run after an upload), so the longest problems start in the first
 * dispatch wave; the answers do not depend on the order.  piadmm_obca_run blocks: it reads the
 * previous run's per-problem work back to the host (a device-to-host copy and stream syncs) and
 * uploads the order before it enqueues its launches, which then run asynchronously on the handle's
 * stream (piadmm_obca_download / _time synchronise). */
int32_t piadmm_obca_upload(piadmm_obca_t h, const double* recs, int32_t n);
int32_t piadmm_obca_run(piadmm_obca_t h, int32_t repeats);
int32_t piadmm_obca_time(piadmm_obca_t h, int32_t repeats, float* ms_per_launch);
int32_t piadmm_obca_download(piadmm_obca_t h, double* out, int32_t* status3, int32_t n);
/* Diagnostic builds (-DPIADMM_STAMPS) only: per-problem cycle sums of the SQP phases and event
 * counts of the last launch (n = 16 x batch uint64); PIADMM_E_STATE otherwise. */
int32_t piadmm_obca_debug_stamps(piadmm_obca_t h, uint64_t* out, int32_t n);

#ifdef __cplusplus
}
#endif

#endif /* PIADMM_H */
