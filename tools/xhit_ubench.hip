// Microbenchmark of the x-step's steady-state solve (pd_qp.h qp_solve on a cached-table hit) on one
// wave: cycles (s_memtime) per call, in isolation, against the same solve inside k_mpc_step (the
// phase stamps, tools/stamps.py).  H = 30, LDS-mode layout (RM_S | RM_T: the transposed G T' / X T'
// tables), an empty working set (m = 0) whose unconstrained answer is feasible, so every call
// certifies on its first reduced solve -- exactly the path of a repeated x-step in the bench.
// Diagnostic only (tools/, never in the library).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I distributed-local-planner-pi-admm_amd/csrc \
//         tools/xhit_ubench.hip -o tools/xhit_ubench && tools/xhit_ubench
#include <cstdio>
#include <vector>

#include "pd_setup.h"
using namespace pd;

constexpr int UB_H = 30;

// OP 0: qp_solve (the agent loop's call);  OP 1: pdas<1>(1 step) = reduced_solve_x + kkt_check;
// OP 2: reduced_solve_x alone;  OP 3: kkt_check alone;  OP 4: the agent loop's x-step block
// (w', qp_solve, around(), the control's LDS store)
// CH: the horizon as a compile-time constant (else the kernel argument, as in k_mpc_step<.., 0>)
// NWV waves per workgroup, each with its own LDS regions and solve (LDS / issue contention on one CU)
constexpr size_t WAVE_LDS = gt_stride(UB_H) + HMAX * XLDT + 512 + HMAX * (HMAX + 2) + 128 + 64;
template <int OP, bool CH, int NWV = 1>
__global__ void __launch_bounds__(256) k_xhit(int reps, int Harg, unsigned long long* out, double* sink,
                                              const int* opaque) {
  extern __shared__ __attribute__((aligned(16))) double lds_all[];
  const int H = CH ? UB_H : Harg, l = lid();
  const int wv = threadIdx.x >> 6;
  double* lds = lds_all + wv * WAVE_LDS;
  double* Gt = lds;                                   // gt_stride(H)
  double* XT = Gt + gt_stride(H);                     // HMAX x XLDT
  double* vb = XT + HMAX * XLDT;                      // 512
  double* fac = vb + 512;                             // HMAX x (HMAX + 2)
  double* fdiag = fac + HMAX * (HMAX + 2);            // 128
  double* uo = fdiag + 128;                           // 64
  __shared__ int ib_all[NWV * 272];
  int* ib = ib_all + wv * 272;
  for (int i = l; i < gt_stride(H); i += 64) Gt[i] = 1e-3 / (1.0 + (i % 7));
  for (int i = l; i < HMAX * XLDT; i += 64) XT[i] = 1e-3 / (2.0 + (i % 5));
  for (int i = l; i < 512; i += 64) vb[i] = 0.0;
  __syncthreads();
  QP<1> P;
  P.H = H;
  P.n = H;
  P.umax = 0.5235987755982988;
  P.dumax = 0.3490658503988659;
  P.h0 = 0.0;
  P.g1 = P.g2 = 0.0;
  P.Pcost2 = 2.0;
  P.beta = 0.0;
  P.rho = 1.0;
  P.sigma = 1e-6;
  P.alpha = 1.6;
  P.tol = 1e-9;
  P.kready = true;
  P.scaled = true;
  P.wraw = false;
  P.Kcache = nullptr;
  P.K = nullptr;
  P.Kf = nullptr;
  P.kf32 = false;
  P.Pinv = nullptr;
  P.G = Gt;
  P.vb = vb;
  P.fac = fac;
  P.XT = XT;
  P.xld = XLDT;
  P.gmem = false;
  P.fdiag = fdiag;
  P.ib = ib;
  P.fstate = ib + 256;
  P.fld = HMAX + 1;
  P.mmax = HMAX;
  P.gws = nullptr;
  P.tstep = 0;
  P.t32 = nullptr;
  P.Y = fac;
  P.ycap = H;
  P.y_in_k = true;
  P.mm[0] = 1.0;
  P.coefP = 1.0;
  P.csig = opaque[threadIdx.x & 63];                  // 0: the tables hold the empty working set
  if (l == 0) P.fstate[0] = 0;
  double xs[1] = {0.0}, zs[2] = {0.0, 0.0}, ys[2] = {0.0, 0.0};
  piadmm_config_t cfg{};
  cfg.dt = 0.1;
  cfg.L = 2.7;
  // labels, signature and w' from memory (opaque to the compiler, as in k_mpc_step)
  signed char lab[2] = {(signed char)opaque[64 + l], (signed char)opaque[128 + l]};
  int na = 0, np = 0, ng = 0, bad = 0;
  double acc = 0.0;
  const double wq0 = 1e-2 * (l < H ? 1.0 + 0.01 * opaque[192 + l] : 0.0);
  wsync();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; ++rep) {
    if constexpr (OP == 0 || OP == 4) {
      double wq = wq0;
      if constexpr (OP == 4) wq = shdn(wq0 + acc * 1e-30, 1);
      P.wq = (l < H) ? wq : 0.0;
      P.qvalid = false;
      double ustar[1];
      const int st = qp_solve<1, false, XGEMV_U, RM_S | RM_T>(P, xs, zs, ys, lab, true, 100, 25, fac, P.fld, ustar,
                                                              na, np, ng, 0);
      bad += st;
      if constexpr (OP == 4) {
        const double u = around(ustar[0], 4);
        if (l < H) uo[l] = u;
        acc += u;
      } else {
        acc += ustar[0];
      }
    } else if constexpr (OP == 1) {
      P.wq = (l < H) ? wq0 : 0.0;
      double x[1], y[2];
      bad += pdas<1, XGEMV_U, true>(P, lab, x, y, np, 1) ? 0 : 1;
      acc += x[0];
    } else if constexpr (OP == 2) {
      P.wq = (l < H) ? wq0 : 0.0;
      double x[1], y[2];
      bad += reduced_solve_x<XGEMV_U, true>(P, lab, x, y) ? 0 : 1;
      acc += x[0];
    } else if constexpr (OP == 3) {
      // (y from memory: the multiplier checks and the wave max are not folded away)
      double x[1] = {acc * 1e-30 + 1e-3 * l}, y[2] = {1e-30 * opaque[l], 1e-30 * opaque[64 + l]};
      signed char nl[2];
      bad += kkt_check(P, lab, x, y, nl) ? 0 : 1;
      acc += x[0];
    } else if constexpr (OP == 5) {
      // reduced_solve_x + kkt_check without the pdas wrapper
      P.wq = (l < H) ? wq0 : 0.0;
      double x[1], y[2];
      signed char nl[2];
      bad += reduced_solve_x<XGEMV_U, true>(P, lab, x, y) ? 0 : 1;
      bad += kkt_check(P, lab, x, y, nl) ? 0 : 1;
      acc += x[0];
    } else if constexpr (OP == 9) {
      // the speculative x-step's lean repeat (pd_qp.h xhit_repeat) + the agent loop's rounding
      P.wq = (l < H) ? wq0 : 0.0;
      double ustar[1];
      bad += xhit_repeat<XGEMV_U>(P, lab, xs, ys, ustar, np) ? 0 : 1;
      const double u = around(ustar[0], 4);
      if (l < H) uo[l] = u;
      acc += u;
    } else if constexpr (OP == 10 || OP == 11) {
      // the speculative loop's protocol: waves 0, 1 run the lean repeat (OP 10) or nothing (OP 11)
      // between barriers A and B, every other wave only takes the two barriers
      if (OP == 10 && wv < 2) {
        P.wq = (l < H) ? wq0 : 0.0;
        double ustar[1];
        bad += xhit_repeat<XGEMV_U>(P, lab, xs, ys, ustar, np) ? 0 : 1;
        const double u = around(ustar[0], 4);
        if (l < H) uo[l] = u;
        acc += u;
      }
      __syncthreads();            // B
      acc += uo[63] * 1e-30;      // (the verdict read)
      __syncthreads();            // A
    } else if constexpr (OP == 12) {
      // a minimal replica of k_mpc_step's speculative loop (piadmm_device.hip agent_part / pair_part /
      // roll_part): waves 0, 1 the agents' lean repeat + rounding + control store; wave 2 the pair's
      // rollout of agent 0, the wait for the roller's flag, the collision test, the residual record
      // and the verdict; wave 3 the roller's rollout of agent 1 and its flag; barriers A and B
      __shared__ double s_u[2][64], s_pos[4][64];
      __shared__ int s_vd[4], s_flag;
      if (rep == 0 && threadIdx.x == 0) s_flag = 0;
      __syncthreads();                                     // A
      if (wv < 2) {
        P.wq = (l < H) ? wq0 : 0.0;
        double ustar[1];
        bad += xhit_repeat<XGEMV_U>(P, lab, xs, ys, ustar, np) ? 0 : 1;
        const double u = around(ustar[0], 4);
        if (l < H) s_u[wv][l] = u;
        acc += u;
      } else if (wv == 2) {
        double px, py, pth;
        const double u = (l < H) ? s_u[0][l] : 0.0;
        rollout_r(1.0, 2.0, 0.3, 10.0, 10.0 / 2.7, u, cfg, H, true, px, py, pth);
        if (l <= H) { s_pos[0][l] = px; s_pos[1][l] = py; }
        while (__hip_atomic_load(&s_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != rep + 1)
          __builtin_amdgcn_s_sleep(1);
        wsync();
        bool hit = false;
        if (l <= H) {
          const double dx = s_pos[0][l] - s_pos[2][l], dy = s_pos[1][l] - s_pos[3][l];
          hit = dx * dx + dy * dy < 1e-6;
        }
        const bool act = wany(hit);
        if (l == 0) {
          sink[64 + (rep & 63)] = act ? 1.0 : 0.0;         // the residual record's global store
          s_vd[0] = act; s_vd[1] = 0; s_vd[2] = 1; s_vd[3] = 0;
        }
      } else {
        double px, py, pth;
        const double u = (l < H) ? s_u[1][l] : 0.0;
        rollout_r(-1.0, 2.0, 1.3, 9.0, 9.0 / 2.7, u, cfg, H, true, px, py, pth);
        if (l <= H) { s_pos[2][l] = px; s_pos[3][l] = py; }
        if (l == 0) __hip_atomic_store(&s_flag, rep + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __syncthreads();                                     // B
      acc += s_vd[0] * 1e-30;                              // (the verdict read)
    } else if constexpr (OP == 6) {
      acc = wmax(acc + 1e-3 * opaque[192 + l]) * 1e-9;
    } else if constexpr (OP == 7) {
      acc += around(acc + 1e-3 * opaque[192 + l], 4) * 1e-9;
    } else if constexpr (OP == 8) {
      // one LDS store + wave sync + load round trip
      uo[l] = acc;
      wsync();
      acc = uo[(l + 1) & 63] * 0.5 + 1e-6;
      wsync();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = (unsigned long long)bad;
  }
  sink[threadIdx.x] = acc;
}

template <int OP, bool CH, int NWV = 1>
static void run(const char* name, int reps) {
  unsigned long long* d_out;
  double* d_sink;
  (void)hipMalloc(&d_out, 16);
  (void)hipMalloc(&d_sink, 256 * 8);
  int* d_op;
  std::vector<int> op(256, 0);
  for (int i = 0; i < 64; ++i) op[192 + i] = i;
  (void)hipMalloc(&d_op, 256 * sizeof(int));
  (void)hipMemcpy(d_op, op.data(), 256 * sizeof(int), hipMemcpyHostToDevice);
  const size_t sh = NWV * WAVE_LDS * sizeof(double);
  (void)hipFuncSetAttribute((const void*)k_xhit<OP, CH, NWV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((k_xhit<OP, CH, NWV>), dim3(1), dim3(64 * NWV), sh, 0, reps, UB_H, d_out, d_sink, d_op);
  unsigned long long h[2];
  (void)hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost);
  // s_memtime counts at the shader clock on gfx950 (the stamps' unit)
  printf("%d wave(s) %s %-34s %8.1f cycles per call  (status/failures %llu)\n", NWV, CH ? "H const  " : "H runtime", name, (double)h[0] / reps, h[1]);
  (void)hipFree(d_out);
  (void)hipFree(d_sink);
  (void)hipFree(d_op);
}

int main() {
  const int reps = 2000;
  run<3, false>("kkt_check (opaque y)", reps);
  run<5, false>("reduced_solve_x + kkt_check", reps);
  run<6, false>("wmax", reps);
  run<7, false>("around", reps);
  run<8, false>("LDS store/sync/load", reps);
  run<9, false>("xhit_repeat + round", reps);
  run<0, false>("qp_solve (hit)", reps);
  run<4, false>("x-step block (w', solve, round)", reps);
  run<1, false>("pdas 1 step", reps);
  run<2, false>("reduced_solve_x", reps);
  run<0, true>("qp_solve (hit)", reps);
  run<4, true>("x-step block (w', solve, round)", reps);
  run<2, true>("reduced_solve_x", reps);
  run<12, false, 4>("speculative-loop replica (4 waves)", reps);
  run<11, false, 4>("2 barriers, 4 waves, no work", reps);
  run<10, false, 4>("lean repeat on 2 waves + 2 barriers", reps);
  run<4, false, 2>("x-step block (w', solve, round)", reps);
  run<4, false, 4>("x-step block (w', solve, round)", reps);
  run<4, true, 2>("x-step block (w', solve, round)", reps);
  return 0;
}
