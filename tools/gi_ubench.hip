// Microbenchmark of the dual active set's per-step LDS passes (pd_qp.h gi_solve) on one wave:
// cycles (s_memtime) per call of S^-1 v, the Y axpy, the bordering update of an append and the
// downdate of a drop, at working-set sizes m.  Diagnostic only (tools/, never in the library).
//   hipcc -O3 --offload-arch=gfx950 -I include -I distributed-local-planner-pi-admm_amd/csrc \
//         tools/gi_ubench.hip -o tools/gi_ubench && tools/gi_ubench
#include <cstdio>
#include <vector>

#include "pd_qp.h"
using namespace pd;

constexpr int UB_H = 30;
constexpr int LDT = 66;                   // row-contiguous S^-1: stride 528 B (4 banks mod 64)
constexpr int LDY = 66;                   // transposed Y: per variable, the m coefficients contiguous
constexpr size_t UB_LDS = (64 * LDT + 2 * UB_H * LDY + 256) * sizeof(double);
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) dv2 ldsd2;

template <int OP>
__global__ void __launch_bounds__(64) k_ub(int m, int reps, unsigned long long* out, double* sink) {
  extern __shared__ double lds[];
  double* Si = lds;
  double* Y = lds + 64 * LDT;
  double* vbuf = Y + 2 * UB_H * LDY;
  ldsd* Yl = lds_ptr(Y);
  const int l = lid();
  for (int i = l; i < 64 * LDT; i += 64) Si[i] = 1.0 / (1.0 + (i % 13));
  for (int i = l; i < 2 * UB_H * LDY; i += 64) Y[i] = 1.0 / (2.0 + (i % 11));
  for (int i = l; i < 256; i += 64) vbuf[i] = 0.0;
  __syncthreads();
  ldsd* Sil = lds_ptr(Si);
  ldsd* vbl = lds_ptr(vbuf);
  double v = 1e-3 * l, z[2] = {0.0, 0.0};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; ++rep) {
    if (OP == 0) {
      v = sinv_gemv(Si, LD, vbuf, v, m) * 1e-3 + 1e-4;
    } else if (OP == 1) {
      y_axpy<2>(Y, UB_H, vbuf, v, m, z);
      v = z[0] * 1e-3 + 1e-4;
    } else if (OP == 2) {
      // append's bordering of S^-1 (r at lanes < m, one row + column)
      const double id = 1.0 / (1.0 + v * v);
      put_bcast(vbl, v, m);
      if (l < m) {
        const double rl = v * id;
        ldsd* col = Sil + l;
        const int mu = unif(m), ldu = unif(LD);
        for (int j0 = 0; j0 < mu; j0 += SINV_U) {
          double sv[SINV_U], rv[SINV_U];
#pragma unroll
          for (int u = 0; u < SINV_U; ++u) {
            sv[u] = col[unif(min(j0 + u, mu - 1) * ldu)];
            rv[u] = vbl[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < SINV_U; ++u)
            if (j0 + u < mu) col[unif((j0 + u) * ldu)] = sv[u] * 0.5 + rv[u] * rl;
        }
        Sil[m * LD + l] = -rl;
        Sil[l * LD + m] = -rl;
      }
      wsync();
      v = v * 0.999 + 1e-4;
    } else if (OP == 3) {
      // a full GI step without the search: S^-1 v, Y axpy, two reductions, bordering
      const double va = v;
      const double r = sinv_gemv(Si, LD, vbuf, va, m);
      y_axpy<2>(Y, UB_H, vbuf, r, m, z);
      const double lpp2 = 1.0 + wsum(va * r);
      const double tdrop = (l < m && r > 0.0) ? 0.5 / r : INFINITY;
      const double t1 = wmin(tdrop);
      v = (r + z[0] * 1e-3) * 1e-3 / lpp2 + fmin(t1, 1.0) * 1e-6;
    } else if (OP == 9 || OP == 12) {
      // S^-1 v along rows at the odd stride LD (8-byte alignment: paired ds_read2_b64)
      const double va = v;
      put_bcast(vbl, va, m);
      const ldsd* row = Sil + ((l < m) ? l : 0) * LD;
      double a0 = 0.0, a1 = 0.0;
      const int mu = unif(m);
      for (int j0 = 0; j0 < mu; j0 += 8) {
        double sv[8], wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          sv[u] = row[j0 + u];
          wv[u] = vbl[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
          a0 += sv[u] * wv[u];
          a1 += sv[u + 1] * wv[u + 1];
        }
      }
      wsync();
      const double r = (l < m) ? a0 + a1 : 0.0;
      if (OP == 9) {
        v = r * 1e-3 + 1e-4;
      } else {
        put_bcast(vbl, r, m);
        const int lc = (l < UB_H) ? l : 0;
        const ldsd* y0 = Yl + lc * LD;
        const ldsd* y1 = Yl + (UB_H + lc) * LD;
        for (int b0 = 0; b0 < mu; b0 += 8) {
          double p[8], q[8], c[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            c[u] = vbl[b0 + u];
            p[u] = y0[b0 + u];
            q[u] = y1[b0 + u];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            z[0] -= c[u] * p[u];
            z[1] -= c[u] * q[u];
          }
        }
        wsync();
        const double lpp2 = 1.0 + wsum(va * r);
        const double tdrop = (l < m && r > 0.0) ? 0.5 / r : INFINITY;
        const double t1 = wmin(tdrop);
        v = (r + z[0] * 1e-3) * 1e-3 / lpp2 + fmin(t1, 1.0) * 1e-6;
      }
    } else if (OP == 10) {
      // bordering along rows at the odd stride LD
      const double id = 1.0 / (1.0 + v * v);
      put_bcast(vbl, v, m);
      if (l < m) {
        const double rl = v * id;
        ldsd* row = Sil + l * LD;
        const int mu = unif(m);
        for (int j0 = 0; j0 < mu; j0 += 8) {
          double sv[8], wv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            sv[u] = row[j0 + u];
            wv[u] = vbl[j0 + u];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (j0 + u < mu) row[j0 + u] = sv[u] * 0.5 + wv[u] * rl;
        }
        Sil[l * LD + m] = -rl;
        Sil[m * LD + l] = -rl;
      }
      wsync();
      v = v * 0.999 + 1e-4;
    } else if (OP == 11) {
      // Y axpy, Y transposed at the odd stride LD
      put_bcast(vbl, v, m);
      const int lc = (l < UB_H) ? l : 0;
      const ldsd* y0 = Yl + lc * LD;
      const ldsd* y1 = Yl + (UB_H + lc) * LD;
      const int mu = unif(m);
      for (int b0 = 0; b0 < mu; b0 += 8) {
        double p[8], q[8], c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          c[u] = vbl[b0 + u];
          p[u] = y0[b0 + u];
          q[u] = y1[b0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          z[0] -= c[u] * p[u];
          z[1] -= c[u] * q[u];
        }
      }
      wsync();
      v = z[0] * 1e-3 + 1e-4;
    } else if (OP == 4 || OP == 8) {
      // S^-1 v, lane = row, the row contiguous (stride LDT), 16-byte loads; vector broadcast
      // from LDS in 16-byte loads (OP 4, batches of 8) or 16 (OP 8)
      constexpr int U = OP == 4 ? 8 : 16;
      put_bcast(vbl, v, m);
      const ldsd2* row = (const ldsd2*)(Sil + ((l < m) ? l : 0) * LDT);
      const ldsd2* vv2 = (const ldsd2*)vbl;
      double a0 = 0.0, a1 = 0.0;
      const int mu = unif(m);
      for (int j0 = 0; j0 < mu; j0 += U) {
        dv2 sv[U / 2], wv[U / 2];
#pragma unroll
        for (int u = 0; u < U / 2; ++u) {
          sv[u] = row[(j0 >> 1) + u];
          wv[u] = vv2[(j0 >> 1) + u];
        }
#pragma unroll
        for (int u = 0; u < U / 2; ++u) {
          a0 += sv[u].x * wv[u].x;
          a1 += sv[u].y * wv[u].y;
        }
      }
      wsync();
      v = ((l < m) ? a0 + a1 : 0.0) * 1e-3 + 1e-4;
    } else if (OP == 5) {
      // Y axpy, Y transposed per vehicle (lane = variable, the m coefficients contiguous)
      put_bcast(vbl, v, m);
      const int lc = (l < UB_H) ? l : 0;
      const ldsd2* y0 = (const ldsd2*)(Yl + lc * LDY);
      const ldsd2* y1 = (const ldsd2*)(Yl + (UB_H + lc) * LDY);
      const ldsd2* vv2 = (const ldsd2*)vbl;
      const int mu = unif(m);
      for (int a0 = 0; a0 < mu; a0 += 8) {
        dv2 p[4], q[4], c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          c[u] = vv2[(a0 >> 1) + u];
          p[u] = y0[(a0 >> 1) + u];
          q[u] = y1[(a0 >> 1) + u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          z[0] -= c[u].x * p[u].x + c[u].y * p[u].y;
          z[1] -= c[u].x * q[u].x + c[u].y * q[u].y;
        }
      }
      wsync();
      v = z[0] * 1e-3 + 1e-4;
    } else if (OP == 6) {
      // bordering, row-contiguous layout, 16-byte loads and stores
      const double id = 1.0 / (1.0 + v * v);
      put_bcast(vbl, v, m);
      if (l < m) {
        const double rl = v * id;
        ldsd2* row = (ldsd2*)(Sil + l * LDT);
        const ldsd2* vv2 = (const ldsd2*)vbl;
        const int mu = unif(m);
        for (int j0 = 0; j0 < mu; j0 += 8) {
          dv2 sv[4], wv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            sv[u] = row[(j0 >> 1) + u];
            wv[u] = vv2[(j0 >> 1) + u];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            sv[u].x = sv[u].x * 0.5 + wv[u].x * rl;
            sv[u].y = sv[u].y * 0.5 + wv[u].y * rl;
            if (j0 + 2 * u < mu) row[(j0 >> 1) + u] = sv[u];   // (pairs past m: padding columns)
          }
        }
        Sil[l * LDT + m] = -rl;
        Sil[m * LDT + l] = -rl;
      }
      wsync();
      v = v * 0.999 + 1e-4;
    } else if (OP == 7) {
      // the GI step on the transposed layouts
      const double va = v;
      put_bcast(vbl, va, m);
      const ldsd2* row = (const ldsd2*)(Sil + ((l < m) ? l : 0) * LDT);
      const ldsd2* vv2 = (const ldsd2*)vbl;
      double a0 = 0.0, a1 = 0.0;
      const int mu = unif(m);
      for (int j0 = 0; j0 < mu; j0 += 8) {
        dv2 sv[4], wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          sv[u] = row[(j0 >> 1) + u];
          wv[u] = vv2[(j0 >> 1) + u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a0 += sv[u].x * wv[u].x;
          a1 += sv[u].y * wv[u].y;
        }
      }
      wsync();
      const double r = (l < m) ? a0 + a1 : 0.0;
      put_bcast(vbl, r, m);
      const int lc = (l < UB_H) ? l : 0;
      const ldsd2* y0 = (const ldsd2*)(Yl + lc * LDY);
      const ldsd2* y1 = (const ldsd2*)(Yl + (UB_H + lc) * LDY);
      for (int b0 = 0; b0 < mu; b0 += 8) {
        dv2 p[4], q[4], c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          c[u] = vv2[(b0 >> 1) + u];
          p[u] = y0[(b0 >> 1) + u];
          q[u] = y1[(b0 >> 1) + u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          z[0] -= c[u].x * p[u].x + c[u].y * p[u].y;
          z[1] -= c[u].x * q[u].x + c[u].y * q[u].y;
        }
      }
      wsync();
      const double lpp2 = 1.0 + wsum(va * r);
      const double tdrop = (l < m && r > 0.0) ? 0.5 / r : INFINITY;
      const double t1 = wmin(tdrop);
      v = (r + z[0] * 1e-3) * 1e-3 / lpp2 + fmin(t1, 1.0) * 1e-6;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (l == 0) out[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + l] = v + z[0] + z[1];
}

template <int OP>
static void run(const char* name, int m, int reps, unsigned long long* d_out, double* d_sink) {
  auto fn = k_ub<OP>;
  hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)UB_LDS);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(fn, dim3(1), dim3(64), UB_LDS, 0, m, 16, d_out, d_sink);
  hipEventRecord(e0);
  hipLaunchKernelGGL(fn, dim3(1), dim3(64), UB_LDS, 0, m, reps, d_out, d_sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long cyc = 0;
  hipMemcpy(&cyc, d_out, sizeof(cyc), hipMemcpyDeviceToHost);
  printf("%-10s m=%2d  %8.1f memtime/call  %7.1f ns/call\n", name, m, (double)cyc / reps, 1e6 * ms / reps);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  unsigned long long* d_out;
  double* d_sink;
  hipMalloc(&d_out, 64 * sizeof(unsigned long long));
  hipMalloc(&d_sink, 64 * 64 * sizeof(double));
  const int reps = 20000;
  for (int m : {8, 16, 32, 50, 63}) {
    run<0>("sinv_gemv", m, reps, d_out, d_sink);
    run<1>("y_axpy", m, reps, d_out, d_sink);
    run<2>("border", m, reps, d_out, d_sink);
    run<3>("gi_step", m, reps, d_out, d_sink);
    run<4>("T sinv", m, reps, d_out, d_sink);
    run<9>("R sinv", m, reps, d_out, d_sink);
    run<10>("R border", m, reps, d_out, d_sink);
    run<11>("R y_axpy", m, reps, d_out, d_sink);
    run<12>("R gi_step", m, reps, d_out, d_sink);
    run<5>("T y_axpy", m, reps, d_out, d_sink);
    run<6>("T border", m, reps, d_out, d_sink);
    run<7>("T gi_step", m, reps, d_out, d_sink);
  }
  hipFree(d_out);
  hipFree(d_sink);
  return 0;
}
