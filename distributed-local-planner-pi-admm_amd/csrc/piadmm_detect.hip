// piadmm_detect.hip -- candidate-pair detection on a uniform grid hash (MI355X, gfx950).
//
// The reference tests every pair of vehicles for a collision in every outer iteration
// (casadi/main.py:110-113: edge_mat[i, j] = any_k |p_i,k - p_j,k|^2 < dis_thres, O(N^2 H)); the
// solver here takes a static candidate graph.  This builds it for large N in O(N): pairs
// (i < j) with |p_i - p_j| <= r_i + r_j.  With p the agents' positions at the start of an MPC
// step and r_i = s_i H dt + d/2 (reach of a constant-speed agent over the horizon plus half the
// collision distance) no pair outside the list can collide within the horizon
// (piadmm.candidates.reach_radii), so the collision test over the candidates is the reference's
// all-pairs test.  SURVEY.md 8f rank 2.
//
// Integer / byte work, HBM- and latency-bound: no MFMA.  Agents are hashed to the cells of a
// grid of cell size cs >= 2 max r (a candidate pair lies in the same or an adjacent cell), a
// counting sort groups them by hash bucket (atomics + one-workgroup scans), each agent scans the
// buckets of its 3 x 3 neighbourhood twice (count, emit) and sorts its own partner list, so the
// output is in (i, j) order, independent of the atomics' order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "piadmm_internal.h"

namespace pd {

namespace {

constexpr int DT = 256;   // threads per workgroup of the per-agent kernels

__device__ __forceinline__ long long cell_of(double v, double inv_cs) {
  double c = floor(v * inv_cs);
  c = fmin(fmax(c, -4.0e18), 4.0e18);
  return (long long)c;
}

__device__ __forceinline__ unsigned bucket_of(long long cx, long long cy, unsigned mask) {
  const unsigned long long h = (unsigned long long)cx * 0x9E3779B97F4A7C15ull ^
                               (unsigned long long)cy * 0xC2B2AE3D27D4EB4Full;
  return (unsigned)((h ^ (h >> 29)) & mask);
}

__global__ void __launch_bounds__(DT) k_hash(const double* xy, int n, double inv_cs, unsigned mask, unsigned* key,
                                             int* cnt) {
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= n) return;
  const unsigned k = bucket_of(cell_of(xy[2 * i], inv_cs), cell_of(xy[2 * i + 1], inv_cs), mask);
  key[i] = k;
  atomicAdd(&cnt[k], 1);
}

// Exclusive scan of m ints in one workgroup (1024 threads, each a contiguous chunk); out[m] =
// total.  m <= a few million: one pass over HBM each way.
__global__ void __launch_bounds__(1024) k_scan(const int* in, int m, int* out, long long* total) {
  __shared__ long long part[1024];
  const int t = threadIdx.x;
  const int chunk = (m + 1023) / 1024;
  const int a = min(m, t * chunk), b = min(m, a + chunk);
  long long s = 0;
  for (int i = a; i < b; ++i) s += in[i];
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const long long v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  long long run = part[t] - s;     // exclusive prefix of this chunk
  for (int i = a; i < b; ++i) {
    const int v = in[i];
    out[i] = (int)run;
    run += v;
  }
  if (t == 1023) {
    out[m] = (int)part[1023];
    if (total) *total = part[1023];
  }
}

__global__ void __launch_bounds__(DT) k_scatter(int n, const unsigned* key, const int* start, int* fill, int* order) {
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= n) return;
  const unsigned k = key[i];
  order[start[k] + atomicAdd(&fill[k], 1)] = i;
}

// Partners j > i of agent i in its 3 x 3 cell neighbourhood (buckets deduplicated: two cells
// of the neighbourhood may hash to one bucket).  EMIT = 0: count into cnt[i]; 1: write them at
// out[off[i] ...] and sort the agent's segment by j.
template <int EMIT>
__global__ void __launch_bounds__(DT) k_pairs(const double* xy, const double* r, int n, double inv_cs, unsigned mask,
                                              const int* start, const int* order, int* cnt, const int* off,
                                              int* out) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= n) return;
  const double xi = xy[2 * i], yi = xy[2 * i + 1], ri = r[i];
  const long long cx = cell_of(xi, inv_cs), cy = cell_of(yi, inv_cs);
  unsigned seen[9];
  int ns = 0, c = 0;
  const int base = EMIT ? off[i] : 0;
  for (int dx = -1; dx <= 1; ++dx) {
    for (int dy = -1; dy <= 1; ++dy) {
      const unsigned k = bucket_of(cx + dx, cy + dy, mask);
      bool dup = false;
      for (int s = 0; s < ns; ++s) dup |= seen[s] == k;
      if (dup) continue;
      seen[ns++] = k;
      const int b0 = start[k], b1 = start[k + 1];
      for (int p = b0; p < b1; ++p) {
        const int j = order[p];
        if (j <= i) continue;
        const double ddx = xy[2 * j] - xi, ddy = xy[2 * j + 1] - yi;
        const double d2 = ddx * ddx + ddy * ddy;
        const double rr = (ri + r[j]) * (ri + r[j]);
        if (d2 <= rr) {
          if (EMIT) out[2 * (base + c) + 1] = j;
          ++c;
        }
      }
    }
  }
  if (!EMIT) {
    cnt[i] = c;
    return;
  }
  // the agent's partners in increasing j (insertion sort: segments are short), then the i column
  int* seg = out + 2 * base;
  for (int a = 1; a < c; ++a) {
    const int v = seg[2 * a + 1];
    int b = a - 1;
    while (b >= 0 && seg[2 * b + 1] > v) {
      seg[2 * (b + 1) + 1] = seg[2 * b + 1];
      --b;
    }
    seg[2 * (b + 1) + 1] = v;
  }
  for (int a = 0; a < c; ++a) seg[2 * a] = i;
}

inline int blocks(int n) { return (n + DT - 1) / DT; }

}  // namespace

// Device part of piadmm_candidate_pairs (piadmm_capi.cpp): all pointers device-resident, sized
// by the caller (key, order, pcnt: n; cnt, fill: T; start: T + 1; off: n + 1; out: 2 * max_pairs).
// Returns 0 after enqueueing the count phase; *total is available after the stream syncs.
int launch_detect_count(const double* xy, const double* r, int n, double inv_cs, unsigned T, unsigned* key, int* cnt,
                        int* start, int* fill, int* order, int* pcnt, int* off, long long* total, hipStream_t s) {
  const unsigned mask = T - 1;
  if (hipMemsetAsync(cnt, 0, (size_t)T * sizeof(int), s) != hipSuccess) return -1;
  if (hipMemsetAsync(fill, 0, (size_t)T * sizeof(int), s) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_hash, dim3(blocks(n)), dim3(DT), 0, s, xy, n, inv_cs, mask, key, cnt);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, cnt, (int)T, start, (long long*)nullptr);
  hipLaunchKernelGGL(k_scatter, dim3(blocks(n)), dim3(DT), 0, s, n, key, start, fill, order);
  hipLaunchKernelGGL(k_pairs<0>, dim3(blocks(n)), dim3(DT), 0, s, xy, r, n, inv_cs, mask, start, order, pcnt,
                     nullptr, nullptr);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, pcnt, n, off, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_detect_emit(const double* xy, const double* r, int n, double inv_cs, unsigned T, const int* start,
                       const int* order, const int* off, int* out, hipStream_t s) {
  hipLaunchKernelGGL(k_pairs<1>, dim3(blocks(n)), dim3(DT), 0, s, xy, r, n, inv_cs, T - 1, start, order, nullptr,
                     off, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pd
