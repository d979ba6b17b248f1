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

__global__ void k_copy_last(const long long* src, int* dst) { *dst = (int)*src; }

__global__ void __launch_bounds__(DT) k_hash(const double* xy, int n, double inv_cs, unsigned mask, unsigned* key,
                                             int* cnt) {
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= n) return;
  const unsigned k = bucket_of(cell_of(xy[2 * i], inv_cs), cell_of(xy[2 * i + 1], inv_cs), mask);
  key[i] = k;
  atomicAdd(&cnt[k], 1);
}

// Exclusive scan of m 64-bit block sums in one workgroup (1024 threads, each a contiguous chunk);
// out[m] = total.  Used for the block sums of the multi-workgroup scan below (<= 2^16 of them):
// 64-bit, so that a dense cluster's pair count (> 2^31 in total) is reported exactly and refused
// by the caller instead of wrapping.
__global__ void __launch_bounds__(1024) k_scan(const long long* in, int m, long long* out, long long* total) {
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
    const long long v = in[i];
    out[i] = run;
    run += v;
  }
  if (t == 1023) {
    out[m] = part[1023];
    if (total) *total = part[1023];
  }
}

// Multi-workgroup exclusive scan: SCAN_B consecutive ints per workgroup (SCAN_T threads x 4,
// coalesced 16-byte loads), (1) the workgroups' sums, (2) their exclusive scan in one
// workgroup (k_scan), (3) each workgroup's local scan plus its offset.
constexpr int SCAN_T = 256, SCAN_B = 4 * SCAN_T;

template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T& tot) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < SCAN_T; o <<= 1) {
    const T a = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  tot = sh[SCAN_T - 1];
  const T incl = sh[t];
  __syncthreads();
  return incl - v;
}

__global__ void __launch_bounds__(SCAN_T) k_scan_sums(const int* in, int m, long long* bsum) {
  __shared__ long long sh[SCAN_T];
  const int i0 = blockIdx.x * SCAN_B + 4 * threadIdx.x;
  long long v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v += (i0 + k < m) ? in[i0 + k] : 0;
  long long tot;
  (void)block_excl_scan(v, sh, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// (int offsets: only used when the caller accepted the 64-bit total, <= 2^30)
__global__ void __launch_bounds__(SCAN_T) k_scan_down(const int* in, int m, const long long* boff, int* out) {
  __shared__ int sh[SCAN_T];
  const int i0 = blockIdx.x * SCAN_B + 4 * threadIdx.x;
  int e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = (i0 + k < m) ? in[i0 + k] : 0;
  int tot;
  int run = block_excl_scan<int>(e[0] + e[1] + e[2] + e[3], sh, tot) + (int)boff[blockIdx.x];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (i0 + k < m) out[i0 + k] = run;
    run += e[k];
  }
}

__global__ void __launch_bounds__(DT) k_scatter(int n, const unsigned* key, const int* start, int* fill, int* order) {
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= n) return;
  const unsigned k = key[i];
  order[start[k] + atomicAdd(&fill[k], 1)] = i;
}

// Positions and radii in bucket order (xs[p] = xy[order[p]]): a bucket is then a contiguous
// run, and the threads of a wave (consecutive sorted positions: spatial neighbours) read the
// same runs -- the gathers of the neighbourhood scans become cache-line reuse.
__global__ void __launch_bounds__(DT) k_permute(const double* xy, const double* r, int n, const int* order, double* xs,
                                                double* rs) {
  const int p = blockIdx.x * DT + threadIdx.x;
  if (p >= n) return;
  const int i = order[p];
  xs[2 * p] = xy[2 * i];
  xs[2 * p + 1] = xy[2 * i + 1];
  rs[p] = r[i];
}

// Partners j > i of agent i = order[p] in its 3 x 3 cell neighbourhood (buckets deduplicated:
// two cells of the neighbourhood may hash to one bucket).  EMIT = 0: count into cnt[i]; 1: write
// them at out[off[i] ...] and sort the agent's segment by j.
template <int EMIT>
__global__ void __launch_bounds__(DT) k_pairs(const double* xs, const double* rs, int n, double inv_cs, unsigned mask,
                                              const int* start, const int* order, int* cnt, const int* off,
                                              int* out) {
#pragma clang fp contract(off)
  const int p0 = blockIdx.x * DT + threadIdx.x;
  if (p0 >= n) return;
  const int i = order[p0];
  const double xi = xs[2 * p0], yi = xs[2 * p0 + 1], ri = rs[p0];
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
        const double ddx = xs[2 * p] - xi, ddy = xs[2 * p + 1] - yi;
        const double d2 = ddx * ddx + ddy * ddy;
        const double rr = (ri + rs[p]) * (ri + rs[p]);
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

// out[0..m) = exclusive scan of in, out[m] = total (and *total); bsum: (m + SCAN_B - 1) / SCAN_B + 1 ints
void scan(const int* in, int m, int* out, long long* bsum, long long* total, hipStream_t s) {
  const int nb = (m + SCAN_B - 1) / SCAN_B;
  hipLaunchKernelGGL(k_scan_sums, dim3(nb), dim3(SCAN_T), 0, s, in, m, bsum);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, s, bsum, nb, bsum, total);   // in place: block offsets
  hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(SCAN_T), 0, s, in, m, bsum, out);
  // out[m] = total = bsum[nb] (k_scan wrote it there)
  hipLaunchKernelGGL(k_copy_last, dim3(1), dim3(1), 0, s, bsum + nb, out + m);
}

}  // namespace

// Device part of piadmm_candidate_pairs (piadmm_capi.cpp): all pointers device-resident, sized
// by the caller (key, order, pcnt, rs: n; xs: 2n; cnt, fill: T; start: T + 1; off: n + 1; out:
// 2 * total).  The emit phase takes the bucket-ordered xs, rs of the count phase.
// Returns 0 after enqueueing the count phase; *total is available after the stream syncs.
int launch_detect_count(const double* xy, const double* r, int n, double inv_cs, unsigned T, unsigned* key, int* cnt,
                        int* start, int* fill, int* order, int* pcnt, int* off, long long* total, long long* bsum,
                        double* xs, double* rs, hipStream_t s) {
  const unsigned mask = T - 1;
  if (hipMemsetAsync(cnt, 0, (size_t)T * sizeof(int), s) != hipSuccess) return -1;
  if (hipMemsetAsync(fill, 0, (size_t)T * sizeof(int), s) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_hash, dim3(blocks(n)), dim3(DT), 0, s, xy, n, inv_cs, mask, key, cnt);
  scan(cnt, (int)T, start, bsum, nullptr, s);
  hipLaunchKernelGGL(k_scatter, dim3(blocks(n)), dim3(DT), 0, s, n, key, start, fill, order);
  hipLaunchKernelGGL(k_permute, dim3(blocks(n)), dim3(DT), 0, s, xy, r, n, order, xs, rs);
  hipLaunchKernelGGL(k_pairs<0>, dim3(blocks(n)), dim3(DT), 0, s, xs, rs, n, inv_cs, mask, start, order, pcnt,
                     nullptr, nullptr);
  scan(pcnt, n, off, bsum, total, s);
  return launch_rc(hipGetLastError());
}

int launch_detect_emit(const double* xs, const double* rs, int n, double inv_cs, unsigned T, const int* start,
                       const int* order, const int* off, int* out, hipStream_t s) {
  hipLaunchKernelGGL(k_pairs<1>, dim3(blocks(n)), dim3(DT), 0, s, xs, rs, n, inv_cs, T - 1, start, order, nullptr,
                     off, out);
  return launch_rc(hipGetLastError());
}

}  // namespace pd
