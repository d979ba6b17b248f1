// gbar_ubench.hip -- development microbenchmark (not shipped): the cost of one in-kernel grid
// barrier of the natural global stop test (piadmm_device.hip iter_tail) on gfx950, per barrier:
//   mode 0: cooperative_groups::this_grid().sync() alone
//   mode 1: a one-counter barrier (agent-scope fetch-add arrival, the last arrival bumps a
//           generation word the others spin on with s_sleep)
//   mode 2: mode 0 + iter_tail's reduction of the C x 5 partials (first 256 threads load, five
//           threads sum the 256 per-thread partials in thread order)
//   mode 3: mode 1 + the reduction of mode 2
//   mode 4: mode 1 + a butterfly reduction (per-thread strided partials, a wave xor-tree, the
//           waves' sums in wave order): a fixed order, the same in every workgroup
//   mode 5: a flag barrier: each workgroup release-stores its epoch into its own word (no
//           read-modify-write to serialise), wave 0 of every workgroup polls all C words
//   mode 6: mode 5 + the serial reduction of mode 2 cut to min(C, 256) terms (the terms of the
//           threads >= C are +0.0: the same sum bit for bit)
// Grid = C workgroups of 256 threads (one per component), cooperative launch.
//   hipcc -O3 --offload-arch=gfx950 tools/gbar_ubench.hip -o tools/gbar_ubench && tools/gbar_ubench
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int NT = 256;

__device__ __forceinline__ void bar1(unsigned* cnt, unsigned* gen, unsigned nb, unsigned& g) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned my = g;
    if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, my + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == my) __builtin_amdgcn_s_sleep(1);
    }
  }
  g = g + 1;
  __syncthreads();
}

__device__ __forceinline__ void bar_flags(unsigned long long* flags, unsigned long long epoch) {
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&flags[blockIdx.x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 64) {
    const int C = gridDim.x;
    while (true) {
      bool ok = true;
      for (int k = threadIdx.x; k < C; k += 64)
        ok = ok && __hip_atomic_load(&flags[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ void __launch_bounds__(NT) k_bar(int mode, int iters, double* part, unsigned* cnt, unsigned* gen, double* out,
                                            unsigned long long* flags, unsigned long long base) {
  __shared__ double red[5 * NT];
  __shared__ double tot[5];
  const int C = gridDim.x;
  unsigned g = 0;
  double acc = 0.0;
  for (int it = 0; it < iters; ++it) {
    double* p = part + (size_t)(it & 1) * C * 5;
    if (threadIdx.x == 0)
      for (int q = 0; q < 5; ++q)
        __hip_atomic_store(&p[blockIdx.x * 5 + q], (double)(blockIdx.x + q + it), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (mode == 0 || mode == 2)
      cooperative_groups::this_grid().sync();
    else if (mode >= 5)
      bar_flags(flags, base + it + 1);
    else
      bar1(cnt, gen, C, g);
    if (mode == 2 || mode == 3 || mode == 6) {
      double v[5] = {0, 0, 0, 0, 0};
      for (int k = threadIdx.x; k < C; k += NT)
        for (int q = 0; q < 5; ++q) v[q] += __hip_atomic_load(&p[k * 5 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int q = 0; q < 5; ++q) red[q * NT + threadIdx.x] = v[q];
      __syncthreads();
      if (threadIdx.x < 5) {
        double s = 0.0;
        const int nk = mode == 6 ? (C < NT ? C : NT) : NT;
        for (int k = 0; k < nk; ++k) s += red[threadIdx.x * NT + k];
        tot[threadIdx.x] = s;
      }
      __syncthreads();
      acc += tot[0] + tot[4];
      __syncthreads();
    } else if (mode == 4) {
      double v[5] = {0, 0, 0, 0, 0};
      for (int k = threadIdx.x; k < C; k += NT)
        for (int q = 0; q < 5; ++q) v[q] += __hip_atomic_load(&p[k * 5 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int q = 0; q < 5; ++q)
        for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o, 64);
      const int w = threadIdx.x >> 6;
      if ((threadIdx.x & 63) == 0)
        for (int q = 0; q < 5; ++q) red[q * 4 + w] = v[q];
      __syncthreads();
      if (threadIdx.x < 5) {
        double s = 0.0;
        for (int k = 0; k < NT / 64; ++k) s += red[threadIdx.x * 4 + k];
        tot[threadIdx.x] = s;
      }
      __syncthreads();
      acc += tot[0] + tot[4];
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

int main() {
  const int iters = 2000;
  double *part, *out;
  unsigned *cnt, *gen;
  CK(hipMalloc(&part, 2 * 1024 * 5 * sizeof(double)));
  CK(hipMalloc(&out, 1024 * sizeof(double)));
  CK(hipMalloc(&cnt, 64));
  CK(hipMalloc(&gen, 64));
  unsigned long long* flags;
  CK(hipMalloc(&flags, 1024 * sizeof(unsigned long long)));
  CK(hipMemset(flags, 0, 1024 * sizeof(unsigned long long)));
  unsigned long long base = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int Cs[] = {32, 64, 128, 256};
  const char* names[] = {"cg sync", "counter barrier", "cg sync + serial reduction", "counter + serial reduction",
                         "counter + butterfly reduction", "flag barrier", "flag barrier + reduction to C"};
  for (int C : Cs) {
    for (int mode = 0; mode < 7; ++mode) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(cnt, 0, 64));
        CK(hipMemset(gen, 0, 64));
        int m = mode, n = iters;
        void* args[] = {&m, &n, &part, &cnt, &gen, &out, &flags, &base};
        CK(hipEventRecord(e0));
        CK(hipLaunchCooperativeKernel((const void*)k_bar, dim3(C), dim3(NT), args, 0, 0));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
        base += iters + 1;                               // epochs never repeat across launches
      }
      std::printf("C=%4d  %-32s %8.3f us per barrier\n", C, names[mode], 1e3f * best / iters);
    }
  }
  return 0;
}
