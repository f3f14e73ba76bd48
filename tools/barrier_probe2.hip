// barrier_probe2.hip -- a hierarchical grid barrier vs the kernel boundary
// (development probe, not part of the product).  barrier_probe.hip measured a
// flat barrier (256 same-address arrivals) at 7.6 us against 2.9 us per launch
// of an empty pass-shaped kernel.  Here the workgroups arrive on G group
// counters (blockIdx % G, so with G = 8 a group is one XCD under round-robin
// dispatch), the last arriver of a group arrives on the top counter, and the
// last one there bumps a generation word every workgroup polls.  Each
// barrier also carries the visibility a pass boundary needs: agent-scope
// release before arriving, acquire after leaving, and every workgroup writes a
// word before and checks its neighbour's after.  Every spin has a bailout.
// Build: hipcc --offload-arch=gfx950 -O3 tools/barrier_probe2.hip -o tools/barrier_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__global__ __launch_bounds__(1024) void k_empty(unsigned* out, unsigned p) {
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = p;
}

// bar layout (unsigned, 32 words = 128 B apart): [0] generation, [32] top
// counter, [64 + 32 g] group g's counter, [64 + 32 * 64] bailout / error flag
// FENCE 1: agent-scope release / acquire fences (L2 writeback / invalidate);
// FENCE 0: none -- the data word itself is written and read with agent-scope
// atomics (they bypass the non-coherent per-XCD L2), as pass data would be
template <int FENCE>
__global__ __launch_bounds__(1024) void k_hbar(unsigned* out, unsigned* bar, int n, int G,
                                               int sleep) {
  const unsigned nb = gridDim.x, b = blockIdx.x;
  const unsigned g = b % (unsigned)G;
  const unsigned gsize = nb / G + (g < nb % G ? 1u : 0u);
  unsigned* gen = bar;
  unsigned* top = bar + 32;
  unsigned* grp = bar + 64 + 32 * g;
  unsigned* flag = bar + 64 + 32 * 64;
  for (int p = 0; p < n; ++p) {
    if (threadIdx.x == 0) {
      if (FENCE)
        out[b] = (unsigned)p + 1;
      else
        __hip_atomic_store(&out[b], (unsigned)p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned my_gen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (atomicAdd(grp, 1u) == gsize - 1) {
        __hip_atomic_store(grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (atomicAdd(top, 1u) == (unsigned)G - 1) {
          __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == my_gen) {
        if (sleep) __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {  // 100 ms
          atomicExch(flag, 1u);
          break;
        }
      }
      if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      // the neighbour's word of this round must be visible
      const unsigned v = __hip_atomic_load(&out[(b + 1) % nb], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (v < (unsigned)p + 1) atomicOr(flag, 2u);
    }
    __syncthreads();
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u) break;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int nb = cus;
  unsigned *out = nullptr, *bar = nullptr;
  const size_t bar_words = 64 + 32 * 64 + 32;
  CK(hipMalloc(&out, sizeof(unsigned) * nb));
  CK(hipMalloc(&bar, sizeof(unsigned) * bar_words));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {
    CK(hipEventRecord(e0, st));
    for (int p = 0; p < n; ++p) hipLaunchKernelGGL(k_empty, dim3(nb), dim3(1024), 0, st, out, (unsigned)p);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("launches: %d x empty pass kernel: %.3f us each\n", n, 1000.0 * ms / n);
    for (int fence = 0; fence < 2; ++fence)
    for (int G : {1, 8, 32}) {
      for (int sl = 0; sl < 2; ++sl) {
        CK(hipMemsetAsync(bar, 0, sizeof(unsigned) * bar_words, st));
        CK(hipMemsetAsync(out, 0, sizeof(unsigned) * nb, st));
        int nn = n, gg = G, ss = sl;
        void* args[] = {&out, &bar, &nn, &gg, &ss};
        CK(hipEventRecord(e0, st));
        CK(hipLaunchCooperativeKernel(fence ? (const void*)k_hbar<1> : (const void*)k_hbar<0>,
                                      dim3(nb), dim3(1024), args, 0, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned h[1];
        CK(hipMemcpy(h, bar + 64 + 32 * 64, sizeof h, hipMemcpyDeviceToHost));
        std::printf("hierarchical barrier fence %d G=%2d sleep %d: %.3f us each (flags %u)\n",
                    fence, G, sl, 1000.0 * ms / n, h[0]);
        if (h[0] & 1u) return 2;
      }
    }
  }
  return 0;
}
