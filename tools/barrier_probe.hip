// barrier_probe.hip -- is a grid barrier between passes cheaper than a kernel
// boundary?  Times (1) N back-to-back launches of a pass-shaped empty kernel
// (one 1024-thread workgroup per CU, a tiny store each) and (2) one cooperative
// launch of the same workgroups doing N grid barriers (agent-scope release /
// acquire, counter polled with s_sleep).  Every spin has a wall-clock bailout.
// Build: hipcc --offload-arch=gfx950 -O3 tools/barrier_probe.hip -o tools/barrier_probe
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

// bar[0]: arrivals (monotone); bar[1]: bailout flag
__global__ __launch_bounds__(1024) void k_barriers(unsigned* out, unsigned* bar, int n, int sleep) {
  const unsigned nb = gridDim.x;
  for (int p = 0; p < n; ++p) {
    if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)p;
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      atomicAdd(&bar[0], 1u);
      const unsigned target = nb * (unsigned)(p + 1);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(&bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (sleep) __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {  // 100 ms
          atomicExch(&bar[1], 1u);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_barriers, 1024, 0));
  const int nb = cus;  // one workgroup per CU, as the pass kernel
  std::printf("CUs %d, k_barriers workgroups/CU %d, grid %d x 1024\n", cus, occ, nb);
  unsigned *out = nullptr, *bar = nullptr;
  CK(hipMalloc(&out, sizeof(unsigned) * nb));
  CK(hipMalloc(&bar, sizeof(unsigned) * 2));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, st));
    for (int p = 0; p < n; ++p) hipLaunchKernelGGL(k_empty, dim3(nb), dim3(1024), 0, st, out, (unsigned)p);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("launches: %d x empty pass kernel: %.3f us each\n", n, 1000.0 * ms / n);
    for (int sl = 0; sl < 2; ++sl) {
      CK(hipMemsetAsync(bar, 0, sizeof(unsigned) * 2, st));
      int nn = n;
      void* args[] = {&out, &bar, &nn, &sl};
      CK(hipEventRecord(e0, st));
      CK(hipLaunchCooperativeKernel((const void*)k_barriers, dim3(nb), dim3(1024), args, 0, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned h[2];
      CK(hipMemcpy(h, bar, sizeof h, hipMemcpyDeviceToHost));
      std::printf("grid barriers (sleep %d): %d: %.3f us each (arrivals %u, bailout %u)\n", sl, n,
                  1000.0 * ms / n, h[0], h[1]);
      if (h[1]) return 2;
    }
  }
  return 0;
}
