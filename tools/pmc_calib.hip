// pmc_calib.hip -- calibrate FETCH_SIZE / WRITE_SIZE for kernel 5's access
// pattern (development probe, not part of the product).  MI355X_MICROARCH.md
// calibrates the counters only for 16-B-per-lane streaming; visit16 loads and
// stores 8 B per lane (lane r*4+q: row r, the 4 doubles of columns 4q..4q+3 of
// a 16x16 tile, one double per instruction).  k_read reads every 16x16 tile of
// an N x N fp64 array exactly once with that pattern; k_write writes it the
// same way.  Known bytes: 8 N^2 each.  Run under rocprofv3 --pmc FETCH_SIZE
// (resp. WRITE_SIZE) and divide.
// Usage: tools/pmc_calib [N] [uc]  (uc: uncached memory, like the product's maps)
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

__global__ __launch_bounds__(256) void k_read(const double* a, int64_t n, double* sink) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane >> 2, q = lane & 3, odd = r & 1;
  const int64_t ntx = n / 16, tiles = ntx * ntx;
  double s = 0;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wv; t < tiles; t += (int64_t)gridDim.x * 4) {
    const int64_t tx = t % ntx, ty = t / ntx;
    const double* row = a + (ty * 16 + r) * n + tx * 16;
    // visit16's order: the two red then the two black cells of the lane
    s += row[4 * q + odd] + row[4 * q + 2 + odd] + row[4 * q + 1 - odd] + row[4 * q + 3 - odd];
  }
  if (s == 12345.678) sink[0] = s;  // keeps the loads
}

__global__ __launch_bounds__(256) void k_write(double* a, int64_t n) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane >> 2, q = lane & 3, odd = r & 1;
  const int64_t ntx = n / 16, tiles = ntx * ntx;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wv; t < tiles; t += (int64_t)gridDim.x * 4) {
    const int64_t tx = t % ntx, ty = t / ntx;
    double* row = a + (ty * 16 + r) * n + tx * 16;
    row[4 * q + odd] = 1.0;
    row[4 * q + 2 + odd] = 2.0;
    row[4 * q + 1 - odd] = 3.0;
    row[4 * q + 3 - odd] = 4.0;
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 16384;
  // "uc": the array in uncached device memory, as dymu_device_alloc's maps (round 6)
  const bool uc = argc > 2 && argv[2][0] == 'u';
  double *a = nullptr, *sink = nullptr;
  if (uc)
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&a), sizeof(double) * n * n,
                             hipDeviceMallocUncached));
  else
    CK(hipMalloc(&a, sizeof(double) * n * n));
  CK(hipMalloc(&sink, sizeof(double)));
  CK(hipMemset(a, 0, sizeof(double) * n * n));
  hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, 0, a, n);
  hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, a, n, sink);
  CK(hipDeviceSynchronize());
  std::printf("bytes per kernel: %lld (n = %lld)\n", (long long)(8 * n * n), (long long)n);
  CK(hipFree(a));
  CK(hipFree(sink));
  return 0;
}
