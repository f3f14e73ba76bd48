// Probe: where do the blocks of a kernel launched on a CU-masked stream run?
// For a few single-bit masks, 16 blocks each record HW_REG_XCC_ID / HW_REG_HW_ID.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_where(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc & 15;
    out[2 * blockIdx.x + 1] = hw;
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  int ncu = p.multiProcessorCount;
  unsigned* d;
  (void)hipMalloc(&d, 8 * 16);
  std::printf("cus %d\n", ncu);
  const int bits[] = {-1, 0, 1, 7, 8, 31, 32, 33, 40, 64, 100, 200, 255};
  for (int b : bits) {
    std::vector<uint32_t> m((ncu + 31) / 32, b < 0 ? ~0u : 0u);
    if (b >= 0) m[b / 32] = 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) != hipSuccess) {
      std::printf("bit %d: create failed\n", b);
      continue;
    }
    (void)hipMemsetAsync(d, 0xff, 8 * 16, s);
    hipLaunchKernelGGL(k_where, dim3(16), dim3(64), 0, s, d);
    unsigned h[32];
    (void)hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    std::printf("bit %4d:", b);
    for (int k = 0; k < 16; ++k) std::printf(" %u/%05x", h[2 * k], (h[2 * k + 1] >> 8) & 0xfffff);
    std::printf("\n");
    (void)hipStreamDestroy(s);
  }
  return 0;
}
