// valu_probe.hip -- issue cost of the fp64 instructions of the sweep update on gfx950
// (development probe).  Every lane runs 8 independent chains of N instructions of one
// kind (inline asm, so nothing folds), 16 waves per CU on every CU; the time per
// instruction per wave at 4 waves per SIMD is the SIMD's issue cost of that opcode.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

template <int OP>
__device__ __forceinline__ void step(double& a, double b) {
  if (OP == 0) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a) : "v"(b));
  if (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));
  if (OP == 2) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a) : "v"(b));
  if (OP == 3) asm volatile("v_rsq_f64 %0, %0" : "+v"(a));
  if (OP == 4) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));
  if (OP == 5) {  // f32 rsq with the two conversions
    float f;
    asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f) : "v"(a));
    asm volatile("v_rsq_f32 %0, %0" : "+v"(f));
    asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(a) : "v"(f));
  }
  if (OP == 6) asm volatile("v_ldexp_f64 %0, %0, -1" : "+v"(a));
}

template <int OP>
__global__ __launch_bounds__(1024) void k_op(double* out, int n) {
  double a[8], b = 1.0000001 + threadIdx.x * 1e-9;
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 1.5 + k;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) step<OP>(a[k], b);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  if (s == 12345.678) out[threadIdx.x] = s;
}

int main() {
  double* out;
  CK(hipMalloc(&out, 8192));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int n = 4096;
  const char* names[] = {"v_fma_f64", "v_mul_f64", "v_min_f64", "v_rsq_f64", "v_add_f64",
                         "cvt+v_rsq_f32+cvt", "v_ldexp_f64"};
  for (int rep = 0; rep < 2; ++rep)
    for (int op = 0; op < 7; ++op) {
      const void* fn = op == 0 ? (const void*)k_op<0> : op == 1 ? (const void*)k_op<1>
                     : op == 2 ? (const void*)k_op<2> : op == 3 ? (const void*)k_op<3>
                     : op == 4 ? (const void*)k_op<4> : op == 5 ? (const void*)k_op<5>
                                                              : (const void*)k_op<6>;
      int nn = n;
      void* args[] = {&out, &nn};
      CK(hipEventRecord(e0, 0));
      CK(hipLaunchKernel(fn, dim3(256), dim3(1024), args, 0, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      // per SIMD: 4 waves x n x 8 instructions, at 2.4 GHz
      const double ns_per = 1e6 * ms / (4.0 * n * 8);
      std::printf("%-20s %.3f ns per wave-instruction per SIMD (%.1f cycles at 2.4 GHz)\n",
                  names[op], ns_per, ns_per * 2.4);
    }
  return 0;
}
