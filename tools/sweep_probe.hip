// sweep_probe.hip -- where does a kernel-5 half-sweep's time go?  (development
// probe, not part of the product)  Every wave of one workgroup per CU runs a
// fixed number of red-black sweep pairs over its own 16x16 tile image in LDS,
// with kernel 5's own update (rb_update2<true, true>, fim_kernels.hip), and the
// kernel is timed with events.  Variants:
//   0  kernel 5's half-sweep: 8 LDS reads, the update, 2 LDS writes
//   1  the same without the LDS writes (reads + VALU)
//   2  LDS reads + writes with a single v_min instead of the update (LDS only)
//   3  the update on register values only (VALU only, no LDS)
// Waves per CU W = 4 / 8 / 12 / 16 give 1..4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iplanning-path_planning_amd/csrc \
//          -Iinclude tools/sweep_probe.hip -o tools/sweep_probe
#include "../planning-path_planning_amd/csrc/fim_kernels.hip"

#include <cstdio>
#include <cstdlib>

namespace probe {
using namespace dymu;

template <int V>
__global__ __launch_bounds__(1024) void k_probe(double* sink, int pairs) {
  __shared__ double s_img[16][IMG16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* img = s_img[wv];
  for (int k = lane; k < IMG16; k += 64) img[k] = 1000.0 + (double)((k * 37) % 101);
  const int r = lane >> 2, q = lane & 3, odd = r & 1;
  const int rb = img16_row(r);
  const int dn = img16_row(r + 1) - rb, ds = rb - img16_row(r - 1);
  double* pr = img + rb + 4 * q + odd;
  double* pb = img + rb + 4 * q + 1 - odd;
  const double *prn = pr + dn, *prs = pr - ds, *pbn = pb + dn, *pbs = pb - ds;
  double fr[2] = {1.5 + 0.01 * lane, 2.5}, fb[2] = {3.0, 1.25 + 0.02 * lane};
  double tr[2] = {pr[0], pr[2]}, tb[2] = {pb[0], pb[2]};
  bool c0, c1, c2, c3;
  __builtin_amdgcn_wave_barrier();
  for (int s = 0; s < pairs; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (V == 0 || V == 1) {
        __builtin_amdgcn_wave_barrier();
        rb_update2<true, true>(pr, prn, prs, fr[0], fr[1], tr[0], tr[1], c0, c1);
        if constexpr (V == 0) {
          pr[0] = tr[0];
          pr[2] = tr[1];
        }
        __builtin_amdgcn_wave_barrier();
        rb_update2<true, true>(pb, pbn, pbs, fb[0], fb[1], tb[0], tb[1], c2, c3);
        if constexpr (V == 0) {
          pb[0] = tb[0];
          pb[2] = tb[1];
        }
      } else if constexpr (V == 2) {
        __builtin_amdgcn_wave_barrier();
        double a0 = pr[-1], a1 = pr[1], a2 = prn[0], a3 = prs[0], a4 = pr[3], a5 = prn[2], a6 = prs[2];
        tr[0] = vmin64(tr[0], vmin64(vmin64(a0, a1), vmin64(a2, a3)));
        tr[1] = vmin64(tr[1], vmin64(vmin64(a1, a4), vmin64(a5, a6)));
        pr[0] = tr[0];
        pr[2] = tr[1];
        __builtin_amdgcn_wave_barrier();
        double b0 = pb[-1], b1 = pb[1], b2 = pbn[0], b3 = pbs[0], b4 = pb[3], b5 = pbn[2], b6 = pbs[2];
        tb[0] = vmin64(tb[0], vmin64(vmin64(b0, b1), vmin64(b2, b3)));
        tb[1] = vmin64(tb[1], vmin64(vmin64(b1, b4), vmin64(b5, b6)));
        pb[0] = tb[0];
        pb[2] = tb[1];
      } else {  // V == 3: the update's arithmetic on registers
        double w0 = tb[0] + 1, e0 = tb[1] + 2, n0 = tb[0] + 3, s0 = tb[1] + 4;
        asm volatile("" : "+v"(w0), "+v"(e0), "+v"(n0), "+v"(s0));
        const double c20 = 2.0 * (fr[0] * fr[0]), c21 = 2.0 * (fr[1] * fr[1]);
        const double tx0 = vmin64(w0, e0), ty0 = vmin64(n0, s0);
        const double tx1 = vmin64(e0, n0), ty1 = vmin64(s0, w0);
        const double m0 = vmin64(tx0, ty0), m1 = vmin64(tx1, ty1);
        const double d0 = tx0 - ty0, d1 = tx1 - ty1;
        double v0, v1;
        two_sided_approx2(ty0, d0, c20, ty1, d1, c21, v0, v1);
        const double u0 = fabs(d0) < fr[0] ? v0 : m0 + fr[0];
        const double u1 = fabs(d1) < fr[1] ? v1 : m1 + fr[1];
        tr[0] = vmin64(tr[0], u0);
        tr[1] = vmin64(tr[1], u1);
        double w1 = tr[0] + 1, e1 = tr[1] + 2, n1 = tr[0] + 3, s1 = tr[1] + 4;
        asm volatile("" : "+v"(w1), "+v"(e1), "+v"(n1), "+v"(s1));
        const double c22 = 2.0 * (fb[0] * fb[0]), c23 = 2.0 * (fb[1] * fb[1]);
        const double tx2 = vmin64(w1, e1), ty2 = vmin64(n1, s1);
        const double tx3 = vmin64(e1, n1), ty3 = vmin64(s1, w1);
        const double m2 = vmin64(tx2, ty2), m3 = vmin64(tx3, ty3);
        const double d2 = tx2 - ty2, d3 = tx3 - ty3;
        double v2, v3;
        two_sided_approx2(ty2, d2, c22, ty3, d3, c23, v2, v3);
        const double u2 = fabs(d2) < fb[0] ? v2 : m2 + fb[0];
        const double u3 = fabs(d3) < fb[1] ? v3 : m3 + fb[1];
        tb[0] = vmin64(tb[0], u2);
        tb[1] = vmin64(tb[1], u3);
      }
    }
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = tr[0] + tr[1] + tb[0] + tb[1] + (c0 + c1 + c2 + c3);
}

}  // namespace probe

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

template <int V>
static void run(double* sink, int cus, int waves, int pairs) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe::k_probe<V>, dim3(cus), dim3(64 * waves), 0, 0, sink, pairs);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(probe::k_probe<V>, dim3(cus), dim3(64 * waves), 0, 0, sink, pairs);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  // one sweep pair = 2 sweeps = 4 half-sweeps (8 cell updates per lane)
  std::printf("variant %d waves/CU %2d (%d per SIMD): %.1f ns per sweep pair per wave\n", V, waves,
              waves / 4, 1e6 * ms / pairs);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int pairs = argc > 1 ? std::atoi(argv[1]) : 20000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  double* sink = nullptr;
  CK(hipMalloc(&sink, sizeof(double) * (size_t)cus * 1024));
  for (int w : {4, 8, 12, 16}) {
    run<0>(sink, cus, w, pairs);
    run<1>(sink, cus, w, pairs);
    run<2>(sink, cus, w, pairs);
    run<3>(sink, cus, w, pairs);
  }
  CK(hipFree(sink));
  return 0;
}
