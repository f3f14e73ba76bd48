// sqrt_probe.hip -- ulp error of the pass kernel's sqrt variants vs the correctly
// rounded sqrt on gfx950, over x = 2C^2 - d^2 with |d| < C (the sweep's operands):
// raw v_rsq_f64 * x, one Goldschmidt step, plus one Newton step; and the kernel's
// fused two-sided candidate (two_sided_approx) in ulps of the candidate.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/sqrt_probe.hip -o tools/sqrt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>

__device__ unsigned long long mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ long long ulps(double a, double b) {  // same sign, finite
  long long ia, ib;
  memcpy(&ia, &a, 8);
  memcpy(&ib, &b, 8);
  return ia > ib ? ia - ib : ib - ia;
}
// out[v*4 + k]: k = 0 max ulp, 1 count of nonzero, 2 count, v = variant (0 raw, 1 g1, 2 g1+n1)
__global__ void k_probe(unsigned long long seed, unsigned long long n, int scale_lo, int scale_hi,
                        unsigned long long* out) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned long long r1 = mix(seed ^ (2 * i)), r2 = mix(seed ^ (2 * i + 1));
    // C in [2^scale_lo, 2^scale_hi) log-uniform, d = C * u with u in (-1, 1)
    const double lg = scale_lo + (scale_hi - scale_lo) * ((r1 >> 11) * 0x1p-53);
    const double C = exp2(lg);
    const double u = ((double)(r2 >> 11) * 0x1p-52) - 1.0;
    const double d = C * u;
    const double x = 2.0 * (C * C) - d * d;
    const double cr = sqrt(x);
    const double y0 = __builtin_amdgcn_rsq(x);
    double s = x * y0;
    double h = y0 * 0.5;
    const double raw = s;
    const double e = __builtin_fma(-h, s, 0.5);
    s = __builtin_fma(s, e, s);
    h = __builtin_fma(h, e, h);
    const double g1 = s;
    const double dd = __builtin_fma(-s, s, x);
    const double n1 = __builtin_fma(dd, h, s);
    // the candidate u of the kernel's fused form (two_sided_approx) vs the reference
    // formula ((Tx + Ty) + sqrt(2C^2 - d^2)) / 2 on the kernel's domain: Tx, Ty >= 0,
    // |Tx - Ty| < C (Tx = T0, Ty = T0 + |d|), so u >= C / sqrt(2)
    const double T0 = C * 1000.0 * (double)((r1 >> 3) & 0xff) / 255.0;
    const double tx = T0, ty = T0 + fabs(d), dv = tx - ty;
    const double c2 = 2.0 * (C * C);
    const double rr = c2 - dv * dv;
    const double uref = ((tx + ty) + sqrt(rr)) * 0.5;
    const double rf = __builtin_fma(-dv, dv, c2);
    const double yf = __builtin_amdgcn_rsq(rf);
    const double sf = rf * yf;
    const double tf = __builtin_fma(-(yf * 0.25), sf, 0.75);
    const double uf = __builtin_fma(sf, tf, __builtin_fma(dv, 0.5, ty));
    const double v[4] = {raw, g1, n1, uf};
    {
      const long long e2 = ulps(uf, uref);
      atomicMax(&out[3 * 4 + 0], (unsigned long long)e2);
      if (e2) atomicAdd(&out[3 * 4 + 1], 1ull);
    }
    (void)v;
    for (int k = 0; k < 3; ++k) {
      const long long e2 = ulps(v[k], cr);
      atomicMax(&out[k * 4 + 0], (unsigned long long)e2);
      if (e2) atomicAdd(&out[k * 4 + 1], 1ull);
    }
  }
}

int main(int argc, char** argv) {
  const unsigned long long n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1ull << 28);
  const int ranges[][2] = {{0, 3}, {-20, 20}, {-380, 380}};
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * 16);
  for (auto& rg : ranges) {
    hipMemset(d, 0, sizeof(unsigned long long) * 16);
    hipLaunchKernelGGL(k_probe, dim3(4096), dim3(256), 0, 0, 0x1234ull + rg[0], n, rg[0], rg[1], d);
    unsigned long long h[16];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* nm[4] = {"raw x*rsq", "1 Goldschmidt step", "+1 Newton step",
                         "fused candidate u (ulp of u)"};
    std::printf("C in [2^%d, 2^%d), %llu samples\n", rg[0], rg[1], n);
    for (int k = 0; k < 4; ++k)
      std::printf("  %-30s max %llu ulp, %.3e of samples not correctly rounded\n", nm[k], h[k * 4],
                  (double)h[k * 4 + 1] / (double)n);
  }
  return 0;
}
