// pair_probe.hip -- development probe (not product): does splitting a 16x16
// tile's red-black sweeps over TWO waves (8 rows each, one red + one black cell
// per lane, the rows across the split read live from the shared LDS image, one
// LDS-counter pair barrier per sweep pair) shorten a tile's sweep latency at the
// same tiles per CU?  Mode 0: kernel 5's one-wave tile (rb_update2, 4 cells per
// lane); mode 1: the pair.  One workgroup per CU, W waves, fixed sweep pairs.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/pair_probe.hip -o tools/pair_probe
#include "../planning-path_planning_amd/csrc/fim_kernels.hip"

#include <cstdio>
#include <cstdlib>

namespace probe {
using namespace dymu;

__device__ __forceinline__ void rb_update1(const double* p, const double* pn, const double* ps,
                                           double f, double& t, bool& ch) {
  double w = p[-1], e = p[1], n = pn[0], s = ps[0];
  asm volatile("" : "+v"(w), "+v"(e), "+v"(n), "+v"(s));
  const double c2 = 2.0 * (f * f);
  const double tx = vmin64(w, e), ty = vmin64(n, s);
  const double m = vmin64(tx, ty);
  const double d = tx - ty;
  const double v = two_sided_approx(ty, d, c2);
  const double u = fabs(d) < f ? v : m + f;
  ch = u < t;
  t = vmin64(t, u);
}

// kernel 5's rb_update2 on two tiles at once (4 cells, two per tile): every
// neighbour read in flight before one wait, then the four chains interleaved
__device__ __forceinline__ void rb_update4(const double* p, const double* pn, const double* ps,
                                           const double* q, const double* qn, const double* qs,
                                           const double (&f)[4], double (&t)[4], bool (&ch)[4]) {
  double w[4] = {p[-1], p[1], q[-1], q[1]}, e[4] = {p[1], p[3], q[1], q[3]};
  double n[4] = {pn[0], pn[2], qn[0], qn[2]}, so[4] = {ps[0], ps[2], qs[0], qs[2]};
  asm volatile("" : "+v"(w[0]), "+v"(e[0]), "+v"(n[0]), "+v"(so[0]), "+v"(w[1]), "+v"(e[1]),
               "+v"(n[1]), "+v"(so[1]));
  asm volatile("" : "+v"(w[2]), "+v"(e[2]), "+v"(n[2]), "+v"(so[2]), "+v"(w[3]), "+v"(e[3]),
               "+v"(n[3]), "+v"(so[3]));
  double c2[4], tx[4], ty[4], m[4], d[4], v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c2[k] = 2.0 * (f[k] * f[k]);
    tx[k] = vmin64(w[k], e[k]);
    ty[k] = vmin64(n[k], so[k]);
    m[k] = vmin64(tx[k], ty[k]);
    d[k] = tx[k] - ty[k];
  }
  two_sided_approx2(ty[0], d[0], c2[0], ty[1], d[1], c2[1], v[0], v[1]);
  two_sided_approx2(ty[2], d[2], c2[2], ty[3], d[3], c2[3], v[2], v[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double u = fabs(d[k]) < f[k] ? v[k] : m[k] + f[k];
    ch[k] = u < t[k];
    t[k] = vmin64(t[k], u);
  }
}

// pair barrier: publish v, wait for the partner's arrival, return its v
struct Pair {
  uint32_t* cnt;  // [2]
  uint32_t* pw;   // [2 parity][2]
  int h;
  uint32_t n;
  __device__ uint32_t exchange(uint32_t v, uint32_t* err) {
    pw[(n & 1) * 2 + h] = v;
    ++n;
    __hip_atomic_store(&cnt[h], n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint32_t spins = 0;
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&cnt[1 - h], __ATOMIC_ACQUIRE,
                                                            __HIP_MEMORY_SCOPE_WORKGROUP)) < n) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        *err = 1u;
        break;
      }
    }
    return pw[((n - 1) & 1) * 2 + 1 - h];
  }
};

template <int MODE>
__global__ __launch_bounds__(1024) void k_probe(double* sink, uint32_t* err, int pairs) {
  __shared__ double s_img[16][IMG16];
  __shared__ uint32_t s_cnt[8][2], s_pw[8][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (MODE == 2) {  // two tiles per wave (waves <= 8: two images each)
    double* imgA = s_img[2 * wv];
    double* imgB = s_img[2 * wv + 1];
    for (int k = lane; k < IMG16; k += 64) {
      imgA[k] = 1000.0 + (double)((k * 37) % 101);
      imgB[k] = 1000.0 + (double)((k * 41) % 103);
    }
    const int r = lane >> 2, q = lane & 3, odd = r & 1;
    const int rb = img16_row(r);
    const int dn = img16_row(r + 1) - rb, ds = rb - img16_row(r - 1);
    double* prA = imgA + rb + 4 * q + odd;
    double* pbA = imgA + rb + 4 * q + 1 - odd;
    double* prB = imgB + rb + 4 * q + odd;
    double* pbB = imgB + rb + 4 * q + 1 - odd;
    const double fr[4] = {1.5 + 0.01 * lane, 2.5, 1.75, 2.25 + 0.01 * lane};
    const double fb[4] = {3.0, 1.25 + 0.02 * lane, 2.0 + 0.01 * lane, 1.5};
    double tr[4] = {prA[0], prA[2], prB[0], prB[2]}, tb[4] = {pbA[0], pbA[2], pbB[0], pbB[2]};
    bool cr[4], cb[4];
    int any = 0;
    __builtin_amdgcn_wave_barrier();
    for (int s = 0; s < pairs; ++s) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        __builtin_amdgcn_wave_barrier();
        rb_update4(prA, prA + dn, prA - ds, prB, prB + dn, prB - ds, fr, tr, cr);
        prA[0] = tr[0];
        prA[2] = tr[1];
        prB[0] = tr[2];
        prB[2] = tr[3];
        __builtin_amdgcn_wave_barrier();
        rb_update4(pbA, pbA + dn, pbA - ds, pbB, pbB + dn, pbB - ds, fb, tb, cb);
        pbA[0] = tb[0];
        pbA[2] = tb[1];
        pbB[0] = tb[2];
        pbB[2] = tb[3];
      }
      any += __any(cr[0] || cr[1] || cr[2] || cr[3] || cb[0] || cb[1] || cb[2] || cb[3]) ? 1 : 0;
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = tr[0] + tr[1] + tr[2] + tr[3] + tb[0] + tb[1] + tb[2] + tb[3] + any;
  } else if (MODE == 0) {
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
    int any = 0;
    __builtin_amdgcn_wave_barrier();
    for (int s = 0; s < pairs; ++s) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        __builtin_amdgcn_wave_barrier();
        rb_update2<true, true>(pr, prn, prs, fr[0], fr[1], tr[0], tr[1], c0, c1);
        pr[0] = tr[0];
        pr[2] = tr[1];
        __builtin_amdgcn_wave_barrier();
        rb_update2<true, true>(pb, pbn, pbs, fb[0], fb[1], tb[0], tb[1], c2, c3);
        pb[0] = tb[0];
        pb[2] = tb[1];
      }
      any += __any(c0 || c1 || c2 || c3) ? 1 : 0;
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = tr[0] + tr[1] + tb[0] + tb[1] + any;
  } else if (MODE == 1) {
    const int p = wv >> 1, h = wv & 1;
    double* img = s_img[p];
    if (lane < 2) s_cnt[p][lane] = 0u;
    if (lane < 4) s_pw[p][lane] = 0u;
    for (int k = lane + 64 * h; k < IMG16; k += 128) img[k] = 1000.0 + (double)((k * 37) % 101);
    __syncthreads();
    Pair P{s_cnt[p], s_pw[p], h, 0u};
    const int r = 8 * h + (lane >> 3), q = lane & 7, odd = r & 1;
    const int rb = img16_row(r);
    const int dn = img16_row(r + 1) - rb, ds = rb - img16_row(r - 1);
    double* pr = img + rb + 2 * q + odd;
    double* pb = img + rb + 2 * q + 1 - odd;
    const double *prn = pr + dn, *prs = pr - ds, *pbn = pb + dn, *pbs = pb - ds;
    const double fr = 1.5 + 0.01 * lane, fb = 1.25 + 0.02 * lane;
    double tr = pr[0], tb = pb[0];
    bool c0 = false, c2 = false;
    int any = 0;
    for (int s = 0; s < pairs; ++s) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        __builtin_amdgcn_wave_barrier();
        rb_update1(pr, prn, prs, fr, tr, c0);
        pr[0] = tr;
        __builtin_amdgcn_wave_barrier();
        rb_update1(pb, pbn, pbs, fb, tb, c2);
        pb[0] = tb;
      }
      const uint32_t mine = __any(c0 || c2) ? 1u : 0u;
      any += (int)(mine | P.exchange(mine, err));
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = tr + tb + any;
  }
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

template <int M>
static void run(double* sink, uint32_t* err, int cus, int waves, int pairs) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe::k_probe<M>, dim3(cus), dim3(64 * waves), 0, 0, sink, err, pairs);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(probe::k_probe<M>, dim3(cus), dim3(64 * waves), 0, 0, sink, err, pairs);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  uint32_t e = 0;
  CK(hipMemcpy(&e, err, sizeof e, hipMemcpyDeviceToHost));
  const int tiles = M == 0 ? waves : M == 2 ? 2 * waves : waves / 2;
  const double ns = 1e6 * ms / pairs;
  std::printf("mode %d waves/CU %2d tiles/CU %2d: %7.1f ns per tile sweep pair, %6.2f tile-pairs/us/CU%s\n",
              M, waves, tiles, ns, 1e3 * tiles / ns, e ? "  [SPIN LIMIT HIT]" : "");
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const int pairs = argc > 1 ? std::atoi(argv[1]) : 20000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  double* sink = nullptr;
  uint32_t* err = nullptr;
  CK(hipMalloc(&sink, sizeof(double) * (size_t)cus * 1024));
  CK(hipMalloc(&err, sizeof(uint32_t)));
  CK(hipMemset(err, 0, sizeof(uint32_t)));
  for (int w : {4, 8, 12, 16}) run<0>(sink, err, cus, w, pairs);
  for (int w : {2, 4, 8, 12, 16}) run<1>(sink, err, cus, w, pairs);
  for (int w : {4, 8}) run<2>(sink, err, cus, w, pairs);
  CK(hipFree(sink));
  CK(hipFree(err));
  return 0;
}
