// group_barrier_probe.hip -- what a 4-wave superblock visit would pay per half-sweep
// (VERDICT r5 "do this" 3: 32x32 superblocks, four waves sharing one LDS image, a barrier
// among them per half-sweep).  (development probe, not part of the product)
// Every wave runs kernel 5's own red-black sweep pairs (rb_update2<true, true>) over its
// own 16x16 LDS image -- the quadrant it would own in a superblock -- and after every
// half-sweep the four waves of its group synchronise:
//   0  no barrier (today's one-wave visit)
//   1  a 4-wave barrier on an LDS counter (each wave's lane 0 adds, spins until the
//      group's count reaches the generation; workgroup-scope release / acquire)
//   2  s_barrier over the whole workgroup (__syncthreads)
// W waves per workgroup, one workgroup per CU: W = 4 is the sparse pass (one wave per
// SIMD, the maze's and the slabs' case), W = 16 a full one.  Prints ns per sweep pair.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iplanning-path_planning_amd/csrc \
//          -Iinclude tools/group_barrier_probe.hip -o tools/group_barrier_probe
#include "../planning-path_planning_amd/csrc/fim_kernels.hip"

#include <cstdio>
#include <cstdlib>

namespace probe {
using namespace dymu;

__device__ __forceinline__ void group_sync(unsigned* ctr, unsigned& gen, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  ++gen;
  if (lane == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4u * gen)
      __builtin_amdgcn_s_sleep(0);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int V>
__global__ __launch_bounds__(1024) void k_probe(double* sink, int pairs) {
  __shared__ double s_img[16][IMG16];
  __shared__ unsigned s_ctr[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < 4) s_ctr[threadIdx.x] = 0u;
  double* img = s_img[wv];
  for (int k = lane; k < IMG16; k += 64) img[k] = 1000.0 + (double)((k * 37) % 101);
  __syncthreads();
  unsigned* ctr = &s_ctr[wv >> 2];
  unsigned gen = 0;
  const int r = lane >> 2, q = lane & 3, odd = r & 1;
  const int rb = img16_row(r);
  const int dn = img16_row(r + 1) - rb, ds = rb - img16_row(r - 1);
  double* pr = img + rb + 4 * q + odd;
  double* pb = img + rb + 4 * q + 1 - odd;
  const double *prn = pr + dn, *prs = pr - ds, *pbn = pb + dn, *pbs = pb - ds;
  double fr[2] = {1.5 + 0.01 * lane, 2.5}, fb[2] = {3.0, 1.25 + 0.02 * lane};
  double tr[2] = {pr[0], pr[2]}, tb[2] = {pb[0], pb[2]};
  bool c0, c1, c2, c3;
  for (int s = 0; s < pairs; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __builtin_amdgcn_wave_barrier();
      rb_update2<true, true>(pr, prn, prs, fr[0], fr[1], tr[0], tr[1], c0, c1);
      pr[0] = tr[0];
      pr[2] = tr[1];
      if constexpr (V == 1) group_sync(ctr, gen, lane);
      if constexpr (V == 2) __syncthreads();
      __builtin_amdgcn_wave_barrier();
      rb_update2<true, true>(pb, pbn, pbs, fb[0], fb[1], tb[0], tb[1], c2, c3);
      pb[0] = tb[0];
      pb[2] = tb[1];
      if constexpr (V == 1) group_sync(ctr, gen, lane);
      if constexpr (V == 2) __syncthreads();
    }
  }
  if (c0 || c1 || c2 || c3) sink[blockIdx.x * 1024 + threadIdx.x] = tr[0] + tr[1] + tb[0] + tb[1];
}

template <int V>
float run(int waves, int pairs, double* sink, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_probe<V>, dim3(blocks), dim3(64 * waves), 0, 0, sink, pairs);  // warm
  (void)hipEventRecord(e0, 0);
  for (int k = 0; k < 5; ++k)
    hipLaunchKernelGGL(k_probe<V>, dim3(blocks), dim3(64 * waves), 0, 0, sink, pairs);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5.f;
}
}  // namespace probe

int main() {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double* sink = nullptr;
  if (hipMalloc(&sink, sizeof(double) * 1024 * (size_t)cus) != hipSuccess) return 1;
  const int pairs = 2000;
  for (const int W : {4, 8, 16}) {
    const float t0 = probe::run<0>(W, pairs, sink, cus);
    const float t1 = probe::run<1>(W, pairs, sink, cus);
    const float t2 = probe::run<2>(W, pairs, sink, cus);
    std::printf("{\"waves_per_cu\": %d, \"ns_per_pair\": {\"none\": %.1f, \"group4_lds\": %.1f, "
                "\"s_barrier\": %.1f}}\n",
                W, t0 * 1e6 / pairs, t1 * 1e6 / pairs, t2 * 1e6 / pairs);
  }
  (void)hipFree(sink);
  return 0;
}
