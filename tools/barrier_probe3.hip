// barrier_probe3.hip -- grid barriers among FEW workgroups (development probe, not
// part of the product; VERDICT r3 "do this" 3).  barrier_probe2 measured 256
// workgroups: 2.7 us with agent-scope atomics for the data, 6.8 us with agent-scope
// release/acquire fences (L2 writeback + invalidate), against 2.8 us per launch.  A
// sparse pass needs only a few workgroups; if they all sit on ONE XCD they share
// its L2, so a pass boundary needs no L2 writeback / invalidate -- only the CU's
// vector L1 must not serve a stale line.  Variants, for W = 4 / 8 / 16 / 32
// workgroups:
//   spread  W workgroups on consecutive block ids (round-robin over the 8 XCDs),
//           agent-scope release / acquire fences (what a pass boundary needs there)
//   xcd0    W workgroups with block id % 8 == 0 (one XCD; the other blocks of the
//           launch exit at once), plain stores, the barrier's own agent-scope
//           atomics, then a vector-L1 invalidate (buffer_inv sc0) before the loads
//   spread-L1  (control) W workgroups over the XCDs, plain stores, L1 invalidate only:
//           a reader on another XCD keeps its own L2's stale line, so stale reads here
//           and none under "xcd0 + L1 invalidate" show the W workgroups share one L2
//   xcc0-reg  W workgroups that READ their XCC id (hardware register XCC_ID) as 0 and
//           draw a ticket below W; plain stores, L1 invalidate (co-location by
//           construction instead of by block-id arithmetic)
// Also prints which XCC each block id of a 256-block launch ran on.
// Every round each workgroup writes a word with a PLAIN store and reads its
// neighbour's with a PLAIN load after the barrier; a stale read sets a flag.
// Every spin has a bailout (100 ms).
// Build: hipcc --offload-arch=gfx950 -O3 tools/barrier_probe3.hip -o tools/barrier_probe3
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

// the XCC (XCD) this wave runs on: hardware register XCC_ID (id 20), bits [3:0]
__device__ __forceinline__ unsigned xcc_id() {
  return (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
}

__global__ void k_xcc(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

// bar: [0] generation, [32] arrival counter, [64] error flags, [96] tickets (mode 4)
// MODE 0: spread + agent fences; 1: xcd0 + L1 invalidate; 2: xcd0, no invalidate;
// 3: spread + L1 invalidate (control); 4: xcc0 by register + L1 invalidate
template <int MODE>
__global__ __launch_bounds__(1024) void k_bar(unsigned* out, unsigned* bar, int n, int W) {
  const unsigned b = blockIdx.x;
  unsigned me;
  __shared__ unsigned s_me;
  if (MODE == 4) {
    if (threadIdx.x == 0) {
      s_me = ~0u;
      if (xcc_id() == 0u) s_me = atomicAdd(bar + 96, 1u);
    }
    __syncthreads();
    me = s_me;
    if (me >= (unsigned)W) return;
  } else if (MODE == 0 || MODE == 3) {
    if (b >= (unsigned)W) return;
    me = b;
  } else {
    if (b % 8u != 0u || b / 8u >= (unsigned)W) return;
    me = b / 8u;
  }
  unsigned* gen = bar;
  unsigned* cnt = bar + 32;
  unsigned* flag = bar + 64;
  for (int p = 0; p < n; ++p) {
    if (threadIdx.x == 0) out[me * 32] = (unsigned)p + 1;  // plain store (write-through L1)
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned my_gen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (MODE == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      else __builtin_amdgcn_s_waitcnt(0);  // the store has reached the XCD's L2
      if (atomicAdd(cnt, 1u) == (unsigned)W - 1) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == my_gen) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {  // 100 ms
          atomicOr(flag, 1u);
          break;
        }
      }
      if (MODE == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (MODE == 1 || MODE == 3 || MODE == 4) asm volatile("buffer_inv sc0" ::: "memory");
      const unsigned v = out[((me + 1) % (unsigned)W) * 32];  // plain load
      if (v < (unsigned)p + 1) atomicOr(flag, 2u);
    }
    __syncthreads();
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u) break;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4000;
  unsigned *out = nullptr, *bar = nullptr;
  CK(hipMalloc(&out, sizeof(unsigned) * 32 * 256));
  CK(hipMalloc(&bar, sizeof(unsigned) * 128));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0;
  for (int W : {8, 32, 256}) {
    CK(hipEventRecord(e0, st));
    for (int p = 0; p < n; ++p)
      hipLaunchKernelGGL(k_empty, dim3(W), dim3(1024), 0, st, out, (unsigned)p);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("launch of %3d empty 1024-thread workgroups: %.3f us each\n", W, 1000.0 * ms / n);
  }
  {
    unsigned h[256];
    hipLaunchKernelGGL(k_xcc, dim3(256), dim3(1024), 0, st, out);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
    std::printf("XCC of block ids 0..31:");
    for (int b = 0; b < 32; ++b) std::printf(" %u", h[b]);
    int per[16] = {0}, mod_ok = 0;
    for (int b = 0; b < 256; ++b) {
      ++per[h[b] & 15u];
      mod_ok += h[b] == h[b % 8];
    }
    std::printf("\nblocks per XCC:");
    for (int x = 0; x < 8; ++x) std::printf(" %d", per[x]);
    std::printf("; blocks with the XCC of block id %% 8: %d / 256\n", mod_ok);
  }
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 5; ++mode)
      for (int W : {4, 8, 16, 32}) {
        CK(hipMemsetAsync(bar, 0, sizeof(unsigned) * 128, st));
        CK(hipMemsetAsync(out, 0, sizeof(unsigned) * 32 * 256, st));
        int nn = n, ww = W;
        const int blocks = (mode == 0 || mode == 3) ? W : mode == 4 ? 256 : 8 * W;
        void* args[] = {&out, &bar, &nn, &ww};
        const void* fn = mode == 0   ? (const void*)k_bar<0>
                         : mode == 1 ? (const void*)k_bar<1>
                         : mode == 2 ? (const void*)k_bar<2>
                         : mode == 3 ? (const void*)k_bar<3>
                                     : (const void*)k_bar<4>;
        CK(hipEventRecord(e0, st));
        CK(hipLaunchCooperativeKernel(fn, dim3(blocks), dim3(1024), args, 0, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned h = 0;
        CK(hipMemcpy(&h, bar + 64, sizeof h, hipMemcpyDeviceToHost));
        std::printf("%s W=%2d: %.3f us per barrier (flags %u)\n",
                    mode == 0   ? "spread + agent fences  "
                    : mode == 1 ? "xcd0 + L1 invalidate   "
                    : mode == 2 ? "xcd0, no invalidate    "
                    : mode == 3 ? "spread + L1 inv (ctrl) "
                                : "xcc0-reg + L1 invalid. ",
                    W, 1000.0 * ms / n, h);
        if (h & 1u) return 2;
      }
  return 0;
}
