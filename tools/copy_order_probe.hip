// copy_order_probe.hip -- which host-to-device copy pattern hands a kernel data the
// copy has not delivered (VERDICT r5 "do this" 1: the round-5 early exit wrote T = 0
// into cell 0 through dymu_scatter).  Each variant runs the call sequence of the old
// dymu_find_equal + dymu_scatter (commit 68c7198^) or one change of it, many times,
// with values tagged per iteration, and a kernel copies what it reads into a plain
// hipMalloc buffer that the host checks after a stream synchronisation.
//
//   A pool + pageable async   hipMallocAsync / pageable hipMemcpyAsync / kernel / hipFreeAsync
//                             after a find_equal-like alloc, blocking D2H, free (the old code)
//   B pool + pinned async     A with the host data in hipHostMalloc memory
//   C malloc + pageable async A with persistent hipMalloc buffers
//   D pool, no earlier free   A without the find_equal-like prologue
//   E pool + pageable + sync  A with hipStreamSynchronize between the copies and the kernel
//   F pool + blocking copy    A with null-stream hipMemcpy for the two copies
//   G pinned, zero copy       the kernel reads the hipHostMalloc buffers directly (the fix)
//   H pool, copy view         A's H2D copies into pool memory read back by a D2H hipMemcpy
//                             (what the copy engine sees; no kernel)
//   I pool, kernel writes     a kernel writes the pool buffers, a D2H hipMemcpy reads them
//                             (the old find_equal direction)
//   J pool, kernel round trip A, then a second kernel reads the buffers again after the
//                             first kernel and a stream synchronisation
//
// Output: one JSON line per (variant, n): iterations, bad elements, of which zero,
// of which stale (the previous iteration's tag).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/copy_order_probe tools/copy_order_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void k_read(const uint64_t* idx, const double* val, uint64_t* oi, double* ov, uint64_t n) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    oi[c] = idx[c];
    ov[c] = val[c];
  }
}

__global__ void k_mark(uint64_t* p, uint64_t n, uint64_t tag) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x)
    p[c] = tag + c;
}

static void launch_read(const uint64_t* di, const double* dv, uint64_t* oi, double* ov, uint64_t n,
                        hipStream_t st) {
  uint64_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  hipLaunchKernelGGL(k_read, dim3((unsigned)b), dim3(256), 0, st, di, dv, oi, ov, n);
  CK(hipGetLastError());
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const uint64_t nmax = 1u << 16;
  uint64_t* oi;
  double* ov;
  CK(hipMalloc(&oi, sizeof(uint64_t) * nmax));
  CK(hipMalloc(&ov, sizeof(double) * nmax));
  uint64_t* pdi;
  double* pdv;
  CK(hipMalloc(&pdi, sizeof(uint64_t) * nmax));
  CK(hipMalloc(&pdv, sizeof(double) * nmax));
  uint64_t* hpi;
  double* hpv;
  CK(hipHostMalloc(&hpi, sizeof(uint64_t) * nmax, hipHostMallocDefault));
  CK(hipHostMalloc(&hpv, sizeof(double) * nmax, hipHostMallocDefault));
  std::vector<uint64_t> hi(nmax), ri(nmax);
  std::vector<double> hv(nmax), rv(nmax);
  std::vector<uint64_t> eq(256);
  const uint64_t sizes[] = {150, 1328, 4096, 65536};
  const char* names = "ABCDEFGHIJ";
  for (int var = 0; var < 10; ++var) {
    for (const uint64_t n : sizes) {
      uint64_t bad = 0, zero = 0, stale = 0, bad_iters = 0;
      // the first bad element seen: index, expected / read index word, read value, and
      // the pool pointers of that iteration
      uint64_t fb_c = ~0ull, fb_exp = 0, fb_got = 0;
      double fb_val = 0.0;
      uintptr_t p_di = 0, p_dv = 0, fb_di = 0, fb_dv = 0;
      for (int it = 0; it < iters; ++it) {
        const uint64_t tag = ((uint64_t)(var * 16 + it) << 32) + 7;
        for (uint64_t c = 0; c < n; ++c) {
          hi[c] = tag + c;
          hv[c] = (double)(tag + c) + 0.5;
        }
        if (var == 1 || var == 6) {
          std::memcpy(hpi, hi.data(), sizeof(uint64_t) * n);
          std::memcpy(hpv, hv.data(), sizeof(double) * n);
        }
        if (var != 3 && var != 2 && var != 6) {  // find_equal-like prologue
          uint64_t* di = nullptr;
          CK(hipMallocAsync(reinterpret_cast<void**>(&di), sizeof(uint64_t) * 256, st));
          hipLaunchKernelGGL(k_mark, dim3(1), dim3(256), 0, st, di, (uint64_t)256, tag ^ 0x5555);
          CK(hipGetLastError());
          CK(hipStreamSynchronize(st));
          CK(hipMemcpy(eq.data(), di, sizeof(uint64_t) * 256, hipMemcpyDeviceToHost));
          CK(hipFreeAsync(di, st));
          CK(hipStreamSynchronize(st));
        }
        const uint64_t* src_i = var == 1 ? hpi : hi.data();
        const double* src_v = var == 1 ? hpv : hv.data();
        if (var == 7 || var == 8) {
          uint64_t* di = nullptr;
          double* dv = nullptr;
          CK(hipMallocAsync(reinterpret_cast<void**>(&di), sizeof(uint64_t) * n, st));
          CK(hipMallocAsync(reinterpret_cast<void**>(&dv), sizeof(double) * n, st));
          p_di = (uintptr_t)di;
          p_dv = (uintptr_t)dv;
          if (var == 7) {
            CK(hipMemcpyAsync(di, hi.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(dv, hv.data(), sizeof(double) * n, hipMemcpyHostToDevice, st));
          } else {
            CK(hipMemcpyAsync(pdi, hi.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(pdv, hv.data(), sizeof(double) * n, hipMemcpyHostToDevice, st));
            launch_read(pdi, pdv, di, dv, n, st);  // kernel writes the pool buffers
          }
          CK(hipStreamSynchronize(st));
          CK(hipMemcpy(ri.data(), di, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
          CK(hipMemcpy(rv.data(), dv, sizeof(double) * n, hipMemcpyDeviceToHost));
          CK(hipFreeAsync(dv, st));
          CK(hipFreeAsync(di, st));
          CK(hipStreamSynchronize(st));
          goto check;
        }
        if (var == 9) {
          uint64_t* di = nullptr;
          double* dv = nullptr;
          CK(hipMallocAsync(reinterpret_cast<void**>(&di), sizeof(uint64_t) * n, st));
          CK(hipMallocAsync(reinterpret_cast<void**>(&dv), sizeof(double) * n, st));
          p_di = (uintptr_t)di;
          p_dv = (uintptr_t)dv;
          CK(hipMemcpyAsync(di, hi.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
          CK(hipMemcpyAsync(dv, hv.data(), sizeof(double) * n, hipMemcpyHostToDevice, st));
          launch_read(di, dv, oi, ov, n, st);
          CK(hipStreamSynchronize(st));
          launch_read(di, dv, oi, ov, n, st);
          CK(hipFreeAsync(dv, st));
          CK(hipFreeAsync(di, st));
        } else if (var == 2) {
          CK(hipMemcpyAsync(pdi, src_i, sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
          CK(hipMemcpyAsync(pdv, src_v, sizeof(double) * n, hipMemcpyHostToDevice, st));
          launch_read(pdi, pdv, oi, ov, n, st);
        } else if (var == 6) {
          uint64_t* gi = nullptr;
          double* gv = nullptr;
          CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&gi), hpi, 0));
          CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&gv), hpv, 0));
          launch_read(gi, gv, oi, ov, n, st);
        } else {
          uint64_t* di = nullptr;
          double* dv = nullptr;
          CK(hipMallocAsync(reinterpret_cast<void**>(&di), sizeof(uint64_t) * n, st));
          CK(hipMallocAsync(reinterpret_cast<void**>(&dv), sizeof(double) * n, st));
          p_di = (uintptr_t)di;
          p_dv = (uintptr_t)dv;
          if (var == 5) {
            CK(hipMemcpy(di, src_i, sizeof(uint64_t) * n, hipMemcpyHostToDevice));
            CK(hipMemcpy(dv, src_v, sizeof(double) * n, hipMemcpyHostToDevice));
          } else {
            CK(hipMemcpyAsync(di, src_i, sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
            CK(hipMemcpyAsync(dv, src_v, sizeof(double) * n, hipMemcpyHostToDevice, st));
          }
          if (var == 4) CK(hipStreamSynchronize(st));
          launch_read(di, dv, oi, ov, n, st);
          CK(hipFreeAsync(dv, st));
          CK(hipFreeAsync(di, st));
        }
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(ri.data(), oi, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(rv.data(), ov, sizeof(double) * n, hipMemcpyDeviceToHost));
      check:
        uint64_t b = 0;
        for (uint64_t c = 0; c < n; ++c) {
          if (ri[c] != hi[c] || rv[c] != hv[c]) {
            ++b;
            if (ri[c] == 0 || rv[c] == 0.0) ++zero;
            if ((ri[c] >> 32) != (hi[c] >> 32)) ++stale;
            if (fb_c == ~0ull) {
              fb_c = c;
              fb_exp = hi[c];
              fb_got = ri[c];
              fb_val = rv[c];
              fb_di = p_di;
              fb_dv = p_dv;
            }
          }
        }
        bad += b;
        bad_iters += b != 0;
      }
      std::printf("{\"variant\": \"%c\", \"n\": %llu, \"iters\": %d, \"bad_iters\": %llu, "
                  "\"bad\": %llu, \"zero\": %llu, \"stale\": %llu, \"first\": [%lld, \"%llx\", "
                  "\"%llx\", %.17g, \"%llx\", \"%llx\"]}\n",
                  names[var], (unsigned long long)n, iters, (unsigned long long)bad_iters,
                  (unsigned long long)bad, (unsigned long long)zero, (unsigned long long)stale,
                  (long long)fb_c, (unsigned long long)fb_exp, (unsigned long long)fb_got, fb_val,
                  (unsigned long long)fb_di, (unsigned long long)fb_dv);
      std::fflush(stdout);
    }
  }
  return 0;
}
