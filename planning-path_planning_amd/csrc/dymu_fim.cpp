// dymu_fim.cpp -- C-ABI runtime (include/dymu_fim.h) around the HIP block-FIM
// kernels (fim_kernels.hip).  Owns the stream, events and the tile workspace;
// drives passes until the active-tile list drains.
//
// Replaces the host loop of computeEntireTotalCostMap
// (src/DyMu_GlobalPathPlanning.cpp:443-468): the reference pops one node per
// iteration from a linear-scan narrow band; here each pass relaxes every
// active tile in parallel and the device builds the next active list itself,
// so the host only reads a 4-byte counter every few passes.
#include "dymu_fim.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fim_kernels.h"

using namespace dymu;

struct dymu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  dymu_opts opts{};
  int cu_count = 256;

  int variant = 2;  // 1: 32x32 tile per workgroup, 2: 8x8 tile per wave (DYMU_KERNEL)

  // tile workspace
  uint32_t tiles_cap = 0;
  uint32_t* d_lists = nullptr;       // 3 lists x kShards shards x tiles_cap
  uint32_t* d_counts = nullptr;      // 3 x kShards words, own block
  uint32_t* d_tile_epoch = nullptr;  // tiles_cap
  unsigned long long* d_stats = nullptr;  // kStatSlots
  uint32_t epoch_base = 0;
  uint32_t* h_count = nullptr;  // pinned

  // host-solve staging
  double* d_F = nullptr;
  double* d_T = nullptr;
  uint64_t cells_cap = 0;

  // profiling
  int profiling = 0;
  std::vector<hipEvent_t> prof_ev;
  double last_pass_ms = 0.0;
  uint64_t last_launches = 0;

  std::string last_error;
};

namespace {

int fail_hip(dymu_ctx* c, hipError_t e, const char* what) {
  if (c) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    c->last_error = buf;
  }
  return e == hipErrorOutOfMemory ? DYMU_ERR_NOMEM : DYMU_ERR_HIP;
}

#define HIPC(ctx, expr)                                  \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return fail_hip(ctx, _e, #expr); \
  } while (0)

int ensure_tiles(dymu_ctx* c, uint32_t ntiles) {
  if (ntiles <= c->tiles_cap) return DYMU_OK;
  if (c->d_lists) (void)hipFree(c->d_lists);
  if (c->d_tile_epoch) (void)hipFree(c->d_tile_epoch);
  c->d_lists = nullptr;
  c->d_tile_epoch = nullptr;
  c->tiles_cap = 0;
  HIPC(c, hipMalloc(&c->d_lists, sizeof(uint32_t) * 3ull * kShards * ntiles));
  HIPC(c, hipMalloc(&c->d_tile_epoch, sizeof(uint32_t) * (uint64_t)ntiles));
  HIPC(c, hipMemsetAsync(c->d_tile_epoch, 0, sizeof(uint32_t) * (uint64_t)ntiles, c->stream));
  c->tiles_cap = ntiles;
  c->epoch_base = 0;
  return DYMU_OK;
}

int ensure_cells(dymu_ctx* c, uint64_t cells) {
  if (cells <= c->cells_cap) return DYMU_OK;
  if (c->d_F) (void)hipFree(c->d_F);
  if (c->d_T) (void)hipFree(c->d_T);
  c->d_F = c->d_T = nullptr;
  c->cells_cap = 0;
  HIPC(c, hipMalloc(&c->d_F, sizeof(double) * cells));
  HIPC(c, hipMalloc(&c->d_T, sizeof(double) * cells));
  c->cells_cap = cells;
  return DYMU_OK;
}

int tile_w(const dymu_ctx* c) { return c->variant == 1 ? kTileW : kWaveTile; }
int tile_h(const dymu_ctx* c) { return c->variant == 1 ? kTileH : kWaveTile; }

int solve_core(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
               uint32_t gi, uint32_t gj, hipStream_t st, dymu_stats* stats) {
  if (!dF || !dT || nx == 0 || ny == 0 || ld < nx || gi >= nx || gj >= ny) return DYMU_ERR_ARG;
  const int TWd = tile_w(c), THd = tile_h(c);
  const uint32_t ntx = (uint32_t)((nx + TWd - 1) / TWd), nty = (uint32_t)((ny + THd - 1) / THd);
  const uint64_t ntiles64 = (uint64_t)ntx * nty;
  if (ntiles64 >= (1ull << 31)) return DYMU_ERR_ARG;
  const uint32_t ntiles = (uint32_t)ntiles64;
  int rc = ensure_tiles(c, ntiles);
  if (rc) return rc;

  const uint64_t max_passes =
      c->opts.max_passes > 0 ? (uint64_t)c->opts.max_passes : 4ull * ntiles + 1024ull;
  if ((uint64_t)c->epoch_base + max_passes + 8 >= 0xFFFFFFF0ull) {
    HIPC(c, hipMemsetAsync(c->d_tile_epoch, 0, sizeof(uint32_t) * (uint64_t)ntiles, st));
    c->epoch_base = 0;
  }
  const uint32_t eb = c->epoch_base;
  const uint64_t lstride = (uint64_t)kShards * ntiles;
  uint32_t* lists[3] = {c->d_lists, c->d_lists + lstride, c->d_lists + 2 * lstride};
  uint32_t* counts[3] = {c->d_counts, c->d_counts + kShards, c->d_counts + 2 * kShards};
  HIPC(c, hipMemsetAsync(c->d_counts, 0, sizeof(uint32_t) * 3 * kShards, st));
  HIPC(c, hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * kShards * kStatSlots, st));
  HIPC(c, launch_fill_inf(dT, ld, nx, 0, ny, st));
  const uint32_t gtile = (gj / THd) * ntx + (gi / TWd);
  HIPC(c, launch_seed(dT, ld, gi, gj, lists[0], counts[0], c->d_tile_epoch, eb + 1, gtile, 1, st));

  PassArgs a{};
  a.F = dF;
  a.T = dT;
  a.ld = (int64_t)ld;
  a.nx = nx;
  a.ny = ny;
  a.ntx = (int)ntx;
  a.nty = (int)nty;
  a.ghost_lo = 0;
  a.ghost_hi = 0;
  a.max_inner = c->opts.max_inner > 0 ? c->opts.max_inner : 4 * (TWd + THd);
  a.shard_cap = ntiles;
  a.tile_epoch = c->d_tile_epoch;
  a.stats = c->d_stats;
  const int blocks = c->opts.grid_blocks > 0 ? c->opts.grid_blocks : c->cu_count * 8;

  const bool prof = c->profiling != 0;
  size_t prof_used = 0;
  HIPC(c, hipEventRecord(c->ev0, st));
  uint64_t p = 0, launches = 0;
  uint64_t K = c->opts.passes_per_check > 0 ? (uint64_t)c->opts.passes_per_check : 4;
  for (;;) {
    for (uint64_t k = 0; k < K; ++k, ++p) {
      a.list_in = lists[p % 3];
      a.count_in = counts[p % 3];
      a.list_out = lists[(p + 1) % 3];
      a.count_out = counts[(p + 1) % 3];
      a.count_clear = counts[(p + 2) % 3];
      a.epoch = eb + (uint32_t)p + 2u;
      if (prof) {
        while (c->prof_ev.size() < prof_used + 2) {
          hipEvent_t e;
          HIPC(c, hipEventCreate(&e));
          c->prof_ev.push_back(e);
        }
        HIPC(c, hipEventRecord(c->prof_ev[prof_used], st));
      }
      HIPC(c, c->variant == 1 ? launch_pass(a, blocks, st) : launch_pass_w8(a, blocks, st));
      if (prof) {
        HIPC(c, hipEventRecord(c->prof_ev[prof_used + 1], st));
        prof_used += 2;
      }
      ++launches;
    }
    HIPC(c, hipMemcpyAsync(c->h_count, counts[p % 3], sizeof(uint32_t) * kShards,
                           hipMemcpyDeviceToHost, st));
    HIPC(c, hipStreamSynchronize(st));
    uint64_t pending = 0;
    for (int q = 0; q < kShards; ++q) pending += c->h_count[q];
    if (pending == 0) break;
    if (p >= max_passes) {
      c->last_error = "pass cap reached before convergence";
      c->epoch_base = eb + (uint32_t)p + 4u;
      return DYMU_ERR_NOT_CONVERGED;
    }
    if (c->opts.passes_per_check <= 0) K = std::min<uint64_t>(K * 2, 64);
  }
  HIPC(c, hipEventRecord(c->ev1, st));
  HIPC(c, hipEventSynchronize(c->ev1));
  c->epoch_base = eb + (uint32_t)p + 4u;

  float ms = 0.f;
  HIPC(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->last_launches = launches;
  c->last_pass_ms = 0.0;
  if (prof) {
    for (size_t q = 0; q + 1 < prof_used; q += 2) {
      float m = 0.f;
      HIPC(c, hipEventElapsedTime(&m, c->prof_ev[q], c->prof_ev[q + 1]));
      c->last_pass_ms += m;
    }
  }
  if (stats) {
    unsigned long long hs[kShards * kStatSlots];
    HIPC(c, hipMemcpy(hs, c->d_stats, sizeof hs, hipMemcpyDeviceToHost));
    unsigned long long h[kStatSlots] = {0};
    for (int q = 0; q < kShards; ++q)
      for (int k = 0; k < kStatSlots; ++k)
        h[k] = (k == kStatMaxActive) ? std::max(h[k], hs[q * kStatSlots + k])
                                     : h[k] + hs[q * kStatSlots + k];
    std::memset(stats, 0, sizeof *stats);
    stats->passes = h[kStatPasses];
    stats->launches = launches;
    stats->tile_visits = h[kStatVisits];
    stats->inner_sweeps = h[kStatSweeps];
    stats->max_active = h[kStatMaxActive];
    stats->rounds = 0;
    stats->ms = ms;
    stats->tile_w = TWd;
    stats->tile_h = THd;
  }
  return DYMU_OK;
}

hipStream_t pick_stream(dymu_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }

}  // namespace

extern "C" {

int dymu_abi_version(void) { return DYMU_ABI_VERSION; }

int dymu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* dymu_strerror(int s) {
  switch (s) {
    case DYMU_OK: return "ok";
    case DYMU_ERR_ARG: return "invalid argument";
    case DYMU_ERR_HIP: return "HIP runtime error";
    case DYMU_ERR_NOMEM: return "device out of memory";
    case DYMU_ERR_NOT_CONVERGED: return "pass cap reached before convergence";
    case DYMU_ERR_NO_DEVICE: return "no HIP device";
    case DYMU_ERR_RCCL: return "RCCL error";
    case DYMU_ERR_STATE: return "call out of sequence";
    default: return "unknown status";
  }
}

const char* dymu_last_error(dymu_ctx* c) { return c ? c->last_error.c_str() : ""; }

int dymu_create(dymu_ctx** out, const dymu_opts* opts) {
  if (!out) return DYMU_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DYMU_ERR_NO_DEVICE;
  dymu_ctx* c = new dymu_ctx();
  if (opts) c->opts = *opts;
  else c->opts.device = -1;
  int dev = c->opts.device;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  if (dev >= ndev) {
    delete c;
    return DYMU_ERR_ARG;
  }
  c->device = dev;
  hipError_t e = hipSetDevice(dev);
  if (e == hipSuccess) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
      c->cu_count = prop.multiProcessorCount;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  }
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (const char* kv = std::getenv("DYMU_KERNEL")) c->variant = std::atoi(kv) == 1 ? 1 : 2;
  if (e == hipSuccess) e = hipMalloc(&c->d_counts, sizeof(uint32_t) * 4 * kShards);
  if (e == hipSuccess)
    e = hipMalloc(&c->d_stats, sizeof(unsigned long long) * kShards * kStatSlots);
  if (e == hipSuccess) e = hipHostMalloc(&c->h_count, sizeof(uint32_t) * 4 * kShards, hipHostMallocDefault);
  if (e != hipSuccess) {
    dymu_destroy(c);
    return e == hipErrorOutOfMemory ? DYMU_ERR_NOMEM : DYMU_ERR_HIP;
  }
  *out = c;
  return DYMU_OK;
}

int dymu_destroy(dymu_ctx* c) {
  if (!c) return DYMU_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->d_lists) (void)hipFree(c->d_lists);
  if (c->d_tile_epoch) (void)hipFree(c->d_tile_epoch);
  if (c->d_counts) (void)hipFree(c->d_counts);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->d_F) (void)hipFree(c->d_F);
  if (c->d_T) (void)hipFree(c->d_T);
  if (c->h_count) (void)hipHostFree(c->h_count);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return DYMU_OK;
}

int dymu_solve_device(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny,
                      uint64_t ld, uint32_t gi, uint32_t gj, void* stream, dymu_stats* stats) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return solve_core(c, dF, dT, nx, ny, ld, gi, gj, pick_stream(c, stream), stats);
}

int dymu_solve(dymu_ctx* c, const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
               double* T_out, dymu_stats* stats) {
  if (!c || !F || !T_out || nx == 0 || ny == 0) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  const uint64_t cells = (uint64_t)nx * ny;
  int rc = ensure_cells(c, cells);
  if (rc) return rc;
  HIPC(c, hipMemcpyAsync(c->d_F, F, sizeof(double) * cells, hipMemcpyHostToDevice, c->stream));
  rc = solve_core(c, c->d_F, c->d_T, nx, ny, nx, gi, gj, c->stream, stats);
  if (rc) return rc;
  HIPC(c, hipMemcpyAsync(T_out, c->d_T, sizeof(double) * cells, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return DYMU_OK;
}

int dymu_synth_speed(dymu_ctx* c, double* dF, uint32_t nx, uint32_t ny, uint64_t ld, uint64_t row0,
                     uint64_t seed, double obst_frac, uint64_t obst_seed, uint32_t gi, uint32_t gj,
                     void* stream) {
  if (!c || !dF || ld < nx) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, stream);
  HIPC(c, launch_synth(dF, ld, nx, ny, row0, seed, obst_frac, obst_seed, gi, gj, st));
  HIPC(c, hipStreamSynchronize(st));
  return DYMU_OK;
}

int dymu_device_alloc(dymu_ctx* c, size_t bytes, void** p) {
  if (!c || !p) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMalloc(p, bytes));
  return DYMU_OK;
}

int dymu_device_free(dymu_ctx* c, void* p) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipFree(p));
  return DYMU_OK;
}

int dymu_memcpy_d2h(dymu_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return DYMU_OK;
}

int dymu_memcpy_h2d(dymu_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return DYMU_OK;
}

int dymu_set_profiling(dymu_ctx* c, int on) {
  if (!c) return DYMU_ERR_ARG;
  c->profiling = on;
  return DYMU_OK;
}

int dymu_last_pass_timing(dymu_ctx* c, double* ms, uint64_t* n) {
  if (!c) return DYMU_ERR_ARG;
  if (ms) *ms = c->last_pass_ms;
  if (n) *n = c->last_launches;
  return DYMU_OK;
}

}  // extern "C"
