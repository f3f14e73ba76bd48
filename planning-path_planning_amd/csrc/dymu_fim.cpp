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
#include <cmath>
#include <chrono>
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
  uint32_t* d_xchg = nullptr;  // k_exchange's block ticket (zero between launches)

  // 3: two 8x8 tiles per wave (red-black), 4: v3 body + priority passes;
  // 5: priority passes on 16x16 tiles (one per wave, 16-wave workgroups);
  // 0 (default): per domain, 5 from prio_min_tiles 8x8 tiles up, else 3.  Since the
  // checkerboard passes (v23) kernel 5 is the faster one at every size measured (256^2:
  // 0.45 vs 0.51 ms, 1024^2: 1.22 vs 1.63, 2048^2: 2.4-2.9 vs 4.1-4.3, 2896^2: 3.52 vs
  // 6.60; profiles/r02/small_grids.txt), so the threshold is 0.
  // DYMU_KERNEL overrides
  int variant = 0;
  uint32_t prio_min_tiles = 0;  // DYMU_PRIO_MIN_TILES
  uint32_t prio_target = 0;  // v4/v5: tiles relaxed per pass; 0 = per-variant default
  double prio_kappa = 0.5;   // v4: histogram bin width / mean F (DYMU_PRIO_KAPPA)
  float prio_frac = 0.0f;    // v4: ... or this fraction of the active list (DYMU_PRIO_FRAC)
  int prio_trace = -1;       // v4: stamp phases of this pass index (DYMU_PRIO_TRACE)
  unsigned long long* d_trace = nullptr;
  int prune = 1;             // v4/v5 exact activation pruning (DYMU_PRUNE=0 disables)
  int occupancy[6] = {0, 0, 0, 6, 5, 1};  // pass workgroups per CU (occupancy API)
  // passes before the first convergence read-back (then doubling to 64): 16 saves two
  // host round trips per solve (4096^2: 5.88 vs 5.96 ms; DYMU_FIRST_BATCH)
  uint64_t first_batch = 16;
  // convergence checks without host round trips: every pass posts the tiles queued for
  // it to a host-coherent mailbox and the host keeps max_batch passes queued ahead of the
  // running one (2, converge_stream; default), or the first pass of each batch posts and
  // the next batch is queued before the host reads it (1, converge_pipelined), or the
  // host synchronises on the counters after each batch (0, converge).  DYMU_PIPELINE,
  // DYMU_MAX_BATCH (passes queued ahead / batch size) override.  16384^2: 35.94 / 36.13 /
  // 36.58 ms, 4096^2: 5.85 / 5.91 / 5.96 ms (profiles/r02/pipe_*.log)
  int pipeline = 2;
  uint64_t max_batch = 4;
  unsigned long long* h_mail = nullptr;  // pinned, host-coherent: (seq << 32) | pending
  unsigned long long* d_mail = nullptr;  // its device address
  uint32_t mail_seq = 0;
  // a post armed by dymu_dom_post for the next launched pass (sharded loop)
  const int32_t* arm_src = nullptr;
  uint32_t arm_seq = 0;
  unsigned long long* arm_dst = nullptr;       // another post target (the peer status ring)
  const unsigned long long* arm_ext = nullptr;  // ... with these 4 status words
  int prio_debug = 0;        // v4: print the state after the first N passes (DYMU_PRIO_DEBUG)

  // tile workspace
  uint32_t tiles_cap = 0;
  uint32_t* d_lists = nullptr;       // 3 lists x kShards shards x tiles_cap
  uint32_t* d_counts = nullptr;      // 3 x kShards words, own block
  uint32_t* d_tile_epoch = nullptr;  // tiles_cap
  unsigned long long* d_stats = nullptr;  // kStatSlots
  // v4 priority state: keys 3 x tiles_cap, hist 3 x kShards x kBins,
  // prio = {minkey[3] (u64), base[3] (f64), delta (f64)}
  unsigned long long* d_keys = nullptr;
  uint32_t keys_cap = 0;
  uint32_t* d_hist = nullptr;
  unsigned long long* d_prio = nullptr;
  uint32_t epoch_base = 0;
  uint32_t* h_count = nullptr;  // pinned
  unsigned long long* h_probe = nullptr;  // pinned [2]: early-exit probe (max T, min key)
  uint64_t* d_band = nullptr;   // early-exit band indices (device)
  uint64_t band_cap = 0;
  // dymu_find_equal / dymu_scatter exchange indices and values through this pinned,
  // host-coherent, device-mapped buffer, which their kernels read and write in place
  void* h_xfer = nullptr;       // host address
  void* d_xfer = nullptr;       // its device address
  uint64_t xfer_cap = 0;        // bytes
  unsigned long long* d_region = nullptr;  // dymu_region_stats' 8 device words
  unsigned long long* d_scratch = nullptr;  // 8 words of per-call device scalars
  double* d_lut = nullptr;      // computeCostMap LUT (device copy)
  size_t lut_cap = 0;

  // host-solve staging
  double* d_F = nullptr;
  double* d_T = nullptr;
  uint64_t cells_cap = 0;
  // the staged d_T holds the converged map of the last host solve of this grid
  bool host_valid = false;
  uint32_t host_nx = 0, host_ny = 0, host_gi = 0, host_gj = 0;

  // current domain (whole grid or one row slab) being solved
  struct Dom {
    bool live = false;
    int variant = 3;
    PassArgs a{};
    uint32_t ntiles = 0;
    uint32_t eb = 0;
    uint64_t p = 0;         // next pass index
    uint64_t launches = 0;
    uint64_t max_passes = 0;
    int blocks = 0;
    bool rehist = false;  // rebuild each list's histogram from its final keys
    uint32_t* lists[3] = {nullptr, nullptr, nullptr};
    uint32_t* counts[3] = {nullptr, nullptr, nullptr};
    size_t prof_used = 0;
  } dom;

  // per-pass statistics (kernel 5; dymu_set_pass_stats): kPassStatCap records of
  // kShards x kPsWords words, pass p at p % kPassStatCap
  int pass_stats = 0;
  uint32_t* d_pstat = nullptr;
  // kernel 5 edge columns (PassArgs::ec): 32 doubles per 16x16 tile; 1.5-2% per
  // 16384^2 solve against the per-row W / E halo loads (profiles/r03/ec)
  int use_ec = 1;
  // device memory kinds (dev_alloc): the maps (dymu_device_alloc, host-solve staging):
  // uncached -- a pass's write-backs leave no dirty L2 lines for its end-of-kernel
  // release (27.52-27.72 vs 28.06-28.28 ms per 16384^2 solve, profiles/r06/map_mem_ab.txt);
  // the tile workspace: cached (uncached lists / keys / edge columns cost +0.6%).
  // DYMU_MAP_MEM / DYMU_WS_MEM override (A/B)
  int map_mem = 2, ws_mem = 0, ec_mem = 0, key_mem = 0;
  double* d_ec = nullptr;
  uint64_t ec_cap = 0;  // tiles
  // windowed updates with increases: theta reset (0, default) or the raise front (1,
  // DYMU_RAISE=1: exact dependency cone, measured slower on config 5 -- 9.5 vs 4.1 ms
  // at 4096^2, profiles/r03/configs_4096_r03c.json); the last
  // update's raise passes, raise visits, cells invalidated
  int raise = 0;
  uint64_t last_update[4] = {0, 0, 0, 0};

  // profiling
  int profiling = 0;
  std::vector<hipEvent_t> prof_ev;
  double last_pass_ms = 0.0;
  uint64_t last_launches = 0;
  uint64_t last_timed = 0;  // sampled launches behind last_pass_ms

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

// Device memory by kind (A/B knobs): 0 hipMalloc (coarse-grained,
// L2-cached), 1 fine-grained, 2 uncached (no L2: nothing dirty for a kernel's
// end-of-pass release to write back)
hipError_t dev_alloc(void** p, size_t bytes, int kind) {
  if (kind == 1) return hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained);
  if (kind == 2) return hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
  return hipMalloc(p, bytes);
}
template <class P>
hipError_t dev_alloc(P** p, size_t bytes, int kind) {
  return dev_alloc(reinterpret_cast<void**>(p), bytes, kind);
}

int ensure_tiles(dymu_ctx* c, uint32_t ntiles, hipStream_t st) {
  if (ntiles <= c->tiles_cap) return DYMU_OK;
  if (c->d_lists) (void)hipFree(c->d_lists);
  if (c->d_tile_epoch) (void)hipFree(c->d_tile_epoch);
  c->d_lists = nullptr;
  c->d_tile_epoch = nullptr;
  c->tiles_cap = 0;
  HIPC(c, dev_alloc(&c->d_lists, sizeof(uint32_t) * 3ull * kShards * ntiles, c->ws_mem));
  HIPC(c, dev_alloc(&c->d_tile_epoch, sizeof(uint32_t) * (uint64_t)ntiles, c->ws_mem));
  HIPC(c, hipMemsetAsync(c->d_tile_epoch, 0, sizeof(uint32_t) * (uint64_t)ntiles, st));
  c->tiles_cap = ntiles;
  c->epoch_base = 0;
  return DYMU_OK;
}

int ensure_prio(dymu_ctx* c, uint32_t ntiles) {
  // 3 list histograms + 2 rebuild buffers (deterministic mode)
  if (!c->d_hist) HIPC(c, hipMalloc(&c->d_hist, sizeof(uint32_t) * 5 * kShards * kBins));
  if (!c->d_prio) HIPC(c, hipMalloc(&c->d_prio, sizeof(unsigned long long) * 8));
  if (ntiles <= c->keys_cap) return DYMU_OK;
  if (c->d_keys) (void)hipFree(c->d_keys);
  c->d_keys = nullptr;
  c->keys_cap = 0;
  HIPC(c, dev_alloc(&c->d_keys, sizeof(unsigned long long) * 3ull * ntiles, c->key_mem));
  c->keys_cap = ntiles;
  return DYMU_OK;
}

// The transfer buffer of dymu_find_equal / dymu_scatter: pinned host memory the
// kernels access in place, so no copy command stands between the host's data and
// the kernel.  Round 5's version staged through hipMallocAsync memory with copies; on
// this stack (ROCm 7.2, gfx950) a stream-ordered pool allocation is not seen alike by
// the copy paths and the kernels beyond its first 4 KiB page -- a kernel read an
// earlier allocation's bytes, whatever the copy's source, synchronicity or ordering
// (tools/copy_order_probe.hip, profiles/r06/copy_order_probe.jsonl).
// Callers synchronise the stream before the buffer is rewritten.
int ensure_xfer(dymu_ctx* c, uint64_t bytes) {
  if (bytes <= c->xfer_cap) return DYMU_OK;
  if (c->h_xfer) HIPC(c, hipHostFree(c->h_xfer));
  c->h_xfer = c->d_xfer = nullptr;
  c->xfer_cap = 0;
  bytes = std::max<uint64_t>(bytes, 1u << 16);
  HIPC(c, hipHostMalloc(&c->h_xfer, bytes, hipHostMallocCoherent | hipHostMallocMapped));
  c->xfer_cap = bytes;
  HIPC(c, hipHostGetDevicePointer(&c->d_xfer, c->h_xfer, 0));
  return DYMU_OK;
}

int ensure_cells(dymu_ctx* c, uint64_t cells) {
  if (cells <= c->cells_cap) return DYMU_OK;
  c->host_valid = false;
  if (c->d_F) (void)hipFree(c->d_F);
  if (c->d_T) (void)hipFree(c->d_T);
  c->d_F = c->d_T = nullptr;
  c->cells_cap = 0;
  HIPC(c, dev_alloc(&c->d_F, sizeof(double) * cells, c->map_mem));
  HIPC(c, dev_alloc(&c->d_T, sizeof(double) * cells, c->map_mem));
  c->cells_cap = cells;
  return DYMU_OK;
}

double* prio_delta(dymu_ctx* c) { return reinterpret_cast<double*>(c->d_prio + 6); }
double* prio_base(dymu_ctx* c, uint64_t q) { return reinterpret_cast<double*>(c->d_prio + 3 + q); }
unsigned long long* prio_minkey(dymu_ctx* c, uint64_t q) { return c->d_prio + q; }
uint32_t* prio_hist(dymu_ctx* c, uint64_t q) { return c->d_hist + q * kShards * kBins; }
unsigned long long* prio_keys(dymu_ctx* c, uint64_t q) {
  return c->d_keys + q * (uint64_t)c->dom.ntiles;
}

int tile_w(int variant) { return variant == 5 ? 16 : kWaveTile; }
int tile_h(int variant) { return variant == 5 ? 16 : kWaveTile; }
bool valid_variant(int v) { return v == 0 || (v >= 3 && v <= 5); }
bool is_prio(int variant) { return variant == 4 || variant == 5; }

// Passes a domain may run beyond max_passes: converge() checks the cap between
// batches of up to 64 launches (converge_pipelined has two such batches queued),
// so epochs up to eb + max_passes + kPassSlack + 2 can be stamped; the epoch-wrap
// guard in dom_begin reserves that many.
constexpr uint64_t kPassSlack = 128;

// Leave the live domain (error paths included): later domains stamp epochs
// above every epoch this one used, so no tile_epoch entry can block them.
void dom_retire(dymu_ctx* c) {
  auto& D = c->dom;
  c->arm_seq = 0;  // a post armed for a pass that will not run
  c->arm_src = nullptr;
  c->arm_dst = nullptr;
  c->arm_ext = nullptr;
  if (!D.live) return;
  c->epoch_base = D.eb + (uint32_t)D.p + 4u;
  D.live = false;
}

// ---- domain primitives (whole grid, or one row slab with ghost rows) ----
// cold = true: T := +inf (incl. ghost rows) and the goal seeded (a fresh solve);
// false: T is kept and the caller seeds list 0 (windowed re-propagation).
// need_keys: the caller needs tile keys (lower bounds on every value the passes can
// still produce, dymu_solve_until_device): the plain FIM kernel 3 has none, kernel 4
// runs instead.
// the pass kernel a domain of nx x nrows cells runs
int dom_variant(const dymu_ctx* c, uint32_t nx, uint32_t nrows, bool need_keys) {
  int variant = c->variant;
  if (variant == 0) {
    const uint64_t t8 = (uint64_t)((nx + kWaveTile - 1) / kWaveTile) *
                        (uint64_t)((nrows + kWaveTile - 1) / kWaveTile);
    variant = t8 >= c->prio_min_tiles ? 5 : 3;
  }
  if (need_keys && !is_prio(variant)) variant = 4;
  if (c->opts.deterministic) variant = 5;
  return variant;
}

int dom_begin(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t nrows, uint64_t ld,
              int ghost_lo, int ghost_hi, int64_t gi, int64_t gj, hipStream_t st,
              bool cold = true, bool need_keys = false) {
  if (!dF || !dT || nx == 0 || nrows == 0 || ld < nx) return DYMU_ERR_ARG;
  const int variant = dom_variant(c, nx, nrows, need_keys);
  const int TWd = tile_w(variant), THd = tile_h(variant);
  if (ghost_hi && (nrows % (uint32_t)THd) != 0) return DYMU_ERR_ARG;
  if (gj >= 0 && (gi < 0 || gi >= (int64_t)nx || gj >= (int64_t)nrows)) return DYMU_ERR_ARG;
  const uint32_t ntx = (uint32_t)((nx + TWd - 1) / TWd), nty = (uint32_t)((nrows + THd - 1) / THd);
  const uint64_t ntiles64 = (uint64_t)ntx * nty;
  if (ntiles64 >= (1ull << 31)) return DYMU_ERR_ARG;
  const uint32_t ntiles = (uint32_t)ntiles64;
  dom_retire(c);  // a domain abandoned mid-solve (an error, or no dom_finish)
  int rc = ensure_tiles(c, ntiles, st);
  if (rc) return rc;
  if (is_prio(variant) && (rc = ensure_prio(c, ntiles)) != DYMU_OK) return rc;
  auto& D = c->dom;
  D = dymu_ctx::Dom{};
  D.variant = variant;
  D.ntiles = ntiles;
  D.max_passes = c->opts.max_passes > 0 ? (uint64_t)c->opts.max_passes : 4ull * ntiles + 1024ull;
  if ((uint64_t)c->epoch_base + D.max_passes + kPassSlack + 8 >= 0xFFFFFFF0ull) {
    HIPC(c, hipMemsetAsync(c->d_tile_epoch, 0, sizeof(uint32_t) * (uint64_t)ntiles, st));
    c->epoch_base = 0;
  }
  D.eb = c->epoch_base;
  c->epoch_base = D.eb + 4u;  // the seed's epoch stays used even if a step below fails
  const uint64_t lstride = (uint64_t)kShards * ntiles;
  for (int q = 0; q < 3; ++q) {
    D.lists[q] = c->d_lists + q * lstride;
    D.counts[q] = c->d_counts + q * kShards;
  }
  HIPC(c, hipMemsetAsync(c->d_counts, 0, sizeof(uint32_t) * 3 * kShards, st));
  HIPC(c, hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * kShards * kStatSlots, st));
  if (cold)
    HIPC(c, launch_fill_inf(dT, ld, nx, ghost_lo ? -1 : 0, (int64_t)nrows + (ghost_hi ? 1 : 0), st));
  PassArgs& a = D.a;
  if (is_prio(D.variant)) {
    HIPC(c, launch_prio_init(dF, (int64_t)ld, nx, nrows, c->d_keys, 3ull * ntiles, c->d_hist,
                             3ull * kShards * kBins, c->d_prio,
                             reinterpret_cast<double*>(c->d_prio + 3), prio_delta(c), c->prio_kappa,
                             st));
    // kernel 5 relaxes one colour of a checkerboard of tiles per pass (PassArgs::checker):
    // no visit then reads a halo another wave is writing, which cuts the tile visits
    // by a third (16384^2: 36.8 -> 33.8 ms, 4096^2: 5.98 -> 5.48 ms, v23,
    // profiles/r02/checker_sweep.txt).  DYMU_CHECKER=0 disables it.
    bool checker = D.variant == 5;
    if (const char* kv = std::getenv("DYMU_CHECKER")) checker = D.variant == 5 && std::atoi(kv);
    if (c->opts.deterministic) checker = true;
    // default per pass: 64 8x8 tiles per CU (v4) / 16x16 tiles per CU (v5), the measured
    // optima: with the checkerboard 6 / 12 / 14 per CU for whole grids below 2^17 /
    // below 2^20 / from 2^20 tiles (4096^2 / 8192^2 / 16384^2), 10 for slabs (8 without:
    // same pass time in the rehearsal, 6% fewer exchange rounds); without it 4 / 8 / 10
    // (v11, v18: profiles/r02/sweep_v18b.log)
    const bool whole5 = D.variant == 5 && !ghost_lo && !ghost_hi;
    const uint32_t per_cu = D.variant != 5                            ? 64u
                            : !whole5                                  ? (checker ? 10u : 8u)
                            : ntiles < (1u << 17)                      ? (checker ? 6u : 4u)
                            : ntiles >= (1u << 20)                     ? (checker ? 14u : 10u)
                                                                       : (checker ? 12u : 8u);
    a.checker = checker;
    a.target = c->prio_target ? c->prio_target : (uint32_t)c->cu_count * per_cu;
    a.target_frac = c->prio_frac;
    a.prune = c->prune;
    a.delta = prio_delta(c);
  }
  if (cold && gj >= 0) {
    const uint32_t gtile = (uint32_t)(gj / THd) * ntx + (uint32_t)(gi / TWd);
    HIPC(c, launch_seed(dT, ld, gi, gj, D.lists[0], D.counts[0], c->d_tile_epoch, D.eb + 1, gtile,
                        1, st));
    if (is_prio(D.variant))
      HIPC(c, launch_prio_seed(c->d_keys, c->d_hist, c->d_prio, gtile, 0.0, st));
  }
  // kernel 5 edge columns: +inf (cold) plus the goal's tile; a warm domain
  // (resolve_core) rebuilds them from T once its seeding kernels have run (ec_sync)
  a.ec = nullptr;
  if (D.variant == 5 && c->use_ec) {
    if (c->ec_cap < ntiles) {
      if (c->d_ec) (void)hipFree(c->d_ec);
      c->d_ec = nullptr;
      c->ec_cap = 0;
      HIPC(c, dev_alloc(&c->d_ec, sizeof(double) * 32 * (uint64_t)ntiles, c->ec_mem));
      c->ec_cap = ntiles;
    }
    a.ec = c->d_ec;
    if (cold) {
      HIPC(c, launch_fill_inf(c->d_ec, 0, 32u * ntiles, 0, 1, st));
      if (gj >= 0) {
        const uint32_t gtile = (uint32_t)(gj / THd) * ntx + (uint32_t)(gi / TWd);
        HIPC(c, launch_ec_rebuild(dT, ld, nx, nrows, c->d_ec, ntx, gtile, gtile + 1, st));
      }
    }
  }
  a.F = dF;
  a.T = dT;
  a.ld = (int64_t)ld;
  a.nx = nx;
  a.ny = nrows;
  a.ntx = (int)ntx;
  a.nty = (int)nty;
  a.ghost_lo = ghost_lo;
  a.ghost_hi = ghost_hi;
  // v5: a sweep cap of 16 bounds the visit (capped tiles re-queue themselves); on large
  // grids a pass is ended by the capped visits of the busiest SIMDs, so there a visit
  // also stops sweeping 14 us into the pass (re-queued like a capped one): 46.0 vs
  // 49.2 ms at 16384^2 (v9), 15.6 vs 16.0 ms at 8192^2 (v11).  Whole grids from 2^18
  // tiles; slabs (more exchange rounds with it) only from 2^20.
  // v33 (13 instead of 16.5 fp64 instructions per update) and the strided entries moved
  // the optimum for those grids to a cap of 18 and a deadline of 15 us: 28.48-28.54 vs
  // 29.90 ms at 16384^2, 1,392 vs 1,562 passes (profiles/r04/v34_knobs.txt)
  const bool big = ntiles >= (1u << 20) || (!ghost_lo && !ghost_hi && ntiles >= (1u << 18));
  a.max_inner = c->opts.max_inner > 0 ? c->opts.max_inner
                : variant == 5            ? (big ? 18 : 16)
                                          : 4 * (TWd + THd);
  if (const char* kv = std::getenv("DYMU_MAX_INNER")) a.max_inner = std::max(1, std::atoi(kv));

  a.sweep_deadline = (variant == 5 && big) ? 1500u : 0u;  // 10-ns s_memrealtime ticks
  if (const char* kv = std::getenv("DYMU_SWEEP_DEADLINE"))
    a.sweep_deadline = (uint32_t)std::max(0, std::atoi(kv));
  // at most 90% of the listed tiles per pass: a short list (the serpentine maze, the first
  // passes of an open grid) is otherwise relaxed whole, and every improvement behind the
  // front re-relaxes the tiles downstream of it; DYMU_PRIO_CAPFRAC=0: off
  a.cap_frac = 0.9f;
  if (const char* kv = std::getenv("DYMU_PRIO_CAPFRAC")) a.cap_frac = (float)std::atof(kv);
  // kernel 5: list entries carry their first-insertion key bin, so a key-deferred entry
  // skips its tile loads (PassArgs::pack_bins); tile indices must fit below the bin field,
  // and deterministic mode's histogram is rebuilt from the current keys instead
  a.pack_bins = variant == 5 && D.ntiles <= kTileMask + 1u && !c->opts.deterministic;
  if (const char* kv = std::getenv("DYMU_PACK_BINS")) a.pack_bins = a.pack_bins && std::atoi(kv);
  a.exact_sqrt = c->opts.exact_sqrt != 0;
  if (const char* kv = std::getenv("DYMU_EXACT_SQRT")) a.exact_sqrt = std::atoi(kv) != 0;
  if (c->opts.deterministic) {
    a.sweep_deadline = 0;  // the deadline makes the schedule timing-dependent
    D.rehist = true;       // and so do the first-insertion keys of the histogram
    HIPC(c, hipMemsetAsync(c->d_hist + (uint64_t)3 * kShards * kBins, 0,
                           sizeof(uint32_t) * 2 * kShards * kBins, st));
  }
  a.shard_cap = ntiles;
  a.tile_epoch = c->d_tile_epoch;
  a.stats = c->d_stats;
  a.goal_tx = gj >= 0 ? (int)(gi / TWd) : 0;
  a.goal_ty = gj >= 0 ? (int)(gj / THd) : 0;
  if (c->pass_stats && D.variant == 5) {
    const size_t bytes = sizeof(uint32_t) * (size_t)kPassStatCap * kShards * kPsWords;
    if (!c->d_pstat) HIPC(c, hipMalloc(&c->d_pstat, bytes));
    HIPC(c, hipMemsetAsync(c->d_pstat, 0, bytes, st));
  }
  // resident workgroups per CU at the kernel's register / LDS budget
  D.blocks = c->opts.grid_blocks > 0 ? c->opts.grid_blocks
                                      : c->cu_count * c->occupancy[D.variant];
  D.live = true;
  return DYMU_OK;
}

// report_seq != 0: the batch's first pass posts (report_seq, tiles pending) to the mailbox
int dom_launch(dymu_ctx* c, uint64_t K, hipStream_t st, uint32_t report_seq = 0) {
  auto& D = c->dom;
  if (!D.live) return DYMU_ERR_STATE;
  if (D.p + K > D.max_passes + kPassSlack) {  // beyond the epochs dom_begin reserved
    c->last_error = "pass cap reached before convergence";
    dom_retire(c);
    return DYMU_ERR_NOT_CONVERGED;
  }
  PassArgs& a = D.a;
  const bool prof = c->profiling != 0;
  for (uint64_t k = 0; k < K; ++k, ++D.p) {
    const uint64_t p = D.p;
    a.list_in = D.lists[p % 3];
    a.count_in = D.counts[p % 3];
    a.list_out = D.lists[(p + 1) % 3];
    a.count_out = D.counts[(p + 1) % 3];
    a.count_clear = D.counts[(p + 2) % 3];
    a.epoch = D.eb + (uint32_t)p + 2u;
    a.checker_parity = (uint32_t)(p & 1u);
    if (is_prio(D.variant)) {
      a.key_in = prio_keys(c, p % 3);
      a.key_out = prio_keys(c, (p + 1) % 3);
      a.hist_in = prio_hist(c, p % 3);
      a.hist_out = prio_hist(c, (p + 1) % 3);
      a.hist_clear = prio_hist(c, (p + 2) % 3);
      a.minkey_in = prio_minkey(c, p % 3);
      a.minkey_out = prio_minkey(c, (p + 1) % 3);
      a.minkey_clear = prio_minkey(c, (p + 2) % 3);
      a.base_in = prio_base(c, p % 3);
      a.base_out = prio_base(c, (p + 1) % 3);
    }
    if (k == 0 && report_seq) {
      a.report = c->d_mail;
      a.report_seq = report_seq;
    } else if (c->arm_seq) {
      a.report = c->arm_dst ? c->arm_dst : c->d_mail;
      a.report_seq = c->arm_seq;
      a.report_src = c->arm_src;
      a.report_ext = c->arm_ext;
      c->arm_seq = 0;
      c->arm_src = nullptr;
      c->arm_dst = nullptr;
      c->arm_ext = nullptr;
    }
    a.pstat = (c->pass_stats && D.variant == 5 && c->d_pstat)
                  ? c->d_pstat + (p % kPassStatCap) * (uint64_t)kShards * kPsWords
                  : nullptr;
    const bool tr = is_prio(D.variant) && c->prio_trace >= 0 && p == (uint64_t)c->prio_trace;
    if (tr) {
      if (!c->d_trace)
        HIPC(c, hipMalloc(&c->d_trace, sizeof(unsigned long long) * kTracePts * 65536));
      HIPC(c, hipMemsetAsync(c->d_trace, 0, sizeof(unsigned long long) * kTracePts * D.blocks, st));
      a.trace = c->d_trace;
    }
    if (D.rehist) {  // deterministic mode: b* from the list's final keys
      uint32_t* rh = c->d_hist + (uint64_t)3 * kShards * kBins;  // 2 alternating buffers
      uint32_t* mine = rh + (p & 1u) * kShards * kBins;
      uint32_t* next = rh + ((p + 1) & 1u) * kShards * kBins;
      HIPC(c, launch_rehist(a.list_in, a.count_in, a.shard_cap, a.key_in, a.base_in, a.delta,
                            mine, next, st));
      a.hist_in = mine;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof && D.launches % (uint64_t)c->profiling == 0) {
      while (c->prof_ev.size() < D.prof_used + 2) {
        hipEvent_t e;
        HIPC(c, hipEventCreate(&e));
        c->prof_ev.push_back(e);
      }
      e0 = c->prof_ev[D.prof_used];
      e1 = c->prof_ev[D.prof_used + 1];
      D.prof_used += 2;
    }
    HIPC(c, D.variant == 4   ? launch_pass_prio(a, D.blocks, st, e0, e1)
            : D.variant == 5 ? launch_pass_prio16(a, D.blocks, st, e0, e1)
                             : launch_pass_rb(a, D.blocks, st, e0, e1));
    ++D.launches;
    a.report = nullptr;
    a.report_src = nullptr;
    a.report_ext = nullptr;
    if (tr) {
      a.trace = nullptr;
      std::vector<unsigned long long> h((size_t)kTracePts * D.blocks);
      HIPC(c, hipStreamSynchronize(st));
      HIPC(c, hipMemcpy(h.data(), c->d_trace, sizeof(unsigned long long) * h.size(),
                        hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull;
      for (int b = 0; b < D.blocks; ++b) t0 = std::min(t0, h[(size_t)b * kTracePts]);
      std::fprintf(stderr, "TRACE pass %llu blocks %d (10ns ticks rel. first start)\n",
                   (unsigned long long)p, D.blocks);
      for (int b = 0; b < D.blocks; ++b) {
        const unsigned long long* t = &h[(size_t)b * kTracePts];
        auto rel = [&](int k) { return t[k] ? (long long)(t[k] - t0) : -1ll; };
        std::fprintf(stderr, "B %d %lld %lld %lld %lld %lld %llu %llu %lld %lld %lld %llu\n", b,
                     rel(0), rel(1), rel(2), rel(3), rel(4), t[5] >> 32, t[5] & 0xffffffffull,
                     rel(6), rel(7), rel(8), t[9]);
      }
    }
    if (is_prio(D.variant) && c->prio_debug && p < (uint64_t)c->prio_debug) {
      unsigned long long pr[8];
      uint32_t h[kShards * kBins], cnt[kShards];
      HIPC(c, hipStreamSynchronize(st));
      HIPC(c, hipMemcpy(pr, c->d_prio, sizeof pr, hipMemcpyDeviceToHost));
      HIPC(c, hipMemcpy(h, prio_hist(c, (p + 1) % 3), sizeof h, hipMemcpyDeviceToHost));
      HIPC(c, hipMemcpy(cnt, D.counts[(p + 1) % 3], sizeof cnt, hipMemcpyDeviceToHost));
      double dd[4];
      std::memcpy(dd, pr + 3, sizeof dd);
      uint32_t n = 0, hs[kBins] = {0};
      for (int q = 0; q < kShards; ++q) n += cnt[q];
      for (int q = 0; q < kShards * kBins; ++q) hs[q % kBins] += h[q];
      double mk[3];
      std::memcpy(mk, pr, sizeof mk);
      std::fprintf(stderr, "pass %llu n_out %u minkey %g %g %g base %g %g %g delta %g hist:",
                   (unsigned long long)p, n, mk[0], mk[1], mk[2], dd[0], dd[1], dd[2], dd[3]);
      for (int b = 0; b < kBins; ++b) if (hs[b]) std::fprintf(stderr, " %d:%u", b, hs[b]);
      std::fprintf(stderr, "\n");
    }
  }
  return DYMU_OK;
}

// tiles queued for the next pass (synchronises the stream)
int dom_pending(dymu_ctx* c, hipStream_t st, uint64_t* out) {
  auto& D = c->dom;
  if (!D.live) return DYMU_ERR_STATE;
  HIPC(c, hipMemcpyAsync(c->h_count, D.counts[D.p % 3], sizeof(uint32_t) * kShards,
                         hipMemcpyDeviceToHost, st));
  HIPC(c, hipStreamSynchronize(st));
  uint64_t pending = 0;
  for (int q = 0; q < kShards; ++q) pending += c->h_count[q];
  *out = pending;
  return DYMU_OK;
}

int dom_merge(dymu_ctx* c, const double* lo, const double* hi, int32_t* d_pending, hipStream_t st) {
  auto& D = c->dom;
  if (!D.live) return DYMU_ERR_STATE;
  if ((lo && !D.a.ghost_lo) || (hi && !D.a.ghost_hi)) return DYMU_ERR_ARG;
  const uint64_t p = D.p;
  if (lo || hi)
    HIPC(c, launch_merge_ghosts(D.a.T, D.a.ld, D.a.nx, D.a.ny, lo, hi, D.a.ntx, D.a.nty,
                                tile_w(D.variant), D.lists[p % 3], D.counts[p % 3], D.ntiles,
                                c->d_tile_epoch, D.eb + (uint32_t)p + 1u,
                                is_prio(D.variant) ? prio_keys(c, p % 3) : nullptr,
                                is_prio(D.variant) ? prio_hist(c, p % 3) : nullptr,
                                is_prio(D.variant) ? prio_minkey(c, p % 3) : nullptr,
                                is_prio(D.variant) ? prio_base(c, p % 3) : nullptr,
                                is_prio(D.variant) ? prio_delta(c) : nullptr, st));
  if (d_pending) HIPC(c, launch_sum_counts(D.counts[p % 3], d_pending, st));
  return DYMU_OK;
}

int dom_exchange(dymu_ctx* c, const double* lo, const double* hi, int32_t* d_total,
                 hipStream_t st) {
  auto& D = c->dom;
  if (!D.live) return DYMU_ERR_STATE;
  if (!d_total || (lo && !D.a.ghost_lo) || (hi && !D.a.ghost_hi)) return DYMU_ERR_ARG;
  const uint64_t p = D.p;
  HIPC(c, launch_exchange(D.a.T, D.a.ld, D.a.nx, D.a.ny, lo, hi, D.a.ntx, D.a.nty,
                          tile_w(D.variant), D.lists[p % 3], D.counts[p % 3], D.ntiles,
                          c->d_tile_epoch, D.eb + (uint32_t)p + 1u,
                          is_prio(D.variant) ? prio_keys(c, p % 3) : nullptr,
                          is_prio(D.variant) ? prio_hist(c, p % 3) : nullptr,
                          is_prio(D.variant) ? prio_minkey(c, p % 3) : nullptr,
                          is_prio(D.variant) ? prio_base(c, p % 3) : nullptr,
                          is_prio(D.variant) ? prio_delta(c) : nullptr, c->d_xchg, d_total, st));
  return DYMU_OK;
}

// One round of the sharded loop with the ghost merge inside the passes (kernel 5,
// K >= 2): the first pass min-merges the rows received after the previous round
// and queues the tiles under improved columns for the second; the second pass
// writes *d_total = tiles queued for the first + for the second pass.  0 on every
// rank is the fixed point: nothing was queued after the previous round, and the
// rows it produced improved no ghost.
bool dom_round_ok(const dymu_ctx* c, uint64_t K) {
  // not in deterministic mode: the in-pass merge writes ghost rows that the same
  // pass's boundary visits may be reading
  return c->dom.live && c->dom.variant == 5 && K >= 2 && !c->opts.deterministic;
}

int dom_round(dymu_ctx* c, uint64_t K, const double* lo, const double* hi, int32_t* d_total,
              hipStream_t st) {
  auto& D = c->dom;
  if (!dom_round_ok(c, K)) return DYMU_ERR_STATE;
  if (!d_total || (lo && !D.a.ghost_lo) || (hi && !D.a.ghost_hi)) return DYMU_ERR_ARG;
  uint32_t* scratch = reinterpret_cast<uint32_t*>(c->d_scratch + 7);
  D.a.merge_lo = lo;
  D.a.merge_hi = hi;
  D.a.tot_save = scratch;
  int rc = dom_launch(c, 1, st);
  D.a.merge_lo = D.a.merge_hi = nullptr;
  D.a.tot_save = nullptr;
  if (rc) return rc;
  D.a.tot_prev = scratch;
  D.a.tot_out = d_total;
  rc = dom_launch(c, 1, st);
  D.a.tot_prev = nullptr;
  D.a.tot_out = nullptr;
  if (rc) return rc;
  return dom_launch(c, K - 2, st);
}

// The peer round (include/dymu_fim.h dymu_dom_round_peer): dom_round whose first pass
// also pushes the owned boundary rows into the neighbours' receive rows with a tag and
// reads its own receive rows after their tags; the second pass records the status.
int dom_round_peer(dymu_ctx* c, uint64_t K, const dymu_peer_links& L, hipStream_t st) {
  auto& D = c->dom;
  if (!dom_round_ok(c, K)) return DYMU_ERR_STATE;
  if (!L.ctl || (L.recv[0] && !D.a.ghost_lo) || (L.recv[1] && !D.a.ghost_hi)) return DYMU_ERR_ARG;
  for (int s = 0; s < 2; ++s)
    if ((L.recv[s] && !L.recv_tag[s]) || (L.send[s] && (!L.send_tag[s] || !L.last[s])))
      return DYMU_ERR_ARG;
  PeerCtl* pc = static_cast<PeerCtl*>(L.ctl);
  uint32_t* scratch = reinterpret_cast<uint32_t*>(c->d_scratch + 7);
  PassArgs& a = D.a;
  a.merge_lo = L.recv[0];
  a.merge_hi = L.recv[1];
  for (int s = 0; s < 2; ++s) {
    a.merge_tag[s] = L.recv[s] ? L.recv_tag[s] : nullptr;
    a.push_dst[s] = L.send[s];
    a.push_tag[s] = L.send_tag[s];
    a.push_last[s] = L.last[s];
  }
  a.peer = pc;
  a.tot_save = scratch;
  int rc = dom_launch(c, 1, st);
  a.merge_lo = a.merge_hi = nullptr;
  for (int s = 0; s < 2; ++s) {
    a.merge_tag[s] = nullptr;
    a.push_dst[s] = nullptr;
    a.push_tag[s] = nullptr;
    a.push_last[s] = nullptr;
  }
  a.tot_save = nullptr;
  if (rc) {
    a.peer = nullptr;
    return rc;
  }
  a.tot_prev = scratch;
  a.tot_out = reinterpret_cast<int32_t*>(&pc->pend);
  rc = dom_launch(c, 1, st);
  a.tot_prev = nullptr;
  a.tot_out = nullptr;
  a.peer = nullptr;
  if (rc) return rc;
  return dom_launch(c, K - 2, st);
}

int dom_finish(dymu_ctx* c, hipStream_t st, dymu_stats* stats, double ms) {
  auto& D = c->dom;
  if (!D.live) return DYMU_ERR_STATE;
  dom_retire(c);
  HIPC(c, hipStreamSynchronize(st));
  c->last_launches = D.launches;
  c->last_pass_ms = 0.0;
  c->last_timed = 0;
  if (c->profiling) {
    c->last_timed = D.prof_used / 2;
    for (size_t q = 0; q + 1 < D.prof_used; q += 2) {
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
    stats->launches = D.launches;
    stats->tile_visits = h[kStatVisits];
    stats->inner_sweeps = h[kStatSweeps];
    stats->max_active = h[kStatMaxActive];
    stats->deferred = h[kStatDeferred];
    stats->rounds = 0;
    stats->ms = ms;
    stats->tile_w = tile_w(D.variant);
    stats->tile_h = tile_h(D.variant);
    stats->kernel = D.variant;
  }
  return DYMU_OK;
}

// passes until no tile is queued, then statistics (the domain must be live).
// probe (priority kernels only): also stop as soon as the probe cells are final --
// every queued tile's key exceeds their largest value -- and return that value in
// *t_probe (+inf if a probe cell is unreachable; then the solve runs to the end).
int converge(dymu_ctx* c, hipStream_t st, dymu_stats* stats, const ProbeCells* probe = nullptr,
             double* t_probe = nullptr) {
  HIPC(c, hipEventRecord(c->ev0, st));
  uint64_t K = c->opts.passes_per_check > 0 ? (uint64_t)c->opts.passes_per_check : c->first_batch;
  for (;;) {
    int rc = dom_launch(c, K, st);
    if (rc == DYMU_OK && probe) {
      auto& D = c->dom;
      const hipError_t e = launch_probe(D.a.T, D.a.ld, *probe, prio_minkey(c, D.p % 3),
                                        c->d_scratch + 2, st);
      rc = e == hipSuccess ? DYMU_OK : fail_hip(c, e, "launch_probe");
      if (rc == DYMU_OK) {
        const hipError_t e2 = hipMemcpyAsync(c->h_probe, c->d_scratch + 2,
                                             2 * sizeof(unsigned long long),
                                             hipMemcpyDeviceToHost, st);
        if (e2 != hipSuccess) rc = fail_hip(c, e2, "probe read-back");
      }
    }
    if (rc == DYMU_OK) {
      uint64_t pending = 0;
      rc = dom_pending(c, st, &pending);
      if (rc == DYMU_OK && probe) {
        double tmax, kmin;
        std::memcpy(&tmax, &c->h_probe[0], sizeof tmax);
        std::memcpy(&kmin, &c->h_probe[1], sizeof kmin);
        *t_probe = tmax;
        if (kmin > tmax) break;  // no pass can lower a value <= tmax any more
      }
      if (rc == DYMU_OK && pending == 0) break;
    }
    if (rc == DYMU_OK && c->dom.p >= c->dom.max_passes) {
      c->last_error = "pass cap reached before convergence";
      rc = DYMU_ERR_NOT_CONVERGED;
    }
    if (rc) {
      dom_retire(c);
      return rc;
    }
    if (c->opts.passes_per_check <= 0) K = std::min<uint64_t>(K * 2, 64);
  }
  HIPC(c, hipEventRecord(c->ev1, st));
  HIPC(c, hipEventSynchronize(c->ev1));
  float ms = 0.f;
  HIPC(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  return dom_finish(c, st, stats, ms);
}

// Wait for the mailbox post seq (converge_pipelined, converge_stream).  The host spins on
// the coherent word; once a wait has lasted 20 ms (far beyond any batch) it asks
// every 5 ms whether the stream has drained, so a faulted or stopped stream ends
// the wait with an error instead of a hang.  (Not earlier: a query of a busy
// stream is not free.)
// Posts carry increasing sequence numbers; this returns the first one seen at or
// after seq (its number in *seen when seen is given).
int wait_mail(dymu_ctx* c, hipStream_t st, uint32_t seq, uint32_t* pending,
              uint32_t* seen = nullptr, double timeout_s = 0.0) {
  auto arrived = [&](unsigned long long v) {
    if ((int32_t)((uint32_t)(v >> 32) - seq) < 0) return false;
    *pending = (uint32_t)v;
    if (seen) *seen = (uint32_t)(v >> 32);
    return true;
  };
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = clk::now();
  clk::time_point next_query = t0 + std::chrono::milliseconds(20);
  for (uint64_t spin = 1;; ++spin) {
    if (arrived(__atomic_load_n(c->h_mail, __ATOMIC_ACQUIRE))) return DYMU_OK;
    if ((spin & 255) == 0 && clk::now() >= next_query) {
      next_query += std::chrono::milliseconds(5);
      if (timeout_s > 0.0 &&
          std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) {
        c->last_error = "convergence mailbox: timed out waiting for a post";
        return DYMU_ERR_HIP;
      }
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) {  // drained: the post, if made, is visible now
        if (arrived(__atomic_load_n(c->h_mail, __ATOMIC_ACQUIRE))) return DYMU_OK;
        c->last_error = "convergence mailbox: batch report missing";
        return DYMU_ERR_HIP;
      }
      if (e != hipErrorNotReady) return fail_hip(c, e, "hipStreamQuery");
    }
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
}

// converge() without host round trips between batches: batch b+1 is queued before
// the host learns batch b's outcome, which batch b+1's first pass posts to the
// mailbox as it starts -- the GPU never waits for the host, and the batch queued
// behind the converged one runs as empty passes (~3 us each).  Results are those of
// converge(): every pass after convergence finds no tile queued and changes nothing.
int converge_pipelined(dymu_ctx* c, hipStream_t st, dymu_stats* stats) {
  HIPC(c, hipEventRecord(c->ev0, st));
  auto& D = c->dom;
  uint64_t K = c->first_batch;
  int rc = dom_launch(c, K, st);
  while (rc == DYMU_OK) {
    const uint64_t done = D.p;  // passes whose outcome the next post reports
    K = std::min<uint64_t>(K * 2, c->max_batch);
    if (++c->mail_seq == 0) c->mail_seq = 1;
    const uint32_t seq = c->mail_seq;
    rc = dom_launch(c, K, st, seq);
    uint32_t pending = 0;
    if (rc == DYMU_OK) rc = wait_mail(c, st, seq, &pending);
    if (rc == DYMU_OK && pending == 0) break;
    if (rc == DYMU_OK && done >= D.max_passes) {
      c->last_error = "pass cap reached before convergence";
      rc = DYMU_ERR_NOT_CONVERGED;
    }
  }
  if (rc) {
    dom_retire(c);
    (void)hipStreamSynchronize(st);
    return rc;
  }
  HIPC(c, hipEventRecord(c->ev1, st));
  HIPC(c, hipEventSynchronize(c->ev1));
  float ms = 0.f;
  HIPC(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  return dom_finish(c, st, stats, ms);
}

// Streaming variant (DYMU_PIPELINE=2): every pass posts, and the host keeps
// c->max_batch passes queued ahead of the one running -- the overshoot after
// convergence is at most that many passes.
// probe (priority kernels): the passes also post whether the probe cells are final
// (PassArgs::probe); the loop stops at the first such post, and *t_probe gets their
// largest value (+inf if one is unreachable: then the solve runs to the end).  The
// <= 4 passes queued behind that post only lower values above *t_probe (every key
// exceeds it), so the cells <= *t_probe are exactly those of converge()'s exit.
int converge_stream(dymu_ctx* c, hipStream_t st, dymu_stats* stats,
                    const ProbeCells* probe = nullptr, double* t_probe = nullptr) {
  HIPC(c, hipEventRecord(c->ev0, st));
  auto& D = c->dom;
  if (probe) D.a.probe = *probe;
  const uint64_t ahead = c->max_batch;
  const uint32_t base = c->mail_seq + 1;  // pass p posts base + p
  auto post_seq = [&](uint64_t p) { uint32_t s = base + (uint32_t)p; return s ? s : 1u; };
  int rc = DYMU_OK;
  for (uint64_t k = 0; k < ahead && rc == DYMU_OK; ++k) rc = dom_launch(c, 1, st, post_seq(D.p));
  uint64_t running = 0;  // pass whose post the host waits for
  while (rc == DYMU_OK) {
    uint32_t pending = 0, seen = 0;
    rc = wait_mail(c, st, post_seq(running), &pending, &seen);
    if (rc) break;
    running = (uint64_t)(uint32_t)(seen - base);
    if ((pending & 0x7FFFFFFFu) == 0 || (pending & 0x80000000u)) break;
    if (running > D.max_passes) {
      c->last_error = "pass cap reached before convergence";
      rc = DYMU_ERR_NOT_CONVERGED;
      break;
    }
    while (rc == DYMU_OK && D.p < running + 1 + ahead) rc = dom_launch(c, 1, st, post_seq(D.p));
    ++running;
  }
  c->mail_seq = base + (uint32_t)D.p + 1;
  D.a.probe.n = 0;
  if (rc) {
    dom_retire(c);
    (void)hipStreamSynchronize(st);
    return rc;
  }
  HIPC(c, hipEventRecord(c->ev1, st));
  if (probe) {
    HIPC(c, launch_probe(D.a.T, D.a.ld, *probe, nullptr, c->d_scratch + 2, st));
    HIPC(c, hipMemcpyAsync(c->h_probe, c->d_scratch + 2, 2 * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st));
  }
  HIPC(c, hipEventSynchronize(c->ev1));
  HIPC(c, hipStreamSynchronize(st));
  if (probe) std::memcpy(t_probe, &c->h_probe[0], sizeof(double));
  float ms = 0.f;
  HIPC(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  return dom_finish(c, st, stats, ms);
}

int converge_auto(dymu_ctx* c, hipStream_t st, dymu_stats* stats) {
  if (c->pipeline == 2 && c->d_mail && c->opts.passes_per_check <= 0)
    return converge_stream(c, st, stats);
  if (c->pipeline && c->d_mail && c->opts.passes_per_check <= 0)
    return converge_pipelined(c, st, stats);
  return converge(c, st, stats);
}

int solve_core(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
               uint32_t gi, uint32_t gj, hipStream_t st, dymu_stats* stats) {
  if (gi >= nx || gj >= ny) return DYMU_ERR_ARG;
  int rc = dom_begin(c, dF, dT, nx, ny, ld, 0, 0, gi, gj, st);
  if (rc) return rc;
  return converge_auto(c, st, stats);
}

// The start cell and its in-grid 4-neighbours (isFullyClosedNode, :424-436).
ProbeCells start_probe(uint32_t nx, uint32_t ny, uint32_t si, uint32_t sj) {
  ProbeCells p{};
  auto add = [&](int64_t i, int64_t j) {
    if (i >= 0 && j >= 0 && i < (int64_t)nx && j < (int64_t)ny) {
      p.ij[p.n][0] = i;
      p.ij[p.n][1] = j;
      ++p.n;
    }
  };
  add(si, sj);
  add(si, (int64_t)sj - 1);
  add((int64_t)si - 1, sj);
  add((int64_t)si + 1, sj);
  add(si, (int64_t)sj + 1);
  return p;
}

int solve_until_core(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny,
                     uint64_t ld, uint32_t gi, uint32_t gj, uint32_t si, uint32_t sj,
                     hipStream_t st, double* t_closed, dymu_stats* stats) {
  if (gi >= nx || gj >= ny || si >= nx || sj >= ny || !t_closed) return DYMU_ERR_ARG;
  int rc = dom_begin(c, dF, dT, nx, ny, ld, 0, 0, gi, gj, st, true, /*need_keys=*/true);
  if (rc) return rc;
  const ProbeCells p = start_probe(nx, ny, si, sj);
  *t_closed = __builtin_inf();
  if (c->pipeline == 2 && c->d_mail && c->opts.passes_per_check <= 0)
    return converge_stream(c, st, stats, &p, t_closed);
  return converge(c, st, stats, &p, t_closed);
}

// Windowed re-propagation (update_kernels.hip): dT holds the converged map of
// the previous speed, dF the new speed, which differs only inside the window.
// decrease_only: the caller guarantees no speed in the window went up; then the
// old map is kept whole and only the window's tiles are seeded (k_seed_window).
// Otherwise (c->raise, default) the raise front invalidates the dependency cone of
// the window (k_raise passes) and the FIM re-solves the cone from
// its boundary plus the window when c->raise (DYMU_RAISE=1); by default every cell
// at or above theta is reset instead (k_reset_seed): a larger region, but one the
// FIM fills in key order from a single level set, where the cone is filled from
// its whole lateral boundary -- 4.1 ms / 192 K visits vs 9.5 ms (252 raise passes +
// 163 K visits) for config 5 at 4096^2.
int resolve_core(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
                 uint32_t gi, uint32_t gj, uint32_t i0, uint32_t j0, uint32_t w, uint32_t h,
                 hipStream_t st, dymu_stats* stats, bool decrease_only = false) {
  if (gi >= nx || gj >= ny || w == 0 || h == 0 || i0 >= nx || j0 >= ny) return DYMU_ERR_ARG;
  std::memset(c->last_update, 0, sizeof c->last_update);
  int rc = dom_begin(c, dF, dT, nx, ny, ld, 0, 0, -1, -1, st, /*cold=*/false);
  if (rc) return rc;
  auto& D = c->dom;
  // theta = min old T over the window plus its 1-cell ring (clipped)
  const uint32_t wi0 = i0 > 0 ? i0 - 1 : 0, wj0 = j0 > 0 ? j0 - 1 : 0;
  const uint32_t wi1 = (uint32_t)std::min<uint64_t>((uint64_t)i0 + w + 1, nx);
  const uint32_t wj1 = (uint32_t)std::min<uint64_t>((uint64_t)j0 + h + 1, ny);
  unsigned long long* theta = c->d_scratch;
  HIPC(c, launch_store_u64(theta, 0x7FF0000000000000ull, st));  // +inf bits
  HIPC(c, launch_window_min(dT, (int64_t)ld, wi0, wj0, wi1, wj1, theta, st));
  UpdateArgs u{};
  u.T = dT;
  u.F = dF;
  u.ld = (int64_t)ld;
  u.nx = nx;
  u.ny = ny;
  u.gi = gi;
  u.gj = gj;
  u.theta_bits = theta;
  u.shard_cap = D.ntiles;
  u.tile_epoch = c->d_tile_epoch;
  const bool raise = !decrease_only && c->raise;
  if (raise) {
    // the raise passes use the domain's lists and epochs (plain FIM lists, 16x16 tiles)
    const uint32_t ntx16 = (nx + 15) / 16, nty16 = (ny + 15) / 16;
    u.list = D.lists[0];
    u.counts = D.counts[0];
    u.epoch = D.eb + 1;
    u.tw = u.th = 16;
    u.ntx = ntx16;
    HIPC(c, launch_seed_window(u, i0, j0, i0 + w, j0 + h, st));  // no keys: u.keys null
    unsigned long long* rst = c->d_scratch + 5;  // [visits, cells]
    HIPC(c, hipMemsetAsync(rst, 0, 2 * sizeof(unsigned long long), st));
    RaiseArgs ra{};
    ra.T = dT;
    ra.F = dF;
    ra.ld = (int64_t)ld;
    ra.nx = nx;
    ra.ny = ny;
    ra.gi = gi;
    ra.gj = gj;
    ra.ntx = ntx16;
    ra.nty = nty16;
    ra.shard_cap = D.ntiles;
    ra.tile_epoch = c->d_tile_epoch;
    ra.tol = 1e-13;
    ra.stats = rst;
    const int blocks = c->cu_count * 2;
    uint64_t K = 4, raise_passes = 0;
    for (;;) {
      for (uint64_t k = 0; k < K; ++k, ++D.p) {
        const uint64_t p = D.p;
        if (p > D.max_passes) {
          c->last_error = "raise: pass cap reached";
          dom_retire(c);
          return DYMU_ERR_NOT_CONVERGED;
        }
        ra.list_in = D.lists[p % 3];
        ra.count_in = D.counts[p % 3];
        ra.list_out = D.lists[(p + 1) % 3];
        ra.count_out = D.counts[(p + 1) % 3];
        ra.count_clear = D.counts[(p + 2) % 3];
        ra.epoch = D.eb + (uint32_t)p + 2u;
        HIPC(c, launch_raise(ra, blocks, st));
        ++raise_passes;
      }
      uint64_t pending = 0;
      rc = dom_pending(c, st, &pending);
      if (rc) {
        dom_retire(c);
        return rc;
      }
      if (pending == 0) break;
      K = std::min<uint64_t>(K * 2, 64);
    }
    unsigned long long hr[2];
    HIPC(c, hipMemcpy(hr, rst, sizeof hr, hipMemcpyDeviceToHost));
    c->last_update[0] = raise_passes;
    c->last_update[1] = hr[0];
    c->last_update[2] = hr[1];
    // a fresh domain for the re-solve: epochs above every raise epoch (dom_retire)
    rc = dom_begin(c, dF, dT, nx, ny, ld, 0, 0, -1, -1, st, /*cold=*/false);
    if (rc) return rc;
    u.shard_cap = D.ntiles;
  }
  u.list = D.lists[0];
  u.counts = D.counts[0];
  u.epoch = D.eb + 1;  // the epoch of list 0 (dom_launch: eb + p + 2 for list p + 1)
  u.tw = (uint32_t)tile_w(D.variant);
  u.th = (uint32_t)tile_h(D.variant);
  u.ntx = (uint32_t)D.a.ntx;
  if (is_prio(D.variant)) {
    u.keys = prio_keys(c, 0);
    u.hist = prio_hist(c, 0);
  }
  if (raise) {  // the cone's boundary, then the window (decreases inside it)
    uint32_t* hist0 = u.hist;
    u.hist = nullptr;  // binned below from the final keys (they differ per tile)
    HIPC(c, launch_cone_seed(u, theta, st));
    HIPC(c, launch_seed_window(u, i0, j0, i0 + w, j0 + h, st));
    if (is_prio(D.variant)) {
      HIPC(c, launch_theta_state(theta, prio_minkey(c, 0), prio_base(c, 0), st));
      // list 0's histogram from its keys (origin theta', the smallest boundary value):
      // the first passes then relax the boundary tiles in key order, not all at once
      HIPC(c, launch_rehist(D.lists[0], D.counts[0], D.ntiles, prio_keys(c, 0), prio_base(c, 0),
                            prio_delta(c), hist0, c->d_hist + (uint64_t)4 * kShards * kBins, st));
    }
    if (D.a.ec)
      HIPC(c, launch_ec_rebuild(dT, ld, nx, ny, D.a.ec, (uint32_t)D.a.ntx, 0, D.ntiles, st));
    return converge_auto(c, st, stats);
  } else if (decrease_only) {
    HIPC(c, launch_seed_window(u, i0, j0, i0 + w, j0 + h, st));
  } else {
    HIPC(c, launch_reset_seed(u, st));
  }
  if (is_prio(D.variant))
    HIPC(c, launch_theta_state(theta, prio_minkey(c, 0), prio_base(c, 0), st));
  if (D.a.ec)  // the reset kernel wrote T
    HIPC(c, launch_ec_rebuild(dT, ld, nx, ny, D.a.ec, (uint32_t)D.a.ntx, 0, D.ntiles, st));
  return converge_auto(c, st, stats);
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

void* dymu_get_stream(dymu_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

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
  if (const char* kv = std::getenv("DYMU_MAP_MEM")) c->map_mem = std::atoi(kv);
  if (const char* kv = std::getenv("DYMU_WS_MEM")) c->ws_mem = c->ec_mem = c->key_mem = std::atoi(kv);
  if (const char* kv = std::getenv("DYMU_EC_MEM")) c->ec_mem = std::atoi(kv);
  if (const char* kv = std::getenv("DYMU_KEY_MEM")) c->key_mem = std::atoi(kv);
  if (const char* kv = std::getenv("DYMU_FIRST_BATCH"))
    c->first_batch = (uint64_t)std::max(1, std::atoi(kv));
  if (const char* kv = std::getenv("DYMU_PIPELINE")) c->pipeline = std::atoi(kv);
  if (const char* kv = std::getenv("DYMU_DETERMINISTIC")) c->opts.deterministic = std::atoi(kv);
  if (const char* kv = std::getenv("DYMU_MAX_BATCH"))
    c->max_batch = (uint64_t)std::min(64, std::max(1, std::atoi(kv)));
  if (e == hipSuccess) {
    for (int v = 3; v <= 5; ++v) c->occupancy[v] = pass_blocks_per_cu(v);
  }
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (!valid_variant(c->opts.kernel) || c->opts.prio_target < 0) {
    dymu_destroy(c);
    return DYMU_ERR_ARG;
  }
  c->variant = c->opts.kernel;
  if (const char* kv = std::getenv("DYMU_KERNEL")) {  // development override
    const int v = std::atoi(kv);
    c->variant = valid_variant(v) ? v : 0;
  }
  if (e == hipSuccess) {
    c->prio_target = (uint32_t)c->opts.prio_target;
    if (const char* kv = std::getenv("DYMU_PRIO_TARGET")) c->prio_target = (uint32_t)std::atol(kv);
    if (const char* kv = std::getenv("DYMU_PRIO_KAPPA")) c->prio_kappa = std::atof(kv);
    if (!(c->prio_kappa > 0.0)) c->prio_kappa = 0.5;
    if (const char* kv = std::getenv("DYMU_GRID_BLOCKS")) c->opts.grid_blocks = std::atoi(kv);
    if (const char* kv = std::getenv("DYMU_PRIO_MIN_TILES"))
      c->prio_min_tiles = (uint32_t)std::atol(kv);
    if (const char* kv = std::getenv("DYMU_PRIO_FRAC")) c->prio_frac = (float)std::atof(kv);
    if (const char* kv = std::getenv("DYMU_PRIO_TRACE")) c->prio_trace = std::atoi(kv);
    if (const char* kv = std::getenv("DYMU_PRUNE")) c->prune = std::atoi(kv);
    if (const char* kv = std::getenv("DYMU_PRIO_DEBUG")) c->prio_debug = std::atoi(kv);
    if (const char* kv = std::getenv("DYMU_RAISE")) c->raise = std::atoi(kv);
  }
  if (e == hipSuccess) e = hipMalloc(&c->d_counts, sizeof(uint32_t) * 4 * kShards);
  if (e == hipSuccess) e = hipMalloc(&c->d_scratch, sizeof(unsigned long long) * 8);
  if (e == hipSuccess) e = hipMalloc(&c->d_xchg, sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(c->d_xchg, 0, sizeof(uint32_t));
  if (e == hipSuccess)
    e = hipMalloc(&c->d_stats, sizeof(unsigned long long) * kShards * kStatSlots);
  if (e == hipSuccess) e = hipHostMalloc(&c->h_count, sizeof(uint32_t) * 4 * kShards, hipHostMallocDefault);
  if (e == hipSuccess)
    e = hipHostMalloc(&c->h_probe, sizeof(unsigned long long) * 2, hipHostMallocDefault);
  if (e == hipSuccess && c->pipeline) {  // without a mailbox: synchronous checks
    if (hipHostMalloc(&c->h_mail, 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess) {
      *c->h_mail = 0ull;
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, c->h_mail, 0) == hipSuccess)
        c->d_mail = static_cast<unsigned long long*>(d);
    }
    (void)hipGetLastError();
  }
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
  if (c->d_keys) (void)hipFree(c->d_keys);
  if (c->d_hist) (void)hipFree(c->d_hist);
  if (c->d_prio) (void)hipFree(c->d_prio);
  if (c->d_trace) (void)hipFree(c->d_trace);
  if (c->d_pstat) (void)hipFree(c->d_pstat);
  if (c->d_ec) (void)hipFree(c->d_ec);
  if (c->d_lut) (void)hipFree(c->d_lut);
  if (c->d_scratch) (void)hipFree(c->d_scratch);
  if (c->d_xchg) (void)hipFree(c->d_xchg);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->d_F) (void)hipFree(c->d_F);
  if (c->d_T) (void)hipFree(c->d_T);
  if (c->h_count) (void)hipHostFree(c->h_count);
  if (c->h_probe) (void)hipHostFree(c->h_probe);
  if (c->h_mail) (void)hipHostFree(c->h_mail);
  if (c->d_band) (void)hipFree(c->d_band);
  if (c->h_xfer) (void)hipHostFree(c->h_xfer);
  if (c->d_region) (void)hipFree(c->d_region);
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
  c->host_valid = false;
  HIPC(c, hipMemcpyAsync(c->d_F, F, sizeof(double) * cells, hipMemcpyHostToDevice, c->stream));
  rc = solve_core(c, c->d_F, c->d_T, nx, ny, nx, gi, gj, c->stream, stats);
  if (rc) return rc;
  HIPC(c, hipMemcpyAsync(T_out, c->d_T, sizeof(double) * cells, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  c->host_valid = true;
  c->host_nx = nx;
  c->host_ny = ny;
  c->host_gi = gi;
  c->host_gj = gj;
  return DYMU_OK;
}

int dymu_solve_until_device(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny,
                            uint64_t ld, uint32_t gi, uint32_t gj, uint32_t si, uint32_t sj,
                            void* stream, double* t_closed, dymu_stats* stats) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return solve_until_core(c, dF, dT, nx, ny, ld, gi, gj, si, sj, pick_stream(c, stream), t_closed,
                          stats);
}

int dymu_early_exit_mask(dymu_ctx* c, const double* dF, double* dT, uint32_t nx, uint32_t ny,
                         uint64_t ld, double t_closed, uint64_t* band_idx, uint64_t cap,
                         uint64_t* n_band, void* stream) {
  if (!c || !dF || !dT || !n_band || nx == 0 || ny == 0 || ld < nx || (cap && !band_idx))
    return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, stream);
  if (cap > c->band_cap) {
    if (c->d_band) HIPC(c, hipFree(c->d_band));
    c->d_band = nullptr;
    c->band_cap = 0;
    HIPC(c, hipMalloc(&c->d_band, sizeof(uint64_t) * cap));
    c->band_cap = cap;
  }
  unsigned long long* cnt = c->d_scratch + 4;
  HIPC(c, hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
  HIPC(c, launch_early_mask(dF, dT, (int64_t)ld, nx, ny, t_closed, c->d_band, cnt, cap, st));
  HIPC(c, hipMemcpyAsync(c->h_probe, cnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPC(c, hipStreamSynchronize(st));
  *n_band = c->h_probe[0];
  const uint64_t m = std::min<uint64_t>(*n_band, cap);
  if (m) HIPC(c, hipMemcpy(band_idx, c->d_band, sizeof(uint64_t) * m, hipMemcpyDeviceToHost));
  return DYMU_OK;
}

int dymu_count_equal(dymu_ctx* c, const double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
                     double value, uint64_t* count, void* stream) {
  if (!c || !dT || !count || ld < nx) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, stream);
  unsigned long long* cnt = c->d_scratch + 4;
  HIPC(c, hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
  HIPC(c, launch_count_equal(dT, (int64_t)ld, nx, ny, value, cnt, nullptr, 0, st));
  HIPC(c, hipMemcpyAsync(c->h_probe, cnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPC(c, hipStreamSynchronize(st));
  *count = c->h_probe[0];
  return DYMU_OK;
}

int dymu_find_equal(dymu_ctx* c, const double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
                    double value, uint64_t* idx, uint64_t cap, uint64_t* count, void* stream) {
  if (!c || !dT || !count || ld < nx || (cap && !idx)) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, stream);
  HIPC(c, hipStreamSynchronize(st));  // no earlier kernel still uses the transfer buffer
  int rc = ensure_xfer(c, sizeof(uint64_t) * (cap ? cap : 1));
  if (rc) return rc;
  uint64_t* di = static_cast<uint64_t*>(c->d_xfer);  // written by the kernel in host memory
  unsigned long long* cnt = c->d_scratch + 4;
  HIPC(c, hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st));
  HIPC(c, launch_count_equal(dT, (int64_t)ld, nx, ny, value, cnt, di, cap, st));
  HIPC(c, hipMemcpyAsync(c->h_probe, cnt, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPC(c, hipStreamSynchronize(st));
  *count = c->h_probe[0];
  const uint64_t m = std::min<uint64_t>(*count, cap);
  if (m) std::memcpy(idx, c->h_xfer, sizeof(uint64_t) * m);
  return DYMU_OK;
}

int dymu_region_stats(dymu_ctx* c, const double* dF, const double* dT, uint32_t nx, uint32_t ny,
                      uint64_t ld, uint32_t gi, uint32_t gj, double thr, double lo, double hi,
                      dymu_region* out, void* stream) {
  if (!c || !dF || !dT || !out || nx == 0 || ny == 0 || ld < nx || gi >= nx || gj >= ny)
    return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, stream);
  HIPC(c, hipStreamSynchronize(st));  // no earlier kernel still uses the transfer buffer
  int rc = ensure_xfer(c, sizeof(unsigned long long) * 8);
  if (rc) return rc;
  if (!c->d_region) HIPC(c, hipMalloc(&c->d_region, sizeof(unsigned long long) * 8));
  // atomics on device words (initialised by memsets), read back into pinned memory
  unsigned long long* d = c->d_region;
  auto* h = static_cast<unsigned long long*>(c->h_xfer);
  HIPC(c, hipMemsetAsync(d, 0xFF, 2 * sizeof(unsigned long long), st));  // min i, min j
  HIPC(c, hipMemsetAsync(d + 2, 0, 3 * sizeof(unsigned long long), st));  // max i, max j, count
  HIPC(c, hipMemsetAsync(d + 5, 0xFF, sizeof(unsigned long long), st));   // min distance^2
  double f0 = 0.0;  // the goal's speed
  HIPC(c, hipMemcpyAsync(h + 7, dF + (uint64_t)gj * ld + gi, sizeof(double), hipMemcpyDeviceToHost,
                         st));
  HIPC(c, launch_region_box(dT, (int64_t)ld, nx, ny, thr, lo, hi, d, st));
  HIPC(c, hipStreamSynchronize(st));
  std::memcpy(&f0, &h[7], sizeof f0);
  HIPC(c, launch_const_radius(dF, (int64_t)ld, nx, ny, gi, gj, f0, d + 5, st));
  HIPC(c, hipMemcpyAsync(h, d, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  HIPC(c, hipStreamSynchronize(st));
  std::memset(out, 0, sizeof *out);
  out->n_range = h[4];
  out->r_const = h[5] == ~0ull ? __builtin_inf() : std::sqrt((double)h[5]);
  if (h[0] > h[2]) {  // no cell at or below thr
    out->i0 = 1;
    out->i1 = 0;
    return DYMU_OK;
  }
  out->i0 = (uint32_t)h[0];
  out->j0 = (uint32_t)h[1];
  out->i1 = (uint32_t)h[2];
  out->j1 = (uint32_t)h[3];
  return DYMU_OK;
}

int dymu_scatter(dymu_ctx* c, double* dT, uint32_t nx, uint64_t ld, const uint64_t* idx,
                 const double* vals, uint64_t n, void* stream) {
  if (!c || !dT || nx == 0 || ld < nx || (n && (!idx || !vals))) return DYMU_ERR_ARG;
  if (n == 0) return DYMU_OK;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t st = pick_stream(c, stream);
  // indices and values written into the pinned transfer buffer on the host and read
  // there by the kernel (ensure_xfer): no copy command, no device staging
  HIPC(c, hipStreamSynchronize(st));  // no earlier kernel still uses the transfer buffer
  int rc = ensure_xfer(c, (sizeof(uint64_t) + sizeof(double)) * n);
  if (rc) return rc;
  std::memcpy(c->h_xfer, idx, sizeof(uint64_t) * n);
  std::memcpy(static_cast<char*>(c->h_xfer) + sizeof(uint64_t) * n, vals, sizeof(double) * n);
  const uint64_t* di = static_cast<const uint64_t*>(c->d_xfer);
  const double* dv = reinterpret_cast<const double*>(di + n);
  HIPC(c, launch_scatter(dT, (int64_t)ld, nx, di, dv, n, st));
  HIPC(c, hipStreamSynchronize(st));
  return DYMU_OK;
}

int dymu_memcpy2d_d2h(dymu_ctx* c, void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width, size_t height) {
  if (!c || !dst || !src) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToHost,
                           c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return DYMU_OK;
}

int dymu_memcpy2d_h2d(dymu_ctx* c, void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width, size_t height) {
  if (!c || !dst || !src) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyHostToDevice,
                           c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return DYMU_OK;
}

int dymu_host_register(dymu_ctx* c, void* p, size_t bytes) {
  if (!c || !p || bytes == 0) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipHostRegister(p, bytes, hipHostRegisterDefault));
  return DYMU_OK;
}

int dymu_host_unregister(dymu_ctx* c, void* p) {
  if (!c || !p) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipHostUnregister(p));
  return DYMU_OK;
}

int dymu_resolve_window_device(dymu_ctx* c, const double* dF, double* dT, uint32_t nx,
                               uint32_t ny, uint64_t ld, uint32_t gi, uint32_t gj, uint32_t i0,
                               uint32_t j0, uint32_t w, uint32_t h, void* stream,
                               dymu_stats* stats) {
  if (!c || !dF || !dT || nx == 0 || ny == 0 || ld < nx) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  w = (uint32_t)std::min<uint64_t>(w, nx > i0 ? nx - i0 : 0);
  h = (uint32_t)std::min<uint64_t>(h, ny > j0 ? ny - j0 : 0);
  return resolve_core(c, dF, dT, nx, ny, ld, gi, gj, i0, j0, w, h, pick_stream(c, stream), stats);
}

int dymu_update_window_device(dymu_ctx* c, const double* dF, double* dT, uint32_t nx,
                              uint32_t ny, uint64_t ld, uint32_t gi, uint32_t gj, uint32_t i0,
                              uint32_t j0, uint32_t w, uint32_t h, int decrease_only, void* stream,
                              dymu_stats* stats) {
  if (!c || !dF || !dT || nx == 0 || ny == 0 || ld < nx) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  w = (uint32_t)std::min<uint64_t>(w, nx > i0 ? nx - i0 : 0);
  h = (uint32_t)std::min<uint64_t>(h, ny > j0 ? ny - j0 : 0);
  return resolve_core(c, dF, dT, nx, ny, ld, gi, gj, i0, j0, w, h, pick_stream(c, stream), stats,
                      decrease_only != 0);
}

int dymu_resolve_window(dymu_ctx* c, const double* F, uint32_t nx, uint32_t ny, uint32_t gi,
                        uint32_t gj, uint32_t i0, uint32_t j0, uint32_t w, uint32_t h,
                        double* T_out, dymu_stats* stats) {
  if (!c || !F || !T_out || nx == 0 || ny == 0) return DYMU_ERR_ARG;
  if (!c->host_valid || c->host_nx != nx || c->host_ny != ny || c->host_gi != gi ||
      c->host_gj != gj) {
    c->last_error = "dymu_resolve_window: no previous dymu_solve of this grid and goal";
    return DYMU_ERR_STATE;
  }
  if (i0 >= nx || j0 >= ny || w == 0 || h == 0) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  w = (uint32_t)std::min<uint64_t>(w, nx - i0);
  h = (uint32_t)std::min<uint64_t>(h, ny - j0);
  c->host_valid = false;
  // only the window of F changed: upload those rows' columns
  const uint64_t off = (uint64_t)j0 * nx + i0;
  HIPC(c, hipMemcpy2DAsync(c->d_F + off, sizeof(double) * nx, F + off, sizeof(double) * nx,
                           sizeof(double) * w, h, hipMemcpyHostToDevice, c->stream));
  int rc = resolve_core(c, c->d_F, c->d_T, nx, ny, nx, gi, gj, i0, j0, w, h, c->stream, stats);
  if (rc) return rc;
  const uint64_t cells = (uint64_t)nx * ny;
  HIPC(c, hipMemcpyAsync(T_out, c->d_T, sizeof(double) * cells, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  c->host_valid = true;
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
  HIPC(c, dev_alloc(p, bytes, c->map_mem));
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
  // ordered after the work queued on the context stream, complete on return
  HIPC(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return DYMU_OK;
}

int dymu_memcpy_h2d(dymu_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return DYMU_OK;
}

int dymu_dom_begin(dymu_ctx* c, const dymu_domain* d, int64_t goal_i, int64_t goal_j_local,
                   void* stream) {
  if (!c || !d) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_begin(c, d->F, d->T, d->nx, d->nrows, d->ld, d->ghost_lo, d->ghost_hi, goal_i,
                   goal_j_local, pick_stream(c, stream));
}

int dymu_dom_run(dymu_ctx* c, uint32_t passes, void* stream) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_launch(c, passes, pick_stream(c, stream));
}

int dymu_dom_merge_ghosts(dymu_ctx* c, const double* new_lo, const double* new_hi,
                          int32_t* d_pending, void* stream) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_merge(c, new_lo, new_hi, d_pending, pick_stream(c, stream));
}

int dymu_dom_exchange(dymu_ctx* c, const double* new_lo, const double* new_hi,
                      int32_t* d_total, void* stream) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_exchange(c, new_lo, new_hi, d_total, pick_stream(c, stream));
}

int dymu_dom_round_supported(dymu_ctx* c, uint32_t passes) {
  return c && dom_round_ok(c, passes) ? 1 : 0;
}

int dymu_dom_round_capable(dymu_ctx* c, uint32_t nx, uint32_t nrows, uint32_t passes) {
  if (!c || nx == 0 || nrows == 0) return 0;
  return dom_variant(c, nx, nrows, false) == 5 && passes >= 2 && !c->opts.deterministic ? 1 : 0;
}

int dymu_dom_round(dymu_ctx* c, uint32_t passes, const double* new_lo, const double* new_hi,
                   int32_t* d_total, void* stream) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_round(c, passes, new_lo, new_hi, d_total, pick_stream(c, stream));
}

int dymu_dom_round_peer(dymu_ctx* c, uint32_t passes, const dymu_peer_links* links,
                        void* stream) {
  if (!c || !links) return DYMU_ERR_ARG;
  static_assert(sizeof(PeerCtl) <= DYMU_PEER_CTL_BYTES, "peer control block");
  HIPC(c, hipSetDevice(c->device));
  return dom_round_peer(c, passes, *links, pick_stream(c, stream));
}

int dymu_dom_post_status(dymu_ctx* c, const void* ctl, unsigned long long* dst, uint32_t seq) {
  if (!c || !ctl || !dst || seq == 0) return DYMU_ERR_ARG;
  if (!c->dom.live) return DYMU_ERR_STATE;
  const PeerCtl* pc = static_cast<const PeerCtl*>(ctl);
  c->arm_src = reinterpret_cast<const int32_t*>(&pc->pend);
  c->arm_ext = pc->ext;
  c->arm_dst = dst;
  c->arm_seq = seq;
  return DYMU_OK;
}

int dymu_dom_post(dymu_ctx* c, const int32_t* d_src, uint32_t* seq) {
  if (!c || !d_src || !seq) return DYMU_ERR_ARG;
  if (!c->d_mail || !c->dom.live) return DYMU_ERR_STATE;
  if (++c->mail_seq == 0) c->mail_seq = 1;
  c->arm_dst = nullptr;
  c->arm_ext = nullptr;
  c->arm_src = d_src;
  c->arm_seq = c->mail_seq;
  *seq = c->mail_seq;
  return DYMU_OK;
}

int dymu_dom_wait_post(dymu_ctx* c, uint32_t seq, double timeout_s, int32_t* value,
                       void* stream) {
  if (!c || !value || seq == 0) return DYMU_ERR_ARG;
  if (!c->d_mail) return DYMU_ERR_STATE;
  uint32_t v = 0;
  const int rc = wait_mail(c, pick_stream(c, stream), seq, &v, nullptr, timeout_s);
  if (rc) return rc;
  *value = (int32_t)v;
  return DYMU_OK;
}

int dymu_dom_pending(dymu_ctx* c, void* stream, uint64_t* pending) {
  if (!c || !pending) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_pending(c, pick_stream(c, stream), pending);
}

int dymu_dom_finish(dymu_ctx* c, void* stream, dymu_stats* stats) {
  if (!c) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  return dom_finish(c, pick_stream(c, stream), stats, 0.0);
}

int dymu_slab_rows(uint32_t ny, uint32_t nranks, uint32_t rank, uint32_t* row0, uint32_t* nrows) {
  if (!row0 || !nrows || nranks == 0 || rank >= nranks) return DYMU_ERR_ARG;
  // slab boundaries on multiples of 32 rows (a whole number of tile rows for
  // every kernel variant), so every slab but the last satisfies ghost_hi.
  const uint32_t A = 32;
  const uint64_t blocks = ((uint64_t)ny + A - 1) / A;
  const uint64_t b0 = blocks * rank / nranks, b1 = blocks * (rank + 1) / nranks;
  uint64_t r0 = b0 * A, r1 = b1 * A;
  if (r1 > ny) r1 = ny;
  if (r0 > ny) r0 = ny;
  *row0 = (uint32_t)r0;
  *nrows = (uint32_t)(r1 - r0);
  return DYMU_OK;
}

int dymu_eikonal_batch(dymu_ctx* c, const double* tx, const double* ty, const double* cc,
                       double* out, uint64_t n, int fast) {
  if (!c || !tx || !ty || !cc || !out) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  HIPC(c, launch_eikonal_batch(tx, ty, cc, out, n, fast, c->stream));
  HIPC(c, hipStreamSynchronize(c->stream));
  return DYMU_OK;
}

namespace {
dymu::CostState cost_state(const dymu_cost_state* s) {
  return dymu::CostState{s->cost,        s->raw_cost, s->slope, s->terrain,
                         s->is_obstacle, s->hazard,   s->traff, s->loc_mode};
}
bool cost_state_ok(const dymu_cost_state* s) {
  return s && s->cost && s->raw_cost && s->slope && s->terrain && s->is_obstacle && s->hazard &&
         s->traff && s->loc_mode;
}
}  // namespace

int dymu_compute_cost_map(dymu_ctx* c, uint32_t nx, uint32_t ny, uint64_t ld, double global_res,
                          const double* lut, int lut_len, const double* slopes, int n_slopes,
                          int n_locs, const double* elevation, const double* terrain_map,
                          const dymu_cost_state* st, double* dF, void* stream) {
  if (!c || !lut || lut_len <= 0 || !slopes || n_slopes <= 0 || n_locs <= 0 || !elevation ||
      !terrain_map || !cost_state_ok(st) || nx < 2 || ny < 2 || ld < nx || !(global_res > 0))
    return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  hipStream_t s = pick_stream(c, stream);
  if ((size_t)lut_len > c->lut_cap) {
    if (c->d_lut) HIPC(c, hipFree(c->d_lut));
    c->d_lut = nullptr;
    c->lut_cap = 0;
    HIPC(c, hipMalloc(&c->d_lut, sizeof(double) * (size_t)lut_len));
    c->lut_cap = (size_t)lut_len;
  }
  // the previous launch reading d_lut must be done before it is overwritten
  HIPC(c, hipStreamSynchronize(s));
  HIPC(c, hipMemcpy(c->d_lut, lut, sizeof(double) * (size_t)lut_len, hipMemcpyHostToDevice));
  dymu::CostArgs a{};
  a.nx = nx;
  a.ny = ny;
  a.ld = (int64_t)ld;
  a.res = global_res;
  a.cmax = lut[0];  // std::max_element (:221)
  for (int k = 1; k < lut_len; ++k)
    if (a.cmax < lut[k]) a.cmax = lut[k];
  a.slope_lo = slopes[0];
  a.slope_hi = slopes[n_slopes - 1];
  a.n_slopes = n_slopes;
  a.n_locs = n_locs;
  a.lut_len = lut_len;
  a.lut = c->d_lut;
  a.elevation = elevation;
  a.terrain_map = terrain_map;
  a.st = cost_state(st);
  a.F = dF;
  HIPC(c, dymu::launch_cost_map(a, s));
  return DYMU_OK;
}

int dymu_pack_speed(dymu_ctx* c, uint32_t nx, uint32_t ny, uint64_t ld, double global_res,
                    const dymu_cost_state* st, double* dF, void* stream) {
  if (!c || !cost_state_ok(st) || !dF || nx == 0 || ny == 0 || ld < nx) return DYMU_ERR_ARG;
  HIPC(c, hipSetDevice(c->device));
  dymu::CostArgs a{};
  a.nx = nx;
  a.ny = ny;
  a.ld = (int64_t)ld;
  a.res = global_res;
  a.st = cost_state(st);
  a.F = dF;
  HIPC(c, dymu::launch_pack_speed(a, pick_stream(c, stream)));
  return DYMU_OK;
}

int dymu_last_update_stats(dymu_ctx* c, uint64_t out[4]) {
  if (!c || !out) return DYMU_ERR_ARG;
  std::memcpy(out, c->last_update, sizeof c->last_update);
  return DYMU_OK;
}

int dymu_set_pass_stats(dymu_ctx* c, int enable) {
  if (!c) return DYMU_ERR_ARG;
  c->pass_stats = enable != 0;
  return DYMU_OK;
}

int dymu_last_pass_stats(dymu_ctx* c, uint32_t* out, uint64_t cap, uint64_t* n) {
  if (!c || !n || (cap && !out)) return DYMU_ERR_ARG;
  *n = 0;
  if (!c->d_pstat || !c->pass_stats) return DYMU_ERR_STATE;
  HIPC(c, hipSetDevice(c->device));
  const uint64_t passes = std::min<uint64_t>(c->last_launches, kPassStatCap);
  *n = passes;
  const uint64_t m = std::min(passes, cap);
  if (!m) return DYMU_OK;
  std::vector<uint32_t> h((size_t)m * kShards * kPsWords);
  HIPC(c, hipMemcpy(h.data(), c->d_pstat, sizeof(uint32_t) * h.size(), hipMemcpyDeviceToHost));
  for (uint64_t p = 0; p < m; ++p) {
    uint32_t* o = out + p * kPsWords;
    std::memset(o, 0, sizeof(uint32_t) * kPsWords);
    for (int q = 0; q < kShards; ++q) {
      const uint32_t* r = &h[(p * kShards + q) * kPsWords];
      for (int w = 0; w < kPsWords; ++w) {
        if (w == kPsRadiusMax || w == kPsRadiusMin) o[w] = std::max(o[w], r[w]);
        else o[w] += r[w];
      }
    }
    o[kPsRadiusMin] = o[kPsRadiusMin] ? ~o[kPsRadiusMin] : 0u;  // stored as ~radius
  }
  return DYMU_OK;
}

int dymu_set_profiling(dymu_ctx* c, int period) {
  if (!c || period < 0) return DYMU_ERR_ARG;
  c->profiling = period;
  return DYMU_OK;
}

int dymu_last_pass_timing(dymu_ctx* c, double* ms, uint64_t* n) {
  if (!c) return DYMU_ERR_ARG;
  if (ms) *ms = c->last_pass_ms;
  if (n) *n = c->last_timed;
  return DYMU_OK;
}

}  // extern "C"
