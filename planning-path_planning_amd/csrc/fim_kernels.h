// fim_kernels.h -- internal interface between the HIP kernels and the
// C-ABI runtime (dymu_fim.cpp).  Not installed; not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dymu {

constexpr int kTileW = 32;  // tile width  (x, columns)
constexpr int kTileH = 32;  // tile height (y, rows)

enum StatSlot : int {
  kStatPasses = 0,
  kStatVisits = 1,
  kStatSweeps = 2,
  kStatMaxActive = 3,
  kStatSlots = 8
};

struct PassArgs {
  const double* F;  // speed, pitch ld
  double* T;        // total cost, pitch ld (row -1 / row ny are ghost rows when flagged)
  int64_t ld;
  int64_t nx, ny;   // local domain
  int ntx, nty;     // tiles
  int ghost_lo;     // row -1 exists in memory (read-only halo)
  int ghost_hi;     // row ny exists in memory (requires ny % kTileH == 0)
  int max_inner;    // cap on in-tile sweeps per visit
  uint32_t epoch;   // epoch stamped on tiles enqueued for the NEXT pass
  const uint32_t* list_in;
  const uint32_t* count_in;
  uint32_t* list_out;
  uint32_t* count_out;
  uint32_t* count_clear;
  uint32_t* tile_epoch;
  unsigned long long* stats;
};

hipError_t launch_fill_inf(double* T, uint64_t ld, uint32_t nx, int64_t row_lo, int64_t row_hi,
                           hipStream_t st);
hipError_t launch_seed(double* T, uint64_t ld, int64_t gi, int64_t gj, uint32_t* list,
                       uint32_t* count, uint32_t* tile_epoch, uint32_t epoch, uint32_t tile,
                       int set_goal, hipStream_t st);
hipError_t launch_pass(const PassArgs& a, int blocks, hipStream_t st);
hipError_t launch_synth(double* F, uint64_t ld, uint32_t nx, uint32_t ny, uint64_t row0,
                        uint64_t seed, double frac, uint64_t oseed, int64_t gi, int64_t gj,
                        hipStream_t st);

}  // namespace dymu
