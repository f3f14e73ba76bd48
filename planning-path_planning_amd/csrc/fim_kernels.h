// fim_kernels.h -- internal interface between the HIP kernels and the
// C-ABI runtime (dymu_fim.cpp).  Not installed; not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dymu {

constexpr int kWaveTile = 8;  // kernels 3/4: 8x8 tiles, two per 64-lane wave (half-wave each)
constexpr int kShards = 16;   // active lists are split in shards to spread the append atomics

enum StatSlot : int {
  kStatPasses = 0,
  kStatVisits = 1,
  kStatSweeps = 2,
  kStatMaxActive = 3,
  kStatDeferred = 4,
  kStatSlots = 8
};

struct ProbeCells {
  int64_t ij[5][2];  // (i, j) of the start cell and its in-grid 4-neighbours
  int n;
};

// Counters of the peer rounds (dymu_dom_round_peer, DESIGN.md s5 "Peer transport"),
// in the rank's own device memory, zeroed at the start of a solve (rmin: all ones).
// side 0 = the link to rank-1, side 1 = the link to rank+1.
struct PeerCtl {
  uint32_t done[2];               // workgroups that finished this pass's push of a side
  uint32_t changed[2];            // some pushed column of the side decreased this pass
  unsigned long long sent[2];     // S: pushes that carried a decrease (= the tags written)
  unsigned long long rmin[2];     // smallest tag a merging workgroup read this round
  unsigned long long merged[2];   // R: the tag of the last complete merge (status pass)
  uint32_t pend;                  // P: tiles queued for the round's first + second pass
  uint32_t pad;
  unsigned long long ext[4];      // the posted status: S0, S1, R0, R1 (with pend)
};

struct PassArgs {
  const double* F;  // speed, pitch ld
  double* T;        // total cost, pitch ld (row -1 / row ny are ghost rows when flagged)
  int64_t ld;
  int64_t nx, ny;   // local domain
  int ntx, nty;     // tiles
  int ghost_lo;     // row -1 exists in memory (read-only halo)
  int ghost_hi;     // row ny exists in memory (requires ny % tile height == 0)
  int max_inner;    // cap on in-tile sweeps per visit
  uint32_t epoch;   // epoch stamped on tiles enqueued for the NEXT pass
  uint32_t shard_cap;  // capacity of one shard (= number of tiles)
  const uint32_t* list_in;   // kShards shards of shard_cap entries
  const uint32_t* count_in;  // kShards counters
  uint32_t* list_out;
  uint32_t* count_out;
  uint32_t* count_clear;
  uint32_t* tile_epoch;
  unsigned long long* stats;  // kShards x kStatSlots
  // ---- v4 (priority passes) only ----
  unsigned long long* key_in;   // per-tile key of list p (double bits), reset to +inf by its reader
  unsigned long long* key_out;  // keys of list p+1 (atomicMin)
  const uint32_t* hist_in;      // kShards x kBins key histogram of list p
  uint32_t* hist_out;           // ... of list p+1
  uint32_t* hist_clear;         // ... of list p+2 (zeroed by block 0)
  const unsigned long long* minkey_in;  // min key of list p
  unsigned long long* minkey_out;
  unsigned long long* minkey_clear;
  const double* base_in;  // histogram origin of list p
  double* base_out;       // ... of list p+1 (= min key of list p, written by block 0)
  const double* delta;    // histogram bin width (k_prio_init)
  uint32_t target;        // tiles to relax per pass; 0 = all (plain FIM)
  float target_frac;      // ... at least this fraction of the active list
  float cap_frac;         // kernel 5: ... and at most this fraction (>= 256 tiles); 0 = off
  int prune;              // activate a neighbour only through edge cells below its halo value
  unsigned long long* trace;  // debug: kTracePts s_memrealtime stamps per block, or null
  uint32_t sweep_deadline;  // kernel 5 (dyn): > 0: a visit stops sweeping this many 10-ns ticks
                            // after its workgroup started the pass (re-queued as if capped)
  int checker;              // kernel 5: relax only tiles with (tx + ty + checker_parity) even
  uint32_t checker_parity;  // (deterministic mode: no tile reads a halo being written)
  int exact_sqrt;  // kernel 5 (dyn): 1 = correctly rounded sweep sqrt (10 VALU), 0 = one
                   // Goldschmidt step (5 VALU, <= 36 ulp)
  // convergence mailbox: when set, block 0 stores (report_seq << 32) | n_active -- the
  // tiles queued by the previous pass -- into this word of host-coherent pinned memory,
  // so the host learns a batch's outcome without a stream synchronisation
  unsigned long long* report;
  uint32_t report_seq;
  const int32_t* report_src;  // post *report_src instead of the pass's count (sharded loop)
  // with report_src: these 4 words are stored at report[1..4] before the (seq | count)
  // word at report[0] (a fresh slot per post: the peer loop's status ring)
  const unsigned long long* report_ext;
  // priority kernels, with report: bit 31 of the posted count is set when every queued
  // tile's key (min key of the input list) exceeds the largest T over these cells -- they
  // are final (the early exit of dymu_solve_until_device); n = 0: off
  ProbeCells probe;
  // ---- kernel 5, sharded rounds (dom_round) ----
  // received neighbour rows (nx doubles, device) min-merged into the ghost rows by this
  // pass; the tiles under improved columns are queued for the NEXT pass
  const double* merge_lo;
  const double* merge_hi;
  uint32_t* tot_save;       // block 0 stores the pass's count here ...
  const uint32_t* tot_prev;  // ... and a later pass stores *tot_prev + its count
  int32_t* tot_out;          //     into *tot_out (the round's termination count)
  // peer rounds (dymu_dom_round_peer): the merge reads merge_tag[s] (the sequence tag
  // the neighbour writes after its push, system scope) before its share of the row,
  // and the pass pushes the owned first (0) / last (1) row's decreased values into the
  // neighbour's receive row push_dst[s] (peer-mapped) and, from the last workgroup,
  // the new tag into push_tag[s]; push_last[s] holds the values last pushed.  With
  // peer set, the status pass (tot_out) also records S / R in *peer.
  const unsigned long long* merge_tag[2];
  double* push_dst[2];
  unsigned long long* push_tag[2];
  double* push_last[2];
  PeerCtl* peer;
  // ---- kernel 5: edge columns (required) ----
  // ec[t * 32 + 0..15] = column 0 (W edge) of tile t's T, ec[t * 32 + 16..31] = column
  // 15 (E edge): an interior tile reads its W / E halo as ONE 128-byte line of its
  // neighbour's edge instead of one line per row; every visit writes its decreased
  // edge cells here too ("Edge columns")
  double* ec;
  // ---- kernel 5, per-pass statistics (dymu_set_pass_stats; off = null) ----
  // this pass's record: kShards rows of kPsWords words (PassStat), one row per
  // workgroup shard, summed (max / min for the radii) by the host
  uint32_t* pstat;
  int goal_tx, goal_ty;  // the goal's tile (radius = Manhattan tile distance from it)
  // ---- kernel 5: list entries carry their first-insertion key bin (kPackShift) ----
  // 1: this pass's enqueues write tile | (bin + 1) << kPackShift; an entry with a bin
  // above the pass's threshold is then deferred on its CURRENT key before any tile
  // load, one at or below it is relaxed without waiting on the key (the current key
  // is never above the first-insertion one, so the decision is the key gate's)
  int pack_bins;
};
// list entries: the tile index in the low kPackShift bits; bits above: 0 = no bin
// (seeding kernels, merges), else the key bin + 1 the entry was first inserted with
constexpr int kPackShift = 25;
constexpr uint32_t kTileMask = (1u << kPackShift) - 1u;

// per-pass statistics words (kernel 5)
enum PassStat : int {
  kPsActive = 0,    // listed entries (block 0)
  kPsVisited = 1,   // tiles relaxed
  kPsColour = 2,    // entries deferred by the checkerboard colour (no tile load)
  kPsKey = 3,       // entries deferred by the key threshold (tile loaded, then skipped)
  kPsCapped = 4,    // visits stopped by the sweep cap (re-queued)
  kPsDeadline = 5,  // visits stopped by the pass deadline (re-queued)
  kPsRadiusMax = 6, // largest tile radius relaxed (atomicMax; 0 = none or the goal tile)
  kPsSweeps = 7,    // in-tile sweeps
  kPsBstar = 8,     // threshold bin (block 0)
  kPsRadiusMin = 9, // ~smallest tile radius relaxed (atomicMin of ~r... stored as 0xFFFFFFFF - r)
  kPsEnqueued = 10, // entries appended to the next list (activations + deferrals)
  kPsWords = 12
};
constexpr uint32_t kPassStatCap = 16384;  // passes kept (a ring; pass p at p % cap)

constexpr int kBins = 64;  // v4/v5 key histogram bins
constexpr int kTracePts = 10;
// resident workgroups per CU of pass kernel variant 3/4/5 (occupancy API)
int pass_blocks_per_cu(int variant);

hipError_t launch_fill_inf(double* T, uint64_t ld, uint32_t nx, int64_t row_lo, int64_t row_hi,
                           hipStream_t st);
hipError_t launch_seed(double* T, uint64_t ld, int64_t gi, int64_t gj, uint32_t* list,
                       uint32_t* count, uint32_t* tile_epoch, uint32_t epoch, uint32_t tile,
                       int set_goal, hipStream_t st);
hipError_t launch_pass_prio(const PassArgs& a, int blocks, hipStream_t st,
                           hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_pass_prio16(const PassArgs& a, int blocks, hipStream_t st,
                             hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);  // kernel 5
hipError_t launch_pass_rb(const PassArgs& a, int blocks, hipStream_t st,
                      hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);     // v3: 2 x 8x8 tiles / wave, red-black
hipError_t launch_merge_ghosts(double* T, int64_t ld, int64_t nx, int64_t nrows,
                               const double* new_lo, const double* new_hi, int ntx, int nty,
                               int tile_w, uint32_t* list, uint32_t* counts, uint32_t cap,
                               uint32_t* tile_epoch, uint32_t epoch, unsigned long long* keys,
                               uint32_t* hist, unsigned long long* minkey, const double* base,
                               const double* delta, hipStream_t st);
hipError_t launch_exchange(double* T, int64_t ld, int64_t nx, int64_t nrows, const double* new_lo,
                           const double* new_hi, int ntx, int nty, int tile_w, uint32_t* list,
                           uint32_t* counts, uint32_t cap, uint32_t* tile_epoch, uint32_t epoch,
                           unsigned long long* keys, uint32_t* hist, unsigned long long* minkey,
                           const double* base, const double* delta, uint32_t* ticket,
                           int32_t* total, hipStream_t st);
hipError_t launch_eikonal_batch(const double* tx, const double* ty, const double* c, double* out,
                                uint64_t n, int fast, hipStream_t st);
hipError_t launch_sum_counts(const uint32_t* counts, int32_t* out, hipStream_t st);
// edge columns of tiles [t0, t1) (16x16 tiles, ntx per row) from T (see PassArgs::ec)
hipError_t launch_ec_rebuild(const double* T, uint64_t ld, uint32_t nx, uint32_t ny, double* ec,
                             uint32_t ntx, uint32_t t0, uint32_t t1, hipStream_t st);
// deterministic mode: rebuild the key histogram of a list from its FINAL keys (the
// enqueue path bins a tile by the key of its first insertion, which depends on the
// order of the insertions) into shard 0's row of `out`; `zero` (the other of two
// alternating buffers) is cleared for the next rebuild
hipError_t launch_rehist(const uint32_t* list, const uint32_t* counts, uint32_t cap,
                         const unsigned long long* keys, const double* base, const double* delta,
                         uint32_t* out, uint32_t* zero, hipStream_t st);
// computeCostMap state (SoA planner node fields, row-major pitch ld)
struct CostState {
  double* cost;
  double* raw_cost;
  double* slope;
  uint32_t* terrain;
  uint8_t* is_obstacle;
  double* hazard;
  double* traff;
  int32_t* loc_mode;
};
struct CostArgs {
  uint32_t nx, ny;
  int64_t ld;
  double res, cmax, slope_lo, slope_hi;
  int n_slopes, n_locs, lut_len;
  const double* lut;  // device copy
  const double* elevation;
  const double* terrain_map;
  CostState st;
  double* F;  // speed output (may be null for launch_cost_map)
};
hipError_t launch_cost_map(const CostArgs& a, hipStream_t st);
hipError_t launch_pack_speed(const CostArgs& a, hipStream_t st);

// windowed re-propagation (update_kernels.hip)
struct UpdateArgs {
  double* T;
  const double* F;
  int64_t ld;
  uint32_t nx, ny, gi, gj;
  const unsigned long long* theta_bits;
  uint32_t* list;    // list 0 (kShards x shard_cap)
  uint32_t* counts;  // its kShards counters
  uint32_t shard_cap;
  uint32_t* tile_epoch;
  uint32_t epoch;
  uint32_t tw, th, ntx;
  unsigned long long* keys;  // priority kernels: keys / histogram of list 0, else null
  uint32_t* hist;
};
hipError_t launch_window_min(const double* T, int64_t ld, uint32_t i0, uint32_t j0, uint32_t i1,
                             uint32_t j1, unsigned long long* out, hipStream_t st);
hipError_t launch_reset_seed(const UpdateArgs& a, hipStream_t st);
// *out += the number of cells of T (nx x ny, pitch ld) whose bits equal value's;
// with idx (device, cap entries) also the first cap of their indices j*nx + i
hipError_t launch_count_equal(const double* T, int64_t ld, uint32_t nx, uint32_t ny, double value,
                              unsigned long long* out, uint64_t* idx, uint64_t cap,
                              hipStream_t st);
// decrease-only window [i0,i1) x [j0,j1): seed the tiles that intersect it, no reset
hipError_t launch_seed_window(const UpdateArgs& a, uint32_t i0, uint32_t j0, uint32_t i1,
                              uint32_t j1, hipStream_t st);
hipError_t launch_theta_state(const unsigned long long* theta_bits, unsigned long long* minkey0,
                              double* base0, hipStream_t st);

// raise front of a windowed update with speed increases (update_kernels.hip): one
// pass over the listed 16x16 tiles; every cell whose converged value is no longer
// supported by the update of its current neighbours under the new speed (u >
// T (1 + tol)) becomes +inf, inside the tile until nothing changes; the tiles
// across an edge with an invalidated cell are listed for the next pass
struct RaiseArgs {
  double* T;
  const double* F;
  int64_t ld;
  uint32_t nx, ny, gi, gj;
  uint32_t ntx, nty;  // 16x16 tiles
  const uint32_t* list_in;
  const uint32_t* count_in;
  uint32_t* list_out;
  uint32_t* count_out;
  uint32_t* count_clear;
  uint32_t shard_cap;
  uint32_t* tile_epoch;
  uint32_t epoch;
  double tol;
  unsigned long long* stats;  // [0] tile visits, [1] cells invalidated
};
hipError_t launch_raise(const RaiseArgs& a, int blocks, hipStream_t st);
// after the raise: list 0 <- every tile holding a finite-speed +inf cell (not the goal)
// next to a finite cell, key = the smallest such neighbour value of the tile (a
// scheduling hint), histogram bin 0; *theta_bits lowered to the smallest key
hipError_t launch_cone_seed(const UpdateArgs& a, unsigned long long* theta_bits, hipStream_t st);

// early exit of computeTotalCostMap (update_kernels.hip)
// out[0] = bits of max T over the probe cells, out[1] = *minkey (or +inf bits if null)
hipError_t launch_probe(const double* T, int64_t ld, const ProbeCells& cells,
                        const unsigned long long* minkey, unsigned long long* out,
                        hipStream_t st);
// reference node states after the early exit: T > t_closed -> +inf unless the cell is a
// finite-speed 4-neighbour of a cell with T <= t_closed (the band: index appended to band)
hipError_t launch_early_mask(const double* F, double* T, int64_t ld, uint32_t nx, uint32_t ny,
                             double t_closed, uint64_t* band, unsigned long long* n_band,
                             uint64_t cap, hipStream_t st);
// the early exit's region: bbox of the cells with T <= thr into out[0..3] (atomic
// min i, min j, max i, max j: initialise to ~0, ~0, 0, 0) and the count of cells with
// lo <= T <= hi added to out[4]
hipError_t launch_region_box(const double* T, int64_t ld, uint32_t nx, uint32_t ny, double thr,
                             double lo, double hi, unsigned long long* out, hipStream_t st);
// least squared distance from (gi, gj) to a cell of speed != f0 into *out (atomic min:
// initialise to ~0)
hipError_t launch_const_radius(const double* F, int64_t ld, uint32_t nx, uint32_t ny, uint32_t gi,
                               uint32_t gj, double f0, unsigned long long* out, hipStream_t st);
// *p = v, in stream order (no host-to-device copy for a per-call scalar)
hipError_t launch_store_u64(unsigned long long* p, unsigned long long v, hipStream_t st);
// T[(idx / nx) * ld + idx % nx] = vals[k]
hipError_t launch_scatter(double* T, int64_t ld, uint32_t nx, const uint64_t* idx,
                          const double* vals, uint64_t n, hipStream_t st);

hipError_t launch_prio_init(const double* F, int64_t ld, int64_t nx, int64_t ny,
                           unsigned long long* keys, uint64_t nkeys, uint32_t* hist, uint64_t nhist,
                           unsigned long long* minkey, double* base, double* delta, double kappa,
                           hipStream_t st);
hipError_t launch_prio_seed(unsigned long long* key0, uint32_t* hist0, unsigned long long* minkey0,
                           uint32_t tile, double keyv, hipStream_t st);
hipError_t launch_synth(double* F, uint64_t ld, uint32_t nx, uint32_t ny, uint64_t row0,
                        uint64_t seed, double frac, uint64_t oseed, int64_t gi, int64_t gj,
                        hipStream_t st);

}  // namespace dymu
