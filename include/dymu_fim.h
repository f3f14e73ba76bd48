/*
 * dymu_fim.h -- C-ABI of the MI355X (gfx950) total-cost propagation engine.
 *
 * This is the drop-in boundary for the DyMu global total-cost propagation
 * (ESA-PRL/planning-path_planning).  It replaces, for the host C++ planner
 * (include/DyMu.hpp), the hot loop of:
 *   - DyMuPathPlanner::computeEntireTotalCostMap   src/DyMu_GlobalPathPlanning.cpp:443-468
 *   - DyMuPathPlanner::computeTotalCostMap         src/DyMu_GlobalPathPlanning.cpp:364-408
 *   - propagateGlobalNode (Eikonal update)          src/DyMu_GlobalPathPlanning.cpp:500-546
 *   - minCostGlobalNode (narrow band)               src/DyMu_GlobalPathPlanning.cpp:551-568
 *   - resetTotalCostMap / resetGlobalNarrowBand     src/DyMu_GlobalPathPlanning.cpp:473-496
 * The reference has no FFI; its boundary is the C++ class in src/DyMu.hpp:397-609.
 * This header is the C surface that class (our include/DyMu.hpp) calls, and
 * the one a cgo / JNI / ctypes binding would bind.
 *
 * Data model: row-major fp64 grids, index = j*ld + i (j = y row, i = x col,
 * reference :52-58).  F[k] is the per-node speed C of reference :527-528,
 *   F = global_res * cost * (2 + hazard_density - trafficability),
 * and +inf (or NaN) for an obstacle.  F must be >= 0 or +inf.  T[k] receives
 * the converged total cost; +inf marks unreachable cells and obstacles; the
 * goal holds 0.  Results equal the reference FMM within |dT| <= 1e-12*max(1,T)
 * with an identical +inf mask for speeds with 2*F*F finite
 * (F < 1.34e154); beyond that the reference update itself is order-dependent.
 *
 * All functions return DYMU_OK (0) or a negative dymu_status.  Contexts are
 * not thread-safe; use one context per host thread.
 */
#ifndef DYMU_FIM_H
#define DYMU_FIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DYMU_ABI_VERSION 5

typedef enum dymu_status {
  DYMU_OK = 0,
  DYMU_ERR_ARG = -1,           /* bad argument (null pointer, size, goal off-grid) */
  DYMU_ERR_HIP = -2,           /* HIP runtime error (see dymu_last_error) */
  DYMU_ERR_NOMEM = -3,         /* device allocation failed */
  DYMU_ERR_NOT_CONVERGED = -4, /* pass cap reached (dymu_opts.max_passes) */
  DYMU_ERR_NO_DEVICE = -5,     /* no HIP device / extension unusable */
  DYMU_ERR_RCCL = -6,          /* RCCL error in the sharded solver */
  DYMU_ERR_STATE = -7          /* call out of sequence (e.g. comm not initialised) */
} dymu_status;

typedef struct dymu_ctx dymu_ctx;

typedef struct dymu_opts {
  int device;           /* HIP device ordinal; -1 = current device */
  int passes_per_check; /* passes launched between convergence read-backs; 0 = adaptive */
  int max_passes;       /* safety cap on FIM passes; 0 = derived from the grid size */
  int max_inner;        /* cap on in-tile sweeps per tile visit; 0 = default */
  int grid_blocks;      /* workgroups per pass launch; 0 = derived from the device */
  int kernel;           /* pass kernel: 0 = auto (by grid size), 3 = plain block FIM
                           (8x8 tiles), 4 = priority passes on 8x8 tiles, 5 = priority
                           passes on 16x16 tiles */
  int prio_target;      /* kernels 4/5: tiles relaxed per pass; 0 = default
                           (64 per CU for 4, 8 per CU for 5) */
  int exact_sqrt;       /* kernel 5: 1 = correctly rounded sqrt in the sweeps; 0 = default:
                           one Goldschmidt step folded into the candidate.  Both use the
                           monotone combine min(Tx,Ty) + h (one rounding at the scale of T,
                           within 1 ulp of the reference candidate plus the sqrt's error),
                           so the FIM's min over history does not accumulate a rounding
                           bias along long paths (DESIGN.md s3, s4 "Monotone combine") */
  int deterministic;    /* 1 = bit-reproducible maps: kernel 5 with checkerboard passes (a
                           pass relaxes tiles of one colour only, so no tile reads a halo
                           another wave is writing) and no sweep deadline; ~2x the passes.
                           0 = default (the last ulps depend on the schedule) */
} dymu_opts;

typedef struct dymu_stats {
  uint64_t passes;       /* FIM passes that had active tiles ("iterations to converge") */
  uint64_t launches;     /* pass kernels launched (incl. speculative empty ones) */
  uint64_t tile_visits;  /* sum over passes of active tiles */
  uint64_t inner_sweeps; /* sum over tile visits of in-tile sweeps */
  uint64_t max_active;   /* largest active-tile list */
  uint64_t rounds;       /* sharded solver: halo-exchange rounds (0 single GPU) */
  double ms;             /* device time of the solve (HIP events), ms */
  int tile_w, tile_h;    /* tile geometry used */
  int kernel;            /* pass kernel that ran (see dymu_opts.kernel) */
  int reserved;
  uint64_t deferred;     /* kernel 5: list entries deferred to a later pass (key above the
                            pass's threshold bin); entries drawn = tile_visits + deferred */
} dymu_stats;

/* Context: owns a HIP stream, events and workspace on one device. */
int dymu_create(dymu_ctx** out, const dymu_opts* opts); /* opts may be NULL */
int dymu_destroy(dymu_ctx* ctx);

/* Host-buffer solve: copies F in, solves, copies T out (the planner path).
 * F, T_out: nx*ny doubles, row-major, caller-owned host memory. */
int dymu_solve(dymu_ctx* ctx, const double* F, uint32_t nx, uint32_t ny, uint32_t goal_i,
               uint32_t goal_j, double* T_out, dymu_stats* stats);

/* Device-resident solve: dF, dT are device pointers with row pitch `ld`
 * elements (ld >= nx).  dT is overwritten (initialised to +inf, goal 0).
 * `stream` is a hipStream_t or NULL for the context's own stream.  Blocks
 * until converged. */
int dymu_solve_device(dymu_ctx* ctx, const double* dF, double* dT, uint32_t nx, uint32_t ny,
                      uint64_t ld, uint32_t goal_i, uint32_t goal_j, void* stream,
                      dymu_stats* stats);

/* ---- computeTotalCostMap's early exit (reference src/DyMu_GlobalPathPlanning.cpp:364-408) ----
 * The reference stops its FMM as soon as the start node and its 4-neighbours
 * are CLOSED (isFullyClosedNode :424-436).  dymu_solve_until_device is
 * dymu_solve_device with that stop: it returns as soon as every queued tile's
 * priority key -- a lower bound on any value the remaining passes can produce --
 * exceeds t = max T over the start (start_i, start_j) and its in-grid
 * 4-neighbours, or when the map has converged.  On return every cell whose
 * converged value is <= *t_closed = t holds that value (the reference's CLOSED
 * set); other cells hold upper bounds.  *t_closed = +inf when the start is
 * unreachable (the whole map is then converged).  Runs a priority kernel (4 or
 * 5) whatever dymu_opts.kernel says. */
int dymu_solve_until_device(dymu_ctx* ctx, const double* dF, double* dT, uint32_t nx,
                            uint32_t ny, uint64_t ld, uint32_t goal_i, uint32_t goal_j,
                            uint32_t start_i, uint32_t start_j, void* stream, double* t_closed,
                            dymu_stats* stats);
/* The node states after that early exit: a cell is CLOSED iff T <= t_closed and
 * keeps T; a finite-speed 4-neighbour of a CLOSED cell is in the narrow band
 * (the reference propagated into it, :462-465) and keeps its current T for the
 * caller to replace with the reference's tentative value; every other cell
 * gets +inf (never reached: -1 in getTotalCostMatrix).  band_idx: host buffer
 * of `cap` entries receiving the band cells' indices j*nx + i (unordered);
 * *n_band = their number -- if it exceeds cap only cap were written, and the
 * call may be repeated with a larger buffer (it is idempotent). */
int dymu_early_exit_mask(dymu_ctx* ctx, const double* dF, double* dT, uint32_t nx, uint32_t ny,
                         uint64_t ld, double t_closed, uint64_t* band_idx, uint64_t cap,
                         uint64_t* n_band, void* stream);
/* *count = the number of cells of dT whose value is bitwise `value` (the early
 * exit's tie test: cells of exactly t_closed other than the last one the
 * reference closes make its CLOSED set depend on its insertion order).
 * Synchronises `stream`. */
int dymu_count_equal(dymu_ctx* ctx, const double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
                     double value, uint64_t* count, void* stream);
/* dymu_count_equal that also lists the cells: *count = their number, idx (host,
 * cap entries) their indices j*nx + i (the first cap found, unordered).  The
 * planner's early exit resolves the reference's order among them. */
int dymu_find_equal(dymu_ctx* ctx, const double* dT, uint32_t nx, uint32_t ny, uint64_t ld,
                    double value, uint64_t* idx, uint64_t cap, uint64_t* count, void* stream);
/* The early exit's region, for the planner's near-tie guard and its exact host
 * replay: the bounding box of the cells with T <= thr (i0, j0, i1, j1
 * inclusive; i0 > i1 when there is none), the number of cells with lo <= T <= hi (the
 * engine's near ties with the exit value), and r_const, the Euclidean distance from
 * the goal (goal_i, goal_j) to the nearest cell whose speed differs from the goal's
 * (+inf: constant speed everywhere).  Synchronises `stream`. */
typedef struct dymu_region {
  uint32_t i0, j0, i1, j1;
  uint64_t n_range;
  double r_const;
} dymu_region;
int dymu_region_stats(dymu_ctx* ctx, const double* dF, const double* dT, uint32_t nx, uint32_t ny,
                      uint64_t ld, uint32_t goal_i, uint32_t goal_j, double thr, double lo,
                      double hi, dymu_region* out, void* stream);
/* dT[(idx[k] / nx) * ld + idx[k] % nx] = vals[k] for k < n (idx, vals: host). */
int dymu_scatter(dymu_ctx* ctx, double* dT, uint32_t nx, uint64_t ld, const uint64_t* idx,
                 const double* vals, uint64_t n, void* stream);

/* ---- row-slab domains (multi-GPU sharding; also single-GPU virtual slabs) ----
 * A rank owns rows [row0, row0+nrows) of an nx-wide global grid.  T points at
 * its first owned row; with ghost_lo the row above it (T - ld) holds the
 * neighbour rank's last row, with ghost_hi the row T + nrows*ld holds the
 * next rank's first row (then nrows must be a multiple of 32).  Ghost rows are
 * read-only halo for the kernels.  Protocol (bench_sharded.py / dymu.sharded):
 *   dymu_dom_begin -> repeat { dymu_dom_run(K passes); exchange boundary rows
 *   (RCCL); dymu_dom_merge_ghosts(received rows) } until the all-reduced
 *   pending count is 0 -> dymu_dom_finish.
 * or, on kernel-5 slabs (include/dymu_dist.h's native loop):
 *   dymu_dom_begin -> repeat { dymu_dom_round(K passes, merging the rows the
 *   previous exchange received); exchange boundary rows } until 0 -> finish.
 * All calls except dymu_dom_pending / dymu_dom_finish are asynchronous on
 * `stream`. */
typedef struct dymu_domain {
  const double* F; /* owned rows, pitch ld (device) */
  double* T;       /* owned row 0 (device); ghost rows at T - ld / T + nrows*ld */
  uint64_t ld;
  uint32_t nx, nrows;
  int32_t ghost_lo, ghost_hi;
} dymu_domain;

/* Partition ny rows over nranks slabs (boundaries on multiples of 32 rows). */
int dymu_slab_rows(uint32_t ny, uint32_t nranks, uint32_t rank, uint32_t* row0, uint32_t* nrows);
/* Initialise T (owned + ghost rows = +inf) and seed the goal if it lies in
 * this slab (goal_j_local = goal row - row0, or -1). */
int dymu_dom_begin(dymu_ctx* ctx, const dymu_domain* dom, int64_t goal_i, int64_t goal_j_local,
                   void* stream);
/* Launch `passes` FIM passes (speculative passes with no active tile are cheap). */
int dymu_dom_run(dymu_ctx* ctx, uint32_t passes, void* stream);
/* Min-merge received neighbour rows (device pointers, nx doubles, or NULL)
 * into the ghost rows and queue the tiles under improved columns; if
 * d_pending != NULL also write the number of queued tiles there (int32). */
int dymu_dom_merge_ghosts(dymu_ctx* ctx, const double* new_lo, const double* new_hi,
                          int32_t* d_pending, void* stream);
/* dymu_dom_merge_ghosts with the queued-tile count in the SAME launch (the
 * native sharded loop's per-round step, include/dymu_dist.h): *d_total (device
 * int32, required) receives the number of tiles queued for the next pass. */
int dymu_dom_exchange(dymu_ctx* ctx, const double* new_lo, const double* new_hi,
                      int32_t* d_total, void* stream);
/* One round with the ghost merge inside the passes: `passes` (>= 2) FIM passes,
 * the first of which min-merges the received rows (device, nx doubles, or NULL)
 * into the ghost rows; *d_total (device int32) receives the tiles queued for
 * the round's first pass plus those queued for its second (0 on every rank =
 * fixed point).  Replaces dymu_dom_run + dymu_dom_exchange for the rows of the
 * PREVIOUS round (one launch per round fewer).  Only for domains on kernel 5:
 * DYMU_ERR_STATE otherwise; dymu_dom_round_supported says which (1 / 0). */
int dymu_dom_round_supported(dymu_ctx* ctx, uint32_t passes);
/* 1 if a domain of nx x nrows cells would support fused rounds of `passes` (the
 * check dymu_dom_round_supported makes after dymu_dom_begin), before any domain
 * exists: the sharded solver's pre-flight rejects an unsupported peer-transport
 * solve on every rank with DYMU_ERR_ARG instead of aborting the communicator. */
int dymu_dom_round_capable(dymu_ctx* ctx, uint32_t nx, uint32_t nrows, uint32_t passes);
int dymu_dom_round(dymu_ctx* ctx, uint32_t passes, const double* new_lo, const double* new_hi,
                   int32_t* d_total, void* stream);
/* Arm a post for the next launched pass: its block 0 stores *d_src (device
 * int32) into the context's host-coherent mailbox with sequence *seq, so the
 * host can read a device value (the all-reduced count) without a copy or a
 * stream synchronisation; dymu_dom_wait_post spins for it (timeout_s > 0:
 * DYMU_ERR_HIP after that long).  DYMU_ERR_STATE without a mailbox. */
int dymu_dom_post(dymu_ctx* ctx, const int32_t* d_src, uint32_t* seq);
int dymu_dom_wait_post(dymu_ctx* ctx, uint32_t seq, double timeout_s, int32_t* value,
                       void* stream);
/* Peer rounds (include/dymu_dist.h's GPU-initiated peer transport):
 * dymu_dom_round whose first pass also PUSHES this rank's first / last owned row
 * into the neighbours' receive rows (peer-mapped device memory) -- only the
 * values below those last pushed -- and, from the pass's last workgroup, writes a
 * sequence tag after them (system-scope release); the merge of the same pass reads
 * this rank's own receive rows after their tags.  No host involvement and no wait
 * on a neighbour: rows arrive whenever the neighbour's pass runs, and any mix of
 * old and new values is a valid upper bound.  The round's second pass records in
 * `ctl` the status a termination check needs: P (tiles queued for the round's two
 * first passes), S per side (pushes that carried a decrease) and R per side (the
 * smallest tag the round's merge read).  Kernel-5 domains, passes >= 2. */
#define DYMU_PEER_CTL_BYTES 128
typedef struct dymu_peer_links {
  const double* recv[2];                 /* own receive rows: from rank-1 (0) / rank+1 (1) */
  const unsigned long long* recv_tag[2]; /* their tags (written by the neighbours) */
  double* send[2];                       /* the neighbours' receive rows for the first (0) /
                                            last (1) owned row (peer-mapped), NULL = none */
  unsigned long long* send_tag[2];       /* ... and their tags */
  double* last[2];                       /* nx values last pushed per side (device) */
  void* ctl;                             /* DYMU_PEER_CTL_BYTES of device memory */
} dymu_peer_links;
int dymu_dom_round_peer(dymu_ctx* ctx, uint32_t passes, const dymu_peer_links* links,
                        void* stream);
/* Arm a status post for the next launched pass: its block 0 stores the status of
 * `ctl` (S0, S1, R0, R1) at dst[1..4], then (seq << 32) | P at dst[0] (release,
 * system scope).  dst: device address of 5 words of host-coherent memory. */
int dymu_dom_post_status(dymu_ctx* ctx, const void* ctl, unsigned long long* dst, uint32_t seq);
/* Tiles queued for the next pass (synchronises `stream`). */
int dymu_dom_pending(dymu_ctx* ctx, void* stream, uint64_t* pending);
/* End the domain solve; fills stats (passes, visits, sweeps). */
int dymu_dom_finish(dymu_ctx* ctx, void* stream, dymu_stats* stats);

/* Synthetic input generator on the device (bench/test data):
 *   F[k] = 1 + 4*u(seed, k),  u(s,k) = (splitmix64(s ^ k) >> 11) * 2^-53,
 *   obstacle (F = +inf) where u(obst_seed, k) < obst_frac, except the 3x3
 *   block around (goal_i, goal_j).  k = j*nx + i is the GLOBAL cell index, so
 *   shards generate identical values: rows [row0, row0+ny) of a grid nx wide. */
int dymu_synth_speed(dymu_ctx* ctx, double* dF, uint32_t nx, uint32_t ny, uint64_t ld,
                     uint64_t row0, uint64_t seed, double obst_frac, uint64_t obst_seed,
                     uint32_t goal_i, uint32_t goal_j, void* stream);

/* Arithmetic self-test: out[k] = the kernels' Eikonal candidate for
 * (Tx[k], Ty[k], C[k]) (reference :531-535), computed by the same device code
 * the pass kernels use (fast = 1: the range-restricted correctly rounded sqrt in
 * the reference's combine, kernels 3/4; fast = 2: kernel 5's default sweep
 * candidate, monotone combine + one Goldschmidt step; fast = 3: kernel 5 with
 * exact_sqrt, monotone combine + correctly rounded sqrt; fast = 4: the v31 sweep
 * candidate, kept for A/B).
 * Device pointers; blocks until done. */
int dymu_eikonal_batch(dymu_ctx* ctx, const double* tx, const double* ty, const double* c,
                       double* out, uint64_t n, int fast);

/* Device memory helpers (so a host without torch can run the device path).
 * dymu_device_alloc returns uncached device memory (hipDeviceMallocUncached: no L2
 * lines of the maps are left dirty for each pass's end-of-kernel release to write
 * back -- 27.5 vs 28.1 ms per 16384^2 solve); DYMU_MAP_MEM=0 gives
 * plain hipMalloc memory, 1 fine-grained.  Any device memory works with the solve
 * entry points.  The copies are ordered after the work queued on the context stream
 * and are complete on return. */
int dymu_device_alloc(dymu_ctx* ctx, size_t bytes, void** dptr);
int dymu_device_free(dymu_ctx* ctx, void* dptr);
int dymu_memcpy_d2h(dymu_ctx* ctx, void* dst, const void* src, size_t bytes);
int dymu_memcpy_h2d(dymu_ctx* ctx, void* dst, const void* src, size_t bytes);
/* pitched copies (hipMemcpy2D: width bytes per row, height rows) */
int dymu_memcpy2d_d2h(dymu_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width, size_t height);
int dymu_memcpy2d_h2d(dymu_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width, size_t height);
/* page-lock a host buffer for full-speed DMA (hipHostRegister) / undo it */
int dymu_host_register(dymu_ctx* ctx, void* p, size_t bytes);
int dymu_host_unregister(dymu_ctx* ctx, void* p);

/* ---- dynamic update: windowed re-propagation ----
 * After the speed changed only inside the window [i0, i0+w) x [j0, j0+h)
 * (the local layer's hazard / trafficability writes, reference
 * src/DyMu_LocalPathRepairing.cpp:264-274, :389-394, entering F through
 * src/DyMu_GlobalPathPlanning.cpp:527-528), bring T from the converged map of
 * the old speed to that of the new one without a cold solve: cells whose old
 * T is below theta = min(old T over the window and its 1-cell ring) provably
 * keep their value; the rest is reset and re-propagated from the boundary of
 * the kept region.  With DYMU_RAISE=1 a raise front instead
 * sets to +inf exactly the cells whose converged value is no longer supported
 * under the new speed (the window's dependency cone; cells supported within
 * 1e-13 relative keep their value) and the FIM re-propagates the cone from its
 * boundary -- exact and smaller, but slower on config 5.
 * Increases and decreases are both handled; the result is the fixed point a
 * cold dymu_solve of the new speed reaches.
 * The window is clipped to the grid. */
int dymu_resolve_window_device(dymu_ctx* ctx, const double* dF, double* dT, uint32_t nx,
                               uint32_t ny, uint64_t ld, uint32_t goal_i, uint32_t goal_j,
                               uint32_t i0, uint32_t j0, uint32_t w, uint32_t h, void* stream,
                               dymu_stats* stats);
/* The same with the caller's knowledge of the change: decrease_only != 0
 * promises that no F in the window increased (F grows with hazard density and
 * falls with trafficability, reference :527-528: e.g. a hazard cleared or a
 * trafficability restored after src/DyMu_LocalPathRepairing.cpp:389-394).  Then
 * the old map is a valid upper bound everywhere and no cell is reset: only the
 * window's tiles are seeded and the passes lower what the cheaper window
 * reaches.  decrease_only = 0 is dymu_resolve_window_device. */
int dymu_update_window_device(dymu_ctx* ctx, const double* dF, double* dT, uint32_t nx,
                              uint32_t ny, uint64_t ld, uint32_t goal_i, uint32_t goal_j,
                              uint32_t i0, uint32_t j0, uint32_t w, uint32_t h, int decrease_only,
                              void* stream, dymu_stats* stats);
/* What the last windowed update did before its re-solve: out[0] raise passes,
 * out[1] tiles visited by them, out[2] cells invalidated (the dependency cone of
 * the window's speed increases; 0s for decrease-only updates), out[3] reserved. */
int dymu_last_update_stats(dymu_ctx* ctx, uint64_t out[4]);
/* Host-buffer form: requires that the previous dymu_solve / dymu_resolve_window
 * on this context solved the same grid size and goal (DYMU_ERR_STATE otherwise);
 * only the window of F is uploaded, the whole new T is written to T_out. */
int dymu_resolve_window(dymu_ctx* ctx, const double* F, uint32_t nx, uint32_t ny, uint32_t goal_i,
                        uint32_t goal_j, uint32_t i0, uint32_t j0, uint32_t w, uint32_t h,
                        double* T_out, dymu_stats* stats);

/* ---- computeCostMap on the device ----
 * Planner node state (the globalNode fields of reference src/DyMu.hpp:69-108
 * that the global layer uses) as device SoA arrays, row-major, pitch ld. */
typedef struct dymu_cost_state {
  double* cost;         /* smoothed cost; its previous value feeds the smoothing (Q1) */
  double* raw_cost;     /* nominal cost before smoothing */
  double* slope;        /* rad */
  uint32_t* terrain;    /* terrain class, 0 on the border */
  uint8_t* is_obstacle; /* sticky */
  double* hazard;       /* hazard_density */
  double* traff;        /* trafficability */
  int32_t* loc_mode;    /* -1 = "DONT_CARE", else the locomotion index */
} dymu_cost_state;

/* computeCostMap (reference src/DyMu_GlobalPathPlanning.cpp:145-181 with
 * calculateSlope :186-210, calculateNominalCost :217-293, smoothCost
 * :297-308; quirks Q1-Q4) over device arrays elevation / terrain_map (class
 * as double, like the reference's vector<vector<double>>); lut and slopes are
 * HOST arrays (the reference's cost_data / slope_values).  If dF is not NULL
 * the speed F = (res*cost)*((2+hazard)-traff), +inf for obstacles (:527-528),
 * is written too.  Asynchronous on `stream` (NULL: the context's stream).
 * nx, ny >= 2.  A terrain class beyond the LUT marks the cell as an obstacle
 * (the reference reads out of bounds there). */
int dymu_compute_cost_map(dymu_ctx* ctx, uint32_t nx, uint32_t ny, uint64_t ld, double global_res,
                          const double* lut, int lut_len, const double* slopes, int n_slopes,
                          int n_locs, const double* elevation, const double* terrain_map,
                          const dymu_cost_state* st, double* dF, void* stream);

/* The speed alone from the state (after hazard / trafficability updates). */
int dymu_pack_speed(dymu_ctx* ctx, uint32_t nx, uint32_t ny, uint64_t ld, double global_res,
                    const dymu_cost_state* st, double* dF, void* stream);

/* Profiling: period > 0 times every period-th pass launch with HIP events
 * (start/stop taken by the dispatch itself); 0 turns it off.  Sampling keeps
 * the event overhead out of the timed region (period 1 costs ~4 us/launch). */
int dymu_set_profiling(dymu_ctx* ctx, int period);

/* Per-pass statistics of kernel 5 (diagnostics; off by default, costs a few
 * atomics per workgroup per pass when on): enable, then after a solve read one
 * record of DYMU_PASS_STAT_WORDS words per pass (the first min(launches, 16384)
 * passes; *n = their number):
 *   [0] listed entries   [1] tiles relaxed    [2] colour-deferred entries
 *   [3] key-deferred entries (tile loaded, key above the pass threshold)
 *   [4] visits stopped by the sweep cap   [5] ... by the pass deadline
 *   [6] largest / [9] smallest Manhattan tile distance from the goal's tile relaxed
 *   [7] in-tile sweeps   [8] threshold bin   [10] entries appended to the next list */
#define DYMU_PASS_STAT_WORDS 12
int dymu_set_pass_stats(dymu_ctx* ctx, int enable);
int dymu_last_pass_stats(dymu_ctx* ctx, uint32_t* out, uint64_t cap_passes, uint64_t* n);

/* Summed kernel time (ms, HIP events on the launch stream) of the most recent
 * solve's SAMPLED pass launches and their count: the mean launch duration is
 * pass_ms_total / n_pass_launches -- the bench's roofline source. */
int dymu_last_pass_timing(dymu_ctx* ctx, double* pass_ms_total, uint64_t* n_pass_launches);

/* The context's own stream (the hipStream_t that NULL `stream` arguments mean). */
void* dymu_get_stream(dymu_ctx* ctx);

const char* dymu_strerror(int status);
const char* dymu_last_error(dymu_ctx* ctx); /* last HIP/RCCL error text */
int dymu_abi_version(void);
int dymu_device_count(void);

#ifdef __cplusplus
}
#endif
#endif
