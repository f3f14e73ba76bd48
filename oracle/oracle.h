/*
 * oracle.h -- CPU restatement of the DyMu global total-cost propagation.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libdymu_fim.so,
 * libdymu_planner.so, the `dymu` Python module) links, loads or calls this
 * library.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it, and only as the checker.
 *
 * Every function restates one piece of the reference
 * (ESA-PRL/planning-path_planning, src/DyMu_GlobalPathPlanning.cpp) and cites
 * the file:line it follows.  Grid convention (reference :52-100): row-major
 * [j][i], j = y row, i = x column, index = j*nx + i.  nb4 order
 * {(i,j-1),(i-1,j),(i+1,j),(i,j+1)} (reference :76-80).
 *
 * Pinning: the reference has no tests and cannot be rebuilt here (it needs
 * Rock base-types/base-logging headers absent from the image).  The
 * restatement is pinned against the reference-run known-answer checksums
 * recorded in SURVEY.md s8(c) (sum of getTotalCostMatrix and T[1][1] at
 * N = 256..4096, mt19937_64(1) inputs) and against closed forms; see
 * tests/test_oracle.py and DESIGN.md s3.
 */
#ifndef DYMU_ORACLE_H
#define DYMU_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- input generators (test/bench data, not reference code) ---- */
/* std::mt19937_64(seed) + std::uniform_real_distribution<double>(lo,hi),
 * drawn row-major (libstdc++ generate_canonical with one 64-bit draw).
 * This is the input of the SURVEY.md s8(c) KATs. */
void oracle_fill_mt19937_uniform(double* out, uint64_t n, uint64_t seed, double lo, double hi);
/* counter-based u(idx) = (splitmix64(seed ^ idx) >> 11) * 2^-53 */
double oracle_u01(uint64_t seed, uint64_t idx);
void oracle_fill_u01(double* out, uint64_t n, uint64_t seed);

/* ---- per-node speed (reference :527-528) ----
 * F = (res*cost) * ((2 + hazard) - traff); obstacles -> +inf.
 * isObstacle may be NULL (no obstacles), hazard NULL (0), traff NULL (1). */
void oracle_pack_speed(const double* cost, const double* hazard, const double* traff,
                       const uint8_t* is_obstacle, uint64_t n, double res, double* F);

/* setCostMap (reference :109-126): cost<=0 => obstacle, traff 0, hazard 1.
 * Arrays are the planner state (in/out); borders are NOT forced. */
void oracle_set_cost_map(const double* cost_map, uint64_t n, double* cost, uint8_t* is_obstacle,
                         double* traff, double* hazard);

/* computeCostMap (reference :145-181, :186-210, :217-293, :297-308),
 * quirks Q1-Q4 of SURVEY s8(a) honoured.  State arrays (cost, is_obstacle,
 * traff, hazard, loc_mode) carry over between calls like the reference's
 * node fields.  loc_mode: -1 = "DONT_CARE", else the locomotion index. */
void oracle_compute_cost_map(uint32_t nx, uint32_t ny, double res, const double* lut, int lut_len,
                             const double* slopes, int n_slopes, int n_locs,
                             const double* elevation, const double* terrain_map,
                             /* state, in/out */
                             double* raw_cost, double* cost, double* slope, uint32_t* terrain,
                             uint8_t* is_obstacle, double* traff, double* hazard,
                             int32_t* loc_mode);

/* setGoal validation (reference :322-357).  Returns 1 and the node on
 * success, 0 if rejected.  is_obstacle may be NULL. */
int oracle_set_goal(uint32_t nx, uint32_t ny, double res, double offx, double offy, double wx,
                    double wy, const uint8_t* is_obstacle, uint32_t* gi, uint32_t* gj);

/* Eikonal node update (reference :500-546), returns the candidate T'. */
double oracle_eikonal(double Tx, double Ty, double C);

/* computeEntireTotalCostMap (reference :443-468) with the reference's own
 * linear-scan narrow band (minCostGlobalNode :551-568: first strict minimum in
 * band order, then erase).  F = +inf marks an obstacle.  T receives +inf for
 * unreachable cells.  If start_i/start_j >= 0 the loop stops early like
 * computeTotalCostMap (reference :390-398, isFullyClosedNode :424-436); T
 * then holds tentative band values and `closed` the node states.
 * Returns: 1 = band non-empty at exit (computeTotalCostMap true),
 *          0 = band empty at exit, -1 bad args.  n_pops receives #pops. */
int oracle_fmm_linear(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                      int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                      uint64_t* n_pops);

/* Same algorithm, same pop order: binary heap keyed (T, first-insertion
 * sequence), which is exactly the linear scan's tie rule because the band
 * vector keeps insertion order under erase.  Bit-identical to
 * oracle_fmm_linear; O(N log N).  This is the CPU baseline ("port"). */
int oracle_fmm_heap(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                    int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                    uint64_t* n_pops);
/* oracle_fmm_heap plus each node's band-insertion sequence number seq[k] (its
 * position in the reference's global_narrowband / global_propagated_nodes when it
 * first became finite; goal 0; UINT64_MAX never reached). */
int oracle_fmm_order(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                     int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                     uint64_t* seq);

/* All-cores CPU baseline (oracle_par.c, SURVEY s8(d) cpu_fim_omp): the same fixed
 * point reached by a block FIM over `threads` OpenMP threads (64 x 64 tiles, a
 * warm-started fast-marching solve inside a tile).  Equals oracle_fmm_heap within ulps.
 * Returns 0, or -1 on bad arguments; *passes = parallel passes. */
int oracle_fim_parallel(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                        double* T, int threads, uint64_t* passes);

/* Jacobi iteration of the same update to its fixed point from T=+inf
 * (SURVEY s8(c)); returns the number of sweeps.  Used by property tests. */
int oracle_jacobi(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj, double* T,
                  int max_sweeps);

/* One Jacobi sweep's max |T - U(T)| over non-obstacle, non-goal cells whose
 * update would DECREASE T (zero residual <=> fixed point). */
double oracle_residual(const double* F, const double* T, uint32_t nx, uint32_t ny, uint32_t gi,
                       uint32_t gj, uint64_t* n_decreasing);

/* getTotalCostMatrix (reference :799-811): +inf -> -1.0 */
void oracle_total_cost_matrix(const double* T, uint64_t n, double* out);

/* computeGlobalPath (reference :615-662, :666-714, :718-772, :776-784).
 * T: total cost (+inf unreachable), elev: elevation (may be NULL => 0),
 * wx/wy/wh: start in grid-local metres + heading (offset already removed, as getPath does
 * at :593-594).  Writes up to max_wp waypoints (x,y,z,heading) into wp.
 * Returns #waypoints (>=0), -1 when the reference returns false at the first
 * NaN check (:628), -2 on "ERROR in trajectory" (:650-656), -3 when more than
 * max_wp waypoints would be produced.  risk_distance sets tau=min(0.4,rd). */
int oracle_global_path(const double* T, const double* elev, uint32_t nx, uint32_t ny, double res,
                       uint32_t gi, uint32_t gj, double goal_heading, double risk_distance,
                       double wx, double wy, double wh, double* wp, int max_wp);

/* computeGlobalPath keeping what it pushed before a failure (see oracle.c). */
int oracle_global_path_partial(const double* T, const double* elev, uint32_t nx, uint32_t ny,
                               double res, uint32_t gi, uint32_t gj, double goal_heading,
                               double risk_distance, double wx, double wy, double wh, double* wp,
                               int max_wp, int* n_out);

/* ---- the local layer (oracle_local.c; reference DyMu_LocalPathRepairing.cpp) ----
 * A context holds a copy of the global layer the local layer reads (obstacle
 * flags, total cost, CLOSED state, elevation, goal) and writes (hazard
 * density, trafficability), current_path and the lazily subdivided sub-grid. */
typedef struct oracle_local oracle_local;
oracle_local* oracle_local_create(uint32_t nx, uint32_t ny, double gres, double lres, double offx,
                                  double offy, double risk_distance, double reconnect_distance,
                                  double risk_ratio, int approach);
void oracle_local_destroy(oracle_local* L);
/* any pointer may be NULL (keeps the current array) */
void oracle_local_set_global(oracle_local* L, const uint8_t* obst, const double* T,
                             const uint8_t* closed, const double* elev, const double* hazard,
                             const double* traff, uint32_t gi, uint32_t gj, double goal_heading);
void oracle_local_get_global(const oracle_local* L, double* hazard, double* traff);
void oracle_local_set_path(oracle_local* L, const double* wp, int n);
int oracle_local_get_path(const oracle_local* L, double* wp, int max_wp);
int oracle_local_reconnecting_index(const oracle_local* L);
int oracle_local_planning(oracle_local* L, double x, double y, double z, double h,
                          const uint8_t* image, uint32_t width, uint32_t height,
                          uint32_t row_size, uint32_t pixel_size, double res);
int oracle_local_get_path_eval(oracle_local* L, double x, double y, double z, double h,
                               double* wp, int max_wp);
void oracle_local_risk_matrix(oracle_local* L, double x, double y, double* out);
void oracle_local_deviation_matrix(oracle_local* L, double x, double y, double* out);
uint64_t oracle_local_map_mask(const oracle_local* L, uint8_t* mask);
int oracle_local_block(const oracle_local* L, uint32_t gi, uint32_t gj, double* dev, double* tc,
                       double* risk, uint8_t* state, uint8_t* obst);

#ifdef __cplusplus
}
#endif
#endif
