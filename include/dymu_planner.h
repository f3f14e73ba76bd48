/*
 * dymu_planner.h -- flat C-ABI over PathPlanning_lib::DyMuPathPlanner
 * (include/DyMu.hpp) for non-C++ callers (ctypes, cgo, JNI).
 *
 * Each entry point forwards to the class method of the same name, which in
 * turn follows the reference method cited in DyMu.hpp.  Boolean methods
 * return 1 (true) / 0 (false); a negative value is a dymu_status error (for
 * example DYMU_ERR_NO_DEVICE when the HIP engine cannot run).  Grids are
 * row-major ny*nx doubles, index j*nx + i.  Waypoints are (x, y, z, heading).
 */
#ifndef DYMU_PLANNER_H
#define DYMU_PLANNER_H

#include <stdint.h>

#include "dymu_fim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dymu_planner dymu_planner;

/* DyMuPathPlanner(risk_distance, reconnect_distance, risk_ratio, approach)
 * (reference src/DyMu_GlobalPathPlanning.cpp:22-33); approach 0 CONSERVATIVE, 1 SWEEPING */
int dymu_planner_create(dymu_planner** out, double risk_distance, double reconnect_distance,
                        double risk_ratio, int approach);
void dymu_planner_destroy(dymu_planner* p);
int dymu_planner_set_engine_options(dymu_planner* p, const dymu_opts* opts);

/* initGlobalLayer (:39-104) */
int dymu_planner_init_global_layer(dymu_planner* p, double globalres, double localres,
                                   uint32_t nx, uint32_t ny, double offx, double offy);
/* setCostMap (:109-126); cost_map: ny*nx */
int dymu_planner_set_cost_map(dymu_planner* p, const double* cost_map, uint32_t nx, uint32_t ny);
/* computeCostMap (:145-181); loc_modes: n_locs C strings */
int dymu_planner_compute_cost_map(dymu_planner* p, const double* lut, int lut_len,
                                  const double* slopes, int n_slopes, const char* const* loc_modes,
                                  int n_locs, const double* elevation, const double* terrain);
/* setGoal (:322-357) */
int dymu_planner_set_goal(dymu_planner* p, double x, double y, double z, double heading);
/* computeTotalCostMap (:364-408) */
int dymu_planner_compute_total_cost_map(dymu_planner* p, double x, double y, double z,
                                        double heading);
/* computeEntireTotalCostMap (:443-468) */
int dymu_planner_compute_entire_total_cost_map(dymu_planner* p);

/* getTotalCostMatrix (:799-811, +inf -> -1), getGlobalCostMatrix (:815-829),
 * getHazardDensityMatrix (:833-842), getTrafficabilityMatrix (:846-855) */
int dymu_planner_get_total_cost_matrix(dymu_planner* p, double* out);
int dymu_planner_get_global_cost_matrix(dymu_planner* p, double* out);
int dymu_planner_get_hazard_density_matrix(dymu_planner* p, double* out);
int dymu_planner_get_trafficability_matrix(dymu_planner* p, double* out);
/* raw total cost (+inf unreachable), ny*nx */
int dymu_planner_get_total_cost_raw(dymu_planner* p, double* out);
/* getTotalCost(Waypoint) (:860-890) */
int dymu_planner_get_total_cost(dymu_planner* p, double x, double y, double z, double heading,
                                double* out);
/* getPath (:589-611): writes up to max_wp waypoints (x,y,z,heading); returns
 * the number of waypoints (>= 0) or a negative status */
int dymu_planner_get_path(dymu_planner* p, double x, double y, double z, double heading,
                          double* out_xyzh, int max_wp);
/* getLocomotionMode (:788-795) into buf (NUL-terminated) */
int dymu_planner_get_locomotion_mode(dymu_planner* p, double x, double y, double z, double heading,
                                     char* buf, int buflen);
/* dynamic feedback (extension): hazard_density / trafficability, ny*nx */
int dymu_planner_set_hazard_density(dymu_planner* p, const double* hd);
int dymu_planner_set_trafficability(dymu_planner* p, const double* tr);
/* windowed forms: w*h values (row-major) for cells [i0, i0+w) x [j0, j0+h) */
int dymu_planner_set_hazard_density_window(dymu_planner* p, uint32_t i0, uint32_t j0, uint32_t w,
                                           uint32_t h, const double* hd);
int dymu_planner_set_trafficability_window(dymu_planner* p, uint32_t i0, uint32_t j0, uint32_t w,
                                           uint32_t h, const double* tr);
/* narrow-band cells left by the last computeTotalCostMap's early exit (0 after
 * computeEntireTotalCostMap) */
int64_t dymu_planner_last_band_size(dymu_planner* p);
/* statistics of the last solve */
int dymu_planner_last_stats(dymu_planner* p, dymu_stats* out);
/* the last computeTotalCostMap's exit-order resolution: out[0] cells
 * of exactly the exit value, out[1] how many of them the reference had not closed,
 * out[2] 1 if the exact host replay ran (degenerate ties only), out[3] host ms,
 * out[4] reference updates the band replay evaluated, out[5] 1 if every band value
 * is the reference's (0: the replay hit its work bound) */
int dymu_planner_last_early_exit(dymu_planner* p, double out[6]);
/* the same, n values of: tied, open_at_limit, exact_replay, resolve_ms, replay_updates,
 * band_exact, near_ties (comparisons of engine values rounding could flip: any sends
 * the exit to the exact host replay), replay_threads (round 6) */
int dymu_planner_last_early_exit_ex(dymu_planner* p, double* out, uint32_t n);
/* how the last solve ran: 0 cold, 1 windowed re-propagation from the window
 * where the speed changed (dymu_resolve_window), 2 previous map reused */
int dymu_planner_last_solve_kind(dymu_planner* p);

/* ---- node-level access (src/DyMu.hpp:500-518, extension of the flat ABI) ---- */
typedef struct dymu_global_node {
  double elevation, slope, raw_cost, cost, hazard_density, trafficability, total_cost;
  uint32_t terrain;
  int32_t state;        /* 0 OPEN, 1 CLOSED */
  int32_t is_obstacle;
  int32_t has_local_map;
} dymu_global_node;
/* getGlobalNode (:313-317): 1 and *out, or 0 (NULL) */
int dymu_planner_get_global_node(dymu_planner* p, uint32_t i, uint32_t j, dymu_global_node* out);
int dymu_planner_is_safe_node(dymu_planner* p, uint32_t i, uint32_t j);          /* :410-422 */
int dymu_planner_is_fully_closed_node(dymu_planner* p, uint32_t i, uint32_t j);  /* :424-436 */
int dymu_planner_reset_total_cost_map(dymu_planner* p);                          /* :473-485 */
/* every node's state in bulk (ny*nx bytes, row-major: 1 CLOSED, 0 OPEN), as
 * dymu_planner_get_global_node reports it one node at a time */
int dymu_planner_get_node_states(dymu_planner* p, uint8_t* out);
/* global_narrowband (:445) as the last computeTotalCostMap left it: the band
 * size; up to max (i, j) pairs written to ij in the reference's insertion order */
int64_t dymu_planner_global_narrowband(dymu_planner* p, uint32_t* ij, int64_t max);
/* minCostGlobalNode (:548-567): 1, the band node of lowest total cost (removed
 * from the band list) in ij[2] and *total_cost; 0 on an empty band */
int dymu_planner_min_cost_global_node(dymu_planner* p, uint32_t* ij, double* total_cost);
int dymu_planner_reset_global_narrow_band(dymu_planner* p);                      /* :487-498 */
/* gradientNode (:718-772): the normalised descent direction at (i, j) in d[2] */
int dymu_planner_gradient_node(dymu_planner* p, uint32_t i, uint32_t j, double* d);
/* propagateGlobalNode (:500-546): the reference update of node (i, j) from its
 * nb4's current total costs on the host copy of the map; a node whose total cost
 * was +inf joins the band (appended) and global_propagated_nodes */
int dymu_planner_propagate_global_node(dymu_planner* p, uint32_t i, uint32_t j);
/* the public globalNode::state (0 OPEN, 1 CLOSED) written by a caller */
int dymu_planner_set_global_node_state(dymu_planner* p, uint32_t i, uint32_t j, int state);
/* global_propagated_nodes (:447): the count (max <= 0: cheap); up to max (i, j) pairs in
 * ij, in the reference's insertion order (DyMuPathPlanner::globalPropagatedIndices) --
 * rebuilt from the values, or from the exact host replay of the reference's FMM where
 * near ties leave it open (from ~2^22 reached nodes: ~34 s for the whole list at 16384^2) */
int64_t dymu_planner_global_propagated_nodes(dymu_planner* p, uint32_t* ij, int64_t max);
/* install a total-cost map (ny*nx, +inf unreachable) as a converged
 * computeEntireTotalCostMap leaves it (every finite node CLOSED) */
int dymu_planner_load_total_cost_map(dymu_planner* p, const double* T);
/* current_path (public member, src/DyMu.hpp:456): n waypoints (x, y, z, heading) */
int dymu_planner_set_current_path(dymu_planner* p, const double* xyzh, int n);
int dymu_planner_get_current_path(dymu_planner* p, double* out_xyzh, int max_wp);

/* ---- local layer (src/DyMu_LocalPathRepairing.cpp) ---- */
/* computeLocalPlanning (:193-291).  image: height rows of row_size bytes, pixel
 * (i, j) at image[j*row_size + i*pixel_size], nonzero = obstacle.  Returns 1
 * when the path was repaired (trajectory = current_path, *n_traj waypoints, at
 * most max_traj written; *local_time_s = repair time), 0 when not blocked. */
int dymu_planner_compute_local_planning(dymu_planner* p, double x, double y, double z,
                                        double heading, const uint8_t* image, uint32_t width,
                                        uint32_t height, uint32_t row_size, uint32_t pixel_size,
                                        double res, double* traj_xyzh, int max_traj,
                                        int* n_traj, double* local_time_s);
/* repairPath (:298-435): the reconnecting index or -1 */
int dymu_planner_repair_path(dymu_planner* p, double x, double y, double z, double heading,
                             uint32_t index);
/* evaluatePath (:1027-1109) */
int dymu_planner_evaluate_path(dymu_planner* p, uint32_t starting_index);
/* expandRisk (:493-523) */
int dymu_planner_expand_risk(dymu_planner* p);
/* computeLocalPropagation (:578-698): 1 and the set node's global pose, or 0 (NULL) */
int dymu_planner_compute_local_propagation(dymu_planner* p, const double* start_xyzh,
                                           const double* overtake_xyzh, double* set_xy);
/* computeLocalWaypointDijkstra (L:851-869) from the sub-cell at waypoint xyzh
 * (getLocalNode: subdivides): 1 and the step's (x, y, z, heading), 0 (NULL) */
int dymu_planner_local_waypoint_dijkstra(dymu_planner* p, const double* xyzh, double* out_xyzh);
/* local_agent (src/DyMu.hpp:460): 1 and its global pose (x, y), or 0 (NULL) */
int dymu_planner_local_agent(dymu_planner* p, double* global_xy);
/* computeLocalPropagation's wall-clock limit (the reference's 5 s, :685-696;
 * <= 0 disables it); it then returns 0 (NULL) like the reference */
int dymu_planner_set_local_timeout(dymu_planner* p, double seconds);
/* getRiskMatrix / getDeviationMatrix (:1111-1211): (21*r)^2 doubles, r = res ratio */
int dymu_planner_get_risk_matrix(dymu_planner* p, double x, double y, double z, double heading,
                                 double* out);
int dymu_planner_get_deviation_matrix(dymu_planner* p, double x, double y, double z,
                                      double heading, double* out);
int dymu_planner_get_reconnecting_index(dymu_planner* p);
int dymu_planner_res_ratio(dymu_planner* p);
/* subdivided global nodes: count, and a ny*nx byte mask (may be NULL) */
int64_t dymu_planner_local_map_mask(dymu_planner* p, uint8_t* mask);
/* a local-layer sub-cell (the reference's localNode, src/DyMu.hpp:42-67); id names
 * it for the calls below (stable while the local map lives) */
typedef struct dymu_local_node {
  double global_x, global_y;  /* global_pose (global units) */
  double deviation, total_cost, risk;
  uint32_t parent_i, parent_j; /* the subdivided global node */
  uint32_t li, lj;             /* the sub-cell inside it */
  int32_t state, is_obstacle;  /* 0 OPEN / 1 CLOSED; 0 / 1 */
  uint64_t id;
} dymu_local_node;
/* getLocalNode(Waypoint) (L:177-189; subdivides): 1 and *out, or 0 (NULL) */
int dymu_planner_get_local_node(dymu_planner* p, double x, double y, dymu_local_node* out);
/* localNode::nb4List[d] of sub-cell id (d: 0 (i,j-1), 1 (i-1,j), 2 (i+1,j),
 * 3 (i,j+1)): 1 and *out, or 0 (NULL) */
int dymu_planner_local_neighbour(dymu_planner* p, uint64_t id, int d, dymu_local_node* out);
/* maxRiskNode (L:525-548): 1 and the popped node, or 0 (empty queue: NULL) */
int dymu_planner_max_risk_node(dymu_planner* p, dymu_local_node* out);
/* propagateRisk (L:550-576) / propagateLocalNode (L:700-750) on sub-cell id */
int dymu_planner_propagate_risk(dymu_planner* p, uint64_t id);
int dymu_planner_propagate_local_node(dymu_planner* p, uint64_t id);
/* the public localNode::state (0 OPEN, 1 CLOSED) written by a caller */
int dymu_planner_set_local_node_state(dymu_planner* p, uint64_t id, int state);
/* minCostLocalNode(Tovertake, minC) (L:752-775) / minCostLocalNode(reachNode)
 * (L:777-805): 1 and the popped band node, or 0 (empty band) */
int dymu_planner_min_cost_local_node(dymu_planner* p, double Tovertake, double minC,
                                     dymu_local_node* out);
int dymu_planner_min_cost_local_node_reach(dymu_planner* p, uint64_t reach_id,
                                           dymu_local_node* out);
/* the public local lists (src/DyMu.hpp:448-454): which = 0 local_narrowband, 1
 * local_expandable_obstacles, 2 local_propagated_nodes; the count, up to max
 * written to out in the list's order */
int64_t dymu_planner_local_list(dymu_planner* p, int which, dymu_local_node* out, int64_t max);
/* one subdivided node's r*r sub-cells ([j][i]); 0 if (i, j) has no local map */
int dymu_planner_local_block(dymu_planner* p, uint32_t i, uint32_t j, double* dev, double* tc,
                             double* risk, uint8_t* state, uint8_t* obst);

#ifdef __cplusplus
}
#endif
#endif
