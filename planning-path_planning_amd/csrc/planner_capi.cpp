// planner_capi.cpp -- extern "C" forwarding layer (include/dymu_planner.h)
// over PathPlanning_lib::DyMuPathPlanner.  Exceptions never cross the ABI:
// an engine failure becomes DYMU_ERR_NO_DEVICE / DYMU_ERR_HIP.
#include <cstring>
#include <exception>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "DyMu.hpp"
#include "dymu_planner.h"

using PathPlanning_lib::DyMuPathPlanner;
using PathPlanning_lib::localNode;
using PathPlanning_lib::CLOSED;
using PathPlanning_lib::OPEN;

struct dymu_planner {
  DyMuPathPlanner pl;
  dymu_planner(double a, double b, double c, PathPlanning_lib::repairingAproach r)
      : pl(a, b, c, r) {}
};

namespace {

base::Waypoint wp(double x, double y, double z, double h) {
  base::Waypoint w;
  w.position[0] = x;
  w.position[1] = y;
  w.position[2] = z;
  w.heading = h;
  return w;
}

int engine_error(const std::exception& e) {
  const std::string m = e.what();
  return m.find("cannot create") != std::string::npos ? DYMU_ERR_NO_DEVICE : DYMU_ERR_HIP;
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return DYMU_ERR_NOMEM;
  } catch (const std::exception& e) {
    return engine_error(e);
  }
}

std::vector<std::vector<double>> to_rows(const double* a, unsigned nx, unsigned ny) {
  std::vector<std::vector<double>> m(ny, std::vector<double>(nx));
  for (unsigned j = 0; j < ny; ++j) std::memcpy(m[j].data(), a + (size_t)j * nx, sizeof(double) * nx);
  return m;
}

void from_rows(const std::vector<std::vector<double>>& m, double* out) {
  size_t off = 0;
  for (const auto& r : m) {
    std::memcpy(out + off, r.data(), sizeof(double) * r.size());
    off += r.size();
  }
}

}  // namespace

extern "C" {

int dymu_planner_create(dymu_planner** out, double risk_distance, double reconnect_distance,
                        double risk_ratio, int approach) {
  if (!out) return DYMU_ERR_ARG;
  return guarded([&] {
    *out = new dymu_planner(risk_distance, reconnect_distance, risk_ratio,
                            approach == 1 ? PathPlanning_lib::SWEEPING
                                          : PathPlanning_lib::CONSERVATIVE);
    return DYMU_OK;
  });
}

void dymu_planner_destroy(dymu_planner* p) { delete p; }

int dymu_planner_set_engine_options(dymu_planner* p, const dymu_opts* o) {
  if (!p || !o) return DYMU_ERR_ARG;
  p->pl.setEngineOptions(*o);
  return DYMU_OK;
}

int dymu_planner_init_global_layer(dymu_planner* p, double globalres, double localres,
                                   uint32_t nx, uint32_t ny, double offx, double offy) {
  if (!p || nx == 0 || ny == 0) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.initGlobalLayer(globalres, localres, nx, ny, {offx, offy}); });
}

int dymu_planner_set_cost_map(dymu_planner* p, const double* cost_map, uint32_t nx, uint32_t ny) {
  if (!p || !cost_map) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.setCostMap(to_rows(cost_map, nx, ny)); });
}

int dymu_planner_compute_cost_map(dymu_planner* p, const double* lut, int lut_len,
                                  const double* slopes, int n_slopes, const char* const* loc_modes,
                                  int n_locs, const double* elevation, const double* terrain) {
  if (!p || !lut || !slopes || !loc_modes || !elevation || !terrain || lut_len <= 0 ||
      n_slopes <= 0 || n_locs <= 0)
    return DYMU_ERR_ARG;
  return guarded([&] {
    std::vector<std::string> modes;
    for (int k = 0; k < n_locs; ++k) modes.emplace_back(loc_modes[k] ? loc_modes[k] : "");
    return (int)p->pl.computeCostMap(std::vector<double>(lut, lut + lut_len),
                                     std::vector<double>(slopes, slopes + n_slopes), modes,
                                     elevation, terrain);
  });
}

int dymu_planner_set_goal(dymu_planner* p, double x, double y, double z, double h) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.setGoal(wp(x, y, z, h)); });
}

int dymu_planner_compute_total_cost_map(dymu_planner* p, double x, double y, double z, double h) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.computeTotalCostMap(wp(x, y, z, h)); });
}

int dymu_planner_compute_entire_total_cost_map(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.computeEntireTotalCostMap(); });
}

int dymu_planner_get_total_cost_matrix(dymu_planner* p, double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { p->pl.copyTotalCost(out, false); return DYMU_OK; });
}

int dymu_planner_get_global_cost_matrix(dymu_planner* p, double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { from_rows(p->pl.getGlobalCostMatrix(), out); return DYMU_OK; });
}

int dymu_planner_get_hazard_density_matrix(dymu_planner* p, double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { from_rows(p->pl.getHazardDensityMatrix(), out); return DYMU_OK; });
}

int dymu_planner_get_trafficability_matrix(dymu_planner* p, double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { from_rows(p->pl.getTrafficabilityMatrix(), out); return DYMU_OK; });
}

int dymu_planner_get_total_cost_raw(dymu_planner* p, double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { p->pl.copyTotalCost(out, true); return DYMU_OK; });
}

int dymu_planner_get_total_cost(dymu_planner* p, double x, double y, double z, double h,
                                double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { *out = p->pl.getTotalCost(wp(x, y, z, h)); return DYMU_OK; });
}

int dymu_planner_get_path(dymu_planner* p, double x, double y, double z, double h,
                          double* out, int max_wp) {
  if (!p || !out || max_wp < 0) return DYMU_ERR_ARG;
  return guarded([&] {
    const std::vector<base::Waypoint> path = p->pl.getPath(wp(x, y, z, h));
    const int n = (int)path.size();
    for (int k = 0; k < n && k < max_wp; ++k) {
      out[4 * k + 0] = path[k].position[0];
      out[4 * k + 1] = path[k].position[1];
      out[4 * k + 2] = path[k].position[2];
      out[4 * k + 3] = path[k].heading;
    }
    return n;
  });
}

int dymu_planner_get_locomotion_mode(dymu_planner* p, double x, double y, double z, double h,
                                     char* buf, int buflen) {
  if (!p || !buf || buflen <= 0) return DYMU_ERR_ARG;
  return guarded([&] {
    const std::string m = p->pl.getLocomotionMode(wp(x, y, z, h));
    std::strncpy(buf, m.c_str(), (size_t)buflen - 1);
    buf[buflen - 1] = '\0';
    return (int)m.size();
  });
}

int dymu_planner_set_hazard_density(dymu_planner* p, const double* hd) {
  if (!p || !hd) return DYMU_ERR_ARG;
  const size_t n = (size_t)p->pl.sizeX() * p->pl.sizeY();
  return guarded([&] { return (int)p->pl.setHazardDensity(std::vector<double>(hd, hd + n)); });
}

int dymu_planner_set_trafficability(dymu_planner* p, const double* tr) {
  if (!p || !tr) return DYMU_ERR_ARG;
  const size_t n = (size_t)p->pl.sizeX() * p->pl.sizeY();
  return guarded([&] { return (int)p->pl.setTrafficability(std::vector<double>(tr, tr + n)); });
}

int dymu_planner_last_stats(dymu_planner* p, dymu_stats* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  *out = p->pl.lastStats();
  return DYMU_OK;
}

int dymu_planner_last_early_exit(dymu_planner* p, double out[6]) {
  if (!p || !out) return DYMU_ERR_ARG;
  const auto& e = p->pl.lastEarlyExitInfo();
  out[0] = (double)e.tied;
  out[1] = (double)e.open_at_limit;
  out[2] = (double)e.exact_replay;
  out[3] = e.resolve_ms;
  out[4] = (double)e.replay_updates;
  out[5] = (double)e.band_exact;
  return DYMU_OK;
}

int dymu_planner_last_early_exit_ex(dymu_planner* p, double* out, uint32_t n) {
  if (!p || (n && !out)) return DYMU_ERR_ARG;
  const auto& e = p->pl.lastEarlyExitInfo();
  const double v[8] = {(double)e.tied,           (double)e.open_at_limit, (double)e.exact_replay,
                       e.resolve_ms,             (double)e.replay_updates, (double)e.band_exact,
                       (double)e.near_ties,      (double)e.replay_threads};
  for (uint32_t q = 0; q < n && q < 8; ++q) out[q] = v[q];
  return DYMU_OK;
}

int dymu_planner_last_solve_kind(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return p->pl.lastSolveKind();
}

int dymu_planner_set_hazard_density_window(dymu_planner* p, uint32_t i0, uint32_t j0, uint32_t w,
                                           uint32_t h, const double* hd) {
  if (!p || !hd) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.setHazardDensityWindow(i0, j0, w, h, hd); });
}

int dymu_planner_set_trafficability_window(dymu_planner* p, uint32_t i0, uint32_t j0, uint32_t w,
                                           uint32_t h, const double* tr) {
  if (!p || !tr) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.setTrafficabilityWindow(i0, j0, w, h, tr); });
}

int64_t dymu_planner_last_band_size(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return (int64_t)p->pl.lastBandSize();
}

int dymu_planner_get_global_node(dymu_planner* p, uint32_t i, uint32_t j, dymu_global_node* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.getGlobalNode(i, j);
    if (!n) return 0;
    out->elevation = n->elevation;
    out->slope = n->slope;
    out->raw_cost = n->raw_cost;
    out->cost = n->cost;
    out->hazard_density = n->hazard_density;
    out->trafficability = n->trafficability;
    out->total_cost = n->total_cost;
    out->terrain = n->terrain;
    out->state = n->state == PathPlanning_lib::CLOSED ? 1 : 0;
    out->is_obstacle = n->isObstacle ? 1 : 0;
    out->has_local_map = n->hasLocalMap ? 1 : 0;
    return 1;
  });
}

int dymu_planner_is_safe_node(dymu_planner* p, uint32_t i, uint32_t j) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.isSafeNode(i, j); });
}

int dymu_planner_is_fully_closed_node(dymu_planner* p, uint32_t i, uint32_t j) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.isFullyClosedNode(i, j); });
}

int64_t dymu_planner_global_narrowband(dymu_planner* p, uint32_t* ij, int64_t max) {
  if (!p || (max > 0 && !ij)) return DYMU_ERR_ARG;
  int64_t n = 0;
  const int rc = guarded([&] {
    const auto band = p->pl.globalNarrowband();
    n = (int64_t)band.size();
    for (int64_t q = 0; q < n && q < max; ++q) {
      ij[2 * q] = (uint32_t)band[q].pose.position[0];
      ij[2 * q + 1] = (uint32_t)band[q].pose.position[1];
    }
    return DYMU_OK;
  });
  return rc < 0 ? rc : n;
}

int dymu_planner_min_cost_global_node(dymu_planner* p, uint32_t* ij, double* total_cost) {
  if (!p || !ij) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.minCostGlobalNode();
    if (!n) return 0;
    ij[0] = (uint32_t)n->pose.position[0];
    ij[1] = (uint32_t)n->pose.position[1];
    if (total_cost) *total_cost = n->total_cost;
    return 1;
  });
}

int dymu_planner_reset_global_narrow_band(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { p->pl.resetGlobalNarrowBand(); return DYMU_OK; });
}

int dymu_planner_gradient_node(dymu_planner* p, uint32_t i, uint32_t j, double* d) {
  if (!p || !d) return DYMU_ERR_ARG;
  return guarded([&] {
    if (i >= p->pl.sizeX() || j >= p->pl.sizeY()) return (int)DYMU_ERR_ARG;
    p->pl.gradientNode(i, j, d[0], d[1]);
    return (int)DYMU_OK;
  });
}

int dymu_planner_propagate_global_node(dymu_planner* p, uint32_t i, uint32_t j) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] {
    if (i >= p->pl.sizeX() || j >= p->pl.sizeY()) return (int)DYMU_ERR_ARG;
    p->pl.propagateGlobalNode(i, j);
    return (int)DYMU_OK;
  });
}

int dymu_planner_set_global_node_state(dymu_planner* p, uint32_t i, uint32_t j, int state) {
  if (!p || (state != 0 && state != 1)) return DYMU_ERR_ARG;
  return guarded([&] {
    if (i >= p->pl.sizeX() || j >= p->pl.sizeY()) return (int)DYMU_ERR_ARG;
    p->pl.setGlobalNodeState(i, j, state ? CLOSED : OPEN);
    return (int)DYMU_OK;
  });
}

int64_t dymu_planner_global_propagated_nodes(dymu_planner* p, uint32_t* ij, int64_t max) {
  if (!p || (max > 0 && !ij)) return DYMU_ERR_ARG;
  int64_t n = 0;
  const int rc = guarded([&] {
    if (max <= 0) {
      n = (int64_t)p->pl.globalPropagatedCount();
      return DYMU_OK;
    }
    const std::vector<uint64_t> ks = p->pl.globalPropagatedIndices();
    const uint64_t nx = p->pl.sizeX();
    n = (int64_t)ks.size();
    for (int64_t q = 0; q < n && q < max; ++q) {
      ij[2 * q] = (uint32_t)(ks[q] % nx);
      ij[2 * q + 1] = (uint32_t)(ks[q] / nx);
    }
    return DYMU_OK;
  });
  return rc < 0 ? rc : n;
}

int dymu_planner_get_node_states(dymu_planner* p, uint8_t* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    p->pl.copyNodeStates(out);
    return (int)DYMU_OK;
  });
}

int dymu_planner_reset_total_cost_map(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  p->pl.resetTotalCostMap();
  return DYMU_OK;
}

int dymu_planner_load_total_cost_map(dymu_planner* p, const double* T) {
  if (!p || !T) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.loadTotalCostMap(T); });
}

int dymu_planner_set_current_path(dymu_planner* p, const double* xyzh, int n) {
  if (!p || n < 0 || (n > 0 && !xyzh)) return DYMU_ERR_ARG;
  return guarded([&] {
    p->pl.current_path.clear();
    for (int k = 0; k < n; ++k)
      p->pl.current_path.push_back(wp(xyzh[4 * k], xyzh[4 * k + 1], xyzh[4 * k + 2], xyzh[4 * k + 3]));
    return DYMU_OK;
  });
}

namespace {
int put_path(const std::vector<base::Waypoint>& path, double* out, int max_wp) {
  const int n = (int)path.size();
  for (int k = 0; k < n && k < max_wp; ++k) {
    out[4 * k + 0] = path[k].position[0];
    out[4 * k + 1] = path[k].position[1];
    out[4 * k + 2] = path[k].position[2];
    out[4 * k + 3] = path[k].heading;
  }
  return n;
}
}  // namespace

int dymu_planner_get_current_path(dymu_planner* p, double* out, int max_wp) {
  if (!p || !out || max_wp < 0) return DYMU_ERR_ARG;
  return put_path(p->pl.current_path, out, max_wp);
}

int dymu_planner_compute_local_planning(dymu_planner* p, double x, double y, double z, double h,
                                        const uint8_t* image, uint32_t width, uint32_t height,
                                        uint32_t row_size, uint32_t pixel_size, double res,
                                        double* traj, int max_traj, int* n_traj,
                                        double* local_time_s) {
  if (!p || (!image && width && height) || max_traj < 0 || (max_traj > 0 && !traj) ||
      (height > 0 && width > 0 && (uint64_t)(height - 1) * row_size + (uint64_t)(width - 1) * pixel_size >= (uint64_t)height * row_size))
    return DYMU_ERR_ARG;
  return guarded([&] {
    base::samples::frame::Frame f;
    f.width = width;
    f.height = height;
    f.row_size = row_size;
    f.pixel_size = pixel_size;
    f.image.assign(image, image + (size_t)height * row_size);
    std::vector<base::Waypoint> trajectory;
    base::Time t;
    const bool r = p->pl.computeLocalPlanning(wp(x, y, z, h), f, res, trajectory, t);
    if (r) {
      const int n = put_path(trajectory, traj, max_traj);
      if (n_traj) *n_traj = n;
      if (local_time_s) *local_time_s = t.toSeconds();
    } else if (n_traj) {
      *n_traj = 0;
    }
    return (int)r;
  });
}

int dymu_planner_repair_path(dymu_planner* p, double x, double y, double z, double h,
                             uint32_t index) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return p->pl.repairPath(wp(x, y, z, h), index); });
}

int dymu_planner_evaluate_path(dymu_planner* p, uint32_t starting_index) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { return (int)p->pl.evaluatePath(starting_index); });
}

int dymu_planner_expand_risk(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { p->pl.expandRisk(); return DYMU_OK; });
}

int dymu_planner_set_local_timeout(dymu_planner* p, double seconds) {
  if (!p) return DYMU_ERR_ARG;
  p->pl.setLocalPropagationTimeout(seconds);
  return DYMU_OK;
}

int dymu_planner_local_waypoint_dijkstra(dymu_planner* p, const double* s, double* out) {
  if (!p || !s || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.getLocalNode(wp(s[0], s[1], s[2], s[3]));
    if (!n) return 0;
    const base::Waypoint w = p->pl.computeLocalWaypointDijkstra(*n);
    out[0] = w.position[0];
    out[1] = w.position[1];
    out[2] = w.position[2];
    out[3] = w.heading;
    return 1;
  });
}

int dymu_planner_local_agent(dymu_planner* p, double* xy) {
  if (!p || !xy) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.localAgent();
    if (!n) return 0;
    xy[0] = n->global_pose.position[0];
    xy[1] = n->global_pose.position[1];
    return 1;
  });
}

namespace {
void flat_local(const localNode& n, dymu_local_node* out) {
  out->global_x = n.global_pose.position[0];
  out->global_y = n.global_pose.position[1];
  out->deviation = n.deviation;
  out->total_cost = n.total_cost;
  out->risk = n.risk;
  out->parent_i = (uint32_t)n.parent_pose.position[0];
  out->parent_j = (uint32_t)n.parent_pose.position[1];
  out->li = (uint32_t)n.pose.position[0];
  out->lj = (uint32_t)n.pose.position[1];
  out->state = n.state == CLOSED ? 1 : 0;
  out->is_obstacle = n.isObstacle ? 1 : 0;
  out->id = n.id;
}
localNode by_id(uint64_t id) {
  localNode n;
  n.id = id;
  return n;
}
}  // namespace

int dymu_planner_get_local_node(dymu_planner* p, double x, double y, dymu_local_node* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.getLocalNode(wp(x, y, 0.0, 0.0));
    if (!n) return 0;
    flat_local(*n, out);
    return 1;
  });
}

int dymu_planner_local_neighbour(dymu_planner* p, uint64_t id, int d, dymu_local_node* out) {
  if (!p || !out || d < 0 || d > 3) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.localNeighbour(by_id(id), d);
    if (!n) return 0;
    flat_local(*n, out);
    return 1;
  });
}

int dymu_planner_max_risk_node(dymu_planner* p, dymu_local_node* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.maxRiskNode();
    if (!n) return 0;
    flat_local(*n, out);
    return 1;
  });
}

int dymu_planner_propagate_risk(dymu_planner* p, uint64_t id) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { p->pl.propagateRisk(by_id(id)); return (int)DYMU_OK; });
}

int dymu_planner_propagate_local_node(dymu_planner* p, uint64_t id) {
  if (!p) return DYMU_ERR_ARG;
  return guarded([&] { p->pl.propagateLocalNode(by_id(id)); return (int)DYMU_OK; });
}

int dymu_planner_set_local_node_state(dymu_planner* p, uint64_t id, int state) {
  if (!p || (state != 0 && state != 1)) return DYMU_ERR_ARG;
  return guarded([&] {
    p->pl.setLocalNodeState(by_id(id), state ? CLOSED : OPEN);
    return (int)DYMU_OK;
  });
}

int dymu_planner_min_cost_local_node(dymu_planner* p, double Tovertake, double minC,
                                     dymu_local_node* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.minCostLocalNode(Tovertake, minC);
    if (!n) return 0;
    flat_local(*n, out);
    return 1;
  });
}

int dymu_planner_min_cost_local_node_reach(dymu_planner* p, uint64_t reach_id,
                                           dymu_local_node* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.minCostLocalNode(by_id(reach_id));
    if (!n) return 0;
    flat_local(*n, out);
    return 1;
  });
}

int64_t dymu_planner_local_list(dymu_planner* p, int which, dymu_local_node* out, int64_t max) {
  if (!p || which < 0 || which > 2 || (max > 0 && !out)) return DYMU_ERR_ARG;
  int64_t n = 0;
  const int rc = guarded([&] {
    const auto v = which == 0   ? p->pl.localNarrowband()
                   : which == 1 ? p->pl.localExpandableObstacles()
                                : p->pl.localPropagatedNodes();
    n = (int64_t)v.size();
    for (int64_t q = 0; q < n && q < max; ++q) flat_local(v[q], &out[q]);
    return DYMU_OK;
  });
  return rc < 0 ? rc : n;
}

int dymu_planner_compute_local_propagation(dymu_planner* p, const double* s, const double* o,
                                           double* set_xy) {
  if (!p || !s || !o) return DYMU_ERR_ARG;
  return guarded([&] {
    const auto n = p->pl.computeLocalPropagation(wp(s[0], s[1], s[2], s[3]), wp(o[0], o[1], o[2], o[3]));
    if (!n) return 0;
    if (set_xy) {
      set_xy[0] = n->global_pose.position[0];
      set_xy[1] = n->global_pose.position[1];
    }
    return 1;
  });
}

int dymu_planner_get_risk_matrix(dymu_planner* p, double x, double y, double z, double h,
                                 double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { from_rows(p->pl.getRiskMatrix(wp(x, y, z, h)), out); return DYMU_OK; });
}

int dymu_planner_get_deviation_matrix(dymu_planner* p, double x, double y, double z, double h,
                                      double* out) {
  if (!p || !out) return DYMU_ERR_ARG;
  return guarded([&] { from_rows(p->pl.getDeviationMatrix(wp(x, y, z, h)), out); return DYMU_OK; });
}

int dymu_planner_get_reconnecting_index(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return p->pl.getReconnectingIndex();
}

int dymu_planner_res_ratio(dymu_planner* p) {
  if (!p) return DYMU_ERR_ARG;
  return (int)p->pl.resRatio();
}

int64_t dymu_planner_local_map_mask(dymu_planner* p, uint8_t* mask) {
  if (!p) return DYMU_ERR_ARG;
  return (int64_t)p->pl.localMapMask(mask);
}

int dymu_planner_local_block(dymu_planner* p, uint32_t i, uint32_t j, double* dev, double* tc,
                             double* risk, uint8_t* state, uint8_t* obst) {
  if (!p) return DYMU_ERR_ARG;
  return (int)p->pl.localBlock(i, j, dev, tc, risk, state, obst);
}

}  // extern "C"
