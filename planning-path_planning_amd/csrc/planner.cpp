// planner.cpp -- PathPlanning_lib::DyMuPathPlanner over SoA arrays (DyMu.hpp).
//
// Host C++ around the MI355X engine: cost-map ingestion, goal validation and
// path extraction run on the host exactly as the reference computes them
// (compiled with -ffp-contract=off so each operation rounds where the
// reference's does); the total-cost propagation -- the reference's FMM loop
// -- is one dymu_solve() call on the GPU.
#include <algorithm>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <limits>
#include <stdexcept>
#include <string>

#include "DyMu.hpp"

namespace PathPlanning_lib {

namespace {
constexpr double kInf = std::numeric_limits<double>::infinity();

void log_warn(const char* m) { std::fprintf(stderr, "[dymu] WARN: %s\n", m); }
void log_error(const char* m) { std::fprintf(stderr, "[dymu] ERROR: %s\n", m); }
}  // namespace

DyMuPathPlanner::DyMuPathPlanner(double risk_distance, double reconnect_distance,
                                 double risk_ratio, repairingAproach input_approach)
    : risk_distance_(risk_distance),
      reconnect_distance_(reconnect_distance),
      risk_ratio_(risk_ratio),
      repairing_approach_(input_approach) {}

DyMuPathPlanner::~DyMuPathPlanner() {
  if (ctx_) dymu_destroy(ctx_);
}

void DyMuPathPlanner::setEngineOptions(const dymu_opts& o) {
  opts_ = o;
  if (ctx_) {
    dymu_destroy(ctx_);
    ctx_ = nullptr;
  }
}

// :39-104.  Node fields start as the globalNode constructor sets them
// (src/DyMu.hpp:88-107): cost 0, raw_cost 0, hazard 0, traff 1, T = +inf,
// OPEN, not an obstacle, locomotion "DONT_CARE".  Neighbour lists are implicit
// in the row-major layout.
bool DyMuPathPlanner::initGlobalLayer(double globalres, double localres, unsigned num_nodes_X,
                                      unsigned num_nodes_Y, std::vector<double> offset) {
  global_res_ = globalres;
  local_res_ = localres;
  solved_ = false;
  nx_ = num_nodes_X;
  ny_ = num_nodes_Y;
  global_offset_ = offset;
  if (global_offset_.size() < 2) global_offset_.resize(2, 0.0);
  const uint64_t n = (uint64_t)nx_ * ny_;
  elevation_.assign(n, 0.0);
  slope_.assign(n, 0.0);
  raw_cost_.assign(n, 0.0);
  cost_.assign(n, 0.0);
  hazard_.assign(n, 0.0);
  traff_.assign(n, 1.0);
  total_cost_.assign(n, kInf);
  terrain_.assign(n, 0u);
  is_obstacle_.assign(n, 0);
  state_.assign(n, OPEN);
  loc_mode_.assign(n, -1);
  has_goal_ = false;
  current_path.clear();
  return true;
}

// :109-126
bool DyMuPathPlanner::setCostMap(std::vector<std::vector<double>> cost_map) {
  if (cost_map.size() != ny_ || cost_map.empty() || cost_map[0].size() != nx_) return false;
  for (unsigned j = 0; j < ny_; ++j) {
    if (cost_map[j].size() != nx_) return false;
    for (unsigned i = 0; i < nx_; ++i) {
      const double c = cost_map[j][i];
      const uint64_t k = idx(i, j);
      cost_[k] = c;
      if (c <= 0) {
        is_obstacle_[k] = 1;
        traff_[k] = 0.0;
        hazard_[k] = 1.0;
      }
    }
  }
  return true;
}

// :145-181, with :186-210 (slope), :217-293 (nominal cost) and :297-308
// (smoothing).  Quirks kept: Q1 smoothing starts from the previous cost; Q2
// locomotion mode 0 skipped when several modes exist; Q3 the neighbour
// "Cmax" loops never run; Q4 LUT indexing differs between range==1 and >1.
bool DyMuPathPlanner::computeCostMap(std::vector<double> cost_data,
                                     std::vector<double> slope_values,
                                     std::vector<std::string> locomotionModes,
                                     std::vector<std::vector<double>> elevation,
                                     std::vector<std::vector<double>> terrainMap) {
  cost_lutable = cost_data;
  slope_range_ = slope_values;
  locomotion_modes_ = locomotionModes;
  if (cost_lutable.empty() || slope_range_.empty() || locomotion_modes_.empty()) return false;
  if (elevation.size() != ny_ || terrainMap.size() != ny_) return false;
  const int range = (int)slope_range_.size();
  const int num_locs = (int)locomotion_modes_.size();
  const double cmax = *std::max_element(cost_lutable.begin(), cost_lutable.end());

  for (unsigned j = 0; j < ny_; ++j) {
    if (elevation[j].size() != nx_ || terrainMap[j].size() != nx_) return false;
    for (unsigned i = 0; i < nx_; ++i) {
      const uint64_t k = idx(i, j);
      raw_cost_[k] = 0;
      elevation_[k] = elevation[j][i];
      terrain_[k] = (i == 0 || j == 0 || i == nx_ - 1 || j == ny_ - 1)
                        ? 0u
                        : (uint32_t)terrainMap[j][i];
    }
  }
  for (unsigned j = 0; j < ny_; ++j) {
    for (unsigned i = 0; i < nx_; ++i) {
      const uint64_t k = idx(i, j);
      // calculateSlope (:186-210)
      double dx, dy;
      if (i == 0)
        dx = (elevation_[k + 1] - elevation_[k]) / global_res_;
      else if (i == nx_ - 1)
        dx = (elevation_[k] - elevation_[k - 1]) / global_res_;
      else
        dx = (elevation_[k + 1] - elevation_[k - 1]) * 0.5 / global_res_;
      if (j == 0)
        dy = (elevation_[k + nx_] - elevation_[k]) / global_res_;
      else if (j == ny_ - 1)
        dy = (elevation_[k] - elevation_[k - nx_]) / global_res_;
      else
        dy = (elevation_[k + nx_] - elevation_[k - nx_]) * 0.5 / global_res_;
      slope_[k] = std::atan(std::sqrt(dx * dx + dy * dy));

      // calculateNominalCost (:217-293)
      const uint32_t t = terrain_[k];
      if (t == 0) {
        raw_cost_[k] = cmax;
        is_obstacle_[k] = 1;
      } else if (range == 1) {
        double cdef = cost_lutable[t * num_locs];
        for (int m = 0; m < num_locs; ++m) cdef = std::min(cdef, cost_lutable[t * num_locs + m]);
        raw_cost_[k] = std::max(raw_cost_[k], cdef);
      } else {
        const double si = slope_[k] * 180 / M_PI / (slope_range_.back() - slope_range_.front()) *
                          (double)(slope_range_.size() - 1);
        if (si > (double)(slope_range_.size() - 1)) {
          raw_cost_[k] = cmax;
          is_obstacle_[k] = 1;
        } else {
          const double smin = std::floor(si), smax = std::ceil(si);
          double cdef = cmax;
          if (num_locs > 1) {
            for (int m = 1; m < num_locs; ++m) {
              const double c1 = cost_lutable[t * range * num_locs + m * range + (int)smin];
              const double c2 = cost_lutable[t * range * num_locs + m * range + (int)smax];
              const double cc = c1 + (c2 - c1) * (si - smin);
              if (cc < cdef) {
                cdef = cc;
                raw_cost_[k] = std::max(raw_cost_[k], cdef);
                loc_mode_[k] = m;
              }
            }
          } else {
            const double c1 = cost_lutable[t * range + (int)smin];
            const double c2 = cost_lutable[t * range + (int)smax];
            cdef = c1 + (c2 - c1) * (si - smin);
            raw_cost_[k] = std::max(raw_cost_[k], cdef);
            loc_mode_[k] = 0;
          }
        }
      }
      if (is_obstacle_[k]) {
        traff_[k] = 0.0;
        hazard_[k] = 1.0;
      }
    }
  }
  // smoothCost (:297-308): own previous cost + neighbours' raw_cost
  for (unsigned j = 0; j < ny_; ++j)
    for (unsigned i = 0; i < nx_; ++i) {
      const uint64_t k = idx(i, j);
      double csum = cost_[k], n = 5;
      if (j == 0) n--; else csum += raw_cost_[k - nx_];
      if (i == 0) n--; else csum += raw_cost_[k - 1];
      if (i == nx_ - 1) n--; else csum += raw_cost_[k + 1];
      if (j == ny_ - 1) n--; else csum += raw_cost_[k + nx_];
      cost_[k] = csum / n;
    }
  return true;
}

// :322-357
bool DyMuPathPlanner::setGoal(base::Waypoint wGoal) {
  const double px = (wGoal.position[0] - global_offset_[0]) / global_res_;
  const double py = (wGoal.position[1] - global_offset_[1]) / global_res_;
  if (px < 0 || py < 0) return false;
  const unsigned i = (unsigned)(px + 0.5), j = (unsigned)(py + 0.5);
  if (i >= nx_ || j >= ny_) return false;
  if (i == 0 || j == 0 || i + 1 >= nx_ || j + 1 >= ny_) return false;  // an nb4 is NULL
  const uint64_t k = idx(i, j);
  if (is_obstacle_[k] || is_obstacle_[k - nx_] || is_obstacle_[k - 1] || is_obstacle_[k + 1] ||
      is_obstacle_[k + nx_])
    return false;
  has_goal_ = true;
  goal_i_ = i;
  goal_j_ = j;
  goal_heading_ = wGoal.heading;
  return true;
}

bool DyMuPathPlanner::setHazardDensity(const std::vector<double>& hd) {
  if (hd.size() != hazard_.size()) return false;
  hazard_ = hd;
  return true;
}

bool DyMuPathPlanner::setTrafficability(const std::vector<double>& tr) {
  if (tr.size() != traff_.size()) return false;
  traff_ = tr;
  return true;
}

// The engine call: F = global_res * cost * (2 + hazard - traff) (:527-528),
// +inf for obstacles; T and node states come back for every cell.
// Incremental path: when the previous solve on this engine was
// of the same grid and goal and the speed changed only inside a window (the
// local layer's hazard / trafficability writes), the engine re-propagates
// from that window (dymu_resolve_window) instead of solving cold; unchanged
// speed reuses the previous map.  Both give the cold solve's fixed point.
bool DyMuPathPlanner::solveFull() {
  const uint64_t n = (uint64_t)nx_ * ny_;
  packed_.resize(n);
  for (uint64_t k = 0; k < n; ++k)
    packed_[k] = is_obstacle_[k] ? kInf : global_res_ * cost_[k] * (2 + hazard_[k] - traff_[k]);
  if (!ctx_) {
    const int rc = dymu_create(&ctx_, &opts_);
    if (rc != DYMU_OK) {
      ctx_ = nullptr;
      throw std::runtime_error(std::string("dymu: cannot create the HIP engine: ") +
                               dymu_strerror(rc));
    }
    solved_ = false;
  }
  int rc = DYMU_ERR_STATE;
  if (solved_ && speed_.size() == n && solved_gi_ == goal_i_ && solved_gj_ == goal_j_) {
    // bounding box of the cells whose speed changed (bitwise)
    unsigned i0 = nx_, i1 = 0, j0 = ny_, j1 = 0;
    for (unsigned j = 0; j < ny_; ++j) {
      const double* a = &packed_[idx(0, j)];
      const double* b = &speed_[idx(0, j)];
      if (std::memcmp(a, b, sizeof(double) * nx_) == 0) continue;
      for (unsigned i = 0; i < nx_; ++i)
        if (std::memcmp(a + i, b + i, sizeof(double)) != 0) {
          i0 = std::min(i0, i);
          i1 = std::max(i1, i + 1);
        }
      j0 = std::min(j0, j);
      j1 = j + 1;
    }
    if (i1 == 0) {  // nothing changed: the map stands
      incremental_ = 2;
      return true;
    }
    if ((uint64_t)(i1 - i0) * (j1 - j0) * 4 <= n) {  // a window: re-propagate from it
      rc = dymu_resolve_window(ctx_, packed_.data(), nx_, ny_, goal_i_, goal_j_, i0, j0, i1 - i0,
                               j1 - j0, total_cost_.data(), &stats_);
      if (rc == DYMU_OK) incremental_ = 1;
    }
  }
  if (rc != DYMU_OK) {
    solved_ = false;
    rc = dymu_solve(ctx_, packed_.data(), nx_, ny_, goal_i_, goal_j_, total_cost_.data(), &stats_);
    if (rc != DYMU_OK)
      throw std::runtime_error(std::string("dymu_solve failed: ") + dymu_strerror(rc) + " " +
                               dymu_last_error(ctx_));
    incremental_ = 0;
  }
  speed_.swap(packed_);
  solved_ = true;
  solved_gi_ = goal_i_;
  solved_gj_ = goal_j_;
  for (uint64_t k = 0; k < n; ++k) state_[k] = total_cost_[k] < kInf ? CLOSED : OPEN;
  return true;
}

// :443-468
bool DyMuPathPlanner::computeEntireTotalCostMap() {
  if (!has_goal_ || is_obstacle_[idx(goal_i_, goal_j_)]) {
    log_warn("The goal is not valid");
    return false;
  }
  return solveFull();
}

// :410-422 (start and its 8 neighbours must be free; border -> false here,
// where the reference dereferences NULL)
bool DyMuPathPlanner::isSafeNode(unsigned i, unsigned j) const {
  if (i == 0 || j == 0 || i + 1 >= nx_ || j + 1 >= ny_) return false;
  for (int dj = -1; dj <= 1; ++dj)
    for (int di = -1; di <= 1; ++di)
      if (is_obstacle_[idx(i + di, j + dj)]) return false;
  return true;
}

// :364-408.  The reference stops its FMM once the start node and its nb4 are
// CLOSED and returns false if the band is empty at that moment (start
// unreachable, or the start's neighbourhood closes last of all).  The engine
// converges the whole map; the return value is recovered from it: false iff
// the start is unreachable or max T over {start, nb4} is the global maximum
// finite T (those nodes close last).
bool DyMuPathPlanner::computeTotalCostMap(base::Waypoint wPos) {
  const double x = wPos.position[0] - global_offset_[0];
  const double y = wPos.position[1] - global_offset_[1];
  if (!has_goal_ || is_obstacle_[idx(goal_i_, goal_j_)]) {
    log_warn("The goal is not valid");
    return false;
  }
  const double fx = x / global_res_ + 0.5, fy = y / global_res_ + 0.5;
  if (!(fx >= 0) || !(fy >= 0) || fx >= (double)nx_ || fy >= (double)ny_) {
    log_error("PLANNER: The rover is located too close to an obstacle");
    return false;
  }
  const unsigned si = (unsigned)fx, sj = (unsigned)fy;
  if (!isSafeNode(si, sj)) {
    log_error("PLANNER: The rover is located too close to an obstacle");
    return false;
  }
  solveFull();
  const uint64_t s = idx(si, sj);
  if (!(total_cost_[s] < kInf)) {
    log_error("The goal is unreachable");
    return false;
  }
  double m = total_cost_[s];
  for (uint64_t nb : {s - nx_, s - 1, s + 1, s + nx_}) m = std::max(m, total_cost_[nb]);
  double tmax = 0;
  for (double t : total_cost_)
    if (t < kInf && t > tmax) tmax = t;
  if (m >= tmax) {
    log_error("The goal is unreachable");
    return false;
  }
  return true;
}

// :589-611.  evaluatePath(0) is the identity without local maps.
std::vector<base::Waypoint> DyMuPathPlanner::getPath(base::Waypoint wPos) {
  wPos.position[0] -= global_offset_[0];
  wPos.position[1] -= global_offset_[1];
  computeGlobalPath(wPos);
  std::vector<base::Waypoint> out = current_path;
  for (auto& w : out) {
    w.position[0] += global_offset_[0];
    w.position[1] += global_offset_[1];
  }
  return out;
}

// :615-662 (gradient descent on T; Q5: a NaN position ends the loop and the
// sink is appended)
bool DyMuPathPlanner::computeGlobalPath(base::Waypoint wPos) {
  current_path.clear();
  if (!has_goal_) return false;
  base::Waypoint sink;
  sink.position[0] = global_res_ * (double)goal_i_;
  sink.position[1] = global_res_ * (double)goal_j_;
  sink.position[2] = elevation_.empty() ? 0.0 : elevation_[idx(goal_i_, goal_j_)];
  sink.heading = goal_heading_;
  const double tau = std::min(0.4, risk_distance_);
  base::Waypoint wNext = computeNextGlobalWaypoint(wPos, tau);
  if (std::isnan(wNext.position[0]) || std::isnan(wNext.position[1])) {
    log_error("PLANNER: Gradient Descent Method failed");
    return false;
  }
  current_path.push_back(wPos);
  wPos = wNext;
  auto dist = [](const base::Waypoint& a, const base::Waypoint& b) {
    const double dx = a.position[0] - b.position[0], dy = a.position[1] - b.position[1];
    return std::sqrt(dx * dx + dy * dy);
  };
  while (dist(wPos, sink) > 2.0 * global_res_) {
    wNext = computeNextGlobalWaypoint(wPos, tau);
    current_path.push_back(wPos);
    if (dist(wPos, wNext) < 0.01 * tau * global_res_) {
      log_error("ERROR in trajectory");
      return false;
    }
    wPos = wNext;
  }
  current_path.push_back(sink);
  return true;
}

// :666-714 (wPos.position[2] is written: elevation, bilinear, with the
// reference's argument order at :699-704)
base::Waypoint DyMuPathPlanner::computeNextGlobalWaypoint(base::Waypoint& wPos, double tau) {
  base::Waypoint wNext;
  const double gx = wPos.position[0] / global_res_, gy = wPos.position[1] / global_res_;
  const unsigned cx = (unsigned)gx, cy = (unsigned)gy;
  const double ax = gx - (double)cx, ay = gy - (double)cy;
  if (cx + 1 >= nx_ || cy + 1 >= ny_) {  // reference: NULL dereference
    wNext.position[0] = wNext.position[1] = std::numeric_limits<double>::quiet_NaN();
    return wNext;
  }
  double gx00, gx10, gx01, gx11, gy00, gy10, gy01, gy11;
  gradientNode(cx, cy, gx00, gy00);
  gradientNode(cx + 1, cy, gx10, gy10);
  gradientNode(cx, cy + 1, gx01, gy01);
  gradientNode(cx + 1, cy + 1, gx11, gy11);
  const double dcx = interpolate(ax, ay, gx00, gx01, gx10, gx11);
  const double dcy = interpolate(ax, ay, gy00, gy01, gy10, gy11);
  const uint64_t k = idx(cx, cy);
  wPos.position[2] =
      interpolate(ax, ay, elevation_[k], elevation_[k + 1], elevation_[k + nx_],
                  elevation_[k + nx_ + 1]);
  wNext.position[0] = wPos.position[0] - global_res_ * tau * dcx;
  wNext.position[1] = wPos.position[1] - global_res_ * tau * dcy;
  wNext.heading = std::atan2(-dcy, -dcx);
  return wNext;
}

// :718-772
void DyMuPathPlanner::gradientNode(unsigned i, unsigned j, double& dnx, double& dny) const {
  const uint64_t k = idx(i, j);
  const bool hw = i > 0, he = i + 1 < nx_, hs = j > 0, hn = j + 1 < ny_;
  const double tw = hw ? total_cost_[k - 1] : kInf, te = he ? total_cost_[k + 1] : kInf;
  const double ts = hs ? total_cost_[k - nx_] : kInf, tn = hn ? total_cost_[k + nx_] : kInf;
  const double t = total_cost_[k];
  double dx, dy;
  if ((!hw && !he) || (hw && he && tw == kInf && te == kInf)) dx = 0;
  else if (!hw || tw == kInf) dx = te - t;
  else if (!he || te == kInf) dx = t - tw;
  else dx = (te - tw) * 0.5;
  if ((!hs && !hn) || (hs && hn && ts == kInf && tn == kInf)) dy = 0;
  else if (!hs || ts == kInf) dy = tn - t;
  else if (!hn || tn == kInf) dy = t - ts;
  else dy = (tn - ts) * 0.5;
  if (dx == 0 && dy == 0) {
    dnx = 0;
    dny = 0;
  } else {
    dnx = dx / std::sqrt(dx * dx + dy * dy);
    dny = dy / std::sqrt(dx * dx + dy * dy);
  }
}

// :776-784
double DyMuPathPlanner::interpolate(double a, double b, double g00, double g01, double g10,
                                    double g11) {
  return g00 + (g10 - g00) * a + (g01 - g00) * b + (g11 + g00 - g10 - g01) * a * b;
}

// :788-795
std::string DyMuPathPlanner::getLocomotionMode(base::Waypoint wPos) {
  const double x = wPos.position[0] - global_offset_[0];
  const double y = wPos.position[1] - global_offset_[1];
  const unsigned i = (unsigned)(x / global_res_ + 0.5), j = (unsigned)(y / global_res_ + 0.5);
  if (i >= nx_ || j >= ny_) return "DONT_CARE";
  const int m = loc_mode_[idx(i, j)];
  if (m < 0 || m >= (int)locomotion_modes_.size()) return "DONT_CARE";
  return locomotion_modes_[m];
}

// :799-811
std::vector<std::vector<double>> DyMuPathPlanner::getTotalCostMatrix() {
  std::vector<std::vector<double>> m(ny_, std::vector<double>(nx_));
  for (unsigned j = 0; j < ny_; ++j)
    for (unsigned i = 0; i < nx_; ++i) {
      const double t = total_cost_[idx(i, j)];
      m[j][i] = (t == kInf) ? -1.0 : t;
    }
  return m;
}

// :815-829
std::vector<std::vector<double>> DyMuPathPlanner::getGlobalCostMatrix() {
  std::vector<std::vector<double>> m(ny_, std::vector<double>(nx_));
  for (unsigned j = 0; j < ny_; ++j)
    for (unsigned i = 0; i < nx_; ++i) {
      const uint64_t k = idx(i, j);
      m[j][i] = is_obstacle_[k] ? -1.0 : cost_[k] * (2 + hazard_[k] - traff_[k]);
    }
  return m;
}

// :833-842
std::vector<std::vector<double>> DyMuPathPlanner::getHazardDensityMatrix() {
  std::vector<std::vector<double>> m(ny_, std::vector<double>(nx_));
  for (unsigned j = 0; j < ny_; ++j)
    for (unsigned i = 0; i < nx_; ++i) m[j][i] = hazard_[idx(i, j)];
  return m;
}

// :846-855
std::vector<std::vector<double>> DyMuPathPlanner::getTrafficabilityMatrix() {
  std::vector<std::vector<double>> m(ny_, std::vector<double>(nx_));
  for (unsigned j = 0; j < ny_; ++j)
    for (unsigned i = 0; i < nx_; ++i) m[j][i] = traff_[idx(i, j)];
  return m;
}

// :860-890 (Q6 kept: a = x - i, not x/res - i)
double DyMuPathPlanner::getTotalCost(base::Waypoint wInt) {
  const double x = wInt.position[0] - global_offset_[0];
  const double y = wInt.position[1] - global_offset_[1];
  const unsigned i = (unsigned)(x / global_res_), j = (unsigned)(y / global_res_);
  const double a = x - (double)i, b = y - (double)j;
  if (i + 1 >= nx_ || j + 1 >= ny_) {  // a corner is NULL
    const unsigned ni = (unsigned)(x / global_res_ + 0.5), nj = (unsigned)(y / global_res_ + 0.5);
    if (ni >= nx_ || nj >= ny_) return kInf;
    return total_cost_[idx(ni, nj)];
  }
  const uint64_t k = idx(i, j);
  const uint64_t k10 = k + 1, k01 = k + nx_, k11 = k + nx_ + 1;
  if (state_[k] == OPEN || state_[k10] == OPEN || state_[k01] == OPEN || state_[k11] == OPEN) {
    const unsigned ni = (unsigned)(x / global_res_ + 0.5), nj = (unsigned)(y / global_res_ + 0.5);
    return total_cost_[idx(ni, nj)];
  }
  const double w00 = total_cost_[k], w10 = total_cost_[k10];
  const double w01 = total_cost_[k01], w11 = total_cost_[k11];
  return w00 + (w10 - w00) * a + (w01 - w00) * b + (w11 + w00 - w10 - w01) * a * b;
}

}  // namespace PathPlanning_lib
