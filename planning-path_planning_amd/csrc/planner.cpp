// planner.cpp -- PathPlanning_lib::DyMuPathPlanner over SoA arrays (DyMu.hpp).
//
// Host C++ around the MI355X engine: cost-map ingestion, goal validation and
// path extraction run on the host exactly as the reference computes them
// (compiled with -ffp-contract=off so each operation rounds where the
// reference's does); the total-cost propagation -- the reference's FMM loop
// -- runs on the GPU over a device-resident speed / total-cost map:
//   * the speed F is packed on the host only for the rows whose node fields
//     changed, and only the rows whose speed changed are uploaded;
//   * the total cost stays on the device; the host mirror fetches blocks of it
//     on first read (path extraction reads a narrow band around the path) or
//     all of it for the matrix getters.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <limits>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "DyMu.hpp"
#include "local_layer.hpp"
#include "pop_order.hpp"

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

namespace {
void release_engine(dymu_ctx*& ctx, double*& dF, double*& dT, void*& reg, uint64_t& cells) {
  if (!ctx) return;
  if (reg) (void)dymu_host_unregister(ctx, reg);
  if (dF) (void)dymu_device_free(ctx, dF);
  if (dT) (void)dymu_device_free(ctx, dT);
  dymu_destroy(ctx);
  ctx = nullptr;
  dF = dT = nullptr;
  reg = nullptr;
  cells = 0;
}
}  // namespace

DyMuPathPlanner::~DyMuPathPlanner() {
  release_engine(ctx_, dF_, dT_, registered_, dcells_);
}

void DyMuPathPlanner::setEngineOptions(const dymu_opts& o) {
  opts_ = o;
  // the solved map lives in dT_: bring the host mirror up to date before the
  // device buffers go, so T(), getPath and the matrix getters keep working
  if (ctx_ && dT_ && blk_missing_) fetchAll();
  release_engine(ctx_, dF_, dT_, registered_, dcells_);
  solved_ = false;
  speed_valid_ = false;
  markDirty(0, ny_);
}

// :39-104.  Node fields start as the globalNode constructor sets them
// (src/DyMu.hpp:88-107): cost 0, raw_cost 0, hazard 0, traff 1, T = +inf,
// OPEN, not an obstacle, locomotion "DONT_CARE".  Neighbour lists are implicit
// in the row-major layout.
bool DyMuPathPlanner::initGlobalLayer(double globalres, double localres, unsigned num_nodes_X,
                                      unsigned num_nodes_Y, std::vector<double> offset) {
  global_res_ = globalres;
  local_res_ = localres;
  {
    const double rr = global_res_ / local_res_;  // :49 res_ratio = (uint)(global_res / local_res)
    res_ratio_ = grid_u32(rr);
  }
  if (!local_) local_ = std::make_unique<LocalLayer>();
  local_->reset(res_ratio_);
  local_agent_ = -1;
  reconnecting_index = 0;
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
  terrain_.assign(n, 0u);
  is_obstacle_.assign(n, 0);
  loc_mode_.assign(n, -1);
  has_goal_ = false;
  current_path.clear();
  // a new grid: new device buffers and an empty total-cost map (every node
  // OPEN at +inf, as the globalNode constructor leaves it)
  release_engine(ctx_, dF_, dT_, registered_, dcells_);
  total_cost_.assign(n, kInf);
  nbx_ = (nx_ + kBlk - 1) / kBlk;
  nby_ = (ny_ + kBlk - 1) / kBlk;
  blk_ok_.assign((uint64_t)nbx_ * nby_, 1);
  blk_missing_ = 0;
  closed_limit_ = 0.0;
  band_cells_.clear();
  band_unordered_ = false;
  band_values_checked_ = true;
  open_at_limit_.clear();
  node_state_.clear();
  propagated_extra_.clear();
  manual_list_ = false;
  speed_.clear();
  speed_valid_ = false;
  markDirty(0, ny_);
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
  markDirty(0, ny_);
  return true;
}

namespace {

// Host threads for the per-node loops of computeCostMap: DYMU_HOST_THREADS, else
// OMP_NUM_THREADS, else the hardware's, at most 64.
unsigned host_threads() {
  for (const char* v : {"DYMU_HOST_THREADS", "OMP_NUM_THREADS"})
    if (const char* kv = std::getenv(v)) {
      const int t = std::atoi(kv);
      if (t > 0) return (unsigned)std::min(t, 64);
    }
  const unsigned h = std::thread::hardware_concurrency();
  return h ? std::min(h, 64u) : 1u;
}

// body(t) for t in [0, nt) on nt threads (the caller's among them).  Exceptions
// thrown by body on a worker thread are carried back and rethrown on the calling
// thread (a throw escaping a std::thread would std::terminate); the started threads
// are joined on every path, a failed thread start included.
template <class Body>
void parallel_tasks(unsigned nt, Body&& body) {
  if (nt <= 1) {
    body(0u);
    return;
  }
  std::vector<std::exception_ptr> errs(nt);
  struct Joiner {
    std::vector<std::thread> pool;
    ~Joiner() {
      for (auto& th : pool)
        if (th.joinable()) th.join();
    }
  } J;
  J.pool.reserve(nt - 1);
  auto run = [&body, &errs](unsigned t) {
    try {
      body(t);
    } catch (...) {
      errs[t] = std::current_exception();
    }
  };
  try {
    for (unsigned t = 1; t < nt; ++t) J.pool.emplace_back(run, t);
  } catch (...) {  // std::system_error from a thread start: finish what started, rethrow
    for (auto& th : J.pool) th.join();
    J.pool.clear();
    throw;
  }
  run(0u);
  for (auto& th : J.pool) th.join();
  J.pool.clear();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// body(j0, j1) over row ranges of [0, ny) on up to host_threads() threads (at
// least 64 rows each).  Every loop run this way writes only the node it visits
// and reads fields no iteration of the same loop writes, so the split changes no
// value -- the results are those of the reference's single raster loop.
template <class Body>
void parallel_rows(unsigned ny, Body&& body) {
  const unsigned nt = std::max(1u, std::min(host_threads(), ny / 64));
  const unsigned step = (ny + nt - 1) / nt;
  parallel_tasks(nt, [&](unsigned t) {
    const unsigned j0 = t * step, j1 = std::min(ny, j0 + step);
    if (t == 0 || j0 < j1) body(j0, j1);
  });
}

// std::sort over up to host_threads() threads: sorted runs, merged pairwise (the merges
// of a round in parallel).  The elements sorted here are distinct (they hold a cell
// index), so the result is the one std::sort gives.
template <class E>
void parallel_sort(std::vector<E>& v) {
  const uint64_t n = v.size();
  const unsigned nt = std::max(1u, std::min(host_threads(), (unsigned)std::min<uint64_t>(n >> 16, 64)));
  if (nt <= 1) {
    std::sort(v.begin(), v.end());
    return;
  }
  std::vector<uint64_t> b(nt + 1);
  for (unsigned t = 0; t <= nt; ++t) b[t] = n * t / nt;
  parallel_tasks(nt, [&](unsigned t) { std::sort(v.begin() + b[t], v.begin() + b[t + 1]); });
  std::vector<E> tmp(n);
  std::vector<E>*src = &v, *dst = &tmp;
  for (unsigned w = 1; w < nt; w *= 2) {
    const unsigned pairs = (nt + 2 * w - 1) / (2 * w);
    parallel_tasks(pairs, [&](unsigned q) {
      const unsigned lo = q * 2 * w, mid = std::min(lo + w, nt), hi = std::min(lo + 2 * w, nt);
      std::merge(src->begin() + b[lo], src->begin() + b[mid], src->begin() + b[mid],
                 src->begin() + b[hi], dst->begin() + b[lo]);
    });
    std::swap(src, dst);
  }
  if (src != &v) v.swap(*src);
}

}  // namespace

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
  if (elevation.size() != ny_ || terrainMap.size() != ny_) return false;
  for (unsigned j = 0; j < ny_; ++j)
    if (elevation[j].size() != nx_ || terrainMap[j].size() != nx_) return false;
  return costMapFromRows([&](unsigned j) { return elevation[j].data(); },
                         [&](unsigned j) { return terrainMap[j].data(); });
}

bool DyMuPathPlanner::computeCostMap(const std::vector<double>& cost_data,
                                     const std::vector<double>& slope_values,
                                     const std::vector<std::string>& locomotionModes,
                                     const double* elevation, const double* terrainMap) {
  cost_lutable = cost_data;
  slope_range_ = slope_values;
  locomotion_modes_ = locomotionModes;
  if (!elevation || !terrainMap) return false;
  const uint64_t nx = nx_;
  return costMapFromRows([=](unsigned j) { return elevation + j * nx; },
                         [=](unsigned j) { return terrainMap + j * nx; });
}

template <class ERows, class TRows>
bool DyMuPathPlanner::costMapFromRows(const ERows& elev_row, const TRows& terr_row) {
  if (cost_lutable.empty() || slope_range_.empty() || locomotion_modes_.empty()) return false;
  const int range = (int)slope_range_.size();
  const int num_locs = (int)locomotion_modes_.size();
  const double cmax = *std::max_element(cost_lutable.begin(), cost_lutable.end());
  parallel_rows(ny_, [&](unsigned j0, unsigned j1) {
    for (unsigned j = j0; j < j1; ++j) {
      const double* e = elev_row(j);
      const double* t = terr_row(j);
      for (unsigned i = 0; i < nx_; ++i) {
        const uint64_t k = idx(i, j);
        raw_cost_[k] = 0;
        elevation_[k] = e[i];
        terrain_[k] = (i == 0 || j == 0 || i == nx_ - 1 || j == ny_ - 1) ? 0u : (uint32_t)t[i];
      }
    }
  });
  // slope reads the elevation only; the nominal cost its own node
  parallel_rows(ny_, [&](unsigned j0, unsigned j1) {
    for (unsigned j = j0; j < j1; ++j)
      for (unsigned i = 0; i < nx_; ++i) {
        calculateSlope(i, j);
        nominalCost(i, j, range, num_locs, cmax);
        const uint64_t k = idx(i, j);
        if (is_obstacle_[k]) {
          traff_[k] = 0.0;
          hazard_[k] = 1.0;
        }
      }
  });
  // smoothing writes cost and reads only raw costs (Q1: its own previous cost)
  parallel_rows(ny_, [&](unsigned j0, unsigned j1) {
    for (unsigned j = j0; j < j1; ++j)
      for (unsigned i = 0; i < nx_; ++i) smoothCost(i, j);
  });
  markDirty(0, ny_);
  return true;
}

// :186-210 (off-grid neighbours: one-sided differences; a 1-wide axis reads
// slope 0 there instead of the reference's NULL dereference)
void DyMuPathPlanner::calculateSlope(unsigned i, unsigned j) {
  if (i >= nx_ || j >= ny_) return;
  const uint64_t k = idx(i, j);
  double dx = 0, dy = 0;
  if (nx_ > 1) {
    if (i == 0)
      dx = (elevation_[k + 1] - elevation_[k]) / global_res_;
    else if (i == nx_ - 1)
      dx = (elevation_[k] - elevation_[k - 1]) / global_res_;
    else
      dx = (elevation_[k + 1] - elevation_[k - 1]) * 0.5 / global_res_;
  }
  if (ny_ > 1) {
    if (j == 0)
      dy = (elevation_[k + nx_] - elevation_[k]) / global_res_;
    else if (j == ny_ - 1)
      dy = (elevation_[k] - elevation_[k - nx_]) / global_res_;
    else
      dy = (elevation_[k + nx_] - elevation_[k - nx_]) * 0.5 / global_res_;
  }
  slope_[k] = std::atan(std::sqrt(dx * dx + dy * dy));
}

// :217-293 (Cmax recomputed per call, as there)
void DyMuPathPlanner::calculateNominalCost(unsigned i, unsigned j, int range, int numLocs) {
  if (i >= nx_ || j >= ny_ || cost_lutable.empty()) return;
  nominalCost(i, j, range, numLocs, *std::max_element(cost_lutable.begin(), cost_lutable.end()));
}

// Q2: locomotion mode 0 is skipped when there are several; Q3: the neighbours'
// "Cmax" loops never run (isObstacle was just set); Q4: range == 1 indexes the
// LUT as terrain * numLocs + m.  A terrain class the LUT does not cover (an
// out-of-bounds read in the reference) makes the cell an obstacle, as the
// device kernel does (cost_kernels.hip).
void DyMuPathPlanner::nominalCost(unsigned i, unsigned j, int range, int num_locs, double cmax) {
  const uint64_t k = idx(i, j);
  const uint32_t t = terrain_[k];
  const size_t nl = cost_lutable.size();
  auto lut = [&](size_t q) { return q < nl ? cost_lutable[q] : cmax; };
  if (t == 0 || (uint64_t)(t + 1) * (uint64_t)range * (uint64_t)num_locs > nl) {
    raw_cost_[k] = cmax;
    is_obstacle_[k] = 1;
  } else if (range == 1) {
    double cdef = lut((size_t)t * num_locs);
    for (int m = 0; m < (int)locomotion_modes_.size(); ++m)
      cdef = std::min(cdef, lut((size_t)t * num_locs + m));
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
        for (int m = 1; m < (int)locomotion_modes_.size(); ++m) {
          const double c1 = lut((size_t)t * range * num_locs + (size_t)m * range + (int)smin);
          const double c2 = lut((size_t)t * range * num_locs + (size_t)m * range + (int)smax);
          const double cc = c1 + (c2 - c1) * (si - smin);
          if (cc < cdef) {
            cdef = cc;
            raw_cost_[k] = std::max(raw_cost_[k], cdef);
            loc_mode_[k] = m;
          }
        }
      } else {
        const double c1 = lut((size_t)t * range + (int)smin);
        const double c2 = lut((size_t)t * range + (int)smax);
        cdef = c1 + (c2 - c1) * (si - smin);
        raw_cost_[k] = std::max(raw_cost_[k], cdef);
        loc_mode_[k] = 0;
      }
    }
  }
}

// :297-308 (Q1: starts from the node's previous cost)
void DyMuPathPlanner::smoothCost(unsigned i, unsigned j) {
  if (i >= nx_ || j >= ny_) return;
  const uint64_t k = idx(i, j);
  double csum = cost_[k], n = 5;
  if (j == 0) n--; else csum += raw_cost_[k - nx_];
  if (i == 0) n--; else csum += raw_cost_[k - 1];
  if (i == nx_ - 1) n--; else csum += raw_cost_[k + 1];
  if (j == ny_ - 1) n--; else csum += raw_cost_[k + nx_];
  cost_[k] = csum / n;
}

// :322-357
bool DyMuPathPlanner::setGoal(base::Waypoint wGoal) {
  const double px = (wGoal.position[0] - global_offset_[0]) / global_res_;
  const double py = (wGoal.position[1] - global_offset_[1]) / global_res_;
  if (px < 0 || py < 0) return false;
  const unsigned i = grid_u32(px + 0.5), j = grid_u32(py + 0.5);
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

namespace {
// rows of a vs b (ny rows of nx) that differ: [*j0, *j1), empty if none
void diff_rows(const double* a, const double* b, unsigned nx, unsigned ny, unsigned* j0,
               unsigned* j1) {
  *j0 = ny;
  *j1 = 0;
  for (unsigned j = 0; j < ny; ++j)
    if (std::memcmp(a + (uint64_t)j * nx, b + (uint64_t)j * nx, sizeof(double) * nx) != 0) {
      if (*j0 == ny) *j0 = j;
      *j1 = j + 1;
    }
}
}  // namespace

void DyMuPathPlanner::markDirty(unsigned j0, unsigned j1) {
  if (j0 >= j1) return;
  if (dirty_j0_ >= dirty_j1_) {
    dirty_j0_ = j0;
    dirty_j1_ = j1;
  } else {
    dirty_j0_ = std::min(dirty_j0_, j0);
    dirty_j1_ = std::max(dirty_j1_, j1);
  }
}

bool DyMuPathPlanner::setHazardDensity(const std::vector<double>& hd) {
  if (hd.size() != hazard_.size()) return false;
  unsigned j0, j1;
  diff_rows(hd.data(), hazard_.data(), nx_, ny_, &j0, &j1);
  if (j0 < j1) {
    std::memcpy(&hazard_[idx(0, j0)], &hd[idx(0, j0)], sizeof(double) * (uint64_t)(j1 - j0) * nx_);
    markDirty(j0, j1);
  }
  return true;
}

bool DyMuPathPlanner::setTrafficability(const std::vector<double>& tr) {
  if (tr.size() != traff_.size()) return false;
  unsigned j0, j1;
  diff_rows(tr.data(), traff_.data(), nx_, ny_, &j0, &j1);
  if (j0 < j1) {
    std::memcpy(&traff_[idx(0, j0)], &tr[idx(0, j0)], sizeof(double) * (uint64_t)(j1 - j0) * nx_);
    markDirty(j0, j1);
  }
  return true;
}

bool DyMuPathPlanner::setHazardDensityWindow(unsigned i0, unsigned j0, unsigned w, unsigned h,
                                             const double* hd) {
  if (!hd || (uint64_t)i0 + w > nx_ || (uint64_t)j0 + h > ny_) return false;
  for (unsigned r = 0; r < h; ++r)
    std::memcpy(&hazard_[idx(i0, j0 + r)], hd + (uint64_t)r * w, sizeof(double) * w);
  markDirty(j0, j0 + h);
  return true;
}

bool DyMuPathPlanner::setTrafficabilityWindow(unsigned i0, unsigned j0, unsigned w, unsigned h,
                                              const double* tr) {
  if (!tr || (uint64_t)i0 + w > nx_ || (uint64_t)j0 + h > ny_) return false;
  for (unsigned r = 0; r < h; ++r)
    std::memcpy(&traff_[idx(i0, j0 + r)], tr + (uint64_t)r * w, sizeof(double) * w);
  markDirty(j0, j0 + h);
  return true;
}

// ---- the device-resident map ----

void DyMuPathPlanner::ensureEngine() {
  const uint64_t n = (uint64_t)nx_ * ny_;
  if (!ctx_) {
    const int rc = dymu_create(&ctx_, &opts_);
    if (rc != DYMU_OK) {
      ctx_ = nullptr;
      throw std::runtime_error(std::string("dymu: cannot create the HIP engine: ") +
                               dymu_strerror(rc));
    }
    solved_ = false;
    speed_valid_ = false;
  }
  if (dcells_ != n) {
    if (dF_) (void)dymu_device_free(ctx_, dF_);
    if (dT_) (void)dymu_device_free(ctx_, dT_);
    dF_ = dT_ = nullptr;
    dcells_ = 0;
    void *f = nullptr, *t = nullptr;
    if (dymu_device_alloc(ctx_, sizeof(double) * n, &f) != DYMU_OK ||
        dymu_device_alloc(ctx_, sizeof(double) * n, &t) != DYMU_OK) {
      if (f) (void)dymu_device_free(ctx_, f);
      throw std::runtime_error("dymu: cannot allocate the device map");
    }
    dF_ = static_cast<double*>(f);
    dT_ = static_cast<double*>(t);
    dcells_ = n;
    solved_ = false;
    speed_valid_ = false;
    // page-lock the host mirror for full-rate downloads (optional: pageable works)
    if (registered_) (void)dymu_host_unregister(ctx_, registered_);
    registered_ = nullptr;
    if (dymu_host_register(ctx_, total_cost_.data(), sizeof(double) * n) == DYMU_OK)
      registered_ = total_cost_.data();
  }
  if (!speed_valid_) {
    speed_.assign(n, 0.0);
    markDirty(0, ny_);
  }
}

// F = global_res * cost * (2 + hazard - traff) (:527-528), +inf for obstacles,
// re-packed for the dirty rows; the rows whose F changed are uploaded.
bool DyMuPathPlanner::syncSpeed(unsigned& i0, unsigned& i1, unsigned& j0, unsigned& j1) {
  i0 = nx_;
  i1 = 0;
  j0 = ny_;
  j1 = 0;
  decrease_only_ = speed_valid_;
  if (dirty_j0_ >= dirty_j1_ && speed_valid_) return false;
  const unsigned d0 = speed_valid_ ? dirty_j0_ : 0, d1 = speed_valid_ ? dirty_j1_ : ny_;
  row_.resize(nx_);
  for (unsigned j = d0; j < d1; ++j) {
    const uint64_t k0 = idx(0, j);
    for (unsigned i = 0; i < nx_; ++i) {
      const uint64_t k = k0 + i;
      row_[i] = is_obstacle_[k] ? kInf : global_res_ * cost_[k] * (2 + hazard_[k] - traff_[k]);
    }
    double* old = &speed_[k0];
    if (speed_valid_ && std::memcmp(row_.data(), old, sizeof(double) * nx_) == 0) continue;
    unsigned a = 0, b = nx_;
    if (speed_valid_) {
      while (std::memcmp(&row_[a], old + a, sizeof(double)) == 0) ++a;
      while (std::memcmp(&row_[b - 1], old + b - 1, sizeof(double)) == 0) --b;
      for (unsigned i = a; i < b && decrease_only_; ++i)
        if (!(row_[i] <= old[i])) decrease_only_ = false;
    }
    std::memcpy(old, row_.data(), sizeof(double) * nx_);
    i0 = std::min(i0, a);
    i1 = std::max(i1, b);
    if (j0 == ny_) j0 = j;
    j1 = j + 1;
  }
  dirty_j0_ = dirty_j1_ = 0;
  if (!speed_valid_) {
    i0 = 0, i1 = nx_, j0 = 0, j1 = ny_;
  }
  speed_valid_ = true;
  if (j0 >= j1) return false;
  const int rc = dymu_memcpy_h2d(ctx_, dF_ + idx(0, j0), &speed_[idx(0, j0)],
                                 sizeof(double) * (uint64_t)(j1 - j0) * nx_);
  if (rc != DYMU_OK) {
    speed_valid_ = false;
    throw std::runtime_error(std::string("dymu: speed upload failed: ") + dymu_last_error(ctx_));
  }
  return true;
}

// Thread-safe (the band replay's threads read through it): a block's flag is read
// with acquire and set with release after its download, downloads one at a time.
double DyMuPathPlanner::T(uint64_t k) const {
  if (__atomic_load_n(&blk_missing_, __ATOMIC_ACQUIRE)) {
    const unsigned j = (unsigned)(k / nx_), i = (unsigned)(k % nx_);
    const uint64_t b = (uint64_t)(j / kBlk) * nbx_ + i / kBlk;
    if (!__atomic_load_n(&blk_ok_[b], __ATOMIC_ACQUIRE)) {
      std::lock_guard<std::mutex> lock(fetch_mu_);
      if (!__atomic_load_n(&blk_ok_[b], __ATOMIC_RELAXED)) {
        const unsigned bi = (i / kBlk) * kBlk, bj = (j / kBlk) * kBlk;
        const unsigned w = std::min(kBlk, nx_ - bi), h = std::min(kBlk, ny_ - bj);
        const uint64_t o = idx(bi, bj);
        if (dymu_memcpy2d_d2h(ctx_, &total_cost_[o], sizeof(double) * nx_, dT_ + o,
                              sizeof(double) * nx_, sizeof(double) * w, h) != DYMU_OK)
          throw std::runtime_error(std::string("dymu: total-cost download failed: ") +
                                   dymu_last_error(ctx_));
        __atomic_store_n(&blk_ok_[b], (uint8_t)1, __ATOMIC_RELEASE);
        __atomic_sub_fetch(&blk_missing_, 1, __ATOMIC_RELEASE);
      }
    }
  }
  return total_cost_[k];
}

void DyMuPathPlanner::fetchAll() const {
  if (!blk_missing_) return;
  if (dymu_memcpy_d2h(ctx_, total_cost_.data(), dT_, sizeof(double) * dcells_) != DYMU_OK)
    throw std::runtime_error(std::string("dymu: total-cost download failed: ") +
                             dymu_last_error(ctx_));
  std::fill(blk_ok_.begin(), blk_ok_.end(), 1);
  blk_missing_ = 0;
}

const double* DyMuPathPlanner::totalCostData() const {
  fetchAll();
  return total_cost_.data();
}

// One pass over the host mirror split in row ranges: at 16384^2 a single-thread
// copy into a caller's fresh buffer (first-touch faults on 2 GiB) costs several
// times the solve itself.
// A stale mirror is downloaded in row chunks and each chunk is handed on while
// the next one downloads.
template <class Body>
void DyMuPathPlanner::streamTotalCost(Body&& body) const {
  constexpr unsigned kChunks = 16;
  if (!blk_missing_ || ny_ < 64 * kChunks) {
    fetchAll();
    body(0u, ny_);
    return;
  }
  const unsigned step = (ny_ + kChunks - 1) / kChunks;
  // the return code is the failure flag (some failures leave no error text)
  int rc = DYMU_OK;
  std::exception_ptr body_err;
  struct Joiner {
    std::thread th;
    ~Joiner() {
      if (th.joinable()) th.join();
    }
  } worker;
  // body_err is written by the worker thread: it is read only after that thread's
  // join (the join is the synchronisation), never while the worker may still run
  for (unsigned r0 = 0; r0 < ny_ && rc == DYMU_OK; r0 += step) {
    const unsigned r1 = std::min(ny_, r0 + step);
    const uint64_t o = idx(0, r0);
    rc = dymu_memcpy_d2h(ctx_, &total_cost_[o], dT_ + o, sizeof(double) * (idx(0, r1) - o));
    if (worker.th.joinable()) worker.th.join();
    if (body_err) break;
    if (rc == DYMU_OK)
      worker.th = std::thread([&body, &body_err, r0, r1] {
        try {
          body(r0, r1);
        } catch (...) {
          body_err = std::current_exception();
        }
      });
  }
  if (worker.th.joinable()) worker.th.join();
  if (rc != DYMU_OK) {
    const char* msg = ctx_ ? dymu_last_error(ctx_) : "";
    throw std::runtime_error(std::string("dymu: total-cost download failed: ") +
                             (msg && *msg ? msg : dymu_strerror(rc)));
  }
  if (body_err) std::rethrow_exception(body_err);
  std::fill(blk_ok_.begin(), blk_ok_.end(), 1);
  blk_missing_ = 0;
}

void DyMuPathPlanner::copyTotalCost(double* out, bool raw) const {
  const double* t = total_cost_.data();
  streamTotalCost([&](unsigned r0, unsigned r1) {
    parallel_rows(r1 - r0, [&](unsigned j0, unsigned j1) {
      const uint64_t a = idx(0, r0 + j0), b = idx(0, r0 + j1);
      if (raw) {
        std::memcpy(out + a, t + a, sizeof(double) * (b - a));
      } else {
        for (uint64_t k = a; k < b; ++k) out[k] = t[k] == kInf ? -1.0 : t[k];
      }
    });
  });
}

bool DyMuPathPlanner::closedCell(uint64_t k) const {
  if (!node_state_.empty()) return node_state_[k] != 0;
  const double t = T(k);
  if (!(t < kInf) || t > closed_limit_) return false;
  return t < closed_limit_ || open_at_limit_.empty() ||
         !std::binary_search(open_at_limit_.begin(), open_at_limit_.end(), k);
}

// One propagation on the engine.  early = computeTotalCostMap (:364-408): stop
// once (si, sj) and its nb4 are final, then rebuild the reference's node states
// (CLOSED / band / never reached) and the band's tentative values.  Otherwise
// computeEntireTotalCostMap (:443-468), incremental where possible: when dT_
// holds the converged map of the same grid and goal and the speed changed only
// inside a window (the local layer's hazard / trafficability writes), the engine
// re-propagates from that window (dymu_update_window_device; without any reset
// when every changed speed went down); unchanged speed
// reuses the map.  Both give the cold solve's fixed point.
// Returns false iff the early exit left an empty band (the reference's "goal
// unreachable" return, :399-403).
bool DyMuPathPlanner::propagate(bool early, unsigned si, unsigned sj) {
  ensureEngine();
  unsigned i0, i1, j0, j1;
  const bool changed = syncSpeed(i0, i1, j0, j1);
  const uint64_t n = (uint64_t)nx_ * ny_;
  int rc = DYMU_ERR_STATE;
  if (!early && solved_ && solved_gi_ == goal_i_ && solved_gj_ == goal_j_) {
    if (!changed) {
      incremental_ = 2;
      return true;
    }
    if ((uint64_t)(i1 - i0) * (j1 - j0) * 4 <= n) {
      rc = dymu_update_window_device(ctx_, dF_, dT_, nx_, ny_, nx_, goal_i_, goal_j_, i0, j0,
                                     i1 - i0, j1 - j0, decrease_only_ ? 1 : 0, nullptr, &stats_);
      if (rc == DYMU_OK) incremental_ = 1;
    }
  }
  double t_closed = kInf;
  if (rc != DYMU_OK) {
    solved_ = false;
    rc = early ? dymu_solve_until_device(ctx_, dF_, dT_, nx_, ny_, nx_, goal_i_, goal_j_, si, sj,
                                         nullptr, &t_closed, &stats_)
               : dymu_solve_device(ctx_, dF_, dT_, nx_, ny_, nx_, goal_i_, goal_j_, nullptr,
                                   &stats_);
    if (rc != DYMU_OK)
      throw std::runtime_error(std::string("dymu solve failed: ") + dymu_strerror(rc) + " " +
                               dymu_last_error(ctx_));
    incremental_ = 0;
  }
  // the host mirror is stale; node states and the propagated list follow the new map
  std::fill(blk_ok_.begin(), blk_ok_.end(), 0);
  blk_missing_ = blk_ok_.size();
  band_cells_.clear();
  band_unordered_ = false;
  band_values_checked_ = true;
  open_at_limit_.clear();
  node_state_.clear();
  propagated_extra_.clear();
  manual_list_ = false;
  early_info_ = EarlyExitInfo{};
  if (!early) {
    closed_limit_ = kInf;
    solved_ = true;
    solved_gi_ = goal_i_;
    solved_gj_ = goal_j_;
    return true;
  }
  // early exit: the reference's CLOSED set is {T <= t_closed}; the band gets its
  // tentative values; every other cell +inf.  dT_ is no longer a converged map.
  solved_ = false;
  closed_limit_ = t_closed;
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t g = idx(goal_i_, goal_j_), s = idx(si, sj);
  // The region the exit is decided on: the cells of T <= t_closed (a margin far above
  // the engine's error) and their band, one cell around; and the near-tie guard over it
  // (pop_order.hpp): the engine's values order cells as the reference's do only where
  // no rounding can flip the order
  dymu_region reg{};
  reg.i0 = 1;
  reg.i1 = 0;
  const double thr = t_closed < kInf ? t_closed * (1 + kRegionMargin) : kInf;
  if (dymu_region_stats(ctx_, dF_, dT_, nx_, ny_, nx_, goal_i_, goal_j_, thr,
                        t_closed * (1 - kTieEps), t_closed * (1 + kTieEps), &reg,
                        nullptr) != DYMU_OK)
    throw std::runtime_error(std::string("dymu_region_stats failed: ") + dymu_last_error(ctx_));
  int64_t box[4] = {0, 0, -1, -1};  // inclusive; empty when nothing was reached
  if (reg.i0 <= reg.i1) {
    box[0] = reg.i0 > 0 ? reg.i0 - 1 : 0;
    box[1] = reg.j0 > 0 ? reg.j0 - 1 : 0;
    box[2] = std::min<int64_t>((int64_t)reg.i1 + 1, nx_ - 1);
    box[3] = std::min<int64_t>((int64_t)reg.j1 + 1, ny_ - 1);
  }
  TieGuard guard(nx_, goal_i_, goal_j_, speed_[g], reg.r_const);
  have_start_ = true;  // for insertionOrder's / minCostGlobalNode's exact fallback
  exit_r_const_ = reg.r_const;
  start_i_ = si;
  start_j_ = sj;
  std::copy(box, box + 4, exit_box_);
  std::vector<uint64_t> band(std::max<uint64_t>(4096, 4 * (uint64_t)(nx_ + ny_)));
  uint64_t nb = 0;
  for (;;) {
    rc = dymu_early_exit_mask(ctx_, dF_, dT_, nx_, ny_, nx_, t_closed, band.data(), band.size(),
                              &nb, nullptr);
    if (rc != DYMU_OK)
      throw std::runtime_error(std::string("dymu_early_exit_mask failed: ") +
                               dymu_last_error(ctx_));
    if (nb <= band.size()) break;
    band.resize(nb);
  }
  band.resize(nb);
  std::sort(band.begin(), band.end());
  PopOrder<MapT> po(MapT{this}, nx_, ny_, g, &guard);
  // the exit moment: the last of the start and its nb4 the reference pops (all five
  // CLOSED; the latest has the largest value, t_closed)
  const uint64_t probes[5] = {s, s - nx_, s - 1, s + 1, s + nx_};
  uint64_t last = s;
  for (int q = 1; q < 5; ++q)
    if (po.popBefore(last, probes[q])) last = probes[q];
  // Cells of exactly t_closed: the reference pops them in insertion order and stops
  // right after `last`, so those it pops later stay in the band (with their value).
  // Resolve which, from the values (pop_order.hpp).  An engine tie with the exit value
  // is the reference's only as a mirror image of a probe of that value; a cell the
  // engine puts within eps of it, but not on it, is a near tie.
  if (t_closed < kInf) {
    std::vector<uint64_t> eq(256);
    uint64_t n_eq = 0;
    for (;;) {
      if (dymu_find_equal(ctx_, dT_, nx_, ny_, nx_, t_closed, eq.data(), eq.size(), &n_eq,
                          nullptr) != DYMU_OK)
        throw std::runtime_error(std::string("dymu_find_equal failed: ") + dymu_last_error(ctx_));
      if (n_eq <= eq.size()) break;
      eq.resize(n_eq);
    }
    eq.resize(n_eq);
    early_info_.tied = n_eq;
    for (const uint64_t x : eq) {
      bool trusted = false;
      for (const uint64_t q : probes)
        trusted = trusted || (T(q) == t_closed && (q == x || guard.mirror(x, q)));
      if (!trusted) ++guard.near;
    }
    guard.near += reg.n_range > n_eq ? reg.n_range - n_eq : 0;
    if (n_eq > 1) {
      for (const uint64_t x : eq)
        if (x != last && po.popBefore(last, x)) open_at_limit_.push_back(x);
      std::sort(open_at_limit_.begin(), open_at_limit_.end());
    }
  }
  const double ms_order =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // an undetermined or near-tied order: the exact host replay decides the exit
  // (DYMU_EXACT_EXIT=1 forces it: measurement and tests of that path)
  static const bool force_exact = [] {
    const char* kv = std::getenv("DYMU_EXACT_EXIT");
    return kv && std::atoi(kv) != 0;
  }();
  bool exact = po.degenerate() || guard.near > 0 || force_exact;
  // the band with the cells the reference left OPEN at t_closed: they join it, and
  // a neighbour of theirs stays in it only if it has another CLOSED neighbour
  // (otherwise it was never reached: +inf)
  std::vector<uint64_t> unreached;
  if (!exact && !open_at_limit_.empty()) {
    std::vector<uint64_t> add(open_at_limit_);
    for (const uint64_t x : open_at_limit_) {
      const unsigned i = (unsigned)(x % nx_), j = (unsigned)(x / nx_);
      const int64_t nb4[4][2] = {{i, (int64_t)j - 1}, {(int64_t)i - 1, j}, {i + 1, j}, {i, j + 1}};
      for (const auto& q : nb4) {
        if (q[0] < 0 || q[1] < 0 || q[0] >= nx_ || q[1] >= ny_) continue;
        const uint64_t y = idx((unsigned)q[0], (unsigned)q[1]);
        if (!std::binary_search(band.begin(), band.end(), y) || T(y) <= t_closed) continue;
        bool reached = false;
        const unsigned yi = (unsigned)q[0], yj = (unsigned)q[1];
        if (yj > 0) reached |= closedCell(y - nx_);
        if (yi > 0) reached |= closedCell(y - 1);
        if (yi + 1 < nx_) reached |= closedCell(y + 1);
        if (yj + 1 < ny_) reached |= closedCell(y + nx_);
        if (!reached) unreached.push_back(y);
      }
    }
    std::sort(unreached.begin(), unreached.end());
    unreached.erase(std::unique(unreached.begin(), unreached.end()), unreached.end());
    std::vector<uint64_t> kept;
    kept.reserve(band.size() + add.size());
    for (const uint64_t y : band)
      if (!std::binary_search(unreached.begin(), unreached.end(), y)) kept.push_back(y);
    kept.insert(kept.end(), add.begin(), add.end());
    std::sort(kept.begin(), kept.end());
    band.swap(kept);
    nb = band.size();
  }
  std::vector<double> vals;
  if (nb && !exact) {
    exact = replayBand(last, band, vals, guard);
  }
  early_info_.near_ties = guard.near;
  early_info_.open_at_limit = open_at_limit_.size();
  if (exact) {
    // the reference replayed exactly on the host over the region (no size limit)
    early_info_.exact_replay = 1;
    if (std::getenv("DYMU_ORDER_DEBUG"))
      std::fprintf(stderr,
                   "[dymu] exact exit: near ties %llu (first (%llu,%llu) %.17g vs (%llu,%llu) "
                   "%.17g; mirror below %.17g), degenerate %d (reason %d)\n",
                   (unsigned long long)guard.near, (unsigned long long)(guard.first[0] % nx_),
                   (unsigned long long)(guard.first[0] / nx_), guard.first_t[0],
                   (unsigned long long)(guard.first[1] % nx_),
                   (unsigned long long)(guard.first[1] / nx_), guard.first_t[1],
                   guard.trust_below, (int)po.degenerate(), po.why());
    const bool r = exactEarlyExit(si, sj, box);
    early_info_.resolve_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return r;
  }
  if (!unreached.empty()) {
    const std::vector<double> inf(unreached.size(), kInf);
    if (dymu_scatter(ctx_, dT_, nx_, nx_, unreached.data(), inf.data(), unreached.size(),
                     nullptr) != DYMU_OK)
      throw std::runtime_error(std::string("dymu_scatter failed: ") + dymu_last_error(ctx_));
    for (const uint64_t y : unreached) {
      (void)T(y);
      total_cost_[y] = kInf;
    }
  }
  if (nb) {
    rc = dymu_scatter(ctx_, dT_, nx_, nx_, band.data(), vals.data(), nb, nullptr);
    if (rc != DYMU_OK)
      throw std::runtime_error(std::string("dymu_scatter failed: ") + dymu_last_error(ctx_));
    // blocks fetched during the replay hold the pre-replay band values
    for (uint64_t q = 0; q < nb; ++q) {
      (void)T(band[q]);
      total_cost_[band[q]] = vals[q];
    }
  }
  early_info_.resolve_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (std::getenv("DYMU_ORDER_DEBUG"))
    std::fprintf(stderr, "[dymu] early exit: t_closed %.17g band %llu tied %llu open %llu, "
                 "%.1f ms order + %.1f ms band on %u threads\n", t_closed,
                 (unsigned long long)nb, (unsigned long long)early_info_.tied,
                 (unsigned long long)open_at_limit_.size(), ms_order,
                 early_info_.resolve_ms - ms_order, early_info_.replay_threads);
  band_cells_ = std::move(band);
  band_unordered_ = band_cells_.size() > 1;
  band_values_checked_ = false;  // minCostGlobalNode checks them for near ties first
  return nb > 0;
}

// The reference's tentative band values at its early exit, from the CLOSED
// values.  A pop of node m updates its OPEN nb4 x from the values x's neighbours
// hold at that moment (:462-465, :500-546), so with "moment c" = just after the pop
// of node c:
//   val(x, c) = min over nb4 m of x CLOSED by moment c of cand(x, m),
// where cand(x, m) is the update with each neighbour n of x at its value at moment
// m: T(n) if n is CLOSED by then (popped no later than m, in the reference's pop
// order -- pop_order.hpp -- which decides ties), else val(n, m).  The band values at
// the exit are val(x, last), last = the last of the start and its nb4 popped.  An
// OPEN value at moment m is >= T(m) >= any CLOSED value then (the FMM invariant), so
// an axis with a CLOSED side takes that side and the recursion only follows axes
// whose two sides are OPEN -- cells next to the front, at strictly earlier pops (x's
// neighbours are not adjacent to each other).
// The band cells are independent given the CLOSED values: host threads take
// contiguous runs of them, each with its own memo and order cache (a walk back stays
// near its band cell, so little work is repeated across threads).  Every comparison
// of two cells' values goes through a copy of the guard; their near ties are summed
// into `guard`.  Returns true when the values are not to be used: the pop order was
// undetermined or near-tied, or a replay hit its work bound -- the caller then
// replays the reference exactly.
bool DyMuPathPlanner::replayBand(uint64_t last, const std::vector<uint64_t>& band,
                                 std::vector<double>& out, TieGuard& guard) {
  using Order = PopOrder<MapT>;
  // open-addressing map uint64 -> double, keys != 0
  struct Memo {
    std::vector<uint64_t> key;
    std::vector<double> v;
    uint64_t n = 0, mask = 0;
    Memo() : key(1u << 12, 0), v(1u << 12), mask((1u << 12) - 1) {}
    static uint64_t h(uint64_t x) { return (x * 0x9E3779B97F4A7C15ull) >> 17; }
    double* find(uint64_t k) {
      for (uint64_t q = h(k) & mask;; q = (q + 1) & mask) {
        if (key[q] == k) return &v[q];
        if (key[q] == 0) return nullptr;
      }
    }
    void put(uint64_t k, double x) {
      if (2 * (n + 1) > key.size()) grow();
      uint64_t q = h(k) & mask;
      while (key[q] != 0 && key[q] != k) q = (q + 1) & mask;
      if (key[q] == 0) ++n;
      key[q] = k;
      v[q] = x;
    }
    void grow() {
      std::vector<uint64_t> ok(key.size() * 2, 0);
      std::vector<double> ov(key.size() * 2);
      ok.swap(key);
      ov.swap(v);
      mask = key.size() - 1;
      n = 0;
      for (size_t q = 0; q < ok.size(); ++q)
        if (ok[q]) put(ok[q], ov[q]);
    }
  };
  struct Replay {
    DyMuPathPlanner& pl;
    TieGuard guard;                // this thread's copy (near ties counted here)
    Order po;
    const double* F;
    int64_t NX, NY;
    uint64_t last;                 // the exit moment
    double lim;                    // closed_limit_ (T(last))
    const std::vector<uint64_t>& open;  // open_at_limit_
    uint64_t budget;               // upd evaluations left before giving up
    Memo memo;                     // upd(k, s), keyed k * 4 + s + 1
    Memo bmemo;                    // band values at the exit, keyed k + 1
    uint64_t band_k = ~0ull;       // the band cell being evaluated at the exit
    bool overrun = false;          // the budget or the depth bound was hit

    Replay(DyMuPathPlanner& p, const TieGuard& g, uint64_t gl, uint64_t lst, uint64_t b)
        : pl(p), guard(g), po(MapT{&p}, p.nx_, p.ny_, gl, &guard),
          F(p.speed_.data()), NX(p.nx_), NY(p.ny_), last(lst), lim(p.closed_limit_),
          open(p.open_at_limit_), budget(b) {
      guard.near = 0;
    }
    bool in_grid(int64_t i, int64_t j) const { return i >= 0 && j >= 0 && i < NX && j < NY; }
    double tv(int64_t i, int64_t j) const { return pl.T((uint64_t)(j * NX + i)); }
    // closedCell with T already loaded (node_state_ is empty here: propagate cleared it)
    bool closed(uint64_t k, double t) {
      if (!(t < kInf)) return false;
      const int c = guard.cmp(k, t, last, lim);
      if (c != 0) return c < 0;
      return open.empty() || !std::binary_search(open.begin(), open.end(), k);
    }
    // value of (i, j) if it is CLOSED by moment c (value tc), else +inf
    double closed_by(int64_t i, int64_t j, uint64_t c, double tc) {
      if (!in_grid(i, j)) return kInf;
      const uint64_t k = (uint64_t)(j * NX + i);
      const double t = tv(i, j);
      if (!closed(k, t)) return kInf;
      if (k == c) return t;
      const int r = guard.cmp(k, t, c, tc);
      if (r != 0) return r < 0 ? t : kInf;
      return po.popBefore(k, c) ? t : kInf;
    }
    // the reference update (:504-535), -ffp-contract=off
    static double eikonal(double tx, double ty, double C) {
      if ((std::fabs(tx - ty) < C) && (tx < kInf) && (ty < kInf))
        return (tx + ty + std::sqrt(2 * (C * C) - (tx - ty) * (tx - ty))) / 2;
      return std::fmin(tx, ty) + C;
    }
    double axis(int64_t ia, int64_t ja, int64_t ib, int64_t jb, uint64_t m, double tm,
                int depth) {
      const double a = closed_by(ia, ja, m, tm), b = closed_by(ib, jb, m, tm);
      if (a < kInf || b < kInf) return std::fmin(a, b);  // OPEN sides are >= T(m) >= it
      const double va = in_grid(ia, ja) ? val(ia, ja, m, tm, depth + 1) : kInf;
      const double vb = in_grid(ib, jb) ? val(ib, jb, m, tm, depth + 1) : kInf;
      return std::fmin(va, vb);
    }
    // val(k, c) = min over the nb4 m of k popped by moment c of upd(k, m): the update
    // of k by m's pop depends on m alone, so it is memoised per (k, m) -- at most four
    // per cell -- and a value at any moment is a min over at most four of them.  When
    // every neighbour that updates k before k's own pop (a CLOSED k) or before the exit
    // (a band k) has been popped by c, the value at c is that final one: T(k), or k's
    // band value -- which cuts the walk back through the front's history short
    double val(int64_t i, int64_t j, uint64_t c, double tc, int depth) {
      const uint64_t k = (uint64_t)(j * NX + i);
      if (!(F[k] < kInf)) return kInf;  // obstacles are never updated
      const int64_t nb[4][2] = {{i, j - 1}, {i - 1, j}, {i + 1, j}, {i, j + 1}};
      const double tk = tv(i, j);
      const bool kc = closed(k, tk);
      bool all = true;
      double byc[4];
      for (int s = 0; s < 4; ++s) {
        byc[s] = closed_by(nb[s][0], nb[s][1], c, tc);
        if (byc[s] < kInf || !all || !in_grid(nb[s][0], nb[s][1])) continue;
        // a neighbour not popped by c: does it update k before k's value is final?
        const uint64_t n = (uint64_t)(nb[s][1] * NX + nb[s][0]);
        if (kc ? n != k && closed_by(nb[s][0], nb[s][1], k, tk) < kInf
               : closed(n, tv(nb[s][0], nb[s][1])))
          all = false;
      }
      if (all && kc) return tk;
      if (all && k != band_k) return bandval(i, j, depth);
      double v = kInf;
      for (int s = 0; s < 4; ++s)
        if (byc[s] < kInf) v = std::fmin(v, upd(i, j, s, depth));
      return v;
    }
    // a band cell's value at the exit, memoised
    double bandval(int64_t i, int64_t j, int depth) {
      const uint64_t k = (uint64_t)(j * NX + i);
      if (const double* hit = bmemo.find(k + 1)) return *hit;
      const uint64_t saved = band_k;
      band_k = k;
      const double v = val(i, j, last, lim, depth + 1);
      band_k = saved;
      bmemo.put(k + 1, v);
      return v;
    }
    // the reference update of k at the pop of its neighbour in nb4 slot s (:462-465)
    double upd(int64_t i, int64_t j, int s, int depth) {
      const uint64_t k = (uint64_t)(j * NX + i);
      const uint64_t key = k * 4 + (uint64_t)s + 1;
      if (const double* hit = memo.find(key)) return *hit;
      if (depth > 3000 || budget == 0) {  // give up (~1 MB of stack)
        overrun = true;
        return tv(i, j);
      }
      --budget;
      memo.put(key, kInf);  // (pops only go back in time: never re-entered)
      const int64_t mi = s == 1 ? i - 1 : s == 2 ? i + 1 : i;
      const int64_t mj = s == 0 ? j - 1 : s == 3 ? j + 1 : j;
      const uint64_t m = (uint64_t)(mj * NX + mi);
      const double tm = tv(mi, mj);
      const double tx = axis(i - 1, j, i + 1, j, m, tm, depth);
      const double ty = axis(i, j - 1, i, j + 1, m, tm, depth);
      const double v = eikonal(tx, ty, F[k]);
      memo.put(key, v);
      return v;
    }
  };
  const uint64_t g = idx(goal_i_, goal_j_);
  // the work bound (DYMU_REPLAY_BUDGET overrides it: tests of the overrun path)
  static const uint64_t budget = [] {
    const char* kv = std::getenv("DYMU_REPLAY_BUDGET");
    return kv && std::atoll(kv) > 0 ? (uint64_t)std::atoll(kv) : kReplayBudget;
  }();
  out.assign(band.size(), kInf);
  // threads: at least 64 band cells each; the work bound is shared out per thread
  const unsigned nt = std::max(1u, std::min(host_threads(), (unsigned)std::min<uint64_t>(
                                                                 band.size() / 64, 1u << 16)));
  std::vector<uint64_t> used(nt, 0);
  std::vector<TieGuard> tg(nt, guard);  // each thread's guard at its end
  std::vector<uint8_t> bad(nt, 0);
  // runs of band cells taken from a shared counter: the work per cell varies by orders
  // of magnitude along the front (where a staircase front walks far back), so static
  // shares leave most threads idle; a thread keeps its memo across its runs
  const uint64_t run = std::max<uint64_t>(16, band.size() / ((uint64_t)nt * 16));
  std::atomic<uint64_t> next_run{0};
  std::vector<double> tms(nt, 0.0);
  const auto tp0 = std::chrono::steady_clock::now();
  parallel_tasks(nt, [&](unsigned t) {
    const auto tt0 = std::chrono::steady_clock::now();
    struct Stamp {
      double& ms;
      std::chrono::steady_clock::time_point t0;
      ~Stamp() {
        ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      }
    } stamp{tms[t], tt0};
    Replay rec(*this, guard, g, last, std::max<uint64_t>(1, budget / nt));
    for (;;) {
      const uint64_t q0 = next_run.fetch_add(run, std::memory_order_relaxed);
      if (q0 >= band.size() || rec.overrun || rec.po.degenerate()) break;
      const uint64_t q1 = std::min<uint64_t>(band.size(), q0 + run);
      for (uint64_t q = q0; q < q1 && !rec.overrun && !rec.po.degenerate(); ++q)
        out[q] = rec.bandval((int64_t)(band[q] % nx_), (int64_t)(band[q] / nx_), 0);
    }
    used[t] = std::max<uint64_t>(1, budget / nt) - rec.budget;
    tg[t] = rec.guard;
    bad[t] = rec.overrun || rec.po.degenerate();
    if (rec.po.degenerate() && std::getenv("DYMU_ORDER_DEBUG")) {
      const uint64_t k = rec.po.whyCell();
      std::fprintf(stderr, "[dymu] order undetermined: reason %d at (%llu, %llu)\n",
                   rec.po.why(), (unsigned long long)(k % nx_), (unsigned long long)(k / nx_));
    }
  });
  if (std::getenv("DYMU_ORDER_DEBUG")) {
    std::fprintf(stderr, "[dymu] band replay %.1f ms, per thread:",
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0)
                     .count());
    for (unsigned t = 0; t < nt; ++t) std::fprintf(stderr, " %.1f/%llu", tms[t], (unsigned long long)used[t]);
    std::fprintf(stderr, "\n");
  }
  early_info_.replay_threads = nt;
  early_info_.replay_updates = 0;
  bool give_up = false;
  for (unsigned t = 0; t < nt; ++t) {
    early_info_.replay_updates += used[t];
    if (!guard.near && tg[t].near) {
      std::copy(tg[t].first, tg[t].first + 2, guard.first);
      std::copy(tg[t].first_t, tg[t].first_t + 2, guard.first_t);
    }
    guard.near += tg[t].near;
    give_up = give_up || bad[t];
  }
  return give_up || guard.near > 0;
}

// band_cells_ after a GPU early exit are in grid order: put them in the reference's
// insertion order (pop_order.hpp) before anyone reads the order.  (The exit has
// already checked the order for near ties: the exact replay ran otherwise.)
void DyMuPathPlanner::orderBand() {
  if (!band_unordered_) return;
  band_unordered_ = false;
  PopOrder<MapT> po(MapT{this}, nx_, ny_, idx(goal_i_, goal_j_));
  std::vector<uint64_t> b(band_cells_);
  std::stable_sort(b.begin(), b.end(),
                   [&po](uint64_t x, uint64_t y) { return po.insBefore(x, y); });
  if (!po.degenerate()) band_cells_.swap(b);  // else keep grid order
}

// The reference FMM replayed exactly on the host: its band as a heap keyed (T,
// first-insertion sequence) -- the pops of the first-strict-minimum scan (:551-568) in
// the same order -- from the goal until the start (si, sj) and its nb4 are CLOSED
// (computeTotalCostMap :364-408; si < 0: until the band empties, :443-468).  It runs
// over a box (inclusive; empty: the whole grid): every cell the reference pops at the
// exit has a value at most t_closed, and the caller's box holds every cell the engine
// puts below t_closed (1 + kRegionMargin) plus a ring; a pop whose neighbour lies
// outside it means the box was short, and the replay restarts on the whole grid.
// The box is stored with a one-cell ring at +inf: off the grid that is the reference's
// "the other neighbour alone" (:504-523, fmin(+inf, x) = x), off the box "never
// reached"; the ring's state says which (4: off the grid, never a neighbour; 3: outside
// the box).  The band is a radix heap (BandQueue below); each pop prefetches the next
// one's neighbourhood while it updates its own.
// O(m log m) for the m cells the reference reaches.
namespace {
// The band in the reference's pop order -- least value, equal values by first insertion
// -- as a radix heap on the values' bit patterns (a non-negative double orders as its
// bits): bucket b > 0 holds the keys whose highest bit differing from the last popped
// key is bit b - 1; `eq` (a heap on the sequence) the keys equal to it.  Every value the
// replay inserts is at least the last popped one in exact arithmetic; one rounded below
// it goes to `below` (a heap on value, then sequence), popped first.  A lowered value
// is pushed again and the entry it supersedes is skipped when popped (its value is no
// longer the cell's).
struct BandQueue {
  struct E {
    uint64_t key, seq, p, k;  // value bits, first insertion, box-local index, grid index
  };
  std::vector<E> b[65], eq, below;
  uint64_t last = 0;
  static bool seq_after(const E& x, const E& y) { return x.seq > y.seq; }
  static bool after(const E& x, const E& y) {
    return x.key > y.key || (x.key == y.key && x.seq > y.seq);
  }
  void push(const E& e) {
    if (e.key < last) {
      below.push_back(e);
      std::push_heap(below.begin(), below.end(), after);
    } else if (e.key == last) {
      eq.push_back(e);
      std::push_heap(eq.begin(), eq.end(), seq_after);
    } else {
      b[64 - __builtin_clzll(e.key ^ last)].push_back(e);
    }
  }
  // the entry the next pop returns (nullptr: empty); the least key's bucket is spread
  // over the lower ones when `eq` has run dry
  const E* next() {
    if (!below.empty()) return &below.front();
    if (eq.empty()) {
      int i = 1;
      while (i <= 64 && b[i].empty()) ++i;
      if (i > 64) return nullptr;
      uint64_t mn = ~0ull;
      for (const E& e : b[i]) mn = std::min(mn, e.key);
      last = mn;
      std::vector<E> v;
      v.swap(b[i]);
      for (const E& e : v) push(e);  // each goes to a bucket below i, or to eq
      v.clear();
      b[i].swap(v);  // the bucket keeps its buffer
    }
    return &eq.front();
  }
  bool pop(E& out) {
    if (!next()) return false;
    const bool lo = !below.empty();
    std::vector<E>& h = lo ? below : eq;
    std::pop_heap(h.begin(), h.end(), lo ? after : seq_after);
    out = h.back();
    h.pop_back();
    return true;
  }
};

uint64_t value_bits(double t) {
  uint64_t u;
  std::memcpy(&u, &t, sizeof u);
  return u;
}
}  // namespace

DyMuPathPlanner::HostFmm DyMuPathPlanner::hostFmm(int64_t si, int64_t sj,
                                                  const int64_t box_in[4]) const {
  const double* F = speed_.data();
  HostFmm r;
  r.bx[0] = r.bx[1] = 0;
  r.bx[2] = (int64_t)nx_ - 1;
  r.bx[3] = (int64_t)ny_ - 1;
  if (box_in && box_in[0] <= box_in[2]) {  // the region grown by two more cells
    r.bx[0] = std::max<int64_t>(0, box_in[0] - 2);
    r.bx[1] = std::max<int64_t>(0, box_in[1] - 2);
    r.bx[2] = std::min<int64_t>(nx_ - 1, box_in[2] + 2);
    r.bx[3] = std::min<int64_t>(ny_ - 1, box_in[3] + 2);
  }
  for (;;) {
    const int64_t* bx = r.bx;
    const int64_t W = bx[2] - bx[0] + 1, H = bx[3] - bx[1] + 1, PW = W + 2;
    r.W = W;
    r.PW = PW;
    const uint64_t m = (uint64_t)PW * (uint64_t)(H + 2);
    r.T.assign(m, kInf);
    r.st.assign(m, 0);  // 1 CLOSED, 2 in the band; the ring 3 / 4
    {
      const uint8_t s_lo = bx[1] > 0 ? 3 : 4, s_hi = bx[3] + 1 < (int64_t)ny_ ? 3 : 4;
      const uint8_t w_lo = bx[0] > 0 ? 3 : 4, w_hi = bx[2] + 1 < (int64_t)nx_ ? 3 : 4;
      for (int64_t c = 0; c < PW; ++c) {
        r.st[(uint64_t)c] = s_lo;
        r.st[(uint64_t)(H + 1) * PW + c] = s_hi;
      }
      for (int64_t q = 1; q <= H; ++q) {
        r.st[(uint64_t)q * PW] = w_lo;
        r.st[(uint64_t)q * PW + W + 1] = w_hi;
      }
    }
    r.order.clear();
    // each band cell's first-insertion sequence (32 bits while the box allows)
    const bool wide = m >= (1ull << 32);
    std::vector<uint32_t> seq32(wide ? 0 : m);
    std::vector<uint64_t> seq64(wide ? m : 0);
    BandQueue band;
    double* T = r.T.data();
    uint8_t* st = r.st.data();
    const uint64_t g = r.at(goal_i_, goal_j_);
    T[g] = 0.0;
    r.order.push_back(idx(goal_i_, goal_j_));
    st[g] = 2;
    band.push({value_bits(0.0), 0, g, idx(goal_i_, goal_j_)});
    r.band = 1;
    bool short_box = false;
    const bool early = si >= 0;
    const uint64_t sl = early ? r.at(si, sj) : 0;
    auto fully_closed = [&] {  // :424-436 (the start is interior: safeNode)
      return early && st[sl] == 1 && st[sl - PW] == 1 && st[sl - 1] == 1 && st[sl + 1] == 1 &&
             st[sl + PW] == 1;
    };
    const int64_t dp[4] = {-PW, -1, 1, PW};  // nb4 order (:76-80)
    const int64_t dk[4] = {-(int64_t)nx_, -1, 1, (int64_t)nx_};
    BandQueue::E top;
    while (r.band > 0 && !fully_closed() && !short_box && band.pop(top)) {
      const uint64_t p = top.p, kp = top.k;
      if (st[p] != 2 || value_bits(T[p]) != top.key) continue;  // a superseded entry
      st[p] = 1;
      --r.band;
      if (const BandQueue::E* nx = band.next()) {  // its neighbourhood, fetched meanwhile
        const uint64_t np = nx->p, nk = nx->k;
        const int64_t NX = (int64_t)nx_, mb = (int64_t)m - 1, ng = (int64_t)nx_ * ny_ - 1;
        auto in = [](int64_t x, int64_t hi) { return x < 0 ? 0 : x > hi ? hi : x; };
        const int64_t dt[8] = {-2 * PW, -PW - 1, -PW + 1, -1, 1, PW - 1, PW + 1, 2 * PW};
        for (const int64_t d : dt) __builtin_prefetch(T + in((int64_t)np + d, mb));
        const int64_t ds[3] = {-PW, 0, PW}, df[3] = {-NX, 0, NX};
        for (const int64_t d : ds) __builtin_prefetch(st + in((int64_t)np + d, mb));
        for (const int64_t d : df) __builtin_prefetch(F + in((int64_t)nk + d, ng));
      }
      for (int s = 0; s < 4; ++s) {
        const uint64_t q = p + dp[s];
        const uint8_t sq = st[q];
        if (sq == 1 || sq == 4) continue;
        if (sq == 3) {
          short_box = true;  // the reference reaches beyond the box
          break;
        }
        const uint64_t kq = kp + dk[s];
        const double C = F[kq];
        if (!(C < kInf)) continue;
        // propagateGlobalNode (:500-546) from the current values
        const double Ty = std::fmin(T[q + PW], T[q - PW]);
        const double Tx = std::fmin(T[q - 1], T[q + 1]);
        double u;
        if ((std::fabs(Tx - Ty) < C) && (Tx < kInf) && (Ty < kInf))
          u = (Tx + Ty + std::sqrt(2 * (C * C) - ((Tx - Ty) * (Tx - Ty)))) / 2;
        else
          u = std::fmin(Tx, Ty) + C;
        if (!(u < T[q])) continue;
        uint64_t seq;
        if (T[q] == kInf) {  // first reached: into the band and the propagated list
          seq = r.order.size();
          if (wide)
            seq64[q] = seq;
          else
            seq32[q] = (uint32_t)seq;
          r.order.push_back(kq);
          st[q] = 2;
          ++r.band;
        } else {
          seq = wide ? seq64[q] : seq32[q];
        }
        T[q] = u;
        band.push({value_bits(u), seq, q, kq});
      }
    }
    if (short_box && !(bx[0] == 0 && bx[1] == 0 && bx[2] == nx_ - 1 && bx[3] == ny_ - 1)) {
      if (std::getenv("DYMU_ORDER_DEBUG"))
        std::fprintf(stderr, "[dymu] exact replay: box short, restarting on the whole grid\n");
      r.bx[0] = r.bx[1] = 0;
      r.bx[2] = (int64_t)nx_ - 1;
      r.bx[3] = (int64_t)ny_ - 1;
      continue;
    }
    return r;
  }
}

// computeTotalCostMap's exit replayed exactly on the host (hostFmm) over the region
// box -- when the values cannot decide the reference's order at the exit (near ties,
// degenerate ties) or the band replay hit its work bound.  The map, the node states,
// the band (insertion order) and global_propagated_nodes become the reference's.
bool DyMuPathPlanner::exactEarlyExit(unsigned si, unsigned sj, const int64_t box[4]) {
  const uint64_t n = (uint64_t)nx_ * ny_;
  HostFmm r = hostFmm(si, sj, box);
  const int64_t* bx = r.bx;
  std::fill(total_cost_.begin(), total_cost_.end(), kInf);
  node_state_.assign(n, 0);
  for (int64_t j = bx[1]; j <= bx[3]; ++j)
    for (int64_t i = bx[0]; i <= bx[2]; ++i) {
      const uint64_t k = r.at(i, j);
      const uint64_t kg = idx((unsigned)i, (unsigned)j);
      total_cost_[kg] = r.T[k];
      node_state_[kg] = r.st[k] == 1 ? 1 : 0;
    }
  std::fill(blk_ok_.begin(), blk_ok_.end(), 1);
  blk_missing_ = 0;
  if (dymu_memcpy_h2d(ctx_, dT_, total_cost_.data(), sizeof(double) * n) != DYMU_OK)
    throw std::runtime_error(std::string("dymu: total-cost upload failed: ") +
                             dymu_last_error(ctx_));
  band_cells_.clear();
  band_unordered_ = false;
  band_values_checked_ = true;
  open_at_limit_.clear();
  for (const uint64_t kg : r.order)
    if (!node_state_[kg]) band_cells_.push_back(kg);  // the reference's band vector, in order
  propagated_extra_.swap(r.order);
  manual_list_ = true;
  solved_ = false;
  return r.band > 0;  // :399-407
}

// global_propagated_nodes (:447, :537-545) after a GPU solve: every reached node in
// the order the reference inserted it, rebuilt from the values like the band's order
// (pop_order.hpp) but for all nodes at once -- the popped (CLOSED) nodes ranked by value,
// equal values by insertion; a node's insertion keyed by the rank of its first-popped
// neighbour (its least CLOSED one) and its slot in that neighbour's nb4 list.  Near ties
// (TieGuard) or an undetermined order: the reference's FMM is replayed on the host for
// the order (hostFmm; its values are not installed).
std::vector<uint64_t> DyMuPathPlanner::insertionOrder() {
  fetchAll();
  const uint64_t n = (uint64_t)nx_ * ny_;
  const double* t = total_cost_.data();
  const uint64_t g = idx(goal_i_, goal_j_);
  std::vector<uint64_t> reached;
  for (uint64_t k = 0; k < n; ++k)
    if (t[k] < kInf) reached.push_back(k);
  // the constant-speed radius around the goal (TieGuard): mirror ties trusted within
  const double f0 = speed_[g];
  double d2 = kInf;
  for (uint64_t k = 0; k < n; ++k)
    if (speed_[k] != f0) {
      const double di = (double)(k % nx_) - goal_i_, dj = (double)(k / nx_) - goal_j_;
      d2 = std::fmin(d2, di * di + dj * dj);
    }
  TieGuard guard(nx_, goal_i_, goal_j_, f0, std::sqrt(d2));
  // DYMU_EXACT_EXIT=1 sends the list to the exact replay too (tests of that path).  So
  // does a list of more than 2^23 nodes: among that many values some two lie within 1e-12
  // of each other (tens of such pairs are expected; none has been seen missing), so the
  // sort below would only find that out
  static const bool force_exact = [] {
    const char* kv = std::getenv("DYMU_EXACT_EXIT");
    return kv && std::atoi(kv) != 0;
  }();
  std::vector<std::pair<double, uint64_t>> popped;
  const bool large = reached.size() > (1ull << 23);
  if (!force_exact && !large) {
    for (const uint64_t k : reached)
      if (closedCell(k)) popped.push_back({t[k], k});
    parallel_sort(popped);
  }
  bool undetermined = force_exact || large || popped.empty() || popped[0].second != g;
  // near ties between consecutive values first (on the host threads): any one of them
  // leaves the pop order to the exact replay, and the keys below would be wasted (the
  // sorted values' mean spacing falls with the cell count: from ~2^22 reached cells on
  // generic terrain some pair lies within 1e-12 of each other)
  {
    const uint64_t m = popped.size();
    const unsigned nt = std::max(1u, std::min(host_threads(), (unsigned)std::min<uint64_t>(m >> 16, 64)));
    std::vector<uint64_t> near(nt, 0);
    parallel_tasks(nt, [&](unsigned th) {
      TieGuard gd(guard);
      gd.near = 0;
      const uint64_t q0 = std::max<uint64_t>(1, m * th / nt), q1 = m * (th + 1) / nt;
      for (uint64_t q = q0; q < q1; ++q)
        if (popped[q].first != popped[q - 1].first)
          (void)gd.cmp(popped[q - 1].second, popped[q - 1].first, popped[q].second, popped[q].first);
      near[th] = gd.near;
    });
    for (const uint64_t x : near) guard.near += x;
  }
  if (guard.near > 0) undetermined = true;
  std::vector<uint64_t> rank(undetermined ? 0 : n, ~0ull);
  // x's first-popped neighbour (least value, equal ones by rank) and x's slot in its list;
  // false when none is ranked (x ties with its least neighbour: undetermined)
  auto first_popped = [&](uint64_t x, uint64_t& key, TieGuard& gd) {
    const unsigned i = (unsigned)(x % nx_), j = (unsigned)(x / nx_);
    uint64_t nb[4];
    int slot[4], m = 0;  // x's slot in nb's list: (i,j-1) sees x as its (i,j+1): 3, ...
    if (j > 0) nb[m] = x - nx_, slot[m++] = 3;
    if (i > 0) nb[m] = x - 1, slot[m++] = 2;
    if (i + 1 < nx_) nb[m] = x + 1, slot[m++] = 1;
    if (j + 1 < ny_) nb[m] = x + nx_, slot[m++] = 0;
    int best = -1;
    for (int q = 0; q < m; ++q) {
      if (rank[nb[q]] == ~0ull) continue;
      if (best < 0) {
        best = q;
        continue;
      }
      const int c = gd.cmp(nb[q], t[nb[q]], nb[best], t[nb[best]]);
      if (c < 0 || (c == 0 && rank[nb[q]] < rank[nb[best]])) best = q;
    }
    if (best < 0) return false;
    if (gd.cmp(nb[best], t[nb[best]], x, t[x]) >= 0) return false;
    key = rank[nb[best]] * 4 + (uint64_t)slot[best];
    return true;
  };
  // pop ranks: value order; a group of equal values in insertion order (a lone value
  // needs no key: its checks run with every node's below)
  uint64_t next = 0;
  std::vector<std::pair<uint64_t, uint64_t>> grp;
  for (size_t a = 0; a < popped.size() && !undetermined;) {
    size_t b = a + 1;
    while (b < popped.size() && popped[b].first == popped[a].first) ++b;
    if (b == a + 1) {
      rank[popped[a].second] = next++;
      a = b;
      continue;
    }
    grp.clear();
    for (size_t q = a; q < b; ++q) {
      const uint64_t x = popped[q].second;
      if (q > a) (void)guard.cmp(popped[a].second, popped[a].first, x, popped[q].first);
      uint64_t key = 0;
      if (x != g && !first_popped(x, key, guard)) undetermined = true;
      grp.push_back({x == g ? 0 : key + 1, x});
    }
    std::sort(grp.begin(), grp.end());
    for (const auto& e : grp) rank[e.second] = next++;
    a = b;
  }
  popped = {};
  // every reached node keyed by its first-popped neighbour's rank and slot, on the host
  // threads (each with its own guard; their near ties are summed)
  std::vector<std::pair<uint64_t, uint64_t>> ins;
  if (!undetermined) {
    ins.resize(reached.size());
    const unsigned nt = std::max(
        1u, std::min(host_threads(), (unsigned)std::min<uint64_t>(reached.size() >> 16, 64)));
    std::vector<TieGuard> tg(nt, guard);
    for (auto& gd : tg) gd.near = 0;
    std::vector<uint8_t> und(nt, 0);
    std::atomic<bool> stop{false};
    parallel_tasks(nt, [&](unsigned th) {
      const uint64_t q0 = reached.size() * th / nt, q1 = reached.size() * (th + 1) / nt;
      for (uint64_t q = q0; q < q1 && !stop.load(std::memory_order_relaxed); ++q) {
        const uint64_t x = reached[q];
        uint64_t key = 0;
        if (x != g && !first_popped(x, key, tg[th])) {
          und[th] = 1;
          stop.store(true, std::memory_order_relaxed);
        }
        ins[q] = {x == g ? 0 : key + 1, x};
      }
    });
    for (unsigned th = 0; th < nt; ++th) {
      guard.near += tg[th].near;
      undetermined = undetermined || und[th];
    }
  }
  std::vector<uint64_t> order;
  if (undetermined || guard.near > 0) {  // the reference's own order, replayed
    const int64_t none[4] = {0, 0, -1, -1};
    const bool early = closed_limit_ < kInf && have_start_;
    HostFmm r = hostFmm(early ? (int64_t)start_i_ : -1, early ? (int64_t)start_j_ : -1,
                        early ? exit_box_ : none);
    order.swap(r.order);
  } else {
    parallel_sort(ins);
    order.reserve(ins.size());
    for (const auto& e : ins) order.push_back(e.second);
  }
  return order;
}

void DyMuPathPlanner::copyNodeStates(uint8_t* out) {
  const uint64_t n = (uint64_t)nx_ * ny_;
  if (!node_state_.empty()) {
    std::memcpy(out, node_state_.data(), n);
    return;
  }
  fetchAll();
  for (uint64_t k = 0; k < n; ++k) out[k] = closedCell(k) ? 1 : 0;
}

// :443-468
bool DyMuPathPlanner::computeEntireTotalCostMap() {
  if (!has_goal_ || is_obstacle_[idx(goal_i_, goal_j_)]) {
    log_warn("The goal is not valid");
    return false;
  }
  return propagate(false, 0, 0);
}

// :410-422 (start and its 8 neighbours must be free; border -> false here,
// where the reference dereferences NULL)
bool DyMuPathPlanner::safeNode(unsigned i, unsigned j) const {
  if (i == 0 || j == 0 || i + 1 >= nx_ || j + 1 >= ny_) return false;
  for (int dj = -1; dj <= 1; ++dj)
    for (int di = -1; di <= 1; ++di)
      if (is_obstacle_[idx(i + di, j + dj)]) return false;
  return true;
}

// :364-408.  The propagation stops once the start node and its nb4 are final
// (dymu_solve_until_device); the return value is the reference's: false iff
// the narrow band is empty at that moment (the start is unreachable, or its
// neighbourhood closed last of all the reachable nodes).
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
  const unsigned si = grid_u32(fx), sj = grid_u32(fy);
  if (!safeNode(si, sj)) {
    log_error("PLANNER: The rover is located too close to an obstacle");
    return false;
  }
  if (!propagate(true, si, sj)) {
    log_error("The goal is unreachable");
    return false;
  }
  return true;
}

// :589-611 (evaluatePath(0) repairs the segments through local risk; it is the
// identity while no global node is subdivided)
std::vector<base::Waypoint> DyMuPathPlanner::getPath(base::Waypoint wPos) {
  wPos.position[0] -= global_offset_[0];
  wPos.position[1] -= global_offset_[1];
  computeGlobalPath(wPos);
  evaluatePath(0);
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
  const unsigned cx = grid_u32(gx), cy = grid_u32(gy);
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

void DyMuPathPlanner::gradientNode(const globalNode& n, double& dnx, double& dny) const {
  const double i = n.pose.position[0], j = n.pose.position[1];
  if (!(i >= 0 && j >= 0 && i < nx_ && j < ny_)) {
    dnx = dny = 0;
    return;
  }
  gradientNode((unsigned)i, (unsigned)j, dnx, dny);
}

// :718-772
void DyMuPathPlanner::gradientNode(unsigned i, unsigned j, double& dnx, double& dny) const {
  const uint64_t k = idx(i, j);
  const bool hw = i > 0, he = i + 1 < nx_, hs = j > 0, hn = j + 1 < ny_;
  const double tw = hw ? T(k - 1) : kInf, te = he ? T(k + 1) : kInf;
  const double ts = hs ? T(k - nx_) : kInf, tn = hn ? T(k + nx_) : kInf;
  const double t = T(k);
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
  const unsigned i = grid_u32(x / global_res_ + 0.5), j = grid_u32(y / global_res_ + 0.5);
  if (i >= nx_ || j >= ny_) return "DONT_CARE";
  const int m = loc_mode_[idx(i, j)];
  if (m < 0 || m >= (int)locomotion_modes_.size()) return "DONT_CARE";
  return locomotion_modes_[m];
}

// :799-811
std::vector<std::vector<double>> DyMuPathPlanner::getTotalCostMatrix() {
  std::vector<std::vector<double>> m(ny_);
  parallel_rows(ny_, [&](unsigned j0, unsigned j1) {
    for (unsigned j = j0; j < j1; ++j) m[j].resize(nx_);
  });
  streamTotalCost([&](unsigned r0, unsigned r1) {
    parallel_rows(r1 - r0, [&](unsigned j0, unsigned j1) {
      for (unsigned j = r0 + j0; j < r0 + j1; ++j) {
        const double* t = &total_cost_[idx(0, j)];
        std::vector<double>& r = m[j];
        for (unsigned i = 0; i < nx_; ++i) r[i] = (t[i] == kInf) ? -1.0 : t[i];
      }
    });
  });
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
  const unsigned i = grid_u32(x / global_res_), j = grid_u32(y / global_res_);
  const double a = x - (double)i, b = y - (double)j;
  if (i >= nx_ || j >= ny_ || i + 1 >= nx_ || j + 1 >= ny_) {  // a corner is NULL
    const unsigned ni = grid_u32(x / global_res_ + 0.5), nj = grid_u32(y / global_res_ + 0.5);
    if (ni >= nx_ || nj >= ny_) return kInf;
    return T(idx(ni, nj));
  }
  const uint64_t k = idx(i, j);
  const uint64_t k10 = k + 1, k01 = k + nx_, k11 = k + nx_ + 1;
  if (!closedCell(k) || !closedCell(k10) || !closedCell(k01) || !closedCell(k11)) {
    const unsigned ni = grid_u32(x / global_res_ + 0.5), nj = grid_u32(y / global_res_ + 0.5);
    return T(idx(ni, nj));
  }
  const double w00 = T(k), w10 = T(k10);
  const double w01 = T(k01), w11 = T(k11);
  return w00 + (w10 - w00) * a + (w01 - w00) * b + (w11 + w00 - w10 - w01) * a * b;
}

// ---- node-level access (src/DyMu.hpp:500-518) ----

std::optional<globalNode> DyMuPathPlanner::snapshot(uint64_t k) {
  globalNode n;
  const unsigned i = (unsigned)(k % nx_), j = (unsigned)(k / nx_);
  n.pose.position[0] = (double)i;
  n.pose.position[1] = (double)j;
  if (has_goal_ && i == goal_i_ && j == goal_j_) n.pose.orientation = goal_heading_;
  n.world_pose.position[0] = (double)i * global_res_;  // globalNode ctor (src/DyMu.hpp:92-93)
  n.world_pose.position[1] = (double)j * global_res_;
  n.elevation = elevation_[k];
  n.slope = slope_[k];
  n.state = closedCell(k) ? CLOSED : OPEN;
  n.isObstacle = is_obstacle_[k] != 0;
  n.hasLocalMap = local_ && local_->block(k) >= 0;
  n.raw_cost = raw_cost_[k];
  n.cost = cost_[k];
  n.hazard_density = hazard_[k];
  n.trafficability = traff_[k];
  n.total_cost = T(k);
  n.terrain = terrain_[k];
  const int m = loc_mode_[k];
  n.nodeLocMode = (m < 0 || m >= (int)locomotion_modes_.size()) ? "DONT_CARE" : locomotion_modes_[m];
  return n;
}

// :313-317
std::optional<globalNode> DyMuPathPlanner::getGlobalNode(unsigned i, unsigned j) {
  if (i >= nx_ || j >= ny_) return std::nullopt;
  return snapshot(idx(i, j));
}

// :570-584
std::optional<globalNode> DyMuPathPlanner::getNearestGlobalNode(base::Pose2D pos) {
  const int64_t k = nearestIndex(pos.position[0], pos.position[1]);
  if (k < 0) return std::nullopt;
  return snapshot((uint64_t)k);
}

std::optional<globalNode> DyMuPathPlanner::getNearestGlobalNode(base::Waypoint wPos) {
  const int64_t k = nearestIndex(wPos.position[0], wPos.position[1]);
  if (k < 0) return std::nullopt;
  return snapshot((uint64_t)k);
}

std::optional<globalNode> DyMuPathPlanner::globalGoal() {
  if (!has_goal_) return std::nullopt;
  return snapshot(idx(goal_i_, goal_j_));
}

bool DyMuPathPlanner::isSafeNode(unsigned i, unsigned j) { return safeNode(i, j); }

// :424-436 (a border node returns false where the reference dereferences NULL)
bool DyMuPathPlanner::isFullyClosedNode(unsigned i, unsigned j) {
  if (i == 0 || j == 0 || i + 1 >= nx_ || j + 1 >= ny_) return false;
  const uint64_t k = idx(i, j);
  return closedCell(k) && closedCell(k - nx_) && closedCell(k - 1) && closedCell(k + 1) &&
         closedCell(k + nx_);
}

// :473-485: every node OPEN at +inf, global_propagated_nodes cleared
void DyMuPathPlanner::resetTotalCostMap() {
  std::fill(total_cost_.begin(), total_cost_.end(), kInf);
  std::fill(blk_ok_.begin(), blk_ok_.end(), 1);
  blk_missing_ = 0;
  closed_limit_ = 0.0;
  band_cells_.clear();
  band_unordered_ = false;
  band_values_checked_ = true;
  open_at_limit_.clear();
  node_state_.assign(total_cost_.size(), 0);
  propagated_extra_.clear();
  manual_list_ = true;
  solved_ = false;
}

// the node states of the last solve made explicit, so a caller can change some
void DyMuPathPlanner::materializeStates() {
  if (!node_state_.empty()) return;
  fetchAll();
  std::vector<uint8_t> st(total_cost_.size());
  for (uint64_t k = 0; k < st.size(); ++k) st[k] = closedCell(k) ? 1 : 0;
  node_state_ = std::move(st);
}

void DyMuPathPlanner::setGlobalNodeState(unsigned i, unsigned j, node_state s) {
  if (i >= nx_ || j >= ny_) return;
  settleBand();
  materializeStates();
  node_state_[idx(i, j)] = s == CLOSED ? 1 : 0;
}

// :500-546, on the host copy of the map (made whole first, so no later download
// of device blocks can overwrite what this writes)
void DyMuPathPlanner::propagateGlobalNode(unsigned i, unsigned j) {
  if (i >= nx_ || j >= ny_) return;
  settleBand();
  orderBand();  // from the solve's values, before this changes any
  fetchAll();
  const uint64_t k = idx(i, j);
  const double* t = total_cost_.data();
  const bool n0 = j > 0, n3 = j + 1 < ny_, n1 = i > 0, n2 = i + 1 < nx_;
  // a NULL neighbour: the other one alone (:504-523); none at all (a 1-wide grid, a
  // NULL dereference in the reference): +inf
  double Ty, Tx;
  if (n0 && n3)
    Ty = std::fmin(t[k + nx_], t[k - nx_]);
  else if (!n0)
    Ty = n3 ? t[k + nx_] : kInf;
  else
    Ty = t[k - nx_];
  if (n1 && n2)
    Tx = std::fmin(t[k - 1], t[k + 1]);
  else if (!n1)
    Tx = n2 ? t[k + 1] : kInf;
  else
    Tx = t[k - 1];
  const double C = global_res_ * (cost_[k]) * (2 + hazard_[k] - traff_[k]);  // :527-528
  double Tn;
  if ((std::fabs(Tx - Ty) < C) && (Tx < kInf) && (Ty < kInf))
    Tn = (Tx + Ty + std::sqrt(2 * (C * C) - ((Tx - Ty) * (Tx - Ty)))) / 2;  // pow(., 2.0) == x*x
  else
    Tn = std::fmin(Tx, Ty) + C;
  if (Tn < total_cost_[k]) {
    if (total_cost_[k] == kInf) {
      propagated_extra_.push_back(k);
      band_cells_.push_back(k);  // insertion order, as the reference's vector
    }
    total_cost_[k] = Tn;
    solved_ = false;  // the device map no longer matches the host's
  }
}

void DyMuPathPlanner::propagateGlobalNode(const globalNode& n) {
  propagateGlobalNode(grid_u32(n.pose.position[0]), grid_u32(n.pose.position[1]));
}

uint64_t DyMuPathPlanner::globalPropagatedCount() {
  if (manual_list_) return propagated_extra_.size();
  uint64_t c = propagated_extra_.size();
  streamTotalCost([&](unsigned r0, unsigned r1) {
    const double* t = total_cost_.data();
    for (uint64_t k = idx(0, r0); k < idx(0, r1); ++k) c += t[k] < kInf ? 1 : 0;
  });
  // nodes propagateGlobalNode made finite are counted in the map already
  return c - propagated_extra_.size();
}

// the reached nodes in the reference's insertion order (insertionOrder: rebuilt from
// the values, or replayed on the host when they cannot decide it), then those
// propagateGlobalNode added since, in the order it added them
std::vector<uint64_t> DyMuPathPlanner::globalPropagatedIndices() {
  std::vector<uint64_t> out;
  if (!manual_list_) {
    out = insertionOrder();
    if (!propagated_extra_.empty()) {
      std::vector<uint8_t> extra(total_cost_.size(), 0);
      for (const uint64_t k : propagated_extra_) extra[k] = 1;
      out.erase(std::remove_if(out.begin(), out.end(), [&](uint64_t k) { return extra[k] != 0; }),
                out.end());
    }
  }
  out.insert(out.end(), propagated_extra_.begin(), propagated_extra_.end());
  return out;
}

std::vector<globalNode> DyMuPathPlanner::globalPropagatedNodes() {
  const std::vector<uint64_t> ks = globalPropagatedIndices();
  std::vector<globalNode> out;
  out.reserve(ks.size());
  for (const uint64_t k : ks) out.push_back(*snapshot(k));
  return out;
}

std::vector<globalNode> DyMuPathPlanner::globalNarrowband() {
  orderBand();
  std::vector<globalNode> out;
  out.reserve(band_cells_.size());
  for (const uint64_t k : band_cells_) out.push_back(*snapshot(k));
  return out;
}

// The band's values after a GPU early exit are the reference's update arithmetic on the
// engine's CLOSED values: equal to the reference's within rounding, so the order of
// minCostGlobalNode's pops is decided by them only if no two are near-tied (TieGuard).
// Checked once, before the first pop or change of the band (it costs a sort); on a near
// tie the exit is replayed exactly on the host and the band and its values become the
// reference's.
void DyMuPathPlanner::settleBand() {
  if (band_values_checked_) return;
  band_values_checked_ = true;
  if (band_cells_.size() < 2) return;
  const uint64_t g = idx(goal_i_, goal_j_);
  TieGuard guard(nx_, goal_i_, goal_j_, speed_[g], exit_r_const_);
  std::vector<std::pair<double, uint64_t>> bv(band_cells_.size());
  for (size_t q = 0; q < bv.size(); ++q) bv[q] = {T(band_cells_[q]), band_cells_[q]};
  std::sort(bv.begin(), bv.end());
  for (size_t q = 1; q < bv.size(); ++q)
    (void)guard.cmp(bv[q - 1].second, bv[q - 1].first, bv[q].second, bv[q].first);
  early_info_.near_ties += guard.near;
  if (guard.near) {
    early_info_.exact_replay = 1;
    (void)exactEarlyExit(start_i_, start_j_, exit_box_);
  }
}

// :548-567 (first strict minimum, then erased from the band)
std::optional<globalNode> DyMuPathPlanner::minCostGlobalNode() {
  settleBand();
  if (band_cells_.empty()) return std::nullopt;
  orderBand();
  size_t best = 0;
  double tmin = T(band_cells_[0]);
  for (size_t q = 1; q < band_cells_.size(); ++q) {
    const double t = T(band_cells_[q]);
    if (t < tmin) {
      tmin = t;
      best = q;
    }
  }
  const uint64_t k = band_cells_[best];
  band_cells_.erase(band_cells_.begin() + (std::ptrdiff_t)best);
  return snapshot(k);
}

// :487-498
void DyMuPathPlanner::resetGlobalNarrowBand() {
  band_cells_.clear();
  band_unordered_ = false;
  band_values_checked_ = true;
  if (!has_goal_ || nx_ == 0) return;
  const uint64_t k = idx(goal_i_, goal_j_);
  (void)T(k);  // the goal's block in the host mirror before the write
  total_cost_[k] = 0.0;
  band_cells_.push_back(k);
  propagated_extra_.push_back(k);  // global_propagated_nodes.push_back(global_goal)
}

bool DyMuPathPlanner::loadTotalCostMap(const double* Tin) {
  const uint64_t n = (uint64_t)nx_ * ny_;
  if (!Tin || n == 0) return false;
  std::memcpy(total_cost_.data(), Tin, sizeof(double) * n);
  std::fill(blk_ok_.begin(), blk_ok_.end(), 1);
  blk_missing_ = 0;
  closed_limit_ = kInf;
  band_cells_.clear();
  band_unordered_ = false;
  band_values_checked_ = true;
  open_at_limit_.clear();
  node_state_.clear();
  propagated_extra_.clear();
  manual_list_ = false;
  solved_ = false;
  if (ctx_ && dT_ && dcells_ == n &&
      dymu_memcpy_h2d(ctx_, dT_, total_cost_.data(), sizeof(double) * n) != DYMU_OK)
    throw std::runtime_error(std::string("dymu: total-cost upload failed: ") +
                             dymu_last_error(ctx_));
  return true;
}

}  // namespace PathPlanning_lib
