// local_layer.cpp -- the DyMu local layer (path repairing around obstacles seen
// by the rover) on the SoA sub-grid of local_layer.hpp.
//
// Host C++: the local layer works on windows of ~10^3-10^5 sub-cells next to
// the rover, serially ordered by its narrow band, and it reads the global
// total cost the MI355X engine produced through the planner's lazily fetched
// host mirror (planner.cpp, T(k)).  Every method follows the reference method
// cited on it (src/DyMu_LocalPathRepairing.cpp, cited :LINE; the global layer
// is src/DyMu_GlobalPathPlanning.cpp, cited G:LINE) with the same arithmetic
// and evaluation order (-ffp-contract=off), so results are bit-identical to
// the oracle restatement (oracle/oracle_local.c, tests/test_local_layer.py).
// Where the reference has undefined behaviour the definitions U1-U5 of
// DESIGN.md s4.7 apply (the oracle defines them the same way).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <limits>

#include "DyMu.hpp"
#include "local_layer.hpp"

namespace PathPlanning_lib {

namespace {
constexpr double kInf = std::numeric_limits<double>::infinity();
constexpr int kMaxLocalSteps = 100000;  // U4

inline double eikonal(double tx, double ty, double C) {
  if ((std::fabs(tx - ty) < C) && (tx < kInf) && (ty < kInf))
    return (tx + ty + std::sqrt(2 * (C * C) - ((tx - ty) * (tx - ty)))) / 2;
  return std::fmin(tx, ty) + C;
}

inline double wdist(const base::Waypoint& a, const base::Waypoint& b) {
  const double dx = a.position[0] - b.position[0], dy = a.position[1] - b.position[1];
  return std::sqrt(dx * dx + dy * dy);
}

base::Waypoint make_wp(double x, double y, double z, double h) {
  base::Waypoint w;
  w.position[0] = x;
  w.position[1] = y;
  w.position[2] = z;
  w.heading = h;
  return w;
}
}  // namespace

// ---- geometry of a sub-cell (createLocalMap, :34-44) ----
namespace {
struct CellPose {
  double px, py;  // parent pose (grid indices)
  double gx, gy;  // global_pose
  double wx, wy;  // world_pose
  unsigned li, lj;
};
inline CellPose cell_pose(const LocalLayer& L, uint64_t p, unsigned nx, double gres) {
  CellPose c;
  const uint64_t g = L.block_g[p / L.rr], q = p % L.rr;
  c.li = (unsigned)(q % L.r);
  c.lj = (unsigned)(q / L.r);
  c.px = (double)(g % nx);
  c.py = (double)(g / nx);
  c.gx = c.px - 0.5 + (0.5 / (double)L.r) + (double)c.li * (1 / (double)L.r);
  c.gy = c.py - 0.5 + (0.5 / (double)L.r) + (double)c.lj * (1 / (double)L.r);
  c.wx = c.gx / gres;
  c.wy = c.gy / gres;
  return c;
}
}  // namespace

// G:570-584 (index of the nearest global node, -1 = NULL)
int64_t DyMuPathPlanner::nearestIndex(double x, double y) const {
  const uint32_t i = grid_u32(x / global_res_ + 0.5), j = grid_u32(y / global_res_ + 0.5);
  if (i >= nx_ || j >= ny_) return -1;
  return (int64_t)idx(i, j);
}

// :150-156
void DyMuPathPlanner::subdivideGlobalNode(unsigned i, unsigned j) {
  if (i >= nx_ || j >= ny_ || !local_) return;  // U1
  LocalLayer& L = *local_;
  const uint64_t g = idx(i, j);
  if (L.block(g) < 0) L.create(g, nx_, ny_);
  static const int d[8][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
  for (const auto& e : d) {
    const uint32_t a = i + (uint32_t)e[0], b = j + (uint32_t)e[1];
    if (a >= nx_ || b >= ny_) continue;
    if (L.block(idx(a, b)) < 0) L.create(idx(a, b), nx_, ny_);
  }
}

// :160-189, by sub-cell id (-1 = NULL)
int64_t DyMuPathPlanner::localAt(double x, double y) {
  const int64_t g = nearestIndex(x, y);
  if (g < 0 || !local_ || local_->r == 0) return -1;  // U1
  const unsigned gi = (unsigned)(g % nx_), gj = (unsigned)(g / nx_);
  subdivideGlobalNode(gi, gj);
  const LocalLayer& L = *local_;
  const double cornerX = (double)gi - global_res_ / 2;
  const double cornerY = (double)gj - global_res_ / 2;
  const double a = x - cornerX, b = y - cornerY;
  const uint32_t li = grid_u32(a * L.r), lj = grid_u32(b * L.r);
  if (li >= L.r || lj >= L.r) return -1;  // U2
  return (int64_t)((uint64_t)L.block(g) * L.rr + (uint64_t)lj * L.r + li);
}

uint64_t DyMuPathPlanner::localCell(uint64_t p, localNode* out) const {
  const LocalLayer& L = *local_;
  const CellPose c = cell_pose(L, p, nx_, global_res_);
  out->pose.position[0] = (double)c.li;
  out->pose.position[1] = (double)c.lj;
  out->parent_pose.position[0] = c.px;
  out->parent_pose.position[1] = c.py;
  out->global_pose.position[0] = c.gx;
  out->global_pose.position[1] = c.gy;
  out->world_pose.position[0] = c.wx;
  out->world_pose.position[1] = c.wy;
  out->deviation = L.dev[p];
  out->total_cost = L.tc[p];
  out->risk = L.risk[p];
  out->state = L.state[p] ? CLOSED : OPEN;
  out->isObstacle = L.obst[p] != 0;
  out->id = p;
  return p;
}

std::optional<localNode> DyMuPathPlanner::getLocalNode(base::Waypoint wPos) {
  const int64_t p = localAt(wPos.position[0], wPos.position[1]);
  if (p < 0) return std::nullopt;
  localNode n;
  localCell((uint64_t)p, &n);
  return n;
}

std::optional<localNode> DyMuPathPlanner::getLocalNode(base::Pose2D pos) {
  const int64_t p = localAt(pos.position[0], pos.position[1]);
  if (p < 0) return std::nullopt;
  localNode n;
  localCell((uint64_t)p, &n);
  return n;
}

// :473-491 (bilinear in the parent's total costs; no CLOSED test)
double DyMuPathPlanner::localTotalCost(uint64_t p) const {
  const CellPose c = cell_pose(*local_, p, nx_, global_res_);
  const uint32_t i = grid_u32(c.gx), j = grid_u32(c.gy);
  const double a = c.gx - (double)i, b = c.gy - (double)j;
  const int64_t n00 = nearestIndex(c.px, c.py);
  if (n00 < 0) return kInf;  // U1
  const unsigned gi = (unsigned)(n00 % nx_), gj = (unsigned)(n00 / nx_);
  const bool e = gi + 1 < nx_, n = gj + 1 < ny_;
  const double w00 = T((uint64_t)n00);
  const double w10 = e ? T((uint64_t)n00 + 1) : kInf;
  const double w01 = n ? T((uint64_t)n00 + nx_) : kInf;
  const double w11 = (e && n) ? T((uint64_t)n00 + nx_ + 1) : kInf;
  return w00 + (w10 - w00) * a + (w01 - w00) * b + (w11 + w00 - w10 - w01) * a * b;
}

double DyMuPathPlanner::getTotalCost(const localNode& lNode) {
  if (!local_ || lNode.id >= local_->dev.size()) return kInf;
  return localTotalCost(lNode.id);
}

// :441-471.  With an index (computeLocalPlanning's pixel loop), the scan starts
// at the first waypoint within risk_distance, found among the index's 3x3
// cells; the reference's loop changes nothing before it.
bool DyMuPathPlanner::isBlockingObstacle(uint64_t p, unsigned& maxIndex, unsigned& minIndex,
                                         const PathIndex* index) const {
  const CellPose c = cell_pose(*local_, p, nx_, global_res_);
  auto near = [&](unsigned i) {
    const double dx = c.wx - current_path[i].position[0], dy = c.wy - current_path[i].position[1];
    return std::sqrt(dx * dx + dy * dy) < risk_distance_;
  };
  unsigned first = 0;
  if (index) {
    const int64_t cx = PathIndex::cell(c.wx, index->cs), cy = PathIndex::cell(c.wy, index->cs);
    uint64_t best = UINT64_MAX;
    for (int64_t a = cx - 1; a <= cx + 1; ++a)
      for (int64_t b = cy - 1; b <= cy + 1; ++b) {
        const auto it = index->cells.find(PathIndex::key(a, b));
        if (it == index->cells.end()) continue;
        for (const uint32_t k : it->second) {
          if (k >= best) break;
          if (near(k)) {
            best = k;
            break;
          }
        }
      }
    if (best == UINT64_MAX) return false;
    first = (unsigned)best;
  }
  bool blocked = false;
  for (unsigned i = first; i < current_path.size(); ++i) {
    if (near(i)) {
      if (!blocked) {
        blocked = true;
        minIndex = (i < minIndex) ? i : minIndex;
      } else {
        maxIndex = (i > maxIndex) ? i : maxIndex;
      }
    } else if (blocked) {
      maxIndex = (i > maxIndex) ? i : maxIndex;
      return blocked;
    }
  }
  if (blocked) maxIndex = (unsigned)current_path.size();
  return blocked;
}

bool DyMuPathPlanner::isBlockingObstacle(const localNode& obNode, unsigned& maxIndex,
                                         unsigned& minIndex) {
  if (!local_ || obNode.id >= local_->dev.size()) return false;
  return isBlockingObstacle(obNode.id, maxIndex, minIndex, nullptr);
}

void DyMuPathPlanner::createLocalMap(unsigned i, unsigned j) { subdivideGlobalNode(i, j); }

std::optional<localNode> DyMuPathPlanner::localAgent() {
  if (!local_ || local_agent_ < 0 || (uint64_t)local_agent_ >= local_->dev.size())
    return std::nullopt;
  localNode n;
  localCell((uint64_t)local_agent_, &n);
  return n;
}

// :493-576 (expandRisk, maxRiskNode, propagateRisk).  The queue keeps the
// reference's order: the front unless it is below 1 and a later entry has a
// higher risk, in which case the first such entry; a node is queued again
// each time its risk rises.
namespace {
// maxRiskNode's choice (:525-548): the front, unless it is below 1 and a later
// entry holds a higher risk -- then the first such entry
size_t max_risk_index(const LocalLayer& L) {
  size_t index = 0;
  double maxRisk = L.risk[L.expandable.front()];
  for (size_t i = 0; i < L.expandable.size(); ++i) {
    if (maxRisk == 1) break;
    if (L.risk[L.expandable[i]] > maxRisk) {
      maxRisk = L.risk[L.expandable[i]];
      index = i;
      break;
    }
  }
  return index;
}
}  // namespace

// propagateRisk (:550-576) on sub-cell q
void DyMuPathPlanner::riskUpdate(uint64_t q) {
  LocalLayer& L = *local_;
  const double C = local_res_ / risk_distance_;
  const int64_t y0 = L.nb(q, 0), y1 = L.nb(q, 3), x0 = L.nb(q, 1), x1 = L.nb(q, 2);
  const double Ry = std::fmax(y0 < 0 ? 0 : L.risk[y0], y1 < 0 ? 0 : L.risk[y1]);
  const double Rx = std::fmax(x0 < 0 ? 0 : L.risk[x0], x1 < 0 ? 0 : L.risk[x1]);
  const double Sx = 1 - Rx, Sy = 1 - Ry;
  double S;
  if (std::fabs(Sx - Sy) < C)
    S = (Sx + Sy + std::sqrt(2 * (C * C) - ((Sx - Sy) * (Sx - Sy)))) / 2;
  else
    S = std::fmin(Sx, Sy) + C;
  const double R = (1 - S < 0.0) ? 0.0 : 1 - S;
  if ((R > 0) && (R > L.risk[q])) {
    L.risk[q] = R;
    L.expandable.push_back(q);
  }
}

void DyMuPathPlanner::expandRisk() {
  if (!local_) return;
  LocalLayer& L = *local_;
  while (!L.expandable.empty()) {
    const size_t index = max_risk_index(L);
    const uint64_t t = L.expandable[index];
    L.expandable.erase(L.expandable.begin() + (std::ptrdiff_t)index);
    const CellPose ct = cell_pose(L, t, nx_, global_res_);
    const int64_t gt = nearestIndex(ct.px, ct.py);
    for (int d = 0; d < 4; ++d) {
      const int64_t q = L.nb(t, d);
      if (q < 0 || L.obst[q]) continue;
      const CellPose cq = cell_pose(L, (uint64_t)q, nx_, global_res_);
      const int64_t g = nearestIndex(cq.px, cq.py);
      if (gt != g && g >= 0) subdivideGlobalNode((unsigned)(g % nx_), (unsigned)(g / nx_));
      riskUpdate((uint64_t)q);
    }
  }
}

// ---- the per-node steps at the class surface (src/DyMu.hpp:553-570) ----

int64_t DyMuPathPlanner::localId(const localNode& n) const {
  if (!local_ || n.id >= local_->dev.size()) return -1;
  return (int64_t)n.id;
}

std::optional<localNode> DyMuPathPlanner::localNeighbour(const localNode& n, int d) {
  const int64_t p = localId(n);
  if (p < 0 || d < 0 || d > 3) return std::nullopt;
  const int64_t q = local_->nb((uint64_t)p, d);
  if (q < 0) return std::nullopt;
  localNode o;
  localCell((uint64_t)q, &o);
  return o;
}

std::optional<localNode> DyMuPathPlanner::maxRiskNode() {
  if (!local_ || local_->expandable.empty()) return std::nullopt;  // :527
  LocalLayer& L = *local_;
  const size_t index = max_risk_index(L);
  const uint64_t t = L.expandable[index];
  L.expandable.erase(L.expandable.begin() + (std::ptrdiff_t)index);
  localNode n;
  localCell(t, &n);
  return n;
}

void DyMuPathPlanner::propagateRisk(const localNode& n) {
  const int64_t q = localId(n);
  if (q >= 0) riskUpdate((uint64_t)q);
}

void DyMuPathPlanner::propagateLocalNode(const localNode& n) {
  const int64_t q = localId(n);
  if (q >= 0) deviationUpdate((uint64_t)q);
}

void DyMuPathPlanner::setLocalNodeState(const localNode& n, node_state s) {
  const int64_t q = localId(n);
  if (q >= 0) local_->state[q] = s == CLOSED ? 1 : 0;
}

// the band in the reference's order: a sub-cell enters local_narrowband exactly when
// it enters local_propagated_nodes (its deviation first becomes finite, :741-747),
// so the band is the propagated list filtered by membership
std::optional<localNode> DyMuPathPlanner::minCostLocalNode(double Tovertake, double minC) {
  (void)Tovertake;  // the reference's key ignores them (the term is commented out, :758)
  (void)minC;
  if (!local_) return std::nullopt;
  LocalLayer& L = *local_;
  int64_t best = -1;
  for (const uint64_t p : L.propagated)
    if (L.in_band[p] && (best < 0 || L.dev[p] < L.dev[best])) best = (int64_t)p;
  if (best < 0) return std::nullopt;  // the reference reads front() of an empty band (U3)
  L.in_band[best] = 0;
  --L.band_count;
  localNode n;
  localCell((uint64_t)best, &n);
  return n;
}

std::optional<localNode> DyMuPathPlanner::minCostLocalNode(const localNode& reachNode) {
  const int64_t r = localId(reachNode);
  if (r < 0) return std::nullopt;
  LocalLayer& L = *local_;
  const CellPose ce = cell_pose(L, (uint64_t)r, nx_, global_res_);
  int64_t best = -1;
  double hmin = 0.0;
  for (const uint64_t p : L.propagated) {
    if (!L.in_band[p]) continue;
    const CellPose c = cell_pose(L, p, nx_, global_res_);
    const double dx = c.wx - ce.wx, dy = c.wy - ce.wy;
    const double h = L.dev[p] + std::sqrt(dx * dx + dy * dy);  // :782-800
    if (best < 0 || h < hmin) {
      hmin = h;
      best = (int64_t)p;
    }
  }
  if (best < 0) return std::nullopt;
  L.in_band[best] = 0;
  --L.band_count;
  localNode n;
  localCell((uint64_t)best, &n);
  return n;
}

std::vector<localNode> DyMuPathPlanner::localNarrowband() {
  std::vector<localNode> out;
  if (!local_) return out;
  for (const uint64_t p : local_->propagated) {
    if (!local_->in_band[p]) continue;
    out.emplace_back();
    localCell(p, &out.back());
  }
  return out;
}

std::vector<localNode> DyMuPathPlanner::localExpandableObstacles() {
  std::vector<localNode> out;
  if (!local_) return out;
  for (const uint64_t p : local_->expandable) {
    out.emplace_back();
    localCell(p, &out.back());
  }
  return out;
}

std::vector<localNode> DyMuPathPlanner::localPropagatedNodes() {
  std::vector<localNode> out;
  if (!local_) return out;
  for (const uint64_t p : local_->propagated) {
    out.emplace_back();
    localCell(p, &out.back());
  }
  return out;
}

// :578-805 (computeLocalPropagation, propagateLocalNode, minCostLocalNode x2);
// returns the set node, -1 = NULL
int64_t DyMuPathPlanner::localPropagation(base::Waypoint start, base::Waypoint over) {
  if (!local_) return -1;
  LocalLayer& L = *local_;
  const double Tover = getTotalCost(over);
  for (const uint64_t p : L.propagated) {
    L.state[p] = 0;
    L.dev[p] = kInf;
    L.tc[p] = kInf;
    L.in_band[p] = 0;
  }
  L.propagated.clear();
  L.heap.clear();
  L.band_count = 0;
  const int64_t agent = localAt(start.position[0], start.position[1]);
  local_agent_ = agent;
  if (agent < 0 || L.obst[agent]) return -1;
  L.dev[agent] = 0;
  L.tc[agent] = localTotalCost((uint64_t)agent);
  L.state[agent] = 1;
  int64_t end = -1;
  if (repairing_approach_ == CONSERVATIVE) {
    end = localAt(over.position[0], over.position[1]);
    if (end < 0 || L.obst[end]) return -1;
  }
  const bool conservative = repairing_approach_ == CONSERVATIVE;
  double ex = 0, ey = 0;
  if (conservative) {
    const CellPose ce = cell_pose(L, (uint64_t)end, nx_, global_res_);
    ex = ce.wx;
    ey = ce.wy;
  }
  // the band key: deviation (SWEEPING, :752-775), deviation + distance to the
  // overtake node (CONSERVATIVE, :777-805)
  auto key = [&](uint64_t p) {
    if (!conservative) return L.dev[p];
    const CellPose c = cell_pose(L, p, nx_, global_res_);
    const double dx = c.wx - ex, dy = c.wy - ey;
    return L.dev[p] + std::sqrt(dx * dx + dy * dy);
  };
  auto later = [](const LocalLayer::Entry& a, const LocalLayer::Entry& b) {
    return a.key > b.key || (a.key == b.key && a.seq > b.seq);
  };
  auto band_push = [&](uint64_t p) {
    L.heap.push_back({key(p), L.seq[p], p});
    std::push_heap(L.heap.begin(), L.heap.end(), later);
  };
  // :685-696: give up (NULL) once the propagation has run longer than the limit
  const auto t_init = std::chrono::steady_clock::now();
  uint64_t pops = 0;
  L.seq[agent] = L.next_seq++;
  L.in_band[agent] = 1;
  L.band_count = 1;
  band_push((uint64_t)agent);
  L.propagated.push_back((uint64_t)agent);

  for (;;) {
    int64_t t = -1;
    while (!L.heap.empty()) {
      std::pop_heap(L.heap.begin(), L.heap.end(), later);
      const LocalLayer::Entry e = L.heap.back();
      L.heap.pop_back();
      if (L.in_band[e.p] && key(e.p) == e.key) {
        t = (int64_t)e.p;
        break;
      }
    }
    if (t < 0) return -1;  // U3
    L.in_band[t] = 0;
    --L.band_count;
    L.state[t] = 1;
    const CellPose ct = cell_pose(L, (uint64_t)t, nx_, global_res_);
    const int64_t gt = nearestIndex(ct.px, ct.py);
    for (int d = 0; d < 4; ++d) {
      int64_t q = L.nb((uint64_t)t, d);
      if (q >= 0) {
        const CellPose cq = cell_pose(L, (uint64_t)q, nx_, global_res_);
        const int64_t g = nearestIndex(cq.px, cq.py);
        if (gt != g && g >= 0) subdivideGlobalNode((unsigned)(g % nx_), (unsigned)(g / nx_));
      }
      q = L.nb((uint64_t)t, d);
      if (q < 0 || L.state[q] || L.obst[q]) continue;
      const double d0 = L.dev[q];
      deviationUpdate((uint64_t)q);  // propagateLocalNode (:700-750)
      if (L.dev[q] < d0) band_push((uint64_t)q);
      if (end < 0 && L.tc[q] < Tover && L.risk[q] == 0) end = q;
    }
    if (end >= 0 && L.state[end]) {
      bool all = true;
      for (int d = 0; d < 4 && all; ++d) {
        const int64_t q = L.nb((uint64_t)end, d);
        all = q >= 0 && L.state[q];  // U1
      }
      if (all) return end;
    }
    if (local_timeout_s_ > 0 && (++pops & 255) == 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t_init).count() >
            local_timeout_s_) {
      std::fprintf(stderr,
                   "computeLocalPropagation: ERROR: no set node after %.3g s (local narrowband "
                   "%llu, propagated nodes %llu)\n",
                   local_timeout_s_, (unsigned long long)L.band_count,
                   (unsigned long long)L.propagated.size());
      return -1;
    }
  }
}

// propagateLocalNode (:700-750) on sub-cell q: the deviation update; a sub-cell whose
// deviation first becomes finite joins the band and the propagated list
void DyMuPathPlanner::deviationUpdate(uint64_t q) {
  LocalLayer& L = *local_;
  const int64_t n0 = L.nb(q, 0), n3 = L.nb(q, 3), n1 = L.nb(q, 1), n2 = L.nb(q, 2);
  double Ty, Tx;
  if (n0 >= 0 && n3 >= 0)
    Ty = std::fmin(L.dev[n3], L.dev[n0]);
  else if (n0 < 0)
    Ty = n3 >= 0 ? L.dev[n3] : kInf;
  else
    Ty = L.dev[n0];
  if (n1 >= 0 && n2 >= 0)
    Tx = std::fmin(L.dev[n1], L.dev[n2]);
  else if (n1 < 0)
    Tx = n2 >= 0 ? L.dev[n2] : kInf;
  else
    Tx = L.dev[n1];
  const double R = L.risk[q];
  if (L.tc[q] == kInf) L.tc[q] = localTotalCost(q);
  const double C = local_res_ * (risk_ratio_ * R + 1);
  const double Tn = eikonal(Tx, Ty, C);
  if (Tn < L.dev[q]) {
    if (L.dev[q] == kInf) {
      L.seq[q] = L.next_seq++;
      L.in_band[q] = 1;
      ++L.band_count;
      L.propagated.push_back(q);
    }
    L.dev[q] = Tn;
  }
}

std::optional<localNode> DyMuPathPlanner::computeLocalPropagation(base::Waypoint wInit,
                                                                  base::Waypoint wOvertake) {
  const int64_t p = localPropagation(wInit, wOvertake);
  if (p < 0) return std::nullopt;
  localNode n;
  localCell((uint64_t)p, &n);
  return n;
}

// ---- local path (:807-1023) ----
namespace {
// :979-1023 gradientNode on the deviation; U1: a NULL neighbour reads +inf
void local_gradient(const LocalLayer& L, uint64_t p, double& dnx, double& dny) {
  const int64_t w = L.nb(p, 1), e = L.nb(p, 2), s = L.nb(p, 0), n = L.nb(p, 3);
  auto dv = [&](int64_t q) { return q < 0 ? kInf : L.dev[q]; };
  const double t = L.dev[p];
  double dx, dy;
  if ((w < 0 && e < 0) || (w >= 0 && e >= 0 && L.dev[w] == kInf && L.dev[e] == kInf))
    dx = 0;
  else if (w < 0 || L.dev[w] == kInf)
    dx = dv(e) - t;
  else if (e < 0 || L.dev[e] == kInf)
    dx = t - L.dev[w];
  else
    dx = (L.dev[e] - L.dev[w]) * 0.5;
  if ((s < 0 && n < 0) || (s >= 0 && n >= 0 && L.dev[s] == kInf && L.dev[n] == kInf))
    dy = 0;
  else if (s < 0 || L.dev[s] == kInf)
    dy = dv(n) - t;
  else if (n < 0 || L.dev[n] == kInf)
    dy = t - L.dev[s];
  else
    dy = (L.dev[n] - L.dev[s]) * 0.5;
  dnx = dx / std::sqrt(dx * dx + dy * dy);
  dny = dy / std::sqrt(dx * dx + dy * dy);
}
}  // namespace

// :877-977
void DyMuPathPlanner::gradientNode(const localNode& n, double& dnx, double& dny) const {
  if (!local_ || n.id >= local_->dev.size()) {
    dnx = dny = 0;
    return;
  }
  local_gradient(*local_, n.id, dnx, dny);
}

bool DyMuPathPlanner::computeLocalWaypointGDM(base::Waypoint& wPos, double tau) {
  const int64_t l = localAt(wPos.position[0], wPos.position[1]);
  if (l < 0) return false;
  const LocalLayer& L = *local_;
  const double gx = wPos.position[0] - global_offset_[0];
  const double gy = wPos.position[1] - global_offset_[1];
  const uint32_t cX = grid_u32(gx / global_res_), cY = grid_u32(gy / global_res_);
  const double dX = gx - (double)cX, dY = gy - (double)cY;
  auto elev = [&](uint32_t i, uint32_t j) {  // U1: a NULL corner reads 0
    return (i < nx_ && j < ny_) ? elevation_[idx(i, j)] : 0.0;
  };
  const bool c00 = cX < nx_ && cY < ny_;
  const bool c10 = c00 && cX + 1 < nx_, c01 = c00 && cY + 1 < ny_, c11 = c10 && cY + 1 < ny_;
  wPos.position[2] = interpolate(dX, dY, c00 ? elev(cX, cY) : 0.0, c10 ? elev(cX + 1, cY) : 0.0,
                                 c01 ? elev(cX, cY + 1) : 0.0, c11 ? elev(cX + 1, cY + 1) : 0.0);
  const CellPose cl = cell_pose(L, (uint64_t)l, nx_, global_res_);
  auto nbn = [&](int64_t q, int d) { return q < 0 ? (int64_t)-1 : L.nb((uint64_t)q, d); };
  int64_t n00, n10, n01, n11;
  double a, b;
  if (cl.wx < wPos.position[0]) {
    if (cl.wy < wPos.position[1]) {
      n00 = l;
      n10 = L.nb(l, 2);
      n01 = L.nb(l, 3);
      n11 = nbn(L.nb(l, 2), 3);
      a = (wPos.position[0] - cl.wx) / local_res_;
      b = (wPos.position[1] - cl.wy) / local_res_;
    } else {
      n00 = L.nb(l, 0);
      n10 = L.nb(l, 2);
      n01 = l;
      n11 = nbn(L.nb(l, 0), 2);
      a = (wPos.position[0] - cl.wx) / local_res_;
      b = 1 + (wPos.position[1] - cl.wy) / local_res_;
    }
  } else {
    if (cl.wy < wPos.position[1]) {
      n00 = L.nb(l, 1);
      n10 = l;
      n01 = L.nb(l, 3);
      n11 = nbn(L.nb(l, 3), 1);
      a = 1 + (wPos.position[0] - cl.wx) / local_res_;
      b = (wPos.position[1] - cl.wy) / local_res_;
    } else {
      n00 = nbn(L.nb(l, 1), 0);
      n10 = L.nb(l, 0);
      n01 = L.nb(l, 1);
      n11 = l;
      a = 1 + (wPos.position[0] - cl.wx) / local_res_;
      b = 1 + (wPos.position[1] - cl.wy) / local_res_;
    }
  }
  if (n00 < 0 || n10 < 0 || n01 < 0 || n11 < 0) return false;  // U1
  double gx00, gx10, gx01, gx11, gy00, gy10, gy01, gy11;
  local_gradient(L, (uint64_t)n00, gx00, gy00);
  local_gradient(L, (uint64_t)n10, gx10, gy10);
  local_gradient(L, (uint64_t)n01, gx01, gy01);
  local_gradient(L, (uint64_t)n11, gx11, gy11);
  const double dcx = interpolate(a, b, gx00, gx01, gx10, gx11);
  const double dcy = interpolate(a, b, gy00, gy01, gy10, gy11);
  if (std::isnan(dcx) || std::isnan(dcy)) return false;
  if (std::sqrt(dcx * dcx + dcy * dcy) < 0.001 * tau * local_res_) return false;
  wPos.position[0] = wPos.position[0] - tau * dcx;
  wPos.position[1] = wPos.position[1] - tau * dcy;
  wPos.heading = std::atan2(dcy, dcx);
  return true;
}

// :851-869: toward the nb4 sub-cell of lowest deviation (U5: none finite -> the
// sub-cell's own position)
base::Waypoint DyMuPathPlanner::dijkstraStep(uint64_t l) const {
  const LocalLayer& L = *local_;
  const CellPose cl = cell_pose(L, l, nx_, global_res_);
  double t = kInf, nxp = cl.wx, nyp = cl.wy;
  for (int d = 0; d < 4; ++d) {
    const int64_t q = L.nb(l, d);
    if (q >= 0 && L.dev[q] < t) {
      t = L.dev[q];
      const CellPose cq = cell_pose(L, (uint64_t)q, nx_, global_res_);
      nxp = cq.wx;
      nyp = cq.wy;
    }
  }
  return make_wp(nxp, nyp, 0.0, std::atan2(nyp - cl.wy, nxp - cl.wx));
}

base::Waypoint DyMuPathPlanner::computeLocalWaypointDijkstra(const localNode& lNode) {
  if (!local_ || lNode.id >= local_->dev.size())
    return make_wp(lNode.world_pose.position[0], lNode.world_pose.position[1], 0.0, 0.0);
  return dijkstraStep(lNode.id);
}

// :807-849 (with :851-869 computeLocalWaypointDijkstra).  The trajectory is
// built back to front and reversed once (the reference inserts at the front).
std::vector<base::Waypoint> DyMuPathPlanner::localPath(uint64_t set, base::Waypoint start) {
  const LocalLayer& L0 = *local_;
  const CellPose cs = cell_pose(L0, set, nx_, global_res_);
  base::Waypoint w = make_wp(cs.gx, cs.gy, 0.0, 0.0);
  const double tau = 0.5 * local_res_;
  std::vector<base::Waypoint> rev;  // rev.back() is the reference's trajectory[0]
  (void)computeLocalWaypointGDM(w, tau * local_res_);
  rev.push_back(w);
  for (int it = 0; it < kMaxLocalSteps; ++it) {  // U4
    if (!(wdist(rev.back(), start) > 1.5 * local_res_)) break;
    bool ok = computeLocalWaypointGDM(w, tau);
    const base::Waypoint& t0 = rev.back();
    const base::Waypoint& t1 = rev.size() > 1 ? rev[rev.size() - 2] : rev.back();  // U4
    const double ex = w.position[0] - t0.position[0], ey = w.position[1] - t1.position[1];
    if (std::sqrt(ex * ex + ey * ey) < 0.01 * tau * local_res_) ok = false;
    if (ok) {
      rev.push_back(w);
    } else {
      const int64_t l = localAt(t0.position[0], t0.position[1]);
      if (l < 0) break;  // U1
      w = dijkstraStep((uint64_t)l);
      rev.push_back(w);
    }
  }
  std::reverse(rev.begin(), rev.end());
  return rev;
}

std::vector<base::Waypoint> DyMuPathPlanner::getLocalPath(const localNode& lSetNode,
                                                          base::Waypoint wInit, double tau) {
  (void)tau;  // overwritten with 0.5 * local_res (:817)
  if (!local_ || lSetNode.id >= local_->dev.size()) return {};
  return localPath(lSetNode.id, wInit);
}

// :298-435
int DyMuPathPlanner::repairPath(base::Waypoint start, unsigned index) {
  std::vector<base::Waypoint>& P = current_path;
  if (P.empty()) return -1;
  double overtake_index;
  if (repairing_approach_ == CONSERVATIVE) {
    overtake_index =
        ((unsigned)reconnecting_index > index) ? (unsigned)reconnecting_index : index;
    index = (unsigned)overtake_index;
  } else {
    overtake_index = index;
  }
  while (index < P.size() && wdist(P[index], P[(size_t)overtake_index]) < reconnect_distance_)
    ++index;
  if (index >= P.size() || index == P.size() - 1) {
    P.clear();
    P.push_back(start);
    return -1;
  }
  const int64_t set = localPropagation(start, P[index]);
  if (set < 0) {
    P.clear();
    P.push_back(start);
    return -1;
  }
  double proximity = wdist(P[0], start), orig = 0, newd = 0;
  unsigned closest = 0;
  for (unsigned k = 1; k < index; ++k)
    if (wdist(P[k], start) < proximity) closest = k;  // proximity not updated (:373)
  for (unsigned k = closest; k < index; ++k) orig += wdist(P[k + 1], P[k]);
  std::vector<base::Waypoint> lp = localPath((uint64_t)set, start);
  const CellPose cs = cell_pose(*local_, (uint64_t)set, nx_, global_res_);
  const base::Waypoint nw = make_wp(cs.gx, cs.gy, 0.0, 0.0);
  if (lp.size() > 1) {
    for (size_t k = 0; k + 1 < lp.size(); ++k) newd += wdist(lp[k + 1], lp[k]);
    for (unsigned k = closest; k < index; ++k) {
      const int64_t g = nearestIndex(P[k].position[0], P[k].position[1]);
      if (g < 0) continue;  // U1
      const double q = orig / newd;
      traff_[g] = (traff_[g] < q) ? traff_[g] : q;
      markDirty((unsigned)(g / nx_), (unsigned)(g / nx_) + 1);
    }
    if (repairing_approach_ == CONSERVATIVE)
      P.erase(P.begin(), P.begin() + index);
    else
      computeGlobalPath(nw);
    lp.pop_back();
    current_path.insert(current_path.begin(), lp.begin(), lp.end());
    return (int)lp.size();
  }
  if (repairing_approach_ == CONSERVATIVE)
    P.erase(P.begin(), P.begin() + index);
  else
    computeGlobalPath(nw);
  return 0;
}

// :1027-1109
bool DyMuPathPlanner::evaluatePath(unsigned starting_index) {
  unsigned minIndex = 0, rect = 0;
  bool blocked = false;
  std::vector<base::Waypoint> fin;
  unsigned iw = starting_index;
  reconnecting_index = 0;
  while (iw < current_path.size()) {
    const int64_t g = nearestIndex(current_path[iw].position[0], current_path[iw].position[1]);
    bool repair = false;
    if (g >= 0 && local_ && local_->block((uint64_t)g) >= 0) {
      const int64_t l = localAt(current_path[iw].position[0], current_path[iw].position[1]);
      if (l >= 0 && local_->risk[l] > 0.0) {
        if (!blocked) {
          blocked = true;
          minIndex = iw;
        }
      } else if (blocked) {
        repair = true;
      }
    } else if (blocked) {
      repair = true;
    }
    if (repair) {
      rect = minIndex;
      while (rect > 0) {
        if (wdist(current_path[minIndex], current_path[rect]) > 2.0) break;
        --rect;
      }
      fin.insert(fin.end(), current_path.begin(), current_path.begin() + rect);
      const base::Waypoint from = current_path[rect];
      iw = (unsigned)repairPath(from, iw);
      blocked = false;
      minIndex = 0;
    }
    if (iw == (unsigned)-1) return false;
    ++iw;
  }
  if (blocked)
    fin.insert(fin.end(), current_path.begin(), current_path.begin() + minIndex);
  else
    fin.insert(fin.end(), current_path.begin() + minIndex, current_path.end());
  current_path = fin;
  return true;
}

// :193-291
bool DyMuPathPlanner::computeLocalPlanning(base::Waypoint wPos,
                                           base::samples::frame::Frame traversabilityMap,
                                           double res, std::vector<base::Waypoint>& trajectory,
                                           base::Time& localTime) {
  if (!local_) return false;
  wPos.position[0] -= global_offset_[0];
  wPos.position[1] -= global_offset_[1];
  const unsigned height = traversabilityMap.getHeight(), width = traversabilityMap.getWidth();
  const uint32_t a = grid_u32(std::fmax(0, ((wPos.position[1] - (double)height / 2 * res) / global_res_)));
  const uint32_t b = grid_u32(std::fmin((double)ny_, ((wPos.position[1] + (double)height / 2 * res) / global_res_)));
  const uint32_t c = grid_u32(std::fmax(0, ((wPos.position[0] - (double)width / 2 * res) / global_res_)));
  const uint32_t d = grid_u32(std::fmin((double)nx_, ((wPos.position[0] + (double)width / 2 * res) / global_res_)));
  for (uint32_t j = a; j < b; ++j)
    for (uint32_t i = c; i < d; ++i) subdivideGlobalNode(i, j);
  unsigned minIndex = (unsigned)current_path.size(), maxIndex = 0;
  bool pathBlocked = false;
  const double offsetX = wPos.position[0] - res * (double)width / 2;
  const double offsetY = wPos.position[1] + res * (double)height / 2;
  const double gsx = global_res_ * (double)nx_ - 0.5, gsy = global_res_ * (double)ny_ - 0.5;
  const double r2 = (double)(res_ratio_ * res_ratio_);
  const uint32_t row = traversabilityMap.getRowSize(), pix = traversabilityMap.getPixelSize();
  PathIndex index;
  bool indexed = false, index_built = false;
  for (uint32_t j = 0; j < height; ++j)
    for (uint32_t i = 0; i < width; ++i) {
      const double px = offsetX + i * res, py = offsetY - j * res;
      if (!((px > -0.5) && (px < gsx) && (py > -0.5) && (py < gsy))) continue;
      const uint8_t value = traversabilityMap.image[(size_t)j * row + (size_t)i * pix];
      const int64_t l = localAt(px, py);
      if (l < 0) continue;  // U2
      LocalLayer& L = *local_;
      const CellPose cl = cell_pose(L, (uint64_t)l, nx_, global_res_);
      const int64_t g = nearestIndex(cl.px, cl.py);
      if (g < 0) continue;  // U1
      if (!L.obst[l] && (value != 0 || is_obstacle_[g])) {
        L.obst[l] = 1;
        L.expandable.push_back((uint64_t)l);
        L.risk[l] = 1.0;
        if (!index_built) {  // current_path does not change inside this loop
          indexed = index.build(current_path, risk_distance_);
          index_built = true;
        }
        const bool blocked =
            isBlockingObstacle((uint64_t)l, maxIndex, minIndex, indexed ? &index : nullptr);
        pathBlocked = pathBlocked ? true : blocked;
        // :264-274 hazard feedback on the global layer (re-propagated by the
        // next computeTotalCostMap as a windowed update)
        const unsigned gi = (unsigned)(g % nx_), gj = (unsigned)(g / nx_);
        const double hv = hazard_[g] + 1.0 / r2;
        hazard_[g] = hv < 1.0 ? hv : 1.0;
        static const int dd[8][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
        for (const auto& e : dd) {
          const uint32_t oi = gi + (uint32_t)e[0], oj = gj + (uint32_t)e[1];
          if (oi >= nx_ || oj >= ny_) continue;
          const double v = hazard_[idx(oi, oj)] + 0.1 / r2;
          hazard_[idx(oi, oj)] = v < 1.0 ? v : 1.0;
        }
        markDirty(gj > 0 ? gj - 1 : 0, std::min(ny_, gj + 2));
      }
    }
  if (pathBlocked && maxIndex > minIndex) {
    const base::Time tInit = base::Time::now();
    expandRisk();
    trajectory.clear();
    reconnecting_index = repairPath(wPos, maxIndex);
    if (repairing_approach_ == SWEEPING) evaluatePath((unsigned)reconnecting_index);
    trajectory = current_path;
    localTime = base::Time::now() - tInit;
    return true;
  }
  return false;
}

// :1111-1211: (21 r)^2 window around the global node nearest rover_pos
void DyMuPathPlanner::windowMatrix(base::Waypoint rover_pos, bool deviation,
                                   std::vector<std::vector<double>>& m) {
  const unsigned half = 10, side = 2 * half + 1, r = res_ratio_, ls = side * r;
  m.assign(ls, std::vector<double>(ls, 0.0));
  const int64_t g = nearestIndex(rover_pos.position[0], rover_pos.position[1]);
  if (g < 0 || !local_) return;  // U1
  const LocalLayer& L = *local_;
  const double gx = (double)(g % nx_), gy = (double)(g / nx_);
  for (unsigned j = 0; j < side; ++j)
    for (unsigned i = 0; i < side; ++i) {
      const int cx = (int)(gx - half + i), cy = (int)(gy - half + j);
      if ((unsigned)cx >= nx_ || (unsigned)cy >= ny_) continue;
      const int64_t b = L.block(idx((unsigned)cx, (unsigned)cy));
      if (b < 0) continue;
      for (unsigned l = 0; l < r; ++l)
        for (unsigned k = 0; k < r; ++k) {
          const uint64_t p = (uint64_t)b * L.rr + (uint64_t)l * r + k;
          m[l + j * r][k + i * r] =
              deviation ? (L.dev[p] == kInf ? -1 : L.dev[p]) : L.risk[p];
        }
    }
}

std::vector<std::vector<double>> DyMuPathPlanner::getRiskMatrix(base::Waypoint rover_pos) {
  std::vector<std::vector<double>> m;
  windowMatrix(rover_pos, false, m);
  return m;
}

std::vector<std::vector<double>> DyMuPathPlanner::getDeviationMatrix(base::Waypoint rover_pos) {
  std::vector<std::vector<double>> m;
  windowMatrix(rover_pos, true, m);
  return m;
}

int DyMuPathPlanner::getReconnectingIndex() { return reconnecting_index; }

uint64_t DyMuPathPlanner::localMapMask(uint8_t* mask) const {
  if (mask) std::fill(mask, mask + (uint64_t)nx_ * ny_, (uint8_t)0);
  if (!local_) return 0;
  if (mask)
    for (const uint64_t g : local_->block_g) mask[g] = 1;
  return local_->block_g.size();
}

bool DyMuPathPlanner::localBlock(unsigned i, unsigned j, double* dev, double* tc, double* risk,
                                 uint8_t* state, uint8_t* obst) const {
  if (!local_ || i >= nx_ || j >= ny_) return false;
  const int64_t b = local_->block(idx(i, j));
  if (b < 0) return false;
  const LocalLayer& L = *local_;
  const uint64_t p0 = (uint64_t)b * L.rr;
  for (uint64_t k = 0; k < L.rr; ++k) {
    if (dev) dev[k] = L.dev[p0 + k];
    if (tc) tc[k] = L.tc[p0 + k];
    if (risk) risk[k] = L.risk[p0 + k];
    if (state) state[k] = L.state[p0 + k];
    if (obst) obst[k] = L.obst[p0 + k];
  }
  return true;
}

}  // namespace PathPlanning_lib
