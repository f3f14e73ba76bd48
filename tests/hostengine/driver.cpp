// driver.cpp -- the planner's host logic over the host-memory engine test double
// (host_engine.c): readback failure handling, engine-option changes after a
// solve, and an early exit on a tie-rich map (tests/test_host_engine.py).
//   driver ok       solve a >= 1024-row grid, read it back, compare with the oracle
//   driver fail     the same with HOST_ENGINE_FAIL_D2H set: the readback must throw
//   driver options  solve, setEngineOptions, then read the map and a path
//   driver ties     constant cost (every distance tie), computeTotalCostMap's early exit
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "DyMu.hpp"
#include "oracle.h"

using namespace PathPlanning_lib;

static base::Waypoint wp(double x, double y) {
  base::Waypoint w;
  w.position[0] = x;
  w.position[1] = y;
  return w;
}

static std::vector<std::vector<double>> random_costs(unsigned nx, unsigned ny, unsigned gi,
                                                     unsigned gj) {
  std::vector<double> u((uint64_t)nx * ny), u2((uint64_t)nx * ny);
  oracle_fill_u01(u.data(), u.size(), 3);
  oracle_fill_u01(u2.data(), u2.size(), 4);
  std::vector<std::vector<double>> c(ny, std::vector<double>(nx));
  for (unsigned j = 0; j < ny; ++j)
    for (unsigned i = 0; i < nx; ++i) {
      const uint64_t k = (uint64_t)j * nx + i;
      const bool near = i + 1 >= gi && i <= gi + 1 && j + 1 >= gj && j <= gj + 1;
      c[j][i] = (u2[k] < 0.02 && !near) ? -1.0 : 1.0 + 4.0 * u[k];
    }
  return c;
}

// the oracle's map of the same input (setCostMap speed, reference :109-126, :527-528)
static std::vector<double> oracle_map(const std::vector<std::vector<double>>& c, unsigned gi,
                                      unsigned gj) {
  const unsigned ny = (unsigned)c.size(), nx = (unsigned)c[0].size();
  const uint64_t n = (uint64_t)nx * ny;
  std::vector<double> flat(n), cost(n, 0.0), traff(n, 1.0), hz(n, 0.0), F(n), T(n);
  std::vector<uint8_t> obst(n, 0);
  for (unsigned j = 0; j < ny; ++j)
    for (unsigned i = 0; i < nx; ++i) flat[(uint64_t)j * nx + i] = c[j][i];
  oracle_set_cost_map(flat.data(), n, cost.data(), obst.data(), traff.data(), hz.data());
  oracle_pack_speed(cost.data(), hz.data(), traff.data(), obst.data(), n, 1.0, F.data());
  uint64_t pops = 0;
  oracle_fmm_heap(F.data(), nx, ny, gi, gj, -1, -1, T.data(), nullptr, &pops);
  return T;
}

static int compare(const std::vector<std::vector<double>>& M, const std::vector<double>& T) {
  const unsigned ny = (unsigned)M.size(), nx = (unsigned)M[0].size();
  for (unsigned j = 0; j < ny; ++j)
    for (unsigned i = 0; i < nx; ++i) {
      const double t = T[(uint64_t)j * nx + i], e = std::isinf(t) ? -1.0 : t;
      if (std::memcmp(&e, &M[j][i], sizeof e) != 0) {
        std::printf("mismatch at (%u,%u): %.17g vs %.17g\n", i, j, M[j][i], e);
        return 1;
      }
    }
  return 0;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "ok";
  if (mode == "ties") {
    // constant cost: every axis distance ties with many others (the early exit's
    // band replay meets equal CLOSED values on both sides of an OPEN pair)
    const unsigned N = 160, gi = 80, gj = 80;
    DyMuPathPlanner p(1.0, 2.0, 5.0, CONSERVATIVE);
    p.initGlobalLayer(1.0, 0.5, N, N, {0.0, 0.0});
    p.setCostMap(std::vector<std::vector<double>>(N, std::vector<double>(N, 1.0)));
    if (!p.setGoal(wp(gi, gj))) return 2;
    const bool r = p.computeTotalCostMap(wp(20, 140));
    const auto M = p.getTotalCostMatrix();
    std::vector<double> F((uint64_t)N * N, 1.0), T((uint64_t)N * N);
    std::vector<uint8_t> closed((uint64_t)N * N);
    uint64_t pops = 0;
    const int rr = oracle_fmm_linear(F.data(), N, N, gi, gj, 20, 140, T.data(), closed.data(), &pops);
    // ties at the exit: the planner replays the reference exactly (exactEarlyExit), so
    // the whole matrix -- CLOSED values, the band's tentative values, -1 elsewhere --
    // and every node state are the reference's, bit for bit
    uint64_t n_closed = 0, bad = 0, band = 0;
    for (uint64_t k = 0; k < T.size(); ++k) {
      const double m = M[k / N][k % N];
      const double want = T[k] < INFINITY ? T[k] : -1.0;
      if (std::memcmp(&m, &want, sizeof m) != 0) ++bad;
      const auto node = p.getGlobalNode((unsigned)(k % N), (unsigned)(k / N));
      if (!node || (node->state == CLOSED) != (closed[k] != 0)) ++bad;
      n_closed += closed[k] ? 1 : 0;
      band += (!closed[k] && T[k] < INFINITY) ? 1 : 0;
    }
    if (p.lastBandSize() != band) ++bad;
    std::printf("ties r=%d oracle=%d closed=%llu band=%llu bad=%llu\n", (int)r, rr,
                (unsigned long long)n_closed, (unsigned long long)band, (unsigned long long)bad);
    return (bad == 0 && (int)r == rr) ? 0 : 1;
  }
  // >= 1024 rows: getTotalCostMatrix streams the download in row chunks
  const unsigned nx = 300, ny = 1100, gi = 150, gj = 550;
  const auto c = random_costs(nx, ny, gi, gj);
  DyMuPathPlanner p(1.0, 2.0, 5.0, CONSERVATIVE);
  p.initGlobalLayer(1.0, 0.5, nx, ny, {0.0, 0.0});
  if (!p.setCostMap(c) || !p.setGoal(wp(gi, gj)) || !p.computeEntireTotalCostMap()) return 2;
  const auto T = oracle_map(c, gi, gj);
  if (mode == "fail") {
    try {
      const auto M = p.getTotalCostMatrix();
      std::printf("no exception: readback returned %zu rows\n", M.size());
      return 1;
    } catch (const std::runtime_error& e) {
      std::printf("threw: %s\n", e.what());
      return 0;
    }
  }
  if (mode == "options") {
    dymu_opts o{};
    o.device = -1;
    p.setEngineOptions(o);  // releases the device buffers: the mirror must survive
    if (compare(p.getTotalCostMatrix(), T)) return 1;
    const auto path = p.getPath(wp(20.0, 30.0));
    std::printf("options ok, path %zu waypoints\n", path.size());
    return path.size() >= 2 ? 0 : 1;
  }
  if (compare(p.getTotalCostMatrix(), T)) return 1;
  std::printf("ok\n");
  return 0;
}
