// driver.cpp -- the planner's host logic over the host-memory engine test double
// (host_engine.c): readback failure handling, engine-option changes after a
// solve, and an early exit on a tie-rich map (tests/test_host_engine.py).
//   driver ok       solve a >= 1024-row grid, read it back, compare with the oracle
//   driver fail     the same with HOST_ENGINE_FAIL_D2H set: the readback must throw
//   driver options  solve, setEngineOptions, then read the map and a path
//   driver ties     constant cost (every distance tie), computeTotalCostMap's early exit
//   driver order    global_propagated_nodes in the reference's insertion order
//   driver exactperf N   the exact host replay's time on a two-valued N^2 map (manual)
// HOST_ENGINE_SHORT_REGION=1 makes the double report a one-cell exit region (ties mode
// with DYMU_EXACT_EXIT=1: the replay must restart on the whole grid)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
  if (mode == "perf") {  // timing of the exit-order resolution on a constant map (manual)
    const unsigned N = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1024;
    DyMuPathPlanner p(1.0, 2.0, 5.0, CONSERVATIVE);
    p.initGlobalLayer(1.0, 0.5, N, N, {0.0, 0.0});
    p.setCostMap(std::vector<std::vector<double>>(N, std::vector<double>(N, 1.0)));
    if (!p.setGoal(wp(N / 2, N / 2))) return 2;
    const bool r = p.computeTotalCostMap(wp(N * 0.7, N * 0.6));
    const auto& info = p.lastEarlyExitInfo();
    std::printf("perf N=%u r=%d band=%llu tied=%llu open=%llu resolve_ms=%.1f\n", N, (int)r,
                (unsigned long long)p.lastBandSize(), (unsigned long long)info.tied,
                (unsigned long long)info.open_at_limit, info.resolve_ms);
    return 0;
  }
  if (mode == "exactperf") {  // the exact host replay's cost: two-valued map, far start (manual)
    const unsigned N = argc > 2 ? (unsigned)std::atoi(argv[2]) : 2048;
    std::vector<std::vector<double>> cost(N, std::vector<double>(N));
    uint64_t h = 12345;
    for (unsigned j = 0; j < N; ++j)
      for (unsigned i = 0; i < N; ++i) {
        h = h * 6364136223846793005ull + 1442695040888963407ull;
        cost[j][i] = (h >> 62) ? 1.0 : 2.0;
      }
    DyMuPathPlanner p(1.0, 2.0, 5.0, CONSERVATIVE);
    p.initGlobalLayer(1.0, 0.5, N, N, {0.0, 0.0});
    p.setCostMap(cost);
    if (!p.setGoal(wp(N / 2, N / 2))) return 2;
    const bool r = p.computeTotalCostMap(wp(N * 0.85, N * 0.8));
    const auto& info = p.lastEarlyExitInfo();
    double sum = 0;
    const auto M = p.getTotalCostMatrix();
    for (const auto& row : M)
      for (const double v : row) sum += v;
    std::printf("exactperf N=%u r=%d band=%llu exact=%d resolve_ms=%.1f sum=%.17g\n", N, (int)r,
                (unsigned long long)p.lastBandSize(), info.exact_replay, info.resolve_ms, sum);
    return 0;
  }
  if (mode == "ties") {
    // constant / two-valued cost: values tie, so which cells of exactly the exit value
    // the reference closed -- and which it reached -- depends on its insertion order
    // (:551-568).  This double solves with the oracle's FMM (exact values); the planner
    // still treats them as an engine's: mirror ties on constant speed are resolved from
    // the values (pop_order.hpp, band replay), any other tie sends the exit to the exact
    // host replay.  Either way the exit state must be the reference's bit for bit: the
    // whole matrix, every node state, the band in insertion order.
    // exact: 1 = the exact host replay must run (two-valued speed: non-mirror ties at the
    // exit decide it), 0 = it must not (constant speed, goal far from the border:
    // every tie a trusted mirror image), -1 = either (mirror images off the grid)
    struct Case {
      unsigned N, gi, gj, si, sj;
      bool two;
      int exact;
    };
    const Case cases[] = {{512, 256, 256, 102, 128, true, -1}, {160, 80, 80, 20, 140, false, 0},
                          {96, 48, 48, 48, 20, false, 0},
                          {97, 30, 30, 60, 60, false, -1},  {64, 2, 5, 40, 40, false, -1},
                          {120, 60, 60, 100, 30, true, -1},  {90, 45, 20, 45, 70, true, 1}};
    uint64_t bad = 0;
    for (const Case& cs : cases) {
      const unsigned N = cs.N;
      std::vector<std::vector<double>> cost(N, std::vector<double>(N, 1.0));
      std::vector<double> F((uint64_t)N * N, 1.0), T((uint64_t)N * N);
      uint64_t h = 12345;
      if (cs.two)
        for (unsigned j = 0; j < N; ++j)
          for (unsigned i = 0; i < N; ++i) {
            h = h * 6364136223846793005ull + 1442695040888963407ull;
            const double v = (h >> 62) ? 1.0 : 2.0;
            cost[j][i] = v;
            F[(uint64_t)j * N + i] = v;
          }
      DyMuPathPlanner p(1.0, 2.0, 5.0, CONSERVATIVE);
      p.initGlobalLayer(1.0, 0.5, N, N, {0.0, 0.0});
      p.setCostMap(cost);
      if (!p.setGoal(wp(cs.gi, cs.gj))) return 2;
      const bool r = p.computeTotalCostMap(wp(cs.si, cs.sj));
      const auto M = p.getTotalCostMatrix();
      std::vector<uint8_t> closed((uint64_t)N * N);
      std::vector<uint64_t> seq((uint64_t)N * N);
      const int rr = oracle_fmm_order(F.data(), N, N, cs.gi, cs.gj, cs.si, cs.sj, T.data(),
                                      closed.data(), seq.data());
      uint64_t cbad = 0, band = 0;
      std::vector<std::pair<uint64_t, uint64_t>> want;  // (seq, k) of the band
      for (uint64_t k = 0; k < T.size(); ++k) {
        const double m = M[k / N][k % N];
        const double w = T[k] < INFINITY ? T[k] : -1.0;
        if (std::memcmp(&m, &w, sizeof m) != 0) ++cbad;
        const auto node = p.getGlobalNode((unsigned)(k % N), (unsigned)(k / N));
        if (!node || (node->state == CLOSED) != (closed[k] != 0)) ++cbad;
        if (!closed[k] && T[k] < INFINITY) {
          ++band;
          want.push_back({seq[k], k});
        }
      }
      std::sort(want.begin(), want.end());
      const auto nb = p.globalNarrowband();
      if (p.lastBandSize() != band || nb.size() != band) ++cbad;
      for (size_t q = 0; q < nb.size() && q < want.size(); ++q) {
        const uint64_t k = (uint64_t)nb[q].pose.position[1] * N + (uint64_t)nb[q].pose.position[0];
        if (k != want[q].second) {
          ++cbad;
          break;
        }
      }
      const int exact_at_exit = p.lastEarlyExitInfo().exact_replay;
      // minCostGlobalNode: the first strict minimum of the band in insertion order
      // (:551-568), with the oracle's values -- near-tied band values are settled first
      if (!want.empty()) {
        size_t best = 0;
        for (size_t q = 1; q < want.size(); ++q)
          if (T[want[q].second] < T[want[best].second]) best = q;
        const auto mn = p.minCostGlobalNode();
        const uint64_t k = mn ? (uint64_t)mn->pose.position[1] * N + (uint64_t)mn->pose.position[0]
                              : ~0ull;
        if (!mn || k != want[best].second ||
            std::memcmp(&mn->total_cost, &T[k], sizeof(double)) != 0)
          ++cbad;
      }
      const auto& info = p.lastEarlyExitInfo();
      // forced through the exact replay (DYMU_EXACT_EXIT, or a band-replay budget it overruns)
      static const bool forced = (std::getenv("DYMU_EXACT_EXIT") && std::atoi(std::getenv("DYMU_EXACT_EXIT"))) ||
                                 std::getenv("DYMU_REPLAY_BUDGET");
      if (!forced && cs.exact >= 0 && exact_at_exit != cs.exact) ++cbad;
      std::printf("ties N=%u r=%d oracle=%d band=%llu tied=%llu open=%llu near=%llu exact=%d "
                  "bad=%llu\n", N, (int)r, rr, (unsigned long long)band,
                  (unsigned long long)info.tied, (unsigned long long)info.open_at_limit,
                  (unsigned long long)info.near_ties, info.exact_replay, (unsigned long long)cbad);
      if ((int)r != rr) ++cbad;
      bad += cbad;
    }
    return bad == 0 ? 0 : 1;
  }
  if (mode == "order") {
    // global_propagated_nodes after computeEntireTotalCostMap and after an early exit:
    // the reached nodes in the reference's insertion order (rebuilt from the values, or
    // replayed on the host where near ties leave them undecided) against the oracle's
    // recorded insertion sequence
    struct Case {
      unsigned N, gi, gj;
      int si, sj;  // -1: full solve
      int kind;    // 0 random U(1,5) + 3% obstacles, 1 constant, 2 two-valued
    };
    const Case cases[] = {{96, 40, 50, -1, -1, 0}, {96, 40, 50, 80, 20, 0}, {64, 32, 32, -1, -1, 1},
                          {80, 30, 41, 60, 60, 1}, {72, 36, 36, -1, -1, 2}, {72, 20, 50, 50, 20, 2},
                          // >= 2^17 reached nodes: the sorts and the keys on several threads
                          {600, 300, 280, -1, -1, 0}, {600, 300, 280, 520, 500, 0}};
    uint64_t bad = 0;
    for (const Case& cs : cases) {
      const unsigned N = cs.N;
      std::vector<std::vector<double>> cost(N, std::vector<double>(N, 1.0));
      std::vector<double> F((uint64_t)N * N, 1.0), T((uint64_t)N * N);
      std::vector<double> u((uint64_t)N * N), u2((uint64_t)N * N);
      oracle_fill_u01(u.data(), u.size(), 5);
      oracle_fill_u01(u2.data(), u2.size(), 6);
      for (unsigned j = 0; j < N; ++j)
        for (unsigned i = 0; i < N; ++i) {
          const uint64_t k = (uint64_t)j * N + i;
          const bool near_goal = i + 1 >= cs.gi && i <= cs.gi + 1 && j + 1 >= cs.gj && j <= cs.gj + 1;
          const bool near_start = cs.si >= 0 && i + 1 >= (unsigned)cs.si && i <= (unsigned)cs.si + 1 &&
                                  j + 1 >= (unsigned)cs.sj && j <= (unsigned)cs.sj + 1;
          double v = 1.0;
          if (cs.kind == 0) v = (u2[k] < 0.03 && !near_goal && !near_start) ? -1.0 : 1.0 + 4.0 * u[k];
          if (cs.kind == 2) v = u[k] < 0.5 ? 1.0 : 2.0;
          cost[j][i] = v;
          F[k] = v > 0 ? v : INFINITY;
        }
      DyMuPathPlanner p(1.0, 2.0, 5.0, CONSERVATIVE);
      p.initGlobalLayer(1.0, 0.5, N, N, {0.0, 0.0});
      p.setCostMap(cost);
      if (!p.setGoal(wp(cs.gi, cs.gj))) return 2;
      if (cs.si < 0)
        p.computeEntireTotalCostMap();
      else
        p.computeTotalCostMap(wp(cs.si, cs.sj));
      std::vector<uint8_t> closed((uint64_t)N * N);
      std::vector<uint64_t> seq((uint64_t)N * N);
      oracle_fmm_order(F.data(), N, N, cs.gi, cs.gj, cs.si, cs.sj, T.data(), closed.data(),
                       seq.data());
      std::vector<std::pair<uint64_t, uint64_t>> want;
      for (uint64_t k = 0; k < T.size(); ++k)
        if (T[k] < INFINITY) want.push_back({seq[k], k});
      std::sort(want.begin(), want.end());
      const auto got = p.globalPropagatedNodes();
      const auto got_k = p.globalPropagatedIndices();  // the flat ABI's form: the same list
      uint64_t cbad = got.size() != want.size() || got_k.size() != got.size();
      for (size_t q = 0; q < got.size() && !cbad; ++q)
        cbad = got_k[q] != (uint64_t)got[q].pose.position[1] * N + (uint64_t)got[q].pose.position[0];
      for (size_t q = 0; q < got.size() && q < want.size() && !cbad; ++q) {
        const uint64_t k =
            (uint64_t)got[q].pose.position[1] * N + (uint64_t)got[q].pose.position[0];
        if (k != want[q].second) {
          std::printf("  first difference at %zu: (%u,%u) vs (%u,%u)\n", q, (unsigned)(k % N),
                      (unsigned)(k / N), (unsigned)(want[q].second % N),
                      (unsigned)(want[q].second / N));
          cbad = 1;
        }
      }
      std::printf("order N=%u kind=%d start=(%d,%d) reached=%zu bad=%llu\n", N, cs.kind, cs.si,
                  cs.sj, want.size(), (unsigned long long)cbad);
      bad += cbad;
    }
    return bad == 0 ? 0 : 1;
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
