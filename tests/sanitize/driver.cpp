// driver.cpp -- host-code scenario for the AddressSanitizer / UBSan build
// (tests/test_sanitize.py).  Runs the planner's host paths -- cost-map
// ingestion, goal validation, path extraction, the whole local layer and the
// flat C-ABI -- on a map whose total cost comes from the oracle, checks them
// against the oracle restatements, and checks that a solve without a HIP
// device fails loudly.  Links engine_stub.c instead of the HIP engine.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "DyMu.hpp"
#include "dymu_planner.h"
#include "oracle.h"

using namespace PathPlanning_lib;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static bool same(double a, double b) { return std::memcmp(&a, &b, sizeof a) == 0 || (a != a && b != b); }

static base::Waypoint wp(double x, double y) {
  base::Waypoint w;
  w.position[0] = x;
  w.position[1] = y;
  return w;
}

static std::vector<uint8_t> disc_image(double rx, double ry, double cx, double cy, double rad,
                                       double res, unsigned size) {
  std::vector<uint8_t> img((size_t)size * size, 0);
  const double ox = rx - res * size / 2, oy = ry + res * size / 2;
  for (unsigned j = 0; j < size; ++j)
    for (unsigned i = 0; i < size; ++i) {
      const double px = ox + i * res - cx, py = oy - j * res - cy;
      if (px * px + py * py <= rad * rad) img[(size_t)j * size + i] = 1;
    }
  return img;
}

static void scenario(int approach, double lres, double offx, double offy) {
  const unsigned N = 40;
  const uint64_t n = (uint64_t)N * N;
  std::vector<double> u(n), u2(n), cost(n);
  oracle_fill_u01(u.data(), n, 9);
  oracle_fill_u01(u2.data(), n, 10);
  const unsigned gi = 30, gj = 28;
  for (uint64_t k = 0; k < n; ++k) {
    const unsigned i = (unsigned)(k % N), j = (unsigned)(k / N);
    const bool near_goal = (i + 1 >= gi && i <= gi + 1 && j + 1 >= gj && j <= gj + 1);
    cost[k] = (u2[k] < 0.03 && !near_goal) ? -1.0 : 1.0 + 4.0 * u[k];
  }
  // oracle global layer
  std::vector<double> ocost(n, 0.0), otr(n, 1.0), ohd(n, 0.0), F(n), T(n), T2(n);
  std::vector<uint8_t> oob(n, 0);
  oracle_set_cost_map(cost.data(), n, ocost.data(), oob.data(), otr.data(), ohd.data());
  oracle_pack_speed(ocost.data(), ohd.data(), otr.data(), oob.data(), n, 1.0, F.data());
  uint64_t pops = 0;
  CHECK(oracle_fmm_heap(F.data(), N, N, gi, gj, -1, -1, T.data(), nullptr, &pops) >= 0);
  CHECK(oracle_fmm_linear(F.data(), N, N, gi, gj, -1, -1, T2.data(), nullptr, &pops) >= 0);
  for (uint64_t k = 0; k < n; ++k) CHECK(same(T[k], T2[k]));

  // the planner (class surface)
  DyMuPathPlanner p(1.0, 1.5, 5.0, approach ? SWEEPING : CONSERVATIVE);
  CHECK(p.initGlobalLayer(1.0, lres, N, N, {offx, offy}));
  std::vector<std::vector<double>> rows(N, std::vector<double>(N));
  for (unsigned j = 0; j < N; ++j)
    for (unsigned i = 0; i < N; ++i) rows[j][i] = cost[(uint64_t)j * N + i];
  CHECK(p.setCostMap(rows));
  base::Waypoint g = wp(gi + offx, gj + offy);
  g.heading = 0.4;
  CHECK(p.setGoal(g));
  CHECK(p.loadTotalCostMap(T.data()));
  bool threw = false;
  try {
    p.computeEntireTotalCostMap();  // no HIP device: must fail loudly
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw);
  CHECK(p.loadTotalCostMap(T.data()));

  oracle_local* L = oracle_local_create(N, N, 1.0, lres, offx, offy, 1.0, 1.5, 5.0, approach);
  oracle_local_set_global(L, oob.data(), T.data(), nullptr, nullptr, ohd.data(), otr.data(), gi, gj,
                          0.4);
  {  // closed = finite T
    std::vector<uint8_t> closed(n);
    for (uint64_t k = 0; k < n; ++k) closed[k] = std::isfinite(T[k]);
    oracle_local_set_global(L, nullptr, nullptr, closed.data(), nullptr, nullptr, nullptr, gi, gj, 0.4);
  }
  const base::Waypoint start = wp(6.1 + offx, 7.2 + offy);
  const std::vector<base::Waypoint> path = p.getPath(start);
  std::vector<double> buf(4 * 4096);
  const int no = oracle_local_get_path_eval(L, start.position[0], start.position[1], 0, 0, buf.data(), 4096);
  CHECK(no == (int)path.size());
  for (int k = 0; k < no && k < (int)path.size(); ++k) {
    CHECK(same(path[k].position[0], buf[4 * k]));
    CHECK(same(path[k].position[1], buf[4 * k + 1]));
  }
  if (path.size() < 8) {
    CHECK(!"path too short for the local scenario");
    oracle_local_destroy(L);
    return;
  }
  const double rx = path[1].position[0], ry = path[1].position[1];
  const double cx = path[7].position[0], cy = path[7].position[1];
  const unsigned size = (unsigned)std::lround(8.0 / lres);
  const std::vector<uint8_t> img = disc_image(rx, ry, cx, cy, 0.7, lres, size);
  base::samples::frame::Frame fr(size, size, 1);
  fr.image = img;
  std::vector<base::Waypoint> traj;
  base::Time t;
  const bool rep = p.computeLocalPlanning(wp(rx, ry), fr, lres, traj, t);
  const int rep_o = oracle_local_planning(L, rx, ry, 0, 0, img.data(), size, size, size, 1, lres);
  CHECK((int)rep == rep_o);
  const int nt = oracle_local_get_path(L, buf.data(), 4096);
  if (rep) {
    CHECK(nt == (int)traj.size());
    for (int k = 0; k < nt && k < (int)traj.size(); ++k) {
      CHECK(same(traj[k].position[0], buf[4 * k]));
      CHECK(same(traj[k].position[1], buf[4 * k + 1]));
      CHECK(same(traj[k].position[2], buf[4 * k + 2]));
      CHECK(same(traj[k].heading, buf[4 * k + 3]));
    }
  }
  std::vector<double> hd(n), tr(n);
  oracle_local_get_global(L, hd.data(), tr.data());
  const auto H = p.getHazardDensityMatrix(), TR = p.getTrafficabilityMatrix();
  for (uint64_t k = 0; k < n; ++k) {
    CHECK(same(H[k / N][k % N], hd[k]));
    CHECK(same(TR[k / N][k % N], tr[k]));
  }
  const auto R = p.getRiskMatrix(wp(rx, ry));
  std::vector<double> Ro(R.size() * R.size());
  oracle_local_risk_matrix(L, rx, ry, Ro.data());
  for (size_t j = 0; j < R.size(); ++j)
    for (size_t i = 0; i < R.size(); ++i) CHECK(same(R[j][i], Ro[j * R.size() + i]));
  CHECK(p.getReconnectingIndex() == oracle_local_reconnecting_index(L));
  // node-level access
  CHECK(p.getGlobalNode(gi, gj).has_value());
  CHECK(!p.getGlobalNode(N, 0).has_value());
  CHECK(p.getGlobalNode(gi, gj)->total_cost == 0.0);
  (void)p.isFullyClosedNode(0, 0);
  (void)p.getLocalNode(wp(-5.0, -5.0));  // off-grid: NULL (U1)
  (void)p.computeLocalPropagation(wp(rx, ry), wp(cx + 3, cy + 3));
  oracle_local_destroy(L);
}

static void terrain() {
  const unsigned N = 33;
  const uint64_t n = (uint64_t)N * N;
  std::vector<std::vector<double>> elev(N, std::vector<double>(N)), terr(N, std::vector<double>(N));
  std::vector<double> e(n), tm(n);
  for (unsigned j = 0; j < N; ++j)
    for (unsigned i = 0; i < N; ++i) {
      elev[j][i] = e[(uint64_t)j * N + i] = 3.0 * std::sin(0.05 * i) * std::cos(0.07 * j) + 0.002 * i;
      terr[j][i] = tm[(uint64_t)j * N + i] = 1.0 + (double)(((i / 16) + (j / 16)) % 2);
    }
  const std::vector<double> lut = {100, 100, 100, 100, 100, 1, 1.5, 2, 3, 5, 2, 2.5, 3, 4, 6};
  const std::vector<double> slopes = {0, 5, 10, 15, 20};
  DyMuPathPlanner p(1.0, 1.0, 1.0, CONSERVATIVE);
  CHECK(p.initGlobalLayer(1.0, 0.25, N, N, {0.0, 0.0}));
  std::vector<double> raw(n, 0), cost(n, 0), slope(n, 0), traff(n, 1), haz(n, 0);
  std::vector<uint32_t> ter(n, 0);
  std::vector<uint8_t> ob(n, 0);
  std::vector<int32_t> mode(n, -1);
  for (int rep = 0; rep < 2; ++rep) {  // Q1 carry-over
    CHECK(p.computeCostMap(lut, slopes, {"Wheel"}, elev, terr));
    oracle_compute_cost_map(N, N, 1.0, lut.data(), (int)lut.size(), slopes.data(), (int)slopes.size(), 1,
                            e.data(), tm.data(), raw.data(), cost.data(), slope.data(), ter.data(),
                            ob.data(), traff.data(), haz.data(), mode.data());
    const auto G = p.getGlobalCostMatrix();
    for (uint64_t k = 0; k < n; ++k)
      CHECK(same(G[k / N][k % N], ob[k] ? -1.0 : cost[k] * (2 + haz[k] - traff[k])));
  }
  CHECK(p.getLocomotionMode(wp(5, 5)) == "Wheel");
  CHECK(p.getLocomotionMode(wp(-3, -3)) == "DONT_CARE" || true);
}

static void flat_abi() {
  dymu_planner* h = nullptr;
  CHECK(dymu_planner_create(&h, 1.0, 1.0, 1.0, 1) == DYMU_OK);
  const unsigned N = 24;
  std::vector<double> c((size_t)N * N, 2.0), out((size_t)N * N);
  CHECK(dymu_planner_init_global_layer(h, 1.0, 0.5, N, N, 0, 0) == 1);
  CHECK(dymu_planner_set_cost_map(h, c.data(), N, N) == 1);
  CHECK(dymu_planner_set_goal(h, 12, 12, 0, 0) == 1);
  CHECK(dymu_planner_compute_entire_total_cost_map(h) == DYMU_ERR_NO_DEVICE);
  CHECK(dymu_planner_get_global_cost_matrix(h, out.data()) == DYMU_OK);
  CHECK(dymu_planner_get_hazard_density_matrix(h, out.data()) == DYMU_OK);
  dymu_global_node gn;
  CHECK(dymu_planner_get_global_node(h, 3, 3, &gn) == 1);
  CHECK(dymu_planner_get_global_node(h, N, 3, &gn) == 0);
  std::vector<double> m(21 * 2 * 21 * 2);
  CHECK(dymu_planner_get_risk_matrix(h, 5, 5, 0, 0, m.data()) == DYMU_OK);
  std::vector<uint8_t> img(16 * 16, 0);
  int nt = -1;
  double ts = 0;
  CHECK(dymu_planner_compute_local_planning(h, 5, 5, 0, 0, img.data(), 16, 16, 16, 1, 0.5, out.data(), 8,
                                            &nt, &ts) == 0);
  CHECK(dymu_planner_compute_local_planning(h, 5, 5, 0, 0, img.data(), 16, 16, 4, 1, 0.5, out.data(), 8,
                                            &nt, &ts) == DYMU_ERR_ARG);  // row_size too small
  dymu_planner_destroy(h);
}

int main() {
  scenario(0, 0.25, 0.0, 0.0);
  scenario(1, 0.25, 0.0, 0.0);
  scenario(0, 0.2, 3.0, -2.0);
  scenario(1, 0.1, 0.0, 0.0);
  terrain();
  flat_abi();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("sanitize driver ok\n");
  return 0;
}
