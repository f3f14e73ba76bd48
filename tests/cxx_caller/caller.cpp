// caller.cpp -- a Rock-style C++ caller of the drop-in class surface
// (include/DyMu.hpp, linked against libdymu_planner.so), written against the
// reference's own signatures (src/DyMu.hpp:484-537): the cost map as
// std::vector<std::vector<double>>, positions as base::Waypoint, the total cost
// back as std::vector<std::vector<double>>.  tests/test_cxx_caller.py builds it
// on the GPU box and compares what it writes with the goldens / the oracle.
//
//   caller cost.bin N goal_i goal_j start_x start_y early.bin full.bin path.bin
// writes: early.bin  getTotalCostMatrix after computeTotalCostMap(start)
//         full.bin   getTotalCostMatrix after computeEntireTotalCostMap()
//         path.bin   getPath(start) as (x, y, z, heading) per waypoint
// prints: "rc <computeTotalCostMap> <computeEntireTotalCostMap> <waypoints>"
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "DyMu.hpp"

using PathPlanning_lib::DyMuPathPlanner;

static bool write_matrix(const char* f, const std::vector<std::vector<double>>& M) {
  FILE* o = std::fopen(f, "wb");
  if (!o) return false;
  for (const auto& row : M) std::fwrite(row.data(), sizeof(double), row.size(), o);
  return std::fclose(o) == 0;
}

int main(int argc, char** argv) {
  if (argc != 10) return 2;
  const unsigned N = (unsigned)std::atoi(argv[2]);
  std::vector<std::vector<double>> cost(N, std::vector<double>(N));
  FILE* in = std::fopen(argv[1], "rb");
  if (!in) return 2;
  for (auto& row : cost)
    if (std::fread(row.data(), sizeof(double), N, in) != N) return 2;
  std::fclose(in);

  DyMuPathPlanner planner(1.0, 2.0, 5.0, PathPlanning_lib::CONSERVATIVE);
  planner.initGlobalLayer(1.0, 0.5, N, N, std::vector<double>{0.0, 0.0});
  if (!planner.setCostMap(cost)) return 3;
  base::Waypoint goal;
  goal.position[0] = std::atof(argv[3]);
  goal.position[1] = std::atof(argv[4]);
  goal.heading = 0.0;
  if (!planner.setGoal(goal)) return 4;
  base::Waypoint start;
  start.position[0] = std::atof(argv[5]);
  start.position[1] = std::atof(argv[6]);
  start.heading = 0.0;
  const bool early = planner.computeTotalCostMap(start);
  if (!write_matrix(argv[7], planner.getTotalCostMatrix())) return 5;
  const bool full = planner.computeEntireTotalCostMap();
  if (!write_matrix(argv[8], planner.getTotalCostMatrix())) return 5;
  const std::vector<base::Waypoint> path = planner.getPath(start);
  FILE* o = std::fopen(argv[9], "wb");
  if (!o) return 5;
  for (const auto& w : path) {
    const double v[4] = {w.position[0], w.position[1], w.position[2], w.heading};
    std::fwrite(v, sizeof(double), 4, o);
  }
  std::fclose(o);
  std::printf("rc %d %d %zu\n", (int)early, (int)full, path.size());
  return 0;
}
