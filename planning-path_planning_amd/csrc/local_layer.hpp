// local_layer.hpp -- storage of the DyMu local layer (sub-grid of the
// subdivided global nodes) behind DyMuPathPlanner (include/DyMu.hpp).
//
// The reference (src/DyMu_LocalPathRepairing.cpp:23-145) allocates one
// localNode record per sub-cell with an nb4 pointer list and links the lists
// across global nodes as they get subdivided.  Here a subdivided global node
// owns a block of res_ratio x res_ratio sub-cells in SoA pools; a sub-cell is
// named by p = block * r*r + lj * r + li, neighbours are implicit inside a
// block and found through a 4-entry block adjacency across blocks (linked in
// both directions when a block is created, so a cross-block neighbour exists
// iff both global nodes are subdivided -- exactly the reference's links).
// Poses are recomputed from (block, li, lj) with the reference's expression
// order instead of being stored.
#pragma once

#include <cmath>
#include <cstdint>
#include <deque>
#include <unordered_map>
#include <vector>

#include "dymu_base.hpp"

namespace PathPlanning_lib {

// (uint) of a double as the reference's x86-64 GCC build converts it: through
// int64 (cvttsd2si), so -1 < d < 0 gives 0 and more negative values wrap to
// huge indices that every bounds test rejects.  A plain cast of a negative
// double to unsigned is undefined behaviour in C++.
inline uint32_t grid_u32(double d) {
  return (d > -9.2e18 && d < 9.2e18) ? (uint32_t)(int64_t)d : 0u;
}

// Waypoints of current_path bucketed on a square grid of cell size 1.5 x
// risk_distance, for isBlockingObstacle (:441-471).  The reference scans the
// whole path for every obstacle pixel; the first waypoint within risk_distance
// of a point can only lie in the 3x3 cells around it (any pair closer than
// risk_distance is less than 2/3 of a cell apart on each axis), and the
// reference's scan changes nothing before that waypoint -- so the index gives
// the same result from a handful of candidates.
struct PathIndex {
  double cs = 0.0;
  std::unordered_map<uint64_t, std::vector<uint32_t>> cells;  // ascending indices
  static int64_t cell(double v, double cs) { return (int64_t)std::floor(v / cs); }
  static uint64_t key(int64_t cx, int64_t cy) {
    return ((uint64_t)(uint32_t)(int32_t)cx << 32) | (uint64_t)(uint32_t)(int32_t)cy;
  }
  // false when the index cannot be used (the caller scans the path instead)
  bool build(const std::vector<base::Waypoint>& path, double rd) {
    cells.clear();
    if (!(rd > 0) || !(rd < 1e300)) return false;
    cs = 1.5 * rd;
    for (uint32_t k = 0; k < path.size(); ++k) {
      const double x = path[k].position[0], y = path[k].position[1];
      if (!(std::fabs(x / cs) < 1e9) || !(std::fabs(y / cs) < 1e9)) return false;  // NaN / far
      cells[key(cell(x, cs), cell(y, cs))].push_back(k);
    }
    return true;
  }
};

struct LocalLayer {
  unsigned r = 1;   // res_ratio
  uint64_t rr = 1;  // r * r
  std::unordered_map<uint64_t, uint32_t> block_of;  // global node -> block
  std::vector<uint64_t> block_g;                     // block -> global node
  std::vector<int32_t> block_nb;                     // 4 per block, -1 = none
  // SoA sub-cell fields (localNode, src/DyMu.hpp:42-67)
  std::vector<double> dev, tc, risk;
  std::vector<uint8_t> state, obst;
  // narrow band of the local FMM: a min-heap of (key, first-insertion
  // sequence) with lazy deletion.  The reference's band is a vector scanned
  // for the first strict minimum (:752-805); it keeps insertion order under
  // erase, so (key, sequence) order pops the same node.
  struct Entry {
    double key;
    uint32_t seq;
    uint64_t p;
  };
  std::vector<Entry> heap;
  std::vector<uint8_t> in_band;
  std::vector<uint32_t> seq;
  uint32_t next_seq = 0;
  uint64_t band_count = 0;
  std::vector<uint64_t> propagated;   // local_propagated_nodes
  std::deque<uint64_t> expandable;    // local_expandable_obstacles

  void reset(unsigned res_ratio) {
    *this = LocalLayer();
    r = res_ratio;
    rr = (uint64_t)r * r;
  }
  int64_t block(uint64_t g) const {
    auto it = block_of.find(g);
    return it == block_of.end() ? -1 : (int64_t)it->second;
  }
  // subdivide global node g = j*nx + i (createLocalMap, :23-145)
  void create(uint64_t g, unsigned nx, unsigned ny) {
    const uint32_t b = (uint32_t)block_g.size();
    block_of.emplace(g, b);
    block_g.push_back(g);
    block_nb.resize(block_nb.size() + 4, -1);
    const uint64_t n = block_g.size() * rr;
    dev.resize(n, kInf());
    tc.resize(n, kInf());
    risk.resize(n, 0.0);
    state.resize(n, 0);
    obst.resize(n, 0);
    in_band.resize(n, 0);
    seq.resize(n, 0);
    const unsigned i = (unsigned)(g % nx), j = (unsigned)(g / nx);
    // nb4 order {(i,j-1), (i-1,j), (i+1,j), (i,j+1)}; opposite of d is 3-d
    const int64_t o[4] = {j > 0 ? (int64_t)(g - nx) : -1, i > 0 ? (int64_t)(g - 1) : -1,
                          i + 1 < nx ? (int64_t)(g + 1) : -1, j + 1 < ny ? (int64_t)(g + nx) : -1};
    for (int d = 0; d < 4; ++d) {
      if (o[d] < 0) continue;
      const int64_t ob = block((uint64_t)o[d]);
      if (ob < 0) continue;
      block_nb[4 * b + d] = (int32_t)ob;
      block_nb[4 * ob + 3 - d] = (int32_t)b;
    }
  }
  // nb4List[d] of sub-cell p, -1 = NULL
  int64_t nb(uint64_t p, int d) const {
    const uint64_t b = p / rr, q = p % rr;
    const unsigned li = (unsigned)(q % r), lj = (unsigned)(q / r);
    switch (d) {
      case 0:
        if (lj > 0) return (int64_t)(p - r);
        return block_nb[4 * b] < 0 ? -1 : (int64_t)(block_nb[4 * b] * rr + (uint64_t)(r - 1) * r + li);
      case 1:
        if (li > 0) return (int64_t)(p - 1);
        return block_nb[4 * b + 1] < 0 ? -1 : (int64_t)(block_nb[4 * b + 1] * rr + (uint64_t)lj * r + r - 1);
      case 2:
        if (li + 1 < r) return (int64_t)(p + 1);
        return block_nb[4 * b + 2] < 0 ? -1 : (int64_t)(block_nb[4 * b + 2] * rr + (uint64_t)lj * r);
      default:
        if (lj + 1 < r) return (int64_t)(p + r);
        return block_nb[4 * b + 3] < 0 ? -1 : (int64_t)(block_nb[4 * b + 3] * rr + li);
    }
  }
  static double kInf() { return __builtin_inf(); }
};

}  // namespace PathPlanning_lib
