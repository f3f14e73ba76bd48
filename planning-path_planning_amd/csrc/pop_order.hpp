// pop_order.hpp -- the reference FMM's pop and insertion order, rebuilt from the
// total costs alone (computeTotalCostMap's exit state).
//
// The reference FMM (src/DyMu_GlobalPathPlanning.cpp:364-408, :443-468) pops the band
// node of least total cost, the first one in band order on ties (minCostGlobalNode
// :551-568).  The band is a vector appended when a node first becomes finite
// (propagateGlobalNode :537-545) and erased in place, so band order is
// first-insertion order.  A node becomes finite when its first neighbour is popped:
// every pop updates its OPEN, non-obstacle nb4 (:392-396, :462-465), and the first
// update of a node always gives a finite value.  One pop inserts in nb4List order
// (i,j-1), (i-1,j), (i+1,j), (i,j+1) (src/DyMu.hpp:76-80).  So, with the final values T:
//
//   pop(x) < pop(y)  <=>  T(x) < T(y),  or  T(x) == T(y) and ins(x) < ins(y)
//   ins(x) < ins(y)  <=>  pop(a(x)) < pop(a(y)),  or  a(x) == a(y) and x precedes y
//                         in a(x)'s nb4 order
//
// where a(x), the first-popped neighbour of x, is its neighbour of least T (ties:
// pop order again); the goal is inserted before everything (:487-498).  A comparison
// thus walks two chains toward the goal, each step to strictly smaller T, with a(.)
// memoised.  When a node's least neighbour has the node's own value (a speed below
// the rounding of the total cost) its insertion is not determined by the values:
// degenerate() is set and the caller must not trust the answers.
//
// The values are the GPU engine's: within ~1e-14 of the reference's, not equal to
// them.  So an order read off them stands for the reference's only
// where no rounding can flip it -- TieGuard: two values more than eps apart
// (relative), or exactly equal at mirror images about the goal where every value
// they depend on lies in a disc of constant speed (the reference computes those two
// values alike, by symmetry).  Any other comparison is a near tie: counted, and
// the caller must not trust the answers (the planner then replays the reference
// exactly on the host).  Without a guard the values are taken as exact (the
// oracle's, in the tests).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <unordered_map>
#include <utility>

namespace PathPlanning_lib {

struct TieGuard {
  double eps = 1e-12;  // relative: well above the engine's measured 1e-14 deviation
  int64_t nx = 0, gi = 0, gj = 0;
  // Mirror ties are trusted below this value: the goal's speed F0 times the distance R
  // from the goal to the nearest cell of another speed (obstacles included).  Every cell
  // whose reference value is below F0 R lies within R of the goal (on constant speed the
  // FMM's values are at least F0 times the Euclidean distance), so those values are the
  // constant-speed plane's -- a value depends only on smaller ones, an upwind neighbour is
  // nearer the goal, and the grid's edges cut off nothing a value depends on -- and the
  // plane's are equal at mirror images about the goal (the update is symmetric in its two
  // axes and in each axis's two sides).
  double trust_below = 0.0;
  uint64_t near = 0;  // near ties met
  uint64_t first[2] = {0, 0};  // the first near tie's cells and values
  double first_t[2] = {0.0, 0.0};

  TieGuard() = default;
  TieGuard(int64_t nx_, int64_t gi_, int64_t gj_, double f0, double r)
      : nx(nx_), gi(gi_), gj(gj_),
        trust_below(f0 < __builtin_inf() && f0 > 0.0 ? f0 * r * (1.0 - 1e-9) : 0.0) {}
  // a and b mirror images of each other about the goal (any of the 8 symmetries of
  // the square lattice)
  bool mirror(uint64_t a, uint64_t b) const {
    int64_t ax = std::llabs((int64_t)(a % (uint64_t)nx) - gi);
    int64_t ay = std::llabs((int64_t)(a / (uint64_t)nx) - gj);
    int64_t bx = std::llabs((int64_t)(b % (uint64_t)nx) - gi);
    int64_t by = std::llabs((int64_t)(b / (uint64_t)nx) - gj);
    if (ax > ay) std::swap(ax, ay);
    if (bx > by) std::swap(bx, by);
    return ax == bx && ay == by;
  }
  // the order of a's value ta against b's value tb: -1, 0 (a tie), +1.  Mirror images
  // within the constant-speed disc tie (the reference's values are equal; the engine's
  // may differ by a few ulps); any other comparison rounding could flip is counted as a
  // near tie (its answer is then the raw one)
  int cmp(uint64_t a, double ta, uint64_t b, double tb) {
    int r = ta < tb ? -1 : ta > tb ? 1 : 0;
    if (a == b || !(ta < __builtin_inf()) || !(tb < __builtin_inf())) return r;  // +inf is exact
    const bool close = r == 0 || std::fabs(ta - tb) <= eps * std::fmax(ta, tb);
    if (!close) return r;
    if (std::fmax(ta, tb) < trust_below && mirror(a, b)) return 0;
    {
      if (near++ == 0) {  // the first one, for diagnostics
        first[0] = a;
        first[1] = b;
        first_t[0] = ta;
        first_t[1] = tb;
      }
    }
    return r;
  }
};

template <class TFn>  // double TFn(uint64_t k): total cost of cell k (+inf unreached)
class PopOrder {
 public:
  // guard: null = the values are exact (trust every comparison)
  PopOrder(TFn t, uint32_t nx, uint32_t ny, uint64_t goal, TieGuard* guard = nullptr)
      : T_(t), nx_(nx), ny_(ny), goal_(goal), guard_(guard) {}

  // the order of two cells' values through the guard (if any)
  int cmp(uint64_t a, double ta, uint64_t b, double tb) {
    if (guard_) return guard_->cmp(a, ta, b, tb);
    return ta < tb ? -1 : ta > tb ? 1 : 0;
  }

  // pop(x) < pop(y) for finite T(x), T(y); false for x == y
  bool popBefore(uint64_t x, uint64_t y) {
    if (x == y) return false;
    const int c = cmp(x, T_(x), y, T_(y));
    if (c != 0) return c < 0;
    return insBefore(x, y);
  }

  // ins(x) < ins(y) (band-insertion order) for reached x, y; false for x == y
  bool insBefore(uint64_t x, uint64_t y) {
    if (++depth_ > kMaxDepth) {  // nested tie walks: give up rather than recurse on
      degenerate_ = true;
      why_ = 1;
      why_cell_ = x;
      --depth_;
      return x < y;
    }
    bool r = x < y;
    for (;;) {
      if (x == y) {
        r = false;
        break;
      }
      if (x == goal_ || y == goal_) {
        r = x == goal_;
        break;
      }
      const int64_t ax = firstPopped(x), ay = firstPopped(y);
      if (ax < 0 || ay < 0) {  // degenerate: keep a deterministic answer
        r = x < y;
        break;
      }
      if (ax == ay) {
        r = nbSlot((uint64_t)ax, x) < nbSlot((uint64_t)ax, y);
        break;
      }
      const int c = cmp((uint64_t)ax, T_((uint64_t)ax), (uint64_t)ay, T_((uint64_t)ay));
      if (c != 0) {
        r = c < 0;
        break;
      }
      x = (uint64_t)ax;  // pop(a(x)) vs pop(a(y)) at equal values: their insertions
      y = (uint64_t)ay;
    }
    --depth_;
    return r;
  }

  // a(x): the neighbour whose pop inserted x; -1 for the goal or when undetermined
  int64_t firstPopped(uint64_t x) {
    if (x == goal_) return -1;
    auto it = memo_.find(x);
    if (it != memo_.end()) return it->second;
    const uint32_t i = (uint32_t)(x % nx_), j = (uint32_t)(x / nx_);
    uint64_t nb[4];
    int m = 0;
    if (j > 0) nb[m++] = x - nx_;
    if (i > 0) nb[m++] = x - 1;
    if (i + 1 < nx_) nb[m++] = x + 1;
    if (j + 1 < ny_) nb[m++] = x + nx_;
    int64_t best = -1;
    double tb = __builtin_inf();
    for (int q = 0; q < m; ++q) {  // the least value (the first such in nb4 order) ...
      const double t = T_(nb[q]);
      if (t < tb) {
        best = (int64_t)nb[q];
        tb = t;
      }
    }
    if (best >= 0) {  // ... and the ones equal to it by their pop order
      const uint64_t least = (uint64_t)best;
      for (int q = 0; q < m; ++q) {
        const double t = T_(nb[q]);
        if (nb[q] == least || !(t < __builtin_inf())) continue;
        if (cmp(nb[q], t, least, tb) == 0 && popBefore(nb[q], (uint64_t)best))
          best = (int64_t)nb[q];
      }
    }
    if (best >= 0 && cmp((uint64_t)best, tb, x, T_(x)) >= 0) {  // the least neighbour ties with x
      degenerate_ = true;
      why_ = 2;
      why_cell_ = x;
      best = -1;
    }
    memo_.emplace(x, best);
    return best;
  }

  bool degenerate() const { return degenerate_; }
  // diagnostics: 1 = tie walks nested too deep, 2 = a node ties with its least
  // neighbour; the node concerned
  int why() const { return why_; }
  uint64_t whyCell() const { return why_cell_; }

 private:
  // position of neighbour x in p's nb4List (0 (i,j-1), 1 (i-1,j), 2 (i+1,j), 3 (i,j+1))
  int nbSlot(uint64_t p, uint64_t x) const {
    if (x + nx_ == p) return 0;
    if (x + 1 == p) return 1;
    if (x == p + 1) return 2;
    return 3;
  }

  static constexpr int kMaxDepth = 4096;
  TFn T_;
  uint32_t nx_, ny_;
  uint64_t goal_;
  TieGuard* guard_;
  std::unordered_map<uint64_t, int64_t> memo_;
  int depth_ = 0;
  bool degenerate_ = false;
  int why_ = 0;
  uint64_t why_cell_ = 0;
};

template <class TFn>
PopOrder<TFn> makePopOrder(TFn t, uint32_t nx, uint32_t ny, uint64_t goal) {
  return PopOrder<TFn>(t, nx, ny, goal);
}

}  // namespace PathPlanning_lib
