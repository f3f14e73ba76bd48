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
#pragma once

#include <cmath>
#include <cstdint>
#include <unordered_map>

namespace PathPlanning_lib {

template <class TFn>  // double TFn(uint64_t k): total cost of cell k (+inf unreached)
class PopOrder {
 public:
  PopOrder(TFn t, uint32_t nx, uint32_t ny, uint64_t goal)
      : T_(t), nx_(nx), ny_(ny), goal_(goal) {}

  // pop(x) < pop(y) for finite T(x), T(y); false for x == y
  bool popBefore(uint64_t x, uint64_t y) {
    if (x == y) return false;
    const double tx = T_(x), ty = T_(y);
    if (tx != ty) return tx < ty;
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
      const double ta = T_((uint64_t)ax), tb = T_((uint64_t)ay);
      if (ta != tb) {
        r = ta < tb;
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
    double tb = __builtin_inf();
    for (int q = 0; q < m; ++q) tb = std::fmin(tb, T_(nb[q]));
    int64_t best = -1;
    if (tb < __builtin_inf())
      for (int q = 0; q < m; ++q)  // the least value; equal ones by their pop order
        if (T_(nb[q]) == tb && (best < 0 || popBefore(nb[q], (uint64_t)best)))
          best = (int64_t)nb[q];
    if (best >= 0 && !(tb < T_(x))) {  // the least neighbour ties with x itself
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
