// Test harness (CPU): exposes csrc/pop_order.hpp over a plain T array so that
// tests/test_pop_order.py can compare the rebuilt order with the oracle's recorded
// band-insertion sequence.  Built by the test with g++; not product code.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "pop_order.hpp"

using PathPlanning_lib::PopOrder;

namespace {
struct ArrayT {
  const double* t;
  double operator()(uint64_t k) const { return t[k]; }
};
}  // namespace

extern "C" {
// cells sorted into insertion order (stable); returns 1 if the order was degenerate
int po_ins_sort(const double* T, uint32_t nx, uint32_t ny, uint64_t goal, uint64_t* cells,
                uint64_t n) {
  PopOrder<ArrayT> po(ArrayT{T}, nx, ny, goal);
  std::stable_sort(cells, cells + n, [&po](uint64_t x, uint64_t y) { return po.insBefore(x, y); });
  return po.degenerate() ? 1 : 0;
}

// out[q] = pop(x[q]) < pop(y[q]); returns 1 if degenerate
int po_pop_before(const double* T, uint32_t nx, uint32_t ny, uint64_t goal, const uint64_t* x,
                  const uint64_t* y, uint64_t n, uint8_t* out) {
  PopOrder<ArrayT> po(ArrayT{T}, nx, ny, goal);
  for (uint64_t q = 0; q < n; ++q) out[q] = po.popBefore(x[q], y[q]) ? 1 : 0;
  return po.degenerate() ? 1 : 0;
}
}
