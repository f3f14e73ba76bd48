// update_kernels.hip -- windowed re-propagation after a local speed change
// (the hazard bumps of reference
// src/DyMu_LocalPathRepairing.cpp:264-274 and trafficability drops :389-394
// change F = res*cost*(2+hd-tr) (src/DyMu_GlobalPathPlanning.cpp:527-528)
// inside a window W).
//
// Causality of the update (:531-535): a cell's converged value exceeds every
// neighbour value it was computed from (one-sided: min + C; two-sided:
// >= max(Tx, Ty) because |Tx-Ty| < C).  Let theta = min of the old T over W and
// its 1-cell ring.  A cell whose old T < theta depends on no cell of W, and no
// path through W can give it a smaller value (such a path leaves the ring at a
// value >= theta), so it keeps its value exactly.  Every other cell may change:
// reset it to +inf, seed the tiles where a reset cell touches a kept finite
// cell, and run the FIM.  New values of reset cells are >= theta, so theta is
// a valid priority key for the seeded tiles.  The result is the fixed point of
// a cold solve -- exactly for the reference arithmetic; with
// kernel 5's default sweep sqrt (a two-sided candidate within 36 ulp, which can
// fall a few ulp below max(Tx, Ty)) the causality bound, and so the result,
// hold within the solve tolerance (tests compare with the oracle at 1e-12).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fim_kernels.h"

namespace dymu {

namespace {

constexpr unsigned long long kInfBits = 0x7FF0000000000000ull;

__device__ __forceinline__ unsigned long long dbits(double v) {
  return (unsigned long long)__double_as_longlong(v);
}

// theta = min T over [i0,i1) x [j0,j1) (window plus ring, clipped); T >= 0 so
// the u64 bit patterns order like the doubles.
__global__ void k_window_min(const double* T, int64_t ld, uint32_t i0, uint32_t j0, uint32_t i1,
                             uint32_t j1, unsigned long long* out) {
  __shared__ unsigned long long s_min;
  if (threadIdx.x == 0) s_min = kInfBits;
  __syncthreads();
  const uint64_t w = i1 - i0, n = w * (uint64_t)(j1 - j0);
  unsigned long long m = kInfBits;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const double v = T[(int64_t)(j0 + c / w) * ld + (i0 + c % w)];
    const unsigned long long b = dbits(v);
    m = b < m ? b : m;
  }
  atomicMin(&s_min, m);
  __syncthreads();
  if (threadIdx.x == 0 && s_min != kInfBits) atomicMin(out, s_min);
}

// number of cells whose value is bitwise `value` (early-exit tie detection); with
// idx, also their indices j*nx + i (the first cap of them, in no particular order)
__global__ void k_count_equal(const double* T, int64_t ld, uint32_t nx, uint32_t ny,
                              unsigned long long vbits, unsigned long long* out, uint64_t* idx,
                              uint64_t cap) {
  const uint64_t n = (uint64_t)nx * ny;
  unsigned long long c = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (uint64_t)gridDim.x * blockDim.x) {
    if (dbits(T[(int64_t)(k / nx) * ld + (int64_t)(k % nx)]) != vbits) continue;
    if (idx) {  // matches are few: one atomic each
      const unsigned long long pos = atomicAdd(out, 1ull);
      if (pos < cap) idx[pos] = k;
    } else {
      ++c;
    }
  }
  if (idx) return;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// Reset every cell with old T >= theta (except the goal) and seed the tiles
// holding a reset, finite-speed cell next to a kept finite cell.  A neighbour
// read may race with its reset, but "old < theta" cells are never written, so
// the test below sees the same answer either way.
__global__ void k_reset_seed(UpdateArgs a) {
  const double theta = __longlong_as_double((long long)*a.theta_bits);
  const uint64_t n = (uint64_t)a.nx * a.ny;
  const uint32_t shard = blockIdx.x % kShards;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = (uint32_t)(c / a.nx), i = (uint32_t)(c % a.nx);
    const int64_t k = (int64_t)j * a.ld + i;
    if (i == a.gi && j == a.gj) continue;
    const double old = a.T[k];
    if (!(old >= theta)) continue;  // kept
    if (old < __builtin_inf()) a.T[k] = __builtin_inf();
    if (!(a.F[k] < __builtin_inf())) continue;  // obstacle: never updated
    // kept neighbour: old T < theta, or the goal (theta = 0 when the goal is in
    // the window or its ring)
    auto kept = [&](uint32_t ii, uint32_t jj, int64_t kk) {
      return a.T[kk] < theta || (ii == a.gi && jj == a.gj);
    };
    bool seed = false;
    if (j > 0) seed |= kept(i, j - 1, k - a.ld);
    if (i > 0) seed |= kept(i - 1, j, k - 1);
    if (i + 1 < a.nx) seed |= kept(i + 1, j, k + 1);
    if (j + 1 < a.ny) seed |= kept(i, j + 1, k + a.ld);
    if (!seed) continue;
    const uint32_t tile = (j / a.th) * a.ntx + (i / a.tw);
    if (atomicMax(&a.tile_epoch[tile], a.epoch) < a.epoch) {
      const uint32_t pos = atomicAdd(&a.counts[shard], 1u);
      a.list[(uint64_t)shard * a.shard_cap + pos] = tile;
      if (a.keys) atomicMin(&a.keys[tile], *a.theta_bits);  // priority kernels: key theta,
      if (a.hist) atomicAdd(&a.hist[shard * kBins], 1u);    // histogram bin 0
    }
  }
}

// Decrease-only change (every speed in W went down or stayed): the old map is a
// valid upper bound of the new fixed point everywhere, so no cell needs a reset.
// theta is a lower bound on every new value the passes can produce: with the goal
// outside W, a cell whose value changes has a new optimal path that enters W from
// its ring, so its new value is above min old T over the ring >= theta; with the
// goal inside W (or its ring) theta = T(goal) = 0, trivially a lower bound.  Seed
// every tile that intersects W (tiles [tx0,tx1) x [ty0,ty1)) with key theta; the
// passes then lower whatever the cheaper window reaches.
__global__ void k_seed_window(UpdateArgs a, uint32_t tx0, uint32_t ty0, uint32_t tx1,
                              uint32_t ty1) {
  const uint32_t w = tx1 - tx0, n = w * (ty1 - ty0);
  const uint32_t shard = blockIdx.x % kShards;
  for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const uint32_t tile = (ty0 + c / w) * a.ntx + (tx0 + c % w);
    if (atomicMax(&a.tile_epoch[tile], a.epoch) < a.epoch) {
      const uint32_t pos = atomicAdd(&a.counts[shard], 1u);
      a.list[(uint64_t)shard * a.shard_cap + pos] = tile;
      if (a.keys) atomicMin(&a.keys[tile], *a.theta_bits);
      if (a.hist) atomicAdd(&a.hist[shard * kBins], 1u);
    }
  }
}

// ---- raise front (increases inside the window) ----
// At a converged map every free non-goal cell satisfies T = u(T) (the update of its
// final neighbours), so after the speed of some cells went up and the cells whose
// support is gone were set to +inf, a cell keeps its value exactly when u, computed
// from its current neighbours under the new speed, does not exceed it.  The raise
// repeats that test until nothing changes, starting in the window: the result is the
// set of cells whose value depended on a raised cell (the dependency cone), every
// other cell keeps a value some path under the new speed still realises -- a valid
// upper bound of the new fixed point.  The FIM then re-solves the cone from its
// boundary.  tol absorbs the last-ulp non-monotonicity of the engine's sweep sqrt
// (<= 36 ulp): a cell kept within tol is off by at most tol relative.
__device__ __forceinline__ double ref_update(double tx, double ty, double c) {
  const double d = tx - ty;
  if ((fabs(d) < c) && (tx < __builtin_inf()) && (ty < __builtin_inf()))
    return (tx + ty + sqrt(2.0 * (c * c) - d * d)) / 2;  // :531-535
  return fmin(tx, ty) + c;
}

constexpr int RT = 16;       // raise tile edge (kernel 5's tiling)
constexpr int RP = RT + 2;   // image pitch

__global__ __launch_bounds__(256) void k_raise(RaiseArgs a) {
  __shared__ uint32_t s_pref[kShards + 1];
  __shared__ double s_img[4][RP * RP];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < kShards; ++k) {
      s_pref[k] = acc;
      acc += a.count_in[k];
    }
    s_pref[kShards] = acc;
  }
  __syncthreads();
  const uint32_t n = s_pref[kShards];
  if (blockIdx.x == 0 && tid < kShards) a.count_clear[tid] = 0u;
  const uint32_t shard = blockIdx.x % kShards;
  double* img = s_img[wv];
  const int r = lane >> 2, q = lane & 3;
  const double inf = __builtin_inf();
  unsigned long long visits = 0, cells = 0;
  const uint32_t nw = gridDim.x * 4u;
  for (uint32_t e = blockIdx.x * 4u + (uint32_t)wv; e < n; e += nw) {  // wave-uniform
    int k = 0;
    for (int s = 1; s < kShards; ++s) k += (e >= s_pref[s]) ? 1 : 0;
    const uint32_t tile = a.list_in[(uint64_t)k * a.shard_cap + (e - s_pref[k])] & kTileMask;
    const int64_t i0 = (int64_t)(tile % a.ntx) * RT, j0 = (int64_t)(tile / a.ntx) * RT;
    auto at = [&](int64_t i, int64_t j) -> double {
      return (i >= 0 && j >= 0 && i < a.nx && j < a.ny) ? a.T[j * a.ld + i] : inf;
    };
    // image: own cells (r, 4q..4q+3) and the halo ring
    double t[4], f[4];
    bool live[4];
    for (int c = 0; c < 4; ++c) {
      const int64_t i = i0 + 4 * q + c, j = j0 + r;
      const bool in = i < a.nx && j < a.ny;
      t[c] = in ? a.T[j * a.ld + i] : inf;
      f[c] = in ? a.F[j * a.ld + i] : inf;
      live[c] = in && t[c] < inf && !(i == a.gi && j == a.gj);
      img[(r + 1) * RP + 4 * q + c + 1] = t[c];
    }
    if (r == 0)
      for (int c = 0; c < 4; ++c) img[4 * q + c + 1] = at(i0 + 4 * q + c, j0 - 1);
    if (r == RT - 1)
      for (int c = 0; c < 4; ++c) img[(RT + 1) * RP + 4 * q + c + 1] = at(i0 + 4 * q + c, j0 + RT);
    if (q == 0) img[(r + 1) * RP] = at(i0 - 1, j0 + r);
    if (q == 3) img[(r + 1) * RP + RT + 1] = at(i0 + RT, j0 + r);
    __builtin_amdgcn_wave_barrier();
    bool gone[4] = {false, false, false, false};
    for (int it = 0; it < RT * RT; ++it) {  // a cascade is at most one cell per sweep
      bool now[4];
      for (int c = 0; c < 4; ++c) {
        const int s = (r + 1) * RP + 4 * q + c + 1;
        const double u = ref_update(fmin(img[s - 1], img[s + 1]), fmin(img[s - RP], img[s + RP]), f[c]);
        // a cell that became an obstacle (F = +inf) loses its value outright
        now[c] = live[c] && !gone[c] && (!(f[c] < inf) || u > t[c] * (1.0 + a.tol));
      }
      __builtin_amdgcn_wave_barrier();
      bool any = false;
      for (int c = 0; c < 4; ++c)
        if (now[c]) {
          gone[c] = true;
          any = true;
          img[(r + 1) * RP + 4 * q + c + 1] = inf;
        }
      __builtin_amdgcn_wave_barrier();
      if (!__any(any)) break;
    }
    bool edge[4] = {false, false, false, false};  // S, W, E, N
    for (int c = 0; c < 4; ++c)
      if (gone[c]) {
        a.T[(j0 + r) * a.ld + i0 + 4 * q + c] = inf;
        ++cells;
        edge[0] |= r == 0;
        edge[3] |= r == RT - 1;
        edge[1] |= q == 0 && c == 0;
        edge[2] |= q == 3 && c == 3;
      }
    const int tx = (int)(tile % a.ntx), ty = (int)(tile / a.ntx);
    const int nbx[4] = {tx, tx - 1, tx + 1, tx}, nby[4] = {ty - 1, ty, ty, ty + 1};
    for (int s = 0; s < 4; ++s) {
      if (!__any(edge[s]) || lane != 0) continue;
      if (nbx[s] < 0 || nby[s] < 0 || nbx[s] >= (int)a.ntx || nby[s] >= (int)a.nty) continue;
      const uint32_t nt = (uint32_t)nby[s] * a.ntx + (uint32_t)nbx[s];
      if (atomicMax(&a.tile_epoch[nt], a.epoch) < a.epoch) {
        const uint32_t pos = atomicAdd(&a.count_out[shard], 1u);
        a.list_out[(uint64_t)shard * a.shard_cap + pos] = nt;
      }
    }
    ++visits;
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0 && visits) atomicAdd(&a.stats[0], visits);
  for (int o = 32; o > 0; o >>= 1) cells += __shfl_xor(cells, o);
  if (lane == 0 && cells) atomicAdd(&a.stats[1], cells);
}

// List 0 after the raise (see launch_cone_seed)
__global__ void k_cone_seed(UpdateArgs a, unsigned long long* theta_bits) {
  const uint64_t n = (uint64_t)a.nx * a.ny;
  const uint32_t shard = blockIdx.x % kShards;
  const double inf = __builtin_inf();
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = (uint32_t)(c / a.nx), i = (uint32_t)(c % a.nx);
    const int64_t k = (int64_t)j * a.ld + i;
    if (!(a.T[k] == inf) || !(a.F[k] < inf) || (i == a.gi && j == a.gj)) continue;
    double m = inf;
    if (j > 0) m = fmin(m, a.T[k - a.ld]);
    if (i > 0) m = fmin(m, a.T[k - 1]);
    if (i + 1 < a.nx) m = fmin(m, a.T[k + 1]);
    if (j + 1 < a.ny) m = fmin(m, a.T[k + a.ld]);
    if (!(m < inf)) continue;
    const uint32_t tile = (j / a.th) * a.ntx + (i / a.tw);
    const unsigned long long mb = dbits(m);
    atomicMin(theta_bits, mb);
    if (a.keys) atomicMin(&a.keys[tile], mb);
    if (atomicMax(&a.tile_epoch[tile], a.epoch) < a.epoch) {
      const uint32_t pos = atomicAdd(&a.counts[shard], 1u);
      a.list[(uint64_t)shard * a.shard_cap + pos] = tile;
      if (a.hist) atomicAdd(&a.hist[shard * kBins], 1u);
    }
  }
}

// Priority-kernel list-0 state: keys of the seeded tiles are theta.
__global__ void k_theta_state(const unsigned long long* theta_bits, unsigned long long* minkey0,
                              double* base0) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *minkey0 = *theta_bits;
    const double th = __longlong_as_double((long long)*theta_bits);
    *base0 = th < __builtin_inf() ? th : 0.0;
  }
}

// ---- early exit of computeTotalCostMap (reference :364-408) ----

__global__ void k_probe(const double* T, int64_t ld, ProbeCells cells,
                        const unsigned long long* minkey, unsigned long long* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned long long m = 0;
  for (int k = 0; k < cells.n; ++k) {
    const unsigned long long b = dbits(T[cells.ij[k][1] * ld + cells.ij[k][0]]);
    m = b > m ? b : m;  // T >= 0: bit order = value order
  }
  out[0] = m;
  out[1] = minkey ? *minkey : kInfBits;
}

// Cells are CLOSED iff T <= t_closed (their values are final).  A cell that is not
// CLOSED keeps its value only if it is in the band (a finite-speed 4-neighbour of a
// CLOSED cell: the reference propagated into it, :462-465); every other cell was
// never reached and gets +inf.  Writes only touch non-CLOSED cells and the test
// reads only CLOSED-ness, so the races between threads do not change any answer.
__global__ void k_early_mask(const double* F, double* T, int64_t ld, uint32_t nx, uint32_t ny,
                             double tc, uint64_t* band, unsigned long long* n_band, uint64_t cap) {
  const uint64_t n = (uint64_t)nx * ny;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = (uint32_t)(c / nx), i = (uint32_t)(c % nx);
    const int64_t k = (int64_t)j * ld + i;
    const double t = T[k];
    if (t <= tc) continue;  // CLOSED
    bool b = false;
    if (F[k] < __builtin_inf()) {
      b = (j > 0 && T[k - ld] <= tc) || (i > 0 && T[k - 1] <= tc) ||
          (i + 1 < nx && T[k + 1] <= tc) || (j + 1 < ny && T[k + ld] <= tc);
    }
    if (b) {
      const unsigned long long pos = atomicAdd(n_band, 1ull);
      if (pos < cap) band[pos] = c;
    } else if (t < __builtin_inf()) {
      T[k] = __builtin_inf();
    }
  }
}

// The early exit's region (dymu_region_stats): over every cell, the bounding box of
// those with T <= thr (out[0..3]: min i, min j, max i, max j; nothing: min > max) and
// the number with lo <= T <= hi (out[4]) -- the engine's near ties with the exit value.
// Wave reductions, then one atomic per wave and word.
__global__ void k_region_box(const double* T, int64_t ld, uint32_t nx, uint32_t ny, double thr,
                             double lo, double hi, unsigned long long* out) {
  const uint64_t n = (uint64_t)nx * ny;
  unsigned long long mi = ~0ull, mj = ~0ull, xi = 0, xj = 0, cnt = 0;
  bool any = false;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = c / nx, i = c % nx;
    const double t = T[(int64_t)j * ld + (int64_t)i];
    if (t <= thr) {
      any = true;
      mi = i < mi ? i : mi;
      mj = j < mj ? j : mj;
      xi = i > xi ? i : xi;
      xj = j > xj ? j : xj;
    }
    cnt += (t >= lo && t <= hi) ? 1u : 0u;
  }
  if (!any) xi = xj = 0;
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(mi, o), b = __shfl_xor(mj, o);
    const unsigned long long e = __shfl_xor(xi, o), f = __shfl_xor(xj, o);
    mi = a < mi ? a : mi;
    mj = b < mj ? b : mj;
    xi = e > xi ? e : xi;
    xj = f > xj ? f : xj;
    cnt += __shfl_xor(cnt, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (mi != ~0ull) {
      atomicMin(&out[0], mi);
      atomicMin(&out[1], mj);
      atomicMax(&out[2], xi);
      atomicMax(&out[3], xj);
    }
    if (cnt) atomicAdd(&out[4], cnt);
  }
}

// The constant-speed radius (dymu_region_stats): the least squared distance from the
// goal (gi, gj) to a cell whose speed differs from f0 (an obstacle included) -> *out
__global__ void k_const_radius(const double* F, int64_t ld, uint32_t nx, uint32_t ny, uint32_t gi,
                               uint32_t gj, double f0, unsigned long long* out) {
  const uint64_t n = (uint64_t)nx * ny;
  unsigned long long m = ~0ull;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = c / nx, i = c % nx;
    if (F[(int64_t)j * ld + (int64_t)i] != f0) {
      const int64_t di = (int64_t)i - gi, dj = (int64_t)j - gj;
      const unsigned long long d2 = (unsigned long long)(di * di + dj * dj);
      m = d2 < m ? d2 : m;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a = __shfl_xor(m, o);
    m = a < m ? a : m;
  }
  if ((threadIdx.x & 63) == 0 && m != ~0ull) atomicMin(out, m);
}

// *p = v (a per-call device scalar initialised in stream order, without a host copy)
__global__ void k_store_u64(unsigned long long* p, unsigned long long v) {
  if (threadIdx.x == 0) *p = v;
}

__global__ void k_scatter(double* T, int64_t ld, uint32_t nx, const uint64_t* idx,
                          const double* vals, uint64_t n) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q = idx[c];
    T[(int64_t)(q / nx) * ld + (int64_t)(q % nx)] = vals[c];
  }
}

}  // namespace

hipError_t launch_probe(const double* T, int64_t ld, const ProbeCells& cells,
                        const unsigned long long* minkey, unsigned long long* out,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, st, T, ld, cells, minkey, out);
  return hipGetLastError();
}

hipError_t launch_early_mask(const double* F, double* T, int64_t ld, uint32_t nx, uint32_t ny,
                             double t_closed, uint64_t* band, unsigned long long* n_band,
                             uint64_t cap, hipStream_t st) {
  uint64_t b = ((uint64_t)nx * ny + 255) / 256;
  if (b > 16384) b = 16384;
  if (b == 0) return hipSuccess;
  hipLaunchKernelGGL(k_early_mask, dim3((unsigned)b), dim3(256), 0, st, F, T, ld, nx, ny,
                     t_closed, band, n_band, cap);
  return hipGetLastError();
}

hipError_t launch_scatter(double* T, int64_t ld, uint32_t nx, const uint64_t* idx,
                          const double* vals, uint64_t n, hipStream_t st) {
  uint64_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)b), dim3(256), 0, st, T, ld, nx, idx, vals, n);
  return hipGetLastError();
}

hipError_t launch_region_box(const double* T, int64_t ld, uint32_t nx, uint32_t ny, double thr,
                             double lo, double hi, unsigned long long* out, hipStream_t st) {
  uint64_t b = ((uint64_t)nx * ny + 255) / 256;
  if (b > 4096) b = 4096;
  if (b == 0) b = 1;
  hipLaunchKernelGGL(k_region_box, dim3((unsigned)b), dim3(256), 0, st, T, ld, nx, ny, thr, lo,
                     hi, out);
  return hipGetLastError();
}

hipError_t launch_const_radius(const double* F, int64_t ld, uint32_t nx, uint32_t ny, uint32_t gi,
                               uint32_t gj, double f0, unsigned long long* out, hipStream_t st) {
  uint64_t b = ((uint64_t)nx * ny + 255) / 256;
  if (b > 4096) b = 4096;
  if (b == 0) b = 1;
  hipLaunchKernelGGL(k_const_radius, dim3((unsigned)b), dim3(256), 0, st, F, ld, nx, ny, gi, gj, f0,
                     out);
  return hipGetLastError();
}

hipError_t launch_store_u64(unsigned long long* p, unsigned long long v, hipStream_t st) {
  hipLaunchKernelGGL(k_store_u64, dim3(1), dim3(64), 0, st, p, v);
  return hipGetLastError();
}

hipError_t launch_window_min(const double* T, int64_t ld, uint32_t i0, uint32_t j0, uint32_t i1,
                             uint32_t j1, unsigned long long* out, hipStream_t st) {
  const uint64_t n = (uint64_t)(i1 - i0) * (j1 - j0);
  uint64_t b = (n + 255) / 256;
  if (b > 1024) b = 1024;
  if (b == 0) b = 1;
  hipLaunchKernelGGL(k_window_min, dim3((unsigned)b), dim3(256), 0, st, T, ld, i0, j0, i1, j1, out);
  return hipGetLastError();
}

hipError_t launch_count_equal(const double* T, int64_t ld, uint32_t nx, uint32_t ny, double value,
                              unsigned long long* out, uint64_t* idx, uint64_t cap,
                              hipStream_t st) {
  uint64_t b = ((uint64_t)nx * ny + 255) / 256;
  if (b > 4096) b = 4096;
  if (b == 0) b = 1;
  hipLaunchKernelGGL(k_count_equal, dim3((unsigned)b), dim3(256), 0, st, T, ld, nx, ny,
                     (unsigned long long)__builtin_bit_cast(unsigned long long, value), out, idx,
                     cap);
  return hipGetLastError();
}

hipError_t launch_reset_seed(const UpdateArgs& a, hipStream_t st) {
  uint64_t b = ((uint64_t)a.nx * a.ny + 255) / 256;
  if (b > 8192) b = 8192;
  if (b == 0) b = 1;
  hipLaunchKernelGGL(k_reset_seed, dim3((unsigned)b), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_seed_window(const UpdateArgs& a, uint32_t i0, uint32_t j0, uint32_t i1,
                              uint32_t j1, hipStream_t st) {
  const uint32_t tx0 = i0 / a.tw, ty0 = j0 / a.th;
  const uint32_t tx1 = (i1 + a.tw - 1) / a.tw, ty1 = (j1 + a.th - 1) / a.th;
  const uint64_t n = (uint64_t)(tx1 - tx0) * (ty1 - ty0);
  uint64_t b = (n + 255) / 256;
  if (b > 1024) b = 1024;
  if (b == 0) return hipSuccess;
  hipLaunchKernelGGL(k_seed_window, dim3((unsigned)b), dim3(256), 0, st, a, tx0, ty0, tx1, ty1);
  return hipGetLastError();
}

hipError_t launch_raise(const RaiseArgs& a, int blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_raise, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_cone_seed(const UpdateArgs& a, unsigned long long* theta_bits, hipStream_t st) {
  uint64_t b = ((uint64_t)a.nx * a.ny + 255) / 256;
  if (b > 8192) b = 8192;
  if (b == 0) b = 1;
  hipLaunchKernelGGL(k_cone_seed, dim3((unsigned)b), dim3(256), 0, st, a, theta_bits);
  return hipGetLastError();
}

hipError_t launch_theta_state(const unsigned long long* theta_bits, unsigned long long* minkey0,
                              double* base0, hipStream_t st) {
  hipLaunchKernelGGL(k_theta_state, dim3(1), dim3(64), 0, st, theta_bits, minkey0, base0);
  return hipGetLastError();
}

}  // namespace dymu
