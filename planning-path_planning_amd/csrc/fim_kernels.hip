// fim_kernels.hip -- MI355X (gfx950) block Fast-Iterative-Method kernels for the
// DyMu global total-cost propagation (reference: src/DyMu_GlobalPathPlanning.cpp).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction:
// every update rounds exactly like the reference's SSE2 build).
//
// Algorithm: the grid is cut into TB_W x TB_H tiles.  A pass
// kernel walks the device-built list of active tiles; each workgroup loads one
// tile of T (plus a 1-cell halo) into LDS and the tile's F into registers,
// relaxes the reference's Eikonal update (:500-546) in place until the tile is
// locally converged, writes back the cells that decreased and enqueues the
// neighbour tiles whose shared edge changed.  Values only decrease and every
// update is the reference's arithmetic -- exactly (kernels 3/4, kernel 5 with
// exact_sqrt) or within 36 ulp on the two-sided candidate (kernel 5's default
// sweep sqrt) -- so the converged map is the fixed point the
// reference FMM reaches, exactly resp. within the stated tolerance (measured
// <= 6e-15 relative).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fim_kernels.h"

namespace dymu {

__device__ __forceinline__ double dinf() { return __builtin_inf(); }

// fmin for operands that are never NaN (T values are >= 0 or +inf): a plain
// compare-select, so the compiler does not canonicalise both inputs first.
__device__ __forceinline__ double minnn(double a, double b) { return b < a ? b : a; }

// Reference :504-535.  Tx = fmin(W,E), Ty = fmin(N,S); off-grid neighbours
// are +inf (a NULL nb4 makes the reference use the other one alone, :508-523).
// 2*pow(C,2.0) - pow(Tx-Ty,2.0) with pow(x,2.0) == x*x; no contraction.
__device__ __forceinline__ double eikonal(double tx, double ty, double c) {
  const double d = tx - ty;
  if ((fabs(d) < c) && (tx < dinf()) && (ty < dinf())) {
    const double cc = c * c;
    const double r = 2.0 * cc - d * d;
    return (tx + ty + sqrt(r)) / 2;
  }
  return minnn(tx, ty) + c;
}

// ---------------------------------------------------------------------------
// T initialisation: +inf everywhere, 0 at the goal (resetTotalCostMap +
// resetGlobalNarrowBand, :473-496).  Ghost rows (sharded mode) are included
// when rows < 0 / >= ny are passed in.
// ---------------------------------------------------------------------------
// rows on blockIdx.y, columns on blockIdx.x (grid-strided; no index division);
// 16-byte stores (two cells per lane) on rows that start 16-byte aligned
__global__ void k_fill_inf(double* T, uint64_t ld, uint32_t nx, int64_t row_lo, int64_t row_hi) {
  const double inf = dinf();
  for (int64_t r = row_lo + blockIdx.y; r < row_hi; r += gridDim.y) {
    double* row = T + r * (int64_t)ld;
    if (((uintptr_t)row & 15) == 0) {  // wave-uniform
      double2* row2 = reinterpret_cast<double2*>(row);
      for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nx / 2;
           c += gridDim.x * blockDim.x)
        row2[c] = make_double2(inf, inf);
      if ((nx & 1) && blockIdx.x == 0 && threadIdx.x == 0) row[nx - 1] = inf;
    } else {
      for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < nx;
           c += gridDim.x * blockDim.x)
        row[c] = inf;
    }
  }
}

__global__ void k_seed(double* T, uint64_t ld, int64_t gi, int64_t gj, uint32_t* list,
                       uint32_t* count, uint32_t* tile_epoch, uint32_t epoch, uint32_t tile,
                       int set_goal) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (set_goal) T[gj * (int64_t)ld + gi] = 0.0;
    if (atomicMax(&tile_epoch[tile], epoch) < epoch) {
      const uint32_t pos = atomicAdd(count, 1u);
      list[pos] = tile;
    }
  }
}

// ---------------------------------------------------------------------------
// Active-tile lists: kShards shards, one wave-or-half-wave per tile, enqueues
// aggregated per workgroup in LDS and published with one atomic per workgroup
// per pass into one shard (same-address atomics serialise at ~11 ns each).
// ---------------------------------------------------------------------------
constexpr int WT = kWaveTile;
constexpr int QCAP = 1024;  // LDS enqueue buffer per workgroup

// shard of a logical list index: the counters are prefix-summed in LDS.
__device__ __forceinline__ uint32_t list_at(const uint32_t* list, uint32_t cap,
                                            const uint32_t* pref, uint32_t li) {
  int k = 0;
#pragma unroll
  for (int q = 1; q < kShards; ++q) k += (li >= pref[q]) ? 1 : 0;
  return list[(uint64_t)k * cap + (li - pref[k])];
}

// list_at for a wave-uniform li: lane q reads pref[q], one ballot counts the
// shards that start at or before li (one LDS read and a few VALU ops instead of
// fifteen reads and a 64-bit add chain)
__device__ __forceinline__ uint32_t list_at_wave(const uint32_t* list, uint32_t cap,
                                                 const uint32_t* pref, uint32_t li, int lane) {
  const uint32_t p = lane < kShards ? pref[lane] : 0u;
  const int k = __popcll(__ballot(lane >= 1 && lane < kShards && li >= p));
  const uint32_t base = __builtin_amdgcn_readlane(p, k);
  return list[(uint64_t)k * cap + (li - base)];
}

// ---------------------------------------------------------------------------
// v3 pass kernel: red-black Gauss-Seidel, two 8x8 tiles per wave.
// Half-wave h (lanes 32h..32h+31) owns one tile; lane (r = l>>2, q = l&3) owns
// the two horizontally adjacent cells (r, 2q) and (r, 2q+1), one of each
// checkerboard colour: red column 2q + (r&1), black column 2q + 1 - (r&1).
// A sweep updates all red cells from the current image, then all black cells
// from the freshly written reds (Gauss-Seidel on the two colours), so a sweep
// moves information two cells for the cost of one Jacobi sweep of 64 lanes.
// Everything else (halo ring, ballot convergence, edge flags, enqueue
// aggregation) is as in v2.
// ---------------------------------------------------------------------------
// Image row pitch 12 doubles: the 32 red (or black) cells of a half-wave, and
// every +-1 / +-pitch shift of them, fall on 32 distinct ds_read_b64 bank pairs
// and 16 distinct ds_write_b64 banks per 16-lane group (pitch 10 was 2-way).
constexpr int IP = 12;
// 16x16 image (kernel 5): row r of a wave's tile image (r = -1 .. 16, the halo
// rows included) starts at slot img16_row(r), and cell (r, c), c = -1 .. 16, sits
// at img16_row(r) + c.  The rows are skewed -- consecutive bases 32, 34, 32, 46
// slots apart -- so that with lane (r = lane>>2, q = lane&3) owning columns
// 4q..4q+3 of row r, every ds_read_b64 of a half-sweep (W, E, N, S of the
// lane's two same-colour cells) lands its 32 lanes on 32 distinct bank pairs and
// every ds_write_b64 its 16-lane groups on distinct banks.  With a constant
// pitch the colour offset (r & 1) leaves only two bank classes per row
// parity: the former pitch-20 image had every read and write 2-way
// (PMC SQ_LDS_BANK_CONFLICT 3.7 G cycles per 16384^2 solve, more than the LDS
// instructions' own 1.9 G).
__device__ __forceinline__ int img16_row(int r) {
  return 47 + 144 * (r >> 2) + 32 * (r & 3) + 2 * ((r >> 1) & 1);
}
constexpr int IMG16 = 640;  // img16_row(16) + 17

// v_min_f64 on operands that are never NaN (T >= 0 or +inf): one instruction,
// no canonicalisation (the compiler cannot prove no-NaN for fmin).
__device__ __forceinline__ double vmin64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// min(|a|, b) in one v_min_f64 (abs source modifier); a NaN operand yields the other
__device__ __forceinline__ double vmin64_abs(double a, double b) {
  double r;
  asm("v_min_f64 %0, |%1|, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Correctly rounded sqrt for x in [2^-767, 2^1023]: LLVM's f64 sqrt expansion
// (rsq + Goldschmidt/Newton refinement) minus its range scaling and special-
// value selects, which are identities on that range.  Bit-identical to sqrt()
// there; x = 2C^2 - d^2 >= C^2 >= 2^-767 whenever C >= 2^-383 (kFastMinF).
__device__ __forceinline__ double sqrt_cr_fast(double x) {
  const double y0 = __builtin_amdgcn_rsq(x);
  double s = x * y0;
  double h = y0 * 0.5;
  const double e = __builtin_fma(-h, s, 0.5);
  s = __builtin_fma(s, e, s);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-s, s, x);
  s = __builtin_fma(d, h, s);
  d = __builtin_fma(-s, s, x);
  s = __builtin_fma(d, h, s);
  return s;
}

// sqrt_cr_fast on two independent operands, step-interleaved so the two
// dependent chains overlap in a single wave (same operations: bit-identical)
// APPROX: stop after the Goldschmidt step (5 instead of 10 VALU instructions):
// <= 36 ulp from the correctly rounded sqrt (tools/sqrt_probe.hip: 805 M operands
// 2C^2 - d^2, |d| < C, C in 2^-380..2^380), the rsq estimate alone is ~2^-23
template <bool APPROX = false>
__device__ __forceinline__ void sqrt_cr_fast2(double x0, double x1, double& r0, double& r1) {
  const double y0 = __builtin_amdgcn_rsq(x0), y1 = __builtin_amdgcn_rsq(x1);
  double s0 = x0 * y0, s1 = x1 * y1;
  double h0 = y0 * 0.5, h1 = y1 * 0.5;
  const double e0 = __builtin_fma(-h0, s0, 0.5), e1 = __builtin_fma(-h1, s1, 0.5);
  s0 = __builtin_fma(s0, e0, s0);
  s1 = __builtin_fma(s1, e1, s1);
  if constexpr (APPROX) {
    r0 = s0;
    r1 = s1;
    return;
  }
  h0 = __builtin_fma(h0, e0, h0);
  h1 = __builtin_fma(h1, e1, h1);
  double d0 = __builtin_fma(-s0, s0, x0), d1 = __builtin_fma(-s1, s1, x1);
  s0 = __builtin_fma(d0, h0, s0);
  s1 = __builtin_fma(d1, h1, s1);
  d0 = __builtin_fma(-s0, s0, x0);
  d1 = __builtin_fma(-s1, s1, x1);
  r0 = __builtin_fma(d0, h0, s0);
  r1 = __builtin_fma(d1, h1, s1);
}
constexpr double kFastMinF = 0x1p-383;

// Kernel 5's default two-sided candidate (Tx + Ty + sqrt(2C^2 - d^2)) / 2 with the
// Goldschmidt step of sqrt_cr_fast2<true> folded into the combine: with y0 = rsq(r),
// s = r*y0, sqrt(r) ~ s*(1.5 - 0.5*y0*s), so u = (Tx+Ty)/2 + s*(0.75 - (y0/4)*s);
// r = fma(-d, d, 2C^2) (one rounding; r >= C^2 on this branch, no cancellation) and
// (Tx+Ty)/2 = fma(d, 0.5, Ty) from the d = Tx - Ty the caller has.
// 7 VALU after d instead of 10 (the exact sqrt: 15).
__device__ __forceinline__ double two_sided_approx(double ty, double d, double c2x2) {
  const double r = __builtin_fma(-d, d, c2x2);
  const double y0 = __builtin_amdgcn_rsq(r);
  const double s = r * y0;
  const double t = __builtin_fma(-(y0 * 0.25), s, 0.75);
  return __builtin_fma(s, t, __builtin_fma(d, 0.5, ty));
}

// The monotone combine (v32, kernel 5's sweeps).  The reference rounds the
// two-sided candidate twice at the scale of T -- RN(RN(Tx + Ty) + sqrt) / 2 --
// so a larger input can round to a smaller candidate by an ulp of T.  The FIM
// evaluates a cell many times while its inputs converge from above and keeps
// the minimum (:537), i.e. the luckiest of those roundings: a downward bias of
// ~0.002 ulp per cell that adds up along a path (1.21e-12 on the 16384^2
// serpentine maze's ~4 M-cell corridors).  Written as
//   T' = min(Tx,Ty) + h,  h = (|Tx - Ty| + sqrt(2C^2 - d^2)) / 2  (two-sided)
//                         h = C                                  (one-sided)
// the candidate is rounded ONCE at the scale of T, the correction h carries
// only errors at the scale of C, and the candidate is monotone in (Tx, Ty)
// up to those C-scale errors: the min over history is then the last
// evaluation's value, and the map is the fixed point of the update rather
// than its luckiest rounding (tools/mono_sim.c: the bias no longer grows with
// the path length).
// The default sweep candidate (v33) also folds the branch into h's argument:
// e = min(|Tx - Ty|, C), T' = m + h(e) -- the two-sided h below C, h(C) = (C +
// sqrt(C^2)) / 2 ~ C at and above it (the one-sided value within the sweep sqrt's
// 36 ulp of C instead of bit for bit; continuous and monotone across |d| = C) -- one
// v_min_f64 instead of a compare and two selects.  The approximate sqrt: y0 =
// rsq(r), s = r*y0, sqrt(r) ~ s*(1.5 - (y0/2)*s) (one Goldschmidt step); at twice
// the scale, t2 = 1.5 - (y0/2) s, h2 = e + s t2 = 2h, T' = fma(h2, 0.5, m) = RN(m + h)
// (scalings by 2 are exact) -- no e/2 multiply.  12 VALU per cell after the
// neighbours' minima, 14 with them (v32: 16.5).  e >= 0.
__device__ __forceinline__ double cand_approx(double e, double c2x2, double m) {
  const double r = __builtin_fma(-e, e, c2x2);
  const double y0 = __builtin_amdgcn_rsq(r);
  const double s = r * y0;
  const double t2 = __builtin_fma(-(y0 * 0.5), s, 1.5);
  return __builtin_fma(__builtin_fma(s, t2, e), 0.5, m);
}

// cand_approx on two independent cells, statement by statement interleaved (same
// operations, bit-identical)
__device__ __forceinline__ void cand_approx2(double e0, double c0, double m0, double e1, double c1,
                                             double m1, double& u0, double& u1) {
  const double r0 = __builtin_fma(-e0, e0, c0);
  const double r1 = __builtin_fma(-e1, e1, c1);
  const double y0 = __builtin_amdgcn_rsq(r0);
  const double y1 = __builtin_amdgcn_rsq(r1);
  const double s0 = r0 * y0;
  const double s1 = r1 * y1;
  const double t0 = __builtin_fma(-(y0 * 0.5), s0, 1.5);
  const double t1 = __builtin_fma(-(y1 * 0.5), s1, 1.5);
  const double h0 = __builtin_fma(s0, t0, e0);
  const double h1 = __builtin_fma(s1, t1, e1);
  u0 = __builtin_fma(h0, 0.5, m0);
  u1 = __builtin_fma(h1, 0.5, m1);
}

// One cell of the reference update (:504-537) against the image.  Preconditions
// (guaranteed by the skip test): f finite and min(Tx,Ty) finite, so the
// reference's "Tx < inf && Ty < inf" is implied by |Tx - Ty| < C.
// c2x2 = 2*(C*C) is precomputed: the same two roundings as 2*pow(C,2.0).
template <bool FAST, int PITCH = IP>
__device__ __forceinline__ bool rb_update(double* img, int slot, double f, double k1, double c2x2,
                                          double& t) {
  const double south = img[slot - PITCH];
  const double west = img[slot - 1];
  const double east = img[slot + 1];
  const double north = img[slot + PITCH];
  const double tx_ = vmin64(west, east), ty_ = vmin64(north, south);
  const double m = vmin64(tx_, ty_);
  if (m + k1 < t) {  // exact skip bound U >= min + C/sqrt(2); k1 = 0.7071*C
    const double dd = tx_ - ty_;
    double u;
    if (fabs(dd) < f) {
      const double r = c2x2 - dd * dd;
      const double sq = FAST ? sqrt_cr_fast(r) : sqrt(r);
      u = ((tx_ + ty_) + sq) * 0.5;  // (Tx + Ty + sqrt(...)) / 2, /2 exact
    } else {
      u = m + f;  // fmin(Tx,Ty) + C
    }
    if (u < t) {  // :537
      t = u;
      return true;
    }
  }
  return false;
}

// The update of rb_update without the skip test, for the arithmetic self-test
// (dymu_eikonal_batch): candidate T' from (Tx, Ty, C) as at :531-535.
// MODE 0: sqrt(), 1: sqrt_cr_fast (bit-identical), 2: kernel 5's default sweep
// candidate (monotone combine, approximate sqrt), 3: kernel 5's exact_sqrt sweep
// candidate (monotone combine, correctly rounded sqrt), 4: v31's sweep candidate
// (two_sided_approx, kept for the A/B of the combine)
template <int MODE>
__device__ __forceinline__ double update_value(double tx_, double ty_, double f) {
  const double m = minnn(tx_, ty_);
  if (!(f < dinf()) || !(m < dinf())) return m + f;  // outside the kernel's fast path
  const double dd = tx_ - ty_;
  if (MODE == 2)  // rb_update2's default candidate, both branches
    return cand_approx(fabs(dd) < f ? fabs(dd) : f, 2.0 * (f * f), m);
  if (fabs(dd) < f) {
    const double r = 2.0 * (f * f) - dd * dd;
    if (MODE == 3) return m + (fabs(dd) + sqrt_cr_fast(__builtin_fma(-dd, dd, 2.0 * (f * f)))) * 0.5;
    if (MODE == 4) return two_sided_approx(ty_, dd, 2.0 * (f * f));
    const double sq = MODE == 1 ? sqrt_cr_fast(r) : sqrt(r);
    return ((tx_ + ty_) + sq) * 0.5;
  }
  return m + f;
}

template <int MODE>
__global__ void k_eikonal_batch(const double* tx, const double* ty, const double* c, double* out,
                                uint64_t n) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (uint64_t)gridDim.x * blockDim.x)
    out[k] = update_value<MODE>(tx[k], ty[k], c[k]);
}

template <bool FAST>
__device__ __forceinline__ int rb_sweeps(double* img, int sr, int sb, double fr, double fb,
                                         double& tr, double& tb, int max_inner, bool& capped) {
  const double k1r = 0.7071 * fr, k1b = 0.7071 * fb;
  const double c2r = 2.0 * (fr * fr), c2b = 2.0 * (fb * fb);
  int sweeps = 0;
  capped = true;
  while (sweeps < max_inner) {
    __builtin_amdgcn_wave_barrier();
    const bool ir = rb_update<FAST>(img, sr, fr, k1r, c2r, tr);  // red from black
    img[sr] = tr;
    __builtin_amdgcn_wave_barrier();
    const bool ib = rb_update<FAST>(img, sb, fb, k1b, c2b, tb);  // black from fresh red
    img[sb] = tb;
    ++sweeps;
    if (!__any(ir || ib)) {
      capped = false;
      break;
    }
  }
  __builtin_amdgcn_wave_barrier();
  return sweeps;
}

// the convergence mailbox (PassArgs::report): a system-scope vector store into
// host-coherent memory, visible to a polling host thread while the stream runs
__device__ __forceinline__ void report_pending(const PassArgs& a, uint32_t n_active) {
  if (a.report) {
    uint32_t v = a.report_src ? (uint32_t)*a.report_src : n_active;
    if (a.probe.n > 0 && a.minkey_in) {  // T, keys >= 0: bit order = value order
      unsigned long long tmax = 0;
      for (int k = 0; k < a.probe.n; ++k) {
        const unsigned long long b =
            __double_as_longlong(a.T[a.probe.ij[k][1] * a.ld + a.probe.ij[k][0]]);
        tmax = b > tmax ? b : tmax;
      }
      if (*a.minkey_in > tmax) v |= 0x80000000u;
    }
    if (a.report_ext) {  // the status words first, then the word the host polls
#pragma unroll
      for (int k = 0; k < 4; ++k)
        __hip_atomic_store(a.report + 1 + k, a.report_ext[k], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.report, ((unsigned long long)a.report_seq << 32) | v, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __hip_atomic_store(a.report, ((unsigned long long)a.report_seq << 32) | v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- peer rounds (dymu_dom_round_peer; DESIGN.md s5 "Peer transport") ----
// The status pass of a round (block 0, thread 0): R per side = the smallest tag the
// round's merging workgroups read (kept when no workgroup merged that side), then
// the status (S0, S1, R0, R1) beside P (pend) for the next check's post.
__device__ __forceinline__ void peer_status(PeerCtl* pc) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const unsigned long long rm = pc->rmin[s];
    if (rm != ~0ull) pc->merged[s] = rm;
    pc->rmin[s] = ~0ull;
  }
  pc->ext[0] = pc->sent[0];
  pc->ext[1] = pc->sent[1];
  pc->ext[2] = pc->merged[0];
  pc->ext[3] = pc->merged[1];
}

// One wave per workgroup pushes the workgroup's column share [m0, m1) of the owned
// first / last row into the neighbour's receive row: only values below the last
// pushed ones (values only decrease), stored at system scope over xGMI (or into
// another process's buffer on the same GPU).  The workgroup then counts itself done;
// the last one of the pass, if any column of the side decreased, bumps S and writes
// it as the neighbour's tag after a system-scope fence -- every workgroup's values
// are visible before the tag that covers them.  No wait on the neighbour anywhere.
__device__ __forceinline__ void peer_push(const PassArgs& a, int64_t m0, int64_t m1, int lane) {
  PeerCtl* pc = a.peer;
  for (int s = 0; s < 2; ++s) {
    double* dst = a.push_dst[s];
    if (!dst) continue;
    const double* row = a.T + (s == 0 ? 0 : (a.ny - 1) * a.ld);
    double* last = a.push_last[s];
    bool ch = false;
    for (int64_t k0 = m0; k0 < m1; k0 += 64) {
      const int64_t k = k0 + lane;
      if (k < m1) {
        const double v = row[k];
        if (v < last[k]) {
          last[k] = v;
          __hip_atomic_store(dst + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          ch = true;
        }
      }
    }
    const bool any = __any(ch);
    __threadfence_system();  // this wave's pushed values before its done count
    if (lane == 0) {
      if (any) __hip_atomic_fetch_or(&pc->changed[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t prev =
          __hip_atomic_fetch_add(&pc->done[s], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == gridDim.x - 1u) {  // the pass's last workgroup for this side
        __hip_atomic_store(&pc->done[s], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_exchange(&pc->changed[s], 0u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)) {
          const unsigned long long S = pc->sent[s] + 1ull;
          pc->sent[s] = S;
          __threadfence_system();
          __hip_atomic_store(a.push_tag[s], S, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_fim_pass_rb(PassArgs a) {
  __shared__ uint32_t s_q[QCAP];
  __shared__ uint32_t s_pref[kShards + 1];
  __shared__ uint32_t s_nq, s_base;
  __shared__ unsigned long long s_visits, s_sweeps;
  __shared__ double s_img[8][(WT + 2) * IP];  // one 10-row image (pitch IP) per half-wave

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int half = lane >> 5;
  const int hl = lane & 31;
  const int r = hl >> 2, q = hl & 3;
  const int cr = 2 * q + (r & 1), cb = 2 * q + 1 - (r & 1);  // red / black column
  const uint32_t shard = blockIdx.x % kShards;

  if (tid == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < kShards; ++k) {
      s_pref[k] = acc;
      acc += a.count_in[k];
    }
    s_pref[kShards] = acc;
    s_nq = 0;
    s_visits = 0;
    s_sweeps = 0;
  }
  __syncthreads();
  const uint32_t n_active = s_pref[kShards];
  if (blockIdx.x == 0) {
    if (tid < kShards) a.count_clear[tid] = 0u;
    if (tid == 0 && n_active > 0) {
      atomicAdd(&a.stats[kStatPasses], 1ull);
      atomicMax(&a.stats[kStatMaxActive], (unsigned long long)n_active);
    }
    if (tid == 0) report_pending(a, n_active);
  }

  unsigned long long my_visits = 0, my_sweeps = 0;
  double* img = s_img[wv * 2 + half];
  const int sr = (r + 1) * IP + (cr + 1);  // red slot
  const int sb = (r + 1) * IP + (cb + 1);  // black slot
  const unsigned long long hmask = half ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull;
  const uint32_t nslots = gridDim.x * 8u;  // tile slots: 4 waves x 2 halves per block
  for (uint32_t base = (blockIdx.x * 4u + (uint32_t)wv) * 2u; base < n_active;
       base += nslots) {
    const uint32_t li = base + (uint32_t)half;
    const bool has = li < n_active;  // the second half may have no tile
    uint32_t tile = 0;
    int tx = 0, ty = 0;
    if (has) {
      tile = list_at(a.list_in, a.shard_cap, s_pref, li) & kTileMask;
      tx = (int)(tile % (uint32_t)a.ntx);
      ty = (int)(tile / (uint32_t)a.ntx);
    }
    const int64_t i0 = (int64_t)tx * WT, j0 = (int64_t)ty * WT;
    const int64_t gj = j0 + r, gir = i0 + cr, gib = i0 + cb;
    const bool rowin = has && gj < a.ny;
    double tr = dinf(), fr = dinf(), tb = dinf(), fb = dinf();
    if (rowin && gir < a.nx) {
      tr = a.T[gj * a.ld + gir];
      fr = a.F[gj * a.ld + gir];
    }
    if (rowin && gib < a.nx) {
      tb = a.T[gj * a.ld + gib];
      fb = a.F[gj * a.ld + gib];
    }
    // halo ring: west/east cells of row r (lanes q==0 / q==3), south/north
    // cells of columns 2q, 2q+1 (lanes r==0 / r==7)
    double hw = dinf(), he = dinf(), hs0 = dinf(), hs1 = dinf(), hn0 = dinf(), hn1 = dinf();
    if (rowin) {
      if (q == 0 && i0 > 0) hw = a.T[gj * a.ld + (i0 - 1)];
      if (q == 3 && i0 + WT < a.nx) he = a.T[gj * a.ld + (i0 + WT)];
    }
    if (has) {
      const int64_t c0 = i0 + 2 * q, c1 = c0 + 1;
      if (r == 0 && (j0 > 0 || a.ghost_lo)) {
        if (c0 < a.nx) hs0 = a.T[(j0 - 1) * a.ld + c0];
        if (c1 < a.nx) hs1 = a.T[(j0 - 1) * a.ld + c1];
      }
      if (r == WT - 1) {
        const int64_t jn = j0 + WT;
        if (jn < a.ny || (jn == a.ny && a.ghost_hi)) {
          if (c0 < a.nx) hn0 = a.T[jn * a.ld + c0];
          if (c1 < a.nx) hn1 = a.T[jn * a.ld + c1];
        }
      }
    }
    {
      const int row = (r + 1) * IP;
      if (q == 0) img[row] = hw;
      if (q == 3) img[row + WT + 1] = he;
      if (r == 0) {
        img[1 + 2 * q] = hs0;
        img[2 + 2 * q] = hs1;
      }
      if (r == WT - 1) {
        img[(WT + 1) * IP + 1 + 2 * q] = hn0;
        img[(WT + 1) * IP + 2 + 2 * q] = hn1;
      }
      img[sb] = tb;
    }
    const double tr0 = tr, tb0 = tb;
    // sqrt without range scaling is exact while every finite C >= 2^-383
    const bool fast = __all(!(fr < kFastMinF) && !(fb < kFastMinF));
    bool capped;
    const int sweeps = fast ? rb_sweeps<true>(img, sr, sb, fr, fb, tr, tb, a.max_inner, capped)
                            : rb_sweeps<false>(img, sr, sb, fr, fb, tr, tb, a.max_inner, capped);
    if (has) {
      my_visits += 1;
      my_sweeps += (unsigned long long)sweeps;
    }
    const bool dr = tr < tr0, db = tb < tb0;
    if (dr) a.T[gj * a.ld + gir] = tr;
    if (db) a.T[gj * a.ld + gib] = tb;
    // edge flags of this half's tile (cells on row 0 / 7, column 0 / 7)
    const bool w_dec = (cr == 0 && dr) || (cb == 0 && db);
    const bool e_dec = (cr == WT - 1 && dr) || (cb == WT - 1 && db);
    const unsigned long long mS = __ballot(r == 0 && (dr || db)) & hmask;
    const unsigned long long mN = __ballot(r == WT - 1 && (dr || db)) & hmask;
    const unsigned long long mW = __ballot(w_dec) & hmask;
    const unsigned long long mE = __ballot(e_dec) & hmask;
    const unsigned long long mC = __ballot(capped && has) & hmask;
    bool want = false;
    int nx_t = tx, ny_t = ty;
    if (has) {
      if (hl == 0) { want = mS && ty > 0; ny_t = ty - 1; }
      else if (hl == 1) { want = mW && tx > 0; nx_t = tx - 1; }
      else if (hl == 2) { want = mE && tx + 1 < a.ntx; nx_t = tx + 1; }
      else if (hl == 3) { want = mN && ty + 1 < a.nty; ny_t = ty + 1; }
      else if (hl == 4) { want = mC != 0ull; }
    }
    if (want) {
      const uint32_t nt = (uint32_t)ny_t * (uint32_t)a.ntx + (uint32_t)nx_t;
      if (a.tile_epoch[nt] < a.epoch && atomicMax(&a.tile_epoch[nt], a.epoch) < a.epoch) {
        const uint32_t pos = atomicAdd(&s_nq, 1u);
        if (pos < QCAP) {
          s_q[pos] = nt;
        } else {
          const uint32_t gp = atomicAdd(&a.count_out[shard], 1u);
          a.list_out[(uint64_t)shard * a.shard_cap + gp] = nt;
        }
      }
    }
  }
  if (lane == 0 && my_visits) {
    atomicAdd(&s_visits, my_visits);
    atomicAdd(&s_sweeps, my_sweeps);
  }
  if (lane == 32 && my_visits) {  // each half counted its own tiles
    atomicAdd(&s_visits, my_visits);
    atomicAdd(&s_sweeps, my_sweeps);
  }
  __syncthreads();
  const uint32_t nq = s_nq < QCAP ? s_nq : QCAP;
  if (tid == 0) {
    if (nq) s_base = atomicAdd(&a.count_out[shard], nq);
    if (s_visits) {
      unsigned long long* st = a.stats + (uint64_t)shard * kStatSlots;
      atomicAdd(&st[kStatVisits], s_visits);
      atomicAdd(&st[kStatSweeps], s_sweeps);
    }
  }
  __syncthreads();
  for (uint32_t k = tid; k < nq; k += blockDim.x)
    a.list_out[(uint64_t)shard * a.shard_cap + s_base + k] = s_q[k];
}

// ---------------------------------------------------------------------------
// v4 pass kernel: priority passes.  Plain FIM relaxes every
// active tile every pass, so on rough fronts (random media) tiles far ahead of
// the true front are relaxed many times with values that later improve again
// (34 visits/tile at 16384^2).  Here every active tile carries a key -- a lower
// bound on the values it can still take (the minimum changed edge value that
// activated it) -- and a per-list key histogram (kBins bins of width delta from
// the list's minimum key) gives every pass a threshold bin b*: only the ~target
// lowest-key tiles are relaxed, the rest are re-appended unchanged (deferred,
// never dropped, so the fixed point and the result are those of v3).
// Keys are T values (>= 0 or +inf), ordered as u64 bit patterns.
// ---------------------------------------------------------------------------
constexpr unsigned long long kInfBits = 0x7FF0000000000000ull;
constexpr int WCAP = 1024;  // LDS worklist of one classify chunk

__device__ __forceinline__ unsigned long long dbits(double v) {
  return (unsigned long long)__double_as_longlong(v);
}
__device__ __forceinline__ double bitsd(unsigned long long b) {
  return __longlong_as_double((long long)b);
}
// Log-spaced bins: 4 per octave of (key - origin) / delta, so 64 bins span
// delta * 2^16 -- fronts hundreds of cells deep -- with ~19% relative
// resolution and no per-list rescaling.  Classification and histogram use this
// same function, so a tile's bin is consistent between the two.
__device__ __forceinline__ int key_bin(double k, double origin, double inv_delta) {
  const float x = (float)((k - origin) * inv_delta);
  if (!(x > 0.0f)) return 0;
  const float b = 4.0f * __builtin_amdgcn_logf(1.0f + x);  // v_log_f32 (log2)
  return b < (float)(kBins - 1) ? (int)b : kBins - 1;
}

// ---- v4 tile visits: load tile + halo into the wave's LDS image, red-black
// sweeps to local convergence, write back decreased cells, and leave in ek[0..3]
// (S, W, E, N) the minimum decreased value on each edge (+inf bits: unchanged).
// Returns the sweep count; capped = the sweep cap was hit.

// 8x8, half-wave per tile (the v3 body): lane (r, q) owns red column cr and
// black column cb of row r.
__device__ __forceinline__ int visit8(const PassArgs& a, double* img, unsigned long long* ek,
                                      bool has, int tx, int ty, int r, int q, int cr, int cb,
                                      bool& capped) {
  const int sr = (r + 1) * IP + (cr + 1);
  const int sb = (r + 1) * IP + (cb + 1);
  const int64_t i0 = (int64_t)tx * WT, j0 = (int64_t)ty * WT;
  const int64_t gj = j0 + r, gir = i0 + cr, gib = i0 + cb;
  const bool rowin = has && gj < a.ny;
  double tr = dinf(), fr = dinf(), tb = dinf(), fb = dinf();
  if (rowin && gir < a.nx) {
    tr = a.T[gj * a.ld + gir];
    fr = a.F[gj * a.ld + gir];
  }
  if (rowin && gib < a.nx) {
    tb = a.T[gj * a.ld + gib];
    fb = a.F[gj * a.ld + gib];
  }
  double hw = dinf(), he = dinf(), hs0 = dinf(), hs1 = dinf(), hn0 = dinf(), hn1 = dinf();
  if (rowin) {
    if (q == 0 && i0 > 0) hw = a.T[gj * a.ld + (i0 - 1)];
    if (q == 3 && i0 + WT < a.nx) he = a.T[gj * a.ld + (i0 + WT)];
  }
  if (has) {
    const int64_t cc0 = i0 + 2 * q, cc1 = cc0 + 1;
    if (r == 0 && (j0 > 0 || a.ghost_lo)) {
      if (cc0 < a.nx) hs0 = a.T[(j0 - 1) * a.ld + cc0];
      if (cc1 < a.nx) hs1 = a.T[(j0 - 1) * a.ld + cc1];
    }
    if (r == WT - 1) {
      const int64_t jn = j0 + WT;
      if (jn < a.ny || (jn == a.ny && a.ghost_hi)) {
        if (cc0 < a.nx) hn0 = a.T[jn * a.ld + cc0];
        if (cc1 < a.nx) hn1 = a.T[jn * a.ld + cc1];
      }
    }
  }
  {
    const int row = (r + 1) * IP;
    if (q == 0) img[row] = hw;
    if (q == 3) img[row + WT + 1] = he;
    if (r == 0) {
      img[1 + 2 * q] = hs0;
      img[2 + 2 * q] = hs1;
    }
    if (r == WT - 1) {
      img[(WT + 1) * IP + 1 + 2 * q] = hn0;
      img[(WT + 1) * IP + 2 + 2 * q] = hn1;
    }
    img[sb] = tb;
  }
  const double tr0 = tr, tb0 = tb;
  const bool fast = __all(!(fr < kFastMinF) && !(fb < kFastMinF));
  const int sweeps = fast ? rb_sweeps<true>(img, sr, sb, fr, fb, tr, tb, a.max_inner, capped)
                          : rb_sweeps<false>(img, sr, sb, fr, fb, tr, tb, a.max_inner, capped);
  const bool dr = tr < tr0, db = tb < tb0;
  if (dr) a.T[gj * a.ld + gir] = tr;
  if (db) a.T[gj * a.ld + gib] = tb;
  const unsigned long long vr = dr ? dbits(tr) : kInfBits;
  const unsigned long long vb = db ? dbits(tb) : kInfBits;
  // An edge cell n can only improve the cell x across the edge if its new value
  // is below x's (every candidate of x's update using n is >= T(n), :531-535);
  // x's halo snapshot is >= its current value, so the test is safe (prune).
  // The halo ring of the image is never written by the sweeps: it is re-read
  // there rather than kept live in registers.
  auto across = [&](unsigned long long v, double hx) {
    return (v != kInfBits && (!a.prune || v < dbits(hx))) ? v : kInfBits;
  };
  const int odd = r & 1;
  if (r == 0) {  // cr = 2q, cb = 2q+1
    const unsigned long long m0 = across(vr, img[1 + 2 * q]), m1 = across(vb, img[2 + 2 * q]);
    const unsigned long long m = m0 < m1 ? m0 : m1;
    if (m != kInfBits) atomicMin(&ek[0], m);
  }
  if (r == WT - 1) {  // cr = 2q+1, cb = 2q
    const unsigned long long m0 = across(vb, img[(WT + 1) * IP + 1 + 2 * q]);
    const unsigned long long m1 = across(vr, img[(WT + 1) * IP + 2 + 2 * q]);
    const unsigned long long m = m0 < m1 ? m0 : m1;
    if (m != kInfBits) atomicMin(&ek[3], m);
  }
  if (q == 0) {  // column 0: red on even rows, black on odd rows
    const unsigned long long m = across(odd ? vb : vr, img[(r + 1) * IP]);
    if (m != kInfBits) atomicMin(&ek[1], m);
  }
  if (q == 3) {  // column 7: red on odd rows, black on even rows
    const unsigned long long m = across(odd ? vr : vb, img[(r + 1) * IP + WT + 1]);
    if (m != kInfBits) atomicMin(&ek[2], m);
  }
  return sweeps;
}

// 16x16, one tile per wave: lane (r = lane>>2, q = lane&3) owns the four
// cells (r, 4q..4q+3): red columns 4q+(r&1), 4q+2+(r&1), black the other two.
// A half-sweep updates two independent cells per lane.
// Two independent cells of one colour per lane (16x16 tiles).  Both skip
// tests first; if any lane of the wave can improve either cell, both candidates
// are evaluated straight-line and the branch the reference takes (:531-535) is
// picked by a select, so the two dependent chains interleave instead of
// running one after the other behind per-cell branches.  Same operations as
// rb_update: bit-identical results (a discarded two-sided candidate may be
// NaN from a negative radicand; it is never selected).
template <bool FAST, bool APPROX = false>
__device__ __forceinline__ void rb_update2(const double* p, const double* pn, const double* ps,
                                           double f0, double f1, double& t0, double& t1,
                                           bool& ch0, bool& ch1) {
  // p: the lane's first cell of this colour (the second is p + 2, same row);
  // pn / ps: the same column in the rows above / below (skewed image rows).
  // All neighbour reads in flight before the first use (cell 1's W is cell 0's E).
  double w0 = p[-1], e0 = p[1], n0 = pn[0], so0 = ps[0];
  double e1 = p[3], n1 = pn[2], so1 = ps[2];
  // one wait for all of them (the v_min asm below would otherwise pin reads behind it);
  // cell 1's W is cell 0's E, one register (a separate asm operand costs a copy)
  asm volatile("" : "+v"(w0), "+v"(e0), "+v"(n0), "+v"(so0), "+v"(e1), "+v"(n1), "+v"(so1));
  const double w1 = e0;
  // No skip test: u < t alone decides (u >= min + C/sqrt(2) > min + 0.7071 C, so
  // the skip test of rb_update never rejects an improving candidate), and the
  // half-sweep is one straight-line dependent chain without a scalar branch.
  const double c20 = 2.0 * (f0 * f0), c21 = 2.0 * (f1 * f1);
  const double tx0 = vmin64(w0, e0), ty0 = vmin64(n0, so0);
  const double tx1 = vmin64(w1, e1), ty1 = vmin64(n1, so1);
  const double m0 = vmin64(tx0, ty0), m1 = vmin64(tx1, ty1);
  {
    const double d0 = tx0 - ty0, d1 = tx1 - ty1;
    // the monotone combine: T' = min + h, h = C on the one-sided branch; the select
    // (or the clamp of cand_approx) comes before the one add at the scale of T
    double h0, h1;  // two-sided half-sums (|d| + sqrt(2C^2 - d^2)) / 2
    if constexpr (FAST && APPROX) {
      // cand_approx: the branch folded into the argument min(|d|, C).  An obstacle
      // (f = inf) gives NaN (rsq(inf) * inf), which v_min ignores; d = NaN (no finite
      // neighbour) gives min(|NaN|, C) = C, and m = inf keeps the candidate at inf
      double u0, u1;
      cand_approx2(vmin64_abs(d0, f0), c20, m0, vmin64_abs(d1, f1), c21, m1, u0, u1);
      ch0 = u0 < t0;
      ch1 = u1 < t1;
      t0 = vmin64(t0, u0);
      t1 = vmin64(t1, u1);
      return;
    } else {
      const double r0 = __builtin_fma(-d0, d0, c20), r1 = __builtin_fma(-d1, d1, c21);
      double q0, q1;
      if constexpr (FAST) {
        sqrt_cr_fast2<APPROX>(r0, r1, q0, q1);
      } else {
        q0 = sqrt(r0);
        q1 = sqrt(r1);
      }
      h0 = (fabs(d0) + q0) * 0.5;
      h1 = (fabs(d1) + q1) * 0.5;
    }
    const double u0 = m0 + (fabs(d0) < f0 ? h0 : f0);
    const double u1 = m1 + (fabs(d1) < f1 ? h1 : f1);
    ch0 = u0 < t0;
    ch1 = u1 < t1;
    // min(t, u) == (u < t ? u : t): one v_min_f64 on the chain to the LDS write
    // (a NaN candidate -- obstacle cells on the FAST path -- leaves t, as v_min does)
    t0 = vmin64(t0, u0);
    t1 = vmin64(t1, u1);
  }
}

// pr / pb: the lane's first red / black cell in the image; dn / ds: slots to the
// same column one row up / down (the lane's row and its neighbours, img16_row)
template <bool FAST, bool APPROX = false>
__device__ __forceinline__ int rb_sweeps4(double* pr, double* pb, int dn, int ds,
                                          const double (&fr)[2], const double (&fb)[2],
                                          double (&tr)[2], double (&tb)[2], int max_inner,
                                          bool& capped, uint32_t stop_at) {
  const double *prn = pr + dn, *prs = pr - ds, *pbn = pb + dn, *pbs = pb - ds;
  int sweeps = 0;
  capped = true;
  // past stop_at (the pass deadline) a visit ends as if capped -- but only after
  // its first sweep pair, so every visit makes progress and the solve terminates
  // (the low 32 bits of the 10-ns clock, compared wrap-safe: scalar instructions only)
  while (sweeps < max_inner &&
         (sweeps == 0 || (int32_t)(stop_at - (uint32_t)__builtin_amdgcn_s_memrealtime()) > 0)) {
    bool i0, i1, i2, i3;
    // two sweeps per convergence test: the second sweep's flags decide (a sweep
    // that changes nothing is the local fixed point)
    __builtin_amdgcn_wave_barrier();
    rb_update2<FAST, APPROX>(pr, prn, prs, fr[0], fr[1], tr[0], tr[1], i0, i1);
    pr[0] = tr[0];
    pr[2] = tr[1];
    __builtin_amdgcn_wave_barrier();
    rb_update2<FAST, APPROX>(pb, pbn, pbs, fb[0], fb[1], tb[0], tb[1], i2, i3);
    pb[0] = tb[0];
    pb[2] = tb[1];
    ++sweeps;
    __builtin_amdgcn_wave_barrier();
    rb_update2<FAST, APPROX>(pr, prn, prs, fr[0], fr[1], tr[0], tr[1], i0, i1);
    pr[0] = tr[0];
    pr[2] = tr[1];
    __builtin_amdgcn_wave_barrier();
    rb_update2<FAST, APPROX>(pb, pbn, pbs, fb[0], fb[1], tb[0], tb[1], i2, i3);
    pb[0] = tb[0];
    pb[2] = tb[1];
    ++sweeps;
    // the lane masks of the four compares, or-ed in scalar registers (no VGPR round trip)
    if ((__builtin_amdgcn_ballot_w64(i0) | __builtin_amdgcn_ballot_w64(i1) |
         __builtin_amdgcn_ballot_w64(i2) | __builtin_amdgcn_ballot_w64(i3)) == 0) {
      capped = false;
      break;
    }
  }
  __builtin_amdgcn_wave_barrier();
  return sweeps;
}

struct NoGate {
  __device__ bool operator()() const { return true; }
};

// gate(): wave-uniform, evaluated after the tile's loads are issued (so a key
// load the gate waits on overlaps them); false = skip the visit, return -1.
template <bool APPROX = false, class Gate = NoGate>
__device__ __forceinline__ int visit16(const PassArgs& a, double* img, unsigned long long* ek,
                                       bool has, int tx, int ty, int lane, bool& capped,
                                       Gate gate, uint32_t stop_at) {
  const int cap = a.max_inner;
  constexpr int TT = 16;
  const int r = lane >> 2, q = lane & 3, odd = r & 1;
  const int cr[2] = {4 * q + odd, 4 * q + 2 + odd};
  const int cb[2] = {4 * q + 1 - odd, 4 * q + 3 - odd};
  const int rb = img16_row(r);  // slot of (r, 0); the halo columns are rb - 1, rb + 16
  const int dn = img16_row(r + 1) - rb, ds = rb - img16_row(r - 1);
  const int sr[2] = {rb + cr[0], rb + cr[1]};
  const int sb[2] = {rb + cb[0], rb + cb[1]};
  const int64_t i0 = (int64_t)tx * TT, j0 = (int64_t)ty * TT;
  const int64_t gj = j0 + r;
  const bool rowin = has && gj < a.ny;
  double tr[2], tb[2], fr[2], fb[2];
  double hw, he, hs[4], hn[4];
  // interior tile (wave-uniform): every cell and halo address is valid, so every
  // lane loads unmasked -- no +inf defaults, bounds tests or exec-mask branches.
  // The halo loads of lanes that do not own a halo cell read valid duplicates
  // of their neighbours' addresses and are never stored to the image.
  const bool interior = has && i0 > 0 && i0 + TT < a.nx && (j0 > 0 || a.ghost_lo) &&
                        (j0 + TT < a.ny || (j0 + TT == a.ny && a.ghost_hi));
  if (interior) {
    const double* Tr = a.T + gj * a.ld + i0;
    const double* Fr = a.F + gj * a.ld + i0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      tr[k] = Tr[cr[k]];
      fr[k] = Fr[cr[k]];
      tb[k] = Tr[cb[k]];
      fb[k] = Fr[cb[k]];
    }
    {  // the neighbours' edge columns: one line each instead of 16
      const double* e = a.ec + ((uint64_t)ty * (uint64_t)a.ntx + (uint64_t)tx) * 32 + r;
      hw = e[-32 + 16];
      he = e[32];
    }
    const double* Ts = a.T + (j0 - 1) * a.ld + i0 + 4 * q;
    const double* Tn = a.T + (j0 + TT) * a.ld + i0 + 4 * q;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hs[k] = Ts[k];
      hn[k] = Tn[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      tr[k] = fr[k] = tb[k] = fb[k] = dinf();
      if (rowin && i0 + cr[k] < a.nx) {
        tr[k] = a.T[gj * a.ld + i0 + cr[k]];
        fr[k] = a.F[gj * a.ld + i0 + cr[k]];
      }
      if (rowin && i0 + cb[k] < a.nx) {
        tb[k] = a.T[gj * a.ld + i0 + cb[k]];
        fb[k] = a.F[gj * a.ld + i0 + cb[k]];
      }
    }
    hw = dinf();
    he = dinf();
    if (rowin) {
      if (q == 0 && i0 > 0) hw = a.T[gj * a.ld + (i0 - 1)];
      if (q == 3 && i0 + TT < a.nx) he = a.T[gj * a.ld + (i0 + TT)];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) hs[k] = hn[k] = dinf();
    if (has) {
      if (r == 0 && (j0 > 0 || a.ghost_lo)) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i0 + 4 * q + k < a.nx) hs[k] = a.T[(j0 - 1) * a.ld + i0 + 4 * q + k];
      }
      if (r == TT - 1) {
        const int64_t jn = j0 + TT;
        if (jn < a.ny || (jn == a.ny && a.ghost_hi)) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (i0 + 4 * q + k < a.nx) hn[k] = a.T[jn * a.ld + i0 + 4 * q + k];
        }
      }
    }
  }
  asm volatile("" ::: "memory");  // the loads above issue before the gate's wait
  if (!gate()) return -1;
  if (q == 0) img[rb - 1] = hw;
  if (q == 3) img[rb + TT] = he;
  if (r == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) img[img16_row(-1) + 4 * q + k] = hs[k];
  }
  if (r == TT - 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) img[img16_row(TT) + 4 * q + k] = hn[k];
  }
  img[sb[0]] = tb[0];
  img[sb[1]] = tb[1];
  const double tr0[2] = {tr[0], tr[1]}, tb0[2] = {tb[0], tb[1]};
  const bool fast = __all(!(fr[0] < kFastMinF) && !(fr[1] < kFastMinF) &&
                          !(fb[0] < kFastMinF) && !(fb[1] < kFastMinF));
  const int sweeps =
      fast ? rb_sweeps4<true, APPROX>(img + sr[0], img + sb[0], dn, ds, fr, fb, tr, tb, cap,
                                      capped, stop_at)
           : rb_sweeps4<false>(img + sr[0], img + sb[0], dn, ds, fr, fb, tr, tb, cap, capped,
                               stop_at);
  // write back decreased cells; dr/db: the decreased value or +inf.  Keys are
  // non-negative doubles, so the u64 order of their bits (ek) is their f64
  // order and the edge minima below are v_min_f64 / v_cmp_f64 work.
  double dr[2], db[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool cr_ = tr[k] < tr0[k], cb_ = tb[k] < tb0[k];
    if (cr_) a.T[gj * a.ld + i0 + cr[k]] = tr[k];
    if (cb_) a.T[gj * a.ld + i0 + cb[k]] = tb[k];
    dr[k] = cr_ ? tr[k] : dinf();
    db[k] = cb_ ? tb[k] : dinf();
  }
  // exact pruning (as visit8): a decreased edge cell counts only if it is below
  // the halo snapshot across the edge, re-read from the image.  "Exact" holds
  // for the reference arithmetic (a candidate through n is >= T(n)); with the
  // default sweep sqrt a two-sided candidate may undercut max(Tx, Ty) by a few
  // ulp, so an activation of that size can be skipped -- a deviation within the
  // solve tolerance, not a change of the fixed point's mask.
  auto across = [&](double v, double hx) { return (!a.prune || v < hx) ? v : dinf(); };
  if (r == 0 || r == TT - 1) {  // S / N edge: rows 0 and 15 (disjoint lanes), halo row beyond
    const int vo = r == 0 ? -ds : dn;
    const double m = vmin64(vmin64(across(dr[0], img[sr[0] + vo]), across(dr[1], img[sr[1] + vo])),
                            vmin64(across(db[0], img[sb[0] + vo]), across(db[1], img[sb[1] + vo])));
    if (m < dinf()) atomicMin(&ek[r == 0 ? 0 : 3], dbits(m));
  }
  if (q == 0 || q == 3) {  // W / E edge: column 0 (cr[0] or cb[0]) / column 15 (cr[1] or cb[1])
    const double c = q == 0 ? (odd ? db[0] : dr[0]) : (odd ? dr[1] : db[1]);
    if (c < dinf()) a.ec[((uint64_t)ty * (uint64_t)a.ntx + (uint64_t)tx) * 32 + (q == 0 ? 0 : 16) + r] = c;
    const double m = across(c, img[q == 0 ? rb - 1 : rb + TT]);
    if (m < dinf()) atomicMin(&ek[q == 0 ? 1 : 2], dbits(m));
  }
  return sweeps;
}

// TS 8: two 8x8 tiles per wave (v3 body); 16: one 16x16 tile per wave.
// WPB waves per workgroup: bigger workgroups pool the ready tiles of bigger
// chunks, so fewer of them overflow their wave slots into a second round.
template <int TS, int WPB = 4>
__global__ __launch_bounds__(64 * WPB, 4) void k_fim_pass_prio(PassArgs a) {
  static_assert(TS == 8, "kernel 4: 8x8 tiles (16x16 tiles are kernel 5, k_fim_pass_dyn)");
  constexpr int TPW = TS == 8 ? 2 : 1;  // tiles per wave
  constexpr int SLOTS = WPB * TPW;       // tile slots per workgroup
  constexpr int IMG = (WT + 2) * IP;
  __shared__ uint32_t s_q[QCAP];
  __shared__ uint32_t s_work[WCAP];
  __shared__ unsigned long long s_wkey[WCAP];
  __shared__ uint32_t s_pref[kShards + 1];
  __shared__ uint32_t s_hout[kBins];
  __shared__ uint32_t s_nq, s_base, s_nwork;
  __shared__ int s_bstar;
  __shared__ unsigned long long s_visits, s_sweeps, s_minout;
  __shared__ unsigned long long s_ek[SLOTS][4];
  __shared__ double s_img[SLOTS][IMG];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int half = lane >> 5;
  const int hl = lane & 31;
  const int r = hl >> 2, q = hl & 3;
  const int cr = 2 * q + (r & 1), cb = 2 * q + 1 - (r & 1);
  const uint32_t shard = blockIdx.x % kShards;
  unsigned long long* trace = a.trace ? a.trace + (uint64_t)blockIdx.x * kTracePts : nullptr;
  if (trace && tid == 0) trace[0] = __builtin_amdgcn_s_memrealtime();

  // scalars first (independent loads, issued before the wave-0 scan)
  const double delta = *a.delta;
  const double origin_in = *a.base_in;            // bins of list p
  const double origin_out = bitsd(*a.minkey_in);  // bins of list p+1
  const double inv_delta = 1.0 / delta;
  if (wv == 0) {
    // list-shard prefix counts and the threshold bin, one wave, no serial loops
    uint32_t c = lane < kShards ? a.count_in[lane] : 0u;
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < kShards; ++k) h += a.hist_in[k * kBins + lane];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t yc = __shfl_up(c, o), yh = __shfl_up(h, o);
      if (lane >= o) {
        c += yc;
        h += yh;
      }
    }
    if (lane < kShards) s_pref[lane + 1] = c;
    const uint32_t n = __shfl(c, kShards - 1);
    const uint32_t fr = (uint32_t)(a.target_frac * (float)n);
    const uint32_t target = a.target > fr ? a.target : fr;
    const unsigned long long m = __ballot(h >= target && lane < kBins - 1);
    if (lane == 0) {
      s_pref[0] = 0u;
      s_bstar = (a.target > 0 && n > target && m) ? (int)__ffsll((long long)m) - 1 : kBins;
      s_nq = 0;
      s_visits = 0;
      s_sweeps = 0;
      s_minout = kInfBits;
    }
  }
  s_hout[tid & (kBins - 1)] = 0u;
  __syncthreads();
  const uint32_t n_active = s_pref[kShards];
  const int bstar = s_bstar;
  if (trace && tid == 0) trace[1] = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0) {
    if (tid < kShards) a.count_clear[tid] = 0u;
    for (int k = tid; k < kShards * kBins; k += blockDim.x) a.hist_clear[k] = 0u;
    if (tid == 0) {
      *a.minkey_clear = kInfBits;
      *a.base_out = origin_out;
      if (n_active > 0) {
        atomicAdd(&a.stats[kStatPasses], 1ull);
        atomicMax(&a.stats[kStatMaxActive], (unsigned long long)n_active);
      }
      report_pending(a, n_active);
    }
  }

  // append tile t with key kb to list p+1 (key = running min over its activations)
  auto enqueue = [&](uint32_t t, unsigned long long kb) {
    atomicMin(&a.key_out[t], kb);
    atomicMin(&s_minout, kb);
    if (atomicMax(&a.tile_epoch[t], a.epoch) < a.epoch) {
      const int bin = key_bin(bitsd(kb), origin_out, inv_delta);
      atomicAdd(&s_hout[bin], 1u);
      const uint32_t ent = a.pack_bins ? (t | ((uint32_t)(bin + 1) << kPackShift)) : t;
      const uint32_t pos = atomicAdd(&s_nq, 1u);
      if (pos < QCAP) {
        s_q[pos] = ent;
      } else {
        const uint32_t gp = atomicAdd(&a.count_out[shard], 1u);
        a.list_out[(uint64_t)shard * a.shard_cap + gp] = ent;
      }
    }
  };

  unsigned long long my_visits = 0, my_sweeps = 0;
  const int slot = TS == 8 ? wv * 2 + half : wv;
  const int sl = TS == 8 ? hl : lane;  // lane within the tile's lane group
  double* img = s_img[slot];
  unsigned long long* ek = s_ek[slot];
  const unsigned long long hmask =
      TS == 16 ? ~0ull : (half ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull);

  // this workgroup's share of the active list: a contiguous chunk
  const uint32_t chunk = (n_active + gridDim.x - 1) / gridDim.x;
  const uint32_t c0 = blockIdx.x * chunk;
  const uint32_t c1 = min(n_active, c0 + chunk);
  for (uint32_t s0 = c0; s0 < c1; s0 += WCAP) {  // block-uniform
    const uint32_t s1 = min(c1, s0 + WCAP);
    if (tid == 0) s_nwork = 0;
    __syncthreads();
    for (uint32_t e = s0 + tid; e < s1; e += blockDim.x) {
      const uint32_t t = list_at(a.list_in, a.shard_cap, s_pref, e) & kTileMask;
      const unsigned long long kb = a.key_in[t];
      a.key_in[t] = kInfBits;
      if (key_bin(bitsd(kb), origin_in, inv_delta) <= bstar) {
        const uint32_t pos = atomicAdd(&s_nwork, 1u);
        s_work[pos] = t;
        s_wkey[pos] = kb;
      } else {
        enqueue(t, kb);  // deferred
      }
    }
    __syncthreads();
    const uint32_t nw = s_nwork;
    if (trace && tid == 0 && s0 == c0) trace[2] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t wb = (uint32_t)(wv * TPW); wb < nw; wb += (uint32_t)SLOTS) {  // wave-uniform
      const uint32_t li = wb + (uint32_t)(TS == 8 ? half : 0);
      const bool has = li < nw;
      uint32_t tile = 0;
      int tx = 0, ty = 0;
      if (has) {
        tile = s_work[li];
        tx = (int)(tile % (uint32_t)a.ntx);
        ty = (int)(tile / (uint32_t)a.ntx);
      }
      if (sl < 4) ek[sl] = kInfBits;
      if (trace && tid == 0 && wb == 0) trace[6] = __builtin_amdgcn_s_memrealtime();
      bool capped;
      int sweeps;
      sweeps = visit8(a, img, ek, has, tx, ty, r, q, cr, cb, capped);
      if (trace && tid == 0 && wb == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        trace[7] = __builtin_amdgcn_s_memrealtime();
        trace[9] = (unsigned long long)sweeps;
      }
      if (has) {
        my_visits += 1;
        my_sweeps += (unsigned long long)sweeps;
      }
      const unsigned long long mC = __ballot(capped && has) & hmask;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      bool want = false;
      int nx_t = tx, ny_t = ty;
      unsigned long long kb = kInfBits;
      if (has && sl < 4) {
        kb = ek[sl];
        if (sl == 0) { want = kb != kInfBits && ty > 0; ny_t = ty - 1; }
        else if (sl == 1) { want = kb != kInfBits && tx > 0; nx_t = tx - 1; }
        else if (sl == 2) { want = kb != kInfBits && tx + 1 < a.ntx; nx_t = tx + 1; }
        else { want = kb != kInfBits && ty + 1 < a.nty; ny_t = ty + 1; }
      } else if (has && sl == 4 && mC != 0ull) {
        want = true;
        kb = s_wkey[li];
      }
      if (want) enqueue((uint32_t)ny_t * (uint32_t)a.ntx + (uint32_t)nx_t, kb);
      __builtin_amdgcn_wave_barrier();
      if (trace && wb == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        if (tid == 0) trace[8] = __builtin_amdgcn_s_memrealtime();
      }
    }
    __syncthreads();
  }
  if (trace && tid == 0) trace[3] = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && my_visits) {
    atomicAdd(&s_visits, my_visits);
    atomicAdd(&s_sweeps, my_sweeps);
  }
  if (TS == 8 && lane == 32 && my_visits) {  // each half counted its own tiles
    atomicAdd(&s_visits, my_visits);
    atomicAdd(&s_sweeps, my_sweeps);
  }
  __syncthreads();
  const uint32_t nq = s_nq < QCAP ? s_nq : QCAP;
  if (tid == 0) {
    if (nq) s_base = atomicAdd(&a.count_out[shard], nq);
    if (s_minout != kInfBits) atomicMin(a.minkey_out, s_minout);
    if (s_visits) {
      unsigned long long* st = a.stats + (uint64_t)shard * kStatSlots;
      atomicAdd(&st[kStatVisits], s_visits);
      atomicAdd(&st[kStatSweeps], s_sweeps);
    }
  }
  if (tid < kBins && s_hout[tid]) atomicAdd(&a.hist_out[shard * kBins + tid], s_hout[tid]);
  __syncthreads();
  for (uint32_t k = tid; k < nq; k += blockDim.x)
    a.list_out[(uint64_t)shard * a.shard_cap + s_base + k] = s_q[k];
  if (trace && tid == 0) {
    trace[4] = __builtin_amdgcn_s_memrealtime();
    trace[5] = ((unsigned long long)(c1 > c0 ? c1 - c0 : 0) << 32) | (unsigned long long)s_visits;
  }
}

// Kernel 5 with wave-level dynamic scheduling (16x16 tiles): each wave takes
// the next entry of its workgroup's chunk from an LDS counter, loads the key
// and the tile together, and either defers the tile (key above the threshold
// bin) or visits it.  No classify phase and no block-wide barrier between
// reading the list and the sweeps: a wave that drew a deferred or a quickly
// converging tile moves on to the next entry while the others still sweep.
// STATS: the per-pass statistics (a.pstat) are counted -- a separate instantiation,
// so the default kernel carries none of it (it cost 2% per solve inline: SGPR
// spills 31 -> 41, profiles/r03/knobs1)
template <int WPB, bool APPROX, bool STATS = false>
__global__ __launch_bounds__(64 * WPB, 4) void k_fim_pass_dyn(PassArgs a) {
  constexpr int IMG = IMG16;
  __shared__ uint32_t s_q[QCAP];
  __shared__ uint32_t s_pref[kShards + 1];
  __shared__ uint32_t s_hout[kBins];
  __shared__ uint32_t s_nq, s_base, s_next, s_merge;
  __shared__ int s_bstar;
  __shared__ unsigned long long s_visits, s_sweeps, s_minout, s_defer;
  __shared__ unsigned long long s_ek[WPB][4];
  __shared__ double s_img[WPB][IMG];
  __shared__ uint32_t s_ps[4];  // pass statistics: colour, capped, deadline, max radius
  __shared__ uint32_t s_psmin;  // ~min radius

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const uint32_t shard = blockIdx.x % kShards;
  unsigned long long* trace = a.trace ? a.trace + (uint64_t)blockIdx.x * kTracePts : nullptr;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  // no deadline: 2^30 ticks (10.7 s) ahead, far beyond any pass
  const uint32_t stop_at = (uint32_t)t_start + (a.sweep_deadline ? a.sweep_deadline : (1u << 30));
  if (trace && tid == 0) trace[0] = t_start;

  const double delta = *a.delta;
  const double origin_in = *a.base_in;
  const double origin_out = bitsd(*a.minkey_in);
  const double inv_delta = 1.0 / delta;
  if (wv == 0) {  // shard prefix counts and the threshold bin (as k_fim_pass_prio)
    uint32_t c = lane < kShards ? a.count_in[lane] : 0u;
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < kShards; ++k) h += a.hist_in[k * kBins + lane];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t yc = __shfl_up(c, o), yh = __shfl_up(h, o);
      if (lane >= o) {
        c += yc;
        h += yh;
      }
    }
    if (lane < kShards) s_pref[lane + 1] = c;
    const uint32_t n = __shfl(c, kShards - 1);
    const uint32_t fr = (uint32_t)(a.target_frac * (float)n);
    uint32_t target = a.target > fr ? a.target : fr;
    if (a.cap_frac > 0.0f) {  // at most this fraction of the list (not below 256 tiles)
      uint32_t cf = (uint32_t)(a.cap_frac * (float)n);
      cf = cf > 256u ? cf : 256u;
      target = target < cf ? target : cf;
    }
    const unsigned long long m = __ballot(h >= target && lane < kBins - 1);
    if (lane == 0) {
      s_pref[0] = 0u;
      s_bstar = (a.target > 0 && n > target && m) ? (int)__ffsll((long long)m) - 1 : kBins;
      s_nq = 0;
      s_next = 0;
      s_merge = 0;
      s_visits = 0;
      s_sweeps = 0;
      s_defer = 0;
      s_minout = kInfBits;
      s_ps[0] = s_ps[1] = s_ps[2] = s_ps[3] = 0u;
      s_psmin = 0u;
    }
  }
  s_hout[tid & (kBins - 1)] = 0u;
  __syncthreads();
  const uint32_t n_active = s_pref[kShards];
  const int bstar = s_bstar;
  if (trace && tid == 0) trace[1] = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0) {
    if (tid < kShards) a.count_clear[tid] = 0u;
    for (int k = tid; k < kShards * kBins; k += blockDim.x) a.hist_clear[k] = 0u;
    if (tid == 0) {
      *a.minkey_clear = kInfBits;
      *a.base_out = origin_out;
      if (n_active > 0) {
        atomicAdd(&a.stats[kStatPasses], 1ull);
        atomicMax(&a.stats[kStatMaxActive], (unsigned long long)n_active);
      }
      if (STATS && a.pstat) {
        a.pstat[kPsActive] = n_active;
        a.pstat[kPsBstar] = (uint32_t)bstar;
      }
      report_pending(a, n_active);
      if (a.tot_save) *a.tot_save = n_active;
      if (a.tot_out) *a.tot_out = (int32_t)(*a.tot_prev + n_active);
      if (a.peer && a.tot_out) peer_status(a.peer);
    }
  }

  auto enqueue = [&](uint32_t t, unsigned long long kb) {
    atomicMin(&a.key_out[t], kb);
    atomicMin(&s_minout, kb);
    if (atomicMax(&a.tile_epoch[t], a.epoch) < a.epoch) {
      const int bin = key_bin(bitsd(kb), origin_out, inv_delta);
      atomicAdd(&s_hout[bin], 1u);
      const uint32_t ent = a.pack_bins ? (t | ((uint32_t)(bin + 1) << kPackShift)) : t;
      const uint32_t pos = atomicAdd(&s_nq, 1u);
      if (pos < QCAP) {
        s_q[pos] = ent;
      } else {
        const uint32_t gp = atomicAdd(&a.count_out[shard], 1u);
        a.list_out[(uint64_t)shard * a.shard_cap + gp] = ent;
      }
    }
  };

  unsigned long long my_visits = 0, my_sweeps = 0, my_defer = 0;
  uint32_t my_cd = 0, my_cap = 0, my_dl = 0, my_rmax = 0, my_rmin = ~0u;  // a.pstat only
  double* img = s_img[wv];
  unsigned long long* ek = s_ek[wv];
  // the workgroup's entries are every gridDim.x-th of the list from its own index, not
  // a contiguous chunk: a producer flushes its queue contiguously, so a chunk holds
  // neighbours of the same visits -- mostly admitted or mostly deferred together -- and
  // a workgroup with more visits than waves ends the pass late; strided, the visits
  // per workgroup spread binomially around the mean
  const uint32_t nb = gridDim.x;
  bool first = true;
  if (trace && tid == 0) trace[2] = __builtin_amdgcn_s_memrealtime();
  for (;;) {  // wave-uniform
    uint32_t e = 0;
    if (lane == 0) e = blockIdx.x + atomicAdd(&s_next, 1u) * nb;
    e = __builtin_amdgcn_readfirstlane(e);
    if (e >= n_active) break;
    const uint32_t ent =
        __builtin_amdgcn_readfirstlane(list_at_wave(a.list_in, a.shard_cap, s_pref, e, lane));
    const uint32_t tile = ent & kTileMask;
    const int pbin = (int)(ent >> kPackShift) - 1;  // first-insertion bin, -1: none
    const int tx = (int)(tile % (uint32_t)a.ntx);
    const int ty = (int)(tile / (uint32_t)a.ntx);
    if (a.checker && ((uint32_t)(tx + ty) + a.checker_parity) % 2u != 0u) {
      // the other colour of the checkerboard: deferred with its key, tile not loaded
      if (lane == 0) {
        const unsigned long long k0 = a.key_in[tile];
        a.key_in[tile] = kInfBits;
        enqueue(tile, k0);
      }
      ++my_defer;
      if (STATS && a.pstat) ++my_cd;
      continue;
    }
    const unsigned long long kb = a.key_in[tile];
    // a packed bin at or below b*: admitted (the current key is no higher); above: the
    // current key decides now, before the tile loads a deferral would waste
    if (pbin > bstar && key_bin(bitsd(kb), origin_in, inv_delta) > bstar) {
      if (lane == 0) {
        a.key_in[tile] = kInfBits;
        enqueue(tile, kb);
      }
      ++my_defer;
      continue;
    }
    const bool decided = pbin >= 0;
    if (lane < 4) ek[lane] = kInfBits;
    if (trace && tid == 0 && first) trace[6] = __builtin_amdgcn_s_memrealtime();
    bool capped = false;
    const int sweeps = visit16<APPROX>(
        a, img, ek, true, tx, ty, lane, capped,
        [&] { return decided || key_bin(bitsd(kb), origin_in, inv_delta) <= bstar; }, stop_at);
    if (lane == 0) a.key_in[tile] = kInfBits;
    if (sweeps < 0) {  // deferred to the next pass with its key
      if (lane == 0) enqueue(tile, kb);
      ++my_defer;
      continue;
    }
    if (trace && tid == 0 && first) {
      __builtin_amdgcn_s_waitcnt(0);
      trace[7] = __builtin_amdgcn_s_memrealtime();
      trace[9] = (unsigned long long)sweeps;
    }
    my_visits += 1;
    my_sweeps += (unsigned long long)sweeps;
    const bool cap = __any(capped);
    if (STATS && a.pstat) {
      if (cap) {
        if (sweeps >= a.max_inner) ++my_cap;
        else ++my_dl;
      }
      const uint32_t rad = (uint32_t)(abs(tx - a.goal_tx) + abs(ty - a.goal_ty));
      my_rmax = rad > my_rmax ? rad : my_rmax;
      my_rmin = rad < my_rmin ? rad : my_rmin;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bool want = false;
    int nx_t = tx, ny_t = ty;
    unsigned long long k2 = kInfBits;
    if (lane < 4) {
      k2 = ek[lane];
      if (lane == 0) { want = k2 != kInfBits && ty > 0; ny_t = ty - 1; }
      else if (lane == 1) { want = k2 != kInfBits && tx > 0; nx_t = tx - 1; }
      else if (lane == 2) { want = k2 != kInfBits && tx + 1 < a.ntx; nx_t = tx + 1; }
      else { want = k2 != kInfBits && ty + 1 < a.nty; ny_t = ty + 1; }
    } else if (lane == 4 && cap) {
      want = true;
      k2 = kb;
    }
    if (want) enqueue((uint32_t)ny_t * (uint32_t)a.ntx + (uint32_t)nx_t, k2);
    __builtin_amdgcn_wave_barrier();
    if (trace && first) {
      __builtin_amdgcn_s_waitcnt(0);
      if (tid == 0) trace[8] = __builtin_amdgcn_s_memrealtime();
    }
    first = false;
  }
  const bool pushes = a.push_dst[0] || a.push_dst[1];  // peer rounds: this pass pushes
  if (a.merge_lo || a.merge_hi || pushes) {  // uniform; the first wave out of the loop merges
    uint32_t mine = 0;
    if (lane == 0) mine = atomicAdd(&s_merge, 1u) == 0u;
    if (__builtin_amdgcn_readfirstlane(mine)) {
      // this workgroup's share of the columns (a whole number of 16-wide tiles): min-merge
      // the received rows into the ghost rows, queue the tile under each improved column
      // group with the smallest improved value as its key (as k_merge_ghosts)
      const int64_t cw = (((int64_t)a.nx + gridDim.x - 1) / gridDim.x + 15) & ~(int64_t)15;
      const int64_t m0 = (int64_t)blockIdx.x * cw;
      const int64_t m1 = min((int64_t)a.nx, m0 + cw);
      for (int side = 0; side < 2; ++side) {
        const double* src = side == 0 ? a.merge_lo : a.merge_hi;
        if (!src) continue;
        const bool tagged = a.merge_tag[side] != nullptr;  // peer rounds: a neighbour writes src
        if (tagged && m0 < m1) {
          // the tag first: the rows of every push up to it are complete (the pusher's
          // release); R = the smallest tag any workgroup read (status pass).  Every lane
          // performs the acquire, so each lane's row loads below are ordered after it by
          // the memory model, not only by the wave's lockstep (one line)
          const unsigned long long t = __hip_atomic_load(a.merge_tag[side], __ATOMIC_ACQUIRE,
                                                         __HIP_MEMORY_SCOPE_SYSTEM);
          if (lane == 0)
            __hip_atomic_fetch_min(&a.peer->rmin[side], t, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        double* gh = a.T + (side == 0 ? -a.ld : a.ny * a.ld);
        const uint32_t trow = side == 0 ? 0u : (uint32_t)(a.nty - 1);
        for (int64_t k0 = m0; k0 < m1; k0 += 64) {
          const int64_t k = k0 + lane;
          double w = dinf();
          if (k < m1) {
            // a row another process's kernel writes while this one runs: system-scope
            // loads (any mix of old and new 8-byte values is a valid upper bound)
            const double v = tagged ? __hip_atomic_load(const_cast<double*>(src) + k,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                    : src[k];
            if (v < gh[k]) {
              gh[k] = v;
              w = v;
            }
          }
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) w = vmin64(w, __shfl_xor(w, o));
          if ((lane & 15) == 0 && k < m1 && w < dinf())
            enqueue(trow * (uint32_t)a.ntx + (uint32_t)(k >> 4), dbits(w));
        }
      }
      if (pushes) peer_push(a, m0, m1, lane);
    }
  }
  if (trace && tid == 0) trace[3] = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && (my_visits || my_defer)) {
    atomicAdd(&s_visits, my_visits);
    atomicAdd(&s_sweeps, my_sweeps);
    atomicAdd(&s_defer, my_defer);
    if (STATS && a.pstat) {
      atomicAdd(&s_ps[0], my_cd);
      atomicAdd(&s_ps[1], my_cap);
      atomicAdd(&s_ps[2], my_dl);
      atomicMax(&s_ps[3], my_rmax);
      if (my_visits) atomicMax(&s_psmin, ~my_rmin);
    }
  }
  __syncthreads();
  const uint32_t nq = s_nq < QCAP ? s_nq : QCAP;
  if (tid == 0) {
    if (nq) s_base = atomicAdd(&a.count_out[shard], nq);
    if (s_minout != kInfBits) atomicMin(a.minkey_out, s_minout);
    if (s_visits || s_defer) {
      unsigned long long* st = a.stats + (uint64_t)shard * kStatSlots;
      atomicAdd(&st[kStatVisits], s_visits);
      atomicAdd(&st[kStatSweeps], s_sweeps);
      if (s_defer) atomicAdd(&st[kStatDeferred], s_defer);
    }
    if (STATS && a.pstat) {  // one row per shard: 16 workgroups per address
      uint32_t* ps = a.pstat + (uint64_t)shard * kPsWords;
      atomicAdd(&ps[kPsVisited], (uint32_t)s_visits);
      atomicAdd(&ps[kPsColour], s_ps[0]);
      atomicAdd(&ps[kPsKey], (uint32_t)s_defer - s_ps[0]);
      atomicAdd(&ps[kPsCapped], s_ps[1]);
      atomicAdd(&ps[kPsDeadline], s_ps[2]);
      atomicMax(&ps[kPsRadiusMax], s_ps[3]);
      atomicAdd(&ps[kPsSweeps], (uint32_t)s_sweeps);
      atomicMax(&ps[kPsRadiusMin], s_psmin);
      atomicAdd(&ps[kPsEnqueued], s_nq);
    }
  }
  if (tid < kBins && s_hout[tid]) atomicAdd(&a.hist_out[shard * kBins + tid], s_hout[tid]);
  __syncthreads();
  for (uint32_t k = tid; k < nq; k += blockDim.x)
    a.list_out[(uint64_t)shard * a.shard_cap + s_base + k] = s_q[k];
  if (trace && tid == 0) {
    trace[4] = __builtin_amdgcn_s_memrealtime();
    const uint32_t mine = n_active > blockIdx.x ? (n_active - blockIdx.x - 1) / nb + 1 : 0u;
    trace[5] = ((unsigned long long)mine << 32) | (unsigned long long)s_visits;
  }
}

// Priority-pass state for a new solve: every key +inf, histograms zero, list-0
// origin 0, bin width delta = kappa * mean finite F over a strided sample.
__global__ void k_prio_init(const double* F, int64_t ld, int64_t nx, int64_t ny,
                            unsigned long long* keys, uint64_t nkeys, uint32_t* hist,
                            uint64_t nhist, unsigned long long* minkey, double* base,
                            double* delta, double kappa) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys;
       k += (uint64_t)gridDim.x * blockDim.x)
    keys[k] = kInfBits;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nhist;
       k += (uint64_t)gridDim.x * blockDim.x)
    hist[k] = 0u;
  if (blockIdx.x == 0) {  // blockDim.x == 256
    __shared__ double s_sum[256];
    __shared__ uint32_t s_cnt[256];
    __shared__ int64_t s_row[256];
    // sample: up to 256 rows spread over the grid, from each a contiguous segment of
    // up to 256 cells at a row-dependent offset (thread t reads cell t of every
    // segment: coalesced, one page per row, 16 rows in flight).  The former scattered
    // 1-D sample (a page walk per load) took ~250 us of dependent latency.
    const int64_t sr = ny < 256 ? ny : 256, sc = nx < 256 ? nx : 256;
    if ((int64_t)threadIdx.x < sr) {
      const int64_t j = ((int64_t)threadIdx.x * ny) / sr;
      const int64_t i0 = (((int64_t)threadIdx.x * 97) % 256) * (nx - sc) / 255;
      s_row[threadIdx.x] = j * ld + i0;
    }
    __syncthreads();
    double sum = 0.0;
    uint32_t cnt = 0;
    if ((int64_t)threadIdx.x < sc) {
      for (int64_t a0 = 0; a0 < sr; a0 += 16) {
        double f[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) f[u] = a0 + u < sr ? F[s_row[a0 + u] + threadIdx.x] : dinf();
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (f[u] < dinf()) {
            sum += f[u];
            ++cnt;
          }
      }
    }
    s_sum[threadIdx.x] = sum;
    s_cnt[threadIdx.x] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      uint32_t c = 0;
      for (int k = 0; k < (int)blockDim.x; ++k) {
        s += s_sum[k];
        c += s_cnt[k];
      }
      const double mean = c ? s / (double)c : 1.0;
      *delta = (mean > 0.0 && mean < dinf()) ? kappa * mean : 1.0;
      for (int k = 0; k < 3; ++k) {
        minkey[k] = kInfBits;
        base[k] = 0.0;
      }
    }
  }
}

// The goal tile (or a re-seeded tile) enters list 0 with key keyv, bin 0.
__global__ void k_prio_seed(unsigned long long* key0, uint32_t* hist0, unsigned long long* minkey0,
                            uint32_t tile, double keyv) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    key0[tile] = dbits(keyv);
    hist0[0] += 1u;
    *minkey0 = dbits(keyv);
  }
}

// ---------------------------------------------------------------------------
// Sharded (row-slab) mode: merge freshly received neighbour rows into the
// ghost rows (values only decrease, so a min-merge) and seed the tiles of the
// first / last tile row under every column that improved, into the list the
// next pass reads.  Also used by the single-GPU virtual-slab tests.
// ---------------------------------------------------------------------------
struct MergeArgs {
  double* T;
  int64_t ld, nx, nrows;
  int ntx, nty, tile_w;
  uint32_t* list;
  uint32_t* counts;
  uint32_t cap;
  uint32_t* tile_epoch;
  uint32_t epoch;
  unsigned long long* keys;
  uint32_t* hist;
  unsigned long long* minkey;
  const double* base;
  const double* delta;
};

// blocks of 256 threads start at multiples of 256 columns and tile_w divides
// 64, so a tile's columns are tile_w consecutive lanes of one wave.
__device__ __forceinline__ void merge_rows(const MergeArgs& g, const double* new_lo,
                                           const double* new_hi) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const uint32_t shard = blockIdx.x % kShards;
  const unsigned long long tmask = g.tile_w >= 64 ? ~0ull : ((1ull << g.tile_w) - 1ull);
  for (int side = 0; side < 2; ++side) {
    const double* src = side == 0 ? new_lo : new_hi;
    if (!src) continue;  // uniform
    bool seed = false;
    double v = dinf();
    if (k < g.nx) {
      double* gh = g.T + (side == 0 ? -g.ld : g.nrows * g.ld) + k;
      v = src[k];
      if (v < *gh) {
        *gh = v;
        seed = true;
      }
    }
    const unsigned long long m = __ballot(seed);
    const uint32_t tile = (uint32_t)((side == 0 ? 0 : g.nty - 1) * (int64_t)g.ntx + k / g.tile_w);
    if (g.keys) {  // v4: key = min improved ghost value under the tile
      if (seed) atomicMin(&g.keys[tile], dbits(v));
      double wm = seed ? v : dinf();
      for (int o = 32; o > 0; o >>= 1) wm = vmin64(wm, __shfl_xor(wm, o));
      if (lane == 0 && wm < dinf()) atomicMin(g.minkey, dbits(wm));
    }
    if (k < g.nx && (k % g.tile_w) == 0 && ((m >> lane) & tmask)) {
      if (atomicMax(&g.tile_epoch[tile], g.epoch) < g.epoch) {
        const uint32_t pos = atomicAdd(&g.counts[shard], 1u);
        g.list[(uint64_t)shard * g.cap + pos] = tile;
        if (g.keys) {
          const double kv = bitsd(g.keys[tile]);
          atomicAdd(&g.hist[shard * kBins + key_bin(kv, *g.base, 1.0 / *g.delta)], 1u);
        }
      }
    }
  }
}

__global__ void k_merge_ghosts(MergeArgs g, const double* new_lo, const double* new_hi) {
  merge_rows(g, new_lo, new_hi);
}

// One launch per round of the native sharded loop (dymu_dist.cpp): merge the
// received rows, then the last block to finish writes *total = the number of
// tiles queued for the next pass (k_merge_ghosts + k_sum_counts fused; the
// per-round launch count is what a short round pays for).  *ticket is reset.
__global__ void k_exchange(MergeArgs g, const double* new_lo, const double* new_hi,
                           uint32_t* ticket, int32_t* total) {
  merge_rows(g, new_lo, new_hi);
  __shared__ bool s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && threadIdx.x < 64) {  // every block's list inserts are in
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    uint32_t c = threadIdx.x < kShards ? atomicAdd(&g.counts[threadIdx.x], 0u) : 0u;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (threadIdx.x == 0) {
      *total = (int32_t)c;
      atomicExch(ticket, 0u);
    }
  }
}

// edge columns (PassArgs::ec) of tiles [t0, t1) from T: one thread per (tile, side, row)
__global__ void k_ec_rebuild(const double* T, uint64_t ld, uint32_t nx, uint32_t ny, double* ec,
                             uint32_t ntx, uint32_t t0, uint32_t t1) {
  const uint64_t n = (uint64_t)(t1 - t0) * 32;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t t = t0 + c / 32;
    const uint32_t k = (uint32_t)(c % 32), side = k / 16, r = k % 16;
    const uint64_t j = (t / ntx) * 16 + r, i = (t % ntx) * 16 + (side ? 15 : 0);
    ec[t * 32 + k] = (i < nx && j < ny) ? T[j * ld + i] : dinf();
  }
}

__global__ void k_sum_counts(const uint32_t* counts, int32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    uint32_t s = 0;
    for (int q = 0; q < kShards; ++q) s += counts[q];
    *out = (int32_t)s;
  }
}

// ---------------------------------------------------------------------------
// Synthetic speed field; k = global row-major index.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
__device__ __forceinline__ double u01(uint64_t seed, uint64_t k) {
  return (double)(splitmix64(seed ^ k) >> 11) * 0x1.0p-53;
}

__global__ void k_synth(double* F, uint64_t ld, uint32_t nx, uint32_t ny, uint64_t row0,
                        uint64_t seed, double frac, uint64_t oseed, int64_t gi, int64_t gj) {
  const uint64_t n = (uint64_t)nx * ny;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = k / nx, cc = k % nx;
    const uint64_t grow = row0 + r;
    const uint64_t gk = grow * nx + cc;
    double v = 1.0 + 4.0 * u01(seed, gk);
    if (frac > 0.0 && u01(oseed, gk) < frac) {
      const int64_t di = (int64_t)cc - gi, dj = (int64_t)grow - gj;
      if (!(di >= -1 && di <= 1 && dj >= -1 && dj <= 1)) v = dinf();
    }
    F[r * ld + cc] = v;
  }
}

// ---------------------------------------------------------------------------
// host-side launch wrappers
// ---------------------------------------------------------------------------
hipError_t launch_fill_inf(double* T, uint64_t ld, uint32_t nx, int64_t row_lo, int64_t row_hi,
                           hipStream_t st) {
  const uint64_t rows = row_hi > row_lo ? (uint64_t)(row_hi - row_lo) : 0;
  if (rows == 0 || nx == 0) return hipSuccess;
  const uint32_t gx = (nx / 2 + 255) / 256 + 1;  // a row per column-block strip (2 cells
                                                // per lane when aligned), ~8192 workgroups
  uint64_t gy = 8192u / gx;
  if (gy < 1) gy = 1;
  if (gy > rows) gy = rows;
  if (gy > 65535) gy = 65535;
  hipLaunchKernelGGL(k_fill_inf, dim3(gx, (unsigned)gy), dim3(256), 0, st, T, ld, nx, row_lo,
                     row_hi);
  return hipGetLastError();
}

hipError_t launch_seed(double* T, uint64_t ld, int64_t gi, int64_t gj, uint32_t* list,
                       uint32_t* count, uint32_t* tile_epoch, uint32_t epoch, uint32_t tile,
                       int set_goal, hipStream_t st) {
  hipLaunchKernelGGL(k_seed, dim3(1), dim3(64), 0, st, T, ld, gi, gj, list, count, tile_epoch,
                     epoch, tile, set_goal);
  return hipGetLastError();
}

hipError_t launch_pass_prio(const PassArgs& a, int blocks, hipStream_t st, hipEvent_t e0,
                            hipEvent_t e1) {
  if (e0 || e1)
    hipExtLaunchKernelGGL(k_fim_pass_prio<8>, dim3(blocks), dim3(256), 0, st, e0, e1, 0, a);
  else
    hipLaunchKernelGGL(k_fim_pass_prio<8>, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <int WPB, bool APPROX, bool STATS = false>
hipError_t launch_dyn_k(const PassArgs& a, int blocks, hipStream_t st, hipEvent_t e0,
                        hipEvent_t e1) {
  if (e0 || e1)
    hipExtLaunchKernelGGL((k_fim_pass_dyn<WPB, APPROX, STATS>), dim3(blocks), dim3(64 * WPB), 0, st, e0,
                          e1, 0, a);
  else
    hipLaunchKernelGGL((k_fim_pass_dyn<WPB, APPROX, STATS>), dim3(blocks), dim3(64 * WPB), 0, st, a);
  return hipGetLastError();
}
// kernel 5: 16-wave workgroups, the sweep sqrt of a.exact_sqrt
hipError_t launch_pass_prio16(const PassArgs& a, int blocks, hipStream_t st, hipEvent_t e0,
                              hipEvent_t e1) {
  if (a.pstat)
    return a.exact_sqrt ? launch_dyn_k<16, false, true>(a, blocks, st, e0, e1)
                        : launch_dyn_k<16, true, true>(a, blocks, st, e0, e1);
  return a.exact_sqrt ? launch_dyn_k<16, false>(a, blocks, st, e0, e1)
                      : launch_dyn_k<16, true>(a, blocks, st, e0, e1);
}

int pass_blocks_per_cu(int variant) {
  int n = 0;
  hipError_t e = hipErrorInvalidValue;
  switch (variant) {
    case 3: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fim_pass_rb, 256, 0); break;
    case 4:
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fim_pass_prio<8>, 256, 0);
      break;
    case 5:
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_fim_pass_dyn<16, true>, 1024, 0);
      break;
    default: break;
  }
  (void)hipGetLastError();
  return (e == hipSuccess && n > 0) ? n : 4;
}

hipError_t launch_prio_init(const double* F, int64_t ld, int64_t nx, int64_t ny,
                            unsigned long long* keys, uint64_t nkeys, uint32_t* hist,
                            uint64_t nhist, unsigned long long* minkey, double* base,
                            double* delta, double kappa, hipStream_t st) {
  uint64_t nb = (nkeys + 255) / 256;
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(k_prio_init, dim3((unsigned)nb), dim3(256), 0, st, F, ld, nx, ny, keys, nkeys,
                     hist, nhist, minkey, base, delta, kappa);
  return hipGetLastError();
}

hipError_t launch_prio_seed(unsigned long long* key0, uint32_t* hist0, unsigned long long* minkey0,
                            uint32_t tile, double keyv, hipStream_t st) {
  hipLaunchKernelGGL(k_prio_seed, dim3(1), dim3(64), 0, st, key0, hist0, minkey0, tile, keyv);
  return hipGetLastError();
}

hipError_t launch_pass_rb(const PassArgs& a, int blocks, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (e0 || e1)  // timestamps taken by the dispatch itself (no extra stream packets)
    hipExtLaunchKernelGGL(k_fim_pass_rb, dim3(blocks), dim3(256), 0, st, e0, e1, 0, a);
  else
    hipLaunchKernelGGL(k_fim_pass_rb, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_eikonal_batch(const double* tx, const double* ty, const double* c, double* out,
                                uint64_t n, int fast, hipStream_t st) {
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return hipSuccess;
  if (fast == 2)
    hipLaunchKernelGGL(k_eikonal_batch<2>, dim3((unsigned)blocks), dim3(256), 0, st, tx, ty, c,
                       out, n);
  else if (fast == 3)
    hipLaunchKernelGGL(k_eikonal_batch<3>, dim3((unsigned)blocks), dim3(256), 0, st, tx, ty, c,
                       out, n);
  else if (fast == 4)
    hipLaunchKernelGGL(k_eikonal_batch<4>, dim3((unsigned)blocks), dim3(256), 0, st, tx, ty, c,
                       out, n);
  else if (fast)
    hipLaunchKernelGGL(k_eikonal_batch<1>, dim3((unsigned)blocks), dim3(256), 0, st, tx, ty, c,
                       out, n);
  else
    hipLaunchKernelGGL(k_eikonal_batch<0>, dim3((unsigned)blocks), dim3(256), 0, st, tx, ty,
                       c, out, n);
  return hipGetLastError();
}

hipError_t launch_merge_ghosts(double* T, int64_t ld, int64_t nx, int64_t nrows,
                               const double* new_lo, const double* new_hi, int ntx, int nty,
                               int tile_w, uint32_t* list, uint32_t* counts, uint32_t cap,
                               uint32_t* tile_epoch, uint32_t epoch, unsigned long long* keys,
                               uint32_t* hist, unsigned long long* minkey, const double* base,
                               const double* delta, hipStream_t st) {
  const unsigned blocks = (unsigned)((nx + 255) / 256);
  if (blocks == 0) return hipSuccess;
  const MergeArgs g{T,    ld,    nx,         nrows, ntx,  nty,    tile_w, list,  counts,
                    cap,  tile_epoch, epoch, keys,  hist, minkey, base,   delta};
  hipLaunchKernelGGL(k_merge_ghosts, dim3(blocks), dim3(256), 0, st, g, new_lo, new_hi);
  return hipGetLastError();
}

hipError_t launch_exchange(double* T, int64_t ld, int64_t nx, int64_t nrows, const double* new_lo,
                           const double* new_hi, int ntx, int nty, int tile_w, uint32_t* list,
                           uint32_t* counts, uint32_t cap, uint32_t* tile_epoch, uint32_t epoch,
                           unsigned long long* keys, uint32_t* hist, unsigned long long* minkey,
                           const double* base, const double* delta, uint32_t* ticket,
                           int32_t* total, hipStream_t st) {
  const unsigned blocks = (unsigned)((nx + 255) / 256);
  if (blocks == 0) return hipErrorInvalidValue;
  const MergeArgs g{T,    ld,    nx,         nrows, ntx,  nty,    tile_w, list,  counts,
                    cap,  tile_epoch, epoch, keys,  hist, minkey, base,   delta};
  hipLaunchKernelGGL(k_exchange, dim3(blocks), dim3(256), 0, st, g, new_lo, new_hi, ticket, total);
  return hipGetLastError();
}

// Deterministic mode: rebuild list p's key histogram from its FINAL keys into
// shard 0's row of `out` (zeroed by the previous pass's rebuild); block (0,0)
// zeroes `zero`, the buffer the next rebuild fills.  Blocks (x, q) take shard q.
__global__ __launch_bounds__(256) void k_rehist(const uint32_t* list, const uint32_t* counts,
                                                uint32_t cap, const unsigned long long* keys,
                                                const double* base, const double* delta,
                                                uint32_t* out, uint32_t* zero) {
  __shared__ uint32_t s_h[kBins];
  const int tid = threadIdx.x;
  const uint32_t q = blockIdx.y;
  if (tid < kBins) s_h[tid] = 0u;
  if (blockIdx.x == 0 && q == 0)
    for (int k = tid; k < kShards * kBins; k += blockDim.x) zero[k] = 0u;
  __syncthreads();
  const uint32_t n = counts[q];
  const double origin = *base, inv = 1.0 / *delta;
  for (uint32_t i = blockIdx.x * blockDim.x + tid; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t t = list[(uint64_t)q * cap + i] & kTileMask;
    atomicAdd(&s_h[key_bin(bitsd(keys[t]), origin, inv)], 1u);
  }
  __syncthreads();
  if (tid < kBins && s_h[tid]) atomicAdd(&out[tid], s_h[tid]);
}

hipError_t launch_rehist(const uint32_t* list, const uint32_t* counts, uint32_t cap,
                         const unsigned long long* keys, const double* base, const double* delta,
                         uint32_t* out, uint32_t* zero, hipStream_t st) {
  hipLaunchKernelGGL(k_rehist, dim3(8, kShards), dim3(256), 0, st, list, counts, cap, keys, base,
                     delta, out, zero);
  return hipGetLastError();
}

hipError_t launch_ec_rebuild(const double* T, uint64_t ld, uint32_t nx, uint32_t ny, double* ec,
                             uint32_t ntx, uint32_t t0, uint32_t t1, hipStream_t st) {
  const uint64_t n = (uint64_t)(t1 - t0) * 32;
  uint64_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  if (b == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ec_rebuild, dim3((unsigned)b), dim3(256), 0, st, T, ld, nx, ny, ec, ntx, t0,
                     t1);
  return hipGetLastError();
}

hipError_t launch_sum_counts(const uint32_t* counts, int32_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_sum_counts, dim3(1), dim3(64), 0, st, counts, out);
  return hipGetLastError();
}

hipError_t launch_synth(double* F, uint64_t ld, uint32_t nx, uint32_t ny, uint64_t row0,
                        uint64_t seed, double frac, uint64_t oseed, int64_t gi, int64_t gj,
                        hipStream_t st) {
  const uint64_t n = (uint64_t)nx * ny;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(256), 0, st, F, ld, nx, ny, row0, seed,
                     frac, oseed, gi, gj);
  return hipGetLastError();
}

}  // namespace dymu
