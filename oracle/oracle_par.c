/*
 * oracle_par.c -- all-cores CPU baseline (SURVEY.md s8(d) "cpu_fim_omp", optional):
 * the reference's fixed point (propagateGlobalNode, src/DyMu_GlobalPathPlanning.cpp
 * :500-546) reached by a block Fast Iterative Method on the host's threads.
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY (see oracle.h): bench.py times it beside
 * the single-thread heap FMM so the GPU number has an all-cores CPU reference too.
 * It is a different schedule of the same update -- like the GPU engine -- so its
 * result equals the FMM's within the same ulps (tests/test_oracle.py checks 1e-12).
 *
 * Tiles of 64 x 64 cells; a pass relaxes every active tile in parallel (OpenMP,
 * dynamic schedule) with a fast-marching solve inside the tile, warm-started from
 * its current values and the halo; a tile whose edge cells decreased activates
 * the neighbour across that edge for the next pass.
 * Concurrent tiles read each other's edge cells while they change: every value
 * ever written is a valid upper bound (values only decrease), and a change made
 * after a neighbour read it re-activates that neighbour, so the passes end at the
 * fixed point.  Shared cells are read and written with relaxed 64-bit atomics
 * (plain moves on x86-64), so the races are defined behaviour.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PB 64 /* tile edge */

static inline double ld_relaxed(const double* p) {
  uint64_t b = __atomic_load_n((const uint64_t*)p, __ATOMIC_RELAXED);
  double v;
  memcpy(&v, &b, sizeof v);
  return v;
}

static inline void st_relaxed(double* p, double v) {
  uint64_t b;
  memcpy(&b, &v, sizeof b);
  __atomic_store_n((uint64_t*)p, b, __ATOMIC_RELAXED);
}

/* :504-535 (pow(x, 2.0) == x * x; no contraction) */
static inline double upd(double tx, double ty, double c) {
  if ((fabs(tx - ty) < c) && (tx < INFINITY) && (ty < INFINITY))
    return (tx + ty + sqrt(2 * (c * c) - (tx - ty) * (tx - ty))) / 2;
  return fmin(tx, ty) + c;
}

/* Per-thread work space of a tile solve: the image with its halo, a binary heap
 * of (value, cell) and each cell's position in it. */
typedef struct {
  double* L;
  double* hv;
  int* hc;
  int* pos;
} Work;

static void heap_up(Work* w, int k) {
  while (k > 0) {
    const int p = (k - 1) / 2;
    if (!(w->hv[k] < w->hv[p])) break;
    double tv = w->hv[k];
    int tc = w->hc[k];
    w->hv[k] = w->hv[p], w->hc[k] = w->hc[p];
    w->hv[p] = tv, w->hc[p] = tc;
    w->pos[w->hc[k]] = k, w->pos[w->hc[p]] = p;
    k = p;
  }
}

static void heap_down(Work* w, int n, int k) {
  for (;;) {
    const int l = 2 * k + 1, r = l + 1;
    int m = k;
    if (l < n && w->hv[l] < w->hv[m]) m = l;
    if (r < n && w->hv[r] < w->hv[m]) m = r;
    if (m == k) break;
    double tv = w->hv[k];
    int tc = w->hc[k];
    w->hv[k] = w->hv[m], w->hc[k] = w->hc[m];
    w->hv[m] = tv, w->hc[m] = tc;
    w->pos[w->hc[k]] = k, w->pos[w->hc[m]] = m;
    k = m;
  }
}

/* relax tile (bx, by) to its exact fixed point given the halo: a fast-marching
 * solve inside the tile, warm-started from the current values (every finite cell
 * is a tentative value; a popped value is final because later updates come from
 * values that are not smaller, :500-546).  Returns a 4-bit mask of the edges
 * whose cells decreased (1 S, 2 W, 4 E, 8 N). */
static int relax_tile(const double* F, double* T, uint32_t nx, uint32_t ny, uint32_t gi,
                      uint32_t gj, uint32_t bx, uint32_t by, Work* w) {
  const int64_t i0 = (int64_t)bx * PB, j0 = (int64_t)by * PB;
  const int tw = (int)((i0 + PB <= nx) ? PB : nx - i0), th = (int)((j0 + PB <= ny) ? PB : ny - j0);
  const int P = PB + 2;
  double* L = w->L;
  for (int r = -1; r <= th; ++r)
    for (int c = -1; c <= tw; ++c) {
      const int64_t i = i0 + c, j = j0 + r;
      const int in = i >= 0 && j >= 0 && i < nx && j < ny;
      L[(r + 1) * P + (c + 1)] = in ? ld_relaxed(&T[j * nx + i]) : INFINITY;
    }
  /* tentative values: the current ones, lowered by one update from the image */
  int n = 0;
  for (int r = 0; r < th; ++r)
    for (int c = 0; c < tw; ++c) {
      const int64_t i = i0 + c, j = j0 + r;
      const int s = (r + 1) * P + (c + 1);
      w->pos[s] = -1;
      const double f = F[j * nx + i];
      if (!(f < INFINITY)) continue;
      if (!(i == gi && j == gj)) {
        const double v = upd(fmin(L[s - 1], L[s + 1]), fmin(L[s - P], L[s + P]), f);
        if (v < L[s]) L[s] = v;
      }
      if (L[s] < INFINITY) {
        w->hv[n] = L[s], w->hc[n] = s, w->pos[s] = n;
        heap_up(w, n++);
      }
    }
  while (n > 0) {
    const int s = w->hc[0];
    w->pos[s] = -2;  /* final */
    --n;
    if (n > 0) {
      w->hv[0] = w->hv[n], w->hc[0] = w->hc[n], w->pos[w->hc[0]] = 0;
      heap_down(w, n, 0);
    }
    const int nb[4] = {s - P, s - 1, s + 1, s + P};
    for (int q = 0; q < 4; ++q) {
      const int x = nb[q];
      const int r = x / P - 1, c = x % P - 1;
      if (r < 0 || c < 0 || r >= th || c >= tw || w->pos[x] == -2) continue;
      const int64_t i = i0 + c, j = j0 + r;
      const double f = F[j * nx + i];
      if (!(f < INFINITY) || (i == gi && j == gj)) continue;
      const double v = upd(fmin(L[x - 1], L[x + 1]), fmin(L[x - P], L[x + P]), f);
      if (!(v < L[x])) continue;
      L[x] = v;
      if (w->pos[x] < 0) {
        w->hv[n] = v, w->hc[n] = x, w->pos[x] = n;
        heap_up(w, n++);
      } else {
        w->hv[w->pos[x]] = v;
        heap_up(w, w->pos[x]);
      }
    }
  }
  int mask = 0;
  for (int r = 0; r < th; ++r)
    for (int c = 0; c < tw; ++c) {
      const int64_t k = (j0 + r) * (int64_t)nx + (i0 + c);
      const double v = L[(r + 1) * P + (c + 1)];
      if (v < ld_relaxed(&T[k])) {
        st_relaxed(&T[k], v);
        if (r == 0) mask |= 1;
        if (c == 0) mask |= 2;
        if (c == tw - 1) mask |= 4;
        if (r == th - 1) mask |= 8;
      }
    }
  return mask;
}

int oracle_fim_parallel(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                        double* T, int threads, uint64_t* passes_out) {
  if (!F || !T || nx == 0 || ny == 0 || gi >= nx || gj >= ny) return -1;
  const uint64_t n = (uint64_t)nx * ny;
  const uint32_t tx = (nx + PB - 1) / PB, ty = (ny + PB - 1) / PB;
  const uint64_t nt = (uint64_t)tx * ty;
  uint8_t* act = calloc(nt, 1);
  uint8_t* nxt = calloc(nt, 1);
  uint32_t* list = malloc(sizeof(uint32_t) * nt);
  if (!act || !nxt || !list) {
    free(act), free(nxt), free(list);
    return -1;
  }
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
  for (uint64_t k = 0; k < n; ++k) T[k] = INFINITY;
  T[(uint64_t)gj * nx + gi] = 0.0;
  act[(gj / PB) * tx + gi / PB] = 1;
  uint64_t passes = 0;
  for (;;) {
    uint64_t m = 0;
    for (uint64_t t = 0; t < nt; ++t)
      if (act[t]) list[m++] = (uint32_t)t;
    if (m == 0) break;
    ++passes;
    memset(nxt, 0, nt);
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
    {
      Work wk;
      wk.L = malloc(sizeof(double) * (PB + 2) * (PB + 2));
      wk.hv = malloc(sizeof(double) * PB * PB);
      wk.hc = malloc(sizeof(int) * PB * PB);
      wk.pos = malloc(sizeof(int) * (PB + 2) * (PB + 2));
#pragma omp for schedule(dynamic, 1)
      for (uint64_t q = 0; q < m; ++q) {
        const uint32_t t = list[q], bx = t % tx, by = t / tx;
        const int mk = relax_tile(F, T, nx, ny, gi, gj, bx, by, &wk);
        if ((mk & 1) && by > 0) __atomic_store_n(&nxt[t - tx], 1, __ATOMIC_RELAXED);
        if ((mk & 2) && bx > 0) __atomic_store_n(&nxt[t - 1], 1, __ATOMIC_RELAXED);
        if ((mk & 4) && bx + 1 < tx) __atomic_store_n(&nxt[t + 1], 1, __ATOMIC_RELAXED);
        if ((mk & 8) && by + 1 < ty) __atomic_store_n(&nxt[t + tx], 1, __ATOMIC_RELAXED);
      }
      free(wk.L), free(wk.hv), free(wk.hc), free(wk.pos);
    }
    uint8_t* s = act;
    act = nxt;
    nxt = s;
  }
  free(act), free(nxt), free(list);
  if (passes_out) *passes_out = passes;
  return 0;
}
