/*
 * host_engine.c -- TEST DOUBLE of the engine C-ABI (include/dymu_fim.h) over host
 * memory, for CPU tests of the planner's host logic (tests/test_host_engine.py).
 * "Device" buffers are malloc'd, copies are memcpy, and a solve is the oracle's
 * heap FMM (oracle/oracle.c).  Never part of the product: the product links the
 * HIP engine (libdymu_fim.so), which has no CPU path.
 *
 * Fault injection: HOST_ENGINE_FAIL_D2H=n makes the n-th device-to-host copy
 * (1-based, dymu_memcpy_d2h and dymu_memcpy2d_d2h together) fail with
 * DYMU_ERR_ARG and NO error text -- the failure the planner must not mistake for
 * success (streamTotalCost keyed its failure flag on the text).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "dymu_fim.h"
#include "oracle.h"

struct dymu_ctx {
  int dummy;
};

static long g_d2h_calls = 0;

static int d2h_fails(void) {
  const char* kv = getenv("HOST_ENGINE_FAIL_D2H");
  ++g_d2h_calls;
  return kv && atol(kv) == g_d2h_calls;
}

int dymu_create(dymu_ctx** out, const dymu_opts* o) {
  (void)o;
  if (!out) return DYMU_ERR_ARG;
  *out = (dymu_ctx*)calloc(1, sizeof(dymu_ctx));
  return *out ? DYMU_OK : DYMU_ERR_NOMEM;
}
int dymu_destroy(dymu_ctx* c) {
  free(c);
  return DYMU_OK;
}
const char* dymu_strerror(int rc) { return rc ? "host engine error" : "ok"; }
const char* dymu_last_error(dymu_ctx* c) {
  (void)c;
  return "";
}
int dymu_device_alloc(dymu_ctx* c, size_t n, void** p) {
  if (!c || !p) return DYMU_ERR_ARG;
  *p = malloc(n ? n : 1);
  return *p ? DYMU_OK : DYMU_ERR_NOMEM;
}
int dymu_device_free(dymu_ctx* c, void* p) {
  if (!c) return DYMU_ERR_ARG;
  free(p);
  return DYMU_OK;
}
int dymu_host_register(dymu_ctx* c, void* p, size_t n) {
  (void)p, (void)n;
  return c ? DYMU_OK : DYMU_ERR_ARG;
}
int dymu_host_unregister(dymu_ctx* c, void* p) {
  (void)p;
  return c ? DYMU_OK : DYMU_ERR_ARG;
}
int dymu_memcpy_d2h(dymu_ctx* c, void* d, const void* s, size_t n) {
  if (!c || d2h_fails()) return DYMU_ERR_ARG;
  memcpy(d, s, n);
  return DYMU_OK;
}
int dymu_memcpy_h2d(dymu_ctx* c, void* d, const void* s, size_t n) {
  if (!c) return DYMU_ERR_ARG;
  memcpy(d, s, n);
  return DYMU_OK;
}
int dymu_memcpy2d_d2h(dymu_ctx* c, void* d, size_t dp, const void* s, size_t sp, size_t w,
                      size_t h) {
  if (!c || d2h_fails()) return DYMU_ERR_ARG;
  for (size_t r = 0; r < h; ++r) memcpy((char*)d + r * dp, (const char*)s + r * sp, w);
  return DYMU_OK;
}

static int solve(const double* F, double* T, uint32_t nx, uint32_t ny, uint64_t ld, uint32_t gi,
                 uint32_t gj, int64_t si, int64_t sj, double* tc, dymu_stats* st) {
  if (ld != nx) return DYMU_ERR_ARG;
  uint64_t pops = 0;
  const int rc = oracle_fmm_heap(F, nx, ny, gi, gj, -1, -1, T, NULL, &pops);
  if (rc < 0) return DYMU_ERR_ARG;
  if (tc) {  /* whole map converged: every cell is final */
    double m = 0;
    const int64_t p[5][2] = {{si, sj}, {si, sj - 1}, {si - 1, sj}, {si + 1, sj}, {si, sj + 1}};
    for (int k = 0; k < 5; ++k)
      if (p[k][0] >= 0 && p[k][1] >= 0 && p[k][0] < nx && p[k][1] < ny) {
        const double v = T[p[k][1] * (int64_t)nx + p[k][0]];
        if (v > m) m = v;
      }
    *tc = m;
  }
  if (st) {
    memset(st, 0, sizeof *st);
    st->passes = pops;
    st->tile_w = st->tile_h = 1;
  }
  return DYMU_OK;
}

int dymu_solve_device(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny, uint64_t ld,
                      uint32_t gi, uint32_t gj, void* s, dymu_stats* st) {
  (void)s;
  if (!c) return DYMU_ERR_ARG;
  return solve(F, T, nx, ny, ld, gi, gj, -1, -1, NULL, st);
}
int dymu_solve_until_device(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny,
                            uint64_t ld, uint32_t gi, uint32_t gj, uint32_t si, uint32_t sj, void* s,
                            double* tc, dymu_stats* st) {
  (void)s;
  if (!c || !tc) return DYMU_ERR_ARG;
  return solve(F, T, nx, ny, ld, gi, gj, si, sj, tc, st);
}
int dymu_early_exit_mask(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny,
                         uint64_t ld, double tc, uint64_t* b, uint64_t cap, uint64_t* nb, void* s) {
  (void)s;
  if (!c || !nb) return DYMU_ERR_ARG;
  uint64_t n = 0;
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) {
      const uint64_t k = (uint64_t)j * ld + i;
      if (T[k] <= tc) continue;
      int band = 0;
      if (F[k] < INFINITY)
        band = (j > 0 && T[k - ld] <= tc) || (i > 0 && T[k - 1] <= tc) ||
               (i + 1 < nx && T[k + 1] <= tc) || (j + 1 < ny && T[k + ld] <= tc);
      if (band) {
        if (n < cap) b[n] = (uint64_t)j * nx + i;
        ++n;
      } else {
        T[k] = INFINITY;
      }
    }
  *nb = n;
  return DYMU_OK;
}
int dymu_count_equal(dymu_ctx* c, const double* T, uint32_t nx, uint32_t ny, uint64_t ld,
                     double v, uint64_t* count, void* s) {
  (void)s;
  if (!c || !count) return DYMU_ERR_ARG;
  uint64_t n = 0;
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) n += memcmp(&T[(uint64_t)j * ld + i], &v, sizeof v) == 0;
  *count = n;
  return DYMU_OK;
}
int dymu_find_equal(dymu_ctx* c, const double* T, uint32_t nx, uint32_t ny, uint64_t ld,
                    double v, uint64_t* idx, uint64_t cap, uint64_t* count, void* s) {
  (void)s;
  if (!c || !count || (cap && !idx)) return DYMU_ERR_ARG;
  uint64_t n = 0;
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i)
      if (memcmp(&T[(uint64_t)j * ld + i], &v, sizeof v) == 0) {
        if (n < cap) idx[n] = (uint64_t)j * nx + i;
        ++n;
      }
  *count = n;
  return DYMU_OK;
}
int dymu_region_stats(dymu_ctx* c, const double* F, const double* T, uint32_t nx, uint32_t ny,
                      uint64_t ld, uint32_t gi, uint32_t gj, double thr, double lo, double hi,
                      dymu_region* out, void* s) {
  (void)s;
  if (!c || !out || gi >= nx || gj >= ny) return DYMU_ERR_ARG;
  memset(out, 0, sizeof *out);
  uint32_t mi = UINT32_MAX, mj = UINT32_MAX, xi = 0, xj = 0;
  const double f0 = F[(uint64_t)gj * ld + gi];
  double d2 = INFINITY;
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) {
      const double t = T[(uint64_t)j * ld + i];
      if (t <= thr) {
        mi = i < mi ? i : mi;
        mj = j < mj ? j : mj;
        xi = i > xi ? i : xi;
        xj = j > xj ? j : xj;
      }
      out->n_range += t >= lo && t <= hi;
      if (F[(uint64_t)j * ld + i] != f0) {
        const double di = (double)i - gi, dj = (double)j - gj;
        d2 = di * di + dj * dj < d2 ? di * di + dj * dj : d2;
      }
    }
  out->r_const = sqrt(d2);
  if (mi == UINT32_MAX) {
    out->i0 = 1;
    return DYMU_OK;
  }
  out->i0 = mi, out->j0 = mj, out->i1 = xi, out->j1 = xj;
  if (getenv("HOST_ENGINE_SHORT_REGION")) {  // a box short of the region: the exact replay
    out->i0 = out->i1 = gi;                   // must notice and restart on the whole grid
    out->j0 = out->j1 = gj;
  }
  return DYMU_OK;
}
int dymu_scatter(dymu_ctx* c, double* T, uint32_t nx, uint64_t ld, const uint64_t* idx,
                 const double* v, uint64_t n, void* s) {
  (void)s;
  if (!c) return DYMU_ERR_ARG;
  for (uint64_t q = 0; q < n; ++q) T[(idx[q] / nx) * ld + idx[q] % nx] = v[q];
  return DYMU_OK;
}
int dymu_update_window_device(dymu_ctx* c, const double* F, double* T, uint32_t nx, uint32_t ny,
                              uint64_t ld, uint32_t gi, uint32_t gj, uint32_t i0, uint32_t j0,
                              uint32_t w, uint32_t h, int dec, void* s, dymu_stats* st) {
  (void)i0, (void)j0, (void)w, (void)h, (void)dec, (void)s;
  if (!c) return DYMU_ERR_ARG;
  return solve(F, T, nx, ny, ld, gi, gj, -1, -1, NULL, st);
}
