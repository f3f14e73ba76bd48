/*
 * oracle.c -- CPU restatement of the DyMu global total-cost propagation.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Compiled with -O2
 * -ffp-contract=off so every floating-point operation rounds exactly where
 * the reference's (x86-64 SSE2, no FMA) build rounds.
 *
 * Reference: /root/reference/src/DyMu_GlobalPathPlanning.cpp (cited as :LINE).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define INF_D (__builtin_inf())

/* ------------------------------------------------------------------ */
/* input generators                                                     */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t mt[312];
  int idx;
} mt64_t;

static void mt64_seed(mt64_t* s, uint64_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < 312; ++i)
    s->mt[i] = 6364136223846793005ULL * (s->mt[i - 1] ^ (s->mt[i - 1] >> 62)) + (uint64_t)i;
  s->idx = 312;
}

static uint64_t mt64_next(mt64_t* s) {
  static const uint64_t UM = 0xFFFFFFFF80000000ULL, LM = 0x7FFFFFFFULL;
  if (s->idx >= 312) {
    for (int i = 0; i < 312; ++i) {
      uint64_t x = (s->mt[i] & UM) | (s->mt[(i + 1) % 312] & LM);
      uint64_t xa = x >> 1;
      if (x & 1ULL) xa ^= 0xB5026F5AA96619E9ULL;
      s->mt[i] = s->mt[(i + 156) % 312] ^ xa;
    }
    s->idx = 0;
  }
  uint64_t y = s->mt[s->idx++];
  y ^= (y >> 29) & 0x5555555555555555ULL;
  y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
  y ^= (y << 37) & 0xFFF7EEE000000000ULL;
  y ^= (y >> 43);
  return y;
}

void oracle_fill_mt19937_uniform(double* out, uint64_t n, uint64_t seed, double lo, double hi) {
  mt64_t s;
  mt64_seed(&s, seed);
  const double r = 18446744073709551616.0; /* 2^64: libstdc++ generate_canonical, k = 1 */
  for (uint64_t k = 0; k < n; ++k) {
    double u = (double)mt64_next(&s) / r;
    if (u >= 1.0) u = nextafter(1.0, 0.0);
    out[k] = u * (hi - lo) + lo;
  }
}

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

double oracle_u01(uint64_t seed, uint64_t idx) {
  return (double)(splitmix64(seed ^ idx) >> 11) * 0x1.0p-53;
}

void oracle_fill_u01(double* out, uint64_t n, uint64_t seed) {
  for (uint64_t k = 0; k < n; ++k) out[k] = oracle_u01(seed, k);
}

/* ------------------------------------------------------------------ */
/* per-node speed and cost-map ingestion                               */
/* ------------------------------------------------------------------ */
/* :527-528  C = global_res * cost * (2 + hazard_density - trafficability) */
void oracle_pack_speed(const double* cost, const double* hazard, const double* traff,
                       const uint8_t* is_obstacle, uint64_t n, double res, double* F) {
  for (uint64_t k = 0; k < n; ++k) {
    if (is_obstacle && is_obstacle[k]) {
      F[k] = INF_D;
      continue;
    }
    double hd = hazard ? hazard[k] : 0.0;
    double tr = traff ? traff[k] : 1.0;
    F[k] = res * cost[k] * (2 + hd - tr);
  }
}

/* :109-126 */
void oracle_set_cost_map(const double* cost_map, uint64_t n, double* cost, uint8_t* is_obstacle,
                         double* traff, double* hazard) {
  for (uint64_t k = 0; k < n; ++k) {
    double c = cost_map[k];
    cost[k] = c;
    if (c <= 0) {
      is_obstacle[k] = 1;
      traff[k] = 0.0;
      hazard[k] = 1.0;
    }
  }
}

/* :186-210 calculateSlope.  Off-grid neighbour => one-sided difference. */
static double calc_slope(const double* E, uint32_t nx, uint32_t ny, uint32_t i, uint32_t j,
                         double res) {
  uint64_t k = (uint64_t)j * nx + i;
  double dx, dy;
  if (i == 0)
    dx = (E[k + 1] - E[k]) / res;
  else if (i == nx - 1)
    dx = (E[k] - E[k - 1]) / res;
  else
    dx = (E[k + 1] - E[k - 1]) * 0.5 / res;
  if (j == 0)
    dy = (E[k + nx] - E[k]) / res;
  else if (j == ny - 1)
    dy = (E[k] - E[k - nx]) / res;
  else
    dy = (E[k + nx] - E[k - nx]) * 0.5 / res;
  return atan(sqrt(dx * dx + dy * dy));
}

static double lut_max(const double* lut, int n) {
  /* :221 std::max_element */
  double m = lut[0];
  for (int i = 1; i < n; ++i)
    if (m < lut[i]) m = lut[i];
  return m;
}

/* :217-293 calculateNominalCost, incl. Q2 (mode 0 skipped when n_locs>1),
 * Q3 (dead neighbour loops omitted: they never execute), Q4 (LUT indexing). */
static void nominal_cost(uint64_t k, double cmax, const double* lut, const double* slopes,
                         int n_slopes, int n_locs, double* raw_cost, const double* slope,
                         const uint32_t* terrain, uint8_t* is_obstacle, int32_t* loc_mode) {
  const uint32_t t = terrain[k];
  if (t == 0) { /* :224-234 */
    raw_cost[k] = cmax;
    is_obstacle[k] = 1;
  } else if (n_slopes == 1) { /* :235-244 */
    double cdef = lut[t * n_locs];
    for (int i = 0; i < n_locs; ++i) {
      double cc = lut[t * n_locs + i];
      if (cc < cdef) cdef = cc;
    }
    raw_cost[k] = raw_cost[k] > cdef ? raw_cost[k] : cdef; /* std::max */
  } else {                                                 /* :245-292 */
    double si = slope[k] * 180 / M_PI / (slopes[n_slopes - 1] - slopes[0]) *
                (double)(uint64_t)(n_slopes - 1);
    if (si > (double)(uint64_t)(n_slopes - 1)) {
      raw_cost[k] = cmax;
      is_obstacle[k] = 1;
    } else {
      double smin = floor(si), smax = ceil(si);
      double cdef = cmax;
      if (n_locs > 1) {
        for (int i = 1; i < n_locs; ++i) {
          double c1 = lut[t * n_slopes * n_locs + i * n_slopes + (int)smin];
          double c2 = lut[t * n_slopes * n_locs + i * n_slopes + (int)smax];
          double cc = c1 + (c2 - c1) * (si - smin);
          if (cc < cdef) {
            cdef = cc;
            raw_cost[k] = raw_cost[k] > cdef ? raw_cost[k] : cdef;
            loc_mode[k] = i;
          }
        }
      } else {
        double c1 = lut[t * n_slopes + (int)smin];
        double c2 = lut[t * n_slopes + (int)smax];
        cdef = c1 + (c2 - c1) * (si - smin);
        raw_cost[k] = raw_cost[k] > cdef ? raw_cost[k] : cdef;
        loc_mode[k] = 0;
      }
    }
  }
}

/* :145-181 computeCostMap (+ :297-308 smoothCost, Q1). */
void oracle_compute_cost_map(uint32_t nx, uint32_t ny, double res, const double* lut, int lut_len,
                             const double* slopes, int n_slopes, int n_locs,
                             const double* elevation, const double* terrain_map, double* raw_cost,
                             double* cost, double* slope, uint32_t* terrain,
                             uint8_t* is_obstacle, double* traff, double* hazard,
                             int32_t* loc_mode) {
  const double cmax = lut_max(lut, lut_len);
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) {
      uint64_t k = (uint64_t)j * nx + i;
      raw_cost[k] = 0;
      if (i == 0 || j == 0 || i == nx - 1 || j == ny - 1)
        terrain[k] = 0; /* :162-163 borders are obstacles */
      else
        terrain[k] = (uint32_t)terrain_map[k];
    }
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) {
      uint64_t k = (uint64_t)j * nx + i;
      slope[k] = calc_slope(elevation, nx, ny, i, j, res);
      nominal_cost(k, cmax, lut, slopes, n_slopes, n_locs, raw_cost, slope, terrain, is_obstacle,
                   loc_mode);
      if (is_obstacle[k]) {
        traff[k] = 0.0;
        hazard[k] = 1.0;
      }
    }
  /* smoothCost reads neighbours' raw_cost only, so the row-major in-place
   * order of :178-179 is order-independent; cost starts from the node's
   * previous cost (Q1). */
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) {
      uint64_t k = (uint64_t)j * nx + i;
      double csum = cost[k], n = 5;
      if (j == 0) n--; else csum += raw_cost[k - nx];          /* nb4[0] */
      if (i == 0) n--; else csum += raw_cost[k - 1];           /* nb4[1] */
      if (i == nx - 1) n--; else csum += raw_cost[k + 1];      /* nb4[2] */
      if (j == ny - 1) n--; else csum += raw_cost[k + nx];     /* nb4[3] */
      cost[k] = csum / n;
    }
}

/* :322-357 setGoal */
int oracle_set_goal(uint32_t nx, uint32_t ny, double res, double offx, double offy, double wx,
                    double wy, const uint8_t* is_obstacle, uint32_t* gi, uint32_t* gj) {
  double px = (wx - offx) / res, py = (wy - offy) / res;
  if (px < 0 || py < 0) return 0;
  uint32_t i = (uint32_t)(px + 0.5), j = (uint32_t)(py + 0.5);
  if (i >= nx || j >= ny) return 0;
  /* any nb4 NULL (border) => reject */
  if (i == 0 || j == 0 || i + 1 >= nx || j + 1 >= ny) return 0;
  if (is_obstacle) {
    uint64_t k = (uint64_t)j * nx + i;
    if (is_obstacle[k] || is_obstacle[k - nx] || is_obstacle[k - 1] || is_obstacle[k + 1] ||
        is_obstacle[k + nx])
      return 0;
  }
  *gi = i;
  *gj = j;
  return 1;
}

/* ------------------------------------------------------------------ */
/* the Eikonal update  (:500-546)                                       */
/* ------------------------------------------------------------------ */
double oracle_eikonal(double Tx, double Ty, double C) {
  /* :531-535, pow(x,2.0) == x*x (exact; GCC folds it) */
  if ((fabs(Tx - Ty) < C) && (Tx < INF_D) && (Ty < INF_D))
    return (Tx + Ty + sqrt(2 * (C * C) - ((Tx - Ty) * (Tx - Ty)))) / 2;
  return fmin(Tx, Ty) + C;
}

/* candidate for cell (i,j) from the current T: off-grid neighbours are
 * NULL in the reference and the other one is used alone (:504-523), which is
 * fmin(+inf, x). */
static inline double candidate(const double* F, const double* T, uint32_t nx, uint32_t ny,
                               uint32_t i, uint32_t j) {
  uint64_t k = (uint64_t)j * nx + i;
  double ts = j > 0 ? T[k - nx] : INF_D;
  double tn = j + 1 < ny ? T[k + nx] : INF_D;
  double tw = i > 0 ? T[k - 1] : INF_D;
  double te = i + 1 < nx ? T[k + 1] : INF_D;
  double Ty = fmin(tn, ts); /* :506 fmin(nb4[3], nb4[0]) */
  double Tx = fmin(tw, te); /* :519 fmin(nb4[1], nb4[2]) */
  return oracle_eikonal(Tx, Ty, F[k]);
}

static inline int is_blocked(double f) { return !(f < INF_D); } /* obstacle / +inf / NaN speed */

/* ------------------------------------------------------------------ */
/* FMM, linear band (:364-408, :443-468, :473-496, :551-568)            */
/* ------------------------------------------------------------------ */
static int fully_closed(const uint8_t* closed, uint32_t nx, uint64_t s) {
  /* :424-436 (start validated interior by the caller) */
  return closed[s] && closed[s - nx] && closed[s - 1] && closed[s + 1] && closed[s + nx];
}

static int check_args(uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj, int64_t si,
                      int64_t sj) {
  if (nx == 0 || ny == 0 || gi >= nx || gj >= ny) return 0;
  if (si >= 0 || sj >= 0) {
    if (si < 1 || sj < 1 || si + 1 >= (int64_t)nx || sj + 1 >= (int64_t)ny) return 0;
  }
  return 1;
}

int oracle_fmm_linear(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                      int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                      uint64_t* n_pops) {
  if (!check_args(nx, ny, gi, gj, start_i, start_j)) return -1;
  const uint64_t n = (uint64_t)nx * ny;
  uint8_t* cl = closed ? closed : (uint8_t*)malloc(n);
  uint64_t* band = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  for (uint64_t k = 0; k < n; ++k) {
    T[k] = INF_D;
    cl[k] = 0;
  }
  const int early = start_i >= 0;
  const uint64_t s = early ? (uint64_t)start_j * nx + (uint64_t)start_i : 0;
  const uint64_t g = (uint64_t)gj * nx + gi;
  uint64_t blen = 0, pops = 0;
  band[blen++] = g; /* :490-496 */
  T[g] = 0;
  while (blen > 0 && !(early && fully_closed(cl, nx, s))) {
    /* :551-568 first strict minimum, then erase (order-preserving) */
    uint64_t bi = 0;
    double mc = T[band[0]];
    for (uint64_t b = 0; b < blen; ++b)
      if (T[band[b]] < mc) {
        mc = T[band[b]];
        bi = b;
      }
    uint64_t node = band[bi];
    memmove(band + bi, band + bi + 1, sizeof(uint64_t) * (blen - bi - 1));
    --blen;
    ++pops;
    cl[node] = 1;
    uint32_t i = (uint32_t)(node % nx), j = (uint32_t)(node / nx);
    for (int q = 0; q < 4; ++q) { /* nb4 order :76-80 */
      int64_t ii = i, jj = j;
      if (q == 0) jj = (int64_t)j - 1;
      else if (q == 1) ii = (int64_t)i - 1;
      else if (q == 2) ii = (int64_t)i + 1;
      else jj = (int64_t)j + 1;
      if (ii < 0 || jj < 0 || ii >= nx || jj >= ny) continue;
      uint64_t nb = (uint64_t)jj * nx + (uint64_t)ii;
      if (cl[nb] || is_blocked(F[nb])) continue;
      double tc = candidate(F, T, nx, ny, (uint32_t)ii, (uint32_t)jj);
      if (tc < T[nb]) { /* :537-545 */
        if (T[nb] == INF_D) band[blen++] = nb;
        T[nb] = tc;
      }
    }
  }
  if (n_pops) *n_pops = pops;
  free(band);
  if (!closed) free(cl);
  return blen > 0 ? 1 : 0;
}

/* ------------------------------------------------------------------ */
/* FMM, heap band with the linear scan's exact pop order                */
/* ------------------------------------------------------------------ */
typedef struct {
  double t;
  uint64_t seq;
  uint64_t node;
} hent_t;

static inline int hless(const hent_t* a, const hent_t* b) {
  return a->t < b->t || (a->t == b->t && a->seq < b->seq);
}

typedef struct {
  hent_t* v;
  uint64_t len, cap;
} heap_t;

static void hpush(heap_t* h, hent_t e) {
  if (h->len == h->cap) {
    h->cap = h->cap ? h->cap * 2 : 1024;
    h->v = (hent_t*)realloc(h->v, sizeof(hent_t) * h->cap);
  }
  uint64_t c = h->len++;
  while (c > 0) {
    uint64_t p = (c - 1) / 2;
    if (!hless(&e, &h->v[p])) break;
    h->v[c] = h->v[p];
    c = p;
  }
  h->v[c] = e;
}

static hent_t hpop(heap_t* h) {
  hent_t top = h->v[0], last = h->v[--h->len];
  uint64_t c = 0;
  for (;;) {
    uint64_t l = 2 * c + 1;
    if (l >= h->len) break;
    uint64_t m = (l + 1 < h->len && hless(&h->v[l + 1], &h->v[l])) ? l + 1 : l;
    if (!hless(&h->v[m], &last)) break;
    h->v[c] = h->v[m];
    c = m;
  }
  if (h->len) h->v[c] = last;
  return top;
}

static int fmm_heap(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                    int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                    uint64_t* n_pops, uint64_t* seq_out) {
  if (!check_args(nx, ny, gi, gj, start_i, start_j)) return -1;
  const uint64_t n = (uint64_t)nx * ny;
  uint8_t* cl = closed ? closed : (uint8_t*)malloc(n);
  uint64_t* seq = seq_out ? seq_out : (uint64_t*)malloc(sizeof(uint64_t) * n);
  for (uint64_t k = 0; k < n; ++k) {
    T[k] = INF_D;
    cl[k] = 0;
    seq[k] = UINT64_MAX;
  }
  const int early = start_i >= 0;
  const uint64_t s = early ? (uint64_t)start_j * nx + (uint64_t)start_i : 0;
  const uint64_t g = (uint64_t)gj * nx + gi;
  heap_t h = {0, 0, 0};
  uint64_t next_seq = 0, live = 0, pops = 0;
  seq[g] = next_seq++;
  T[g] = 0;
  live = 1;
  hent_t e0 = {0.0, seq[g], g};
  hpush(&h, e0);
  while (live > 0 && !(early && fully_closed(cl, nx, s))) {
    hent_t e = hpop(&h);
    if (cl[e.node] || e.t != T[e.node]) continue; /* stale entry */
    uint64_t node = e.node;
    --live;
    ++pops;
    cl[node] = 1;
    uint32_t i = (uint32_t)(node % nx), j = (uint32_t)(node / nx);
    for (int q = 0; q < 4; ++q) {
      int64_t ii = i, jj = j;
      if (q == 0) jj = (int64_t)j - 1;
      else if (q == 1) ii = (int64_t)i - 1;
      else if (q == 2) ii = (int64_t)i + 1;
      else jj = (int64_t)j + 1;
      if (ii < 0 || jj < 0 || ii >= nx || jj >= ny) continue;
      uint64_t nb = (uint64_t)jj * nx + (uint64_t)ii;
      if (cl[nb] || is_blocked(F[nb])) continue;
      double tc = candidate(F, T, nx, ny, (uint32_t)ii, (uint32_t)jj);
      if (tc < T[nb]) {
        if (T[nb] == INF_D) {
          seq[nb] = next_seq++;
          ++live;
        }
        T[nb] = tc;
        hent_t en = {tc, seq[nb], nb};
        hpush(&h, en);
      }
    }
  }
  if (n_pops) *n_pops = pops;
  free(h.v);
  if (!seq_out) free(seq);
  if (!closed) free(cl);
  return live > 0 ? 1 : 0;
}

int oracle_fmm_heap(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                    int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                    uint64_t* n_pops) {
  return fmm_heap(F, nx, ny, gi, gj, start_i, start_j, T, closed, n_pops, NULL);
}

/* The same FMM, also returning each node's band-insertion sequence number (the
 * position it takes in global_narrowband / global_propagated_nodes when it first
 * becomes finite, :537-545; the goal 0, :487-498; UINT64_MAX never reached). */
int oracle_fmm_order(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj,
                     int64_t start_i, int64_t start_j, double* T, uint8_t* closed,
                     uint64_t* seq) {
  return fmm_heap(F, nx, ny, gi, gj, start_i, start_j, T, closed, NULL, seq);
}

/* ------------------------------------------------------------------ */
/* Jacobi fixed point and residual                                     */
/* ------------------------------------------------------------------ */
int oracle_jacobi(const double* F, uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj, double* T,
                  int max_sweeps) {
  const uint64_t n = (uint64_t)nx * ny, g = (uint64_t)gj * nx + gi;
  double* Tn = (double*)malloc(sizeof(double) * n);
  for (uint64_t k = 0; k < n; ++k) T[k] = INF_D;
  T[g] = 0;
  int sweeps = 0;
  for (; sweeps < max_sweeps; ++sweeps) {
    int changed = 0;
    for (uint32_t j = 0; j < ny; ++j)
      for (uint32_t i = 0; i < nx; ++i) {
        uint64_t k = (uint64_t)j * nx + i;
        Tn[k] = T[k];
        if (k == g || is_blocked(F[k])) continue;
        double tc = candidate(F, T, nx, ny, i, j);
        if (tc < T[k]) {
          Tn[k] = tc;
          changed = 1;
        }
      }
    memcpy(T, Tn, sizeof(double) * n);
    if (!changed) break;
  }
  free(Tn);
  return sweeps;
}

double oracle_residual(const double* F, const double* T, uint32_t nx, uint32_t ny, uint32_t gi,
                       uint32_t gj, uint64_t* n_decreasing) {
  const uint64_t g = (uint64_t)gj * nx + gi;
  double worst = 0;
  uint64_t cnt = 0;
  for (uint32_t j = 0; j < ny; ++j)
    for (uint32_t i = 0; i < nx; ++i) {
      uint64_t k = (uint64_t)j * nx + i;
      if (k == g || is_blocked(F[k])) continue;
      double tc = candidate(F, T, nx, ny, i, j);
      if (tc < T[k]) {
        ++cnt;
        double d = (T[k] == INF_D) ? INF_D : (T[k] - tc);
        if (d > worst) worst = d;
      }
    }
  if (n_decreasing) *n_decreasing = cnt;
  return worst;
}

void oracle_total_cost_matrix(const double* T, uint64_t n, double* out) {
  for (uint64_t k = 0; k < n; ++k) out[k] = (T[k] == INF_D) ? -1.0 : T[k]; /* :806-809 */
}

/* ------------------------------------------------------------------ */
/* path extraction (:615-784)                                          */
/* ------------------------------------------------------------------ */
/* :718-772 gradientNode; off-grid neighbours are NULL.  The reference would
 * dereference NULL in two corner cases; those read +inf here. */
static void gradient_node(const double* T, uint32_t nx, uint32_t ny, uint32_t i, uint32_t j,
                          double* dnx, double* dny) {
  uint64_t k = (uint64_t)j * nx + i;
  const int hw = i > 0, he = i + 1 < nx, hs = j > 0, hn = j + 1 < ny;
  const double tw = hw ? T[k - 1] : INF_D, te = he ? T[k + 1] : INF_D;
  const double ts = hs ? T[k - nx] : INF_D, tn = hn ? T[k + nx] : INF_D;
  double dx, dy;
  if ((!hw && !he) || (hw && he && tw == INF_D && te == INF_D))
    dx = 0;
  else if (!hw || tw == INF_D)
    dx = te - T[k];
  else if (!he || te == INF_D)
    dx = T[k] - tw;
  else
    dx = (te - tw) * 0.5;
  if ((!hs && !hn) || (hs && hn && ts == INF_D && tn == INF_D))
    dy = 0;
  else if (!hs || ts == INF_D)
    dy = tn - T[k];
  else if (!hn || tn == INF_D)
    dy = T[k] - ts;
  else
    dy = (tn - ts) * 0.5;
  if (dx == 0 && dy == 0) {
    *dnx = 0;
    *dny = 0;
  } else {
    *dnx = dx / sqrt(dx * dx + dy * dy);
    *dny = dy / sqrt(dx * dx + dy * dy);
  }
}

/* :776-784 */
static double interp(double a, double b, double g00, double g01, double g10, double g11) {
  return g00 + (g10 - g00) * a + (g01 - g00) * b + (g11 + g00 - g10 - g01) * a * b;
}

typedef struct {
  double x, y, z, h;
} wp_t;

/* :666-714; writes wpos->z (passed by reference in the reference). */
static wp_t next_waypoint(const double* T, const double* E, uint32_t nx, uint32_t ny, double res,
                          wp_t* wpos, double tau) {
  double gx = wpos->x / res, gy = wpos->y / res;
  uint32_t cx = (uint32_t)gx, cy = (uint32_t)gy;
  double ax = gx - (double)cx, ay = gy - (double)cy;
  double gx00, gx10, gx01, gx11, gy00, gy10, gy01, gy11;
  gradient_node(T, nx, ny, cx, cy, &gx00, &gy00);
  gradient_node(T, nx, ny, cx + 1, cy, &gx10, &gy10);
  gradient_node(T, nx, ny, cx, cy + 1, &gx01, &gy01);
  gradient_node(T, nx, ny, cx + 1, cy + 1, &gx11, &gy11);
  double dcx = interp(ax, ay, gx00, gx01, gx10, gx11);
  double dcy = interp(ax, ay, gy00, gy01, gy10, gy11);
  uint64_t k00 = (uint64_t)cy * nx + cx;
  double e00 = E ? E[k00] : 0, e10 = E ? E[k00 + 1] : 0;
  double e01 = E ? E[k00 + nx] : 0, e11 = E ? E[k00 + nx + 1] : 0;
  /* :699-704 argument order as in the reference (g01 <- e10, g10 <- e01) */
  wpos->z = interp(ax, ay, e00, e10, e01, e11);
  wp_t w;
  w.x = wpos->x - res * tau * dcx;
  w.y = wpos->y - res * tau * dcy;
  w.z = 0;
  w.h = atan2(-dcy, -dcx);
  return w;
}

static int push_wp(double* out, int* n, int max_wp, wp_t w) {
  if (*n >= max_wp) return 0;
  out[4 * *n + 0] = w.x;
  out[4 * *n + 1] = w.y;
  out[4 * *n + 2] = w.z;
  out[4 * *n + 3] = w.h;
  ++*n;
  return 1;
}

/* :615-662.  Returns 1 (true), 0 (false at :628-633 or :650-656: the
 * waypoints pushed so far are kept, as current_path keeps them), -3 when more
 * than max_wp waypoints would be produced; *n_out = #waypoints written. */
int oracle_global_path_partial(const double* T, const double* elev, uint32_t nx, uint32_t ny,
                               double res, uint32_t gi, uint32_t gj, double goal_heading,
                               double risk_distance, double wx, double wy, double wh, double* wp,
                               int max_wp, int* n_out) {
  wp_t sink = {res * (double)gi, res * (double)gj, elev ? elev[(uint64_t)gj * nx + gi] : 0,
               goal_heading};
  wp_t pos = {wx, wy, 0, wh};
  int n = 0;
  *n_out = 0;
  double tau = 0.4 < risk_distance ? 0.4 : risk_distance; /* std::min(0.4, rd) */
  wp_t nxt = next_waypoint(T, elev, nx, ny, res, &pos, tau);
  if (isnan(nxt.x) || isnan(nxt.y)) return 0; /* :628-633 */
  if (!push_wp(wp, &n, max_wp, pos)) return -3;
  pos = nxt;
  while (sqrt((pos.x - sink.x) * (pos.x - sink.x) + (pos.y - sink.y) * (pos.y - sink.y)) >
         2.0 * res) {
    nxt = next_waypoint(T, elev, nx, ny, res, &pos, tau);
    if (!push_wp(wp, &n, max_wp, pos)) return -3;
    *n_out = n;
    if (sqrt((pos.x - nxt.x) * (pos.x - nxt.x) + (pos.y - nxt.y) * (pos.y - nxt.y)) <
        0.01 * tau * res)
      return 0; /* :650-656 */
    pos = nxt;
  }
  if (!push_wp(wp, &n, max_wp, sink)) return -3;
  *n_out = n;
  return 1;
}

int oracle_global_path(const double* T, const double* elev, uint32_t nx, uint32_t ny, double res,
                       uint32_t gi, uint32_t gj, double goal_heading, double risk_distance,
                       double wx, double wy, double wh, double* wp, int max_wp) {
  int n = 0;
  wp_t probe = {wx, wy, 0, wh};
  double tau = 0.4 < risk_distance ? 0.4 : risk_distance;
  wp_t nxt = next_waypoint(T, elev, nx, ny, res, &probe, tau);
  if (isnan(nxt.x) || isnan(nxt.y)) return -1;
  int st = oracle_global_path_partial(T, elev, nx, ny, res, gi, gj, goal_heading, risk_distance,
                                      wx, wy, wh, wp, max_wp, &n);
  if (st == -3) return -3;
  return st == 1 ? n : -2;
}
