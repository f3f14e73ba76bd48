// diamond_sim.c -- CPU model of kernel 5's schedule (development tool, not product):
// pass-synchronous priority block-FIM with checkerboard colours, a key threshold
// admitting ~target tiles per pass, red-black in-tile sweeps (convergence tested
// per sweep pair, cap C), exact activation pruning -- for two tile shapes:
//   square  16x16 tiles (kernel 5)
//   diamond tiles: S x S squares in the rotated frame u = x + y, v = x - y + N - 1
//           (S^2 / 2 cells; S = 22: 242 cells, 121 per colour)
// Reports passes, visits, sweeps and a pass-time model sum(fixed + a * max sweeps).
//   gcc -O2 -ffp-contract=off -o /tmp/dsim tools/diamond_sim.c -lm
//   /tmp/dsim N shape(0 square,1 diamond) S target cap [obst_frac]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int N, SHAPE, S, TARGET, CAP;
static double *F, *T, INF;
static int *tile_of, *loc_of;       // per cell
static int ntiles, *toff, *tcell;   // tile cell lists (CSR)
static int *tcol;                   // tile colour (checkerboard of the tile grid)
static int TA, TB;                  // tile grid extents

static uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static double u01(uint64_t k) { return (double)(sm64(k * 7919u + 13u) >> 11) * 0x1.0p-53; }

static void tile_ab(int x, int y, int* a, int* b) {
  if (SHAPE == 0) {
    *a = x / 16, *b = y / 16;
  } else {
    const int u = x + y, v = x - y + N - 1;
    *a = u / S, *b = v / S;
  }
}

static double eik(double tx, double ty, double c) {
  if (fabs(tx - ty) < c && tx < INF && ty < INF)
    return (tx + ty + sqrt(2 * (c * c) - (tx - ty) * (tx - ty))) / 2;
  return fmin(tx, ty) + c;
}

// visit state
static double* val;  // local values
static int maxcells;

typedef struct {
  int t;
  double key;
} Ent;

static int cmp_ent(const void* p, const void* q) {
  const double a = ((const Ent*)p)->key, b = ((const Ent*)q)->key;
  return a < b ? -1 : a > b;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s N shape S target cap [obst]\n", argv[0]);
    return 1;
  }
  N = atoi(argv[1]);
  SHAPE = atoi(argv[2]);
  S = atoi(argv[3]);
  TARGET = atoi(argv[4]);
  CAP = atoi(argv[5]);
  const double obst = argc > 6 ? atof(argv[6]) : 0.02;
  INF = INFINITY;
  const int64_t n = (int64_t)N * N;
  F = malloc(sizeof(double) * n);
  T = malloc(sizeof(double) * n);
  tile_of = malloc(sizeof(int) * n);
  loc_of = malloc(sizeof(int) * n);
  const int gx = N / 2, gy = N / 2;
  for (int64_t k = 0; k < n; ++k) {
    F[k] = obst < 0 ? 1.0 : 1.0 + 4.0 * u01((uint64_t)k);
    if (u01((uint64_t)k + 0x5555555555ull) < obst) F[k] = INF;
    T[k] = INF;
  }
  F[(int64_t)gy * N + gx] = 1.0;
  if (SHAPE == 0) {
    TA = (N + 15) / 16, TB = (N + 15) / 16;
  } else {
    TA = (2 * N - 1 + S - 1) / S, TB = TA;
  }
  // tiles: CSR over the tile grid (empty diamond tiles outside the map stay empty)
  const int64_t ng = (int64_t)TA * TB;
  int* cnt = calloc(ng + 1, sizeof(int));
  for (int y = 0; y < N; ++y)
    for (int x = 0; x < N; ++x) {
      int a, b;
      tile_ab(x, y, &a, &b);
      cnt[(int64_t)b * TA + a + 1]++;
    }
  for (int64_t t = 0; t < ng; ++t) cnt[t + 1] += cnt[t];
  ntiles = (int)ng;
  toff = cnt;
  tcell = malloc(sizeof(int) * n);
  int* fill = calloc(ng, sizeof(int));
  maxcells = 0;
  for (int y = 0; y < N; ++y)
    for (int x = 0; x < N; ++x) {
      int a, b;
      tile_ab(x, y, &a, &b);
      const int64_t t = (int64_t)b * TA + a;
      const int64_t k = (int64_t)y * N + x;
      tile_of[k] = (int)t;
      loc_of[k] = fill[t];
      tcell[toff[t] + fill[t]++] = (int)k;
    }
  int nonempty = 0;
  for (int64_t t = 0; t < ng; ++t) {
    const int c = toff[t + 1] - toff[t];
    if (c > maxcells) maxcells = c;
    nonempty += c > 0;
  }
  tcol = malloc(sizeof(int) * ng);
  for (int64_t t = 0; t < ng; ++t) tcol[t] = (int)((t % TA + t / TA) & 1);
  val = malloc(sizeof(double) * maxcells);
  double* key = malloc(sizeof(double) * ng);
  char* listed = calloc(ng, 1);
  for (int64_t t = 0; t < ng; ++t) key[t] = INF;
  Ent* list = malloc(sizeof(Ent) * ng);
  Ent* next = malloc(sizeof(Ent) * ng);
  int nl = 0, nn = 0;
  const int64_t gk = (int64_t)gy * N + gx;
  T[gk] = 0.0;
  list[nl++] = (Ent){tile_of[gk], 0.0};
  listed[tile_of[gk]] = 1;
  key[tile_of[gk]] = 0.0;
  long long passes = 0, visits = 0, sweeps = 0, deferred = 0, capped = 0;
  double tmodel = 0.0;  // sum over passes of (4 + 0.75 * max sweeps) us
  double* snap_key = malloc(sizeof(double) * ng);
  Ent* sorted = malloc(sizeof(Ent) * ng);
  // per visit: which neighbour tiles got a decreased edge cell, with the min value
  int* act_t = malloc(sizeof(int) * 4 * maxcells);
  double* act_v = malloc(sizeof(double) * 4 * maxcells);
  while (nl > 0) {
    const int parity = (int)(passes & 1);
    ++passes;
    // threshold: the TARGET-th smallest key over the whole list (both colours)
    double thr = INF;
    if (TARGET > 0 && nl > TARGET) {
      memcpy(sorted, list, sizeof(Ent) * nl);
      qsort(sorted, nl, sizeof(Ent), cmp_ent);
      thr = sorted[TARGET - 1].key;
    }
    for (int q = 0; q < nl; ++q) snap_key[list[q].t] = key[list[q].t];
    nn = 0;
    int maxsw = 0;
    for (int q = 0; q < nl; ++q) listed[list[q].t] = 0;
    for (int q = 0; q < nl; ++q) {
      const int t = list[q].t;
      const double kt = snap_key[t];
      if (tcol[t] != parity || kt > thr) {  // deferred with its key
        ++deferred;
        if (!listed[t]) {
          listed[t] = 1;
          next[nn++] = (Ent){t, kt};
        }
        continue;
      }
      key[t] = INF;
      // visit: local values, sweeps
      const int c0 = toff[t], nc = toff[t + 1] - c0;
      for (int l = 0; l < nc; ++l) val[l] = T[tcell[c0 + l]];
      int sw = 0, cap = 1;
      while (sw < CAP) {
        int changed = 0;
        for (int h = 0; h < 2; ++h) {  // two sweeps per test
          for (int col = 0; col < 2; ++col)
            for (int l = 0; l < nc; ++l) {
              const int k = tcell[c0 + l];
              const int x = k % N, y = k / N;
              if (((x + y) & 1) != col) continue;
              if (k == gk || !(F[k] < INF)) continue;
              double nb[4];
              const int xs[4] = {x - 1, x + 1, x, x}, ys[4] = {y, y, y - 1, y + 1};
              for (int d = 0; d < 4; ++d) {
                if (xs[d] < 0 || ys[d] < 0 || xs[d] >= N || ys[d] >= N) {
                  nb[d] = INF;
                  continue;
                }
                const int64_t m = (int64_t)ys[d] * N + xs[d];
                nb[d] = tile_of[m] == t ? val[loc_of[m]] : T[m];
              }
              const double u = eik(fmin(nb[0], nb[1]), fmin(nb[2], nb[3]), F[k]);
              if (u < val[l]) {
                val[l] = u;
                if (h == 1) changed = 1;
              }
            }
          ++sw;
        }
        if (!changed) {
          cap = 0;
          break;
        }
      }
      ++visits;
      sweeps += sw;
      capped += cap;
      if (sw > maxsw) maxsw = sw;
      // write back + activations (exact pruning: a decreased cell activates the
      // neighbour tile across only if it is below that neighbour cell's value)
      int na = 0;
      for (int l = 0; l < nc; ++l) {
        const int k = tcell[c0 + l];
        if (!(val[l] < T[k])) continue;
        T[k] = val[l];
        const int x = k % N, y = k / N;
        const int xs[4] = {x - 1, x + 1, x, x}, ys[4] = {y, y, y - 1, y + 1};
        for (int d = 0; d < 4; ++d) {
          if (xs[d] < 0 || ys[d] < 0 || xs[d] >= N || ys[d] >= N) continue;
          const int64_t m = (int64_t)ys[d] * N + xs[d];
          if (tile_of[m] == t || !(val[l] < T[m])) continue;
          act_t[na] = tile_of[m];
          act_v[na++] = val[l];
        }
      }
      for (int z = 0; z < na; ++z) {
        const int u = act_t[z];
        if (act_v[z] < key[u]) key[u] = act_v[z];
        if (!listed[u]) {
          listed[u] = 1;
          next[nn++] = (Ent){u, 0};
        }
      }
      if (cap) {
        if (kt < key[t]) key[t] = kt;
        if (!listed[t]) {
          listed[t] = 1;
          next[nn++] = (Ent){t, 0};
        }
      }
    }
    for (int q = 0; q < nn; ++q) next[q].key = key[next[q].t];
    tmodel += 4.0 + 0.75 * maxsw;
    Ent* s = list;
    list = next;
    next = s;
    nl = nn;
  }
  // check against a plain fixed point residual
  double res = 0;
  for (int y = 1; y < N - 1; ++y)
    for (int x = 1; x < N - 1; ++x) {
      const int64_t k = (int64_t)y * N + x;
      if (k == gk || !(F[k] < INF)) continue;
      const double u = eik(fmin(T[k - 1], T[k + 1]), fmin(T[k - N], T[k + N]), F[k]);
      if (T[k] < INF && u < T[k]) {
        const double r = (T[k] - u) / T[k];
        if (r > res) res = r;
      }
    }
  double sum = 0;
  for (int64_t k = 0; k < n; ++k)
    if (T[k] < INF) sum += T[k];
  printf("N %d shape %s S %d target %d cap %d: tiles %d passes %lld visits %lld (%.2f/tile) "
         "sweeps %lld (%.2f/visit) capped %.1f%% deferred %lld model %.2f ms residual %.2e sum %.10e\n",
         N, SHAPE ? "diamond" : "square", SHAPE ? S : 16, TARGET, CAP, nonempty, passes, visits,
         (double)visits / nonempty, sweeps, (double)sweeps / visits, 100.0 * capped / visits,
         deferred, tmodel / 1000.0, res, sum);
  return 0;
}
