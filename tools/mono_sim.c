/* mono_sim.c -- CPU model of the FIM's min-over-history rounding bias.
 *
 * The serpentine maze of tools/maze_bench.py (U(1,5) speed, 2% obstacles, walls every
 * 64 rows with one gap at alternating ends, goal at the centre) is solved by
 *   - the reference FMM (heap, reference update :531-535, accept if smaller :537), and
 *   - a label-correcting tile FIM (red-black sweeps per 16x16 tile, FIFO tile queue),
 *     which evaluates every cell many times as its inputs converge from above and keeps
 *     the minimum -- the GPU engine's accept rule,
 * with several candidate arithmetics for the FIM:
 *   0 reference      (Tx + Ty + sqrt(2C^2 - d^2)) / 2, correctly rounded sqrt
 *   1 kernel-5 v31   fma(s, t, fma(d, 0.5, Ty)), one Goldschmidt step on rsq (~2^-22 model)
 *   2 monotone       min(Tx,Ty) + (|d| < C ? fma(s, t, |d|/2) : C), same sqrt model
 *   3 monotone exact min(Tx,Ty) + (|d| < C ? (|d| + sqrt(r))/2 : C)
 * and prints the max relative deviation from the FMM, split into above / below.
 * Build: gcc -O2 -ffp-contract=off -o /tmp/mono_sim tools/mono_sim.c -lm
 * Usage: /tmp/mono_sim N [period]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static inline double u01(uint64_t seed, uint64_t k) {
  return (double)(splitmix64(seed ^ k) >> 11) * 0x1p-53;
}

/* v_rsq_f64 model: 1/sqrt(x) with a deterministic relative error up to 2^-22 */
static inline double rsq_model(double x) {
  uint64_t b;
  memcpy(&b, &x, 8);
  const double e = ((double)(splitmix64(b) >> 11) * 0x1p-53 * 2.0 - 1.0) * 0x1p-22;
  return (1.0 / sqrt(x)) * (1.0 + e);
}

static int MODE;

static inline double cand(double tx, double ty, double c) {
  const double m = ty < tx ? ty : tx;
  if (!(c < INFINITY) || !(m < INFINITY)) return m + c;
  const double d = tx - ty;
  if (!(fabs(d) < c)) return m + c;
  const double c2 = 2.0 * (c * c);
  if (MODE == 0) return (tx + ty + sqrt(c2 - d * d)) / 2;
  const double r = fma(-d, d, c2);
  if (MODE == 3) return m + (fabs(d) + sqrt(r)) * 0.5;
  const double y0 = rsq_model(r);
  const double s = r * y0;
  const double t = fma(-(y0 * 0.25), s, 0.75);
  if (MODE == 1) return fma(s, t, fma(d, 0.5, ty));
  return m + fma(s, t, fabs(d) * 0.5);
}

static uint32_t NX, NY;
static const double* F;

static inline double update(const double* T, uint32_t i, uint32_t j) {
  const uint64_t k = (uint64_t)j * NX + i;
  const double w = i > 0 ? T[k - 1] : INFINITY, e = i + 1 < NX ? T[k + 1] : INFINITY;
  const double s = j > 0 ? T[k - NX] : INFINITY, n = j + 1 < NY ? T[k + NX] : INFINITY;
  return cand(w < e ? w : e, s < n ? s : n, F[k]);
}

/* reference FMM: binary heap keyed (T, insertion sequence) */
typedef struct { double t; uint64_t seq; uint32_t k; } hent;
static hent* H;
static size_t HN;
static inline int hl(const hent* a, const hent* b) { return a->t < b->t || (a->t == b->t && a->seq < b->seq); }
static void hpush(hent e) {
  size_t i = HN++;
  while (i) { size_t p = (i - 1) / 2; if (!hl(&e, &H[p])) break; H[i] = H[p]; i = p; }
  H[i] = e;
}
static hent hpop(void) {
  hent top = H[0], e = H[--HN];
  size_t i = 0;
  for (;;) {
    size_t c = 2 * i + 1;
    if (c >= HN) break;
    if (c + 1 < HN && hl(&H[c + 1], &H[c])) ++c;
    if (!hl(&H[c], &e)) break;
    H[i] = H[c]; i = c;
  }
  H[i] = e;
  return top;
}

static void fmm(double* T, uint32_t gi, uint32_t gj) {
  const uint64_t n = (uint64_t)NX * NY;
  uint8_t* closed = calloc(n, 1);
  for (uint64_t k = 0; k < n; ++k) T[k] = INFINITY;
  H = malloc(sizeof(hent) * (n * 4 + 8));
  HN = 0;
  uint64_t seq = 0;
  const uint64_t g = (uint64_t)gj * NX + gi;
  T[g] = 0;
  hpush((hent){0.0, seq++, (uint32_t)g});
  const int di[4] = {0, -1, 1, 0}, dj[4] = {-1, 0, 0, 1};
  while (HN) {
    hent e = hpop();
    if (closed[e.k] || e.t != T[e.k]) continue;
    closed[e.k] = 1;
    const uint32_t i = e.k % NX, j = e.k / NX;
    for (int q = 0; q < 4; ++q) {
      const int64_t a = (int64_t)i + di[q], b = (int64_t)j + dj[q];
      if (a < 0 || b < 0 || a >= NX || b >= NY) continue;
      const uint64_t k = (uint64_t)b * NX + a;
      if (closed[k] || !(F[k] < INFINITY)) continue;
      const int sm = MODE;
      MODE = 0;
      const double u = update(T, a, b);
      MODE = sm;
      if (u < T[k]) { T[k] = u; hpush((hent){u, seq++, (uint32_t)k}); }
    }
  }
  free(H);
  free(closed);
}

/* label-correcting tile FIM: FIFO queue of 16x16 tiles, red-black sweeps to convergence */
static uint64_t fim(double* T, uint32_t gi, uint32_t gj) {
  const uint32_t B = 16, ntx = (NX + B - 1) / B, nty = (NY + B - 1) / B;
  const uint64_t n = (uint64_t)NX * NY, nt = (uint64_t)ntx * nty;
  for (uint64_t k = 0; k < n; ++k) T[k] = INFINITY;
  T[(uint64_t)gj * NX + gi] = 0;
  uint32_t* q = malloc(sizeof(uint32_t) * (nt + 1));
  uint8_t* inq = calloc(nt, 1);
  uint64_t head = 0, tail = 0, evals = 0;
  const uint32_t t0 = (gj / B) * ntx + gi / B;
  q[tail++ % (nt + 1)] = t0;
  inq[t0] = 1;
  while (head != tail) {
    const uint32_t t = q[head++ % (nt + 1)];
    inq[t] = 0;
    const uint32_t tx = t % ntx, ty = t / ntx;
    const uint32_t i0 = tx * B, j0 = ty * B;
    const uint32_t i1 = i0 + B < NX ? i0 + B : NX, j1 = j0 + B < NY ? j0 + B : NY;
    int edge[4] = {0, 0, 0, 0};
    for (int sweep = 0; sweep < 64; ++sweep) {
      int changed = 0;
      for (int col = 0; col < 2; ++col)
        for (uint32_t j = j0; j < j1; ++j)
          for (uint32_t i = i0 + ((j + col) & 1); i < i1; i += 2) {
            const uint64_t k = (uint64_t)j * NX + i;
            if (!(F[k] < INFINITY) || (i == gi && j == gj)) continue;
            const double u = update(T, i, j);
            ++evals;
            if (u < T[k]) {
              T[k] = u;
              changed = 1;
              if (j == j0) edge[0] = 1;
              if (i == i0) edge[1] = 1;
              if (i + 1 == i1) edge[2] = 1;
              if (j + 1 == j1) edge[3] = 1;
            }
          }
      if (!changed) break;
    }
    const int dx[4] = {0, -1, 1, 0}, dy[4] = {-1, 0, 0, 1};
    for (int e = 0; e < 4; ++e) {
      if (!edge[e]) continue;
      const int64_t a = (int64_t)tx + dx[e], b = (int64_t)ty + dy[e];
      if (a < 0 || b < 0 || a >= ntx || b >= nty) continue;
      const uint32_t u = (uint32_t)(b * ntx + a);
      if (!inq[u]) { inq[u] = 1; q[tail++ % (nt + 1)] = u; }
    }
  }
  free(q);
  free(inq);
  return evals;
}

int main(int argc, char** argv) {
  const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 2048;
  const uint32_t period = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
  const int maze = period > 0;
  NX = NY = N;
  const uint64_t n = (uint64_t)N * N;
  double* Fm = malloc(8 * n);
  const uint32_t gi = N / 2, gj = N / 2;
  for (uint64_t k = 0; k < n; ++k) {
    Fm[k] = 1.0 + 4.0 * u01(1, k);
    const uint32_t i = k % N, j = k / N;
    const int ng = (i + 1 >= gi && i <= gi + 1 && j + 1 >= gj && j <= gj + 1);
    if (!ng && u01(3, k) < 0.02) Fm[k] = INFINITY;
  }
  if (maze)
    for (uint32_t j = period / 2, kk = 0; j < N; j += period, ++kk) {
      for (uint32_t i = 0; i < N; ++i) Fm[(uint64_t)j * N + i] = INFINITY;
      Fm[(uint64_t)j * N + (kk % 2 == 0 ? 1 : N - 2)] = 2.0;
    }
  F = Fm;
  double* Tr = malloc(8 * n);
  double* T = malloc(8 * n);
  MODE = 0;
  fmm(Tr, gi, gj);
  for (int mode = 0; mode < 4; ++mode) {
    MODE = mode;
    const uint64_t ev = fim(T, gi, gj);
    double up = 0, dn = 0, sbias = 0;
    uint64_t nf = 0, mism = 0, eq = 0;
    for (uint64_t k = 0; k < n; ++k) {
      const int fa = T[k] < INFINITY, fb = Tr[k] < INFINITY;
      if (fa != fb) { ++mism; continue; }
      if (!fa) continue;
      ++nf;
      const double rel = (T[k] - Tr[k]) / (Tr[k] > 1 ? Tr[k] : 1);
      if (rel > up) up = rel;
      if (-rel > dn) dn = -rel;
      sbias += rel;
      eq += T[k] == Tr[k];
    }
    printf("N=%u maze=%d mode=%d evals/cell=%.1f mask_mismatch=%llu max_above=%.3e max_below=%.3e "
           "mean_rel=%.3e equal=%.1f%%\n",
           N, maze, mode, (double)ev / (double)nf, (unsigned long long)mism, up, dn, sbias / (double)nf,
           100.0 * (double)eq / (double)nf);
    fflush(stdout);
  }
  return 0;
}
