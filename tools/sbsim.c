// sbsim.c -- CPU model of the pass schedule with SUPERBLOCKS (development tool).
// A superblock of B x B cells is relaxed by one workgroup: its S x S sub-tiles
// (one wave each) run red-black sweep pairs in lockstep (a workgroup barrier per
// half-sweep), a sub-tile sweeping only while it or a neighbouring sub-tile
// changed in the previous pair.  B == S is the current one-wave-per-tile design.
// Counts passes, the per-pass critical chain (max sweep pairs of a visit), the
// sub-tile sweep pairs (VALU work) and cell updates.
//   gcc -O2 -ffp-contract=off -o /tmp/sbsim tools/sbsim.c -lm
//   /tmp/sbsim N B S target cap [deferral]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static double INF;
static int N, B, S, NS, nbx;
static double *F, *T, *SNAP;

static inline uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static double u01(uint64_t s, uint64_t k) { return (double)(sm64(s ^ k) >> 11) * 0x1.0p-53; }
static inline double eik(double tx, double ty, double c) {
  if (fabs(tx - ty) < c) return (tx + ty + sqrt(2 * (c * c) - (tx - ty) * (tx - ty))) / 2;
  return fmin(tx, ty) + c;
}

static double* L;  // (B+2)^2 image
#define LI(r, c) ((r) * (B + 2) + (c))
static long long updates, subpairs;
static int chg[64 * 64], act[64 * 64];

// one superblock visit; returns pairs run, sets *edge (bit0 N,1 W,2 E,3 S) and *capped
static int visit(int bx, int by, int cap, unsigned* edge, int* capped, const double* fl) {
  int i0 = bx * B, j0 = by * B;
  static double* t0 = 0;
  if (!t0) t0 = malloc(sizeof(double) * B * B);
  for (int r = 0; r < B + 2; r++)
    for (int c = 0; c < B + 2; c++) {
      int j = j0 + r - 1, i = i0 + c - 1;
      int inside = r >= 1 && r <= B && c >= 1 && c <= B;
      double v = INF;
      if (j >= 0 && j < N && i >= 0 && i < N) v = inside ? T[(size_t)j * N + i] : SNAP[(size_t)j * N + i];
      L[LI(r, c)] = v;
    }
  for (int r = 0; r < B; r++)
    for (int c = 0; c < B; c++) t0[r * B + c] = L[LI(r + 1, c + 1)];
  for (int q = 0; q < NS * NS; q++) act[q] = 1;
  int pairs = 0;
  for (;;) {
    int any = 0;
    for (int q = 0; q < NS * NS; q++) any |= act[q];
    if (!any) break;
    if (pairs >= cap) { *capped = 1; break; }
    pairs++;
    memset(chg, 0, sizeof(int) * NS * NS);
    for (int color = 0; color < 2; color++)
      for (int q = 0; q < NS * NS; q++) {
        if (!act[q]) continue;
        int sr = (q / NS) * S, sc = (q % NS) * S;
        for (int r = sr + 1; r <= sr + S; r++)
          for (int c = sc + 1; c <= sc + S; c++) {
            if (((r + c) & 1) != color) continue;
            int j = j0 + r - 1, i = i0 + c - 1;
            if (j >= N || i >= N) continue;
            double f = fl[(size_t)j * N + i];
            if (!(f < INF)) continue;
            updates++;
            double v = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]), f);
            if (v < L[LI(r, c)]) { L[LI(r, c)] = v; chg[q] = 1; }
          }
      }
    for (int q = 0; q < NS * NS; q++) subpairs += act[q];
    int sx, sy;
    for (int q = 0; q < NS * NS; q++) {
      sy = q / NS; sx = q % NS;
      int a = chg[q];
      if (sx > 0) a |= chg[q - 1];
      if (sx + 1 < NS) a |= chg[q + 1];
      if (sy > 0) a |= chg[q - NS];
      if (sy + 1 < NS) a |= chg[q + NS];
      act[q] = a;
    }
  }
  unsigned e = 0;
  for (int r = 0; r < B; r++)
    for (int c = 0; c < B; c++) {
      int j = j0 + r, i = i0 + c;
      if (j >= N || i >= N) continue;
      double v = L[LI(r + 1, c + 1)];
      if (v < t0[r * B + c]) {
        T[(size_t)j * N + i] = v;
        if (r == 0) e |= 1;
        if (c == 0) e |= 2;
        if (c == B - 1) e |= 4;
        if (r == B - 1) e |= 8;
      }
    }
  *edge = e;
  return pairs;
}

static int cmpd(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  INF = __builtin_inf();
  N = atoi(argv[1]); B = atoi(argv[2]); S = atoi(argv[3]);
  int TARGET = atoi(argv[4]), CAP = atoi(argv[5]);
  NS = B / S;
  size_t n = (size_t)N * N;
  F = malloc(8 * n); T = malloc(8 * n); SNAP = malloc(8 * n);
  int gi = N / 2, gj = N / 2;
  for (size_t k = 0; k < n; k++) {
    double v = 1 + 4 * u01(1, k);
    int i = k % N, j = k / N;
    if (u01(3, k) < 0.02 && !(abs(i - gi) <= 1 && abs(j - gj) <= 1)) v = INF;
    F[k] = v; T[k] = INF;
  }
  T[(size_t)gj * N + gi] = 0;
  nbx = (N + B - 1) / B;
  int nt = nbx * nbx;
  L = malloc(sizeof(double) * (B + 2) * (B + 2));
  int *cur = malloc(sizeof(int) * nt), *nxt = malloc(sizeof(int) * nt), *mark = calloc(nt, sizeof(int));
  double* key = malloc(sizeof(double) * nt);
  double* kk = malloc(sizeof(double) * nt);
  for (int q = 0; q < nt; q++) key[q] = INF;
  int nc = 1, nn;
  cur[0] = (gj / B) * nbx + gi / B;
  key[cur[0]] = 0;
  long long visits = 0, chain = 0, pairsum = 0, capped_n = 0;
  int passes = 0;
  while (nc > 0) {
    passes++;
    memcpy(SNAP, T, 8 * n);
    double thr = INF;
    if (nc > TARGET) {
      for (int q = 0; q < nc; q++) kk[q] = key[cur[q]];
      qsort(kk, nc, sizeof(double), cmpd);
      thr = kk[TARGET - 1];
    }
    nn = 0;
    int pmax = 0;
    for (int q = 0; q < nc; q++) {
      int t = cur[q];
      if (key[t] > thr) {
        if (mark[t] != passes) { mark[t] = passes; nxt[nn++] = t; }
        continue;
      }
      double k0 = key[t];
      key[t] = INF;
      unsigned e; int capped = 0;
      int p = visit(t % nbx, t / nbx, CAP, &e, &capped, F);
      visits++; pairsum += p; capped_n += capped;
      if (p > pmax) pmax = p;
      int tx = t % nbx, ty = t / nbx, cand[5], m = 0;
      if ((e & 1) && ty > 0) cand[m++] = t - nbx;
      if ((e & 2) && tx > 0) cand[m++] = t - 1;
      if ((e & 4) && tx + 1 < nbx) cand[m++] = t + 1;
      if ((e & 8) && ty + 1 < nbx) cand[m++] = t + nbx;
      if (capped) cand[m++] = t;
      for (int z = 0; z < m; z++) {
        int u = cand[z], ux = u % nbx, uy = u / nbx;
        double kv = INF;
        int i0 = tx * B, j0 = ty * B;
        if (uy < ty) for (int c = 0; c < B && i0 + c < N; c++) kv = fmin(kv, T[(size_t)j0 * N + i0 + c]);
        else if (uy > ty) { int jj = j0 + B - 1 < N ? j0 + B - 1 : N - 1; for (int c = 0; c < B && i0 + c < N; c++) kv = fmin(kv, T[(size_t)jj * N + i0 + c]); }
        else if (ux < tx) for (int r = 0; r < B && j0 + r < N; r++) kv = fmin(kv, T[(size_t)(j0 + r) * N + i0]);
        else if (ux > tx) { int ii = i0 + B - 1 < N ? i0 + B - 1 : N - 1; for (int r = 0; r < B && j0 + r < N; r++) kv = fmin(kv, T[(size_t)(j0 + r) * N + ii]); }
        else kv = k0;
        if (kv < key[u]) key[u] = kv;
        if (mark[u] != passes) { mark[u] = passes; nxt[nn++] = u; }
      }
    }
    chain += pmax;
    int* tmp = cur; cur = nxt; nxt = tmp; nc = nn;
  }
  double sum = 0;
  for (size_t k = 0; k < n; k++) if (T[k] < INF) sum += T[k];
  printf("N=%d B=%d S=%d target=%d cap=%d passes=%d visits=%lld (%.2f/block) pairs/visit=%.1f capped=%.1f%% "
         "chain=%lld (sum of per-pass max pairs) subtile-pairs/cell-tile=%.1f updates/cell=%.1f sum=%.10e\n",
         N, B, S, TARGET, CAP, passes, visits, (double)visits / nt, (double)pairsum / visits,
         100.0 * capped_n / visits, chain, (double)subpairs / ((double)n / (S * S)), (double)updates / n, sum);
  return 0;
}
