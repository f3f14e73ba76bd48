// fimsim.c -- CPU simulator of the tile-FIM schedule (development tool).
// Counts passes, tile visits, in-tile sweeps and cell updates for several
// in-tile solvers and tile sizes, to choose the GPU design before writing it.
//   gcc -O2 -ffp-contract=off -o /tmp/fimsim tools/fimsim.c -lm
//   /tmp/fimsim N W H method [bucket]
// methods: 0 = strip Jacobi (v1 kernel model: chaotic Jacobi, 4-row GS strips)
//          1 = 4-direction Gauss-Seidel sweeps (fast sweeping) until no change
//          2 = pure Jacobi sweeps
//          3 = 2-direction (up-right / down-left) GS sweeps (skewed-wave model)
// Halo values are snapshotted at the start of each pass (pessimistic model of
// concurrent tiles).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static double INF;
static int N, W, H, M;
static double *F, *T, *S;  // S = snapshot
static int ntx, nty;

static inline uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static double u01(uint64_t s, uint64_t k) { return (double)(sm64(s ^ k) >> 11) * 0x1.0p-53; }

static inline double eik(double tx, double ty, double c) {
  if (fabs(tx - ty) < c && tx < INF && ty < INF)
    return (tx + ty + sqrt(2 * (c * c) - (tx - ty) * (tx - ty))) / 2;
  return fmin(tx, ty) + c;
}

// local tile buffer with halo
static double* L;  // (H+2)*(W+2)
#define LI(r, c) ((r) * (W + 2) + (c))
static long long cell_updates;
static long long subpasses, subvisits;
static int SB = 8;
static int PRUNE = 0;
static int GROUP = 64;
static double EPSR = 0;
static long long hist[6];

static int relax(int r, int c, const double* f) {
  double v = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]),
                 f[(r - 1) * W + (c - 1)]);
  cell_updates++;
  if (v < L[LI(r, c)]) {
    L[LI(r, c)] = v;
    return 1;
  }
  return 0;
}

static int solve_tile(int tx, int ty, int method, int maxs, int* sweeps_out, unsigned* edge) {
  int i0 = tx * W, j0 = ty * H;
  static double* f = 0;
  static double* t0 = 0;
  if (!f) {
    f = malloc(sizeof(double) * W * H);
    t0 = malloc(sizeof(double) * W * H);
  }
  for (int r = 0; r < H + 2; r++)
    for (int c = 0; c < W + 2; c++) {
      int j = j0 + r - 1, i = i0 + c - 1;
      double v = INF;
      int inside = r >= 1 && r <= H && c >= 1 && c <= W;
      if (j >= 0 && j < N && i >= 0 && i < N) v = inside ? T[(size_t)j * N + i] : S[(size_t)j * N + i];
      L[LI(r, c)] = v;
    }
  for (int r = 0; r < H; r++)
    for (int c = 0; c < W; c++) {
      int j = j0 + r, i = i0 + c;
      f[r * W + c] = (j < N && i < N) ? F[(size_t)j * N + i] : INF;
      t0[r * W + c] = L[LI(r + 1, c + 1)];
    }
  int s = 0, changed = 1;
  while (changed && s < maxs) {
    changed = 0;
    if (method == 2) {  // pure Jacobi
      static double* nl = 0;
      if (!nl) nl = malloc(sizeof(double) * (H + 2) * (W + 2));
      memcpy(nl, L, sizeof(double) * (H + 2) * (W + 2));
      for (int r = 1; r <= H; r++)
        for (int c = 1; c <= W; c++) {
          double v = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]),
                         fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]), f[(r - 1) * W + (c - 1)]);
          cell_updates++;
          if (v < nl[LI(r, c)]) { nl[LI(r, c)] = v; changed = 1; }
        }
      memcpy(L, nl, sizeof(double) * (H + 2) * (W + 2));
    } else if (method == 0) {  // strip model: rows in strips of 4 (GS in strip, alternating), Jacobi across
      static double* nl = 0;
      if (!nl) nl = malloc(sizeof(double) * (H + 2) * (W + 2));
      memcpy(nl, L, sizeof(double) * (H + 2) * (W + 2));
      int up = (s & 1) == 0;
      for (int st = 0; st < H / 4; st++)
        for (int c = 1; c <= W; c++)
          for (int kk = 0; kk < 4; kk++) {
            int k = up ? kk : 3 - kk;
            int r = st * 4 + k + 1;
            double south = (k == 0) ? L[LI(r - 1, c)] : nl[LI(r - 1, c)];
            double north = (k == 3) ? L[LI(r + 1, c)] : nl[LI(r + 1, c)];
            double v = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(north, south),
                           f[(r - 1) * W + (c - 1)]);
            cell_updates++;
            if (v < nl[LI(r, c)]) { nl[LI(r, c)] = v; changed = 1; }
          }
      memcpy(L, nl, sizeof(double) * (H + 2) * (W + 2));
    } else if (method == 1) {  // 4-dir GS
      int d = s & 3;
      int rs = (d & 1) ? H : 1, re = (d & 1) ? 0 : H + 1, rd = (d & 1) ? -1 : 1;
      int cs = (d & 2) ? W : 1, ce = (d & 2) ? 0 : W + 1, cd = (d & 2) ? -1 : 1;
      for (int r = rs; r != re; r += rd)
        for (int c = cs; c != ce; c += cd) changed |= relax(r, c, f);
      // any complete sweep without a change is a fixed point
    } else if (method == 4 || method == 5) {
      // lockstep line sweeps: all lanes (columns or rows) advance one step at a
      // time; method 4 = column lines only (up/down), 5 = alternate
      // columns-up, rows-right, columns-down, rows-left.
      static double* buf = 0;
      if (!buf) buf = malloc(sizeof(double) * (W > H ? W : H));
      int d = (method == 4) ? ((s & 1) ? 2 : 0) : (s & 3);
      if (d == 0 || d == 2) {  // columns, rows advance
        for (int q = 0; q < H; q++) {
          int r = (d == 0) ? q + 1 : H - q;
          for (int c = 1; c <= W; c++)
            buf[c - 1] = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]), f[(r - 1) * W + (c - 1)]);
          for (int c = 1; c <= W; c++) { cell_updates++; if (buf[c - 1] < L[LI(r, c)]) { L[LI(r, c)] = buf[c - 1]; changed = 1; } }
        }
      } else {  // rows, columns advance
        for (int q = 0; q < W; q++) {
          int c = (d == 1) ? q + 1 : W - q;
          for (int r = 1; r <= H; r++)
            buf[r - 1] = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]), f[(r - 1) * W + (c - 1)]);
          for (int r = 1; r <= H; r++) { cell_updates++; if (buf[r - 1] < L[LI(r, c)]) { L[LI(r, c)] = buf[r - 1]; changed = 1; } }
        }
      }
      int period = (method == 4) ? 2 : 4;
      if (!changed && (s % period) != period - 1) changed = 1;
    } else if (method == 6) {
      // hierarchical: sub-block FIM inside the tile; this "sweep" is one
      // sub-pass over the active sub-blocks (snapshot halos between
      // sub-blocks), each Jacobi-iterated to local convergence.
      static unsigned char* act = 0; static unsigned char* nact = 0; static double* snap = 0; static double* nl = 0;
      int nbx = W / SB, nby = H / SB;
      if (!act) { act = calloc(4096, 1); nact = calloc(4096, 1); snap = malloc(sizeof(double) * (H + 2) * (W + 2)); nl = malloc(sizeof(double) * (H + 2) * (W + 2)); }
      if (s == 0) for (int q = 0; q < nbx * nby; q++) act[q] = 1;
      memcpy(snap, L, sizeof(double) * (H + 2) * (W + 2));
      memset(nact, 0, nbx * nby);
      int any = 0;
      subpasses++;
      for (int by = 0; by < nby; by++) for (int bx = 0; bx < nbx; bx++) {
        if (!act[by * nbx + bx]) continue;
        subvisits++;
        int r0 = by * SB + 1, c0 = bx * SB + 1;
        // local buffer: sub-block from L, halo from snapshot
        int ch = 1, e = 0;
        // iterate Jacobi on the sub-block using halo from snap and interior from L
        while (ch) {
          ch = 0;
          for (int r = r0; r < r0 + SB; r++) for (int c = c0; c < c0 + SB; c++) {
            #define GV(rr, cc) (((rr) >= r0 && (rr) < r0 + SB && (cc) >= c0 && (cc) < c0 + SB) ? L[LI(rr, cc)] : snap[LI(rr, cc)])
            nl[LI(r, c)] = eik(fmin(GV(r, c - 1), GV(r, c + 1)), fmin(GV(r - 1, c), GV(r + 1, c)), f[(r - 1) * W + (c - 1)]);
            cell_updates++;
          }
          for (int r = r0; r < r0 + SB; r++) for (int c = c0; c < c0 + SB; c++)
            if (nl[LI(r, c)] < L[LI(r, c)]) {
              L[LI(r, c)] = nl[LI(r, c)]; ch = 1; changed = 1;
              if (r == r0) e |= 1; if (c == c0) e |= 2; if (c == c0 + SB - 1) e |= 4; if (r == r0 + SB - 1) e |= 8;
            }
        }
        if ((e & 1) && by > 0) nact[(by - 1) * nbx + bx] = 1;
        if ((e & 2) && bx > 0) nact[by * nbx + bx - 1] = 1;
        if ((e & 4) && bx + 1 < nbx) nact[by * nbx + bx + 1] = 1;
        if ((e & 8) && by + 1 < nby) nact[(by + 1) * nbx + bx] = 1;
        any = 1;
      }
      memcpy(act, nact, nbx * nby);
      changed = 0;
      for (int q = 0; q < nbx * nby; q++) if (act[q]) changed = 1;
    } else if (method == 8 || method == 9) {
      // lockstep segments: every lane owns a 4-cell segment (method 8: rows in
      // even sweeps, columns in odd ones; method 9: rows only) and all lanes
      // update their k-th cell at step k from the current image (so the other
      // segments' cells are as of their own step), direction alternating every
      // two sweeps
      static double* buf = 0;
      if (!buf) buf = malloc(sizeof(double) * W * H);
      const int orient = method == 9 ? 0 : (s & 1), dir = method == 9 ? (s & 1) : ((s >> 1) & 1);
      for (int k = 0; k < 4; k++) {
        const int kk = dir ? 3 - k : k;
        int nb = 0;
        if (orient == 0) {
          for (int r = 1; r <= H; r++)
            for (int sg = 0; sg < W / 4; sg++) {
              const int c = sg * 4 + kk + 1;
              buf[nb++] = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]), f[(r - 1) * W + (c - 1)]);
            }
          nb = 0;
          for (int r = 1; r <= H; r++)
            for (int sg = 0; sg < W / 4; sg++) {
              const int c = sg * 4 + kk + 1;
              cell_updates++;
              if (buf[nb] < L[LI(r, c)]) { L[LI(r, c)] = buf[nb]; changed = 1; }
              nb++;
            }
        } else {
          for (int c = 1; c <= W; c++)
            for (int sg = 0; sg < H / 4; sg++) {
              const int r = sg * 4 + kk + 1;
              buf[nb++] = eik(fmin(L[LI(r, c - 1)], L[LI(r, c + 1)]), fmin(L[LI(r - 1, c)], L[LI(r + 1, c)]), f[(r - 1) * W + (c - 1)]);
            }
          nb = 0;
          for (int c = 1; c <= W; c++)
            for (int sg = 0; sg < H / 4; sg++) {
              const int r = sg * 4 + kk + 1;
              cell_updates++;
              if (buf[nb] < L[LI(r, c)]) { L[LI(r, c)] = buf[nb]; changed = 1; }
              nb++;
            }
        }
      }
    } else if (method == 7) {  // red-black (checkerboard) GS: red half-sweep then black
      for (int color = 0; color < 2; color++)
        for (int r = 1; r <= H; r++)
          for (int c = 1; c <= W; c++)
            if (((r + c) & 1) == color) changed |= relax(r, c, f);
    } else if (method == 3) {  // 2-direction GS: up-right, down-left
      if ((s & 1) == 0) {
        for (int r = 1; r <= H; r++) for (int c = 1; c <= W; c++) changed |= relax(r, c, f);
      } else {
        for (int r = H; r >= 1; r--) for (int c = W; c >= 1; c--) changed |= relax(r, c, f);
      }
      if (!changed && (s & 1) == 0) changed = 1;
    }
    s++;
  }
  *sweeps_out = s;
  unsigned e = 0;
  double maxrel = 0;
  for (int r = 0; r < H; r++)
    for (int c = 0; c < W; c++) {
      int j = j0 + r, i = i0 + c;
      if (j >= N || i >= N) continue;
      double v = L[LI(r + 1, c + 1)];
      if (v < t0[r * W + c]) {
        T[(size_t)j * N + i] = v;
        double rel = (t0[r * W + c] == INF) ? 1.0 : (t0[r * W + c] - v) / v;
        if (rel > maxrel) maxrel = rel;
        if (rel <= EPSR) continue;  // below the activation threshold
        // prune: the neighbour cell across the edge can only improve through
        // this cell if v < its current value (U >= max(Tx,Ty) two-sided)
        if (r == 0 && (!PRUNE || v < L[LI(0, c + 1)])) e |= 1;
        if (c == 0 && (!PRUNE || v < L[LI(r + 1, 0)])) e |= 2;
        if (c == W - 1 && (!PRUNE || v < L[LI(r + 1, W + 1)])) e |= 4;
        if (r == H - 1 && (!PRUNE || v < L[LI(H + 1, c + 1)])) e |= 8;
      }
    }
  *edge = e;
  int b = maxrel >= 1.0 ? 0 : maxrel > 1e-6 ? 1 : maxrel > 1e-10 ? 2 : maxrel > 1e-13 ? 3 : maxrel > 0 ? 4 : 5;
  hist[b]++;
  return s >= maxs;
}

int cmpd(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  INF = __builtin_inf();
  N = atoi(argv[1]);
  W = atoi(argv[2]);
  H = atoi(argv[3]);
  M = atoi(argv[4]);
  if (argc > 5) SB = atoi(argv[5]);
  double DELTA = argc > 6 ? atof(argv[6]) : 0;
  int CAP = argc > 7 ? atoi(argv[7]) : 0;
  PRUNE = argc > 8 ? atoi(argv[8]) : 0;
  EPSR = argc > 9 ? atof(argv[9]) : 0;
  if (getenv("GROUP")) GROUP = atoi(getenv("GROUP"));
  long long group_cost = 0; int gmax = 0, gcnt = 0;
  double frac = 0.02;
  size_t n = (size_t)N * N;
  F = malloc(8 * n); T = malloc(8 * n); S = malloc(8 * n);
  int gi = N / 2, gj = N / 2;
  for (size_t k = 0; k < n; k++) {
    double v = 1 + 4 * u01(1, k);
    int i = k % N, j = k / N;
    if (u01(3, k) < frac && !(abs(i - gi) <= 1 && abs(j - gj) <= 1)) v = INF;
    F[k] = v;
    T[k] = INF;
  }
  T[(size_t)gj * N + gi] = 0;
  ntx = (N + W - 1) / W; nty = (N + H - 1) / H;
  int nt = ntx * nty;
  L = malloc(sizeof(double) * (H + 2) * (W + 2));
  int* cur = malloc(sizeof(int) * nt), *nxt = malloc(sizeof(int) * nt);
  int* mark = calloc(nt, sizeof(int));
  int nc = 1, nn;
  cur[0] = (gj / H) * ntx + gi / W;
  long long visits = 0, sweeps = 0;
  int passes = 0;
  int maxs = 4 * (W + H);
  if (CAP > 0) maxs = CAP;
  double* key = malloc(sizeof(double) * nt);
  for (int q = 0; q < nt; q++) key[q] = INF;
  key[cur[0]] = 0;
  long long deferred = 0;
  while (nc > 0) {
    passes++;
    memcpy(S, T, 8 * n);
    nn = 0;
    double kmin = INF;
    for (int q = 0; q < nc; q++) if (key[cur[q]] < kmin) kmin = key[cur[q]];
    double thr = DELTA > 0 ? kmin + DELTA : INF;
    if (getenv("TARGET")) {  // relax the TARGET lowest keys (v4 model)
      int P = atoi(getenv("TARGET"));
      if (nc > P) {
        static double* kk = 0;
        static int kcap = 0;
        if (kcap < nc) { kk = realloc(kk, sizeof(double) * nc); kcap = nc; }
        for (int q = 0; q < nc; q++) kk[q] = key[cur[q]];
        int cmpd(const void* a, const void* b);
        qsort(kk, nc, sizeof(double), cmpd);
        thr = kk[P - 1];
      }
    }
    for (int q = 0; q < nc; q++) {
      int t = cur[q], tx = t % ntx, ty = t / ntx, sw;
      if (key[t] > thr) {  // deferred: stays active
        if (mark[t] != passes) { mark[t] = passes; nxt[nn++] = t; }
        deferred++;
        continue;
      }
      unsigned e;
      key[t] = INF;
      int capped = solve_tile(tx, ty, M, maxs, &sw, &e);
      visits++;
      sweeps += sw;
      if (sw > gmax) gmax = sw;
      if (++gcnt == GROUP) { group_cost += gmax; gmax = 0; gcnt = 0; }
      int cand[5], ncand = 0;
      if ((e & 1) && ty > 0) cand[ncand++] = t - ntx;
      if ((e & 2) && tx > 0) cand[ncand++] = t - 1;
      if ((e & 4) && tx + 1 < ntx) cand[ncand++] = t + 1;
      if ((e & 8) && ty + 1 < nty) cand[ncand++] = t + ntx;
      if (capped) cand[ncand++] = t;
      // key of an enqueued neighbour: min T on the shared edge (this tile's edge values)
      for (int z = 0; z < ncand; z++) {
        int u = cand[z];
        int ux = u % ntx, uy = u / ntx;
        double kv = INF;
        int i0 = tx * W, j0 = ty * H;
        if (uy < ty) for (int c = 0; c < W && i0 + c < N; c++) kv = fmin(kv, T[(size_t)j0 * N + i0 + c]);
        else if (uy > ty) for (int c = 0; c < W && i0 + c < N; c++) kv = fmin(kv, T[(size_t)(j0 + H - 1 < N ? j0 + H - 1 : N - 1) * N + i0 + c]);
        else if (ux < tx) for (int r = 0; r < H && j0 + r < N; r++) kv = fmin(kv, T[(size_t)(j0 + r) * N + i0]);
        else if (ux > tx) for (int r = 0; r < H && j0 + r < N; r++) kv = fmin(kv, T[(size_t)(j0 + r) * N + (i0 + W - 1 < N ? i0 + W - 1 : N - 1)]);
        else kv = 0;
        if (kv < key[u]) key[u] = kv;
        if (mark[u] != passes) { mark[u] = passes; nxt[nn++] = u; }
      }
    }
    if (gcnt) { group_cost += gmax; gmax = 0; gcnt = 0; }
    int* tmp = cur; cur = nxt; nxt = tmp; nc = nn;
  }
  printf("  visit max-rel-improvement histogram: new=%lld >1e-6=%lld >1e-10=%lld >1e-13=%lld >0=%lld none=%lld\n", hist[0], hist[1], hist[2], hist[3], hist[4], hist[5]);
  printf("  lane-per-tile wave cost: %lld group-sweeps => %.1f sweeps per tile-visit (incl. max-over-64)\n", group_cost, (double)GROUP * group_cost / visits);
  if (DELTA > 0) printf("  delta=%.1f deferred=%lld\n", DELTA, deferred);
  double sum = 0;
  for (size_t k = 0; k < n; k++) if (T[k] < INF) sum += T[k];
  if (M == 6) printf("  subpasses=%lld (%.1f/visit) subvisits=%lld (%.2f/subblock-visit-per-tile-visit)\n", subpasses, (double)subpasses / visits, subvisits, (double)subvisits / visits / ((W / SB) * (H / SB)));
  printf("N=%d tile=%dx%d method=%d passes=%d visits=%lld (%.2f/tile) sweeps=%lld (%.1f/visit) "
         "updates/cell=%.1f sum=%.10e\n",
         N, W, H, M, passes, visits, (double)visits / nt, sweeps, (double)sweeps / visits,
         (double)cell_updates / n, sum);
  return 0;
}
