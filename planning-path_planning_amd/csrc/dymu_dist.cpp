// dymu_dist.cpp -- row-slab sharded solve driven from C++ (include/dymu_dist.h).
//
// The loop the Python SlabSolver (dymu/sharded.py) runs over torch.distributed,
// here natively on the engine's stream: K passes (dymu_dom_run) -> grouped
// ncclSend/ncclRecv of the two boundary rows with rank-1 / rank+1 -> min-merge
// into the ghost rows (dymu_dom_merge_ghosts, which also writes the number of
// queued tiles) -> ncclAllReduce of that count -> async copy to pinned host
// memory + event.  The host checks the count of the previous round, so it
// never drains the device queue; one extra round (K speculative, empty passes)
// runs after convergence.
//
// Reference: the propagation loop this distributes is computeEntireTotalCostMap
// (src/DyMu_GlobalPathPlanning.cpp:443-468); the per-cell update it converges
// is propagateGlobalNode (:500-546).  SURVEY.md s8(e).
#include "dymu_dist.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

struct dymu_dist {
  dymu_ctx* ctx = nullptr;
  int device = 0;
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  double* d_recv = nullptr;  // 2 x cap doubles: rows from rank-1 (lo) and rank+1 (hi)
  uint64_t recv_cap = 0;
  int32_t* d_cnt = nullptr;  // [0] local queued tiles, [1..kRing] all-reduced rounds
  int32_t* h_cnt = nullptr;  // pinned, kRing
  hipEvent_t ev[2] = {nullptr, nullptr};
  std::string last_error;
};

namespace {

constexpr int kRing = 2;  // rounds in flight: the host reads round m-1 while m is queued
constexpr uint32_t kDefaultK = 16;

int fail(std::string* err, const char* what, const char* detail, int code) {
  if (err) {
    char buf[320];
    std::snprintf(buf, sizeof buf, "%s: %s", what, detail);
    *err = buf;
  }
  return code;
}

#define DHIP(err, expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return fail(err, #expr, hipGetErrorString(_e),                                     \
                  _e == hipErrorOutOfMemory ? DYMU_ERR_NOMEM : DYMU_ERR_HIP);            \
  } while (0)

#define DNCCL(err, expr)                                                                 \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess) return fail(err, #expr, ncclGetErrorString(_r), DYMU_ERR_RCCL); \
  } while (0)

#define DCALL(expr)           \
  do {                        \
    int _rc = (expr);         \
    if (_rc != DYMU_OK) return _rc; \
  } while (0)

// geometry of one rank's slab and its domain descriptor
struct Slab {
  uint32_t row0 = 0, nrows = 0;
  bool lo = false, hi = false;
  dymu_domain dom{};
  int64_t goal_local = -1;
};

int make_slab(const double* F, double* T_buf, uint64_t ld, uint32_t nx, uint32_t ny, uint32_t gj,
              int rank, int world, Slab* s) {
  DCALL(dymu_slab_rows(ny, (uint32_t)world, (uint32_t)rank, &s->row0, &s->nrows));
  if (s->nrows == 0 || !F || !T_buf || ld < nx) return DYMU_ERR_ARG;
  s->lo = rank > 0;
  s->hi = rank < world - 1;
  s->dom.F = F;
  s->dom.T = T_buf + ld;  // owned row 0; ghost rows at T - ld and T + nrows*ld
  s->dom.ld = ld;
  s->dom.nx = nx;
  s->dom.nrows = s->nrows;
  s->dom.ghost_lo = s->lo;
  s->dom.ghost_hi = s->hi;
  s->goal_local = (gj >= s->row0 && gj < s->row0 + s->nrows) ? (int64_t)(gj - s->row0) : -1;
  return DYMU_OK;
}

// safety cap on exchange rounds (the engine's own cap is 4 x tiles + 1024 passes)
uint64_t max_rounds(uint32_t nx, uint32_t ny, uint32_t K) {
  const uint64_t t8 = ((uint64_t)nx / 8 + 1) * ((uint64_t)ny / 8 + 1);
  return (4 * t8 + 1024) / K + 2;
}

}  // namespace

extern "C" {

int dymu_dist_unique_id(unsigned char id[DYMU_DIST_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == DYMU_DIST_ID_BYTES, "ncclUniqueId size");
  if (!id) return DYMU_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return DYMU_ERR_RCCL;
  std::memcpy(id, &u, sizeof u);
  return DYMU_OK;
}

int dymu_dist_create(dymu_dist** out, dymu_ctx* ctx, int device,
                     const unsigned char id[DYMU_DIST_ID_BYTES], int rank, int world) {
  if (!out || !ctx || !id || world < 1 || rank < 0 || rank >= world) return DYMU_ERR_ARG;
  *out = nullptr;
  auto* d = new dymu_dist;
  d->ctx = ctx;
  d->device = device;
  d->rank = rank;
  d->world = world;
  auto bail = [&](int rc) {
    dymu_dist_destroy(d);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(DYMU_ERR_HIP);
  if (hipMalloc(&d->d_cnt, sizeof(int32_t) * (1 + kRing)) != hipSuccess) return bail(DYMU_ERR_NOMEM);
  if (hipHostMalloc(&d->h_cnt, sizeof(int32_t) * kRing, hipHostMallocDefault) != hipSuccess)
    return bail(DYMU_ERR_NOMEM);
  for (auto& e : d->ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return bail(DYMU_ERR_HIP);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  if (ncclCommInitRank(&d->comm, world, u, rank) != ncclSuccess) {
    d->comm = nullptr;
    return bail(DYMU_ERR_RCCL);
  }
  *out = d;
  return DYMU_OK;
}

int dymu_dist_destroy(dymu_dist* d) {
  if (!d) return DYMU_OK;
  (void)hipSetDevice(d->device);
  if (d->comm) (void)ncclCommDestroy(d->comm);
  for (auto& e : d->ev)
    if (e) (void)hipEventDestroy(e);
  if (d->d_recv) (void)hipFree(d->d_recv);
  if (d->d_cnt) (void)hipFree(d->d_cnt);
  if (d->h_cnt) (void)hipHostFree(d->h_cnt);
  delete d;
  return DYMU_OK;
}

const char* dymu_dist_last_error(dymu_dist* d) { return d ? d->last_error.c_str() : ""; }

int dymu_dist_solve(dymu_dist* d, const double* F_slab, double* T_buf, uint64_t ld, uint32_t nx,
                    uint32_t ny, uint32_t goal_i, uint32_t goal_j, uint32_t K, void* stream,
                    dymu_stats* stats) {
  if (!d || nx == 0 || ny == 0 || goal_i >= nx || goal_j >= ny) return DYMU_ERR_ARG;
  std::string* err = &d->last_error;
  if (K == 0) K = kDefaultK;
  Slab s;
  DCALL(make_slab(F_slab, T_buf, ld, nx, ny, goal_j, d->rank, d->world, &s));
  DHIP(err, hipSetDevice(d->device));
  if (d->recv_cap < nx) {
    if (d->d_recv) DHIP(err, hipFree(d->d_recv));
    d->d_recv = nullptr;
    d->recv_cap = 0;
    DHIP(err, hipMalloc(&d->d_recv, sizeof(double) * 2 * nx));
    d->recv_cap = nx;
  }
  // RCCL and the domain primitives must share one stream: NULL = the context's
  if (!stream) stream = dymu_get_stream(d->ctx);
  hipStream_t st = static_cast<hipStream_t>(stream);
  double* recv_lo = d->d_recv;
  double* recv_hi = d->d_recv + d->recv_cap;
  const int32_t* pending = d->d_cnt;
  DCALL(dymu_dom_begin(d->ctx, &s.dom, s.goal_local >= 0 ? goal_i : 0, s.goal_local, stream));
  const uint64_t cap = max_rounds(nx, ny, K);
  uint64_t m = 0;
  bool done = false;
  for (; !done; ++m) {
    if (m >= cap) {
      (void)dymu_dom_finish(d->ctx, stream, nullptr);
      return fail(err, "dymu_dist_solve", "exchange-round cap reached", DYMU_ERR_NOT_CONVERGED);
    }
    DCALL(dymu_dom_run(d->ctx, K, stream));
    if (s.lo || s.hi) {
      DNCCL(err, ncclGroupStart());
      if (s.lo) {
        DNCCL(err, ncclSend(s.dom.T, nx, ncclDouble, d->rank - 1, d->comm, st));
        DNCCL(err, ncclRecv(recv_lo, nx, ncclDouble, d->rank - 1, d->comm, st));
      }
      if (s.hi) {
        DNCCL(err, ncclSend(s.dom.T + (uint64_t)(s.nrows - 1) * ld, nx, ncclDouble, d->rank + 1,
                            d->comm, st));
        DNCCL(err, ncclRecv(recv_hi, nx, ncclDouble, d->rank + 1, d->comm, st));
      }
      DNCCL(err, ncclGroupEnd());
    }
    DCALL(dymu_dom_merge_ghosts(d->ctx, s.lo ? recv_lo : nullptr, s.hi ? recv_hi : nullptr,
                                d->d_cnt, stream));
    const int slot = (int)(m % kRing);
    int32_t* sum = d->d_cnt + 1 + slot;
    DNCCL(err, ncclAllReduce(pending, sum, 1, ncclInt32, ncclSum, d->comm, st));
    DHIP(err, hipMemcpyAsync(d->h_cnt + slot, sum, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    DHIP(err, hipEventRecord(d->ev[slot], st));
    if (m >= 1) {  // round m-1's global count (round m stays queued meanwhile)
      const int prev = (int)((m - 1) % kRing);
      DHIP(err, hipEventSynchronize(d->ev[prev]));
      done = d->h_cnt[prev] == 0;
    }
  }
  DCALL(dymu_dom_finish(d->ctx, stream, stats));
  if (stats) stats->rounds = m;
  return DYMU_OK;
}

int dymu_vdist_solve(dymu_ctx* const* ctxs, int world, const double* const* F_slabs,
                     double* const* T_bufs, uint64_t ld, uint32_t nx, uint32_t ny,
                     uint32_t goal_i, uint32_t goal_j, uint32_t K, void* stream,
                     dymu_stats* stats) {
  if (!ctxs || !F_slabs || !T_bufs || !stream || world < 1 || nx == 0 || ny == 0 ||
      goal_i >= nx || goal_j >= ny)
    return DYMU_ERR_ARG;
  if (K == 0) K = kDefaultK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<Slab> s(world);
  for (int r = 0; r < world; ++r) {
    if (!ctxs[r]) return DYMU_ERR_ARG;
    DCALL(make_slab(F_slabs[r], T_bufs[r], ld, nx, ny, goal_j, r, world, &s[r]));
  }
  // per rank: recv_lo, recv_hi (nx each); counts: world x (1 + kRing) int32
  double* d_recv = nullptr;
  int32_t* d_cnt = nullptr;
  int32_t* h_cnt = nullptr;
  hipEvent_t ev[kRing] = {nullptr, nullptr};
  struct Cleanup {
    double*& a;
    int32_t*& b;
    int32_t*& c;
    hipEvent_t* e;
    ~Cleanup() {
      if (a) (void)hipFree(a);
      if (b) (void)hipFree(b);
      if (c) (void)hipHostFree(c);
      for (int k = 0; k < kRing; ++k)
        if (e[k]) (void)hipEventDestroy(e[k]);
    }
  } cleanup{d_recv, d_cnt, h_cnt, ev};
  DHIP(nullptr, hipMalloc(&d_recv, sizeof(double) * 2 * nx * (uint64_t)world));
  DHIP(nullptr, hipMalloc(&d_cnt, sizeof(int32_t) * world));
  DHIP(nullptr, hipHostMalloc(&h_cnt, sizeof(int32_t) * kRing * world, hipHostMallocDefault));
  for (auto& e : ev) DHIP(nullptr, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  auto recv = [&](int r, int side) { return d_recv + ((uint64_t)r * 2 + side) * nx; };
  for (int r = 0; r < world; ++r)
    DCALL(dymu_dom_begin(ctxs[r], &s[r].dom, s[r].goal_local >= 0 ? goal_i : 0, s[r].goal_local,
                         stream));
  const uint64_t cap = max_rounds(nx, ny, K);
  uint64_t m = 0;
  bool done = false;
  int rc = DYMU_OK;
  for (; !done && rc == DYMU_OK; ++m) {
    if (m >= cap) {
      rc = DYMU_ERR_NOT_CONVERGED;
      break;
    }
    for (int r = 0; r < world && rc == DYMU_OK; ++r) rc = dymu_dom_run(ctxs[r], K, stream);
    if (rc) break;
    // the exchange: rank r's first owned row -> rank r-1's hi ghost, its last -> rank r+1's lo
    for (int r = 0; r < world; ++r) {
      if (s[r].lo)
        DHIP(nullptr, hipMemcpyAsync(recv(r, 0), s[r - 1].dom.T + (uint64_t)(s[r - 1].nrows - 1) * ld,
                                     sizeof(double) * nx, hipMemcpyDeviceToDevice, st));
      if (s[r].hi)
        DHIP(nullptr, hipMemcpyAsync(recv(r, 1), s[r + 1].dom.T, sizeof(double) * nx,
                                     hipMemcpyDeviceToDevice, st));
    }
    const int slot = (int)(m % kRing);
    for (int r = 0; r < world && rc == DYMU_OK; ++r) {
      rc = dymu_dom_merge_ghosts(ctxs[r], s[r].lo ? recv(r, 0) : nullptr,
                                 s[r].hi ? recv(r, 1) : nullptr, d_cnt + r, stream);
      if (rc == DYMU_OK && hipMemcpyAsync(h_cnt + slot * world + r, d_cnt + r, sizeof(int32_t),
                                          hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = DYMU_ERR_HIP;
    }
    if (rc) break;
    DHIP(nullptr, hipEventRecord(ev[slot], st));
    if (m >= 1) {
      const int prev = (int)((m - 1) % kRing);
      DHIP(nullptr, hipEventSynchronize(ev[prev]));
      int64_t tot = 0;
      for (int r = 0; r < world; ++r) tot += h_cnt[prev * world + r];
      done = tot == 0;
    }
  }
  for (int r = 0; r < world; ++r) {
    dymu_stats tmp;
    const int rf = dymu_dom_finish(ctxs[r], stream, stats ? &stats[r] : &tmp);
    if (rc == DYMU_OK) rc = rf;
    if (stats) stats[r].rounds = m;
  }
  return rc;
}

}  // extern "C"
