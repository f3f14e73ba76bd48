// dymu_dist.cpp -- row-slab sharded solve driven from C++ (include/dymu_dist.h).
//
// The loop the Python SlabSolver (dymu/sharded.py) runs over torch.distributed,
// here natively, every step on the engine's stream.  Round m:
//   K passes (dymu_dom_run)
//   -> grouped ncclSend/ncclRecv: the first / last owned rows straight from T
//      to rank-1 / rank+1, theirs into two receive rows
//   -> one exchange launch: min-merge the received rows into the ghost rows and
//      count the tiles queued for the next pass (dymu_dom_exchange)
//   -> every kCheckEvery-th round: ncclAllReduce of that count -> 4-byte copy to
//      pinned host memory + event.
// The host reads the previous check's count after queueing the current one, so
// it never drains the device queue; up to two check intervals of (empty) rounds
// run after convergence.  With kernel-5 slabs (dymu_dom_round) the received rows
// are instead merged by the next round's first pass -- no exchange launch -- and
// the all-reduced count reaches the host through the engine's mailbox: the next
// round's first pass stores it into host-coherent memory (no copy, no event).
//
// Why one stream and no overlap: the pass kernel is one 1024-thread workgroup
// per CU at full register use, back to back, so a kernel on a second stream
// (RCCL's) only gets CUs between passes and the pass stream then waits for it
// anyway -- measured at N=1: a two-stream pipeline cost ~20 us per round, a
// CU-masked pass stream (1 CU per XCD left to RCCL) 50% per pass.
//
// Reference: the propagation loop this distributes is computeEntireTotalCostMap
// (src/DyMu_GlobalPathPlanning.cpp:443-468); the per-cell update it converges
// is propagateGlobalNode (:500-546).  SURVEY.md s8(e).
#include "dymu_dist.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

// Per-rank exchange buffers: r = the rows received from rank-1 (side 0) and
// rank+1 (side 1); d_cnt = [queued tiles of this round, its all-reduced value]
// for two round parities (the host reads round m-1's while round m is queued).
struct Pipe {
  double* rbuf = nullptr;    // [2 side][cap]
  int32_t* d_cnt = nullptr;  // [2 parity][2], then the pre-flight flag
  uint64_t cap = 0;
  double* r(int side) const { return rbuf + (uint64_t)side * cap; }
  int32_t* tot(int par) const { return d_cnt + 2 * par; }
  int32_t* sum(int par) const { return d_cnt + 2 * par + 1; }
  int32_t* flag() const { return d_cnt + 4; }
};

struct dymu_dist {
  dymu_ctx* ctx = nullptr;
  int device = 0;
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  bool aborted = false;  // the communicator was aborted after an error (no further solves)
  Pipe pipe;
  int32_t* h_sum = nullptr;  // pinned [2 parity + the pre-flight flag]
  hipEvent_t ev[2] = {nullptr, nullptr};
  std::string last_error;
};

namespace {

// passes per round: a round costs one RCCL P2P group + one exchange launch + one
// 4-byte all-reduce on the pass stream (~8 us at N=1 without the P2P), and ghost
// rows are at most K passes stale.  16384^2 rehearsal (tools/vdist_rehearsal.py,
// max per-rank pass time): K = 4 -> 37.4 / 27.4 / 21.8 ms at 2 / 4 / 8 ranks in
// 338 / 327 / 302 rounds; K = 8 -> 44.6 / 32.8 / 27.2 ms in 156 / 163 / 156.
constexpr uint32_t kDefaultK = 4;
// rounds per termination check: the 4-byte all-reduce (and its copy to the host)
// sits on the pass stream, so it runs on every kCheckEvery-th round only.  A zero
// global count after ANY round is the fixed point (no rank has work and no ghost
// improved), so checking a subset of rounds is exact; the solve ends at most two
// check intervals of empty rounds later.
constexpr uint64_t kCheckEvery = 4;

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

#define DCALL(expr)                 \
  do {                              \
    int _rc = (expr);               \
    if (_rc != DYMU_OK) return _rc; \
  } while (0)

// geometry of one rank's slab and its domain descriptor
struct Slab {
  uint32_t row0 = 0, nrows = 0;
  bool lo = false, hi = false;
  dymu_domain dom{};
  int64_t goal_local = -1;
  const double* row(int side) const {  // the owned row shared with rank-1 (0) / rank+1 (1)
    return side == 0 ? dom.T : dom.T + (uint64_t)(nrows - 1) * dom.ld;
  }
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
  return (4 * t8 + 1024) / K + 4;
}

int pipe_alloc(Pipe* p, uint64_t nx) {
  if (p->cap >= nx) return DYMU_OK;
  if (p->rbuf) (void)hipFree(p->rbuf);
  if (p->d_cnt) (void)hipFree(p->d_cnt);
  *p = Pipe{};
  if (hipMalloc(&p->rbuf, sizeof(double) * 2 * nx) != hipSuccess ||
      hipMalloc(&p->d_cnt, sizeof(int32_t) * 5) != hipSuccess)
    return DYMU_ERR_NOMEM;
  p->cap = nx;
  return DYMU_OK;
}

void pipe_free(Pipe* p) {
  if (p->rbuf) (void)hipFree(p->rbuf);
  if (p->d_cnt) (void)hipFree(p->d_cnt);
  *p = Pipe{};
}

// Host wait on an event queued behind RCCL work, bounded: a peer that died or
// left the collective sequence would otherwise block this rank forever.
// DYMU_DIST_TIMEOUT_S (default 300 s) bounds one wait.
double dist_timeout_s() {
  static const double limit_s = [] {
    const char* kv = std::getenv("DYMU_DIST_TIMEOUT_S");
    const double v = kv ? std::atof(kv) : 0.0;
    return v > 0.0 ? v : 300.0;
  }();
  return limit_s;
}

int wait_event(hipEvent_t ev, std::string* err) {
  const double limit_s = dist_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0;; ++spin) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return DYMU_OK;
    if (e != hipErrorNotReady) return fail(err, "hipEventQuery", hipGetErrorString(e), DYMU_ERR_HIP);
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    if ((spin & 1023) == 1023 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
      return fail(err, "dymu_dist_solve", "timed out waiting for the exchange (a peer rank failed?)",
                  DYMU_ERR_RCCL);
  }
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
  if (hipHostMalloc(&d->h_sum, sizeof(int32_t) * 3, hipHostMallocDefault) != hipSuccess)
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
  pipe_free(&d->pipe);
  if (d->h_sum) (void)hipHostFree(d->h_sum);
  delete d;
  return DYMU_OK;
}

const char* dymu_dist_last_error(dymu_dist* d) { return d ? d->last_error.c_str() : ""; }

int dymu_dist_comm_count(dymu_dist* d, int* ranks) {
  if (!d || !ranks) return DYMU_ERR_ARG;
  if (!d->comm) return DYMU_ERR_STATE;
  int n = 0;
  if (ncclCommCount(d->comm, &n) != ncclSuccess) return DYMU_ERR_RCCL;
  *ranks = n;
  return DYMU_OK;
}

}  // extern "C"

namespace {

// The round loop of dymu_dist_solve (the domain is live on entry).  Any error
// return leaves the communicator in an unknown collective state; the caller
// aborts it.
int dist_rounds(dymu_dist* d, const Slab& s, uint32_t nx, uint32_t ny, uint32_t K, void* stream,
                uint64_t* rounds) {
  std::string* err = &d->last_error;
  const Pipe& p = d->pipe;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint64_t cap = max_rounds(nx, ny, K) + 2 * kCheckEvery;
  // fused: the rows received after round m are merged by round m+1's first pass
  // (dymu_dom_round) instead of a k_exchange launch after the transfer
  const bool fused = dymu_dom_round_supported(d->ctx, K) == 1;
  bool mail = true;  // checks read through the context's mailbox while it has one
  uint32_t prev_seq = 0;
  uint64_t m = 0, checks = 0;
  bool done = false, have_rows = false;
  for (; !done; ++m) {
    if (m >= cap) return fail(err, "dymu_dist_solve", "exchange-round cap reached",
                              DYMU_ERR_NOT_CONVERGED);
    const bool check = (m % kCheckEvery) == kCheckEvery - 1;
    const int par = (int)(checks & 1);
    int rc = fused ? dymu_dom_round(d->ctx, K, have_rows && s.lo ? p.r(0) : nullptr,
                                    have_rows && s.hi ? p.r(1) : nullptr, p.tot(par), stream)
                   : dymu_dom_run(d->ctx, K, stream);
    if (rc) return fail(err, fused ? "dymu_dom_round" : "dymu_dom_run", dymu_last_error(d->ctx), rc);
    if (s.lo || s.hi) {
      DNCCL(err, ncclGroupStart());
      if (s.lo) {
        DNCCL(err, ncclSend(s.row(0), nx, ncclDouble, d->rank - 1, d->comm, st));
        DNCCL(err, ncclRecv(p.r(0), nx, ncclDouble, d->rank - 1, d->comm, st));
      }
      if (s.hi) {
        DNCCL(err, ncclSend(s.row(1), nx, ncclDouble, d->rank + 1, d->comm, st));
        DNCCL(err, ncclRecv(p.r(1), nx, ncclDouble, d->rank + 1, d->comm, st));
      }
      DNCCL(err, ncclGroupEnd());
    }
    have_rows = true;
    if (!fused) {
      rc = dymu_dom_exchange(d->ctx, s.lo ? p.r(0) : nullptr, s.hi ? p.r(1) : nullptr, p.tot(par),
                             stream);
      if (rc) return fail(err, "dymu_dom_exchange", dymu_last_error(d->ctx), rc);
    }
    if (!check) continue;
    DNCCL(err, ncclAllReduce(p.tot(par), p.sum(par), 1, ncclInt32, ncclSum, d->comm, st));
    if (mail) {  // the next round's first pass posts the sum; read the previous check's
      uint32_t seq = 0;
      rc = dymu_dom_post(d->ctx, p.sum(par), &seq);
      if (rc == DYMU_ERR_STATE && checks == 0) {
        mail = false;
      } else if (rc) {
        return fail(err, "dymu_dom_post", dymu_last_error(d->ctx), rc);
      } else {
        if (checks >= 1) {
          int32_t v = 0;
          rc = dymu_dom_wait_post(d->ctx, prev_seq, dist_timeout_s(), &v, stream);
          if (rc) return fail(err, "dymu_dom_wait_post", dymu_last_error(d->ctx), DYMU_ERR_RCCL);
          done = v == 0;
        }
        prev_seq = seq;
      }
    }
    if (!mail) {
      DHIP(err, hipMemcpyAsync(d->h_sum + par, p.sum(par), sizeof(int32_t),
                               hipMemcpyDeviceToHost, st));
      DHIP(err, hipEventRecord(d->ev[par], st));
      if (checks >= 1) {  // the previous check's global count; this one stays queued meanwhile
        rc = wait_event(d->ev[par ^ 1], err);
        if (rc) return rc;
        done = d->h_sum[par ^ 1] == 0;
      }
    }
    ++checks;
  }
  *rounds = m;
  return DYMU_OK;
}

// Collective pre-flight: every rank learns whether every rank can solve, so a
// rank-local argument error (an empty slab, a null buffer) fails all ranks
// together instead of leaving the others blocked in their first exchange.
int preflight(dymu_dist* d, bool ok, hipStream_t st) {
  std::string* err = &d->last_error;
  const Pipe& p = d->pipe;
  d->h_sum[2] = ok ? 1 : 0;
  DHIP(err, hipMemcpyAsync(p.flag(), d->h_sum + 2, sizeof(int32_t), hipMemcpyHostToDevice, st));
  DNCCL(err, ncclAllReduce(p.flag(), p.flag(), 1, ncclInt32, ncclMin, d->comm, st));
  DHIP(err, hipMemcpyAsync(d->h_sum + 2, p.flag(), sizeof(int32_t), hipMemcpyDeviceToHost, st));
  DHIP(err, hipEventRecord(d->ev[0], st));
  int rc = wait_event(d->ev[0], err);
  if (rc) return rc;
  if (d->h_sum[2] != 1)
    return fail(err, "dymu_dist_solve", ok ? "another rank rejected its slab" : "invalid slab",
                DYMU_ERR_ARG);
  return DYMU_OK;
}

// After an error inside the collective sequence: abort the communicator (its
// peers may be blocked in a send/recv this rank will never post), leave the
// domain, and refuse further solves on this handle.
int abort_comm(dymu_dist* d, int rc) {
  if (d->comm) (void)ncclCommAbort(d->comm);
  d->comm = nullptr;
  d->aborted = true;
  return rc;
}

}  // namespace

extern "C" {

int dymu_dist_solve(dymu_dist* d, const double* F_slab, double* T_buf, uint64_t ld, uint32_t nx,
                    uint32_t ny, uint32_t goal_i, uint32_t goal_j, uint32_t K, void* stream,
                    dymu_stats* stats) {
  if (!d) return DYMU_ERR_ARG;
  std::string* err = &d->last_error;
  if (d->aborted || !d->comm)
    return fail(err, "dymu_dist_solve", "communicator aborted by an earlier error", DYMU_ERR_STATE);
  if (K == 0) K = kDefaultK;
  DHIP(err, hipSetDevice(d->device));
  if (pipe_alloc(&d->pipe, nx ? nx : 1) != DYMU_OK)
    return abort_comm(d, fail(err, "pipe_alloc", "out of memory", DYMU_ERR_NOMEM));
  // RCCL and the domain primitives share one stream: NULL = the context's
  if (!stream) stream = dymu_get_stream(d->ctx);
  hipStream_t st = static_cast<hipStream_t>(stream);
  Slab s;
  const bool ok = nx > 0 && ny > 0 && goal_i < nx && goal_j < ny &&
                  make_slab(F_slab, T_buf, ld, nx, ny, goal_j, d->rank, d->world, &s) == DYMU_OK;
  int rc = preflight(d, ok, st);
  if (rc) return rc == DYMU_ERR_ARG ? rc : abort_comm(d, rc);
  rc = dymu_dom_begin(d->ctx, &s.dom, s.goal_local >= 0 ? goal_i : 0, s.goal_local, stream);
  if (rc) return abort_comm(d, fail(err, "dymu_dom_begin", dymu_last_error(d->ctx), rc));
  uint64_t rounds = 0;
  rc = dist_rounds(d, s, nx, ny, K, stream, &rounds);
  const int rf = dymu_dom_finish(d->ctx, stream, stats);
  if (rc) return abort_comm(d, rc);
  if (rf) return abort_comm(d, fail(err, "dymu_dom_finish", dymu_last_error(d->ctx), rf));
  if (stats) stats->rounds = rounds;
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
  std::vector<Pipe> p(world);
  int32_t* h_tot = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  struct Cleanup {
    std::vector<Pipe>& p;
    int32_t*& h;
    hipEvent_t* e;
    ~Cleanup() {
      for (auto& q : p) pipe_free(&q);
      if (h) (void)hipHostFree(h);
      for (int k = 0; k < 2; ++k)
        if (e[k]) (void)hipEventDestroy(e[k]);
    }
  } cleanup{p, h_tot, ev};
  for (auto& q : p) DCALL(pipe_alloc(&q, nx));
  DHIP(nullptr, hipHostMalloc(&h_tot, sizeof(int32_t) * 2 * world, hipHostMallocDefault));
  for (auto& e : ev) DHIP(nullptr, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (int r = 0; r < world; ++r)
    DCALL(dymu_dom_begin(ctxs[r], &s[r].dom, s[r].goal_local >= 0 ? goal_i : 0, s[r].goal_local,
                         stream));
  const uint64_t cap = max_rounds(nx, ny, K) + 2 * kCheckEvery;
  uint64_t m = 0, checks = 0;
  bool done = false;
  int rc = DYMU_OK;
  // the schedule of dymu_dist_solve with every rank's work serialised on one
  // stream: device-to-device row copies for RCCL P2P, a host sum for the
  // all-reduce
  // fused rounds (kernel 5 slabs): as dist_rounds, the copied rows are merged by
  // each rank's next round
  bool fused = true;
  for (int r = 0; r < world; ++r) fused = fused && dymu_dom_round_supported(ctxs[r], K) == 1;
  bool have_rows = false;
  for (; !done && rc == DYMU_OK; ++m) {
    if (m >= cap) {
      rc = DYMU_ERR_NOT_CONVERGED;
      break;
    }
    const bool check = (m % kCheckEvery) == kCheckEvery - 1;
    const int par = (int)(checks & 1);
    for (int r = 0; r < world && rc == DYMU_OK; ++r)
      rc = fused ? dymu_dom_round(ctxs[r], K, have_rows && s[r].lo ? p[r].r(0) : nullptr,
                                  have_rows && s[r].hi ? p[r].r(1) : nullptr, p[r].tot(par), stream)
                 : dymu_dom_run(ctxs[r], K, stream);
    if (rc) break;
    for (int r = 0; r < world; ++r) {  // rank r-1's last row / rank r+1's first row
      if (s[r].lo)
        DHIP(nullptr, hipMemcpyAsync(p[r].r(0), s[r - 1].row(1), sizeof(double) * nx,
                                     hipMemcpyDeviceToDevice, st));
      if (s[r].hi)
        DHIP(nullptr, hipMemcpyAsync(p[r].r(1), s[r + 1].row(0), sizeof(double) * nx,
                                     hipMemcpyDeviceToDevice, st));
    }
    have_rows = true;
    for (int r = 0; r < world && rc == DYMU_OK; ++r) {
      if (!fused)
        rc = dymu_dom_exchange(ctxs[r], s[r].lo ? p[r].r(0) : nullptr,
                               s[r].hi ? p[r].r(1) : nullptr, p[r].tot(par), stream);
      if (rc == DYMU_OK && check &&
          hipMemcpyAsync(h_tot + par * world + r, p[r].tot(par), sizeof(int32_t),
                         hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = DYMU_ERR_HIP;
    }
    if (rc) break;
    if (!check) continue;
    DHIP(nullptr, hipEventRecord(ev[par], st));
    if (checks >= 1) {
      DHIP(nullptr, hipEventSynchronize(ev[par ^ 1]));
      int64_t tot = 0;
      for (int r = 0; r < world; ++r) tot += h_tot[(par ^ 1) * world + r];
      done = tot == 0;
    }
    ++checks;
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
