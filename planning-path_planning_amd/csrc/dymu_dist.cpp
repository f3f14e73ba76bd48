// dymu_dist.cpp -- row-slab sharded solve driven from C++ (include/dymu_dist.h).
//
// The loop the Python SlabSolver (dymu/sharded.py) runs over torch.distributed,
// here natively, as a two-stream pipeline per round m:
//   pass stream:  K passes (dymu_dom_run) -> min-merge the rows received in
//                 round m-1 into the ghost rows (dymu_dom_merge_ghosts, which
//                 writes the queued-tile count) -> pack this round's boundary
//                 rows into send buffers (+ a changed-since-last-round flag)
//   comm stream:  grouped ncclSend/ncclRecv of those rows with rank-1 / rank+1
//                 and ncclAllReduce of the count -> pinned host copy + event
// so the xGMI transfer of round m overlaps the passes of round m+1.  The host
// reads the count of round m-1 after queueing round m and never drains the
// device queue; one extra round of (empty) passes runs after convergence.
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

// Exchange buffers of one rank, doubled by round parity so that round m's rows
// can be in flight while round m+1's passes run: s = rows sent, r = rows
// received, side 0 = the row shared with rank-1, side 1 = with rank+1.
struct Pipe {
  double* sbuf = nullptr;   // [2 parity][2 side][cap]
  double* rbuf = nullptr;   // [2 parity][2 side][cap]
  int32_t* d_tot = nullptr; // [2 parity] queued tiles + changed-row flag of the round
  int32_t* d_sum = nullptr; // [2 parity] its all-reduced value
  uint64_t cap = 0;
  double* s(int par, int side) const { return sbuf + ((uint64_t)par * 2 + side) * cap; }
  double* r(int par, int side) const { return rbuf + ((uint64_t)par * 2 + side) * cap; }
};

struct dymu_dist {
  dymu_ctx* ctx = nullptr;
  int device = 0;
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  hipStream_t comm_stream = nullptr;  // RCCL runs here, beside the pass stream
  Pipe pipe;
  int32_t* h_sum = nullptr;  // pinned [2 parity]
  hipEvent_t ev_pack[2] = {nullptr, nullptr};  // rows of the round packed (pass stream)
  hipEvent_t ev_comm[2] = {nullptr, nullptr};  // rows received + count reduced (comm stream)
  std::string last_error;
};

namespace {

// passes per round: the rows of round m are merged after round m+1's passes, so
// a round must be short (16384^2 rehearsal, 8 virtual ranks: K = 4 -> 1252
// launches per rank, 8 -> 1472, 16 -> 2400; tools/vdist_rehearsal.py)
constexpr uint32_t kDefaultK = 4;

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
  if (p->sbuf) (void)hipFree(p->sbuf);
  if (p->rbuf) (void)hipFree(p->rbuf);
  if (p->d_tot) (void)hipFree(p->d_tot);
  *p = Pipe{};
  if (hipMalloc(&p->sbuf, sizeof(double) * 4 * nx) != hipSuccess ||
      hipMalloc(&p->rbuf, sizeof(double) * 4 * nx) != hipSuccess ||
      hipMalloc(&p->d_tot, sizeof(int32_t) * 4) != hipSuccess)
    return DYMU_ERR_NOMEM;
  p->d_sum = p->d_tot + 2;
  p->cap = nx;
  return DYMU_OK;
}

void pipe_free(Pipe* p) {
  if (p->sbuf) (void)hipFree(p->sbuf);
  if (p->rbuf) (void)hipFree(p->rbuf);
  if (p->d_tot) (void)hipFree(p->d_tot);
  *p = Pipe{};
}

// Copy the boundary rows into this round's send buffers and add 1 to *tot per
// wave that saw a cell differ from the previous round's rows (prev NULL: the
// first round, every finite cell counts).  Values only decrease, so equal rows
// mean nothing new for the neighbour.
__global__ void k_pack_rows(const double* row_lo, const double* row_hi, double* s_lo,
                            double* s_hi, const double* prev_lo, const double* prev_hi,
                            uint32_t nx, int32_t* tot) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool ch = false;
  if (k < nx) {
    if (row_lo) {
      const double v = row_lo[k];
      s_lo[k] = v;
      ch |= prev_lo ? v != prev_lo[k] : v < __builtin_inf();
    }
    if (row_hi) {
      const double v = row_hi[k];
      s_hi[k] = v;
      ch |= prev_hi ? v != prev_hi[k] : v < __builtin_inf();
    }
  }
  if (__any(ch) && (threadIdx.x & 63) == 0) atomicAdd(tot, 1);
}

hipError_t pack_rows(const Slab& s, const Pipe& p, uint64_t m, hipStream_t st) {
  const int par = (int)(m & 1);
  const uint32_t nx = s.dom.nx;
  if (!s.lo && !s.hi) return hipSuccess;
  hipLaunchKernelGGL(k_pack_rows, dim3((nx + 255) / 256), dim3(256), 0, st,
                     s.lo ? s.row(0) : nullptr, s.hi ? s.row(1) : nullptr, p.s(par, 0),
                     p.s(par, 1), m ? p.s(par ^ 1, 0) : nullptr, m ? p.s(par ^ 1, 1) : nullptr,
                     nx, p.d_tot + par);
  return hipGetLastError();
}

// Round m on the pass stream: K passes, then merge the rows received in round
// m-1 into the ghost rows (writes the queued-tile count to d_tot[par]), then
// pack this round's rows (adds the changed-row flag).  The sum over ranks of
// d_tot[par] is 0 exactly when no rank has queued work and no boundary row
// changed since the rows every neighbour has already merged: the fixed point.
int round_compute(dymu_ctx* ctx, const Slab& s, const Pipe& p, uint64_t m, uint32_t K,
                  hipStream_t st, hipEvent_t rows_in) {
  const int par = (int)(m & 1);
  DCALL(dymu_dom_run(ctx, K, st));
  if (m && rows_in) DHIP(nullptr, hipStreamWaitEvent(st, rows_in, 0));
  DCALL(dymu_dom_merge_ghosts(ctx, m && s.lo ? p.r(par ^ 1, 0) : nullptr,
                              m && s.hi ? p.r(par ^ 1, 1) : nullptr, p.d_tot + par, st));
  DHIP(nullptr, pack_rows(s, p, m, st));
  return DYMU_OK;
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
  if (hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking) != hipSuccess)
    return bail(DYMU_ERR_HIP);
  if (hipHostMalloc(&d->h_sum, sizeof(int32_t) * 2, hipHostMallocDefault) != hipSuccess)
    return bail(DYMU_ERR_NOMEM);
  for (int k = 0; k < 2; ++k)
    if (hipEventCreateWithFlags(&d->ev_pack[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&d->ev_comm[k], hipEventDisableTiming) != hipSuccess)
      return bail(DYMU_ERR_HIP);
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
  if (d->comm_stream) (void)hipStreamSynchronize(d->comm_stream);
  if (d->comm) (void)ncclCommDestroy(d->comm);
  for (int k = 0; k < 2; ++k) {
    if (d->ev_pack[k]) (void)hipEventDestroy(d->ev_pack[k]);
    if (d->ev_comm[k]) (void)hipEventDestroy(d->ev_comm[k]);
  }
  pipe_free(&d->pipe);
  if (d->h_sum) (void)hipHostFree(d->h_sum);
  if (d->comm_stream) (void)hipStreamDestroy(d->comm_stream);
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
  if (pipe_alloc(&d->pipe, nx) != DYMU_OK) return fail(err, "pipe_alloc", "out of memory", DYMU_ERR_NOMEM);
  const Pipe& p = d->pipe;
  // the domain primitives and the pass-stream side of the pipeline share one
  // stream (NULL = the context's); RCCL runs on comm_stream beside it
  if (!stream) stream = dymu_get_stream(d->ctx);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipStream_t cs = d->comm_stream;
  DCALL(dymu_dom_begin(d->ctx, &s.dom, s.goal_local >= 0 ? goal_i : 0, s.goal_local, stream));
  const uint64_t cap = max_rounds(nx, ny, K);
  uint64_t m = 0;
  bool done = false;
  for (; !done; ++m) {
    if (m >= cap) {
      (void)hipStreamSynchronize(cs);
      (void)dymu_dom_finish(d->ctx, stream, nullptr);
      return fail(err, "dymu_dist_solve", "exchange-round cap reached", DYMU_ERR_NOT_CONVERGED);
    }
    const int par = (int)(m & 1);
    // pass stream: K passes | merge round m-1's rows | pack round m's rows
    DCALL(round_compute(d->ctx, s, p, m, K, st, d->ev_comm[par ^ 1]));
    DHIP(err, hipEventRecord(d->ev_pack[par], st));
    // comm stream: round m's rows to rank-1 / rank+1 and the all-reduced count,
    // in flight while round m+1's passes run
    DHIP(err, hipStreamWaitEvent(cs, d->ev_pack[par], 0));
    DNCCL(err, ncclGroupStart());
    if (s.lo) {
      DNCCL(err, ncclSend(p.s(par, 0), nx, ncclDouble, d->rank - 1, d->comm, cs));
      DNCCL(err, ncclRecv(p.r(par, 0), nx, ncclDouble, d->rank - 1, d->comm, cs));
    }
    if (s.hi) {
      DNCCL(err, ncclSend(p.s(par, 1), nx, ncclDouble, d->rank + 1, d->comm, cs));
      DNCCL(err, ncclRecv(p.r(par, 1), nx, ncclDouble, d->rank + 1, d->comm, cs));
    }
    DNCCL(err, ncclAllReduce(p.d_tot + par, p.d_sum + par, 1, ncclInt32, ncclSum, d->comm, cs));
    DNCCL(err, ncclGroupEnd());
    DHIP(err, hipMemcpyAsync(d->h_sum + par, p.d_sum + par, sizeof(int32_t),
                             hipMemcpyDeviceToHost, cs));
    DHIP(err, hipEventRecord(d->ev_comm[par], cs));
    if (m >= 1) {  // round m-1's global count; round m stays queued meanwhile
      DHIP(err, hipEventSynchronize(d->ev_comm[par ^ 1]));
      done = d->h_sum[par ^ 1] == 0;
    }
  }
  DHIP(err, hipStreamSynchronize(cs));
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
  const uint64_t cap = max_rounds(nx, ny, K);
  uint64_t m = 0;
  bool done = false;
  int rc = DYMU_OK;
  // the schedule of dymu_dist_solve, serialised on one stream: round m's rows
  // are merged after round m+1's passes
  for (; !done && rc == DYMU_OK; ++m) {
    if (m >= cap) {
      rc = DYMU_ERR_NOT_CONVERGED;
      break;
    }
    const int par = (int)(m & 1);
    for (int r = 0; r < world && rc == DYMU_OK; ++r)
      rc = round_compute(ctxs[r], s[r], p[r], m, K, st, nullptr);
    if (rc) break;
    // delivery: rank r's side-0 row -> rank r-1's side-1 receive buffer, and back
    for (int r = 0; r < world; ++r) {
      if (s[r].lo)
        DHIP(nullptr, hipMemcpyAsync(p[r].r(par, 0), p[r - 1].s(par, 1), sizeof(double) * nx,
                                     hipMemcpyDeviceToDevice, st));
      if (s[r].hi)
        DHIP(nullptr, hipMemcpyAsync(p[r].r(par, 1), p[r + 1].s(par, 0), sizeof(double) * nx,
                                     hipMemcpyDeviceToDevice, st));
      DHIP(nullptr, hipMemcpyAsync(h_tot + par * world + r, p[r].d_tot + par, sizeof(int32_t),
                                   hipMemcpyDeviceToHost, st));
    }
    DHIP(nullptr, hipEventRecord(ev[par], st));
    if (m >= 1) {
      DHIP(nullptr, hipEventSynchronize(ev[par ^ 1]));
      int64_t tot = 0;
      for (int r = 0; r < world; ++r) tot += h_tot[(par ^ 1) * world + r];
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
