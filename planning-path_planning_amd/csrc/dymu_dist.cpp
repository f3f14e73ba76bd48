// dymu_dist.cpp -- row-slab sharded solve driven from C++ (include/dymu_dist.h).
//
// ONE round loop (run_rounds) for every way the slabs can talk; a Transport
// moves the boundary rows and reduces the termination count:
//   RcclTransport     one rank per process, grouped ncclSend/ncclRecv of the
//                     boundary rows over xGMI + ncclAllReduce of the count (the
//                     bench's multi-GPU path, dymu_dist_solve)
//   IpcTransport      one rank per process, the rows pushed into the neighbours'
//                     hipIpc-mapped receive rows, the count reduced through a
//                     host shared-memory board (dymu_dist_create_ipc; runs with
//                     several ranks on ONE GPU, where RCCL refuses duplicates)
//   VirtualTransport  every rank in one process on one stream, device-to-device
//                     row copies and a device sum (dymu_vdist_solve: rehearsal)
// so the tests of the IPC and virtual transports run the loop, the pre-flight,
// the fused rounds and the mailbox posts that the RCCL bench runs.  Round m:
//   K passes (dymu_dom_round: the first pass min-merges the rows received after
//   round m-1 into the ghost rows; the second writes the round's count = tiles
//   queued for the first + for the second pass)
//   -> exchange: the first / last owned rows to rank-1 / rank+1
//   -> every kCheckEvery-th round: reduce the count over the ranks; the next
//      round's first pass posts it into the engine's host-coherent mailbox
//      (dymu_dom_post); the host reads the PREVIOUS check's post after queueing
//      this one, so the device queue never drains.
// A zero global count after a round is the fixed point: no rank had a tile
// queued after round m-1, and the rows the ranks held after round m-1 (merged
// in round m) improved no ghost row -- so every ghost row equals its
// neighbour's final row and every slab is converged against it.  The exchange
// must therefore deliver, before round m+1's merge, rows at least as new as the
// sender's state after round m: RCCL orders the receive after the send on both
// streams, the virtual copies are on the one stream, and the IPC push is
// host-synchronised per round (exchange() returns once this rank's push of
// round m completed and both neighbours have reported theirs).  The IPC receive
// rows are double-buffered by round parity, so a push never lands in the rows
// the neighbour's current round is merging: round m's push fills parity m % 2,
// round m+1's merge reads it, and the push of round m+2 into the same parity
// starts only after the neighbour reported round m+1's push -- after its round
// m+1 passes, merge included, completed.
// Kernel 3/4 slabs (no fused round) keep the v1 round: dymu_dom_run, the
// transfer, then one dymu_dom_exchange launch that merges and counts.
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

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "fim_kernels.h"
#include "peer_rule.hpp"

namespace {

// passes per round: a round costs one exchange + (every 4th round) one 4-byte
// reduction on the pass stream, and ghost rows are at most K passes stale.
// 16384^2 rehearsal (tools/vdist_rehearsal.py, max per-rank pass time, v26):
// K = 2 / 3 / 4 / 6 / 8 -> 26.6 / 26.5 / 26.4 / 27.4 / 30.4 ms at 2 ranks
// (profiles/r02/vdist_K_v26.txt).
constexpr uint32_t kDefaultK = 4;
// rounds per termination check: a zero global count after ANY round is the fixed
// point, so checking a subset of rounds is exact; the solve ends at most two
// check intervals of empty rounds later.
constexpr uint64_t kCheckEvery = 4;
// ranks of one shared-memory board / one virtual world
constexpr int kMaxWorld = 64;

int fail(std::string* err, const char* what, const char* detail, int code) {
  if (err) {
    char buf[320];
    std::snprintf(buf, sizeof buf, "%s: %s", what, detail);
    *err = buf;
  }
  return code;
}

// the arguments every rank of one solve must agree on (a rank with another grid, goal
// or K would run other rounds and leave its peers waiting), folded into 62 bits so that
// its negation is an int64 too (the RCCL pre-flight reduces min(sig) and min(-sig))
uint64_t call_signature(uint32_t nx, uint32_t ny, uint32_t gi, uint32_t gj, uint32_t K) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (uint64_t v : {(uint64_t)nx, (uint64_t)ny, (uint64_t)gi, (uint64_t)gj, (uint64_t)K}) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
  }
  return (h ^ (h >> 31)) & ((1ull << 62) - 1);
}

constexpr const char* kSigMismatch = "the ranks passed different grids, goals or K";

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

// Host waits on a peer (an event queued behind RCCL work, a board entry another
// process writes) are bounded: a peer that died or left the sequence would
// otherwise block this rank forever.  DYMU_DIST_TIMEOUT_S (default 300 s), or the
// process-wide override of dymu_dist_set_timeout (the bench's candidate tuning).
std::atomic<double> g_timeout_override{0.0};

double dist_timeout_s() {
  static const double limit_s = [] {
    const char* kv = std::getenv("DYMU_DIST_TIMEOUT_S");
    const double v = kv ? std::atof(kv) : 0.0;
    return v > 0.0 ? v : 300.0;
  }();
  const double o = g_timeout_override.load(std::memory_order_relaxed);
  return o > 0.0 ? o : limit_s;
}

// spin on cond() with a pause, then short sleeps; false after the timeout
template <class Cond>
bool spin_until(Cond&& cond) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0;; ++spin) {
    if (cond()) return true;
    if (spin > 256) std::this_thread::sleep_for(std::chrono::microseconds(20));
#if defined(__x86_64__)
    else __builtin_ia32_pause();
#endif
    if ((spin & 255) == 255 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
            dist_timeout_s())
      return false;
  }
}

int wait_event(hipEvent_t ev, std::string* err) {
  hipError_t e = hipErrorNotReady;
  const bool ok = spin_until([&] {
    e = hipEventQuery(ev);
    return e != hipErrorNotReady;
  });
  if (!ok)
    return fail(err, "dymu_dist_solve", "timed out waiting for the exchange (a peer rank failed?)",
                DYMU_ERR_RCCL);
  if (e != hipSuccess) return fail(err, "hipEventQuery", hipGetErrorString(e), DYMU_ERR_HIP);
  return DYMU_OK;
}

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

// A rank this process drives: its context, slab and receive rows (owned by the
// transport; side 0 = rank-1's last row, side 1 = rank+1's first row).
struct Local {
  dymu_ctx* ctx = nullptr;
  int rank = 0;
  Slab s;
  double* recv = nullptr;
  uint64_t cap = 0;
  double* r(int side) const { return recv + (uint64_t)side * cap; }
};

// Per-round counts live in device memory the transport owns: tot(l, par) is
// what local rank l's round writes at a check of parity par, post_src(par) the
// device word the check's mailbox post carries (the reduced count, or the local
// one when the transport reduces on the host, combine()).
class Transport {
 public:
  virtual ~Transport() = default;
  // receive rows and count words for an nx-wide grid (local; sets L[l].recv)
  virtual int alloc(std::vector<Local>& L, uint32_t nx, std::string* err) = 0;
  // collective: every rank learns whether every rank can solve, and whether every
  // rank passed the same solve signature (grid, goal, K: call_signature)
  virtual int preflight(bool ok, uint64_t sig, hipStream_t st, std::string* err) = 0;
  // collective, after a successful pre-flight: peers' buffers mapped
  virtual int connect(std::string* err) {
    (void)err;
    return DYMU_OK;
  }
  virtual int32_t* tot(int l, int par) = 0;
  virtual const int32_t* post_src(int par) = 0;
  virtual int exchange(std::vector<Local>& L, uint32_t nx, hipStream_t st, std::string* err) = 0;
  virtual int reduce(int par, hipStream_t st, std::string* err) = 0;
  virtual int combine(int32_t posted, int64_t* global, std::string* err) {
    (void)err;
    *global = posted;
    return DYMU_OK;
  }
  virtual int ranks_seen() = 0;
  // after an error inside the collective sequence (peers may be blocked)
  virtual void abort() {}
};

// pinned host words + events of the fallback checks (a context without a mailbox)
struct LoopRes {
  int32_t* h = nullptr;  // [2 parity + 1 pre-flight]
  hipEvent_t ev[2] = {nullptr, nullptr};
  int init(std::string* err) {
    if (h) return DYMU_OK;
    DHIP(err, hipHostMalloc(&h, sizeof(int32_t) * 3, hipHostMallocDefault));
    for (auto& e : ev) DHIP(err, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return DYMU_OK;
  }
  ~LoopRes() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (h) (void)hipHostFree(h);
  }
};

// ---- the round loop (the domains are live on entry) ----
// An error return leaves the collective sequence in an unknown state; the caller
// aborts the transport.
int run_rounds(std::vector<Local>& L, Transport& X, LoopRes& R, uint32_t nx, uint32_t ny,
               uint32_t K, hipStream_t st, std::string* err, uint64_t* rounds) {
  const uint64_t cap = max_rounds(nx, ny, K) + 2 * kCheckEvery;
  // fused: the rows received after round m are merged by round m+1's first pass
  // (dymu_dom_round) instead of a dymu_dom_exchange launch after the transfer
  bool fused = true;
  for (auto& l : L) fused = fused && dymu_dom_round_supported(l.ctx, K) == 1;
  dymu_ctx* mctx = L[0].ctx;  // the first local rank's mailbox carries the checks
  bool mail = true;
  uint32_t prev_seq = 0;
  uint64_t m = 0, checks = 0;
  bool done = false, have_rows = false;
  for (; !done; ++m) {
    if (m >= cap)
      return fail(err, "dymu_dist_solve", "exchange-round cap reached", DYMU_ERR_NOT_CONVERGED);
    const bool check = (m % kCheckEvery) == kCheckEvery - 1;
    const int par = (int)(checks & 1);
    for (size_t q = 0; q < L.size(); ++q) {
      const Local& l = L[q];
      const int rc =
          fused ? dymu_dom_round(l.ctx, K, have_rows && l.s.lo ? l.r(0) : nullptr,
                                 have_rows && l.s.hi ? l.r(1) : nullptr, X.tot((int)q, par), st)
                : dymu_dom_run(l.ctx, K, st);
      if (rc) return fail(err, fused ? "dymu_dom_round" : "dymu_dom_run", dymu_last_error(l.ctx), rc);
    }
    DCALL(X.exchange(L, nx, st, err));
    have_rows = true;
    if (!fused) {
      for (size_t q = 0; q < L.size(); ++q) {
        const Local& l = L[q];
        const int rc = dymu_dom_exchange(l.ctx, l.s.lo ? l.r(0) : nullptr,
                                         l.s.hi ? l.r(1) : nullptr, X.tot((int)q, par), st);
        if (rc) return fail(err, "dymu_dom_exchange", dymu_last_error(l.ctx), rc);
      }
    }
    if (!check) continue;
    DCALL(X.reduce(par, st, err));
    if (mail) {  // the next round's first pass posts the count; read the previous check's
      uint32_t seq = 0;
      const int rc = dymu_dom_post(mctx, X.post_src(par), &seq);
      if (rc == DYMU_ERR_STATE && checks == 0) {
        mail = false;
      } else if (rc) {
        return fail(err, "dymu_dom_post", dymu_last_error(mctx), rc);
      } else {
        if (checks >= 1) {
          int32_t v = 0;
          if (dymu_dom_wait_post(mctx, prev_seq, dist_timeout_s(), &v, st) != DYMU_OK)
            return fail(err, "dymu_dom_wait_post", dymu_last_error(mctx), DYMU_ERR_RCCL);
          int64_t g = 0;
          DCALL(X.combine(v, &g, err));
          done = g == 0;
        }
        prev_seq = seq;
      }
    }
    if (!mail) {
      DCALL(R.init(err));
      DHIP(err, hipMemcpyAsync(R.h + par, X.post_src(par), sizeof(int32_t), hipMemcpyDeviceToHost,
                               st));
      DHIP(err, hipEventRecord(R.ev[par], st));
      if (checks >= 1) {  // the previous check's count; this one stays queued meanwhile
        DCALL(wait_event(R.ev[par ^ 1], err));
        int64_t g = 0;
        DCALL(X.combine(R.h[par ^ 1], &g, err));
        done = g == 0;
      }
    }
    ++checks;
  }
  *rounds = m;
  return DYMU_OK;
}

// ---------------------------------------------------------------------------
// RCCL: grouped ncclSend/ncclRecv + ncclAllReduce, all on the engine's stream
// ---------------------------------------------------------------------------
class RcclTransport final : public Transport {
 public:
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  double* rbuf = nullptr;    // [2 side][cap]
  int32_t* d_cnt = nullptr;  // [2 parity][tot, sum], then the pre-flight flag
  uint64_t cap = 0;
  LoopRes pre;
  int64_t* h_pre = nullptr;  // pre-flight (ok, sig, -sig): pinned host / device
  int64_t* d_pre = nullptr;

  ~RcclTransport() override {
    if (comm) (void)ncclCommDestroy(comm);
    release();
    if (h_pre) (void)hipHostFree(h_pre);
    if (d_pre) (void)hipFree(d_pre);
  }
  void release() {
    if (rbuf) (void)hipFree(rbuf);
    if (d_cnt) (void)hipFree(d_cnt);
    rbuf = nullptr;
    d_cnt = nullptr;
    cap = 0;
  }
  int alloc(std::vector<Local>& L, uint32_t nx, std::string* err) override {
    if (cap < nx) {
      release();
      DHIP(err, hipMalloc(&rbuf, sizeof(double) * 2 * (uint64_t)nx));
      DHIP(err, hipMalloc(&d_cnt, sizeof(int32_t) * 5));
      cap = nx;
    }
    L[0].recv = rbuf;
    L[0].cap = cap;
    return DYMU_OK;
  }
  int preflight(bool ok, uint64_t sig, hipStream_t st, std::string* err) override {
    if (!h_pre) DHIP(err, hipHostMalloc(&h_pre, sizeof(int64_t) * 3, hipHostMallocDefault));
    if (!d_pre) DHIP(err, hipMalloc(&d_pre, sizeof(int64_t) * 3));
    DCALL(pre.init(err));
    // min over ranks of (ok, sig, -sig): every rank ok, and min(sig) == max(sig)
    h_pre[0] = ok ? 1 : 0;
    h_pre[1] = (int64_t)sig;
    h_pre[2] = -(int64_t)sig;
    DHIP(err, hipMemcpyAsync(d_pre, h_pre, sizeof(int64_t) * 3, hipMemcpyHostToDevice, st));
    DNCCL(err, ncclAllReduce(d_pre, d_pre, 3, ncclInt64, ncclMin, comm, st));
    DHIP(err, hipMemcpyAsync(h_pre, d_pre, sizeof(int64_t) * 3, hipMemcpyDeviceToHost, st));
    DHIP(err, hipEventRecord(pre.ev[0], st));
    DCALL(wait_event(pre.ev[0], err));
    if (h_pre[0] != 1)
      return fail(err, "dymu_dist_solve", ok ? "another rank rejected its slab" : "invalid slab",
                  DYMU_ERR_ARG);
    if (h_pre[1] != -h_pre[2]) return fail(err, "dymu_dist_solve", kSigMismatch, DYMU_ERR_ARG);
    return DYMU_OK;
  }
  int32_t* tot(int, int par) override { return d_cnt + 2 * par; }
  const int32_t* post_src(int par) override { return d_cnt + 2 * par + 1; }
  int exchange(std::vector<Local>& L, uint32_t nx, hipStream_t st, std::string* err) override {
    const Local& l = L[0];
    if (!l.s.lo && !l.s.hi) return DYMU_OK;
    DNCCL(err, ncclGroupStart());
    if (l.s.lo) {
      DNCCL(err, ncclSend(l.s.row(0), nx, ncclDouble, rank - 1, comm, st));
      DNCCL(err, ncclRecv(l.r(0), nx, ncclDouble, rank - 1, comm, st));
    }
    if (l.s.hi) {
      DNCCL(err, ncclSend(l.s.row(1), nx, ncclDouble, rank + 1, comm, st));
      DNCCL(err, ncclRecv(l.r(1), nx, ncclDouble, rank + 1, comm, st));
    }
    DNCCL(err, ncclGroupEnd());
    return DYMU_OK;
  }
  int reduce(int par, hipStream_t st, std::string* err) override {
    DNCCL(err, ncclAllReduce(d_cnt + 2 * par, d_cnt + 2 * par + 1, 1, ncclInt32, ncclSum, comm, st));
    return DYMU_OK;
  }
  int ranks_seen() override {
    int n = 0;
    return comm && ncclCommCount(comm, &n) == ncclSuccess ? n : 0;
  }
  void abort() override {
    if (comm) (void)ncclCommAbort(comm);
    comm = nullptr;
  }
};

// ---------------------------------------------------------------------------
// The shared-memory board of the IPC and peer transports: one POSIX shared-memory
// segment (/dev/shm) per communicator, one slot per rank.  Joining, the collective
// pre-flight, the receive buffers' IPC handles, the per-check status and the abort
// flag go through it; every host wait on it is bounded (DYMU_DIST_TIMEOUT_S) and
// gives up at once when a rank has aborted.
// ---------------------------------------------------------------------------
struct BoardSlot {
  std::atomic<uint64_t> gen;       // generation of the published receive buffer
  std::atomic<uint64_t> cap;       // its elements per side
  std::atomic<uint64_t> pre[2];    // (solve << 1) | ok, in slot solve % 2
  std::atomic<uint64_t> sig[2];    // call_signature of that solve (stored before pre)
  std::atomic<uint64_t> pushed;    // IPC: rounds whose push completed (running count)
  std::atomic<uint64_t> check[4];  // IPC: ((check + 1) << 32) | count, slot check % 4
  std::atomic<uint64_t> joined;    // 1 once the rank opened the board
  std::atomic<uint64_t> aborted;   // 1 once the rank gave up the collective sequence
  // peer: the status of check c in slot c % 4 -- P, S0, S1, R0, R1, then the tag
  // (solve << 32) | (c + 1), stored last (release)
  std::atomic<uint64_t> stat[4][6];
  unsigned char handle[HIP_IPC_HANDLE_SIZE];
  unsigned char pad[512 - 37 * 8 - HIP_IPC_HANDLE_SIZE];
};
static_assert(sizeof(BoardSlot) == 512, "board slot");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "board atomics");

class BoardTransport : public Transport {
 public:
  int rank = 0, world = 1;
  std::string name;
  bool owner = false;
  BoardSlot* board = nullptr;
  size_t board_bytes = 0;
  uint64_t solves = 0;
  // the exported receive buffer and the neighbours' (mapped)
  void* exported = nullptr;
  uint64_t cap = 0, gen = 0;
  void* peer[2] = {nullptr, nullptr};  // rank-1's / rank+1's exported buffer
  uint64_t peer_gen[2] = {0, 0}, peer_cap[2] = {0, 0};

  ~BoardTransport() override {
    for (auto& p : peer)
      if (p) (void)hipIpcCloseMemHandle(p);
    if (board) munmap(board, board_bytes);
    if (owner && !name.empty()) shm_unlink(name.c_str());
  }
  // spin_until that also gives up as soon as any rank has aborted (its abort() after
  // an error): the peers fail at once instead of after the full timeout
  bool peer_aborted() const {
    for (int q = 0; q < world; ++q)
      if (board[q].aborted.load(std::memory_order_acquire)) return true;
    return false;
  }
  template <class Cond>
  int wait(Cond&& cond, const char* what, std::string* err) {
    bool gone = false;
    const bool ok = spin_until([&] {
      if (cond()) return true;
      gone = peer_aborted();
      return gone;
    });
    if (gone) return fail(err, "dymu_dist_solve", "a peer rank aborted the solve", DYMU_ERR_RCCL);
    if (!ok) return fail(err, "dymu_dist_solve", what, DYMU_ERR_RCCL);
    return DYMU_OK;
  }
  void abort() override {
    if (board) board[rank].aborted.store(1, std::memory_order_release);
  }
  int open(const char* shm, int r, int w, std::string* err) {
    rank = r;
    world = w;
    name = shm;
    owner = r == 0;
    board_bytes = sizeof(BoardSlot) * kMaxWorld;
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return fail(err, "shm_open", std::strerror(errno), DYMU_ERR_STATE);
    if (ftruncate(fd, (off_t)board_bytes) != 0) {
      close(fd);
      return fail(err, "ftruncate", std::strerror(errno), DYMU_ERR_STATE);
    }
    void* p = mmap(nullptr, board_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return fail(err, "mmap", std::strerror(errno), DYMU_ERR_STATE);
    board = static_cast<BoardSlot*>(p);
    DCALL(open_local(err));
    // collective, like ncclCommInitRank: every rank has joined on return
    board[rank].joined.store(1, std::memory_order_release);
    for (int q = 0; q < world; ++q)
      if (!spin_until([&] { return board[q].joined.load(std::memory_order_acquire) != 0; }))
        return fail(err, "dymu_dist_create", "timed out waiting for the other ranks",
                    DYMU_ERR_RCCL);
    return DYMU_OK;
  }
  virtual int open_local(std::string* err) = 0;
  int preflight(bool ok, uint64_t sig, hipStream_t, std::string* err) override {
    // One slot per solve parity: a rank that leaves this pre-flight may post the next
    // solve's before a slower peer has read this one's ok bit, and a single slot would
    // hand that peer the NEXT solve's bit (a rejected slab read as accepted: the other
    // ranks then entered the rounds of a solve the rejecting rank had abandoned).  A
    // rank cannot get two solves ahead (the next pre-flight waits for every rank's post).
    const uint64_t s = ++solves;
    board[rank].sig[s & 1].store(sig, std::memory_order_relaxed);
    board[rank].pre[s & 1].store((s << 1) | (ok ? 1u : 0u), std::memory_order_release);
    bool all = true, same = true;
    for (int q = 0; q < world; ++q) {
      uint64_t v = 0;
      const uint64_t seen0 = std::max(board[q].pre[0].load() >> 1, board[q].pre[1].load() >> 1);
      const std::string why = "timed out in the pre-flight of solve " + std::to_string(s) +
                              " waiting for rank " + std::to_string(q) + " (at solve " +
                              std::to_string(seen0) + "; a peer rank failed?)";
      DCALL(wait([&] {
              v = board[q].pre[s & 1].load(std::memory_order_acquire);
              return (v >> 1) >= s;
            }, why.c_str(), err));
      all = all && (v & 1u);
      same = same && board[q].sig[s & 1].load(std::memory_order_relaxed) == sig;
    }
    if (!all)
      return fail(err, "dymu_dist_solve", ok ? "another rank rejected its slab" : "invalid slab",
                  DYMU_ERR_ARG);
    if (!same) return fail(err, "dymu_dist_solve", kSigMismatch, DYMU_ERR_ARG);
    return DYMU_OK;
  }
  // publish `exported` (generation gen, cap elements per side) if it is new, and map
  // both neighbours' current buffers
  int connect(std::string* err) override {
    if (board[rank].gen.load(std::memory_order_acquire) != gen) {  // publish a new buffer
      hipIpcMemHandle_t h;
      DHIP(err, hipIpcGetMemHandle(&h, exported));
      std::memcpy(board[rank].handle, &h, sizeof h);
      board[rank].cap.store(cap, std::memory_order_relaxed);
      board[rank].gen.store(gen, std::memory_order_release);
    }
    for (int side = 0; side < 2; ++side) {
      const int q = side == 0 ? rank - 1 : rank + 1;
      if (q < 0 || q >= world) continue;
      // every rank allocates after the same accepted pre-flights (the signature pins nx):
      // the same generation
      DCALL(wait([&] { return board[q].gen.load(std::memory_order_acquire) >= gen; },
                 "timed out waiting for a peer's receive rows", err));
      const uint64_t g = board[q].gen.load(std::memory_order_acquire);
      if (g == peer_gen[side] && peer[side]) continue;
      if (peer[side]) DHIP(err, hipIpcCloseMemHandle(peer[side]));
      peer[side] = nullptr;
      hipIpcMemHandle_t h;
      std::memcpy(&h, board[q].handle, sizeof h);
      void* p = nullptr;
      DHIP(err, hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peer[side] = p;
      peer_gen[side] = g;
      peer_cap[side] = board[q].cap.load(std::memory_order_relaxed);
    }
    return DYMU_OK;
  }
  int ranks_seen() override {  // ranks that joined the board
    int n = 0;
    for (int q = 0; q < kMaxWorld; ++q) n += board[q].joined.load(std::memory_order_acquire) ? 1 : 0;
    return n;
  }
};

// ---------------------------------------------------------------------------
// IPC: rows pushed into the neighbours' hipIpc-mapped receive rows, counts
// reduced through the board; one node, any number of ranks per GPU.  Per round
// the host waits for its own push and for both neighbours' (the exactness
// condition in the header comment); the reduction is a host sum over the board.
// ---------------------------------------------------------------------------
class IpcTransport final : public BoardTransport {
 public:
  double* recv = nullptr;  // [2 parity][2 side][cap], exported
  int32_t* d_cnt = nullptr;  // [2 parity] local counts
  uint64_t rounds = 0, checks = 0;
  hipEvent_t ev = nullptr;

  ~IpcTransport() override {
    for (auto& p : peer)
      if (p) (void)hipIpcCloseMemHandle(p);
    peer[0] = peer[1] = nullptr;
    if (recv) (void)hipFree(recv);
    if (d_cnt) (void)hipFree(d_cnt);
    if (ev) (void)hipEventDestroy(ev);
  }
  int open_local(std::string* err) override {
    DHIP(err, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    DHIP(err, hipMalloc(&d_cnt, sizeof(int32_t) * 2));
    return DYMU_OK;
  }
  int alloc(std::vector<Local>& L, uint32_t nx, std::string* err) override {
    if (cap < nx) {
      if (recv) DHIP(err, hipFree(recv));
      recv = nullptr;
      exported = nullptr;
      cap = 0;
      DHIP(err, hipMalloc(&recv, sizeof(double) * 4 * (uint64_t)nx));
      exported = recv;
      cap = nx;
      ++gen;
    }
    L[0].recv = recv + (rounds & 1) * 2 * cap;  // the parity the next merge reads
    L[0].cap = cap;
    return DYMU_OK;
  }
  int32_t* tot(int, int par) override { return d_cnt + par; }
  const int32_t* post_src(int par) override { return d_cnt + par; }
  int exchange(std::vector<Local>& L, uint32_t nx, hipStream_t st, std::string* err) override {
    Local& l = L[0];
    double* const p0 = static_cast<double*>(peer[0]);
    double* const p1 = static_cast<double*>(peer[1]);
    // push: my first row into rank-1's "from rank+1" row, my last into rank+1's
    // "from rank-1" row (ordered after this round's passes on my stream), both in
    // the receive parity of this round
    const uint64_t par = rounds & 1;
    if (l.s.lo)
      DHIP(err, hipMemcpyAsync(p0 + (2 * par + 1) * peer_cap[0], l.s.row(0), sizeof(double) * nx,
                               hipMemcpyDeviceToDevice, st));
    if (l.s.hi)
      DHIP(err, hipMemcpyAsync(p1 + 2 * par * peer_cap[1], l.s.row(1), sizeof(double) * nx,
                               hipMemcpyDeviceToDevice, st));
    const uint64_t m = ++rounds;
    l.recv = recv + par * 2 * cap;  // the next round merges what the neighbours pushed now
    if (!l.s.lo && !l.s.hi) return DYMU_OK;
    DHIP(err, hipEventRecord(ev, st));
    DCALL(wait_event(ev, err));
    board[rank].pushed.store(m, std::memory_order_release);
    for (int side = 0; side < 2; ++side) {
      const int q = side == 0 ? rank - 1 : rank + 1;
      if ((side == 0 && !l.s.lo) || (side == 1 && !l.s.hi)) continue;
      DCALL(wait([&] { return board[q].pushed.load(std::memory_order_acquire) >= m; },
                 "timed out waiting for a neighbour's rows", err));
    }
    return DYMU_OK;
  }
  int reduce(int, hipStream_t, std::string*) override { return DYMU_OK; }
  int combine(int32_t posted, int64_t* global, std::string* err) override {
    const uint64_t c = checks++;
    const uint64_t tag = (c + 1) << 32;
    board[rank].check[c % 4].store(tag | (uint32_t)posted, std::memory_order_release);
    int64_t g = 0;
    for (int q = 0; q < world; ++q) {
      uint64_t v = 0;
      DCALL(wait([&] {
              v = board[q].check[c % 4].load(std::memory_order_acquire);
              return (v >> 32) >= c + 1;
            }, "timed out in the count reduction", err));
      g += (int64_t)(uint32_t)v;
    }
    *global = g;
    return DYMU_OK;
  }
};

// ---------------------------------------------------------------------------
// Peer: GPU-initiated pushes, no host step per round (DESIGN.md s5 "Peer
// transport").  Every round's first pass pushes the decreased values of this
// rank's boundary rows straight into the neighbours' receive rows (peer-mapped,
// over xGMI between GPUs) and then a per-link sequence tag; the merge of the same
// pass reads this rank's receive rows after their tags (dymu_dom_round_peer).
// Nothing waits for a neighbour: the host queues rounds back to back, and every
// kCheckEvery-th round posts the status of the round before (P: tiles queued;
// per link S: pushes that carried a decrease, R: the tag merged) into a
// host-coherent ring, which the host copies onto the board one check late.
// Termination (every rank decides alike from the same board entries): two
// consecutive checks c-1, c in which every rank had P = 0, every link had R = S,
// and no S moved between them.  Then every change ever made reached a boundary
// row, was pushed (P = 0 means the round did nothing after its push), merged (R =
// S) and improved nothing (P = 0 again), and nothing was pushed since -- the
// global fixed point, checked like RCCL's zero count but without a collective.
// The receive rows and tags live in fine-grained device memory
// (hipDeviceMallocFinegrained: coherent while kernels run) and are read with
// system-scope loads.
// ---------------------------------------------------------------------------
class PeerTransport final : public BoardTransport {
 public:
  // exported: [2 side][cap] receive rows, then 2 tags (own 128-byte line)
  double* rx = nullptr;
  unsigned long long* rtag = nullptr;
  double* last = nullptr;      // [2 side][cap], local
  void* ctl = nullptr;         // PeerCtl, local
  unsigned long long* ring = nullptr;    // [kRing][8] words, host-coherent pinned
  unsigned long long* d_ring = nullptr;  // its device address
  static constexpr int kRing = 8;
  bool fine = true;  // fine-grained receive rows (DYMU_PEER_COARSE=1: hipMalloc, A/B)

  static uint64_t rx_bytes(uint64_t n) { return (sizeof(double) * 2 * n + 127) / 128 * 128 + 128; }
  ~PeerTransport() override {
    for (auto& p : peer)
      if (p) (void)hipIpcCloseMemHandle(p);
    peer[0] = peer[1] = nullptr;
    if (rx) (void)hipFree(rx);
    if (last) (void)hipFree(last);
    if (ctl) (void)hipFree(ctl);
    if (ring) (void)hipHostFree(ring);
  }
  int open_local(std::string* err) override {
    if (const char* kv = std::getenv("DYMU_PEER_COARSE")) fine = std::atoi(kv) == 0;
    DHIP(err, hipMalloc(&ctl, DYMU_PEER_CTL_BYTES));
    DHIP(err, hipHostMalloc(&ring, sizeof(unsigned long long) * 8 * kRing,
                            hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(ring, 0, sizeof(unsigned long long) * 8 * kRing);
    void* d = nullptr;
    DHIP(err, hipHostGetDevicePointer(&d, ring, 0));
    d_ring = static_cast<unsigned long long*>(d);
    return DYMU_OK;
  }
  int alloc(std::vector<Local>& L, uint32_t nx, std::string* err) override {
    if (cap < nx) {
      if (rx) DHIP(err, hipFree(rx));
      if (last) DHIP(err, hipFree(last));
      rx = nullptr;
      last = nullptr;
      exported = nullptr;
      cap = 0;
      void* p = nullptr;
      if (fine)
        DHIP(err, hipExtMallocWithFlags(&p, rx_bytes(nx), hipDeviceMallocFinegrained));
      else
        DHIP(err, hipMalloc(&p, rx_bytes(nx)));
      rx = static_cast<double*>(p);
      DHIP(err, hipMalloc(&last, sizeof(double) * 2 * (uint64_t)nx));
      exported = rx;
      cap = nx;
      ++gen;
    }
    rtag = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(rx) + rx_bytes(cap) - 128);
    L[0].recv = rx;
    L[0].cap = cap;
    return DYMU_OK;
  }
  // before the pre-flight (so no neighbour can push into them yet): receive rows and
  // the values last pushed +inf, tags 0, counters 0 (rmin all ones)
  int reset(hipStream_t st, std::string* err) {
    DHIP(err, dymu::launch_fill_inf(rx, 0, (uint32_t)(2 * cap), 0, 1, st));
    DHIP(err, hipMemsetAsync(rtag, 0, 128, st));
    DHIP(err, dymu::launch_fill_inf(last, 0, (uint32_t)(2 * cap), 0, 1, st));
    DHIP(err, hipMemsetAsync(ctl, 0, DYMU_PEER_CTL_BYTES, st));
    DHIP(err, hipMemsetAsync(static_cast<char*>(ctl) + offsetof(dymu::PeerCtl, rmin), 0xFF,
                             2 * sizeof(unsigned long long), st));
    DHIP(err, hipStreamSynchronize(st));
    return DYMU_OK;
  }
  // after connect(): every rank has reset its buffers before any rank starts pushing
  // (a board barrier: the pushes of this solve follow it)
  int ready(hipStream_t st, std::string* err) {
    DCALL(reset(st, err));
    board[rank].pushed.store(solves, std::memory_order_release);
    for (int q = 0; q < world; ++q)
      DCALL(wait([&] { return board[q].pushed.load(std::memory_order_acquire) >= solves; },
                 "timed out waiting for the peers to reset", err));
    return DYMU_OK;
  }
  int32_t* tot(int, int) override { return nullptr; }
  const int32_t* post_src(int) override { return nullptr; }
  int exchange(std::vector<Local>&, uint32_t, hipStream_t, std::string*) override { return DYMU_OK; }
  int reduce(int, hipStream_t, std::string*) override { return DYMU_OK; }

  using Status = dymu_peer::Status;
  // the rounds; the domain is live on entry
  int run(Local& l, uint32_t nx, uint32_t ny, uint32_t K, hipStream_t st, std::string* err,
          uint64_t* rounds_out) {
    dymu_peer_links links{};
    for (int side = 0; side < 2; ++side) {
      const bool has = side == 0 ? l.s.lo : l.s.hi;
      if (!has) continue;
      links.recv[side] = rx + (uint64_t)side * cap;
      links.recv_tag[side] = rtag + side;
      // my first row goes into rank-1's "from rank+1" row (side 1 of its buffer), my
      // last into rank+1's "from rank-1" row (side 0)
      double* pb = static_cast<double*>(peer[side]);
      const uint64_t pc = peer_cap[side];
      links.send[side] = pb + (side == 0 ? pc : 0);
      links.send_tag[side] = reinterpret_cast<unsigned long long*>(
                                 reinterpret_cast<char*>(pb) + rx_bytes(pc) - 128) +
                             (side == 0 ? 1 : 0);
      links.last[side] = last + (uint64_t)side * cap;
    }
    links.ctl = ctl;
    const uint64_t cap_r = max_rounds(nx, ny, K) + 2 * kCheckEvery;
    const uint64_t solve = solves;
    std::vector<Status> prev(world), cur(world);
    bool prev_quiet = false;
    uint64_t checks = 0, m = 0;
    for (bool done = false; !done; ++m) {
      if (m >= cap_r)
        return fail(err, "dymu_dist_solve", "exchange-round cap reached", DYMU_ERR_NOT_CONVERGED);
      int rc = dymu_dom_round_peer(l.ctx, K, &links, st);
      if (rc) return fail(err, "dymu_dom_round_peer", dymu_last_error(l.ctx), rc);
      if ((m % kCheckEvery) != kCheckEvery - 1) continue;
      // this round's status is posted by the next launched pass into ring slot c
      const uint64_t c = checks++;
      unsigned long long* slot = ring + (c % kRing) * 8;
      __atomic_store_n(slot, 0ull, __ATOMIC_RELEASE);
      rc = dymu_dom_post_status(l.ctx, ctl, d_ring + (c % kRing) * 8, (uint32_t)(c + 1));
      if (rc) return fail(err, "dymu_dom_post_status", dymu_last_error(l.ctx), rc);
      if (c == 0) continue;
      // the previous check's status (its post ran at the start of this round)
      const uint64_t k = c - 1;
      unsigned long long* ps = ring + (k % kRing) * 8;
      uint64_t w0 = 0;
      DCALL(wait([&] {
              w0 = __atomic_load_n(ps, __ATOMIC_ACQUIRE);
              return (w0 >> 32) == k + 1;
            }, "timed out waiting for the device's status post", err));
      BoardSlot& me = board[rank];
      me.stat[k % 4][0].store((uint32_t)w0, std::memory_order_relaxed);
      for (int q = 0; q < 4; ++q)
        me.stat[k % 4][1 + q].store(__atomic_load_n(ps + 1 + q, __ATOMIC_RELAXED),
                                    std::memory_order_relaxed);
      me.stat[k % 4][5].store((solve << 32) | (k + 1), std::memory_order_release);
      for (int q = 0; q < world; ++q) {
        DCALL(wait([&] { return board[q].stat[k % 4][5].load(std::memory_order_acquire) ==
                                ((solve << 32) | (k + 1)); },
                   "timed out waiting for a peer's status", err));
        Status& sq = cur[q];
        sq.P = board[q].stat[k % 4][0].load(std::memory_order_relaxed);
        for (int side = 0; side < 2; ++side) {
          sq.S[side] = board[q].stat[k % 4][1 + side].load(std::memory_order_relaxed);
          sq.R[side] = board[q].stat[k % 4][3 + side].load(std::memory_order_relaxed);
        }
      }
      done = dymu_peer::done(prev, prev_quiet, cur);  // csrc/peer_rule.hpp
      prev_quiet = dymu_peer::quiet(cur);
      prev.swap(cur);
    }
    *rounds_out = m;
    return DYMU_OK;
  }
};

// ---------------------------------------------------------------------------
// Virtual ranks: every rank in this process, one stream; D2D copies for the
// rows, the count summed on the device (k_sum_counts over 16 words per parity)
// ---------------------------------------------------------------------------
class VirtualTransport final : public Transport {
 public:
  std::vector<double*> rows;
  uint32_t* cnt = nullptr;  // [2 parity][16]: tot of local rank l at [par][l]
  int32_t* sum = nullptr;   // [2 parity]

  ~VirtualTransport() override {
    for (double* p : rows)
      if (p) (void)hipFree(p);
    if (cnt) (void)hipFree(cnt);
    if (sum) (void)hipFree(sum);
  }
  int alloc(std::vector<Local>& L, uint32_t nx, std::string* err) override {
    if ((int)L.size() > dymu::kShards)
      return fail(err, "dymu_vdist_solve", "at most 16 virtual ranks", DYMU_ERR_ARG);
    rows.assign(L.size(), nullptr);
    for (size_t q = 0; q < L.size(); ++q) {
      DHIP(err, hipMalloc(&rows[q], sizeof(double) * 2 * (uint64_t)nx));
      L[q].recv = rows[q];
      L[q].cap = nx;
    }
    DHIP(err, hipMalloc(&cnt, sizeof(uint32_t) * 2 * dymu::kShards));
    DHIP(err, hipMemset(cnt, 0, sizeof(uint32_t) * 2 * dymu::kShards));
    DHIP(err, hipMalloc(&sum, sizeof(int32_t) * 2));
    return DYMU_OK;
  }
  int preflight(bool ok, uint64_t, hipStream_t, std::string* err) override {
    return ok ? DYMU_OK : fail(err, "dymu_vdist_solve", "invalid slab", DYMU_ERR_ARG);
  }
  int32_t* tot(int l, int par) override {
    return reinterpret_cast<int32_t*>(cnt + par * dymu::kShards + l);
  }
  const int32_t* post_src(int par) override { return sum + par; }
  int exchange(std::vector<Local>& L, uint32_t nx, hipStream_t st, std::string* err) override {
    for (size_t q = 0; q < L.size(); ++q) {  // rank q-1's last row / rank q+1's first row
      if (L[q].s.lo)
        DHIP(err, hipMemcpyAsync(L[q].r(0), L[q - 1].s.row(1), sizeof(double) * nx,
                                 hipMemcpyDeviceToDevice, st));
      if (L[q].s.hi)
        DHIP(err, hipMemcpyAsync(L[q].r(1), L[q + 1].s.row(0), sizeof(double) * nx,
                                 hipMemcpyDeviceToDevice, st));
    }
    return DYMU_OK;
  }
  int reduce(int par, hipStream_t st, std::string* err) override {
    DHIP(err, dymu::launch_sum_counts(cnt + par * dymu::kShards, sum + par, st));
    return DYMU_OK;
  }
  int ranks_seen() override { return (int)rows.size(); }
};

}  // namespace

struct dymu_dist {
  dymu_ctx* ctx = nullptr;
  int device = 0;
  int rank = 0, world = 1;
  int kind = DYMU_DIST_RCCL;
  std::unique_ptr<Transport> xp;
  LoopRes res;
  bool aborted = false;  // the transport was aborted after an error (no further solves)
  std::string last_error;
};

namespace {

// After an error inside the collective sequence: abort the transport (its peers
// may be blocked in an exchange this rank will never post; they are released by
// their own wait timeout), and refuse further solves on this handle.
int abort_dist(dymu_dist* d, int rc) {
  if (d->xp) d->xp->abort();
  d->aborted = true;
  return rc;
}

dymu_dist* new_dist(dymu_ctx* ctx, int device, int rank, int world, int kind) {
  auto* d = new dymu_dist;
  d->ctx = ctx;
  d->device = device;
  d->rank = rank;
  d->world = world;
  d->kind = kind;
  return d;
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
  dymu_dist* d = new_dist(ctx, device, rank, world, DYMU_DIST_RCCL);
  auto bail = [&](int rc) {
    dymu_dist_destroy(d);
    return rc;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(DYMU_ERR_HIP);
  auto x = std::make_unique<RcclTransport>();
  x->rank = rank;
  x->world = world;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  if (ncclCommInitRank(&x->comm, world, u, rank) != ncclSuccess) {
    x->comm = nullptr;
    return bail(DYMU_ERR_RCCL);
  }
  d->xp = std::move(x);
  *out = d;
  return DYMU_OK;
}

int dymu_dist_ipc_unique_id(unsigned char id[DYMU_DIST_ID_BYTES]) {
  if (!id) return DYMU_ERR_ARG;
  std::random_device rd;
  char name[64];
  std::snprintf(name, sizeof name, "/dymu_ipc_%d_%08x%08x", (int)getpid(), (unsigned)rd(),
                (unsigned)rd());
  std::memset(id, 0, DYMU_DIST_ID_BYTES);
  std::memcpy(id, name, std::strlen(name));
  return DYMU_OK;
}

int dymu_dist_create_ipc(dymu_dist** out, dymu_ctx* ctx, int device,
                         const unsigned char id[DYMU_DIST_ID_BYTES], int rank, int world) {
  if (!out || !ctx || !id || world < 1 || world > kMaxWorld || rank < 0 || rank >= world)
    return DYMU_ERR_ARG;
  *out = nullptr;
  char name[DYMU_DIST_ID_BYTES + 1];
  std::memcpy(name, id, DYMU_DIST_ID_BYTES);
  name[DYMU_DIST_ID_BYTES] = 0;
  if (name[0] != '/' || std::strchr(name + 1, '/')) return DYMU_ERR_ARG;
  dymu_dist* d = new_dist(ctx, device, rank, world, DYMU_DIST_IPC);
  if (hipSetDevice(device) != hipSuccess) {
    dymu_dist_destroy(d);
    return DYMU_ERR_HIP;
  }
  auto x = std::make_unique<IpcTransport>();
  const int rc = x->open(name, rank, world, &d->last_error);
  d->xp = std::move(x);
  if (rc) {
    dymu_dist_destroy(d);
    return rc;
  }
  *out = d;
  return DYMU_OK;
}

int dymu_dist_create_peer(dymu_dist** out, dymu_ctx* ctx, int device,
                          const unsigned char id[DYMU_DIST_ID_BYTES], int rank, int world) {
  if (!out || !ctx || !id || world < 1 || world > kMaxWorld || rank < 0 || rank >= world)
    return DYMU_ERR_ARG;
  *out = nullptr;
  char name[DYMU_DIST_ID_BYTES + 1];
  std::memcpy(name, id, DYMU_DIST_ID_BYTES);
  name[DYMU_DIST_ID_BYTES] = 0;
  if (name[0] != '/' || std::strchr(name + 1, '/')) return DYMU_ERR_ARG;
  dymu_dist* d = new_dist(ctx, device, rank, world, DYMU_DIST_PEER);
  if (hipSetDevice(device) != hipSuccess) {
    dymu_dist_destroy(d);
    return DYMU_ERR_HIP;
  }
  auto x = std::make_unique<PeerTransport>();
  const int rc = x->open(name, rank, world, &d->last_error);
  d->xp = std::move(x);
  if (rc) {
    dymu_dist_destroy(d);
    return rc;
  }
  *out = d;
  return DYMU_OK;
}

int dymu_dist_destroy(dymu_dist* d) {
  if (!d) return DYMU_OK;
  (void)hipSetDevice(d->device);
  d->xp.reset();
  delete d;
  return DYMU_OK;
}

const char* dymu_dist_last_error(dymu_dist* d) { return d ? d->last_error.c_str() : ""; }

int dymu_dist_transport(dymu_dist* d) { return d ? d->kind : DYMU_ERR_ARG; }

double dymu_dist_set_timeout(double seconds) {
  const double prev = g_timeout_override.exchange(seconds > 0.0 ? seconds : 0.0);
  (void)prev;
  return dist_timeout_s();
}

int dymu_dist_comm_count(dymu_dist* d, int* ranks) {
  if (!d || !ranks) return DYMU_ERR_ARG;
  if (!d->xp || d->aborted) return DYMU_ERR_STATE;
  const int n = d->xp->ranks_seen();
  if (n <= 0) return DYMU_ERR_RCCL;
  *ranks = n;
  return DYMU_OK;
}

int dymu_dist_solve(dymu_dist* d, const double* F_slab, double* T_buf, uint64_t ld, uint32_t nx,
                    uint32_t ny, uint32_t goal_i, uint32_t goal_j, uint32_t K, void* stream,
                    dymu_stats* stats) {
  if (!d) return DYMU_ERR_ARG;
  std::string* err = &d->last_error;
  if (d->aborted || !d->xp)
    return fail(err, "dymu_dist_solve", "transport aborted by an earlier error", DYMU_ERR_STATE);
  if (K == 0) K = kDefaultK;
  DHIP(err, hipSetDevice(d->device));
  // the transport and the domain primitives share one stream: NULL = the context's
  if (!stream) stream = dymu_get_stream(d->ctx);
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<Local> L(1);
  L[0].ctx = d->ctx;
  L[0].rank = d->rank;
  bool ok = nx > 0 && ny > 0 && goal_i < nx && goal_j < ny &&
            make_slab(F_slab, T_buf, ld, nx, ny, goal_j, d->rank, d->world, &L[0].s) == DYMU_OK;
  // the peer transport runs fused kernel-5 rounds (K >= 2, not deterministic): an
  // unsupported solve is an argument error on every rank, before any collective
  // state changes, so the communicator stays usable
  const bool peer_ok = d->kind != DYMU_DIST_PEER || !ok ||
                       dymu_dom_round_capable(d->ctx, nx, L[0].s.dom.nrows, K) == 1;
  ok = ok && peer_ok;
  int rc = d->xp->preflight(ok, call_signature(nx, ny, goal_i, goal_j, K), st, err);
  if (rc == DYMU_ERR_ARG && !peer_ok)
    return fail(err, "dymu_dist_solve",
                "the peer transport needs kernel-5 slabs, K >= 2 and a non-deterministic engine",
                DYMU_ERR_ARG);
  if (rc) return rc == DYMU_ERR_ARG ? rc : abort_dist(d, rc);
  // receive rows only after every rank accepted this solve (its signature pins nx): a
  // rank whose arguments were rejected must not re-allocate (and re-publish) alone, or
  // the next valid solve would wait for a buffer generation its peers never reach
  if (d->xp->alloc(L, nx, err) != DYMU_OK)
    return abort_dist(d, fail(err, "dymu_dist_solve", "receive rows: out of memory",
                              DYMU_ERR_NOMEM));
  rc = d->xp->connect(err);
  if (rc) return abort_dist(d, rc);
  auto* peer = d->kind == DYMU_DIST_PEER ? static_cast<PeerTransport*>(d->xp.get()) : nullptr;
  if (peer && (rc = peer->ready(st, err)) != DYMU_OK) return abort_dist(d, rc);
  const Slab& s = L[0].s;
  rc = dymu_dom_begin(d->ctx, &s.dom, s.goal_local >= 0 ? goal_i : 0, s.goal_local, stream);
  if (rc) return abort_dist(d, fail(err, "dymu_dom_begin", dymu_last_error(d->ctx), rc));
  if (peer && dymu_dom_round_supported(d->ctx, K) != 1) {
    (void)dymu_dom_finish(d->ctx, stream, nullptr);
    return abort_dist(d, fail(err, "dymu_dist_solve",
                              "the peer transport needs kernel-5 slabs and K >= 2", DYMU_ERR_STATE));
  }
  uint64_t rounds = 0;
  rc = peer ? peer->run(L[0], nx, ny, K, st, err, &rounds)
            : run_rounds(L, *d->xp, d->res, nx, ny, K, st, err, &rounds);
  const int rf = dymu_dom_finish(d->ctx, stream, stats);
  if (rc) return abort_dist(d, rc);
  if (rf) return abort_dist(d, fail(err, "dymu_dom_finish", dymu_last_error(d->ctx), rf));
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
  std::vector<Local> L(world);
  for (int r = 0; r < world; ++r) {
    if (!ctxs[r]) return DYMU_ERR_ARG;
    L[r].ctx = ctxs[r];
    L[r].rank = r;
    DCALL(make_slab(F_slabs[r], T_bufs[r], ld, nx, ny, goal_j, r, world, &L[r].s));
  }
  VirtualTransport X;
  LoopRes R;
  std::string err;
  DCALL(X.alloc(L, nx, &err));
  DCALL(X.preflight(true, call_signature(nx, ny, goal_i, goal_j, K), st, &err));
  for (int r = 0; r < world; ++r)
    DCALL(dymu_dom_begin(ctxs[r], &L[r].s.dom, L[r].s.goal_local >= 0 ? goal_i : 0,
                         L[r].s.goal_local, stream));
  uint64_t rounds = 0;
  int rc = run_rounds(L, X, R, nx, ny, K, st, &err, &rounds);
  if (rc && std::getenv("DYMU_DIST_DEBUG")) std::fprintf(stderr, "dymu_vdist_solve: %s\n", err.c_str());
  for (int r = 0; r < world; ++r) {
    dymu_stats tmp;
    const int rf = dymu_dom_finish(ctxs[r], stream, stats ? &stats[r] : &tmp);
    if (rc == DYMU_OK) rc = rf;
    if (stats) stats[r].rounds = rounds;
  }
  return rc;
}

}  // extern "C"
