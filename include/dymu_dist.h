/*
 * dymu_dist.h -- C-ABI of the row-slab sharded solve driven natively (one C++
 * round loop on the engine's stream, behind a transport).
 *
 * One process per rank.  The global ny x nx grid is cut into row slabs
 * (dymu_slab_rows); rank r owns rows [row0, row0+nrows) and solves them with
 * the engine's domain primitives (dymu_dom_*, include/dymu_fim.h).  Every
 * `passes_per_exchange` passes (one round) the ranks swap their boundary rows
 * with rank-1 / rank+1 (nx x 8 B per neighbour), the next round's first pass
 * min-merges them into the ghost rows, and on every 4th round the ranks reduce
 * the round's queued-tile count (4 bytes); the host reads the reduced count of
 * the PREVIOUS check through the engine's mailbox, so the device always has
 * work queued.  A zero count after a round means the global fixed point was
 * reached.  Transports (the same loop for all of them):
 *   DYMU_DIST_RCCL  grouped ncclSend/ncclRecv over xGMI + ncclAllReduce, one GPU
 *                   per rank (dymu_dist_create; the bench's multi-GPU path)
 *   DYMU_DIST_IPC   rows pushed into the neighbours' hipIpc-mapped receive rows,
 *                   counts reduced through a POSIX shared-memory board; ranks of
 *                   one node, several per GPU allowed (dymu_dist_create_ipc)
 *   DYMU_DIST_PEER  GPU-initiated: every round's first pass pushes its boundary
 *                   rows' decreases straight into the neighbours' peer-mapped
 *                   receive rows with a sequence tag and merges its own after
 *                   theirs (dymu_dom_round_peer); no host step and no collective
 *                   per round, the termination check (every 4th round) compares
 *                   the ranks' posted status on the board; ranks of one node,
 *                   several per GPU allowed (dymu_dist_create_peer)
 *   virtual         all ranks in one process (dymu_vdist_solve)
 *
 * This replaces, for a grid too large or too slow for one GPU, the reference's
 * single-threaded propagation loop computeEntireTotalCostMap
 * (src/DyMu_GlobalPathPlanning.cpp:443-468); the result is the single-GPU
 * fixed point (values only decrease; ghost rows are valid upper bounds).
 *
 * Slab buffers (device, pitch ld >= nx):
 *   F_slab: nrows rows (the rank's rows of F)
 *   T_buf:  nrows + 2 rows; row 0 = ghost row (rank-1's last row), rows
 *           1..nrows = owned rows, row nrows+1 = ghost row (rank+1's first row)
 */
#ifndef DYMU_DIST_H
#define DYMU_DIST_H

#include <stdint.h>

#include "dymu_fim.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DYMU_DIST_ID_BYTES 128 /* sizeof(ncclUniqueId) */
#define DYMU_DIST_RCCL 0
#define DYMU_DIST_IPC 1
#define DYMU_DIST_PEER 2

typedef struct dymu_dist dymu_dist;

/* Rank 0 creates the communicator id; the caller broadcasts the 128 bytes
 * (e.g. torch.distributed over TCP/gloo) to every rank. */
int dymu_dist_unique_id(unsigned char id[DYMU_DIST_ID_BYTES]);

/* Collective over the `world` ranks: creates the RCCL communicator on `device`
 * (the device of `ctx`).  `ctx` stays owned by the caller and must outlive the
 * dymu_dist. */
int dymu_dist_create(dymu_dist** out, dymu_ctx* ctx, int device,
                     const unsigned char id[DYMU_DIST_ID_BYTES], int rank, int world);
int dymu_dist_destroy(dymu_dist* d);

/* The IPC transport.  Rank 0 makes the id (the name of a fresh shared-memory
 * board, /dev/shm) and the caller broadcasts its 128 bytes; creation is
 * collective (returns once every rank has joined the board).  Every rank must
 * run on the same node; the ranks may share a GPU.  Per round the host waits
 * for its own push and both neighbours' (DYMU_DIST_TIMEOUT_S bounds each wait). */
int dymu_dist_ipc_unique_id(unsigned char id[DYMU_DIST_ID_BYTES]);
int dymu_dist_create_ipc(dymu_dist** out, dymu_ctx* ctx, int device,
                         const unsigned char id[DYMU_DIST_ID_BYTES], int rank, int world);
/* The peer transport: the same id (dymu_dist_ipc_unique_id) and collective
 * creation; the boundary rows move GPU to GPU inside the pass kernels (DESIGN.md
 * s5 "Peer transport").  Kernel-5 slabs, passes_per_exchange >= 2. */
int dymu_dist_create_peer(dymu_dist** out, dymu_ctx* ctx, int device,
                          const unsigned char id[DYMU_DIST_ID_BYTES], int rank, int world);
/* DYMU_DIST_RCCL, DYMU_DIST_IPC or DYMU_DIST_PEER */
int dymu_dist_transport(dymu_dist* d);
/* Bound on every host wait on a peer rank, process-wide: seconds > 0 overrides
 * DYMU_DIST_TIMEOUT_S (default 300 s), 0 restores it.  Returns the bound now in
 * force.  The bench shortens it while it tries candidate transports, so a candidate
 * that hangs costs seconds, not the run. */
double dymu_dist_set_timeout(double seconds);

/* Sharded solve of the global grid (nx x ny, goal (goal_i, goal_j) in global
 * coordinates); this rank's slab geometry comes from dymu_slab_rows.
 * Collective: every rank calls it with the same nx, ny, goal and
 * passes_per_exchange (0 = 4).  `stream` NULL = the context's stream.
 * Blocks until converged; stats are this rank's (rounds = exchange rounds).
 * Errors: a collective pre-flight first checks every rank's arguments, so a
 * rank-local argument error returns DYMU_ERR_ARG on every rank.  Any later
 * error aborts the transport (ncclCommAbort for RCCL: peers blocked in an exchange
 * this rank will not post are released by their own wait timeout,
 * DYMU_DIST_TIMEOUT_S, default 300 s) and every further solve on this handle
 * returns DYMU_ERR_STATE. */
int dymu_dist_solve(dymu_dist* d, const double* F_slab, double* T_buf, uint64_t ld, uint32_t nx,
                    uint32_t ny, uint32_t goal_i, uint32_t goal_j, uint32_t passes_per_exchange,
                    void* stream, dymu_stats* stats);

/* The same loop with `world` (<= 16) virtual ranks in one process (tests,
 * rehearsal): ctxs[r] / F_slabs[r] / T_bufs[r] are rank r's context and slab
 * buffers, all on the current device; the exchange is device-to-device copies
 * and the reduction a device sum posted through ctxs[0]'s mailbox, all ordered
 * on `stream` (required, not NULL).  stats: `world` entries (may be NULL). */
int dymu_vdist_solve(dymu_ctx* const* ctxs, int world, const double* const* F_slabs,
                     double* const* T_bufs, uint64_t ld, uint32_t nx, uint32_t ny,
                     uint32_t goal_i, uint32_t goal_j, uint32_t passes_per_exchange,
                     void* stream, dymu_stats* stats);

const char* dymu_dist_last_error(dymu_dist* d);

/* Ranks in the communicator (ncclCommCount) or on the IPC board: what the
 * transport actually sees, for the bench line's `ranks_seen`. */
int dymu_dist_comm_count(dymu_dist* d, int* ranks);

#ifdef __cplusplus
}
#endif
#endif
