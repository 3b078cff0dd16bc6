// pnol_comm.hpp -- the process-wide communicator used by the *_MPI drop-ins (internal).
#pragma once

#include <cstddef>
#include <functional>
#include <vector>

#include "pnol_amd.h"

namespace pnol {

int comm_size();
int comm_rank();
// bind the MPI launcher's communicator if none is bound (every *_MPI entry point calls this
// first); PNOL_ERR_COMM when a multi-rank launch has no communicator
int comm_bind_launcher();
int launcher_world_size();
// ranks sharing one GPU (the host backend with several ranks)
bool comm_shares_device();
// contiguous ceil-sized column block of `rank`
void block_range(int ncols, int nranks, int rank, int* begin, int* count);
// cost-balanced FD column tiles (PNOL_FD_TILE columns each, dealt in snake order)
constexpr int kFdTileCols = PNOL_FD_TILE;
int fd_tile_owner(int tile, int nranks);
void fd_tiles_of(int ncols, int nranks, int rank, std::vector<int>& start, std::vector<int>& count);
// every rank ends with all ncols rows of buf (row c at buf + c * ld), owners per fd_tiles_of
int comm_share_rows(pnol_ctx* ctx, double* buf, size_t ld, int ncols);
// recv[r*count + i] = send_r[i]; host buffers (any backend)
int comm_allgather_host(pnol_ctx* ctx, const double* send, double* recv, size_t count);
// device buffers (RCCL backend native; host backend bounces through host memory); stream:
// nullptr = the context stream
int comm_allgather_device(pnol_ctx* ctx, const double* send, double* recv, size_t count, void* stream = nullptr);
// one int per rank, gathered on every rank (host memory; setup-time agreement checks)
int comm_allgather_int(pnol_ctx* ctx, int mine, std::vector<int>& all);
// Point-to-point exchange of device blocks: blocks(src, dst, out) lists what rank src sends to
// rank dst (src != dst) -- soff into the sender's sbase, roff into the receiver's rbase, count
// doubles -- and must give the same list on every rank.  RCCL: one group of sends / receives
// on `stream` (nullptr: the context stream); host backend: packed through one allgather, the
// copies on `stream` (the host waits for that stream only).
struct XBlock {
    size_t soff, roff, count;
};
int comm_exchange(pnol_ctx* ctx, const double* sbase, double* rbase,
                  const std::function<void(int, int, std::vector<XBlock>&)>& blocks, void* stream = nullptr);
// process default GPU context (nullptr when no gfx950 device is visible)
pnol_ctx* default_ctx_or_null();

}  // namespace pnol
