// pnol_comm.hpp -- the process-wide communicator used by the *_MPI drop-ins (internal).
#pragma once

#include <cstddef>

#include "pnol_amd.h"

namespace pnol {

int comm_size();
int comm_rank();
// contiguous ceil-sized column block of `rank`
void block_range(int ncols, int nranks, int rank, int* begin, int* count);
// recv[r*count + i] = send_r[i]; host buffers (any backend)
int comm_allgather_host(pnol_ctx* ctx, const double* send, double* recv, size_t count);
// device buffers (RCCL backend native; host backend bounces through host memory)
int comm_allgather_device(pnol_ctx* ctx, const double* send, double* recv, size_t count);
// process default GPU context (nullptr when no gfx950 device is visible)
pnol_ctx* default_ctx_or_null();

}  // namespace pnol
