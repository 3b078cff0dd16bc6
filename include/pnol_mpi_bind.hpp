/*
 * pnol_mpi_bind.hpp  (MI355X-native PNOL drop-in)
 *
 * Binds the *_MPI classes to MPI_COMM_WORLD of an unmodified reference program run under
 * `mpirun -n P ./app`.  The reference's MPI classes read P and the rank from MPI_COMM_WORLD
 * (LevenbergMarquardtMPI.cpp:16-17, PNOL_Objective.cpp:102-103 / 227-228,
 * BFGS_with_linesearch_MPI.cpp:231-235, BFGS_bnd_linesearch_MPI_SW.cpp:229 / 490,
 * GeneticAlgorithmMPI.cpp:17-18); libpnol_amd.so links no MPI, so this header -- included by
 * PNOL_Objective.hpp whenever <mpi.h> is on the include path, as it is for every program the
 * reference builds (its PNOL_Objective.hpp:20 includes <mpi.h>) -- compiles the binding into
 * the program against the program's own MPI and registers it with the library before main().
 * The library runs it at the first *_MPI call:
 *
 *   - MPI not initialised (or finalised): nothing is bound; the call is retried at the next
 *     *_MPI use.  A job whose launcher announced more than one rank is then refused by the
 *     library (pnol_comm_bind_launcher) instead of running as one rank.
 *   - P = 1: nothing to bind (single process).
 *   - P > 1: the GPU of the node-local rank (MPI_Comm_split_type SHARED) becomes the default
 *     context's device; when every node-local rank has a GPU of its own, rank 0's RCCL unique
 *     id is broadcast over MPI_COMM_WORLD and every rank joins the RCCL communicator (xGMI);
 *     when node-local ranks outnumber the GPUs (or no GPU is visible), the library's host
 *     backend runs over MPI_Allgather instead.  PNOL_MPI_COMM=host|rccl forces either; the
 *     choice is agreed over all ranks (MPI_Allreduce, min).
 *
 * The allgathers of the host backend may be issued from the bounded solvers' worker thread
 * (one thread at a time, while the calling thread waits): MPI_THREAD_SERIALIZED usage.
 * Define PNOL_AMD_NO_MPI_BIND before the include to keep the binding out.
 */
#ifndef PNOL_AMD_MPI_BIND_HPP_
#define PNOL_AMD_MPI_BIND_HPP_

#include <mpi.h>

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pnol_amd.h"

namespace pnol_mpi_bind {

// the library's host backend: recv[r * bytes + i] = send_r[i] over MPI_COMM_WORLD
inline int allgather(const void* send, void* recv, size_t bytes, void* user) {
    (void)user;
    // doubles as the element type when they fit an int count (up to 16 GiB per rank)
    if (bytes % sizeof(double) == 0 && bytes / sizeof(double) <= (size_t)INT_MAX)
        return MPI_Allgather(send, (int)(bytes / sizeof(double)), MPI_DOUBLE, recv, (int)(bytes / sizeof(double)),
                             MPI_DOUBLE, MPI_COMM_WORLD) == MPI_SUCCESS ? 0 : 1;
    if (bytes <= (size_t)INT_MAX)
        return MPI_Allgather(send, (int)bytes, MPI_BYTE, recv, (int)bytes, MPI_BYTE, MPI_COMM_WORLD) == MPI_SUCCESS
                   ? 0 : 1;
    return 1;
}

inline int bind() {
    int inited = 0, finalized = 0;
    MPI_Initialized(&inited);
    MPI_Finalized(&finalized);
    if (!inited || finalized) return 1;
    int P = 1, rank = 0;
    MPI_Comm_size(MPI_COMM_WORLD, &P);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (P == 1) return 0;
    MPI_Comm node;
    if (MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node) != MPI_SUCCESS) return -1;
    int local_rank = 0, local_size = 1;
    MPI_Comm_rank(node, &local_rank);
    MPI_Comm_size(node, &local_size);
    MPI_Comm_free(&node);
    int ndev = 0;
    if (pnol_device_count(&ndev) != PNOL_OK) ndev = 0;
    int rccl = (ndev > 0 && local_size <= ndev) ? 1 : 0;
    if (const char* e = std::getenv("PNOL_MPI_COMM")) {
        if (std::strcmp(e, "host") == 0) rccl = 0;
        else if (std::strcmp(e, "rccl") == 0 && ndev > 0) rccl = 1;
    }
    MPI_Allreduce(MPI_IN_PLACE, &rccl, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    if (ndev > 0 && pnol_set_default_device(local_rank % ndev) != PNOL_OK)
        std::fprintf(stderr, "pnol_amd: rank %d keeps its default GPU (its context existed before MPI binding)\n", rank);
    if (!rccl) return pnol_comm_init_host(P, rank, &allgather, nullptr) == PNOL_OK ? 0 : -2;
    char id[128];
    std::memset(id, 0, sizeof(id));
    int ok = rank == 0 ? (pnol_comm_unique_id(id) == PNOL_OK) : 1;
    MPI_Allreduce(MPI_IN_PLACE, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    if (!ok) return -3;
    MPI_Bcast(id, 128, MPI_BYTE, 0, MPI_COMM_WORLD);
    pnol_ctx* ctx = nullptr;
    int st = pnol_default_ctx(&ctx);
    if (st == PNOL_OK) st = pnol_comm_init_rccl(ctx, P, rank, id);
    int all_ok = st == PNOL_OK;
    MPI_Allreduce(MPI_IN_PLACE, &all_ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    if (!all_ok) {
        pnol_comm_finalize();
        return -4;
    }
    return 0;
}

struct Registrar {
    Registrar() { pnol_comm_set_launcher_hook(&bind); }
};
inline Registrar registrar;   // one registration per program (C++17 inline variable)

}  // namespace pnol_mpi_bind

#endif /* PNOL_AMD_MPI_BIND_HPP_ */
