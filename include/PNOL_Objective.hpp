/*
 * PNOL_Objective.hpp  (MI355X-native PNOL drop-in)
 *
 * The two objective interfaces of PNOL with their finite-difference engine.  Source
 * compatible with the reference header (Source/PNOL_Objective.hpp:25-62): same classes,
 * same pure virtual objEval signatures, same non-virtual FD members.  What changes is
 * where the work runs:
 *
 *   - A host objective (only objEval overridden) is evaluated on the host exactly as the
 *     reference does, point by point.  The *MPI members shard the points over the active
 *     communicator (RCCL over xGMI, one process per GPU) instead of MPI_COMM_WORLD.
 *   - An objective that returns a device objective from deviceObjective(n) is evaluated on
 *     the GPU: all N+1 forward-difference points in one batched launch
 *     (pnol_fd_gradient_d / pnol_fd_jacobian_d), bitwise equal to the host values for the
 *     transcendental-free objectives.  countEvals() lets such an objective keep its
 *     evaluation counter in step with the reference (one count per point).
 *   - Any objective may override objEvalBatch(): the FD engine hands it every batch of
 *     independent points at once (the N+1 gradient points, the Jacobian columns, the FD
 *     Hessian's triples) and the line searches hand it their trial points (the Wolfe pair
 *     phi(alpha), phi(alpha + dalpha); the MPI classes' pools).  The default loops over
 *     objEval in the reference's evaluation order, so a plain objEval-only objective sees
 *     exactly the reference's calls.  Overriding it is how a user objective runs its own batch
 *     on the GPU (or on host threads) without becoming a built-in device objective.
 */
#ifndef PNOL_AMD_OBJECTIVE_HPP_
#define PNOL_AMD_OBJECTIVE_HPP_

#ifndef ROOT_ID
#define ROOT_ID 0
#endif

#include <vector>

#include "pnol_amd.h"

// A program compiled with <mpi.h> on its include path (every reference program: the reference
// header includes it, PNOL_Objective.hpp:20) gets the *_MPI classes bound to MPI_COMM_WORLD
// with no code change (pnol_mpi_bind.hpp).  The library's own sources never include it.
#if !defined(PNOL_AMD_BUILDING_LIBRARY) && !defined(PNOL_AMD_NO_MPI_BIND) && defined(__has_include)
#if __has_include(<mpi.h>)
#include "pnol_mpi_bind.hpp"
#endif
#endif

using namespace std;  // the reference header exports namespace std to its users

class Objective {
  public:
    virtual ~Objective() {}

    // f(X) for one point (reference: PNOL_Objective.hpp:29)
    virtual double objEval(vector<double>& X) = 0;

    // --- MI355X extension hooks (defaults keep the reference's host behaviour) ---
    // f[k] = f(point k) for the nPts points of Xs (row-major nPts x n); default: objEval in order
    virtual void objEvalBatch(const double* Xs, int nPts, int n, double* f);
    // device objective for n-parameter points, or nullptr for host evaluation
    virtual pnol_dobj* deviceObjective(int n) { (void)n; return nullptr; }
    virtual void countEvals(long points) { (void)points; }

    // forward differences g_i = (f(X + dX_i e_i) - f(X)) / dX_i  (PNOL_Objective.cpp:12-34)
    void gradientApproximation(vector<double>& X, vector<double>& dX, vector<double>& dFdX);
    // upper triangle by 3 evaluations per pair, mirrored (PNOL_Objective.cpp:38-85)
    void hessianApproximation(vector<double>& X, vector<double>& dX, vector<vector<double>>& H);
    // the same gradient with the points sharded over the communicator (PNOL_Objective.cpp:88-159)
    void gradientApproximationMPI(vector<double>& X, vector<double>& dX, vector<double>& dFdX);
    // evaluation / gradient with frozen coordinates (PNOL_Objective.cpp:303-459)
    double objEvalRecur(vector<double>& Xrecur, vector<double>& constantX, vector<bool>& constantIndicator);
    void gradientApproximationRecur(vector<double>& X, vector<double>& dX, vector<double>& dFdX,
                                    vector<double>& constantX, vector<bool>& constantIndicator);
    void gradientApproximationMPIRecur(vector<double>& X, vector<double>& dX, vector<double>& dFdX,
                                       vector<double>& constantX, vector<bool>& constantIndicator);
};

class MultiObjective {
  public:
    virtual ~MultiObjective() {}

    // F(X), one residual per data point (reference: PNOL_Objective.hpp:57); F is pre-sized
    virtual void objEval(vector<double>& X, vector<double>& F) = 0;

    // F rows k*m .. k*m+m-1 = F(point k) for the nPts points of Xs (nPts x n); default: objEval in order
    virtual void objEvalBatch(const double* Xs, int nPts, int n, double* F, int m);
    virtual pnol_dobj* deviceObjective() { return nullptr; }
    virtual void countEvals(long points) { (void)points; }

    // J[i][j] = (F_i(X + dX_j e_j) - F_i(X)) / dX_j ; J is caller-sized m x n (PNOL_Objective.cpp:165-197)
    void gradientApproximation(vector<double>& X, vector<double>& dX, vector<vector<double>>& J);
    // columns sharded over the communicator, one allgather (PNOL_Objective.cpp:202-299)
    void gradientApproximationMPI(vector<double>& X, vector<double>& dX, vector<vector<double>>& J);
};

#endif /* PNOL_AMD_OBJECTIVE_HPP_ */
