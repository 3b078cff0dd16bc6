/*
 * LevenbergMarquardtMPI.hpp  (MI355X-native PNOL drop-in)
 *
 * LevMarq with the finite-difference Jacobian columns sharded over the communicator --
 * the reference class LevMarqMPI (Source/LevenbergMarquardtMPI.hpp:27-60), which evaluates
 * contiguous column blocks and assembles J with n zero-padded MPI_Allreduce calls
 * (PNOL_Objective.cpp:279-288).  Here, for linear-residual device objectives:
 *  - each rank evaluates a cost-balanced set of 128-column FD tiles (snake order,
 *    pnol_fd_tiles) for every residual row;
 *  - the residual rows are cut into 8 m-slices; each slice of those tiles goes to the rank
 *    that holds the slice (one group of RCCL point-to-point transfers, pnol_lm_jacobian_mpi_d);
 *  - each rank forms J^T J and -J^T F over its slices; the slice sums are combined by one
 *    fixed tree (nodes to each tile's owner, then one allgather, pnol_lm_normal_mpi_d).
 * Other objectives keep column tiles with the rows shared point-to-point and the tile-split
 * J^T J.  A, -J^T F and the whole trajectory are bitwise independent of the rank count, as in
 * the reference.  Messages print on rank 0.
 */
#ifndef PNOL_AMD_LEVENBERGMARQUARDT_MPI_HPP_
#define PNOL_AMD_LEVENBERGMARQUARDT_MPI_HPP_

#include <vector>

#include "PNOL_Algorithm.hpp"

class LevMarqMPI : public MultiAlgorithm {
  private:
    double lambda0;
    double dXGrad;
    double xMinDiff;
    int maxIter;
    double lambdaFactor;
    int verbose;
    int stepCounts[2] = {0, 0};   // accepted, rejected loop trips of the last findMin

  public:
    void findMin(vector<double>& X, vector<double>& f0, vector<double>& fOpt);

    void setParams(double lambda0In, double lambdaFactorIn, double dXGradIn, double maxIterIn, double xMinDiffIn,
                   int verboseIn) {
        maxIter = (int)maxIterIn; xMinDiff = xMinDiffIn; verbose = verboseIn; dXGrad = dXGradIn;
        lambda0 = lambda0In; lambdaFactor = lambdaFactorIn;
    }
    // additive: how many loop trips of the last findMin were accepted / rejected steps
    int getAcceptedSteps() const { return stepCounts[0]; }
    int getRejectedSteps() const { return stepCounts[1]; }

    LevMarqMPI() : lambda0(0.001), dXGrad(1e-7), xMinDiff(1e-7), maxIter(10000), lambdaFactor(10), verbose(1) {}
    ~LevMarqMPI() {}
};

#endif /* PNOL_AMD_LEVENBERGMARQUARDT_MPI_HPP_ */
