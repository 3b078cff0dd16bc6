/*
 * LevenbergMarquardtMPI.hpp  (MI355X-native PNOL drop-in)
 *
 * LevMarq with the finite-difference Jacobian columns sharded over the communicator --
 * the reference class LevMarqMPI (Source/LevenbergMarquardtMPI.hpp:27-60).  Each rank
 * evaluates a contiguous block of ceil(n / ranks) columns on its GPU; one RCCL allgather
 * over xGMI assembles J^T on every rank (replacing the n zero-padded MPI_Allreduce calls of
 * PNOL_Objective.cpp:279-288).  The assembled J is bitwise independent of the rank count,
 * so the whole trajectory is too, as in the reference.  Messages print on rank 0.
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

  public:
    void findMin(vector<double>& X, vector<double>& f0, vector<double>& fOpt);

    void setParams(double lambda0In, double lambdaFactorIn, double dXGradIn, double maxIterIn, double xMinDiffIn,
                   int verboseIn) {
        maxIter = (int)maxIterIn; xMinDiff = xMinDiffIn; verbose = verboseIn; dXGrad = dXGradIn;
        lambda0 = lambda0In; lambdaFactor = lambdaFactorIn;
    }

    LevMarqMPI() : lambda0(0.001), dXGrad(1e-7), xMinDiff(1e-7), maxIter(10000), lambdaFactor(10), verbose(1) {}
    ~LevMarqMPI() {}
};

#endif /* PNOL_AMD_LEVENBERGMARQUARDT_MPI_HPP_ */
