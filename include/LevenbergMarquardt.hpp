/*
 * LevenbergMarquardt.hpp  (MI355X-native PNOL drop-in)
 *
 * Marquardt-scaled damped Gauss-Newton on a forward-difference Jacobian -- the reference
 * class LevMarq (Source/LevenbergMarquardt.hpp:24-57): same setParams order, defaults and
 * verbosity contract (final summary whenever verbose >= 0).  Per loop trip, on the GPU:
 * the FD Jacobian (batched device objective, or host objEval columns uploaded once), J^T J
 * on fp64 MFMA with A_ii = (1 + lambda) (J^T J)_ii, rhs = -J^T F, the damped solve
 * (Cholesky; LU in the reference order for n <= PNOL_SEQ_MAX or a non-SPD A), F(X + sigma).
 * The accept/reject test and the lambda schedule run on the host exactly as the reference.
 */
#ifndef PNOL_AMD_LEVENBERGMARQUARDT_HPP_
#define PNOL_AMD_LEVENBERGMARQUARDT_HPP_

#include <vector>

#include "PNOL_Algorithm.hpp"

class LevMarq : public MultiAlgorithm {
  private:
    double lambda0;
    double dXGrad;
    double xMinDiff;
    int maxIter;
    double lambdaFactor;   // > 1
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

    LevMarq() : lambda0(0.001), dXGrad(1e-7), xMinDiff(1e-7), maxIter(10000), lambdaFactor(10), verbose(1) {}
    ~LevMarq() {}
};

#endif /* PNOL_AMD_LEVENBERGMARQUARDT_HPP_ */
