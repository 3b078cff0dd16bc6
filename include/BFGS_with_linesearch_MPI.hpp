/*
 * BFGS_with_linesearch_MPI.hpp  (MI355X-native PNOL drop-in)
 *
 * BFGS with the finite-difference gradient sharded over the communicator and a pooled
 * secant line search that evaluates Npool step sizes at once -- the reference class
 * BFGS_MPI (Source/BFGS_with_linesearch_MPI.hpp:29-103), same members and defaults.
 * Npool defaults to the number of ranks (:235), as in the reference, which makes the
 * trajectory depend on the rank count; setPoolSize() fixes it independently of ranks.
 * The reference's zero-pool behaviour (a line search that ends in its first phase returns
 * alpha = 0, F = 0) is kept by default for drop-in fidelity;
 * setFixZeroPool(true) returns the best evaluated pool point instead.
 */
#ifndef PNOL_AMD_BFGS_WITH_LINESEARCH_MPI_HPP_
#define PNOL_AMD_BFGS_WITH_LINESEARCH_MPI_HPP_

#include <vector>

#include "PNOL_Algorithm.hpp"

class BFGS_MPI : public Algorithm {
  private:
    double c1, c2;
    double maxAlphaMult;
    double alphaGuess;
    int maxIterLineSearch;
    double dXGrad;
    double dXHess;
    double xMinDiff;
    double minGrad2Norm;
    int maxIter;
    bool initHessFD;
    bool verbose;
    int poolSize = 0;        // 0: number of ranks (reference behaviour)
    bool fixZeroPool = false;
    int updateMode = 0;

  public:
    void findMin(vector<double>& X, double& f0, double& fOpt);
    double lineSearchObj(double alpha, vector<double>& X, vector<double>& p);
    void evalAlphaPoolMPI(vector<double>& alphaPool, vector<double>& phiPool, vector<double>& X, vector<double>& p);
    void secantLineSearch(vector<double>& X, double FX, vector<double>& dFdX, vector<double>& p, double& alphaOpt,
                          double& Fopt);

    void setParams(double c1In, double c2In, double maxAlphaMultIn, double alphaGuessIn, int maxIterLineSearchIn,
                   double dXGradIn, double dXHessIn, double maxIterIn, double xMinDiffIn, double minGrad2NormIn,
                   bool initHessFDIn, bool verboseIn) {
        c1 = c1In; c2 = c2In; maxAlphaMult = maxAlphaMultIn; alphaGuess = alphaGuessIn;
        maxIterLineSearch = maxIterLineSearchIn; dXGrad = dXGradIn; dXHess = dXHessIn; maxIter = (int)maxIterIn;
        xMinDiff = xMinDiffIn; minGrad2Norm = minGrad2NormIn; initHessFD = initHessFDIn; verbose = verboseIn;
    }
    void setPoolSize(int npool) { poolSize = npool; }
    void setFixZeroPool(bool fix) { fixZeroPool = fix; }
    void setUpdateMode(int mode) { updateMode = mode; }

    BFGS_MPI()
        : c1(1e-4), c2(0.1), maxAlphaMult(4), alphaGuess(1), maxIterLineSearch(1000), dXGrad(1e-6), dXHess(1e-3),
          xMinDiff(1e-5), minGrad2Norm(1e-5), maxIter(10000), initHessFD(false), verbose(false) {}
    ~BFGS_MPI() {}
};

// findPoolBounds, BFGS_with_linesearch_MPI.cpp:496-530
void findPoolBounds(vector<double>& alphaPool, vector<double>& phiPool, double alpha0, double phi0, double& alpha1,
                    double& alpha2, double& phi1, double& phi2);

#endif /* PNOL_AMD_BFGS_WITH_LINESEARCH_MPI_HPP_ */
