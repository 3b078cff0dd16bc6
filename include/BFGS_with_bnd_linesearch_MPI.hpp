/*
 * BFGS_with_bnd_linesearch_MPI.hpp  (MI355X-native PNOL drop-in)
 *
 * Box-bounded BFGS with a pooled secant line search -- the reference class BFGSBnd_MPI
 * (Source/BFGS_with_bnd_linesearch_MPI.hpp:35-122), same members, setParams order and
 * defaults.  Each line-search round evaluates Npool step sizes at once (round-robin over the
 * ranks, one allgather); the pool is clipped to the box by checkAlphaPoolBnd.  A coordinate
 * on a bound whose search direction points out of the box is frozen and the reduced problem
 * is re-optimised from the free-free block of D (gathered on the device), then released when
 * the gradient points back inside.  D of every level is a device matrix.
 *
 * Npool defaults to the number of ranks (BFGS_with_bnd_linsearch_MPI.cpp:373), which makes
 * the trajectory depend on the rank count; setPoolSize() fixes it independently of ranks.
 * The reference exits the process (exit(0)) on a NaN / inf pool value (:327-333); here
 * findMinBnd throws std::runtime_error instead.
 */
#ifndef PNOL_AMD_BFGS_WITH_BND_LINESEARCH_MPI_HPP_
#define PNOL_AMD_BFGS_WITH_BND_LINESEARCH_MPI_HPP_

#include <vector>

#include "BFGS_with_linesearch_MPI.hpp"   // findPoolBounds
#include "Box_boundary_functions.hpp"
#include "PNOL_Algorithm.hpp"

namespace pnol { class DenseInverseHessian; }

class BFGSBnd_MPI : public AlgorithmBnd {
  private:
    // line search parameters
    double c1, c2;
    double maxAlphaMult;
    double alphaGuess;
    int maxIterLineSearch;
    double alphaMin;
    // BFGS parameters
    double dXGrad;
    double dXHess;
    double xMinDiff;
    double minGrad2Norm;
    double FStepTolerance;
    int maxIter;
    bool initHessFD;
    bool verbose;
    int poolSize = 0;     // 0: number of ranks (reference behaviour)
    int updateMode = 0;

  public:
    void findMinBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0, double& fOpt);
    void mainBFGSLoop(double& F, vector<double>& X, vector<double>& dFdX, pnol::DenseInverseHessian& D,
                      vector<double>& Xlb, vector<double>& Xub, vector<double>& dX, vector<double>& constantX,
                      vector<bool>& constantIndicator, bool& optimFlag, bool& recurFlag);
    double lineSearchObj(double alpha, vector<double>& X, vector<double>& p, vector<double>& constantX,
                         vector<bool>& constantIndicator);
    void evalAlphaPoolMPI(vector<double>& alphaPool, vector<double>& phiPool, vector<double>& X, vector<double>& p,
                          vector<double>& constantX, vector<bool>& constantIndicator);
    void secantLineSearchBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double FX,
                             vector<double>& dFdX, vector<double>& p, double& alphaOpt, double& Fopt,
                             vector<double>& constantX, vector<bool>& constantIndicator);
    void boundaryAssessment(double& F, vector<double>& X, vector<double>& p, vector<double>& dFdX,
                            pnol::DenseInverseHessian& D, vector<double>& Xlb, vector<double>& Xub,
                            vector<double>& dX, vector<double>& constantX, vector<bool>& constantIndicator,
                            bool& optimFlag, bool& recurFlag);

    // same order as the reference (BFGS_with_bnd_linesearch_MPI.hpp:79-96)
    void setParams(double c1In, double c2In, double alphaMinIn, double maxAlphaMultIn, double alphaGuessIn,
                   int maxIterLineSearchIn, double dXGradIn, double dXHessIn, double maxIterIn, double xMinDiffIn,
                   double minGrad2NormIn, double FStepToleranceIn, bool initHessFDIn, bool verboseIn) {
        c1 = c1In; c2 = c2In; alphaMin = alphaMinIn; maxAlphaMult = maxAlphaMultIn; alphaGuess = alphaGuessIn;
        maxIterLineSearch = maxIterLineSearchIn; dXGrad = dXGradIn; dXHess = dXHessIn; maxIter = (int)maxIterIn;
        xMinDiff = xMinDiffIn; minGrad2Norm = minGrad2NormIn; FStepTolerance = FStepToleranceIn;
        initHessFD = initHessFDIn; verbose = verboseIn;
    }
    void setPoolSize(int npool) { poolSize = npool; }
    void setUpdateMode(int mode) { updateMode = mode; }

    BFGSBnd_MPI()
        : c1(1e-4), c2(0.1), maxAlphaMult(4), alphaGuess(1), maxIterLineSearch(1000), alphaMin(1e-16),
          dXGrad(1e-6), dXHess(1e-3), xMinDiff(1e-5), minGrad2Norm(1e-5), FStepTolerance(1e-5), maxIter(10000),
          initHessFD(false), verbose(false) {}
    ~BFGSBnd_MPI() {}
};

// checkAlphaPoolBnd, BFGS_with_bnd_linsearch_MPI.cpp:711-743: a pool reaching past the box
// edge is replaced by Npool equal steps up to it; negative steps are clamped to 0.
void checkAlphaPoolBnd(bool& bndIndicator, vector<double>& alphaPool, vector<double>& X, vector<double>& Xlb,
                       vector<double>& Xub, vector<double>& p, vector<double>& constantX,
                       vector<bool>& constantIndicator);

#endif /* PNOL_AMD_BFGS_WITH_BND_LINESEARCH_MPI_HPP_ */
