/*
 * BFGS_bnd_linesearch_MPI_SW.hpp  (MI355X-native PNOL drop-in)
 *
 * Box-bounded BFGS whose Wolfe line search evaluates a pool of step sizes, each with its
 * forward-difference slope, per round -- the reference class BFGS_Bnd_MPI_SW
 * (Source/BFGS_bnd_linesearch_MPI_SW.hpp:30-165), same members, setParams order (identical to
 * BFGS_Bnd's) and defaults.  The bracketing phase evaluates Nprocs new steps per round
 * (pool of Nprocs + 1 with alpha = 0), the zoom phase Nprocs interior points between the
 * bracket ends, one of them the cubic-interpolation minimiser (pool of Nprocs + 2).  Pool
 * entries are dealt round-robin to the ranks and gathered with one allgather.  The
 * active-set recursion is BFGS_Bnd's, with the gradients sharded over the ranks.
 *
 * Nprocs is the number of ranks, as in the reference; setPoolSize(k) uses k in its place
 * (the pool of a k-rank run, evaluated by however many ranks there are).  A NaN / inf pool
 * value is replaced by 1e10 and stops the optimisation after the current step
 * (BFGS_bnd_linesearch_MPI_SW.cpp:657-693), as in the reference.
 */
#ifndef PNOL_AMD_BFGS_BND_LINESEARCH_MPI_SW_HPP_
#define PNOL_AMD_BFGS_BND_LINESEARCH_MPI_SW_HPP_

#include <vector>

#include "BFGS_bnd_linesearch.hpp"   // cubicInterpMinSimple
#include "Box_boundary_functions.hpp"
#include "PNOL_Algorithm.hpp"

namespace pnol { class DenseInverseHessian; }

class BFGS_Bnd_MPI_SW : public AlgorithmBnd {
  private:
    // line search parameters
    double c1, c2;
    double dalpha;
    double alphaGuess;
    double alphaTol;
    double alphaMult;
    int maxIterLineSearch;
    // BFGS parameters
    double bndTol;
    double dXGrad;
    double dXHess;
    double xMinDiff;
    double minGrad2Norm;
    vector<double> dXGradVec;
    vector<double> initialScalingVec;
    int maxIter;
    int totalIter;
    bool initHessFD;
    int verbose;
    // local variables
    int Nprocs;
    int procID;
    bool optimFlag;
    int recurFlag;
    int poolSize = 0;    // 0: Nprocs = number of ranks (reference behaviour)
    int updateMode = 0;

  public:
    void findMinBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0, double& fOpt);
    void findMinBndBody(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0, double& fOpt);
    void mainBFGSLoop(double& F, vector<double>& X, vector<double>& dFdX, pnol::DenseInverseHessian& D,
                      vector<double>& Xlb, vector<double>& Xub, vector<double>& dX, vector<double>& constantX,
                      vector<bool>& constantIndicator);
    void evaluateAlphaPoolAndDerivativesIndicator(vector<double>& alphaPool, vector<int> evalIndicator,
                                                  vector<double>& X, vector<double>& p, vector<double>& constantX,
                                                  vector<bool>& constantIndicator, vector<double>& phiPool,
                                                  vector<double>& dphidalphaPool);
    void evaluateAlphaPoolAndDerivatives(vector<double>& alphaPool, vector<double>& X, vector<double>& p,
                                         vector<double>& constantX, vector<bool>& constantIndicator,
                                         vector<double>& phiPool, vector<double>& dphidalphaPool);
    double lineSearchObj(double alpha, vector<double>& X, vector<double>& p, vector<double>& constantX,
                         vector<bool>& constantIndicator);
    double lineSearchFDDerivative(double alpha, double phialpha, vector<double>& X, vector<double>& p,
                                  vector<double>& constantX, vector<bool>& constantIndicator);
    void lineSearchZoomBnd(double alpha_a, double alpha_b, double phi_a, double phi_b, double dphi_a_dalpha,
                           double dphi_b_dalpha, double phi0, double dphi0dalpha, vector<double>& X, vector<double>& p,
                           vector<double>& constantX, vector<bool>& constantIndicator, int& iter_ls, double& alphaOpt,
                           double& phiOpt, double& dphiOptdalpha);
    void cubicInterpolationLineSearchBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double FX,
                                         vector<double>& dFdX, vector<double>& p, vector<double>& constantX,
                                         vector<bool>& constantIndicator, double& alphaOpt, double& Fopt);
    void boundaryAssessment(double& F, vector<double>& X, vector<double>& p, vector<double>& dFdX,
                            pnol::DenseInverseHessian& D, vector<double>& Xlb, vector<double>& Xub, vector<double>& dX,
                            vector<double>& constantX, vector<bool>& constantIndicator);

    // same order as the reference (BFGS_bnd_linesearch_MPI_SW.hpp:80-99)
    void setParams(double c1In, double c2In, double dalphaIn, double alphaGuessIn, double alphaTolIn,
                   double alphaMultIn, int maxIterLineSearchIn, double bndTolIn, double dXGradIn, double dXHessIn,
                   double maxIterIn, double xMinDiffIn, double minGrad2NormIn, bool initHessFDIn, int verboseIn) {
        c1 = c1In; c2 = c2In; dalpha = dalphaIn; alphaGuess = alphaGuessIn; alphaTol = alphaTolIn;
        alphaMult = alphaMultIn; maxIterLineSearch = maxIterLineSearchIn; bndTol = bndTolIn; dXGrad = dXGradIn;
        dXHess = dXHessIn; maxIter = (int)maxIterIn; xMinDiff = xMinDiffIn; minGrad2Norm = minGrad2NormIn;
        initHessFD = initHessFDIn; verbose = verboseIn;
    }
    void setGradVec(vector<double>& v) { dXGradVec.assign(v.begin(), v.end()); }
    void setinitialScalingVec(vector<double>& v) { initialScalingVec.assign(v.begin(), v.end()); }
    void setPoolSize(int nprocsEquivalent) { poolSize = nprocsEquivalent; }
    void setUpdateMode(int mode) { updateMode = mode; }

    BFGS_Bnd_MPI_SW();
    ~BFGS_Bnd_MPI_SW() {}
};

// computeZoomRegion, BFGS_bnd_linesearch_MPI_SW.cpp:399-431: the bracket around the pool
// minimum (to its left when the slope there is positive, else to its right)
void computeZoomRegion(vector<double>& alphaPool, vector<double>& phiPool, vector<double>& dphidalphaPool,
                       double& alpha_a, double& alpha_b, double& phi_a, double& phi_b, double& dphi_a_dalpha,
                       double& dphi_b_dalpha);

#endif /* PNOL_AMD_BFGS_BND_LINESEARCH_MPI_SW_HPP_ */
