/*
 * BFGS_bnd_linesearch.hpp  (MI355X-native PNOL drop-in)
 *
 * Box-bounded BFGS -- the reference class BFGS_Bnd (Source/BFGS_bnd_linesearch.hpp:31-145).
 * The Wolfe line search caps the step at the box edge (computeAlphaBnd); a coordinate that
 * reaches a bound with an outward search direction or gradient is frozen and the reduced
 * problem is re-optimised recursively from D = I (active-set recursion, not projected
 * gradient), then released if the gradient points back inside.  D of every recursion level
 * is a device matrix; the frozen-coordinate evaluations go through objEvalRecur.
 */
#ifndef PNOL_AMD_BFGS_BND_LINESEARCH_HPP_
#define PNOL_AMD_BFGS_BND_LINESEARCH_HPP_

#include <vector>

#include "Box_boundary_functions.hpp"
#include "PNOL_Algorithm.hpp"

namespace pnol { class DenseInverseHessian; }

class BFGS_Bnd : public AlgorithmBnd {
  private:
    double c1, c2;
    double dalpha;
    double alphaGuess;
    double alphaTol;
    double alphaMult;
    int maxIterLineSearch;
    double bndTol;
    double dXGrad;
    double dXHess;
    double xMinDiff;
    double minGrad2Norm;
    vector<double> dXGradVec;
    vector<double> initialScalingVec;
    int maxIter;
    bool initHessFD;
    int verbose;
    int totalIter;
    int updateMode = 0;
    bool assessRecursed = false;          // the last boundaryAssessment re-optimised a reduced problem
    vector<double>* fTrace = nullptr;     // extension: F after every iteration (any recursion level)
    double* profile = nullptr;            // extension: per-phase seconds and counts
    int depth = 0;
    // host bookkeeping of the active-set recursion (no reference counterpart): freeIdx[k] is the
    // full-space index of the current level's coordinate k while freeIdxLive, and the caller's
    // pending next direction is released while a reduced problem runs
    vector<int> freeIdx;
    bool freeIdxLive = false;
    vector<double>* pnextHeld = nullptr;

  public:
    void findMinBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0, double& fOpt);
    void findMinBndBody(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0, double& fOpt);
    void mainBFGSLoop(double& F, vector<double>& X, vector<double>& dFdX, pnol::DenseInverseHessian& D,
                      vector<double>& Xlb, vector<double>& Xub, vector<double>& dX, vector<double>& constantX,
                      vector<bool>& constantIndicator, bool& optimFlag, int& recurFlag);
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
                            vector<double>& constantX, vector<bool>& constantIndicator, bool& optimFlag,
                            int& recurFlag);

    // same order as the reference (BFGS_bnd_linesearch.hpp:80-99)
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
    void setUpdateMode(int mode) { updateMode = mode; }
    // --- MI355X extensions (diagnostics; the reference has no counterpart) ---
    void setFTrace(vector<double>* trace) { fTrace = trace; }
    // 8 doubles: iterations, total, FD gradient, line search, D update seconds, line-search
    // points, gradient calls, deepest recursion level
    void setProfile(double* prof) { profile = prof; }
    int getTotalIter() const { return totalIter; }

    BFGS_Bnd()
        : c1(1e-4), c2(0.9), dalpha(1e-6), alphaGuess(1), alphaTol(1e-20), alphaMult(2), maxIterLineSearch(50),
          bndTol(1e-5), dXGrad(1e-6), dXHess(1e-3), xMinDiff(1e-5), minGrad2Norm(1e-5), maxIter(10000),
          initHessFD(false), verbose(0), totalIter(0) {}
    ~BFGS_Bnd() {}
};

// cubicInterpMinSimple, BFGS_bnd_linesearch.cpp:736-750 (assumes alpha_a < alpha_b)
double cubicInterpMinSimple(double alpha_a, double alpha_b, double phi_a, double phi_b, double dphi_a_dalpha,
                            double dphi_b_dalpha);

#endif /* PNOL_AMD_BFGS_BND_LINESEARCH_HPP_ */
