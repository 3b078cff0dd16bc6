/*
 * BFGS_with_linesearch.hpp  (MI355X-native PNOL drop-in)
 *
 * Quasi-Newton minimisation with a dense inverse Hessian D and a cubic-interpolation Wolfe
 * line search (Nocedal & Wright, Alg. 3.5/3.6) -- the reference class BFGS
 * (Source/BFGS_with_linesearch.hpp:27-101) with the same public members, setParams order
 * and defaults.  D lives in HBM; every iteration touches it once:
 *   - n <= PNOL_SEQ_MAX ("exact" mode): p = -D g and updateHessianInv run in the reference's
 *     operation order on the GPU, so small problems reproduce the CPU path bit for bit;
 *   - larger n ("fast" mode): one fused streaming pass per iteration reads D, applies the
 *     previous rank-2 correction, writes D back and produces D y, D^T y and D g at once
 *     (16 n^2 bytes instead of the reference's 4 n^3 flops).  See DESIGN.md.
 */
#ifndef PNOL_AMD_BFGS_WITH_LINESEARCH_HPP_
#define PNOL_AMD_BFGS_WITH_LINESEARCH_HPP_

#include <vector>

#include "PNOL_Algorithm.hpp"

class BFGS : public Algorithm {
  private:
    // line search
    double c1, c2;
    double dalpha;
    double alphaGuess;
    int maxIterLineSearch;
    // outer iteration
    double dXGrad;
    double dXHess;
    double xMinDiff;
    double minGrad2Norm;
    int maxIter;
    bool initHessFD;
    bool verbose;
    // MI355X: 0 = auto (exact for n <= PNOL_SEQ_MAX), 1 = exact, 2 = fast
    int updateMode = 0;
    double* profile = nullptr;   // extension: per-phase seconds and counts (pnol_run_bfgs_ex)

  public:
    void findMin(vector<double>& X, double& f0, double& fOpt);
    double lineSearchObj(double alpha, vector<double>& X, vector<double>& p);
    double lineSearchFDDerivative(double alpha, double phialpha, vector<double>& X, vector<double>& p);
    void lineSearchZoom(double alpha_lo, double alpha_hi, double phi_lo, double phi_hi, double dphi_lo_dalpha,
                        double dphi_hi_dalpha, double phi0, double dphi0dalpha, vector<double>& X, vector<double>& p,
                        double& alphaOpt, double& phiOpt, double& dphiOptdalpha);
    void cubicInterpolationLineSearch(vector<double>& X, double FX, vector<double>& dFdX, vector<double>& p,
                                      double& alphaOpt, double& Fopt);

    // same order as the reference (BFGS_with_linesearch.hpp:62); maxIter arrives as a double
    void setParams(double c1In, double c2In, double dalphaIn, double alphaGuessIn, int maxIterLineSearchIn,
                   double dXGradIn, double dXHessIn, double maxIterIn, double xMinDiffIn, double minGrad2NormIn,
                   bool initHessFDIn, bool verboseIn) {
        c1 = c1In; c2 = c2In; dalpha = dalphaIn; alphaGuess = alphaGuessIn;
        maxIterLineSearch = maxIterLineSearchIn; dXGrad = dXGradIn; dXHess = dXHessIn;
        maxIter = (int)maxIterIn; xMinDiff = xMinDiffIn; minGrad2Norm = minGrad2NormIn;
        initHessFD = initHessFDIn; verbose = verboseIn;
    }
    void setUpdateMode(int mode) { updateMode = mode; }
    // --- MI355X extension (diagnostics): 8 doubles -- iterations, total, FD gradient, line
    // search and D update seconds, line-search points, gradient calls, unused
    void setProfile(double* prof) { profile = prof; }

    BFGS()
        : c1(1e-4), c2(0.9), dalpha(1e-6), alphaGuess(1), maxIterLineSearch(1000), dXGrad(1e-6), dXHess(1e-3),
          xMinDiff(1e-5), minGrad2Norm(1e-5), maxIter(10000), initHessFD(false), verbose(false) {}
    ~BFGS() {}
};

// free helpers of the reference (BFGS_with_linesearch.hpp:104-106)
double cubicInterpMin(double alpha_lo, double alpha_hi, double phi_lo, double phi_hi, double dphi_lo_dalpha,
                      double dphi_hi_dalpha, vector<double>& X, vector<double>& p);
// updateHessianInv on host vectors, executed on the default GPU in the reference order
void updateHessianInv(vector<vector<double>>& D, vector<double>& g, vector<double>& s);

#endif /* PNOL_AMD_BFGS_WITH_LINESEARCH_HPP_ */
