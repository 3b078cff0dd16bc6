// bfgs_bnd_mpi.cpp -- BFGSBnd_MPI: box-bounded BFGS with a pooled secant line search and
// active-set recursion (drop-in for Source/BFGS_with_bnd_linsearch_MPI.cpp).  The pool is
// evaluated round-robin over the ranks and gathered with one allgather per round (the
// reference's zero-padded MPI_Reduce + Bcast, :314-344, is exact for one owner per entry).
// The reduced problem starts from the free-free block of D, gathered on the device (:822-843).
#include <cmath>
#include <cstdio>
#include <iostream>
#include <stdexcept>

#include "../pnol_comm.hpp"
#include "BFGS_with_bnd_linesearch_MPI.hpp"
#include "dense_hessian.hpp"
#include "line_points.hpp"

using namespace pnol;

namespace {

void vector_min(const std::vector<double>& v, double& val, int& idx) {
    val = v[0]; idx = 0;
    for (size_t i = 1; i < v.size(); ++i) if (v[i] < val) { val = v[i]; idx = (int)i; }
}
double vector_max(const std::vector<double>& v) {
    double m = v[0];
    for (size_t i = 1; i < v.size(); ++i) if (v[i] > m) m = v[i];
    return m;
}
void linspace(double a, double b, int N, std::vector<double>& v) {
    v.resize(N);
    for (int i = 0; i < N; ++i) v[i] = a + i * (b - a) / (N - 1);
}
void print_vec(const std::vector<double>& v) {
    for (double x : v) std::printf("%.17g ", x);
    std::printf("\n");
}

}  // namespace

void checkAlphaPoolBnd(bool& bndIndicator, vector<double>& alphaPool, vector<double>& X, vector<double>& Xlb,
                       vector<double>& Xub, vector<double>& p, vector<double>&, vector<bool>&) {
    // BFGS_with_bnd_linsearch_MPI.cpp:711-743
    const int Npool = (int)alphaPool.size();
    bndIndicator = false;
    const double alphaBnd = computeAlphaBnd(X, Xlb, Xub, p);
    for (int i = 0; i < Npool; ++i)
        if (alphaPool[i] > alphaBnd) bndIndicator = true;
    if (bndIndicator) {
        const double deltaAlpha = alphaBnd / (Npool);
        for (int i = 0; i < Npool; ++i) alphaPool[i] = deltaAlpha * (i + 1);
    }
    for (int i = 0; i < Npool; ++i)
        if (alphaPool[i] < 0) alphaPool[i] = 0;
}

double BFGSBnd_MPI::lineSearchObj(double alpha, vector<double>& X, vector<double>& p, vector<double>& cX,
                                  vector<bool>& cI) {
    // :246-258
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + alpha * p[i];
    return objPtr->objEvalRecur(Xa, cX, cI);
}

void BFGSBnd_MPI::evalAlphaPoolMPI(vector<double>& alphaPool, vector<double>& phiPool, vector<double>& X,
                                   vector<double>& p, vector<double>& cX, vector<bool>& cI) {
    // :262-354: entry k is owned by rank k mod P; one allgather of ceil(N/P) values per rank
    const int N = (int)phiPool.size();
    const int P = comm_size(), r = comm_rank();
    const int per = (N + P - 1) / P;
    std::vector<double> mine(per, 0.0), all((size_t)per * P, 0.0);
    std::vector<double> mya;   // this rank's entries, one batch
    for (int k = r; k < N; k += P) mya.push_back(alphaPool[k]);
    eval_line_points_recur(objPtr, X, p, mya.data(), (int)mya.size(), cX, cI, mine.data());
    check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)per), "allgather(alpha pool)");
    for (int k = 0; k < N; ++k) phiPool[k] = all[(size_t)(k % P) * per + k / P];
    for (int k = 0; k < N; ++k)
        if (phiPool[k] != phiPool[k] || std::isinf(phiPool[k]))
            throw std::runtime_error("BFGSBnd_MPI: line search produced a NaN/inf objective value");
}

void BFGSBnd_MPI::secantLineSearchBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double FX,
                                      vector<double>& dFdX, vector<double>& p, double& alphaOpt, double& Fopt,
                                      vector<double>& cX, vector<bool>& cI) {
    // :358-660
    const int Npool = poolSize > 0 ? poolSize : comm_size();
    std::vector<double> alphaPool(Npool, 0.0), phiPool(Npool, 0.0), alphaPoolPrev(Npool, -1.0),
        phiPoolPrev(Npool, 0.0), slope(Npool, 0.0);
    alphaOpt = 0;
    Fopt = FX;
    const double alpha0 = 0, phi0 = FX, dphi0 = seq_dot(dFdX, p);
    bool bndIndicator = false;

    int idxMin = -(int)std::ceil((Npool - 1.0) / 2.0);
    const int idxMax = (int)std::floor((Npool - 1.0) / 2.0);
    double r = std::pow(maxAlphaMult, 1.0 / (double)idxMax);
    for (int k = 0, idx = idxMin; k < Npool; ++k, ++idx) alphaPool[k] = alphaGuess * std::pow(r, idx);

    bool firstFlag = true, zoomFlag = false;
    for (int iter = 0; iter < maxIterLineSearch && firstFlag; ++iter) {
        checkAlphaPoolBnd(bndIndicator, alphaPool, X, Xlb, Xub, p, cX, cI);
        evalAlphaPoolMPI(alphaPool, phiPool, X, p, cX, cI);
        // 1. sufficient decrease
        for (int i = 0; i < Npool; ++i)
            if (phiPool[i] > phi0 + c1 * alphaPool[i] * dphi0) { zoomFlag = true; firstFlag = false; }
        // 2. curvature against the secant slopes
        slope[0] = (phiPool[0] - phi0) / (alphaPool[0] - alpha0);
        for (int i = 1; i < Npool; ++i) slope[i] = (phiPool[i] - phiPool[i - 1]) / (alphaPool[i] - alphaPool[i - 1]);
        if (firstFlag)
            for (int i = 0; i < Npool; ++i)
                if (std::fabs(slope[i]) <= std::fabs(c2 * dphi0)) { zoomFlag = false; firstFlag = false; }
        // 3. a non-negative secant slope brackets a minimum
        if (firstFlag)
            for (int i = 0; i < Npool; ++i)
                if (slope[i] >= 0) { zoomFlag = true; firstFlag = false; }
        // 4. extend the pool, unless it was clipped to the box
        if (firstFlag && !bndIndicator) {
            const double alphaMax = vector_max(alphaPool);
            r = std::pow(maxAlphaMult, 1.0 / (double)Npool);
            for (int i = 0; i < Npool; ++i) {
                alphaPoolPrev[i] = alphaPool[i];
                phiPoolPrev[i] = phiPool[i];
                const double power = i + 1;
                alphaPool[i] = alphaMax * std::pow(r, power);
            }
        } else if (bndIndicator) {
            firstFlag = false;
            if (verbose && comm_rank() == ROOT_ID) {
                std::cout << std::endl << "Line search reached boundary. Attempting to find an acceptable point in "
                          << "the domain interior." << std::endl << "alpha = ";
                print_vec(alphaPool);
                std::cout << "phi = ";
                print_vec(phiPool);
            }
        }
    }

    double alo, ahi, plo, phi;
    if (alphaPoolPrev[0] < 0) {
        findPoolBounds(alphaPool, phiPool, alpha0, phi0, alo, ahi, plo, phi);
    } else {
        std::vector<double> ae(2 * Npool), pe(2 * Npool);
        for (int i = 0; i < Npool; ++i) {
            ae[i] = alphaPoolPrev[i]; ae[i + Npool] = alphaPool[i];
            pe[i] = phiPoolPrev[i]; pe[i + Npool] = phiPool[i];
        }
        findPoolBounds(ae, pe, alpha0, phi0, alo, ahi, plo, phi);
    }

    // zoom: Npool interior points of [alpha_lo, alpha_hi] per round (:547-648)
    std::vector<double> alphaPool2(Npool + 2, 0.0), phiPool2(Npool + 2, 0.0);
    for (int iter = 0; iter < maxIterLineSearch && zoomFlag; ++iter) {
        linspace(alo, ahi, Npool + 2, alphaPool2);
        phiPool2[0] = plo; phiPool2[Npool + 1] = phi;
        alphaPool2[0] = alo; alphaPool2[Npool + 1] = ahi;
        for (int i = 0; i < Npool; ++i) { alphaPool[i] = alphaPool2[i + 1]; phiPool[i] = phiPool2[i + 1]; }
        evalAlphaPoolMPI(alphaPool, phiPool, X, p, cX, cI);
        for (int i = 0; i < Npool; ++i) { alphaPool2[i + 1] = alphaPool[i]; phiPool2[i + 1] = phiPool[i]; }
        for (int i = 0; i < Npool; ++i)
            slope[i] = (phiPool2[i + 1] - phiPool2[i]) / (alphaPool2[i + 1] - alphaPool2[i]);
        for (int i = 0; i < Npool; ++i)
            if (std::fabs(slope[i]) <= std::fabs(c2 * dphi0)) zoomFlag = false;
        if (zoomFlag) findPoolBounds(alphaPool2, phiPool2, alpha0, phi0, alo, ahi, plo, phi);
        if (vector_max(alphaPool2) < alphaMin) zoomFlag = false;
    }

    // the minimum of the last evaluated pool (:651-655)
    double phiMin;
    vector_min(phiPool, phiMin, idxMin);
    alphaOpt = alphaPool[idxMin];
    Fopt = phiMin;
}

void BFGSBnd_MPI::boundaryAssessment(double& F, vector<double>& X, vector<double>& p, vector<double>& dFdX,
                                     DenseInverseHessian& D, vector<double>& Xlb, vector<double>& Xub,
                                     vector<double>& dX, vector<double>& cX, vector<bool>& cI, bool& optimFlag,
                                     bool& recurFlag) {
    // :748-934.  Called only at the top level (recurFlag false), where X has all Ndim entries.
    const int Ndim = (int)cX.size();
    bool bndFlag = false;
    int iRecur = 0;
    for (int i = 0; i < Ndim; ++i) {
        if (cI[i]) continue;
        if ((std::fabs(X[iRecur] - Xlb[iRecur]) < dXGrad) && (p[iRecur] < 0)) {
            bndFlag = true; cI[i] = true; cX[i] = X[iRecur];
        } else if (std::fabs(X[iRecur] - Xub[iRecur]) < dXGrad && (p[iRecur] > 0)) {
            bndFlag = true; cI[i] = true; cX[i] = X[iRecur];
        }
        iRecur++;
    }
    int Nconst = 0;
    for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
    if (bndFlag && verbose && comm_rank() == ROOT_ID) {
        std::cout << std::endl << " Optimizer reached box boundary and found that the steepest descent is directed "
                  << "outside of the boundary at " << Nconst << " coordinate(s)." << std::endl << "    X = ";
        print_vec(X);
        std::cout << "    F = " << F << std::endl;
    }
    const int nr = Ndim - Nconst;
    if (!(bndFlag && nr > 0)) return;

    double FRecur = F;
    std::vector<double> XR, gR, lbR, ubR, dXR;
    std::vector<int> idx;
    for (int i = 0; i < Ndim; ++i)
        if (!cI[i]) {
            XR.push_back(X[i]); gR.push_back(dFdX[i]); lbR.push_back(Xlb[i]); ubR.push_back(Xub[i]);
            dXR.push_back(dX[i]); idx.push_back(i);
        }
    DenseInverseHessian DR(require_ctx(), nr, updateMode, true);
    DR.setSubmatrixOf(D, idx);
    recurFlag = true;
    mainBFGSLoop(FRecur, XR, gR, DR, lbR, ubR, dXR, cX, cI, optimFlag, recurFlag);

    // the reduced solution goes back into X; F keeps its pre-recursion value, as in the
    // reference (FRecur is not copied back, :845-864)
    for (int a = 0; a < nr; ++a) {
        const int i = idx[a];
        X[i] = XR[a]; dFdX[i] = gR[a]; Xlb[i] = lbR[a]; Xub[i] = ubR[a]; dX[i] = dXR[a];
    }
    D.setIdentity();
    objPtr->gradientApproximationMPI(X, dX, dFdX);

    // release everything, then re-freeze where the gradient still points out of the box
    for (int i = 0; i < Ndim; ++i) {
        cI[i] = false;
        if ((std::fabs(X[i] - Xlb[i]) < dXGrad) && (dFdX[i] > 0)) {
            bndFlag = true; cI[i] = true; cX[i] = X[i];
        } else if (std::fabs(X[i] - Xub[i]) < dXGrad && (dFdX[i] < 0)) {
            bndFlag = true; cI[i] = true; cX[i] = X[i];
        }
    }
    Nconst = 0;
    for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
    optimFlag = Nconst == 0;
    recurFlag = false;
    if (verbose && comm_rank() == ROOT_ID)
        std::cout << (optimFlag ? "Optimization continuing after recursive boundary optimization, as the gradient "
                                  "through the boundary points to the domain interior."
                                : "Optimization exiting after recursive boundary optimization, as the gradient "
                                  "through the boundary still points out of the domain.")
                  << std::endl;
}

void BFGSBnd_MPI::mainBFGSLoop(double& F, vector<double>& X, vector<double>& dFdX, DenseInverseHessian& D,
                               vector<double>& Xlb, vector<double>& Xub, vector<double>& dX, vector<double>& cX,
                               vector<bool>& cI, bool& optimFlag, bool& recurFlag) {
    // :84-243
    const int n = (int)X.size();
    double Fprev = 2 * F;
    if (verbose && comm_rank() == ROOT_ID) {
        std::cout << std::endl << "Starting bounded BFGS loop with F(X) = " << F << " over " << n << " variables."
                  << std::endl << "    X = ";
        print_vec(X);
    }
    std::vector<double> Xprev(n, 0.0), dFdXprev = dFdX, p(n), s(n), g(n);
    D.direction(dFdX, p);
    int iter = 0;
    double xdiff = xMinDiff * 2, grad2Norm = 2 * minGrad2Norm, alpha = alphaMin * 2;
    while (iter < maxIter && xdiff > xMinDiff && grad2Norm > minGrad2Norm && alpha > alphaMin && optimFlag) {
        double Fopt = 0;
        secantLineSearchBnd(X, Xlb, Xub, F, dFdX, p, alpha, Fopt, cX, cI);
        // a step that misses the tolerance is retried along steepest descent (:153-166)
        if (F - Fopt < FStepTolerance) {
            // printed on the root rank whatever the verbosity (BFGS_with_bnd_linsearch_MPI.cpp:156-158)
            if (comm_rank() == ROOT_ID)
                std::cout << "Line search failed in the quasi-newton direction. Recomputing gradient and "
                          << "attempting steepest descent instead." << std::endl;
            objPtr->gradientApproximationMPIRecur(X, dX, dFdX, cX, cI);
            for (int i = 0; i < n; ++i) p[i] = -dFdX[i];
            secantLineSearchBnd(X, Xlb, Xub, F, dFdX, p, alpha, Fopt, cX, cI);
        }
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        Fprev = F;
        F = Fopt;
        objPtr->gradientApproximationMPIRecur(X, dX, dFdX, cX, cI);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; g[i] = dFdX[i] - dFdXprev[i]; }
        // the update is skipped on a zero curvature product (:189-192)
        if (seq_dot(g, s) != 0) D.update(g, s, &dFdX, &p);
        else D.direction(dFdX, p);
        dFdXprev = dFdX;
        if (F > Fprev) optimFlag = false;
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += std::fabs(X[i] - Xprev[i]);
        grad2Norm = std::sqrt(seq_dot(dFdX, dFdX));
        if (verbose && comm_rank() == ROOT_ID) {
            std::cout << std::endl << "---> At iter = " << iter << " the mean abs xdiff is " << xdiff
                      << " and the grad2norm = " << grad2Norm << std::endl << "    X = ";
            print_vec(X);
            std::cout << "    with a minimum function evaluation of " << F << std::endl;
        }
        if (!recurFlag) boundaryAssessment(F, X, p, dFdX, D, Xlb, Xub, dX, cX, cI, optimFlag, recurFlag);
        iter = iter + 1;
    }
}

void BFGSBnd_MPI::findMinBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0,
                             double& fOpt) {
    // :14-81
    require_comm("BFGSBnd_MPI::findMinBnd");
    const int n = (int)X.size();
    std::vector<double> cX(n, 0.0), dX(n, dXGrad), dFdX(n, 0.0);
    std::vector<bool> cI(n, false);
    checkBoxBounds(X, Xlb, Xub);
    DenseInverseHessian D(require_ctx(), n, updateMode, true);   // row-sharded over the ranks
    if (initHessFD) init_from_fd_hessian(objPtr, X, dXHess, D);
    else D.setIdentity();
    objPtr->gradientApproximationMPI(X, dX, dFdX);
    double F = objPtr->objEval(X);
    f0 = F;
    bool optimFlag = true, recurFlag = false;
    mainBFGSLoop(F, X, dFdX, D, Xlb, Xub, dX, cX, cI, optimFlag, recurFlag);
    fOpt = F;
    if (verbose && comm_rank() == ROOT_ID) {
        std::cout << std::endl << "Completed bounded bfgs." << std::endl << "f0 = " << f0 << ", fOpt = " << fOpt
                  << " with variable:" << std::endl << "X = ";
        print_vec(X);
    }
}
