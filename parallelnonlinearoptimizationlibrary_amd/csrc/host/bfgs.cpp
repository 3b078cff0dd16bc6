// bfgs.cpp -- BFGS with the cubic-interpolation Wolfe line search (drop-in for
// Source/BFGS_with_linesearch.cpp).  The line-search control flow is host logic, restated
// from the reference; D and its products run on the GPU through DenseInverseHessian.
#include <cmath>
#include <cstdio>
#include <iostream>

#include "BFGS_with_linesearch.hpp"
#include "dense_hessian.hpp"
#include "line_points.hpp"

using namespace pnol;

namespace {

double sign_of(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }

void print_vec(const std::vector<double>& v) {
    for (double x : v) std::printf("%.17g ", x);
    std::printf("\n");
}

}  // namespace

double cubicInterpMin(double alo, double ahi, double plo, double phi, double dlo, double dhi, vector<double>& X,
                      vector<double>& p) {
    (void)X; (void)p;
    // BFGS_with_linesearch.cpp:359-385
    const double d1 = dlo + dhi - 3 * (plo - phi) / (alo - ahi);
    const double d2 = sign_of(ahi - alo) * std::sqrt(d1 * d1 - dlo * dhi);
    double an = ahi - (ahi - alo) * (dhi + d2 - d1) / (dhi - dlo + 2 * d2);
    if (alo < ahi) {
        if (an < alo) an = (ahi + alo) / 2;
    } else {
        if (an < ahi) an = (ahi + alo) / 2;
    }
    return an;
}

void updateHessianInv(vector<vector<double>>& D, vector<double>& g, vector<double>& s) {
    DenseInverseHessian H(require_ctx(), (int)g.size(), 1);
    H.setMatrix(D);
    H.update(g, s, nullptr, nullptr);
    H.getMatrix(D);
}

double BFGS::lineSearchObj(double alpha, vector<double>& X, vector<double>& p) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + alpha * p[i];
    return objPtr->objEval(Xa);
}

double BFGS::lineSearchFDDerivative(double alpha, double phialpha, vector<double>& X, vector<double>& p) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + (alpha + dalpha) * p[i];
    const double Fa = objPtr->objEval(Xa);
    return (Fa - phialpha) / dalpha;
}

void BFGS::lineSearchZoom(double alo, double ahi, double plo, double phi, double dlo, double dhi, double phi0,
                          double dphi0, vector<double>& X, vector<double>& p, double& alphaOpt, double& phiOpt,
                          double& dphiOpt) {
    // BFGS_with_linesearch.cpp:296-356
    int it = 0;
    for (; it < maxIterLineSearch; ++it) {
        const double aj = cubicInterpMin(alo, ahi, plo, phi, dlo, dhi, X, p);
        // lineSearchObj + lineSearchFDDerivative as one batch of two points
        const double a2[2] = {aj, aj + dalpha};
        double f2[2];
        eval_line_points(objPtr, X, p, a2, 2, f2);
        if (profile) profile[kProfPoints] += 2;
        const double pj = f2[0];
        const double dj = (f2[1] - pj) / dalpha;
        if (pj > phi0 + c1 * aj * dphi0 || pj >= plo) {
            ahi = aj; phi = pj; dhi = dj;
            continue;
        }
        if (std::fabs(dj) <= std::fabs(c2 * dphi0)) {
            alphaOpt = aj; phiOpt = pj; dphiOpt = dj;
            if (verbose) std::cout << "Zoom ending after " << it << " iterations and satisfying curvature condition." << std::endl;
            return;
        }
        if (dj * (ahi - alo) >= 0) { ahi = alo; phi = plo; dhi = dlo; }
        alo = aj; plo = pj; dlo = dj;
    }
}

void BFGS::cubicInterpolationLineSearch(vector<double>& X, double FX, vector<double>& dFdX, vector<double>& p,
                                        double& alphaOpt, double& Fopt) {
    // BFGS_with_linesearch.cpp:177-291
    double dphiOpt = 0;
    alphaOpt = 0;
    Fopt = FX;
    const double phi0 = FX, dphi0 = seq_dot(dFdX, p);
    double aim1 = 0, pim1 = phi0, dim1 = dphi0;
    double ai = alphaGuess;
    for (int it = 0; it < maxIterLineSearch; ++it) {
        const double a2[2] = {ai, ai + dalpha};
        double f2[2];
        eval_line_points(objPtr, X, p, a2, 2, f2);
        if (profile) profile[kProfPoints] += 2;
        const double pi = f2[0];
        const double di = (f2[1] - pi) / dalpha;
        if ((pi > phi0 + c1 * ai * dphi0) || (pi >= pim1 && it > 1)) {
            lineSearchZoom(aim1, ai, pim1, pi, dim1, di, phi0, dphi0, X, p, alphaOpt, Fopt, dphiOpt);
            return;
        }
        if (std::fabs(di) <= std::fabs(c2 * dphi0)) {
            alphaOpt = ai;
            Fopt = pi;
            return;
        }
        if (di >= 0) {
            lineSearchZoom(ai, aim1, pi, pim1, di, dim1, phi0, dphi0, X, p, alphaOpt, Fopt, dphiOpt);
            return;
        }
        aim1 = ai; pim1 = pi; dim1 = di;
        ai = 2 * ai;
    }
}

void BFGS::findMin(vector<double>& X, double& f0, double& fOpt) {
    // BFGS_with_linesearch.cpp:12-139
    const int n = (int)X.size();
    PhaseClock total(prof_slot(profile, kProfTotal));
    pnol_ctx* ctx = require_ctx();
    DenseInverseHessian D(ctx, n, updateMode);
    if (initHessFD) init_from_fd_hessian(objPtr, X, dXHess, D);
    else D.setIdentity();

    std::vector<double> dX(n, dXGrad), dFdX(n), dFdXprev(n), p(n), pnext(n), s(n), y(n), Xprev(n);
    {
        PhaseClock t(prof_slot(profile, kProfGrad));
        objPtr->gradientApproximation(X, dX, dFdX);
        if (profile) profile[kProfGradCalls] += 1;
    }
    double F = objPtr->objEval(X);
    f0 = F;
    int iter = 0;
    double xdiff = xMinDiff * 2, gnorm = 2 * minGrad2Norm;
    bool have_next = false;
    while (iter < maxIter && xdiff > xMinDiff && gnorm > minGrad2Norm) {
        dFdXprev = dFdX;
        if (have_next) {
            p = pnext;
        } else {
            PhaseClock t(prof_slot(profile, kProfUpdate));
            D.direction(dFdX, p);
        }
        double alpha = 0, Fopt = 0;
        {
            PhaseClock t(prof_slot(profile, kProfLineSearch));
            cubicInterpolationLineSearch(X, F, dFdX, p, alpha, Fopt);
        }
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        F = Fopt;
        {
            PhaseClock t(prof_slot(profile, kProfGrad));
            objPtr->gradientApproximation(X, dX, dFdX);
            if (profile) profile[kProfGradCalls] += 1;
        }
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = dFdX[i] - dFdXprev[i]; }
        {
            PhaseClock t(prof_slot(profile, kProfUpdate));
            D.update(y, s, &dFdX, &pnext);
        }
        have_next = true;
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += std::fabs(X[i] - Xprev[i]);
        gnorm = std::sqrt(seq_dot(dFdX, dFdX));
        if (verbose) {
            std::cout << "At iter = " << iter << " the mean abs xdiff is " << xdiff << " and the grad2norm = " << gnorm
                      << std::endl;
            std::cout << " with a minimum function evaluation of " << F << std::endl;
        }
        iter = iter + 1;
    }
    if (profile) profile[kProfIters] = iter;
    fOpt = F;
    if (verbose) {
        std::cout << std::endl << "-----------------------------------------------------------------------------------" << std::endl;
        std::cout << "Completed bfgs." << std::endl;
        std::cout << "f0 = " << f0 << ", fOpt = " << fOpt << " with variable:" << std::endl;
        std::cout << "X = ";
        print_vec(X);
        std::cout << "-----------------------------------------------------------------------------------" << std::endl << std::endl;
    }
}
