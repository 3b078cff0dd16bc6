// bfgs_mpi.cpp -- BFGS_MPI: sharded FD gradient + pooled secant line search (drop-in for
// Source/BFGS_with_linesearch_MPI.cpp).  The pool of trial step sizes is evaluated round-robin
// over the ranks and gathered with one allgather per round (:163-223).
#include <cmath>
#include <cstdio>
#include <iostream>

#include "../pnol_comm.hpp"
#include "BFGS_with_linesearch_MPI.hpp"
#include "dense_hessian.hpp"
#include "line_points.hpp"

using namespace pnol;

namespace {

void vector_min(const std::vector<double>& v, size_t n, double& val, int& idx) {
    val = v[0]; idx = 0;
    for (size_t i = 1; i < n; ++i) if (v[i] < val) { val = v[i]; idx = (int)i; }
}
void vector_max(const std::vector<double>& v, size_t n, double& val, int& idx) {
    val = v[0]; idx = 0;
    for (size_t i = 1; i < n; ++i) if (v[i] > val) { val = v[i]; idx = (int)i; }
}
void linspace(double a, double b, int N, std::vector<double>& v) {
    v.resize(N);
    for (int i = 0; i < N; ++i) v[i] = a + i * (b - a) / (N - 1);
}

}  // namespace

void findPoolBounds(vector<double>& ap, vector<double>& pp, double a0, double p0, double& a1, double& a2, double& p1,
                    double& p2) {
    // BFGS_with_linesearch_MPI.cpp:496-530.  The reference reads past the pool end when the
    // minimum is its last entry (undefined behaviour); the index is clamped to the pool.
    double pmin; int imin;
    vector_min(pp, pp.size(), pmin, imin);
    const int N = (int)pp.size();
    const int hi = imin + 1 < N ? imin + 1 : N - 1;
    if (p0 < pmin) {
        a1 = a0; a2 = ap[0]; p1 = p0; p2 = pp[0];
    } else if (p0 >= pmin && imin == 0) {
        a1 = a0; a2 = ap[hi]; p1 = p0; p2 = pp[hi];
    } else {
        a1 = ap[imin - 1]; a2 = ap[hi]; p1 = pp[imin - 1]; p2 = pp[hi];
    }
}

double BFGS_MPI::lineSearchObj(double alpha, vector<double>& X, vector<double>& p) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + alpha * p[i];
    return objPtr->objEval(Xa);
}

void BFGS_MPI::evalAlphaPoolMPI(vector<double>& alphaPool, vector<double>& phiPool, vector<double>& X,
                                vector<double>& p) {
    // entry k is owned by rank k mod P (:186-197); one allgather of ceil(N/P) values per rank
    const int N = (int)phiPool.size();
    const int P = comm_size(), r = comm_rank();
    const int per = (N + P - 1) / P;
    std::vector<double> mine(per, 0.0), all((size_t)per * P, 0.0);
    std::vector<double> mya;   // this rank's entries, one batch
    for (int k = r; k < N; k += P) mya.push_back(alphaPool[k]);
    eval_line_points(objPtr, X, p, mya.data(), (int)mya.size(), mine.data());
    check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)per), "allgather(alpha pool)");
    for (int k = 0; k < N; ++k) phiPool[k] = all[(size_t)(k % P) * per + k / P];
}

void BFGS_MPI::secantLineSearch(vector<double>& X, double FX, vector<double>& dFdX, vector<double>& p,
                                double& alphaOpt, double& Fopt) {
    // BFGS_with_linesearch_MPI.cpp:226-492
    const int Np = poolSize > 0 ? poolSize : comm_size();
    std::vector<double> ap(Np, 0.0), pp(Np, 0.0), apPrev(Np, -1.0), ppPrev(Np, 0.0), slope(Np, 0.0);
    alphaOpt = 0;
    Fopt = FX;
    const double a0 = 0, phi0 = FX, dphi0 = seq_dot(dFdX, p);
    int idxMin = -(int)std::ceil((Np - 1.0) / 2.0);
    const int idxMax = (int)std::floor((Np - 1.0) / 2.0);
    double r = std::pow(maxAlphaMult, 1.0 / (double)idxMax);
    for (int k = 0, idx = idxMin; k < Np; ++k, ++idx) ap[k] = alphaGuess * std::pow(r, idx);

    bool first = true, zoom = false;
    // best point seen, for the optional zero-pool fix
    double bestA = 0, bestP = phi0;
    for (int it = 0; it < maxIterLineSearch && first; ++it) {
        evalAlphaPoolMPI(ap, pp, X, p);
        for (int i = 0; i < Np; ++i) if (pp[i] < bestP) { bestP = pp[i]; bestA = ap[i]; }
        for (int i = 0; i < Np; ++i)
            if (pp[i] > phi0 + c1 * ap[i] * dphi0) { zoom = true; first = false; }
        slope[0] = (pp[0] - phi0) / (ap[0] - a0);
        for (int i = 1; i < Np; ++i) slope[i] = (pp[i] - pp[i - 1]) / (ap[i] - ap[i - 1]);
        if (first)
            for (int i = 0; i < Np; ++i)
                if (std::fabs(slope[i]) <= std::fabs(c2 * dphi0)) { zoom = false; first = false; }
        if (first)
            for (int i = 0; i < Np; ++i)
                if (slope[i] >= 0) { zoom = true; first = false; }
        if (first) {
            double amax; int imax;
            vector_max(ap, ap.size(), amax, imax);
            r = std::pow(maxAlphaMult, 1.0 / (double)Np);
            for (int i = 0; i < Np; ++i) {
                apPrev[i] = ap[i];
                ppPrev[i] = pp[i];
                const double power = i + 1;
                ap[i] = amax * std::pow(r, power);
            }
        }
    }
    double alo, ahi, plo, phi;
    if (apPrev[0] < 0) {
        findPoolBounds(ap, pp, a0, phi0, alo, ahi, plo, phi);
    } else {
        std::vector<double> ae(2 * Np), pe(2 * Np);
        for (int i = 0; i < Np; ++i) { ae[i] = apPrev[i]; ae[i + Np] = ap[i]; pe[i] = ppPrev[i]; pe[i + Np] = pp[i]; }
        findPoolBounds(ae, pe, a0, phi0, alo, ahi, plo, phi);
    }
    std::vector<double> ap2(Np + 2, 0.0), pp2(Np + 2, 0.0);
    const bool zoomed = zoom;
    for (int it = 0; it < maxIterLineSearch && zoom; ++it) {
        linspace(alo, ahi, Np + 2, ap2);
        pp2[0] = plo; pp2[Np + 1] = phi; ap2[0] = alo; ap2[Np + 1] = ahi;
        for (int i = 0; i < Np; ++i) { ap[i] = ap2[i + 1]; pp[i] = pp2[i + 1]; }
        evalAlphaPoolMPI(ap, pp, X, p);
        for (int i = 0; i < Np; ++i) { ap2[i + 1] = ap[i]; pp2[i + 1] = pp[i]; }
        for (int i = 0; i < Np; ++i) slope[i] = (pp2[i + 1] - pp2[i]) / (ap2[i + 1] - ap2[i]);
        for (int i = 0; i < Np; ++i)
            if (std::fabs(slope[i]) <= std::fabs(c2 * dphi0)) zoom = false;
        if (zoom) findPoolBounds(ap2, pp2, a0, phi0, alo, ahi, plo, phi);
    }
    if (!zoomed && fixZeroPool) {
        // the reference would report the untouched zero pool (alpha 0, F 0, :483-488)
        alphaOpt = bestA;
        Fopt = bestP;
        return;
    }
    double pmin; int imin;
    vector_min(pp2, pp2.size(), pmin, imin);
    alphaOpt = ap2[imin];
    Fopt = pmin;
}

void BFGS_MPI::findMin(vector<double>& X, double& f0, double& fOpt) {
    // BFGS_with_linesearch_MPI.cpp:12-142
    require_comm("BFGS_MPI::findMin");   // Npool = Nprocs of MPI_COMM_WORLD (:231-235)
    const int n = (int)X.size();
    const int rank = comm_rank();
    pnol_ctx* ctx = require_ctx();
    DenseInverseHessian D(ctx, n, updateMode, true);   // row-sharded over the ranks
    if (initHessFD) {
        init_from_fd_hessian(objPtr, X, dXHess, D);
    } else {
        D.setIdentity();
    }
    std::vector<double> dX(n, dXGrad), dFdX(n), dFdXprev(n), p(n), pnext(n), s(n), y(n), Xprev(n);
    objPtr->gradientApproximationMPI(X, dX, dFdX);
    double F = objPtr->objEval(X);
    f0 = F;
    int iter = 0;
    double xdiff = xMinDiff * 2, gnorm = 2 * minGrad2Norm;
    bool have_next = false;
    while (iter < maxIter && xdiff > xMinDiff && gnorm > minGrad2Norm) {
        dFdXprev = dFdX;
        if (have_next) p = pnext;
        else D.direction(dFdX, p);
        double alpha = 0, Fopt = 0;
        secantLineSearch(X, F, dFdX, p, alpha, Fopt);
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        F = Fopt;
        objPtr->gradientApproximationMPI(X, dX, dFdX);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = dFdX[i] - dFdXprev[i]; }
        D.update(y, s, &dFdX, &pnext);
        have_next = true;
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += std::fabs(X[i] - Xprev[i]);
        gnorm = std::sqrt(seq_dot(dFdX, dFdX));
        if (verbose && rank == 0) {
            std::cout << "---> At iter = " << iter << " the mean abs xdiff is " << xdiff << " and the grad2norm = "
                      << gnorm << std::endl;
            std::cout << "                 with a minimum function evaluation of " << F << std::endl;
        }
        iter = iter + 1;
    }
    fOpt = F;
    if (verbose && rank == 0) {
        std::cout << std::endl << "-----------------------------------------------------------------------------------" << std::endl;
        std::cout << "Completed bfgs." << std::endl;
        std::cout << "f0 = " << f0 << ", fOpt = " << fOpt << " with variable:" << std::endl << "X = ";
        for (double v : X) std::printf("%.17g ", v);
        std::printf("\n");
        std::cout << "-----------------------------------------------------------------------------------" << std::endl << std::endl;
    }
}
