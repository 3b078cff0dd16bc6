// bfgs_bnd_mpi_sw.cpp -- BFGS_Bnd_MPI_SW: bounded BFGS with a pooled Wolfe line search (each
// pool entry is a step size and its forward-difference slope) and BFGS_Bnd's active-set
// recursion (drop-in for Source/BFGS_bnd_linesearch_MPI_SW.cpp).  Pool entries go round-robin
// to the ranks and come back with one allgather (the reference's zero-padded Reduce + Bcast,
// :646-682, is exact for one owner per entry); the gradients are sharded (MPIRecur).
#include <cmath>
#include <cstdio>
#include <iostream>

#include "../pnol_comm.hpp"
#include "BFGS_bnd_linesearch_MPI_SW.hpp"
#include "deep_stack.hpp"
#include "dense_hessian.hpp"
#include "line_points.hpp"

using namespace pnol;

namespace {

void vector_min(const std::vector<double>& v, double& val, int& idx) {
    val = v[0]; idx = 0;
    for (size_t i = 1; i < v.size(); ++i) if (v[i] < val) { val = v[i]; idx = (int)i; }
}
void linspace(double a, double b, int N, std::vector<double>& v) {
    v.resize(N);
    for (int i = 0; i < N; ++i) v[i] = a + i * (b - a) / (N - 1);
}
void print_vec(const std::vector<double>& v) {
    for (double x : v) std::printf("%.17g ", x);
    std::printf("\n");
}

// computeZoomPool, BFGS_bnd_linesearch_MPI_SW.cpp:434-482: Npool points from alpha_a to
// alpha_b, one of them the cubic-interpolation minimiser; the two ends are already known
void compute_zoom_pool(double aa, double ab, double pa, double pb, double da, double db, std::vector<double>& ap,
                       std::vector<double>& pp, std::vector<double>& dp, std::vector<int>& ev) {
    const int Npool = (int)ap.size();
    double ac = cubicInterpMinSimple(aa, ab, pa, pb, da, db);
    if (ac == (aa + ab) / 2) {
        linspace(aa, ab, Npool, ap);
    } else {
        std::vector<double> al;
        linspace(aa, ab, Npool - 1, al);
        ap[0] = al[0];
        int il = 1;
        for (int i = 1; i < Npool; ++i) {
            // after the insertion ac = -1 fails the first test, so al[il] is never read past its end
            if (ac >= al[il - 1] && ac <= al[il]) { ap[i] = ac; ac = -1; }
            else { ap[i] = al[il]; il++; }
        }
    }
    for (int i = 0; i < Npool; ++i) ev[i] = 1;
    pp[0] = pa; dp[0] = da; ev[0] = 0;
    pp[Npool - 1] = pb; dp[Npool - 1] = db; ev[Npool - 1] = 0;
}

}  // namespace

void computeZoomRegion(vector<double>& ap, vector<double>& pp, vector<double>& dp, double& aa, double& ab,
                       double& pa, double& pb, double& da, double& db) {
    // :399-431.  The reference reads one entry past the pool when the minimum sits on its first
    // entry with a positive slope (or on its last with a non-positive one); that read is
    // undefined behaviour, so the neighbour index is clamped to the pool (a zero-width bracket).
    double pmin; int im;
    vector_min(pp, pmin, im);
    const int N = (int)pp.size();
    int lo, hi;
    if (dp[im] > 0) { lo = im - 1 >= 0 ? im - 1 : 0; hi = im; }
    else { lo = im; hi = im + 1 < N ? im + 1 : N - 1; }
    aa = ap[lo]; ab = ap[hi]; pa = pp[lo]; pb = pp[hi]; da = dp[lo]; db = dp[hi];
}

BFGS_Bnd_MPI_SW::BFGS_Bnd_MPI_SW()
    : c1(1e-4), c2(0.9), dalpha(1e-6), alphaGuess(1), alphaTol(1e-20), alphaMult(2), maxIterLineSearch(50),
      bndTol(1e-5), dXGrad(1e-6), dXHess(1e-3), xMinDiff(1e-5), minGrad2Norm(1e-5), maxIter(10000), totalIter(0),
      initHessFD(false), verbose(0), Nprocs(comm_size()), procID(comm_rank()), optimFlag(true), recurFlag(0) {}

double BFGS_Bnd_MPI_SW::lineSearchObj(double alpha, vector<double>& X, vector<double>& p, vector<double>& cX,
                                      vector<bool>& cI) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + alpha * p[i];
    return objPtr->objEvalRecur(Xa, cX, cI);
}

double BFGS_Bnd_MPI_SW::lineSearchFDDerivative(double alpha, double phialpha, vector<double>& X, vector<double>& p,
                                               vector<double>& cX, vector<bool>& cI) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + (alpha + dalpha) * p[i];
    const double Fa = objPtr->objEvalRecur(Xa, cX, cI);
    return (Fa - phialpha) / dalpha;
}

void BFGS_Bnd_MPI_SW::evaluateAlphaPoolAndDerivatives(vector<double>& ap, vector<double>& X, vector<double>& p,
                                                      vector<double>& cX, vector<bool>& cI, vector<double>& pp,
                                                      vector<double>& dp) {
    // :599-699: entry k is owned by rank k mod P; (phi, dphi) pairs, one allgather
    const int N = (int)ap.size();
    const int P = comm_size(), r = comm_rank();
    const int per = (N + P - 1) / P > 0 ? (N + P - 1) / P : 1;
    std::vector<double> mine(2 * (size_t)per, 0.0), all(2 * (size_t)per * P, 0.0);
    // this rank's entries as one batch of (alpha, alpha + dalpha) pairs, in the reference's order
    std::vector<double> mya, fv;
    for (int k = r; k < N; k += P) { mya.push_back(ap[k]); mya.push_back(ap[k] + dalpha); }
    fv.resize(mya.size());
    eval_line_points_recur(objPtr, X, p, mya.data(), (int)mya.size(), cX, cI, fv.data());
    for (int q = 0; q < per; ++q) {
        const int k = r + q * P;
        if (k >= N) continue;
        double phi = fv[2 * q];
        const double dphi = (fv[2 * q + 1] - phi) / dalpha;
        if (phi != phi || std::isinf(phi)) {
            phi = 1e10;
            std::cout << "Line search crashed with " << std::endl << phi << std::endl << "Ending search..." << std::endl;
        }
        mine[2 * q] = phi;
        mine[2 * q + 1] = dphi;
    }
    check(comm_allgather_host(nullptr, mine.data(), all.data(), 2 * (size_t)per), "allgather(alpha pool)");
    for (int k = 0; k < N; ++k) {
        const size_t at = 2 * ((size_t)(k % P) * per + k / P);
        pp[k] = all[at];
        dp[k] = all[at + 1];
    }
    for (int k = 0; k < N; ++k)
        if (pp[k] == 1e10) {
            std::cout << "Line search crashed ... ending search..." << std::endl;
            optimFlag = false;
        }
}

void BFGS_Bnd_MPI_SW::evaluateAlphaPoolAndDerivativesIndicator(vector<double>& ap, vector<int> ev, vector<double>& X,
                                                               vector<double>& p, vector<double>& cX, vector<bool>& cI,
                                                               vector<double>& pp, vector<double>& dp) {
    // :552-594: evaluate the flagged entries only
    std::vector<double> at, pt, dt;
    for (size_t i = 0; i < ev.size(); ++i)
        if (ev[i] == 1) { at.push_back(ap[i]); pt.push_back(pp[i]); dt.push_back(dp[i]); }
    evaluateAlphaPoolAndDerivatives(at, X, p, cX, cI, pt, dt);
    size_t t = 0;
    for (size_t i = 0; i < ev.size(); ++i)
        if (ev[i] == 1) { ap[i] = at[t]; pp[i] = pt[t]; dp[i] = dt[t]; t++; }
    if (verbose > 2 && procID == ROOT_ID) {
        std::cout << "alphaPool = "; print_vec(ap);
        std::cout << "phiPool = "; print_vec(pp);
        std::cout << "dphidalphaPool = "; print_vec(dp);
    }
}

void BFGS_Bnd_MPI_SW::lineSearchZoomBnd(double aa, double ab, double pa, double pb, double da, double db, double phi0,
                                        double dphi0, vector<double>& X, vector<double>& p, vector<double>& cX,
                                        vector<bool>& cI, int& iter_ls, double& aOpt, double& pOpt, double& dOpt) {
    // :484-548: Nprocs interior points per round
    const int Npool = (poolSize > 0 ? poolSize : Nprocs) + 2;
    std::vector<int> ev(Npool, 1);
    std::vector<double> ap(Npool, 0.0), pp(Npool, 0.0), dp(Npool, 0.0);
    bool zoomFlag = true, success = false;
    while (iter_ls < maxIterLineSearch && (ab - aa > alphaTol) && zoomFlag) {
        compute_zoom_pool(aa, ab, pa, pb, da, db, ap, pp, dp, ev);
        evaluateAlphaPoolAndDerivativesIndicator(ap, ev, X, p, cX, cI, pp, dp);
        for (int i = 1; i < Npool - 1; ++i)
            if ((pp[i] <= phi0 + c1 * ap[i] * dphi0) && (std::fabs(dp[i]) <= std::fabs(c2 * dphi0))) {
                zoomFlag = false;
                success = true;
            }
        if (!success) computeZoomRegion(ap, pp, dp, aa, ab, pa, pb, da, db);
        iter_ls++;
    }
    // the best member of the last pool (all zeros if the loop did not run, as in the reference)
    double pmin; int im;
    vector_min(pp, pmin, im);
    aOpt = ap[im];
    pOpt = pmin;
    dOpt = dp[im];
}

void BFGS_Bnd_MPI_SW::cubicInterpolationLineSearchBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub,
                                                      double FX, vector<double>& dFdX, vector<double>& p,
                                                      vector<double>& cX, vector<bool>& cI, double& aOpt,
                                                      double& Fopt) {
    // :209-397
    const int procs = poolSize > 0 ? poolSize : Nprocs;
    bool bndIndicator = false;
    double pOpt = FX, dOpt = 0;
    aOpt = 0;
    Fopt = FX;
    const double phi0 = FX, dphi0 = seq_dot(dFdX, p);
    const int Npool = procs + 1;
    std::vector<int> ev(Npool, 1);
    std::vector<double> ap(Npool, 0.0), pp(Npool, 0.0), dp(Npool, 0.0);
    ev[0] = 0;            // alpha = 0 is known
    ap[0] = 0;
    pp[0] = phi0;
    dp[0] = dphi0;
    const double alphaMax = computeAlphaBnd(X, Xlb, Xub, p);
    double ai = alphaGuess;
    if (ai > alphaMax) ai = alphaMax;
    const double delta = ai / procs;
    for (int i = 1; i < Npool; ++i) ap[i] = delta * i;

    int iter_ls = 0;
    bool extendFlag = true, zoomFlag = false;
    while (iter_ls < maxIterLineSearch && extendFlag) {
        evaluateAlphaPoolAndDerivativesIndicator(ap, ev, X, p, cX, cI, pp, dp);
        // 1. the interval is large enough (value)
        for (int i = 1; i < Npool; ++i)
            if ((pp[i] > phi0 + c1 * ap[i] * dphi0) || (pp[i] >= pp[0] && iter_ls > 1)) {
                extendFlag = false; zoomFlag = true;
            }
        // 2. a point meets the curvature condition
        for (int i = 1; i < Npool; ++i)
            if (std::fabs(dp[i]) <= std::fabs(c2 * dphi0)) { extendFlag = false; zoomFlag = false; }
        // 3. the interval is large enough (slope)
        for (int i = 1; i < Npool; ++i)
            if (dp[i] >= 0) { extendFlag = false; zoomFlag = true; }
        // 4. still extending but already at the box edge
        if (extendFlag && ap[Npool - 1] == alphaMax) {
            extendFlag = false; zoomFlag = false; bndIndicator = true;
        }
        // 5. extend from the last point
        if (extendFlag) {
            double an = (procs + 1) * ap[Npool - 1];
            if (an > alphaMax) an = alphaMax;
            linspace(ap[Npool - 1], an, Npool, ap);
            for (int i = 0; i < Npool; ++i) ev[i] = 1;
            ev[0] = 0;
            pp[0] = pp[Npool - 1];
            dp[0] = dp[Npool - 1];
        }
        iter_ls++;
    }

    if (zoomFlag) {
        double aa, ab, pa, pb, da, db;
        computeZoomRegion(ap, pp, dp, aa, ab, pa, pb, da, db);
        if (ab - aa > alphaTol) {
            lineSearchZoomBnd(aa, ab, pa, pb, da, db, phi0, dphi0, X, p, cX, cI, iter_ls, aOpt, pOpt, dOpt);
        } else {
            double pmin; int im;
            vector_min(pp, pmin, im);
            aOpt = ap[im]; pOpt = pmin; dOpt = dp[im];
        }
        Fopt = pOpt;
    } else {
        double pmin; int im;
        vector_min(pp, pmin, im);
        aOpt = ap[im]; pOpt = pmin; dOpt = dp[im];
        Fopt = pOpt;
    }
    if (verbose > 0 && procID == ROOT_ID) {
        if (!bndIndicator)
            std::cout << "  Line search completed with alpha = " << aOpt << " and F = " << Fopt << " after " << iter_ls
                      << " iterations. Note: alphaMax = " << alphaMax << std::endl;
        else
            std::cout << "  ! Line search terminated at boundary with alpha = " << aOpt << " and F = " << Fopt
                      << " after " << iter_ls << " iterations. Note: alphaMax = " << alphaMax << std::endl;
    }
}

void BFGS_Bnd_MPI_SW::boundaryAssessment(double& F, vector<double>& X, vector<double>& p, vector<double>& dFdX,
                                         DenseInverseHessian& D, vector<double>& Xlb, vector<double>& Xub,
                                         vector<double>& dX, vector<double>& cX, vector<bool>& cI) {
    // :741-967 (BFGS_Bnd's recursion with the gradients sharded)
    const int ncur = (int)X.size();
    const int Ndim = (int)cX.size();
    std::vector<bool> cIcur(ncur, false);
    std::vector<int> frozen;
    bool bndFlag = false;
    int icur = 0;
    for (int i = 0; i < Ndim; ++i) {
        if (cI[i]) continue;
        if ((std::fabs(X[icur] - Xlb[icur]) < bndTol) && ((p[icur] < 0) || (dFdX[icur] > 0))) {
            bndFlag = true; cI[i] = true; cX[i] = X[icur]; cIcur[icur] = true; frozen.push_back(i);
        } else if ((std::fabs(X[icur] - Xub[icur]) < bndTol) && ((p[icur] > 0) || (dFdX[icur] < 0))) {
            bndFlag = true; cI[i] = true; cX[i] = X[icur]; cIcur[icur] = true; frozen.push_back(i);
        }
        icur++;
    }
    int Nconst = 0;
    for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
    if (bndFlag && verbose > 0 && procID == ROOT_ID) {
        std::cout << std::endl << "Optimizer reached box boundary and found that the steepest descent is directed "
                  << "outside of the boundary at " << frozen.size() << " coordinate(s)." << std::endl << "    X = ";
        print_vec(X);
        std::cout << "    F = " << F << std::endl;
    }
    const int nr = Ndim - Nconst;
    if (bndFlag && nr > 0) {
        double FR = F;
        std::vector<double> XR, gR, lbR, ubR, dXR;
        for (icur = 0; icur < ncur; ++icur)
            if (!cIcur[icur]) {
                XR.push_back(X[icur]); gR.push_back(dFdX[icur]); lbR.push_back(Xlb[icur]);
                ubR.push_back(Xub[icur]); dXR.push_back(dX[icur]);
            }
        // the reduced problem starts along steepest descent (scaled if a scaling was set)
        DenseInverseHessian DR(D, nr, updateMode, true);   // D's buffer: it is reset on return
        if (!initialScalingVec.empty()) {
            std::vector<double> scaleR;
            for (int i = 0; i < Ndim; ++i) if (!cI[i]) scaleR.push_back(initialScalingVec[i]);
            DR.setIdentity(&scaleR);
        } else {
            DR.setIdentity();
        }
        recurFlag = true;
        mainBFGSLoop(FR, XR, gR, DR, lbR, ubR, dXR, cX, cI);
        int ir = 0;
        for (icur = 0; icur < ncur; ++icur)
            if (!cIcur[icur]) {
                F = FR; X[icur] = XR[ir]; dFdX[icur] = gR[ir]; Xlb[icur] = lbR[ir]; Xub[icur] = ubR[ir];
                dX[icur] = dXR[ir];
                ir++;
            }
        for (int k : frozen) cI[k] = false;
        if (!initialScalingVec.empty()) {
            std::vector<double> scale;
            for (int i = 0; i < Ndim; ++i) if (!cI[i]) scale.push_back(initialScalingVec[i]);
            scale.resize(ncur, 1.0);
            D.setIdentity(&scale);
        } else {
            D.setIdentity();
        }
        objPtr->gradientApproximationMPIRecur(X, dX, dFdX, cX, cI);
        bool cont = false;
        for (icur = 0; icur < ncur; ++icur)
            if (cIcur[icur]) {
                if ((std::fabs(X[icur] - Xlb[icur]) < bndTol) && (dFdX[icur] < 0)) cont = true;
                else if ((std::fabs(X[icur] - Xub[icur]) < bndTol) && (dFdX[icur] > 0)) cont = true;
            }
        Nconst = 0;
        for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
        if (Nconst == 0) recurFlag = false;
        optimFlag = cont;
        if (verbose > 1 && procID == ROOT_ID)
            std::cout << (cont ? "     Optimization continuing after recursive boundary optimization."
                               : "     Optimization exiting after recursive boundary optimization.")
                      << std::endl;
    } else if (nr == 0) {
        optimFlag = false;
        if (verbose > 1 && procID == ROOT_ID) std::cout << "      NO VARIABLES LEFT TO OPTIMIZE!!!! " << std::endl;
    }
}

void BFGS_Bnd_MPI_SW::mainBFGSLoop(double& F, vector<double>& X, vector<double>& dFdX, DenseInverseHessian& D,
                                   vector<double>& Xlb, vector<double>& Xub, vector<double>& dX, vector<double>& cX,
                                   vector<bool>& cI) {
    // :116-207
    const int n = (int)X.size();
    std::vector<double> gprev = dFdX, p(n), s(n), y(n), Xprev(n);
    int iter = 0;
    double xdiff = xMinDiff * 2, gnorm = 2 * minGrad2Norm;
    while (optimFlag && iter < maxIter && xdiff > xMinDiff && gnorm > minGrad2Norm && totalIter < maxIter) {
        if (verbose > 0 && procID == ROOT_ID)
            std::cout << std::endl << "Iter = " << iter << " of bounded BFGS search starting with previous F = " << F
                      << "." << std::endl;
        D.direction(dFdX, p);
        double alpha = 0, Fopt = 0;
        cubicInterpolationLineSearchBnd(X, Xlb, Xub, F, dFdX, p, cX, cI, alpha, Fopt);
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        F = Fopt;
        gprev = dFdX;
        objPtr->gradientApproximationMPIRecur(X, dX, dFdX, cX, cI);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = dFdX[i] - gprev[i]; }
        D.update(y, s, nullptr, nullptr);
        boundaryAssessment(F, X, p, dFdX, D, Xlb, Xub, dX, cX, cI);
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += std::fabs(X[i] - Xprev[i]);
        gnorm = std::sqrt(seq_dot(dFdX, dFdX));
        if (verbose > 0 && procID == ROOT_ID) {
            std::cout << "  Step completed with F = " << F << " and mean abs xdiff is " << xdiff
                      << " and the grad2norm = " << gnorm << std::endl;
            if (verbose > 1) { std::cout << "  X = "; print_vec(X); }
        }
        iter = iter + 1;
        totalIter = totalIter + 1;
    }
}

void BFGS_Bnd_MPI_SW::findMinBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0,
                                 double& fOpt) {
    // the communicator is bound on the calling thread; the active-set recursion is one level
    // per frozen coordinate (deep_stack.hpp)
    require_comm("BFGS_Bnd_MPI_SW::findMinBnd");
    run_deep([&] { findMinBndBody(X, Xlb, Xub, f0, fOpt); });
}

void BFGS_Bnd_MPI_SW::findMinBndBody(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0,
                                     double& fOpt) {
    // :12-113
    totalIter = 0;
    Nprocs = comm_size();
    procID = comm_rank();
    if (verbose >= 0 && procID == ROOT_ID) {
        std::cout << std::endl << "  Starting parallel bounded BFGS with line search. " << std::endl << "  X0 = ";
        print_vec(X);
    }
    const int n = (int)X.size();
    checkBoxBounds(X, Xlb, Xub);
    std::vector<double> cX(n, 0.0), X0 = X, dX(n, dXGrad), dFdX(n, 0.0);
    std::vector<bool> cI(n, false);
    if (!dXGradVec.empty())
        for (int i = 0; i < n; ++i) dX[i] = dXGradVec[i];
    DenseInverseHessian D(require_ctx(), n, updateMode, true);   // row-sharded over the ranks
    if (initHessFD) init_from_fd_hessian(objPtr, X, dXHess, D);
    else if (!initialScalingVec.empty()) D.setIdentity(&initialScalingVec);
    else D.setIdentity();
    objPtr->gradientApproximationMPIRecur(X, dX, dFdX, cX, cI);
    double F = objPtr->objEvalRecur(X, cX, cI);
    f0 = F;
    optimFlag = true;
    recurFlag = 0;
    mainBFGSLoop(F, X, dFdX, D, Xlb, Xub, dX, cX, cI);
    fOpt = F;
    if (verbose >= 0 && procID == ROOT_ID) {
        std::cout << std::endl << "  Completed bounded BFGS." << std::endl << "  X0 = ";
        print_vec(X0);
        std::cout << "  Xopt = ";
        print_vec(X);
        std::cout << "  f0 = " << f0 << ", fOpt = " << fOpt << std::endl << std::endl;
    }
}
