// bfgs_bnd.cpp -- bounded BFGS with active-set recursion (drop-in for
// Source/BFGS_bnd_linesearch.cpp) plus the box helpers (Box_boundary_functions.cpp:11-40,
// BFGS_with_bnd_linsearch_MPI.cpp:665-708).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "../pnol_comm.hpp"
#include "BFGS_bnd_linesearch.hpp"
#include "deep_stack.hpp"
#include "dense_hessian.hpp"
#include "line_points.hpp"
#include "recur_simd.hpp"

using namespace pnol;

namespace {
double sign_of(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }
// PNOL_BND_DETAIL=1: where the host time of the "other" phase goes (diagnostics, stderr)
enum { kDetFreeze, kDetGather, kDetCopyBack, kDetIterLoops, kDetCount };
thread_local double g_det[kDetCount];
double* det_slot(int k) {
    static const bool on = [] {
        const char* e = std::getenv("PNOL_BND_DETAIL");
        return e && std::atoi(e) != 0;
    }();
    return on ? &g_det[k] : nullptr;
}
// drop positions fk (ascending) of v[0, n): the kept entries slide down run by run
template <class T>
void drop_positions(std::vector<T>& v, const std::vector<int>& fk, int n) {
    if (fk.empty()) return;
    int dst = fk[0];
    for (size_t f = 0; f < fk.size(); ++f) {
        const int b = fk[f] + 1, e = f + 1 < fk.size() ? fk[f + 1] : n;
        std::copy(v.begin() + b, v.begin() + e, v.begin() + dst);
        dst += e - b;
    }
}
// the inverse: reopen the gaps at positions fk of v[0, n) (their contents are the caller's)
template <class T>
void reopen_positions(std::vector<T>& v, const std::vector<int>& fk, int n) {
    int hi = n;
    for (int f = (int)fk.size() - 1; f >= 0; --f) {
        const int b = fk[f] + 1;
        std::copy_backward(v.begin() + (b - f - 1), v.begin() + (hi - f - 1), v.begin() + hi);
        hi = fk[f];
    }
}
void print_vec(const std::vector<double>& v) {
    for (double x : v) std::printf("%.17g ", x);
    std::printf("\n");
}
}  // namespace

void checkBoxBounds(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub) {
    for (size_t i = 0; i < X.size(); ++i) {
        if (X[i] - Xlb[i] < -std::fabs(Xlb[i]) / 1000 || X[i] - Xub[i] > std::fabs(Xub[i]) / 1000) {
            if (comm_rank() == 0)
                std::cout << std::endl << "!!!!----------------- WARNING -----------------!!!!" << std::endl
                          << "X[" << i << "] = " << X[i] << " is outside of bounds Xlb[i] = " << Xlb[i]
                          << ", Xub[i] = " << Xub[i] << std::endl;
            X[i] = (Xlb[i] + Xub[i]) / 2.0;
            if (comm_rank() == 0)
                std::cout << " Replaced X[" << i << "] with " << X[i] << std::endl
                          << "!!!!----------------- END WARNING -----------------!!!!" << std::endl << std::endl;
        }
    }
}

double computeAlphaBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub,
                       std::vector<double>& p) {
    // the same value as the reference's loop: recur::alpha_bnd (eight quotients per AVX-512 step)
    return recur::alpha_bnd(X.data(), Xlb.data(), Xub.data(), p.data(), X.size());
}

double cubicInterpMinSimple(double aa, double ab, double pa, double pb, double da, double db) {
    const double d1 = da + db - 3 * (pa - pb) / (aa - ab);
    const double d2 = sign_of(ab - aa) * std::sqrt(d1 * d1 - da * db);
    double an = ab - (ab - aa) * (db + d2 - d1) / (db - da + 2 * d2);
    if (an < aa || an > ab || an != an) an = (aa + ab) / 2;
    return an;
}

double BFGS_Bnd::lineSearchObj(double alpha, vector<double>& X, vector<double>& p, vector<double>& cX,
                               vector<bool>& cI) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + alpha * p[i];
    return objPtr->objEvalRecur(Xa, cX, cI);
}

double BFGS_Bnd::lineSearchFDDerivative(double alpha, double phialpha, vector<double>& X, vector<double>& p,
                                        vector<double>& cX, vector<bool>& cI) {
    std::vector<double> Xa(X.size());
    for (size_t i = 0; i < X.size(); ++i) Xa[i] = X[i] + (alpha + dalpha) * p[i];
    const double Fa = objPtr->objEvalRecur(Xa, cX, cI);
    return (Fa - phialpha) / dalpha;
}

void BFGS_Bnd::lineSearchZoomBnd(double aa, double ab, double pa, double pb, double da, double db, double phi0,
                                 double dphi0, vector<double>& X, vector<double>& p, vector<double>& cX,
                                 vector<bool>& cI, int& iter_ls, double& aOpt, double& pOpt, double& dOpt) {
    // BFGS_bnd_linesearch.cpp:358-457
    bool success = false;
    while (iter_ls < maxIterLineSearch && (ab - aa > alphaTol)) {
        const double ac = cubicInterpMinSimple(aa, ab, pa, pb, da, db);
        const double a2[2] = {ac, ac + dalpha};   // the (phi, FD slope) pair as one batch
        double f2[2];
        eval_line_points_recur(objPtr, X, p, a2, 2, cX, cI, f2);
        if (profile) profile[kProfPoints] += 2;
        const double pc = f2[0];
        const double dc = (f2[1] - pc) / dalpha;
        double pmin = pa;
        if (pb < pa) pmin = pb;
        if (pc > phi0 + c1 * ac * dphi0 || pc >= pmin) {
            if (pa < pb) { ab = ac; pb = pc; db = dc; }
            else { aa = ac; pa = pc; da = dc; }
        } else {
            if (std::fabs(dc) <= std::fabs(c2 * dphi0)) {
                aOpt = ac; pOpt = pc; dOpt = dc; success = true;
                break;
            }
            if (dc < 0) { aa = ac; pa = pc; da = dc; }
            else { ab = ac; pb = pc; db = dc; }
        }
        iter_ls++;
    }
    if (!success) {
        if (pa < pb) { aOpt = aa; pOpt = pa; dOpt = da; }
        else { aOpt = ab; pOpt = pb; dOpt = db; }
    }
}

void BFGS_Bnd::cubicInterpolationLineSearchBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub,
                                               double FX, vector<double>& dFdX, vector<double>& p, vector<double>& cX,
                                               vector<bool>& cI, double& aOpt, double& Fopt) {
    // BFGS_bnd_linesearch.cpp:203-353
    bool success = false, atBound = false;
    double dOpt = 0, phii = 0;
    aOpt = 0;
    Fopt = FX;
    const double phi0 = FX, dphi0 = seq_dot(dFdX, p);
    double aim1 = 0, pim1 = phi0, dim1 = dphi0;
    const double amax = computeAlphaBnd(X, Xlb, Xub, p);
    double ai = alphaGuess;
    if (ai > amax) ai = amax;
    int iter_ls = 0;
    while (iter_ls < maxIterLineSearch) {
        const double a2[2] = {ai, ai + dalpha};
        double f2[2];
        eval_line_points_recur(objPtr, X, p, a2, 2, cX, cI, f2);
        if (profile) profile[kProfPoints] += 2;
        phii = f2[0];
        const double di = (f2[1] - phii) / dalpha;
        if ((phii > phi0 + c1 * ai * dphi0) || (phii >= pim1 && iter_ls > 1)) {
            lineSearchZoomBnd(aim1, ai, pim1, phii, dim1, di, phi0, dphi0, X, p, cX, cI, iter_ls, aOpt, Fopt, dOpt);
            success = true;
            break;
        }
        if (std::fabs(di) <= std::fabs(c2 * dphi0)) { aOpt = ai; Fopt = phii; success = true; break; }
        if (di >= 0) {
            lineSearchZoomBnd(aim1, ai, pim1, phii, dim1, di, phi0, dphi0, X, p, cX, cI, iter_ls, aOpt, Fopt, dOpt);
            success = true;
            break;
        }
        if (ai == amax) { aOpt = ai; Fopt = phii; atBound = true; success = true; break; }
        aim1 = ai; pim1 = phii; dim1 = di;
        ai = 2 * ai;
        if (ai > amax) ai = amax;
        iter_ls++;
    }
    if (!success) {
        if (pim1 < phii) { aOpt = aim1; Fopt = pim1; }
        else if (phi0 < phii) { aOpt = 0; Fopt = phi0; }
        else { aOpt = ai; Fopt = phii; }
    }
    if (verbose > 0 && comm_rank() == ROOT_ID) {
        if (!atBound)
            std::cout << "  Line search completed with alpha = " << aOpt << " and F = " << Fopt << " after " << iter_ls
                      << " iterations. Note: alphaMax = " << amax << std::endl << std::endl;
        else
            std::cout << "  ! Line search terminated at boundary with alpha = " << aOpt << " and F = " << Fopt
                      << " after " << iter_ls << " iterations. Note: alphaMax = " << amax << std::endl << std::endl;
    }
}

void BFGS_Bnd::boundaryAssessment(double& F, vector<double>& X, vector<double>& p, vector<double>& dFdX,
                                  DenseInverseHessian& D, vector<double>& Xlb, vector<double>& Xub, vector<double>& dX,
                                  vector<double>& cX, vector<bool>& cI, bool& optimFlag, int& recurFlag) {
    // BFGS_bnd_linesearch.cpp:503-728
    const int ncur = (int)X.size();
    const int Ndim = (int)cX.size();
    PhaseClock tf(det_slot(kDetFreeze));
    std::vector<int> fk, fi;   // positions in X frozen by this assessment (ascending), their full indices
    bool bndFlag = false;
    int Nconst = 0;            // coordinates frozen after the tests
    if (freeIdxLive && (int)freeIdx.size() == ncur) {
        // the level's coordinates are the free ones of cI in order (freeIdx): the reference's
        // walk over all Ndim indicators reduces to the tests over X's own positions
        recur::bound_hits(X.data(), Xlb.data(), Xub.data(), p.data(), dFdX.data(), (size_t)ncur, bndTol, fk);
        for (int k : fk) {
            const int i = freeIdx[k];
            cI[i] = true; cX[i] = X[k]; fi.push_back(i);
        }
        bndFlag = !fk.empty();
        Nconst = Ndim - ncur + (int)fk.size();
    } else {
        // any constantIndicator: the reference's walk, evaluated without short-circuit
        // branches (only a coordinate that hits a bound takes one)
        freeIdxLive = false;
        const int klast = ncur > 0 ? ncur - 1 : 0;
        int icur = 0;
        for (int i = 0; i < Ndim; ++i) {
            const bool c = cI[i];
            Nconst += c;
            if (ncur == 0) continue;
            const int k = icur < klast ? icur : klast;
            const double xk = X[k], pk = p[k], gk = dFdX[k];
            const bool lo = (std::fabs(xk - Xlb[k]) < bndTol) & ((pk < 0) | (gk > 0));
            const bool hi = (std::fabs(xk - Xub[k]) < bndTol) & ((pk > 0) | (gk < 0));
            if (!c & (lo | hi)) {
                bndFlag = true; cI[i] = true; cX[i] = xk; fi.push_back(i);
                if (icur < ncur) fk.push_back(icur);
            }
            icur += !c;
        }
        Nconst += (int)fi.size();   // == the count of cI after the freezes
    }
    if (bndFlag && verbose && comm_rank() == ROOT_ID) {
        std::cout << std::endl << "Optimizer reached box boundary; steepest descent points outside the box at "
                  << fi.size() << " coordinate(s); recursing on the remaining ones." << std::endl;
    }
    const int nr = Ndim - Nconst;
    tf.stop();
    if (bndFlag && nr > 0) {
        PhaseClock tg(det_slot(kDetGather));
        // The reduced problem runs on these same vectors: the frozen entries are set aside and
        // the others slide down in place (the reference gathers them into fresh vectors at every
        // level), so one set of n-vectors serves the whole recursion -- about 11k levels at
        // n = 16384 -- instead of five new ones per level.
        const int nf = (int)fk.size(), nk = ncur - nf;
        std::vector<double> held((size_t)nf * 5);
        for (int f = 0; f < nf; ++f) {
            const int k = fk[f];
            double* h = &held[(size_t)f * 5];
            h[0] = X[k]; h[1] = dFdX[k]; h[2] = Xlb[k]; h[3] = Xub[k]; h[4] = dX[k];
        }
        const bool idx = freeIdxLive;
        for (vector<double>* v : {&X, &dFdX, &Xlb, &Xub, &dX}) {
            drop_positions(*v, fk, ncur);
            v->resize(nr);
            // the fallback walk (freeIdxLive off, e.g. below a level that froze every coordinate)
            // can leave nr != nk: entries past the nk kept ones read 0.0, as the reference's
            // fresh XR(nr) would hold them (never stale values from the compaction)
            if (nr > nk) std::fill(v->begin() + nk, v->end(), 0.0);
        }
        if (idx) {
            drop_positions(freeIdx, fk, ncur);
            freeIdx.resize(nr);
        }
        const double FR = F;
        double Fr = F;
        // the outer D is discarded while the reduced problem runs (reset below), so the
        // reduced D takes over its device buffer: one n x n matrix for the whole recursion
        DenseInverseHessian DR(D, nr, updateMode);
        if (!initialScalingVec.empty()) {
            std::vector<double> scaleR;
            if (idx) {
                scaleR.resize(nr);
                for (int k = 0; k < nr; ++k) scaleR[k] = initialScalingVec[freeIdx[k]];
            } else {
                for (int i = 0; i < Ndim; ++i) if (!cI[i]) scaleR.push_back(initialScalingVec[i]);
            }
            DR.setIdentity(&scaleR);
        } else {
            DR.setIdentity();
        }
        recurFlag = true;
        // the caller's direction (and the next one its update prepared) are recomputed after
        // the recursion: release them while it runs
        std::vector<double>().swap(p);
        if (pnextHeld) std::vector<double>().swap(*pnextHeld);
        pnextHeld = nullptr;
        tg.stop();
        ++depth;
        if (profile && depth > profile[kProfDepth]) profile[kProfDepth] = depth;
        mainBFGSLoop(Fr, X, dFdX, DR, Xlb, Xub, dX, cX, cI, optimFlag, recurFlag);
        --depth;
        assessRecursed = true;   // after the reduced loop, which clears it for its own levels
        PhaseClock tc(det_slot(kDetCopyBack));
        F = nk > 0 ? Fr : FR;
        for (vector<double>* v : {&X, &dFdX, &Xlb, &Xub, &dX}) {
            v->resize(ncur);
            reopen_positions(*v, fk, ncur);
        }
        for (int f = 0; f < nf; ++f) {
            const int k = fk[f];
            const double* h = &held[(size_t)f * 5];
            X[k] = h[0]; dFdX[k] = h[1]; Xlb[k] = h[2]; Xub[k] = h[3]; dX[k] = h[4];
        }
        if (idx && freeIdxLive) {   // (a level below may have dropped the index map)
            freeIdx.resize(ncur);
            reopen_positions(freeIdx, fk, ncur);
            for (int f = 0; f < nf; ++f) freeIdx[fk[f]] = fi[f];
        }
        for (int i : fi) cI[i] = false;
        if (!initialScalingVec.empty()) {
            std::vector<double> scale;
            if (freeIdxLive) {
                scale.resize(ncur);
                for (int k = 0; k < ncur; ++k) scale[k] = initialScalingVec[freeIdx[k]];
            } else {
                for (int i = 0; i < Ndim; ++i) if (!cI[i]) scale.push_back(initialScalingVec[i]);
                scale.resize(ncur, 1.0);
            }
            D.setIdentity(&scale);
        } else {
            D.setIdentity();
        }
        tc.stop();
        {
            PhaseClock t(prof_slot(profile, kProfGrad));
            objPtr->gradientApproximationRecur(X, dX, dFdX, cX, cI);
            if (profile) profile[kProfGradCalls] += 1;
        }
        PhaseClock tc2(det_slot(kDetCopyBack));
        bool cont = false;
        for (int k : fk) {
            if ((std::fabs(X[k] - Xlb[k]) < bndTol) && (dFdX[k] < 0)) cont = true;
            else if ((std::fabs(X[k] - Xub[k]) < bndTol) && (dFdX[k] > 0)) cont = true;
        }
        if (freeIdxLive) {
            Nconst = Ndim - ncur;
        } else {
            Nconst = 0;
            for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
        }
        if (Nconst == 0) recurFlag = false;
        optimFlag = cont;
        if (verbose > 0 && comm_rank() == ROOT_ID)
            std::cout << (cont ? "     Optimization continuing after recursive boundary optimization."
                               : "     Optimization exiting after recursive boundary optimization.")
                      << std::endl;
    } else if (nr == 0) {
        // the coordinates frozen here stay frozen (as in the reference): cI no longer matches
        // the levels above, so they fall back to the full walk
        freeIdxLive = false;
        optimFlag = false;
        if (verbose > 0 && comm_rank() == ROOT_ID) std::cout << "      NO VARIABLES LEFT TO OPTIMIZE!!!! " << std::endl;
    }
}

void BFGS_Bnd::mainBFGSLoop(double& F, vector<double>& X, vector<double>& dFdX, DenseInverseHessian& D,
                            vector<double>& Xlb, vector<double>& Xub, vector<double>& dX, vector<double>& cX,
                            vector<bool>& cI, bool& optimFlag, int& recurFlag) {
    // BFGS_bnd_linesearch.cpp:116-201
    const int n = (int)X.size();
    std::vector<double> p(n), pnext, Xprev(n);
    bool have_next = false;
    int iter = 0;
    double xdiff = xMinDiff * 2, gnorm = 2 * minGrad2Norm;
    while (optimFlag && iter < maxIter && xdiff > xMinDiff && gnorm > minGrad2Norm && totalIter < maxIter) {
        if (verbose > 0 && comm_rank() == ROOT_ID)
            std::cout << std::endl << "Iter = " << iter << " of bounded BFGS search starting with previous F = " << F
                      << "." << std::endl;
        // p = -D g (:142-143); after an iteration without recursion it came out of the update's
        // pass (the same bits: D and g are what the update left)
        if (have_next) {
            p.swap(pnext);
        } else {
            PhaseClock t(prof_slot(profile, kProfUpdate));
            D.direction(dFdX, p);
        }
        double alpha = 0, Fopt = 0;
        {
            PhaseClock t(prof_slot(profile, kProfLineSearch));
            cubicInterpolationLineSearchBnd(X, Xlb, Xub, F, dFdX, p, cX, cI, alpha, Fopt);
        }
        PhaseClock tl(det_slot(kDetIterLoops));
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        F = Fopt;
        {
            // per-iteration scratch (not live across the recursion below, so one set per thread)
            thread_local std::vector<double> gprev, s, y;
            gprev.assign(dFdX.begin(), dFdX.end());
            s.resize(n);
            y.resize(n);
            tl.stop();
            {
                PhaseClock t(prof_slot(profile, kProfGrad));
                objPtr->gradientApproximationRecur(X, dX, dFdX, cX, cI);
                if (profile) profile[kProfGradCalls] += 1;
            }
            for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = dFdX[i] - gprev[i]; }
            PhaseClock t(prof_slot(profile, kProfUpdate));
            D.update(y, s, &dFdX, &pnext);
        }
        assessRecursed = false;
        pnextHeld = &pnext;
        boundaryAssessment(F, X, p, dFdX, D, Xlb, Xub, dX, cX, cI, optimFlag, recurFlag);
        pnextHeld = nullptr;
        // a recursion reset D to I and recomputed the gradient: the fused direction is stale
        have_next = !assessRecursed;
        if (!have_next) std::vector<double>().swap(pnext);
        // the step's sum |X - Xprev| and the gradient's sum of squares: two independent
        // sequential chains (each in the reference's order), one loop
        PhaseClock tl2(det_slot(kDetIterLoops));
        xdiff = 0;
        double gg = 0.0;
        for (int i = 0; i < n; ++i) {
            xdiff += std::fabs(X[i] - Xprev[i]);
            gg = gg + dFdX[i] * dFdX[i];
        }
        gnorm = std::sqrt(gg);
        if (fTrace) fTrace->push_back(F);
        if (verbose > 1 && comm_rank() == ROOT_ID) {
            std::cout << "  Step completed with F = " << F << " and mean abs xdiff is " << xdiff
                      << " and the grad2norm = " << gnorm << std::endl << "  X = ";
            print_vec(X);
        }
        iter = iter + 1;
        totalIter = totalIter + 1;
    }
}

void BFGS_Bnd::findMinBnd(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0, double& fOpt) {
    // the active-set recursion goes one level deeper per frozen coordinate (about 11k levels
    // at n = 16384, SURVEY 8(d) cfg 5): run it on a thread with a stack sized for that
    PhaseClock total(prof_slot(profile, kProfTotal));
    depth = 0;
    run_deep([&] {
        for (double& v : g_det) v = 0.0;
        for (int k = 0; k < kRdCount; ++k)
            if (double* s = recur_detail(k)) *s = 0.0;
        findMinBndBody(X, Xlb, Xub, f0, fOpt);
        if (det_slot(0)) {
            std::fprintf(stderr, "[pnol_amd] BFGS_Bnd host detail (s): freeze %.3f gather+alloc %.3f copyback %.3f iter-loops %.3f\n",
                         g_det[kDetFreeze], g_det[kDetGather], g_det[kDetCopyBack], g_det[kDetIterLoops]);
            std::fprintf(stderr, "[pnol_amd] Recur FD gradient detail (s): build %.3f check %.3f device %.3f redo %.3f gather %.3f\n",
                         *recur_detail(kRdBuild), *recur_detail(kRdCheck), *recur_detail(kRdDevice),
                         *recur_detail(kRdRedo), *recur_detail(kRdGather));
        }
    });
    if (profile) profile[kProfIters] = totalIter;
}

void BFGS_Bnd::findMinBndBody(vector<double>& X, vector<double>& Xlb, vector<double>& Xub, double& f0,
                              double& fOpt) {
    // BFGS_bnd_linesearch.cpp:15-113
    totalIter = 0;
    if (verbose >= 0 && comm_rank() == ROOT_ID) {
        std::cout << std::endl << "  Starting bounded BFGS with line search. " << std::endl << "  X0 = ";
        print_vec(X);
    }
    const int n = (int)X.size();
    checkBoxBounds(X, Xlb, Xub);
    std::vector<double> cX(n, 0.0), X0 = X;
    std::vector<bool> cI(n, false);
    std::vector<double> dX(n, dXGrad);
    if (!dXGradVec.empty())
        for (int i = 0; i < n; ++i) dX[i] = dXGradVec[i];
    std::vector<double> dFdX(n, 0.0);
    pnol_ctx* ctx = require_ctx();
    DenseInverseHessian D(ctx, n, updateMode);
    if (initHessFD) {
        init_from_fd_hessian(objPtr, X, dXHess, D);
    } else if (!initialScalingVec.empty()) {
        D.setIdentity(&initialScalingVec);
    } else {
        D.setIdentity();
    }
    {
        PhaseClock t(prof_slot(profile, kProfGrad));
        objPtr->gradientApproximationRecur(X, dX, dFdX, cX, cI);
        if (profile) profile[kProfGradCalls] += 1;
    }
    double F = objPtr->objEvalRecur(X, cX, cI);
    f0 = F;
    bool optimFlag = true;
    int recurFlag = 0;
    freeIdx.resize(n);
    for (int i = 0; i < n; ++i) freeIdx[i] = i;
    freeIdxLive = true;
    try {
        mainBFGSLoop(F, X, dFdX, D, Xlb, Xub, dX, cX, cI, optimFlag, recurFlag);
    } catch (...) {
        freeIdxLive = false;
        throw;
    }
    freeIdxLive = false;
    std::vector<int>().swap(freeIdx);
    fOpt = F;
    if (verbose >= 0 && comm_rank() == ROOT_ID) {
        std::cout << std::endl << "  Completed bounded BFGS." << std::endl << "  X0 = ";
        print_vec(X0);
        std::cout << "  Xopt = ";
        print_vec(X);
        std::cout << "  f0 = " << f0 << ", fOpt = " << fOpt << std::endl << std::endl;
    }
}
