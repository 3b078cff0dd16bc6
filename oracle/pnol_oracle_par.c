/*
 * pnol_oracle_par.c -- the oracle's LevMarq::findMin (orc_lm_findmin, LevenbergMarquardt.cpp:
 * 11-167) with its independent work spread over host threads.  TEST INFRASTRUCTURE ONLY: it
 * exists to produce the full-size (cfg 3: m = 16384, n = 2048) golden trips that
 * tests/golden/make_cfg3_lm_trips.py writes, in minutes instead of hours.
 *
 * Every value is formed by exactly the oracle's operations in the oracle's order, so the
 * results are bitwise orc_lm_findmin's (tests/test_oracle_golden.py checks that at small
 * sizes):
 *   - FD Jacobian (orc_fd_jacobian, PNOL_Objective.cpp:165-197): column j is
 *     orc_obj_eval_multi(X + dX_j e_j), then (FdX - F) / dX_j -- columns are independent;
 *   - JTJ = JT J (orc_util_matmul, i-j-l order): entry (i, j) is s = 0.0, then
 *     s = s + J[l][i] * J[l][j] for l ascending.  Here every entry of a (64 x 256) tile
 *     accumulates its own s over the same l sequence (the loop over l outermost inside the
 *     tile): the same products, rounded, added in the same order to the same partial sums;
 *   - rhs = -(JT F) (orc_util_matvec): row i's sum over l ascending, then negated;
 *   - luSolve: orc_util_lusolve as is (sequential);
 *   - F norms, the accept / reject test and the lambda update: orc_lm_findmin's statements.
 * Compiled with -ffp-contract=off like the oracle, so no multiply-add is fused.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "pnol_oracle.h"

/* the FD Jacobian, columns over the threads; each thread evaluates with its own copy of the
 * objective (the shared one's eval counter would race) */
static void fd_jacobian_par(orc_objective* o, const double* X, const double* dX, const double* F, double* J,
                            int n, int m, long* evals) {
    long ev = 0;
#pragma omp parallel reduction(+ : ev)
    {
        orc_objective oc = *o;
        oc.evals = 0;
        double* FdX = (double*)malloc(sizeof(double) * (size_t)m);
        double* XdX = (double*)malloc(sizeof(double) * (size_t)n);
#pragma omp for schedule(dynamic, 1)
        for (int j = 0; j < n; ++j) {
            memcpy(XdX, X, sizeof(double) * (size_t)n);
            XdX[j] = XdX[j] + dX[j];
            orc_obj_eval_multi(&oc, XdX, FdX);
            for (int i = 0; i < m; ++i) J[(size_t)i * n + j] = (FdX[i] - F[i]) / dX[j];
        }
        ev += oc.evals;
        free(FdX);
        free(XdX);
    }
    *evals += ev;
}

/* JTJ (n x n) = J^T J with orc_util_matmul's per-entry sums (see the header comment) */
static void jtj_par(const double* J, double* JTJ, int m, int n) {
    enum { TI = 64, TJ = 256 };
    const int ti = (n + TI - 1) / TI, tj = (n + TJ - 1) / TJ;
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
    for (int bi = 0; bi < ti; ++bi)
        for (int bj = 0; bj < tj; ++bj) {
            const int i0 = bi * TI, i1 = i0 + TI < n ? i0 + TI : n;
            const int j0 = bj * TJ, j1 = j0 + TJ < n ? j0 + TJ : n;
            const int w = j1 - j0;
            double* s = (double*)malloc(sizeof(double) * TI * TJ);
            for (int k = 0; k < TI * TJ; ++k) s[k] = 0.0;
            for (int l = 0; l < m; ++l) {
                const double* row = J + (size_t)l * n;
                for (int i = i0; i < i1; ++i) {
                    const double a = row[i];
                    double* si = s + (size_t)(i - i0) * TJ;
                    for (int q = 0; q < w; ++q) si[q] = si[q] + a * row[j0 + q];
                }
            }
            for (int i = i0; i < i1; ++i)
                for (int q = 0; q < w; ++q) JTJ[(size_t)i * n + j0 + q] = s[(size_t)(i - i0) * TJ + q];
            free(s);
        }
}

/* rhs_i = -(sum_l J[l][i] F[l]), orc_util_matvec on JT then the negation of orc_lm_step */
static void jtr_par(const double* J, const double* F, double* rhs, int m, int n) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int l = 0; l < m; ++l) s = s + J[(size_t)l * n + i] * F[l];
        rhs[i] = -s;
    }
}

/* orc_lm_findmin with the parallel pieces above; trace_x (trace_cap x n), trace_chi and
 * trace_lambda (trace_cap) receive X, chiSq and lambda after every loop trip. */
int orc_lm_findmin_par(orc_objective* o, const orc_lm_params* prm, double* X, int n, double* F0, double* FOpt, int m,
                       orc_result* res, double* trace_x, double* trace_chi, double* trace_lambda, int trace_cap) {
    int maxIter = (int)prm->maxIter;
    double lambda = prm->lambda0;
    double* J = (double*)malloc(sizeof(double) * (size_t)m * n);
    double* JTJ = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* A = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* rhs = (double*)malloc(sizeof(double) * (size_t)n);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* F = (double*)malloc(sizeof(double) * (size_t)m);
    double* Fb = (double*)malloc(sizeof(double) * (size_t)m);
    double* Fprev = (double*)malloc(sizeof(double) * (size_t)m);
    double* sigma = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xprev = (double*)malloc(sizeof(double) * (size_t)n);
    if (!J || !JTJ || !A || !rhs || !dX || !F || !Fb || !Fprev || !sigma || !Xprev) return -1;
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    long ev = 0;
    const long ev0 = o->evals;
    orc_obj_eval_multi(o, X, F0);
    memcpy(F, F0, sizeof(double) * (size_t)m);
    memcpy(Fprev, F, sizeof(double) * (size_t)m);
    memcpy(Xprev, X, sizeof(double) * (size_t)n);
    double nrm = orc_util_norm2(F, m);
    double chiSq = nrm * nrm;
    res->f0 = chiSq;
    int iter = 0;
    while (iter < maxIter) {
        /* orc_fd_jacobian: F(X) first, then the n columns */
        orc_obj_eval_multi(o, X, Fb);
        fd_jacobian_par(o, X, dX, Fb, J, n, m, &ev);
        /* orc_lm_step */
        jtj_par(J, JTJ, m, n);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                A[(size_t)i * n + j] = JTJ[(size_t)i * n + j];
                if (i == j) A[(size_t)i * n + j] = (1 + lambda) * JTJ[(size_t)i * n + j];
            }
        jtr_par(J, F, rhs, m, n);
        orc_util_lusolve(A, rhs, sigma, n);
        memcpy(Xprev, X, sizeof(double) * (size_t)n);
        memcpy(Fprev, F, sizeof(double) * (size_t)m);
        for (int i = 0; i < n; ++i) X[i] = X[i] + sigma[i];
        orc_obj_eval_multi(o, X, F);
        double chiSqPrev = chiSq;
        nrm = orc_util_norm2(F, m);
        chiSq = nrm * nrm;
        int stop = 0;
        if (chiSq >= chiSqPrev || chiSq != chiSq) {
            chiSq = chiSqPrev;
            memcpy(X, Xprev, sizeof(double) * (size_t)n);
            memcpy(F, Fprev, sizeof(double) * (size_t)m);
            lambda = lambda * prm->lambdaFactor;
        } else {
            lambda = lambda / prm->lambdaFactor;
            if (orc_util_norm2(sigma, n) < prm->xMinDiff) stop = 1;
        }
        if (iter < trace_cap) {
            if (trace_x) memcpy(trace_x + (size_t)iter * n, X, sizeof(double) * (size_t)n);
            if (trace_chi) trace_chi[iter] = chiSq;
            if (trace_lambda) trace_lambda[iter] = lambda;
        }
        if (stop) break;
        iter++;
    }
    memcpy(FOpt, F, sizeof(double) * (size_t)m);
    o->evals += ev;
    res->fopt = chiSq;
    res->iters = iter;
    res->evals = o->evals - ev0;
    free(J); free(JTJ); free(A); free(rhs); free(dX); free(F); free(Fb); free(Fprev); free(sigma); free(Xprev);
    return 0;
}
