/* asan_check.c -- drives every restated algorithm of the oracle under AddressSanitizer +
 * UndefinedBehaviorSanitizer (the reference has no sanitizer runs; it reads one past a
 * 1-entry pool in findPoolBounds, BFGS_with_linesearch_MPI.cpp:516 -- the restatement clamps that
 * index, and this run is what shows the clamp holds).  TEST INFRASTRUCTURE ONLY
 * (oracle/Makefile `asan`; tests/test_oracle_golden.py runs it).  Exit 0 = clean. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pnol_oracle.h"

static orc_objective obj(int kind, int n, int m, const double* p0, const double* p1, double power) {
    orc_objective o = {kind, n, m, p0, p1, power, 0};
    return o;
}

int main(void) {
    orc_result r;
    /* BFGS on Rosenbrock (Examples.cpp testBFGS params) and with initHessFD */
    for (int fd = 0; fd < 2; ++fd) {
        orc_bfgs_params P = {1e-4, 0.9, 1e-6, 1, 1000, 1e-7, 1e-3, 100, 1e-5, 1e-5, fd, 0};
        double X[5] = {3, 3, 3, 3, 3};
        orc_objective o = obj(ORC_ROSENBROCK, 5, 0, NULL, NULL, 2);
        orc_bfgs_findmin(&o, &P, X, 5, &r, NULL, 0);
    }
    /* BFGS_MPI pools 1..8 (pool 1: the findPoolBounds end-of-pool index) */
    for (int np = 1; np <= 8; ++np) {
        orc_bfgs_mpi_params P = {1e-4, 0.1, 4, 1, 1000, 1e-7, 1e-3, 50, 1e-5, 1e-5, 0, 0};
        double X[10];
        for (int i = 0; i < 10; ++i) X[i] = 10.0;
        orc_objective o = obj(ORC_ROSENBROCK, 10, 0, NULL, NULL, 2);
        orc_bfgs_mpi_findmin(&o, &P, np, X, 10, &r);
    }
    /* LM: ExpCurve, Cubic, a dense linear residual */
    {
        double xd[100], yd[100];
        orc_make_expcurve_data(100, xd, yd);
        orc_objective o = obj(ORC_EXPCURVE, 3, 100, xd, yd, 2);
        orc_lm_params P = {0.001, 10, 1e-7, 100, 1e-7, -1};
        double X[3] = {0.1, 0.1, 0.1}, F0[100], FO[100];
        orc_lm_findmin(&o, &P, X, 3, F0, FO, 100, &r, NULL, 0);
        orc_make_cubic_data(100, xd, yd);
        orc_objective c = obj(ORC_CUBIC, 4, 100, xd, yd, 2);
        double Xc[4] = {0.1, 0.1, 0.1, 0.1};
        orc_lm_findmin(&c, &P, Xc, 4, F0, FO, 100, &r, NULL, 0);
    }
    {
        const int m = 300, n = 70;
        double* A = malloc(sizeof(double) * m * n);
        double *xs = malloc(sizeof(double) * n), *y = malloc(sizeof(double) * m);
        double *X = calloc(n, sizeof(double)), *F0 = malloc(sizeof(double) * m), *FO = malloc(sizeof(double) * m);
        orc_make_linres(0x5EED2018ULL, m, n, A, xs, y);
        orc_objective o = obj(ORC_LINRES, n, m, A, y, 2);
        orc_lm_params P = {0.001, 10, 1e-7, 8, 0.0, -1};
        orc_lm_findmin(&o, &P, X, n, F0, FO, m, &r, NULL, 0);
        double* J = malloc(sizeof(double) * m * n);
        double* h = malloc(sizeof(double) * n);
        for (int i = 0; i < n; ++i) h[i] = 1e-7;
        for (int np = 1; np <= 5; ++np) orc_fd_jacobian_sharded(&o, X, h, J, n, m, np);
        free(A); free(xs); free(y); free(X); free(F0); free(FO); free(J); free(h);
    }
    /* bounded: BFGS_Bnd (with the rank-2 form, trace and depth), BFGSBnd_MPI, BFGS_Bnd_MPI_SW */
    {
        orc_bfgs_bnd_params P = {1e-4, 0.8, 1e-6, 1, 1e-10, 2, 50, 1e-5, 1e-6, 1e-3, 200, 1e-5, 1e-5, 0, -1};
        const int n = 64;
        double d[64], b[64], X[64], lb[64], ub[64], tr[4096];
        orc_make_quadratic(0x5EED2018ULL, n, d, b);
        for (int i = 0; i < n; ++i) { b[i] *= 4; X[i] = 0; lb[i] = -0.5; ub[i] = 0.5; }
        orc_objective q = obj(ORC_QUADRATIC, n, 0, d, b, 2);
        int depth = 0;
        orc_bfgs_bnd_findmin_ex(&q, &P, X, lb, ub, n, &r, 1, tr, 4096, &depth);
        for (int i = 0; i < n; ++i) X[i] = 0;
        orc_bfgs_bnd_findmin(&q, &P, X, lb, ub, n, &r);
        double Xr[3] = {-1, 2, 2}, lr[3] = {-1, -1, -1}, ur[3] = {5, 5, 5};
        orc_objective ro = obj(ORC_ROSENBROCK, 3, 0, NULL, NULL, 2);
        for (int np = 1; np <= 8; ++np) {
            double Xs[3] = {-1, 2, 2};
            orc_bfgs_bnd_mpi_sw_findmin(&ro, &P, np, Xs, lr, ur, 3, &r);
        }
        orc_bfgs_bnd_mpi_params Q = {1e-4, 0.1, 1e-16, 4, 1, 1000, 1e-7, 1e-3, 200, 1e-5, 1e-5, 1e-5, 0, 0};
        for (int np = 2; np <= 8; ++np) {
            double Xs[3] = {-1, 2, 2};
            orc_bfgs_bnd_mpi_findmin(&ro, &Q, np, np, Xs, lr, ur, 3, &r);
        }
        (void)Xr;
    }
    /* utility layer: inverse, FD Hessian */
    {
        const int n = 9;
        double B[81], Bi[81], X[9], h[9];
        for (int i = 0; i < n * n; ++i) B[i] = (i % 7) * 0.1 + (i % (n + 1) == 0 ? 3.0 : 0.0);
        orc_util_matinv(B, Bi, n);
        for (int i = 0; i < n; ++i) { X[i] = 0.3 * i; h[i] = 1e-3; }
        orc_objective o = obj(ORC_ROSENBROCK, n, 0, NULL, NULL, 2);
        orc_fd_hessian(&o, X, h, B, n);
    }
    /* genetic algorithm (row f4), serial and at 1..4 ranks */
    {
        const int n = 4;
        double lb[4] = {-2, -2, -2, -2}, ub[4] = {2, 2, 2, 2};
        const double prm[9] = {30, 40, 0.1, 0.3, 0.2, 0.5, 0.01, 0.5, 10};
        orc_objective o = obj(ORC_ROSENBROCK, n, 0, NULL, NULL, 2);
        orc_result r;
        for (int np = 0; np <= 4; ++np) {
            double X[4] = {-1, -1, -1, -1};
            orc_ga_findmin(&o, prm, 12345ull + np, np, X, lb, ub, n, &r);
        }
    }
    printf("asan_check: clean\n");
    return 0;
}
