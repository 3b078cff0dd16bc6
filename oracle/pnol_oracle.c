/*
 * pnol_oracle.c -- CPU restatement of the PNOL BFGS / Levenberg-Marquardt hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see pnol_oracle.h).  Fresh C, written from the behaviour of
 * the reference (MPL-2.0, not copied); each function cites the reference lines it follows.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off), output oracle/_build/liboracle.so.
 */
#include "pnol_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* objectives                                                                             */
/* ------------------------------------------------------------------------------------ */

/* RosenbrockObject::objEval, ExampleObjectives.hpp:87-103 */
static double obj_rosenbrock(const double* X, int n) {
    double value = 0.0;
    for (int k = 0; k + 1 < n; ++k) {
        double xk2 = X[k] * X[k];
        double t = X[k + 1] - xk2;
        double u = 1.0 - X[k];
        value = value + (100.0 * (t * t) + u * u);
    }
    return value;
}

/* PowerObject::objEval, ExampleObjectives.hpp:214-224 (pow with the integer power) */
static double obj_power(const double* X, int n, double power) {
    double value = 0.0;
    for (int k = 0; k < n; ++k) value = value + (power == 2.0 ? X[k] * X[k] : pow(X[k], power));
    return value;
}

/* GoldsteinFunction::objEval, ExampleObjectives.hpp:27-39 */
static double obj_goldstein(const double* X) {
    double x = X[0], y = X[1];
    double a = x + y + 1, b = 2 * x - 3 * y;
    return (1 + (a * a) * (19 - 14 * x + 3 * (x * x) - 14 * y + 6 * x * y + 3 * (y * y))) *
           (30 + (b * b) * (18 - 32 * x + 12 * (x * x) + 48 * y - 36 * x * y + 27 * (y * y)));
}

/* BoothFunction::objEval, ExampleObjectives.hpp:58-69 */
static double obj_booth(const double* X) {
    double a = X[0] + 2 * X[1] - 7, b = 2 * X[0] + X[1] - 5;
    return a * a + b * b;
}

/* Synthetic convex quadratic of SURVEY 8(d) cfg 2/5.  Summation order is part of the
 * objective's definition (the device batch evaluates the identical chain):
 *   f = sum_i ( (0.5*d_i*x_i)*x_i - b_i*x_i + [i+1<n] (0.25*x_i)*x_{i+1} ), i ascending. */
static double obj_quadratic(const double* X, int n, const double* d, const double* b) {
    double f = 0.0;
    for (int i = 0; i < n; ++i) {
        double t = (0.5 * d[i] * X[i]) * X[i] - b[i] * X[i];
        if (i + 1 < n) t = t + (0.25 * X[i]) * X[i + 1];
        f = f + t;
    }
    return f;
}

double orc_obj_eval(orc_objective* o, const double* x) {
    o->evals++;
    switch (o->kind) {
        case ORC_ROSENBROCK: return obj_rosenbrock(x, o->n);
        case ORC_POWER: return obj_power(x, o->n, o->power);
        case ORC_GOLDSTEIN: return obj_goldstein(x);
        case ORC_BOOTH: return obj_booth(x);
        case ORC_QUADRATIC: return obj_quadratic(x, o->n, o->p0, o->p1);
        default: return NAN;
    }
}

void orc_obj_eval_multi(orc_objective* o, const double* X, double* F) {
    o->evals++;
    const double* xd = o->p0;
    const double* yd = o->p1;
    switch (o->kind) {
        case ORC_EXPCURVE: /* ExpCurveObjective::objEval, ExampleObjectives.hpp:123-132 */
            for (int k = 0; k < o->m; ++k) {
                double func = X[0] * exp(X[1] * xd[k]) + X[2];
                F[k] = yd[k] - func;
            }
            break;
        case ORC_CUBIC: /* CubicObjective::objEval, ExampleObjectives.hpp:170-179 */
            for (int k = 0; k < o->m; ++k) {
                double x = xd[k];
                double func = X[0] * pow(x, 3.0) + X[1] * (x * x) + X[2] * x + X[3];
                F[k] = yd[k] - func;
            }
            break;
        case ORC_LINRES: /* r = A x - y, fma chain over k ascending (the objective's definition) */
            for (int i = 0; i < o->m; ++i) {
                const double* a = o->p0 + (size_t)i * o->n;
                double acc = 0.0;
                for (int k = 0; k < o->n; ++k) acc = fma(a[k], X[k], acc);
                F[i] = acc - o->p1[i];
            }
            break;
        default:
            for (int k = 0; k < o->m; ++k) F[k] = NAN;
    }
}

/* ------------------------------------------------------------------------------------ */
/* utility layer (UtilityFunctionLibrary restatement)                        */
/* ------------------------------------------------------------------------------------ */

double orc_util_dot(const double* a, const double* b, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s = s + a[i] * b[i];
    return s;
}

double orc_util_norm2(const double* a, int n) { return sqrt(orc_util_dot(a, a, n)); }

void orc_util_matvec(const double* A, const double* x, double* y, int rows, int cols) {
    for (int i = 0; i < rows; ++i) {
        double s = 0.0;
        const double* a = A + (size_t)i * cols;
        for (int j = 0; j < cols; ++j) s = s + a[j] * x[j];
        y[i] = s;
    }
}

void orc_util_matmul(const double* A, const double* B, double* C, int n, int k, int m) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s = s + A[(size_t)i * k + l] * B[(size_t)l * m + j];
            C[(size_t)i * m + j] = s;
        }
}

/* Gaussian elimination with partial pivoting on a copy; back substitution j ascending. */
int orc_util_lusolve(const double* Ain, const double* bin, double* x, int n) {
    double* A = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* b = (double*)malloc(sizeof(double) * (size_t)n);
    if (!A || !b) { free(A); free(b); return -1; }
    memcpy(A, Ain, sizeof(double) * (size_t)n * n);
    memcpy(b, bin, sizeof(double) * (size_t)n);
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double best = fabs(A[(size_t)k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = fabs(A[(size_t)i * n + k]);
            if (v > best) { best = v; piv = i; }
        }
        if (piv != k) {
            for (int j = 0; j < n; ++j) {
                double t = A[(size_t)k * n + j];
                A[(size_t)k * n + j] = A[(size_t)piv * n + j];
                A[(size_t)piv * n + j] = t;
            }
            double t = b[k]; b[k] = b[piv]; b[piv] = t;
        }
        double akk = A[(size_t)k * n + k];
        for (int i = k + 1; i < n; ++i) {
            double f = A[(size_t)i * n + k] / akk;
            for (int j = k; j < n; ++j) A[(size_t)i * n + j] = A[(size_t)i * n + j] - f * A[(size_t)k * n + j];
            b[i] = b[i] - f * b[k];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int j = i + 1; j < n; ++j) s = s - A[(size_t)i * n + j] * x[j];
        x[i] = s / A[(size_t)i * n + i];
    }
    free(A); free(b);
    return 0;
}

int orc_util_matinv(const double* A, double* Ainv, int n) {
    double* e = (double*)calloc((size_t)n, sizeof(double));
    double* c = (double*)malloc(sizeof(double) * (size_t)n);
    if (!e || !c) { free(e); free(c); return -1; }
    for (int j = 0; j < n; ++j) {
        e[j] = 1.0;
        orc_util_lusolve(A, e, c, n);
        for (int i = 0; i < n; ++i) Ainv[(size_t)i * n + j] = c[i];
        e[j] = 0.0;
    }
    free(e); free(c);
    return 0;
}

void orc_util_linspace(double a, double b, int N, double* v) {
    for (int i = 0; i < N; ++i) v[i] = a + i * (b - a) / (N - 1);
}

static void vector_min(const double* v, int n, double* val, int* idx) {
    *val = v[0]; *idx = 0;
    for (int i = 1; i < n; ++i) if (v[i] < *val) { *val = v[i]; *idx = i; }
}

static void vector_max(const double* v, int n, double* val, int* idx) {
    *val = v[0]; *idx = 0;
    for (int i = 1; i < n; ++i) if (v[i] > *val) { *val = v[i]; *idx = i; }
}

static double sign_of(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0); }

/* ------------------------------------------------------------------------------------ */
/* FD engine, PNOL_Objective.cpp                                                         */
/* ------------------------------------------------------------------------------------ */

/* Objective::gradientApproximation, PNOL_Objective.cpp:12-34 */
void orc_fd_gradient(orc_objective* o, const double* X, const double* dX, double* dFdX, int n) {
    double* XdX = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double F = orc_obj_eval(o, X);
    for (int i = 0; i < n; ++i) {
        memcpy(XdX, X, sizeof(double) * (size_t)n);
        XdX[i] = XdX[i] + dX[i];
        double FdX = orc_obj_eval(o, XdX);
        dFdX[i] = (FdX - F) / dX[i];
    }
    free(XdX);
}

/* Objective::gradientApproximationMPI, PNOL_Objective.cpp:88-159: owner(k) = k mod P,
 * zero-padded Allreduce(SUM).  Adding zeros is exact, so each owner's value survives
 * bit for bit; the restatement evaluates owner by owner to keep the evaluation order. */
void orc_fd_gradient_sharded(orc_objective* o, const double* X, const double* dX, double* dFdX,
                             int n, int nprocs) {
    double* FdX = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double* XdX = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    double F = 0.0;
    for (int rank = 0; rank < nprocs; ++rank)
        for (int k = rank; k <= n; k += nprocs) {
            if (k < n) {
                memcpy(XdX, X, sizeof(double) * (size_t)n);
                XdX[k] = XdX[k] + dX[k];
                FdX[k] = 0.0 + orc_obj_eval(o, XdX);
            } else {
                F = 0.0 + orc_obj_eval(o, X);
            }
        }
    for (int i = 0; i < n; ++i) dFdX[i] = (FdX[i] - F) / dX[i];
    free(FdX); free(XdX);
}

/* MultiObjective::gradientApproximation, PNOL_Objective.cpp:165-197 (J m x n row-major) */
void orc_fd_jacobian(orc_objective* o, const double* X, const double* dX, double* J, int n, int m) {
    double* F = (double*)malloc(sizeof(double) * (size_t)m);
    double* FdX = (double*)malloc(sizeof(double) * (size_t)m);
    double* XdX = (double*)malloc(sizeof(double) * (size_t)n);
    orc_obj_eval_multi(o, X, F);
    for (int j = 0; j < n; ++j) {
        memcpy(XdX, X, sizeof(double) * (size_t)n);
        XdX[j] = XdX[j] + dX[j];
        orc_obj_eval_multi(o, XdX, FdX);
        for (int i = 0; i < m; ++i) J[(size_t)i * n + j] = (FdX[i] - F[i]) / dX[j];
    }
    free(F); free(FdX); free(XdX);
}

/* MultiObjective::gradientApproximationMPI, PNOL_Objective.cpp:202-299 */
void orc_fd_jacobian_sharded(orc_objective* o, const double* X, const double* dX, double* J,
                             int n, int m, int nprocs) {
    double* F = (double*)calloc((size_t)m, sizeof(double));
    double* Fl = (double*)malloc(sizeof(double) * (size_t)m);
    double* cols = (double*)calloc((size_t)n * m, sizeof(double));
    double* XdX = (double*)malloc(sizeof(double) * (size_t)n);
    for (int rank = 0; rank < nprocs; ++rank)
        for (int j = rank; j <= n; j += nprocs) {
            if (j < n) {
                memcpy(XdX, X, sizeof(double) * (size_t)n);
                XdX[j] = XdX[j] + dX[j];
                orc_obj_eval_multi(o, XdX, Fl);
                for (int k = 0; k < m; ++k) cols[(size_t)j * m + k] = 0.0 + Fl[k];
            } else {
                orc_obj_eval_multi(o, X, Fl);
                for (int k = 0; k < m; ++k) F[k] = 0.0 + Fl[k];
            }
        }
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) J[(size_t)i * n + j] = (cols[(size_t)j * m + i] - F[i]) / dX[j];
    free(F); free(Fl); free(cols); free(XdX);
}

/* Objective::hessianApproximation, PNOL_Objective.cpp:38-85 */
void orc_fd_hessian(orc_objective* o, const double* X, const double* dX, double* B, int n) {
    double* Xi = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xj = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xij = (double*)malloc(sizeof(double) * (size_t)n);
    double F = orc_obj_eval(o, X);
    for (int i = 0; i < n; ++i)
        for (int j = i; j < n; ++j) {
            memcpy(Xi, X, sizeof(double) * (size_t)n);
            memcpy(Xj, X, sizeof(double) * (size_t)n);
            memcpy(Xij, X, sizeof(double) * (size_t)n);
            Xi[i] = Xi[i] + dX[i];
            Xj[j] = Xj[j] + dX[j];
            Xij[i] = Xij[i] + dX[i];
            Xij[j] = Xij[j] + dX[j];
            double Fi = orc_obj_eval(o, Xi);
            double Fj = orc_obj_eval(o, Xj);
            double Fij = orc_obj_eval(o, Xij);
            B[(size_t)i * n + j] = (Fij - Fi - Fj + F) / (dX[i] * dX[j]);
        }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) B[(size_t)i * n + j] = B[(size_t)j * n + i];
    free(Xi); free(Xj); free(Xij);
}

/* Objective::objEvalRecur, PNOL_Objective.cpp:303-333 */
double orc_obj_eval_recur(orc_objective* o, const double* Xr, const double* constX,
                          const unsigned char* constInd, int nfull) {
    double* X = (double*)malloc(sizeof(double) * (size_t)(nfull > 0 ? nfull : 1));
    int ir = 0;
    for (int i = 0; i < nfull; ++i) X[i] = constInd[i] ? constX[i] : Xr[ir++];
    double F = orc_obj_eval(o, X);
    free(X);
    return F;
}

/* Objective::gradientApproximationRecur, PNOL_Objective.cpp:337-360 */
void orc_fd_gradient_recur(orc_objective* o, const double* X, const double* dX, double* dFdX, int nr,
                           const double* constX, const unsigned char* constInd, int nfull) {
    double* XdX = (double*)malloc(sizeof(double) * (size_t)(nr > 0 ? nr : 1));
    double F = orc_obj_eval_recur(o, X, constX, constInd, nfull);
    for (int i = 0; i < nr; ++i) {
        memcpy(XdX, X, sizeof(double) * (size_t)nr);
        XdX[i] = XdX[i] + dX[i];
        double FdX = orc_obj_eval_recur(o, XdX, constX, constInd, nfull);
        dFdX[i] = (FdX - F) / dX[i];
    }
    free(XdX);
}

/* ------------------------------------------------------------------------------------ */
/* BFGS inverse-Hessian update                                                           */
/* ------------------------------------------------------------------------------------ */

/* updateHessianInv, BFGS_with_linesearch.cpp:389-432: D <- M1 D M2 + M3 by two GEMMs. */
void orc_update_hessian_inv(double* D, const double* g, const double* s, int n) {
    size_t nn = (size_t)n * n;
    double* M1 = (double*)malloc(sizeof(double) * nn);
    double* M2 = (double*)malloc(sizeof(double) * nn);
    double* M3 = (double*)malloc(sizeof(double) * nn);
    double* A = (double*)malloc(sizeof(double) * nn);
    double rho = 1 / orc_util_dot(g, s, n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double e = (i == j) ? 1.0 : 0.0;
            M1[(size_t)i * n + j] = e - rho * s[i] * g[j];
            M2[(size_t)i * n + j] = e - rho * g[i] * s[j];
            M3[(size_t)i * n + j] = rho * s[i] * s[j];
        }
    orc_util_matmul(M1, D, A, n, n, n);
    orc_util_matmul(A, M2, D, n, n, n);
    for (size_t k = 0; k < nn; ++k) D[k] = D[k] + M3[k];
    free(M1); free(M2); free(M3); free(A);
}

/* The same update in its O(n^2) rank-2 form (what the device kernel computes):
 *   u = D y, w = D^T y, beta = y.u, c = rho^2 beta + rho,
 *   D_ij += s_i (c s_j - rho w_j) - rho u_i s_j.                                       */
void orc_update_hessian_inv_rank2(double* D, const double* y, const double* s, int n) {
    double* u = (double*)calloc((size_t)n, sizeof(double));
    double* w = (double*)calloc((size_t)n, sizeof(double));
    double rho = 1 / orc_util_dot(y, s, n);
    for (int i = 0; i < n; ++i) {
        double acc = 0.0;
        for (int j = 0; j < n; ++j) acc = acc + D[(size_t)i * n + j] * y[j];
        u[i] = acc;
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) w[j] = w[j] + D[(size_t)i * n + j] * y[i];
    double beta = orc_util_dot(y, u, n);
    double c = rho * rho * beta + rho;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            D[(size_t)i * n + j] = D[(size_t)i * n + j] + s[i] * (c * s[j] - rho * w[j]) - rho * u[i] * s[j];
    free(u); free(w);
}

/* ------------------------------------------------------------------------------------ */
/* BFGS with cubic-interpolation Wolfe line search, BFGS_with_linesearch.cpp              */
/* ------------------------------------------------------------------------------------ */

typedef struct {
    orc_objective* o;
    const orc_bfgs_params* prm;
    double* work;
    int n;
} bfgs_ctx;

/* BFGS::lineSearchObj, :144-156 */
static double ls_obj(bfgs_ctx* c, double alpha, const double* X, const double* p) {
    for (int i = 0; i < c->n; ++i) c->work[i] = X[i] + alpha * p[i];
    return orc_obj_eval(c->o, c->work);
}

/* BFGS::lineSearchFDDerivative, :160-174 */
static double ls_fd_deriv(bfgs_ctx* c, double alpha, double phialpha, const double* X, const double* p) {
    for (int i = 0; i < c->n; ++i) c->work[i] = X[i] + (alpha + c->prm->dalpha) * p[i];
    double Fa = orc_obj_eval(c->o, c->work);
    return (Fa - phialpha) / c->prm->dalpha;
}

/* cubicInterpMin, :359-385 */
static double cubic_interp_min(double alo, double ahi, double plo, double phi, double dlo, double dhi) {
    double d1 = dlo + dhi - 3 * (plo - phi) / (alo - ahi);
    double d2 = sign_of(ahi - alo) * sqrt(d1 * d1 - dlo * dhi);
    double an = ahi - (ahi - alo) * (dhi + d2 - d1) / (dhi - dlo + 2 * d2);
    if (alo < ahi) {
        if (an < alo) an = (ahi + alo) / 2;
    } else {
        if (an < ahi) an = (ahi + alo) / 2;
    }
    return an;
}

/* BFGS::lineSearchZoom, :296-356 */
static void ls_zoom(bfgs_ctx* c, double alo, double ahi, double plo, double phi, double dlo, double dhi,
                    double phi0, double dphi0, const double* X, const double* p,
                    double* alphaOpt, double* phiOpt) {
    const orc_bfgs_params* P = c->prm;
    for (int it = 0; it < P->maxIterLineSearch; ++it) {
        double aj = cubic_interp_min(alo, ahi, plo, phi, dlo, dhi);
        double pj = ls_obj(c, aj, X, p);
        double dj = ls_fd_deriv(c, aj, pj, X, p);
        if (pj > phi0 + P->c1 * aj * dphi0 || pj >= plo) {
            ahi = aj; phi = pj; dhi = dj;
        } else {
            if (fabs(dj) <= fabs(P->c2 * dphi0)) { *alphaOpt = aj; *phiOpt = pj; return; }
            if (dj * (ahi - alo) >= 0) { ahi = alo; phi = plo; dhi = dlo; }
            alo = aj; plo = pj; dlo = dj;
        }
    }
}

/* BFGS::cubicInterpolationLineSearch, :177-291 */
static void ls_cubic(bfgs_ctx* c, const double* X, double FX, const double* g, const double* p,
                     double* alphaOpt, double* Fopt) {
    const orc_bfgs_params* P = c->prm;
    *alphaOpt = 0; *Fopt = FX;
    double phi0 = FX, dphi0 = orc_util_dot(g, p, c->n);
    double aim1 = 0, pim1 = phi0, dim1 = dphi0;
    double ai = P->alphaGuess;
    for (int it = 0; it < P->maxIterLineSearch; ++it) {
        double pi = ls_obj(c, ai, X, p);
        double di = ls_fd_deriv(c, ai, pi, X, p);
        if ((pi > phi0 + P->c1 * ai * dphi0) || (pi >= pim1 && it > 1)) {
            ls_zoom(c, aim1, ai, pim1, pi, dim1, di, phi0, dphi0, X, p, alphaOpt, Fopt);
            return;
        }
        if (fabs(di) <= fabs(P->c2 * dphi0)) { *alphaOpt = ai; *Fopt = pi; return; }
        if (di >= 0) {
            ls_zoom(c, ai, aim1, pi, pim1, di, dim1, phi0, dphi0, X, p, alphaOpt, Fopt);
            return;
        }
        aim1 = ai; pim1 = pi; dim1 = di;
        ai = 2 * ai;
    }
}

static void set_identity(double* D, int n) {
    memset(D, 0, sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) D[(size_t)i * n + i] = 1.0;
}

/* BFGS::findMin, BFGS_with_linesearch.cpp:12-139 */
int orc_bfgs_findmin(orc_objective* o, const orc_bfgs_params* prm, double* X, int n, orc_result* res,
                     double* trace, int trace_cap) {
    return orc_bfgs_findmin_ex(o, prm, X, n, res, trace, trace_cap, 0);
}

/* rank2 = 1: updateHessianInv in its O(n^2) rank-2 form (orc_update_hessian_inv_rank2), so the
 * large-n configs (cfg 2, n = 4096) run in seconds; everything else as orc_bfgs_findmin */
int orc_bfgs_findmin_ex(orc_objective* o, const orc_bfgs_params* prm, double* X, int n, orc_result* res,
                        double* trace, int trace_cap, int rank2) {
    int maxIter = (int)prm->maxIter; /* int member set from a double (hpp:62,72) */
    double* D = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* g = (double*)malloc(sizeof(double) * (size_t)n);
    double* gprev = (double*)malloc(sizeof(double) * (size_t)n);
    double* p = (double*)malloc(sizeof(double) * (size_t)n);
    double* s = (double*)malloc(sizeof(double) * (size_t)n);
    double* y = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xprev = (double*)malloc(sizeof(double) * (size_t)n);
    double* work = (double*)malloc(sizeof(double) * (size_t)n);
    bfgs_ctx c = {o, prm, work, n};
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    if (prm->initHessFD) {
        double* B = (double*)malloc(sizeof(double) * (size_t)n * n);
        double* dXH = (double*)malloc(sizeof(double) * (size_t)n);
        for (int i = 0; i < n; ++i) dXH[i] = prm->dXHess;
        orc_fd_hessian(o, X, dXH, B, n);
        orc_util_matinv(B, D, n);
        free(B); free(dXH);
    } else {
        set_identity(D, n);
    }
    long ev0 = o->evals;
    orc_fd_gradient(o, X, dX, g, n);
    double F = orc_obj_eval(o, X);
    res->f0 = F;
    int iter = 0;
    double xdiff = prm->xMinDiff * 2, gnorm = 2 * prm->minGrad2Norm;
    while (iter < maxIter && xdiff > prm->xMinDiff && gnorm > prm->minGrad2Norm) {
        memcpy(gprev, g, sizeof(double) * (size_t)n);
        orc_util_matvec(D, g, p, n, n);
        for (int i = 0; i < n; ++i) p[i] = -p[i];
        double alpha, Fopt;
        ls_cubic(&c, X, F, g, p, &alpha, &Fopt);
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        F = Fopt;
        orc_fd_gradient(o, X, dX, g, n);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = g[i] - gprev[i]; }
        if (rank2) orc_update_hessian_inv_rank2(D, y, s, n);
        else orc_update_hessian_inv(D, y, s, n);
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += fabs(X[i] - Xprev[i]);
        gnorm = orc_util_norm2(g, n);
        if (trace && iter < trace_cap) memcpy(trace + (size_t)iter * n, X, sizeof(double) * (size_t)n);
        iter++;
    }
    res->fopt = F; res->iters = iter; res->evals = o->evals - ev0;
    free(D); free(dX); free(g); free(gprev); free(p); free(s); free(y); free(Xprev); free(work);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* BFGS_MPI: pool secant line search, BFGS_with_linesearch_MPI.cpp                       */
/* ------------------------------------------------------------------------------------ */

typedef struct {
    orc_objective* o; const orc_bfgs_mpi_params* prm; double* work; int n; int npool;
} bfgs_mpi_ctx;

/* BFGS_MPI::evalAlphaPoolMPI, :163-223 (rank-ordered evaluation, zero-padded sum) */
static void eval_alpha_pool(bfgs_mpi_ctx* c, const double* alpha, double* phi, int N,
                            const double* X, const double* p) {
    for (int rank = 0; rank < c->npool; ++rank)
        for (int i = rank; i < N; i += c->npool) {
            for (int k = 0; k < c->n; ++k) c->work[k] = X[k] + alpha[i] * p[k];
            phi[i] = 0.0 + orc_obj_eval(c->o, c->work);
        }
}

/* findPoolBounds, :496-530.  The reference reads one past either end of the pool when
 * the minimum sits on the last entry (or a 1-entry pool's first); that read is undefined
 * behaviour, so the restatement clamps the index to the pool (documented in DESIGN.md). */
static void find_pool_bounds(const double* ap, const double* pp, int N, double a0, double p0,
                             double* a1, double* a2, double* p1, double* p2) {
    double pmin; int imin;
    vector_min(pp, N, &pmin, &imin);
    int hi = imin + 1 < N ? imin + 1 : N - 1;
    if (p0 < pmin) {
        *a1 = a0; *a2 = ap[0]; *p1 = p0; *p2 = pp[0];
    } else if (p0 >= pmin && imin == 0) {
        *a1 = a0; *a2 = ap[hi]; *p1 = p0; *p2 = pp[hi];
    } else {
        *a1 = ap[imin - 1]; *a2 = ap[hi]; *p1 = pp[imin - 1]; *p2 = pp[hi];
    }
}

/* BFGS_MPI::secantLineSearch, :226-492 */
static void ls_secant(bfgs_mpi_ctx* c, const double* X, double FX, const double* g, const double* p,
                      double* alphaOpt, double* Fopt) {
    const orc_bfgs_mpi_params* P = c->prm;
    int Np = c->npool;
    double* ap = (double*)calloc((size_t)Np, sizeof(double));
    double* pp = (double*)calloc((size_t)Np, sizeof(double));
    double* apPrev = (double*)malloc(sizeof(double) * (size_t)Np);
    double* ppPrev = (double*)calloc((size_t)Np, sizeof(double));
    double* slope = (double*)calloc((size_t)Np, sizeof(double));
    double* ap2 = (double*)calloc((size_t)Np + 2, sizeof(double));
    double* pp2 = (double*)calloc((size_t)Np + 2, sizeof(double));
    for (int i = 0; i < Np; ++i) apPrev[i] = -1;
    *alphaOpt = 0; *Fopt = FX;
    double a0 = 0, phi0 = FX, dphi0 = orc_util_dot(g, p, c->n);
    int idxMin = -(int)ceil((Np - 1.0) / 2.0);
    int idxMax = (int)floor((Np - 1.0) / 2.0);
    double r = pow(P->maxAlphaMult, 1.0 / (double)idxMax);
    int idx = idxMin;
    for (int k = 0; k < Np; ++k) { ap[k] = P->alphaGuess * pow(r, idx); idx++; }
    int first = 1, zoom = 0;
    for (int it = 0; it < P->maxIterLineSearch && first; ++it) {
        eval_alpha_pool(c, ap, pp, Np, X, p);
        for (int i = 0; i < Np; ++i)
            if (pp[i] > phi0 + P->c1 * ap[i] * dphi0) { zoom = 1; first = 0; }
        slope[0] = (pp[0] - phi0) / (ap[0] - a0);
        for (int i = 1; i < Np; ++i) slope[i] = (pp[i] - pp[i - 1]) / (ap[i] - ap[i - 1]);
        if (first)
            for (int i = 0; i < Np; ++i)
                if (fabs(slope[i]) <= fabs(P->c2 * dphi0)) { zoom = 0; first = 0; }
        if (first)
            for (int i = 0; i < Np; ++i)
                if (slope[i] >= 0) { zoom = 1; first = 0; }
        if (first) {
            double amax; int imax;
            vector_max(ap, Np, &amax, &imax);
            r = pow(P->maxAlphaMult, 1.0 / (double)Np);
            for (int i = 0; i < Np; ++i) {
                apPrev[i] = ap[i]; ppPrev[i] = pp[i];
                double power = i + 1;
                ap[i] = amax * pow(r, power);
            }
        }
    }
    double alo, ahi, plo, phi;
    if (apPrev[0] < 0) {
        find_pool_bounds(ap, pp, Np, a0, phi0, &alo, &ahi, &plo, &phi);
    } else {
        double* ae = (double*)malloc(sizeof(double) * 2 * (size_t)Np);
        double* pe = (double*)malloc(sizeof(double) * 2 * (size_t)Np);
        for (int i = 0; i < Np; ++i) { ae[i] = apPrev[i]; ae[i + Np] = ap[i]; pe[i] = ppPrev[i]; pe[i + Np] = pp[i]; }
        find_pool_bounds(ae, pe, 2 * Np, a0, phi0, &alo, &ahi, &plo, &phi);
        free(ae); free(pe);
    }
    for (int it = 0; it < P->maxIterLineSearch && zoom; ++it) {
        orc_util_linspace(alo, ahi, Np + 2, ap2);
        pp2[0] = plo; pp2[Np + 1] = phi; ap2[0] = alo; ap2[Np + 1] = ahi;
        for (int i = 0; i < Np; ++i) { ap[i] = ap2[i + 1]; pp[i] = pp2[i + 1]; }
        eval_alpha_pool(c, ap, pp, Np, X, p);
        for (int i = 0; i < Np; ++i) { ap2[i + 1] = ap[i]; pp2[i + 1] = pp[i]; }
        for (int i = 0; i < Np; ++i) slope[i] = (pp2[i + 1] - pp2[i]) / (ap2[i + 1] - ap2[i]);
        for (int i = 0; i < Np; ++i)
            if (fabs(slope[i]) <= fabs(P->c2 * dphi0)) zoom = 0;
        if (zoom) find_pool_bounds(ap2, pp2, Np + 2, a0, phi0, &alo, &ahi, &plo, &phi);
    }
    /* A10 defect kept: when the first phase ends on the curvature test the zoom never runs
     * and ap2/pp2 are still zero, so the minimum is (alpha 0, phi 0) (:483-488). */
    double pmin; int imin;
    vector_min(pp2, Np + 2, &pmin, &imin);
    *alphaOpt = ap2[imin];
    *Fopt = pmin;
    free(ap); free(pp); free(apPrev); free(ppPrev); free(slope); free(ap2); free(pp2);
}

/* BFGS_MPI::findMin, BFGS_with_linesearch_MPI.cpp:12-142 */
int orc_bfgs_mpi_findmin(orc_objective* o, const orc_bfgs_mpi_params* prm, int nprocs, double* X, int n,
                         orc_result* res) {
    int maxIter = (int)prm->maxIter;
    double* D = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* g = (double*)malloc(sizeof(double) * (size_t)n);
    double* gprev = (double*)malloc(sizeof(double) * (size_t)n);
    double* p = (double*)malloc(sizeof(double) * (size_t)n);
    double* s = (double*)malloc(sizeof(double) * (size_t)n);
    double* y = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xprev = (double*)malloc(sizeof(double) * (size_t)n);
    double* work = (double*)malloc(sizeof(double) * (size_t)n);
    bfgs_mpi_ctx c = {o, prm, work, n, nprocs};
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    if (prm->initHessFD) {
        double* B = (double*)malloc(sizeof(double) * (size_t)n * n);
        double* dXH = (double*)malloc(sizeof(double) * (size_t)n);
        for (int i = 0; i < n; ++i) dXH[i] = prm->dXHess;
        orc_fd_hessian(o, X, dXH, B, n);
        orc_util_matinv(B, D, n);
        free(B); free(dXH);
    } else {
        set_identity(D, n);
    }
    long ev0 = o->evals;
    orc_fd_gradient_sharded(o, X, dX, g, n, nprocs);
    double F = orc_obj_eval(o, X);
    res->f0 = F;
    int iter = 0;
    double xdiff = prm->xMinDiff * 2, gnorm = 2 * prm->minGrad2Norm;
    while (iter < maxIter && xdiff > prm->xMinDiff && gnorm > prm->minGrad2Norm) {
        memcpy(gprev, g, sizeof(double) * (size_t)n);
        orc_util_matvec(D, g, p, n, n);
        for (int i = 0; i < n; ++i) p[i] = -p[i];
        double alpha, Fopt;
        ls_secant(&c, X, F, g, p, &alpha, &Fopt);
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        F = Fopt;
        orc_fd_gradient_sharded(o, X, dX, g, n, nprocs);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = g[i] - gprev[i]; }
        orc_update_hessian_inv(D, y, s, n);
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += fabs(X[i] - Xprev[i]);
        gnorm = orc_util_norm2(g, n);
        iter++;
    }
    res->fopt = F; res->iters = iter; res->evals = o->evals - ev0;
    free(D); free(dX); free(g); free(gprev); free(p); free(s); free(y); free(Xprev); free(work);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Levenberg-Marquardt, LevenbergMarquardt.cpp                                            */
/* ------------------------------------------------------------------------------------ */

/* LevenbergMarquardt.cpp:59-83: JT = J^T; JTJ = JT J; A = JTJ, A_ii = (1+lambda) JTJ_ii;
 * rhs = -(JT F); sigma = luSolve(A, rhs). */
int orc_lm_step(const double* J, const double* F, double lambda, int m, int n,
                double* JTJ, double* A, double* rhs, double* sigma) {
    double* JT = (double*)malloc(sizeof(double) * (size_t)n * m);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) JT[(size_t)j * m + i] = J[(size_t)i * n + j];
    orc_util_matmul(JT, J, JTJ, n, m, n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            A[(size_t)i * n + j] = JTJ[(size_t)i * n + j];
            if (i == j) A[(size_t)i * n + j] = (1 + lambda) * JTJ[(size_t)i * n + j];
        }
    orc_util_matvec(JT, F, rhs, n, m);
    for (int i = 0; i < n; ++i) rhs[i] = -rhs[i];
    int rc = orc_util_lusolve(A, rhs, sigma, n);
    free(JT);
    return rc;
}

/* LevMarq::findMin, LevenbergMarquardt.cpp:11-167 */
int orc_lm_findmin(orc_objective* o, const orc_lm_params* prm, double* X, int n, double* F0, double* FOpt,
                   int m, orc_result* res, double* trace, int trace_cap) {
    int maxIter = (int)prm->maxIter;
    double lambda = prm->lambda0;
    double* J = (double*)malloc(sizeof(double) * (size_t)m * n);
    double* JTJ = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* A = (double*)malloc(sizeof(double) * (size_t)n * n);
    double* rhs = (double*)malloc(sizeof(double) * (size_t)n);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* F = (double*)malloc(sizeof(double) * (size_t)m);
    double* Fprev = (double*)malloc(sizeof(double) * (size_t)m);
    double* sigma = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xprev = (double*)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    long ev0 = o->evals;
    orc_obj_eval_multi(o, X, F0);
    memcpy(F, F0, sizeof(double) * (size_t)m);
    memcpy(Fprev, F, sizeof(double) * (size_t)m);
    memcpy(Xprev, X, sizeof(double) * (size_t)n);
    double nrm = orc_util_norm2(F, m);
    double chiSq = nrm * nrm;
    res->f0 = chiSq;
    int iter = 0;
    while (iter < maxIter) {
        orc_fd_jacobian(o, X, dX, J, n, m);
        orc_lm_step(J, F, lambda, m, n, JTJ, A, rhs, sigma);
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
        if (trace && iter < trace_cap) memcpy(trace + (size_t)iter * n, X, sizeof(double) * (size_t)n);
        if (stop) break;
        iter++;
    }
    memcpy(FOpt, F, sizeof(double) * (size_t)m);
    res->fopt = chiSq; res->iters = iter; res->evals = o->evals - ev0;
    free(J); free(JTJ); free(A); free(rhs); free(dX); free(F); free(Fprev); free(sigma); free(Xprev);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Bounded BFGS, BFGS_bnd_linesearch.cpp + computeAlphaBnd + checkBoxBounds              */
/* ------------------------------------------------------------------------------------ */

/* computeAlphaBnd, BFGS_with_bnd_linsearch_MPI.cpp:665-708 */
double orc_compute_alpha_bnd(const double* X, const double* Xlb, const double* Xub, const double* p, int n) {
    double bnd = 0;
    for (int i = 0; i < n; ++i) {
        double a1 = (Xub[i] - X[i]) / p[i];
        double a2 = (Xlb[i] - X[i]) / p[i];
        double ai;
        if (a1 > 0) ai = a1;
        else if (a2 > 0) ai = a2;
        else ai = 0;
        if (i == 0) bnd = ai;
        if (bnd > ai) bnd = ai;
    }
    return bnd;
}

/* checkBoxBounds, Box_boundary_functions.cpp:11-40 */
void orc_check_box_bounds(double* X, const double* Xlb, const double* Xub, int n) {
    for (int i = 0; i < n; ++i)
        if (X[i] - Xlb[i] < -fabs(Xlb[i]) / 1000 || X[i] - Xub[i] > fabs(Xub[i]) / 1000)
            X[i] = (Xlb[i] + Xub[i]) / 2.0;
}

/* cubicInterpMinSimple, BFGS_bnd_linesearch.cpp:736-750 */
static double cubic_interp_min_simple(double aa, double ab, double pa, double pb, double da, double db) {
    double d1 = da + db - 3 * (pa - pb) / (aa - ab);
    double d2 = sign_of(ab - aa) * sqrt(d1 * d1 - da * db);
    double an = ab - (ab - aa) * (db + d2 - d1) / (db - da + 2 * d2);
    if (an < aa || an > ab || an != an) an = (aa + ab) / 2;
    return an;
}

typedef struct {
    orc_objective* o; const orc_bfgs_bnd_params* prm; int nfull; int totalIter; int maxIter;
    int sw;             /* 1: BFGS_Bnd_MPI_SW's pooled line search (Nprocs = procs) */
    int procs;
    int* optimFlag;     /* the SW class member, cleared by a NaN / inf pool value */
    int rank2;          /* 1: updateHessianInv in its O(n^2) rank-2 form (large-n parity runs) */
    double* ftrace;     /* optional: F after every mainBFGSLoop iteration (any recursion level) */
    int trace_cap;
    int depth, max_depth; /* boundaryAssessment recursion depth (diagnostics) */
} bnd_ctx;

/* BFGS_Bnd::lineSearchObj / lineSearchFDDerivative, :465-496 */
static double bnd_ls_obj(bnd_ctx* c, double alpha, const double* X, const double* p, int n,
                         const double* cX, const unsigned char* cI) {
    double* w = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) w[i] = X[i] + alpha * p[i];
    double v = orc_obj_eval_recur(c->o, w, cX, cI, c->nfull);
    free(w);
    return v;
}
static double bnd_ls_deriv(bnd_ctx* c, double alpha, double phia, const double* X, const double* p, int n,
                           const double* cX, const unsigned char* cI) {
    double* w = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) w[i] = X[i] + (alpha + c->prm->dalpha) * p[i];
    double Fa = orc_obj_eval_recur(c->o, w, cX, cI, c->nfull);
    free(w);
    return (Fa - phia) / c->prm->dalpha;
}

/* BFGS_Bnd::lineSearchZoomBnd, :358-457 */
static void bnd_zoom(bnd_ctx* c, double aa, double ab, double pa, double pb, double da, double db,
                     double phi0, double dphi0, const double* X, const double* p, int n,
                     const double* cX, const unsigned char* cI, int* iter_ls,
                     double* aOpt, double* pOpt) {
    const orc_bfgs_bnd_params* P = c->prm;
    int success = 0;
    while (*iter_ls < P->maxIterLineSearch && (ab - aa > P->alphaTol)) {
        double ac = cubic_interp_min_simple(aa, ab, pa, pb, da, db);
        double pc = bnd_ls_obj(c, ac, X, p, n, cX, cI);
        double dc = bnd_ls_deriv(c, ac, pc, X, p, n, cX, cI);
        double pmin = pa;
        if (pb < pa) pmin = pb;
        if (pc > phi0 + P->c1 * ac * dphi0 || pc >= pmin) {
            if (pa < pb) { ab = ac; pb = pc; db = dc; }
            else { aa = ac; pa = pc; da = dc; }
        } else {
            if (fabs(dc) <= fabs(P->c2 * dphi0)) { *aOpt = ac; *pOpt = pc; success = 1; break; }
            if (dc < 0) { aa = ac; pa = pc; da = dc; }
            else { ab = ac; pb = pc; db = dc; }
        }
        (*iter_ls)++;
    }
    if (!success) {
        if (pa < pb) { *aOpt = aa; *pOpt = pa; }
        else { *aOpt = ab; *pOpt = pb; }
    }
}

/* BFGS_Bnd::cubicInterpolationLineSearchBnd, :203-353 */
static void bnd_line_search(bnd_ctx* c, const double* X, const double* Xlb, const double* Xub, double FX,
                            const double* g, const double* p, int n, const double* cX,
                            const unsigned char* cI, double* aOpt, double* Fopt) {
    const orc_bfgs_bnd_params* P = c->prm;
    int success = 0;
    double phii = 0;
    *aOpt = 0; *Fopt = FX;
    double phi0 = FX, dphi0 = orc_util_dot(g, p, n);
    double aim1 = 0, pim1 = phi0, dim1 = dphi0;
    double amax = orc_compute_alpha_bnd(X, Xlb, Xub, p, n);
    double ai = P->alphaGuess;
    if (ai > amax) ai = amax;
    int iter_ls = 0;
    while (iter_ls < P->maxIterLineSearch) {
        phii = bnd_ls_obj(c, ai, X, p, n, cX, cI);
        double di = bnd_ls_deriv(c, ai, phii, X, p, n, cX, cI);
        if ((phii > phi0 + P->c1 * ai * dphi0) || (phii >= pim1 && iter_ls > 1)) {
            bnd_zoom(c, aim1, ai, pim1, phii, dim1, di, phi0, dphi0, X, p, n, cX, cI, &iter_ls, aOpt, Fopt);
            success = 1; break;
        }
        if (fabs(di) <= fabs(P->c2 * dphi0)) { *aOpt = ai; *Fopt = phii; success = 1; break; }
        if (di >= 0) {
            bnd_zoom(c, aim1, ai, pim1, phii, dim1, di, phi0, dphi0, X, p, n, cX, cI, &iter_ls, aOpt, Fopt);
            success = 1; break;
        }
        if (ai == amax) { *aOpt = ai; *Fopt = phii; success = 1; break; }
        aim1 = ai; pim1 = phii; dim1 = di;
        ai = 2 * ai;
        if (ai > amax) ai = amax;
        iter_ls++;
    }
    if (!success) {
        if (pim1 < phii) { *aOpt = aim1; *Fopt = pim1; }
        else if (phi0 < phii) { *aOpt = 0; *Fopt = phi0; }
        else { *aOpt = ai; *Fopt = phii; }
    }
}

/* ---- BFGS_Bnd_MPI_SW's pooled Wolfe search, BFGS_bnd_linesearch_MPI_SW.cpp ---- */

/* evaluateAlphaPoolAndDerivativesIndicator / evaluateAlphaPoolAndDerivatives, :552-699:
 * flagged entries, dealt round-robin to the ranks; a NaN / inf value becomes 1e10 and
 * clears optimFlag */
static void sw_eval_pool(bnd_ctx* c, const double* ap, double* pp, double* dp, const int* ev, int N,
                         const double* X, const double* p, int n, const double* cX, const unsigned char* cI) {
    int* sel = (int*)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
    int ns = 0;
    for (int i = 0; i < N; ++i) if (ev[i] == 1) sel[ns++] = i;
    for (int rank = 0; rank < c->procs; ++rank)
        for (int t = rank; t < ns; t += c->procs) {
            int i = sel[t];
            double phi = bnd_ls_obj(c, ap[i], X, p, n, cX, cI);
            double dphi = bnd_ls_deriv(c, ap[i], phi, X, p, n, cX, cI);
            if (phi != phi || isinf(phi)) phi = 1e10;
            pp[i] = 0.0 + phi;
            dp[i] = 0.0 + dphi;
        }
    for (int t = 0; t < ns; ++t)
        if (pp[sel[t]] == 1e10) *c->optimFlag = 0;
    free(sel);
}

/* computeZoomRegion, :399-431 (neighbour index clamped to the pool, see the C++ note) */
static void sw_zoom_region(const double* ap, const double* pp, const double* dp, int N, double* aa, double* ab,
                           double* pa, double* pb, double* da, double* db) {
    double pmin; int im;
    vector_min(pp, N, &pmin, &im);
    int lo, hi;
    if (dp[im] > 0) { lo = im - 1 >= 0 ? im - 1 : 0; hi = im; }
    else { lo = im; hi = im + 1 < N ? im + 1 : N - 1; }
    *aa = ap[lo]; *ab = ap[hi]; *pa = pp[lo]; *pb = pp[hi]; *da = dp[lo]; *db = dp[hi];
}

/* computeZoomPool, :434-482 */
static void sw_zoom_pool(double aa, double ab, double pa, double pb, double da, double db, double* ap, double* pp,
                         double* dp, int* ev, int N) {
    double ac = cubic_interp_min_simple(aa, ab, pa, pb, da, db);
    if (ac == (aa + ab) / 2) {
        orc_util_linspace(aa, ab, N, ap);
    } else {
        double* al = (double*)malloc(sizeof(double) * (size_t)(N - 1));
        orc_util_linspace(aa, ab, N - 1, al);
        ap[0] = al[0];
        int il = 1;
        for (int i = 1; i < N; ++i) {
            if (ac >= al[il - 1] && ac <= al[il]) { ap[i] = ac; ac = -1; }
            else { ap[i] = al[il]; il++; }
        }
        free(al);
    }
    for (int i = 0; i < N; ++i) ev[i] = 1;
    pp[0] = pa; dp[0] = da; ev[0] = 0;
    pp[N - 1] = pb; dp[N - 1] = db; ev[N - 1] = 0;
}

/* BFGS_Bnd_MPI_SW::lineSearchZoomBnd, :484-548 */
static void sw_zoom(bnd_ctx* c, double aa, double ab, double pa, double pb, double da, double db, double phi0,
                    double dphi0, const double* X, const double* p, int n, const double* cX,
                    const unsigned char* cI, int* iter_ls, double* aOpt, double* pOpt) {
    const orc_bfgs_bnd_params* P = c->prm;
    int N = c->procs + 2;
    int* ev = (int*)malloc(sizeof(int) * (size_t)N);
    double* ap = (double*)calloc((size_t)N, sizeof(double));
    double* pp = (double*)calloc((size_t)N, sizeof(double));
    double* dp = (double*)calloc((size_t)N, sizeof(double));
    int zoom = 1, success = 0;
    while (*iter_ls < P->maxIterLineSearch && (ab - aa > P->alphaTol) && zoom) {
        sw_zoom_pool(aa, ab, pa, pb, da, db, ap, pp, dp, ev, N);
        sw_eval_pool(c, ap, pp, dp, ev, N, X, p, n, cX, cI);
        for (int i = 1; i < N - 1; ++i)
            if ((pp[i] <= phi0 + P->c1 * ap[i] * dphi0) && (fabs(dp[i]) <= fabs(P->c2 * dphi0))) {
                zoom = 0; success = 1;
            }
        if (!success) sw_zoom_region(ap, pp, dp, N, &aa, &ab, &pa, &pb, &da, &db);
        (*iter_ls)++;
    }
    double pmin; int im;
    vector_min(pp, N, &pmin, &im);
    *aOpt = ap[im]; *pOpt = pmin;
    free(ev); free(ap); free(pp); free(dp);
}

/* BFGS_Bnd_MPI_SW::cubicInterpolationLineSearchBnd, :209-397 */
static void sw_line_search(bnd_ctx* c, const double* X, const double* Xlb, const double* Xub, double FX,
                           const double* g, const double* p, int n, const double* cX, const unsigned char* cI,
                           double* aOpt, double* Fopt) {
    const orc_bfgs_bnd_params* P = c->prm;
    int procs = c->procs, N = procs + 1;
    int* ev = (int*)malloc(sizeof(int) * (size_t)N);
    double* ap = (double*)calloc((size_t)N, sizeof(double));
    double* pp = (double*)calloc((size_t)N, sizeof(double));
    double* dp = (double*)calloc((size_t)N, sizeof(double));
    double phi0 = FX, dphi0 = orc_util_dot(g, p, n), pOpt = FX;
    *aOpt = 0; *Fopt = FX;
    for (int i = 0; i < N; ++i) ev[i] = 1;
    ev[0] = 0; ap[0] = 0; pp[0] = phi0; dp[0] = dphi0;
    double amax = orc_compute_alpha_bnd(X, Xlb, Xub, p, n);
    double ai = P->alphaGuess;
    if (ai > amax) ai = amax;
    double delta = ai / procs;
    for (int i = 1; i < N; ++i) ap[i] = delta * i;
    int iter_ls = 0, extend = 1, zoom = 0;
    while (iter_ls < P->maxIterLineSearch && extend) {
        sw_eval_pool(c, ap, pp, dp, ev, N, X, p, n, cX, cI);
        for (int i = 1; i < N; ++i)
            if ((pp[i] > phi0 + P->c1 * ap[i] * dphi0) || (pp[i] >= pp[0] && iter_ls > 1)) { extend = 0; zoom = 1; }
        for (int i = 1; i < N; ++i)
            if (fabs(dp[i]) <= fabs(P->c2 * dphi0)) { extend = 0; zoom = 0; }
        for (int i = 1; i < N; ++i)
            if (dp[i] >= 0) { extend = 0; zoom = 1; }
        if (extend && ap[N - 1] == amax) { extend = 0; zoom = 0; }
        if (extend) {
            double an = (procs + 1) * ap[N - 1];
            if (an > amax) an = amax;
            orc_util_linspace(ap[N - 1], an, N, ap);
            for (int i = 0; i < N; ++i) ev[i] = 1;
            ev[0] = 0;
            pp[0] = pp[N - 1];
            dp[0] = dp[N - 1];
        }
        iter_ls++;
    }
    double pmin; int im;
    if (zoom) {
        double aa, ab, pa, pb, da, db;
        sw_zoom_region(ap, pp, dp, N, &aa, &ab, &pa, &pb, &da, &db);
        if (ab - aa > P->alphaTol) {
            sw_zoom(c, aa, ab, pa, pb, da, db, phi0, dphi0, X, p, n, cX, cI, &iter_ls, aOpt, &pOpt);
        } else {
            vector_min(pp, N, &pmin, &im);
            *aOpt = ap[im]; pOpt = pmin;
        }
    } else {
        vector_min(pp, N, &pmin, &im);
        *aOpt = ap[im]; pOpt = pmin;
    }
    *Fopt = pOpt;
    free(ev); free(ap); free(pp); free(dp);
}

static void bnd_main_loop(bnd_ctx* c, double* F, double* X, double* g, double* D, double* Xlb, double* Xub,
                          double* dX, int n, double* cX, unsigned char* cI, int* optimFlag, int* recurFlag);

/* BFGS_Bnd::boundaryAssessment, :503-728 */
static void bnd_assess(bnd_ctx* c, double* F, double* X, const double* p, double* g, double* D, double* Xlb,
                       double* Xub, double* dX, int ncur, double* cX, unsigned char* cI, int* optimFlag,
                       int* recurFlag) {
    const orc_bfgs_bnd_params* P = c->prm;
    int Ndim = c->nfull;
    unsigned char* cIcur = (unsigned char*)calloc((size_t)(ncur > 0 ? ncur : 1), 1);
    int* frozen = (int*)malloc(sizeof(int) * (size_t)(Ndim > 0 ? Ndim : 1));
    int nfrozen = 0, bndFlag = 0;
    int icur = 0;
    for (int i = 0; i < Ndim; ++i) {
        if (!cI[i]) {
            if ((fabs(X[icur] - Xlb[icur]) < P->bndTol) && ((p[icur] < 0) || (g[icur] > 0))) {
                bndFlag = 1; cI[i] = 1; cX[i] = X[icur]; cIcur[icur] = 1; frozen[nfrozen++] = i;
            } else if ((fabs(X[icur] - Xub[icur]) < P->bndTol) && ((p[icur] > 0) || (g[icur] < 0))) {
                bndFlag = 1; cI[i] = 1; cX[i] = X[icur]; cIcur[icur] = 1; frozen[nfrozen++] = i;
            }
            icur++;
        }
    }
    int Nconst = 0;
    for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
    int nr = Ndim - Nconst;
    if (bndFlag && nr > 0) {
        double FR = *F;
        double* XR = (double*)malloc(sizeof(double) * (size_t)nr);
        double* gR = (double*)malloc(sizeof(double) * (size_t)nr);
        double* lbR = (double*)malloc(sizeof(double) * (size_t)nr);
        double* ubR = (double*)malloc(sizeof(double) * (size_t)nr);
        double* dXR = (double*)malloc(sizeof(double) * (size_t)nr);
        double* DR = (double*)malloc(sizeof(double) * (size_t)nr * nr);
        int ir = 0;
        for (icur = 0; icur < ncur; ++icur)
            if (!cIcur[icur]) {
                XR[ir] = X[icur]; gR[ir] = g[icur]; lbR[ir] = Xlb[icur]; ubR[ir] = Xub[icur]; dXR[ir] = dX[icur];
                ir++;
            }
        set_identity(DR, nr);
        *recurFlag = 1;
        if (++c->depth > c->max_depth) c->max_depth = c->depth;
        bnd_main_loop(c, &FR, XR, gR, DR, lbR, ubR, dXR, nr, cX, cI, optimFlag, recurFlag);
        c->depth--;
        ir = 0;
        for (icur = 0; icur < ncur; ++icur)
            if (!cIcur[icur]) {
                *F = FR; X[icur] = XR[ir]; g[icur] = gR[ir]; Xlb[icur] = lbR[ir]; Xub[icur] = ubR[ir];
                dX[icur] = dXR[ir];
                ir++;
            }
        for (int k = 0; k < nfrozen; ++k) cI[frozen[k]] = 0;
        set_identity(D, ncur);
        orc_fd_gradient_recur(c->o, X, dX, g, ncur, cX, cI, Ndim);
        int cont = 0;
        for (icur = 0; icur < ncur; ++icur)
            if (cIcur[icur]) {
                if ((fabs(X[icur] - Xlb[icur]) < P->bndTol) && (g[icur] < 0)) cont = 1;
                else if ((fabs(X[icur] - Xub[icur]) < P->bndTol) && (g[icur] > 0)) cont = 1;
            }
        Nconst = 0;
        for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
        if (Nconst == 0) *recurFlag = 0;
        *optimFlag = cont;
        free(XR); free(gR); free(lbR); free(ubR); free(dXR); free(DR);
    } else if (nr == 0) {
        *optimFlag = 0;
    }
    free(cIcur); free(frozen);
}

/* BFGS_Bnd::mainBFGSLoop, :116-201 */
static void bnd_main_loop(bnd_ctx* c, double* F, double* X, double* g, double* D, double* Xlb, double* Xub,
                          double* dX, int n, double* cX, unsigned char* cI, int* optimFlag, int* recurFlag) {
    const orc_bfgs_bnd_params* P = c->prm;
    size_t nb = sizeof(double) * (size_t)(n > 0 ? n : 1);
    double* gprev = (double*)malloc(nb);
    double* p = (double*)malloc(nb);
    double* s = (double*)malloc(nb);
    double* y = (double*)malloc(nb);
    double* Xprev = (double*)malloc(nb);
    memcpy(gprev, g, sizeof(double) * (size_t)n);
    int iter = 0;
    double xdiff = P->xMinDiff * 2, gnorm = 2 * P->minGrad2Norm;
    while (*optimFlag && iter < c->maxIter && xdiff > P->xMinDiff && gnorm > P->minGrad2Norm &&
           c->totalIter < c->maxIter) {
        orc_util_matvec(D, g, p, n, n);
        for (int i = 0; i < n; ++i) p[i] = -p[i];
        double alpha, Fopt;
        if (c->sw) sw_line_search(c, X, Xlb, Xub, *F, g, p, n, cX, cI, &alpha, &Fopt);
        else bnd_line_search(c, X, Xlb, Xub, *F, g, p, n, cX, cI, &alpha, &Fopt);
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        *F = Fopt;
        memcpy(gprev, g, sizeof(double) * (size_t)n);
        orc_fd_gradient_recur(c->o, X, dX, g, n, cX, cI, c->nfull);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = g[i] - gprev[i]; }
        if (c->rank2) orc_update_hessian_inv_rank2(D, y, s, n);
        else orc_update_hessian_inv(D, y, s, n);
        bnd_assess(c, F, X, p, g, D, Xlb, Xub, dX, n, cX, cI, optimFlag, recurFlag);
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += fabs(X[i] - Xprev[i]);
        gnorm = orc_util_norm2(g, n);
        if (c->ftrace && c->totalIter < c->trace_cap) c->ftrace[c->totalIter] = *F;
        iter++;
        c->totalIter++;
    }
    free(gprev); free(p); free(s); free(y); free(Xprev);
}

/* BFGS_Bnd::findMinBnd, BFGS_bnd_linesearch.cpp:15-113 (no dXGradVec / initialScalingVec) */
int orc_bfgs_bnd_findmin(orc_objective* o, const orc_bfgs_bnd_params* prm, double* X, const double* Xlb_in,
                         const double* Xub_in, int n, orc_result* res) {
    return orc_bfgs_bnd_findmin_ex(o, prm, X, Xlb_in, Xub_in, n, res, 0, NULL, 0, NULL);
}

int orc_bfgs_bnd_findmin_ex(orc_objective* o, const orc_bfgs_bnd_params* prm, double* X, const double* Xlb_in,
                            const double* Xub_in, int n, orc_result* res, int rank2, double* ftrace, int trace_cap,
                            int* max_depth) {
    bnd_ctx c = {o, prm, n, 0, (int)prm->maxIter, 0, 1, NULL, rank2, ftrace, trace_cap, 0, 0};
    double* Xlb = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xub = (double*)malloc(sizeof(double) * (size_t)n);
    memcpy(Xlb, Xlb_in, sizeof(double) * (size_t)n);
    memcpy(Xub, Xub_in, sizeof(double) * (size_t)n);
    orc_check_box_bounds(X, Xlb, Xub, n);
    double* cX = (double*)calloc((size_t)n, sizeof(double));
    unsigned char* cI = (unsigned char*)calloc((size_t)n, 1);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* g = (double*)calloc((size_t)n, sizeof(double));
    double* D = (double*)malloc(sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    if (prm->initHessFD) {
        double* B = (double*)malloc(sizeof(double) * (size_t)n * n);
        double* dXH = (double*)malloc(sizeof(double) * (size_t)n);
        for (int i = 0; i < n; ++i) dXH[i] = prm->dXHess;
        orc_fd_hessian(o, X, dXH, B, n);
        orc_util_matinv(B, D, n);
        free(B); free(dXH);
    } else {
        set_identity(D, n);
    }
    long ev0 = o->evals;
    orc_fd_gradient_recur(o, X, dX, g, n, cX, cI, n);
    double F = orc_obj_eval_recur(o, X, cX, cI, n);
    res->f0 = F;
    int optimFlag = 1, recurFlag = 0;
    bnd_main_loop(&c, &F, X, g, D, Xlb, Xub, dX, n, cX, cI, &optimFlag, &recurFlag);
    res->fopt = F; res->iters = c.totalIter; res->evals = o->evals - ev0;
    if (max_depth) *max_depth = c.max_depth;
    free(Xlb); free(Xub); free(cX); free(cI); free(dX); free(g); free(D);
    return 0;
}

/* BFGS_Bnd_MPI_SW::findMinBnd, BFGS_bnd_linesearch_MPI_SW.cpp:12-113, with Nprocs = procs
 * (gradients through the Recur FD engine: the sharded MPIRecur form gives the same values) */
int orc_bfgs_bnd_mpi_sw_findmin(orc_objective* o, const orc_bfgs_bnd_params* prm, int procs, double* X,
                                const double* Xlb_in, const double* Xub_in, int n, orc_result* res) {
    int optimFlag = 1, recurFlag = 0;
    bnd_ctx c = {o, prm, n, 0, (int)prm->maxIter, 1, procs, &optimFlag, 0, NULL, 0, 0, 0};
    double* Xlb = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xub = (double*)malloc(sizeof(double) * (size_t)n);
    memcpy(Xlb, Xlb_in, sizeof(double) * (size_t)n);
    memcpy(Xub, Xub_in, sizeof(double) * (size_t)n);
    orc_check_box_bounds(X, Xlb, Xub, n);
    double* cX = (double*)calloc((size_t)n, sizeof(double));
    unsigned char* cI = (unsigned char*)calloc((size_t)n, 1);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* g = (double*)calloc((size_t)n, sizeof(double));
    double* D = (double*)malloc(sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    if (prm->initHessFD) {
        double* B = (double*)malloc(sizeof(double) * (size_t)n * n);
        double* dXH = (double*)malloc(sizeof(double) * (size_t)n);
        for (int i = 0; i < n; ++i) dXH[i] = prm->dXHess;
        orc_fd_hessian(o, X, dXH, B, n);
        orc_util_matinv(B, D, n);
        free(B); free(dXH);
    } else {
        set_identity(D, n);
    }
    long ev0 = o->evals;
    orc_fd_gradient_recur(o, X, dX, g, n, cX, cI, n);
    double F = orc_obj_eval_recur(o, X, cX, cI, n);
    res->f0 = F;
    bnd_main_loop(&c, &F, X, g, D, Xlb, Xub, dX, n, cX, cI, &optimFlag, &recurFlag);
    res->fopt = F; res->iters = c.totalIter; res->evals = o->evals - ev0;
    free(Xlb); free(Xub); free(cX); free(cI); free(dX); free(g); free(D);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Bounded BFGS with a pooled secant line search, BFGS_with_bnd_linsearch_MPI.cpp         */
/* ------------------------------------------------------------------------------------ */

typedef struct {
    orc_objective* o; const orc_bfgs_bnd_mpi_params* prm; int nfull; int npool; int nprocs; int failed;
} bndmpi_ctx;

/* checkAlphaPoolBnd, :711-743 */
void orc_check_alpha_pool_bnd(int* bndIndicator, double* ap, int Np, const double* X, const double* Xlb,
                              const double* Xub, const double* p, int n) {
    *bndIndicator = 0;
    double alphaBnd = orc_compute_alpha_bnd(X, Xlb, Xub, p, n);
    for (int i = 0; i < Np; ++i)
        if (ap[i] > alphaBnd) *bndIndicator = 1;
    if (*bndIndicator) {
        double deltaAlpha = alphaBnd / (Np);
        for (int i = 0; i < Np; ++i) ap[i] = deltaAlpha * (i + 1);
    }
    for (int i = 0; i < Np; ++i)
        if (ap[i] < 0) ap[i] = 0;
}

/* BFGSBnd_MPI::evalAlphaPoolMPI / lineSearchObj, :246-354 (rank-ordered, zero-padded sum;
 * a NaN / inf value ends the solve, where the reference calls exit(0)) */
static void bndmpi_eval_pool(bndmpi_ctx* c, const double* ap, double* pp, int N, const double* X,
                             const double* p, int n, const double* cX, const unsigned char* cI) {
    double* w = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int rank = 0; rank < c->nprocs; ++rank)
        for (int i = rank; i < N; i += c->nprocs) {
            for (int k = 0; k < n; ++k) w[k] = X[k] + ap[i] * p[k];
            pp[i] = 0.0 + orc_obj_eval_recur(c->o, w, cX, cI, c->nfull);
            if (pp[i] != pp[i] || isinf(pp[i])) c->failed = 1;
        }
    free(w);
}

/* BFGSBnd_MPI::secantLineSearchBnd, :358-660 */
static void bndmpi_line_search(bndmpi_ctx* c, const double* X, const double* Xlb, const double* Xub, double FX,
                               const double* g, const double* p, int n, const double* cX,
                               const unsigned char* cI, double* alphaOpt, double* Fopt) {
    const orc_bfgs_bnd_mpi_params* P = c->prm;
    int Np = c->npool;
    double* ap = (double*)calloc((size_t)Np, sizeof(double));
    double* pp = (double*)calloc((size_t)Np, sizeof(double));
    double* apPrev = (double*)malloc(sizeof(double) * (size_t)Np);
    double* ppPrev = (double*)calloc((size_t)Np, sizeof(double));
    double* slope = (double*)calloc((size_t)Np, sizeof(double));
    double* ap2 = (double*)calloc((size_t)Np + 2, sizeof(double));
    double* pp2 = (double*)calloc((size_t)Np + 2, sizeof(double));
    for (int i = 0; i < Np; ++i) apPrev[i] = -1;
    *alphaOpt = 0; *Fopt = FX;
    double a0 = 0, phi0 = FX, dphi0 = orc_util_dot(g, p, n);
    int bnd = 0;
    int idxMin = -(int)ceil((Np - 1.0) / 2.0);
    int idxMax = (int)floor((Np - 1.0) / 2.0);
    double r = pow(P->maxAlphaMult, 1.0 / (double)idxMax);
    int idx = idxMin;
    for (int k = 0; k < Np; ++k) { ap[k] = P->alphaGuess * pow(r, idx); idx++; }
    int first = 1, zoom = 0;
    for (int it = 0; it < P->maxIterLineSearch && first && !c->failed; ++it) {
        orc_check_alpha_pool_bnd(&bnd, ap, Np, X, Xlb, Xub, p, n);
        bndmpi_eval_pool(c, ap, pp, Np, X, p, n, cX, cI);
        for (int i = 0; i < Np; ++i)
            if (pp[i] > phi0 + P->c1 * ap[i] * dphi0) { zoom = 1; first = 0; }
        slope[0] = (pp[0] - phi0) / (ap[0] - a0);
        for (int i = 1; i < Np; ++i) slope[i] = (pp[i] - pp[i - 1]) / (ap[i] - ap[i - 1]);
        if (first)
            for (int i = 0; i < Np; ++i)
                if (fabs(slope[i]) <= fabs(P->c2 * dphi0)) { zoom = 0; first = 0; }
        if (first)
            for (int i = 0; i < Np; ++i)
                if (slope[i] >= 0) { zoom = 1; first = 0; }
        if (first && !bnd) {
            double amax; int imax;
            vector_max(ap, Np, &amax, &imax);
            r = pow(P->maxAlphaMult, 1.0 / (double)Np);
            for (int i = 0; i < Np; ++i) {
                apPrev[i] = ap[i]; ppPrev[i] = pp[i];
                double power = i + 1;
                ap[i] = amax * pow(r, power);
            }
        } else if (bnd) {
            first = 0;
        }
    }
    double alo, ahi, plo, phi;
    if (apPrev[0] < 0) {
        find_pool_bounds(ap, pp, Np, a0, phi0, &alo, &ahi, &plo, &phi);
    } else {
        double* ae = (double*)malloc(sizeof(double) * 2 * (size_t)Np);
        double* pe = (double*)malloc(sizeof(double) * 2 * (size_t)Np);
        for (int i = 0; i < Np; ++i) { ae[i] = apPrev[i]; ae[i + Np] = ap[i]; pe[i] = ppPrev[i]; pe[i + Np] = pp[i]; }
        find_pool_bounds(ae, pe, 2 * Np, a0, phi0, &alo, &ahi, &plo, &phi);
        free(ae); free(pe);
    }
    for (int it = 0; it < P->maxIterLineSearch && zoom && !c->failed; ++it) {
        orc_util_linspace(alo, ahi, Np + 2, ap2);
        pp2[0] = plo; pp2[Np + 1] = phi; ap2[0] = alo; ap2[Np + 1] = ahi;
        for (int i = 0; i < Np; ++i) { ap[i] = ap2[i + 1]; pp[i] = pp2[i + 1]; }
        bndmpi_eval_pool(c, ap, pp, Np, X, p, n, cX, cI);
        for (int i = 0; i < Np; ++i) { ap2[i + 1] = ap[i]; pp2[i + 1] = pp[i]; }
        for (int i = 0; i < Np; ++i) slope[i] = (pp2[i + 1] - pp2[i]) / (ap2[i + 1] - ap2[i]);
        for (int i = 0; i < Np; ++i)
            if (fabs(slope[i]) <= fabs(P->c2 * dphi0)) zoom = 0;
        if (zoom) find_pool_bounds(ap2, pp2, Np + 2, a0, phi0, &alo, &ahi, &plo, &phi);
        double a2max; int i2max;
        vector_max(ap2, Np + 2, &a2max, &i2max);
        if (a2max < P->alphaMin) zoom = 0;
    }
    /* minimum of the last evaluated pool, :651-655 */
    double pmin; int imin;
    vector_min(pp, Np, &pmin, &imin);
    *alphaOpt = ap[imin];
    *Fopt = pmin;
    free(ap); free(pp); free(apPrev); free(ppPrev); free(slope); free(ap2); free(pp2);
}

static void bndmpi_main_loop(bndmpi_ctx* c, double* F, double* X, double* g, double* D, double* Xlb, double* Xub,
                             double* dX, int n, double* cX, unsigned char* cI, int* optimFlag, int* recurFlag);

/* BFGSBnd_MPI::boundaryAssessment, :748-934 (top level only: n == nfull) */
static void bndmpi_assess(bndmpi_ctx* c, double* F, double* X, const double* p, double* g, double* D,
                          double* Xlb, double* Xub, double* dX, double* cX, unsigned char* cI, int* optimFlag,
                          int* recurFlag) {
    const orc_bfgs_bnd_mpi_params* P = c->prm;
    int Ndim = c->nfull, bndFlag = 0, iR = 0;
    for (int i = 0; i < Ndim; ++i) {
        if (!cI[i]) {
            if ((fabs(X[iR] - Xlb[iR]) < P->dXGrad) && (p[iR] < 0)) { bndFlag = 1; cI[i] = 1; cX[i] = X[iR]; }
            else if (fabs(X[iR] - Xub[iR]) < P->dXGrad && (p[iR] > 0)) { bndFlag = 1; cI[i] = 1; cX[i] = X[iR]; }
            iR++;
        }
    }
    int Nconst = 0;
    for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
    int nr = Ndim - Nconst;
    if (!(bndFlag && nr > 0)) return;
    double FR = *F;
    double* XR = (double*)malloc(sizeof(double) * (size_t)nr);
    double* gR = (double*)malloc(sizeof(double) * (size_t)nr);
    double* lbR = (double*)malloc(sizeof(double) * (size_t)nr);
    double* ubR = (double*)malloc(sizeof(double) * (size_t)nr);
    double* dXR = (double*)malloc(sizeof(double) * (size_t)nr);
    double* DR = (double*)malloc(sizeof(double) * (size_t)nr * nr);
    int ir = 0;
    for (int i = 0; i < Ndim; ++i) {
        if (cI[i]) continue;
        XR[ir] = X[i]; gR[ir] = g[i]; lbR[ir] = Xlb[i]; ubR[ir] = Xub[i]; dXR[ir] = dX[i];
        int jr = 0;
        for (int j = 0; j < Ndim; ++j)
            if (!cI[j]) { DR[(size_t)ir * nr + jr] = D[(size_t)i * Ndim + j]; jr++; }
        ir++;
    }
    *recurFlag = 1;
    bndmpi_main_loop(c, &FR, XR, gR, DR, lbR, ubR, dXR, nr, cX, cI, optimFlag, recurFlag);
    ir = 0;
    for (int i = 0; i < Ndim; ++i)
        if (!cI[i]) { X[i] = XR[ir]; g[i] = gR[ir]; Xlb[i] = lbR[ir]; Xub[i] = ubR[ir]; dX[i] = dXR[ir]; ir++; }
    /* F keeps its pre-recursion value (FRecur is not copied back, :845-864) */
    set_identity(D, Ndim);
    orc_fd_gradient_sharded(c->o, X, dX, g, Ndim, c->nprocs);
    for (int i = 0; i < Ndim; ++i) {
        cI[i] = 0;
        if ((fabs(X[i] - Xlb[i]) < P->dXGrad) && (g[i] > 0)) { cI[i] = 1; cX[i] = X[i]; }
        else if (fabs(X[i] - Xub[i]) < P->dXGrad && (g[i] < 0)) { cI[i] = 1; cX[i] = X[i]; }
    }
    Nconst = 0;
    for (int i = 0; i < Ndim; ++i) Nconst += cI[i];
    *optimFlag = Nconst == 0;
    *recurFlag = 0;
    free(XR); free(gR); free(lbR); free(ubR); free(dXR); free(DR);
}

/* BFGSBnd_MPI::mainBFGSLoop, :84-243 */
static void bndmpi_main_loop(bndmpi_ctx* c, double* F, double* X, double* g, double* D, double* Xlb, double* Xub,
                             double* dX, int n, double* cX, unsigned char* cI, int* optimFlag, int* recurFlag) {
    const orc_bfgs_bnd_mpi_params* P = c->prm;
    size_t nb = sizeof(double) * (size_t)(n > 0 ? n : 1);
    double* gprev = (double*)malloc(nb);
    double* p = (double*)malloc(nb);
    double* s = (double*)malloc(nb);
    double* y = (double*)malloc(nb);
    double* Xprev = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    double Fprev = 2 * *F;
    memcpy(gprev, g, sizeof(double) * (size_t)n);
    orc_util_matvec(D, g, p, n, n);
    for (int i = 0; i < n; ++i) p[i] = -p[i];
    int iter = 0, maxIter = (int)P->maxIter;
    double xdiff = P->xMinDiff * 2, gnorm = 2 * P->minGrad2Norm, alpha = P->alphaMin * 2;
    while (iter < maxIter && xdiff > P->xMinDiff && gnorm > P->minGrad2Norm && alpha > P->alphaMin && *optimFlag &&
           !c->failed) {
        double Fopt;
        bndmpi_line_search(c, X, Xlb, Xub, *F, g, p, n, cX, cI, &alpha, &Fopt);
        if (*F - Fopt < P->FStepTolerance) {
            orc_fd_gradient_recur(c->o, X, dX, g, n, cX, cI, c->nfull);
            for (int i = 0; i < n; ++i) p[i] = -g[i];
            bndmpi_line_search(c, X, Xlb, Xub, *F, g, p, n, cX, cI, &alpha, &Fopt);
        }
        if (c->failed) break;
        for (int i = 0; i < n; ++i) { Xprev[i] = X[i]; X[i] = X[i] + alpha * p[i]; }
        Fprev = *F;
        *F = Fopt;
        orc_fd_gradient_recur(c->o, X, dX, g, n, cX, cI, c->nfull);
        for (int i = 0; i < n; ++i) { s[i] = alpha * p[i]; y[i] = g[i] - gprev[i]; }
        if (orc_util_dot(y, s, n) != 0) orc_update_hessian_inv(D, y, s, n);
        memcpy(gprev, g, sizeof(double) * (size_t)n);
        orc_util_matvec(D, g, p, n, n);
        for (int i = 0; i < n; ++i) p[i] = -p[i];
        if (*F > Fprev) *optimFlag = 0;
        xdiff = 0;
        for (int i = 0; i < n; ++i) xdiff += fabs(X[i] - Xprev[i]);
        gnorm = orc_util_norm2(g, n);
        if (!*recurFlag) bndmpi_assess(c, F, X, p, g, D, Xlb, Xub, dX, cX, cI, optimFlag, recurFlag);
        iter++;
    }
    free(gprev); free(p); free(s); free(y); free(Xprev);
}

/* BFGSBnd_MPI::findMinBnd, BFGS_with_bnd_linsearch_MPI.cpp:14-81, with Npool = npool and the
 * FD gradients sharded over nprocs owners (values do not depend on nprocs).  Returns -1
 * when a pool value is NaN / inf (the reference's exit(0) path). */
int orc_bfgs_bnd_mpi_findmin(orc_objective* o, const orc_bfgs_bnd_mpi_params* prm, int npool, int nprocs,
                             double* X, const double* Xlb_in, const double* Xub_in, int n, orc_result* res) {
    bndmpi_ctx c = {o, prm, n, npool, nprocs, 0};
    double* Xlb = (double*)malloc(sizeof(double) * (size_t)n);
    double* Xub = (double*)malloc(sizeof(double) * (size_t)n);
    memcpy(Xlb, Xlb_in, sizeof(double) * (size_t)n);
    memcpy(Xub, Xub_in, sizeof(double) * (size_t)n);
    double* cX = (double*)calloc((size_t)n, sizeof(double));
    unsigned char* cI = (unsigned char*)calloc((size_t)n, 1);
    double* dX = (double*)malloc(sizeof(double) * (size_t)n);
    double* g = (double*)calloc((size_t)n, sizeof(double));
    double* D = (double*)malloc(sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) dX[i] = prm->dXGrad;
    orc_check_box_bounds(X, Xlb, Xub, n);
    if (prm->initHessFD) {
        double* B = (double*)malloc(sizeof(double) * (size_t)n * n);
        double* dXH = (double*)malloc(sizeof(double) * (size_t)n);
        for (int i = 0; i < n; ++i) dXH[i] = prm->dXHess;
        orc_fd_hessian(o, X, dXH, B, n);
        orc_util_matinv(B, D, n);
        free(B); free(dXH);
    } else {
        set_identity(D, n);
    }
    long ev0 = o->evals;
    orc_fd_gradient_sharded(o, X, dX, g, n, nprocs);
    double F = orc_obj_eval(o, X);
    res->f0 = F;
    int optimFlag = 1, recurFlag = 0;
    bndmpi_main_loop(&c, &F, X, g, D, Xlb, Xub, dX, n, cX, cI, &optimFlag, &recurFlag);
    res->fopt = F; res->iters = 0; res->evals = o->evals - ev0;
    free(Xlb); free(Xub); free(cX); free(cI); free(dX); free(g); free(D);
    return c.failed ? -1 : 0;
}

/* ------------------------------------------------------------------------------------ */
/* synthetic inputs                                                                       */
/* ------------------------------------------------------------------------------------ */

/* counter form of splitmix64: the idx-th output of a generator seeded with `seed` */
double orc_splitmix_u01(unsigned long long seed, unsigned long long idx) {
    unsigned long long z = seed + (idx + 1ULL) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    return (double)(z >> 11) * 0x1.0p-53;
}

/* d_i = 1 + 3u (stream 0..n-1), b_i = 2u - 1 (stream n..2n-1) */
void orc_make_quadratic(unsigned long long seed, int n, double* d, double* b) {
    for (int i = 0; i < n; ++i) d[i] = 1.0 + 3.0 * orc_splitmix_u01(seed, (unsigned long long)i);
    for (int i = 0; i < n; ++i) b[i] = 2.0 * orc_splitmix_u01(seed, (unsigned long long)(n + i)) - 1.0;
}

/* A_ij = (2u-1)/sqrt(n) (stream i*n+j), x*_j = 2u-1 (stream m*n + j), y = A x* (fma chain) */
void orc_make_linres(unsigned long long seed, int m, int n, double* A, double* xstar, double* y) {
    double scale = 1.0 / sqrt((double)n);
    size_t mn = (size_t)m * n;
    for (size_t k = 0; k < mn; ++k) A[k] = (2.0 * orc_splitmix_u01(seed, k) - 1.0) * scale;
    for (int j = 0; j < n; ++j) xstar[j] = 2.0 * orc_splitmix_u01(seed, mn + (size_t)j) - 1.0;
    for (int i = 0; i < m; ++i) {
        double acc = 0.0;
        for (int k = 0; k < n; ++k) acc = fma(A[(size_t)i * n + k], xstar[k], acc);
        y[i] = acc;
    }
}

void orc_make_expcurve_data(int m, double* xData, double* yData) {
    orc_util_linspace(0, 5, m, xData);
    for (int k = 0; k < m; ++k) yData[k] = 10.2 * exp(0.4 * xData[k]) + 0.1;
}

void orc_make_cubic_data(int m, double* xData, double* yData) {
    orc_util_linspace(-5, 5, m, xData);
    for (int k = 0; k < m; ++k) {
        double x = xData[k];
        yData[k] = 0.3 * pow(x, 3.0) + 1.1 * (x * x) - 4.3 * x + 7.3;
    }
}

/* ------------------------------------------------------------------------------------ */
/* genetic algorithm                                                  */
/* ------------------------------------------------------------------------------------ */
/* GeneticAlgorithm::findMinBnd (GeneticAlgorithm.cpp:12-297) and GeneticAlgorithmMPI
 * (GeneticAlgorithmMPI.cpp:12-414).  timeRand() (UtilityFunctionLibrary, absent) is restated
 * as a uniform double in [0, 1) from a splitmix64 stream; the three documented repairs of the
 * product (include/GeneticAlgorithm.hpp: clamped selection index, uniform selection when every
 * fitness is 0, first-minimum sort) are applied the same way here.  nprocs > 1: the population
 * evaluation is dealt round-robin over nprocs ranks and every value comes back as v + 0.0 (the
 * reference's zero-padded MPI_Allreduce); nprocs == 0: the serial class. */
typedef struct {
    unsigned long long state;
} ga_rng;

static double ga_next(ga_rng* r) {
    unsigned long long z = (r->state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1.0p-53;
}

/* GeneticAlgorithm.cpp:312-340 */
static void ga_identical(double* Xp, int Npop, int n, const double* lb, const double* ub, int* ind, ga_rng* r) {
    for (int i = 0; i < Npop; i++)
        for (int k = i + 1; k < Npop; k++) {
            int same = 0;
            for (int j = 0; j < n; j++)
                if (Xp[i * n + j] == Xp[k * n + j]) same++;
            if (same == n) {
                for (int j = 0; j < n; j++) Xp[i * n + j] = lb[j] + (ub[j] - lb[j]) * ga_next(r);
                ind[i] = 1;
            }
        }
}

/* GeneticAlgorithm.cpp:343-362 */
static void ga_bounds(double* Xp, int Npop, int n, const double* lb, const double* ub, int* ind, ga_rng* r) {
    for (int i = 0; i < Npop; i++)
        for (int j = 0; j < n; j++)
            if (Xp[i * n + j] > ub[j] || Xp[i * n + j] < lb[j]) {
                Xp[i * n + j] = lb[j] + (ub[j] - lb[j]) * ga_next(r);
                ind[i] = 1;
            }
}

/* GeneticAlgorithm.cpp:367-406: repeated first minimum among the members not yet placed */
static void ga_sort(double* Xp, double* F, int Npop, int n, double* Xt, double* Ft, int* taken) {
    for (int i = 0; i < Npop; i++) taken[i] = 0;
    for (int k = 0; k < Npop; k++) {
        int best = -1;
        for (int i = 0; i < Npop; i++)
            if (!taken[i] && (best < 0 || F[i] < F[best])) best = i;
        taken[best] = 1;
        memcpy(Xt + (size_t)k * n, Xp + (size_t)best * n, sizeof(double) * n);
        Ft[k] = F[best];
    }
    memcpy(Xp, Xt, sizeof(double) * (size_t)Npop * n);
    memcpy(F, Ft, sizeof(double) * Npop);
}

/* GeneticAlgorithm::evaluatePopulation (:301-310) / evaluatePopulationParallel (MPI :283-414) */
static void ga_pad(double* Xp, double* F, int Npop, int n) {   /* the zero-padded sums, P > 1 */
    for (int i = 0; i < Npop; i++) {
        F[i] = F[i] + 0.0;
        for (int j = 0; j < n; j++) Xp[(size_t)i * n + j] = Xp[(size_t)i * n + j] + 0.0;
    }
}

/* which rank evaluates a member changes no value: only the padding of the two exchanges shows */
static void ga_evaluate(orc_objective* o, double* Xp, double* F, const int* ind, int Npop, int n, int nprocs) {
    if (nprocs > 1) ga_pad(Xp, F, Npop, n);   /* the root's population to every rank */
    for (int i = 0; i < Npop; i++)
        if (ind[i]) F[i] = orc_obj_eval(o, Xp + (size_t)i * n);
    if (nprocs > 1) ga_pad(Xp, F, Npop, n);   /* the values back */
}

static int ga_select(ga_rng* r, const double* fitness, double maxFitness, int Npop) {
    /* repair: uniform over 1..Npop-1 when no member past the best has positive fitness (all
     * tie with the worst; the weighted draw would accept only u == 0 and loop forever) */
    int flat = 1;
    for (int k = 1; k < Npop; k++)
        if (fitness[k] > 0.0) { flat = 0; break; }
    int index = 0;
    while (index == 0) {
        int k = (int)round(ga_next(r) * Npop);
        if (k > Npop - 1) k = Npop - 1;
        const double u = ga_next(r);
        if (flat || maxFitness == 0.0 || u <= fitness[k] / maxFitness) index = k;
    }
    return index;
}

/* params: Npop, maxGenerations, eliteFrac, crossFrac, eliteMutationFrac, mutationSize,
 * eliteMutationSize, initialPopScaling, NstaticGenerations; res->iters = generations */
int orc_ga_findmin(orc_objective* o, const double* prm, unsigned long long seed, int nprocs, double* X,
                   const double* lb, const double* ub, int n, orc_result* res) {
    const int Npop = (int)prm[0], maxGen = (int)prm[1];
    const double eliteFrac = prm[2], crossFrac = prm[3], eliteMutFrac = prm[4], mutSize = prm[5], eliteMutSize = prm[6];
    const double Nstatic_max = prm[8];
    const int Nelite = (int)ceil(eliteFrac * Npop), NeliteMut = (int)ceil(eliteMutFrac * Npop),
              Ncross = (int)ceil(crossFrac * Npop), Nrand = Npop - Nelite - NeliteMut - Ncross;
    if (Nrand <= 0 || Npop < 2) return -1;
    const size_t pn = (size_t)Npop * n;
    double* Xp = calloc(pn, sizeof(double));
    double* Xn = calloc(pn, sizeof(double));
    double* Xt = calloc(pn, sizeof(double));
    double* F = calloc(Npop, sizeof(double));
    double* Fn = calloc(Npop, sizeof(double));
    double* Ft = calloc(Npop, sizeof(double));
    double* fit = calloc(Npop, sizeof(double));
    int* ind = calloc(Npop, sizeof(int));
    int* taken = calloc(Npop, sizeof(int));
    int* idx = calloc(n, sizeof(int));
    ga_rng r = {seed};
    o->evals = 0;
    for (int i = 0; i < Npop; i++) ind[i] = 1;
    for (int j = 0; j < n; j++) Xp[j] = X[j];
    for (int i = 1; i < Npop; i++)
        for (int j = 0; j < n; j++) Xp[(size_t)i * n + j] = Xp[j] + ((ub[j] - lb[j]) * ga_next(&r) + lb[j]);
    ga_identical(Xn, Npop, n, lb, ub, ind, &r);   /* the reference checks XpopNew (zeros) here */
    ga_bounds(Xp, Npop, n, lb, ub, ind, &r);
    ga_evaluate(o, Xp, F, ind, Npop, n, nprocs);
    res->f0 = F[0];
    ga_sort(Xp, F, Npop, n, Xt, Ft, taken);
    double FbestPrev = F[0];
    int Nstatic = 0, iter = 0;
    while (iter < maxGen) {
        for (int k = 0; k < Npop; k++) fit[k] = pow(F[Npop - 1] - F[k], 2);
        const double maxFit = fit[0];
        for (int k = 0; k < Npop; k++) ind[k] = 1;
        int p = 0;
        for (int k = 0; k < Nelite; k++, p++) {
            memcpy(Xn + (size_t)p * n, Xp + (size_t)p * n, sizeof(double) * n);
            Fn[p] = F[p];
            ind[p] = 0;
        }
        for (int k = 0; k < Ncross; k++, p++) {
            for (int i = 0; i < n; i++) idx[i] = ga_select(&r, fit, maxFit, Npop);
            for (int i = 0; i < n; i++) Xn[(size_t)p * n + i] = Xp[(size_t)idx[i] * n + i];
        }
        const double spread = mutSize * (maxGen - iter) / maxGen;
        for (int k = 0; k < Nrand; k++, p++) {
            const int s = ga_select(&r, fit, maxFit, Npop);
            for (int j = 0; j < n; j++) {
                const double mut = spread * (ub[j] - lb[j]) * ga_next(&r);
                Xn[(size_t)p * n + j] = Xp[(size_t)s * n + j] + mut;
            }
        }
        for (int k = 0; k < NeliteMut; k++, p++)
            for (int j = 0; j < n; j++) {
                int e = (int)round(ga_next(&r) * Nelite);
                if (e > Npop - 1) e = Npop - 1;
                const double mut = eliteMutSize * (ub[j] - lb[j]) * ga_next(&r);
                Xn[(size_t)p * n + j] = Xp[(size_t)e * n + j] + mut;
            }
        ga_identical(Xn, Npop, n, lb, ub, ind, &r);
        ga_bounds(Xn, Npop, n, lb, ub, ind, &r);
        ga_evaluate(o, Xn, Fn, ind, Npop, n, nprocs);
        ga_sort(Xn, Fn, Npop, n, Xt, Ft, taken);
        memcpy(F, Fn, sizeof(double) * Npop);
        memcpy(Xp, Xn, sizeof(double) * pn);
        const double Fbest = F[0];
        Nstatic = (Fbest == FbestPrev) ? Nstatic + 1 : 0;
        if (Nstatic > Nstatic_max) break;
        FbestPrev = Fbest;
        iter++;
    }
    res->iters = iter;
    res->evals = o->evals;
    res->fopt = F[0];
    for (int j = 0; j < n; j++) X[j] = Xp[j];
    free(Xp); free(Xn); free(Xt); free(F); free(Fn); free(Ft); free(fit); free(ind); free(taken); free(idx);
    return 0;
}
