/*
 * pnol_oracle.h -- CPU restatement of the PNOL hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is the parity oracle for the MI355X build.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker / the timed CPU
 * baseline -- never as the thing measured or shipped.
 *
 * Every function restates, loop for loop, the reference algorithm it names (file:line
 * under /root/reference/Source).  The reference's dense linear algebra lives in the
 * un-vendored UtilityFunctionLibrary; the orc_util_* functions
 * restate it with the semantics pinned in SURVEY.md sec. 8(c): sequential summation
 * from 0.0, Gaussian elimination with partial pivoting on a copy, first index of an
 * extremum.  That layer is "parity unpinned" (no reference test holds its outputs);
 * the algorithms above it are pinned to the converged vectors the survey recorded from
 * the reference (tests/golden/, tests/test_oracle_golden.py).
 *
 * Arithmetic contract: compiled with -ffp-contract=off, squares written x*x (what GCC
 * folds the reference's pow(x,2) to), every other pow/exp/sqrt a libm call.
 */
#ifndef PNOL_ORACLE_H_
#define PNOL_ORACLE_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- objectives (ExampleObjectives.hpp + the survey's synthetic configs) ---- */
enum orc_obj_kind {
    ORC_ROSENBROCK = 0,   /* ExampleObjectives.hpp:79-111 */
    ORC_POWER = 1,        /* :206-234, params[0] = power */
    ORC_GOLDSTEIN = 2,    /* :19-47 */
    ORC_BOOTH = 3,        /* :50-77 */
    ORC_QUADRATIC = 4,    /* SURVEY 8(d) cfg 2/5: params = d[n], b[n] */
    ORC_EXPCURVE = 10,    /* multi, :113-154, params = xData[m], yData[m] */
    ORC_CUBIC = 11,       /* multi, :160-201, params = xData[m], yData[m] */
    ORC_LINRES = 12       /* multi, SURVEY 8(d) cfg 3/4: r = A x - y; params = A[m*n] row-major, y[m] */
};

typedef struct {
    int kind;
    int n;              /* parameters */
    int m;              /* residuals (multi objectives) */
    const double* p0;   /* kind-specific data (see enum) */
    const double* p1;
    double power;
    long evals;         /* objEval counter, as ExampleObjectives keep `evals` */
} orc_objective;

double orc_obj_eval(orc_objective* o, const double* x);                 /* Objective::objEval */
void   orc_obj_eval_multi(orc_objective* o, const double* x, double* F); /* MultiObjective::objEval */

/* ---- utility layer restatement (UtilityFunctionLibrary, absent) ---- */
double orc_util_dot(const double* a, const double* b, int n);
double orc_util_norm2(const double* a, int n);
void   orc_util_matvec(const double* A, const double* x, double* y, int rows, int cols); /* y=A x */
void   orc_util_matmul(const double* A, const double* B, double* C, int n, int k, int m); /* C=A B */
int    orc_util_lusolve(const double* A, const double* b, double* x, int n);
int    orc_util_matinv(const double* A, double* Ainv, int n);
void   orc_util_linspace(double a, double b, int N, double* v);

/* ---- FD engine, PNOL_Objective.cpp ---- */
void orc_fd_gradient(orc_objective* o, const double* X, const double* dX, double* dFdX, int n);   /* :12-34 */
void orc_fd_gradient_sharded(orc_objective* o, const double* X, const double* dX, double* dFdX,
                             int n, int nprocs);                                                 /* :88-159 */
void orc_fd_jacobian(orc_objective* o, const double* X, const double* dX, double* J, int n, int m); /* :165-197, J m x n row-major */
void orc_fd_jacobian_sharded(orc_objective* o, const double* X, const double* dX, double* J,
                             int n, int m, int nprocs);                                          /* :202-299 */
void orc_fd_hessian(orc_objective* o, const double* X, const double* dX, double* B, int n);      /* :38-85 */
double orc_obj_eval_recur(orc_objective* o, const double* Xr, const double* constX,
                          const unsigned char* constInd, int nfull);                             /* :303-333 */
void orc_fd_gradient_recur(orc_objective* o, const double* X, const double* dX, double* dFdX, int nr,
                           const double* constX, const unsigned char* constInd, int nfull);      /* :337-360 */

/* ---- BFGS inverse-Hessian update, BFGS_with_linesearch.cpp:389-432 ---- */
void orc_update_hessian_inv(double* D, const double* y, const double* s, int n);      /* reference O(n^3) form */
void orc_update_hessian_inv_rank2(double* D, const double* y, const double* s, int n); /* O(n^2) restatement */

/* ---- algorithms ---- */
typedef struct {   /* BFGS::setParams, BFGS_with_linesearch.hpp:62 */
    double c1, c2, dalpha, alphaGuess; int maxIterLineSearch;
    double dXGrad, dXHess; double maxIter; double xMinDiff, minGrad2Norm; int initHessFD; int verbose;
} orc_bfgs_params;

typedef struct {
    int iters; long evals; double f0, fopt;
} orc_result;

/* BFGS::findMin, BFGS_with_linesearch.cpp:12-139 ; trace (optional) gets X after every iteration */
int orc_bfgs_findmin(orc_objective* o, const orc_bfgs_params* prm, double* X, int n, orc_result* res,
                     double* trace, int trace_cap);
int orc_bfgs_findmin_ex(orc_objective* o, const orc_bfgs_params* prm, double* X, int n, orc_result* res,
                        double* trace, int trace_cap, int rank2);   /* rank2: O(n^2) update form */

typedef struct {   /* BFGS_MPI::setParams, BFGS_with_linesearch_MPI.hpp:64 */
    double c1, c2, maxAlphaMult, alphaGuess; int maxIterLineSearch;
    double dXGrad, dXHess; double maxIter; double xMinDiff, minGrad2Norm; int initHessFD; int verbose;
} orc_bfgs_mpi_params;
/* BFGS_MPI::findMin, BFGS_with_linesearch_MPI.cpp:12-142, with Npool = nprocs (:235) */
int orc_bfgs_mpi_findmin(orc_objective* o, const orc_bfgs_mpi_params* prm, int nprocs, double* X, int n,
                         orc_result* res);

typedef struct {   /* LevMarq::setParams, LevenbergMarquardt.hpp:41 */
    double lambda0, lambdaFactor, dXGrad; double maxIter; double xMinDiff; int verbose;
} orc_lm_params;
/* LevMarq::findMin, LevenbergMarquardt.cpp:11-167 (LevMarqMPI is identical up to the FD sharding) */
int orc_lm_findmin(orc_objective* o, const orc_lm_params* prm, double* X, int n, double* F0, double* FOpt,
                   int m, orc_result* res, double* trace, int trace_cap);
/* orc_lm_findmin with its independent work over OpenMP threads (pnol_oracle_par.c, liboracle_par.so
 * only): bitwise the same results; X / chiSq / lambda recorded after every trip */
int orc_lm_findmin_par(orc_objective* o, const orc_lm_params* prm, double* X, int n, double* F0, double* FOpt, int m,
                       orc_result* res, double* trace_x, double* trace_chi, double* trace_lambda, int trace_cap);
/* one LM loop trip's linear algebra, LevenbergMarquardt.cpp:55-83: J -> JTJ, A, rhs, sigma */
int orc_lm_step(const double* J, const double* F, double lambda, int m, int n,
                double* JTJ, double* A, double* rhs, double* sigma);

typedef struct {   /* BFGS_Bnd::setParams, BFGS_bnd_linesearch.hpp:80 */
    double c1, c2, dalpha, alphaGuess, alphaTol, alphaMult; int maxIterLineSearch;
    double bndTol, dXGrad, dXHess; double maxIter; double xMinDiff, minGrad2Norm; int initHessFD; int verbose;
} orc_bfgs_bnd_params;
/* BFGS_Bnd::findMinBnd, BFGS_bnd_linesearch.cpp:15-113 */
int orc_bfgs_bnd_findmin(orc_objective* o, const orc_bfgs_bnd_params* prm, double* X, const double* Xlb,
                         const double* Xub, int n, orc_result* res);
/* the same with the rank-2 O(n^2) form of updateHessianInv when rank2 != 0 (tractable at large n;
 * the reference form sums in another order), F after every iteration in ftrace (nullable) and
 * the deepest boundaryAssessment recursion in max_depth (nullable) */
int orc_bfgs_bnd_findmin_ex(orc_objective* o, const orc_bfgs_bnd_params* prm, double* X, const double* Xlb,
                            const double* Xub, int n, orc_result* res, int rank2, double* ftrace, int trace_cap,
                            int* max_depth);
/* BFGS_Bnd_MPI_SW::findMinBnd, BFGS_bnd_linesearch_MPI_SW.cpp:12-113 (same setParams as BFGS_Bnd;
 * Nprocs = procs: pools of procs + 1 / procs + 2) */
int orc_bfgs_bnd_mpi_sw_findmin(orc_objective* o, const orc_bfgs_bnd_params* prm, int procs, double* X,
                                const double* Xlb, const double* Xub, int n, orc_result* res);
typedef struct {   /* BFGSBnd_MPI::setParams, BFGS_with_bnd_linesearch_MPI.hpp:79 */
    double c1, c2, alphaMin, maxAlphaMult, alphaGuess; int maxIterLineSearch;
    double dXGrad, dXHess; double maxIter; double xMinDiff, minGrad2Norm, FStepTolerance; int initHessFD;
    int verbose;
} orc_bfgs_bnd_mpi_params;
/* BFGSBnd_MPI::findMinBnd, BFGS_with_bnd_linsearch_MPI.cpp:14-81 (Npool = npool, FD over nprocs) */
int orc_bfgs_bnd_mpi_findmin(orc_objective* o, const orc_bfgs_bnd_mpi_params* prm, int npool, int nprocs,
                             double* X, const double* Xlb, const double* Xub, int n, orc_result* res);
/* checkAlphaPoolBnd, BFGS_with_bnd_linsearch_MPI.cpp:711-743 */
void orc_check_alpha_pool_bnd(int* bndIndicator, double* alphaPool, int npool, const double* X, const double* Xlb,
                              const double* Xub, const double* p, int n);
double orc_compute_alpha_bnd(const double* X, const double* Xlb, const double* Xub, const double* p, int n);
void orc_check_box_bounds(double* X, const double* Xlb, const double* Xub, int n);

/* ---- deterministic synthetic inputs: splitmix64, seed 0x5EED2018 ---- */
double orc_splitmix_u01(unsigned long long seed, unsigned long long idx); /* idx-th draw in [0,1) */
void orc_make_quadratic(unsigned long long seed, int n, double* d, double* b);
void orc_make_linres(unsigned long long seed, int m, int n, double* A, double* xstar, double* y);
/* ExpCurveObjective / CubicObjective constructors, ExampleObjectives.hpp:139-147, :186-193 */
void orc_make_expcurve_data(int m, double* xData, double* yData);
void orc_make_cubic_data(int m, double* xData, double* yData);

#ifdef __cplusplus
}
#endif
/* GeneticAlgorithm / GeneticAlgorithmMPI (GeneticAlgorithm.cpp:12-436, GeneticAlgorithmMPI.cpp:12-414):
 * prm = Npop, maxGenerations, eliteFrac, crossFrac, eliteMutationFrac, mutationSize,
 * eliteMutationSize, initialPopScaling, NstaticGenerations; nprocs 0 = the serial class. */
int orc_ga_findmin(orc_objective* o, const double* prm, unsigned long long seed, int nprocs, double* X,
                   const double* lb, const double* ub, int n, orc_result* res);

#endif
