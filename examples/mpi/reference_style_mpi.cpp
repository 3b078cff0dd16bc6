// A reference-style MPI program (the shape of the reference's Examples.cpp drivers: MPI_Init,
// then the *_MPI classes, then MPI_Finalize), built against the drop-in headers with <mpi.h>
// on the include path and run as `mpiexec -n P ./reference_style_mpi <case> <out>`.  Nothing in
// it bootstraps a communicator: the *_MPI classes bind MPI_COMM_WORLD themselves
// (include/pnol_mpi_bind.hpp).  Rank 0 writes the results to <out> as hex floats for the tests.
//
// cases:
//   grad      testGradientApproxMultMPI (Examples.cpp:560-590) on the program's OWN host
//             MultiObjective: serial and MPI Jacobians, plus each rank's evaluation count
//   bfgs_mpi  testBFGS_MPI (Examples.cpp:163-188), RosenbrockObject, verbose off
//   lm_mpi    testLMExpMPI (Examples.cpp:128-158), ExpCurveObjective, verbose off
#include <mpi.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "BFGS_with_linesearch_MPI.hpp"
#include "ExampleObjectives.hpp"
#include "LevenbergMarquardtMPI.hpp"

// the program's own host objective: F_k = y_k - (c0 + c1 t + c2 t^2 + c3 t^3), t = k / 10
class UserCubic : public MultiObjective {
  public:
    long evals = 0;
    void objEval(vector<double>& X, vector<double>& F) {
        ++evals;
        for (size_t k = 0; k < F.size(); ++k) {
            const double t = 0.1 * (double)k;
            F[k] = (0.3 + 1.1 * t - 4.3 * t * t + 7.3 * t * t * t) - (X[0] + X[1] * t + X[2] * t * t + X[3] * t * t * t);
        }
    }
};

static void put(FILE* f, const char* key, const std::vector<double>& v) {
    std::fprintf(f, "%s", key);
    for (double x : v) std::fprintf(f, " %a", x);
    std::fprintf(f, "\n");
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int Nprocs = 1, procID = 0;
    MPI_Comm_size(MPI_COMM_WORLD, &Nprocs);
    MPI_Comm_rank(MPI_COMM_WORLD, &procID);
    const std::string which = argc > 1 ? argv[1] : "grad";
    const char* out = argc > 2 ? argv[2] : nullptr;
    FILE* f = (procID == 0 && out) ? std::fopen(out, "w") : nullptr;
    int rc = 0;
    try {
        if (which == "grad") {
            const int Nparam = 4, Ndata = 50;
            vector<double> X(Nparam, 0.1), dX(Nparam, 1e-6);
            UserCubic mObj;
            vector<vector<double>> J(Ndata, vector<double>(Nparam)), Jm(Ndata, vector<double>(Nparam));
            mObj.gradientApproximation(X, dX, J);
            const long serial_evals = mObj.evals;
            mObj.gradientApproximationMPI(X, dX, Jm);
            long mpi_evals = mObj.evals - serial_evals;
            std::vector<long> per(Nprocs);
            MPI_Gather(&mpi_evals, 1, MPI_LONG, per.data(), 1, MPI_LONG, 0, MPI_COMM_WORLD);
            int P = 0, r = 0;
            pnol_comm_size(&P, &r);
            if (f) {
                std::vector<double> js, jm;
                for (int i = 0; i < Ndata; ++i)
                    for (int j = 0; j < Nparam; ++j) {
                        js.push_back(J[i][j]);
                        jm.push_back(Jm[i][j]);
                    }
                std::fprintf(f, "nprocs %d pnol_size %d serial_evals %ld\n", Nprocs, P, serial_evals);
                std::fprintf(f, "rank_evals");
                for (long e : per) std::fprintf(f, " %ld", e);
                std::fprintf(f, "\n");
                put(f, "J", js);
                put(f, "Jmpi", jm);
            }
        } else if (which == "bfgs_mpi") {
            RosenbrockObject obj;
            int Nparam = 10;
            vector<double> X(Nparam, 10);
            BFGS_MPI bfgs;
            bfgs.setObjPtr(obj);
            bfgs.setParams(1e-4, 0.1, 4, 1, 1000, 1e-7, 1e-3, 200, 1e-5, 1e-5, 0, 0);
            double f0, fOpt;
            bfgs.findMin(X, f0, fOpt);
            if (f) {
                put(f, "X", X);
                put(f, "fopt", {fOpt});
                std::fprintf(f, "nprocs %d\n", Nprocs);
            }
        } else if (which == "lm_mpi") {
            int Nparam = 3;
            vector<double> X(Nparam, 0.1), dX(X.size(), 1e-6);
            ExpCurveObjective mObj;
            int Ndata = mObj.getDataSize();
            vector<vector<double>> J(Ndata, vector<double>(Nparam));
            vector<double> F0(Ndata, 0.0), FOpt(Ndata, 0.0);
            mObj.gradientApproximationMPI(X, dX, J);
            LevMarqMPI lmOptimizer;
            lmOptimizer.setObjPtr(mObj);
            lmOptimizer.setParams(0.001, 10, 1e-6, 100, 1e-6, false);
            lmOptimizer.findMin(X, F0, FOpt);
            if (f) {
                put(f, "X", X);
                std::fprintf(f, "nprocs %d\n", Nprocs);
            }
        } else {
            std::fprintf(stderr, "unknown case %s\n", which.c_str());
            rc = 2;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: %s\n", procID, e.what());
        rc = 3;
    }
    if (f) std::fclose(f);
    if (rc) MPI_Abort(MPI_COMM_WORLD, rc);
    MPI_Finalize();
    return 0;
}
