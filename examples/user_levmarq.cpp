// user_levmarq.cpp -- a PNOL user program, written against the reference's headers as a user
// of briandaniel/ParallelNonlinearOptimizationLibrary would (LevenbergMarquardt.hpp,
// PNOL_Objective.hpp), built with INTEGRATION.md's line and linked to libpnol_amd.so.
//
// The residual is the user's own MultiObjective -- not a built-in device objective -- so the FD
// Jacobian is evaluated on the host through objEvalBatch, which this class overrides to spread
// each batch of points over host threads (each point's arithmetic is unchanged, so the results
// are the same bits in any thread count).  J^T J, the Marquardt diagonal, -J^T F and the damped
// solve run on the GPU inside LevMarq::findMin.
//
//   user_levmarq <in.bin> <out.bin>
//   in.bin : int32 m, n, threads; double lambda0, lambdaFactor, dXGrad, maxIter, xMinDiff;
//            A (m x n, row-major), y (m), x0 (n)
//   out.bin: double X (n), chi^2(F0), chi^2(FOpt); int64 objEval calls, batches
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "LevenbergMarquardt.hpp"
#include "PNOL_Objective.hpp"

// r_i(x) = sum_k A_ik x_k - y_i, accumulated as one fma chain over k (the oracle's LINRES form)
class DenseResidual : public MultiObjective {
  public:
    DenseResidual(std::vector<double> A, std::vector<double> y, int n, int threads)
        : A_(std::move(A)), y_(std::move(y)), n_(n), m_((int)y_.size()), threads_(threads) {}

    void objEval(vector<double>& X, vector<double>& F) override {
        ++evals;
        residual(X.data(), F.data());
    }

    // the batch hook: the points of one FD batch (or the LM trial point) on host threads
    void objEvalBatch(const double* Xs, int nPts, int n, double* F, int m) override {
        (void)n;
        ++batches;
        evals += nPts;
        std::atomic<int> next{0};
        auto work = [&] {
            for (int k = next++; k < nPts; k = next++) residual(Xs + (size_t)k * n_, F + (size_t)k * m);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < threads_ && t < nPts; ++t) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();
    }

    long evals = 0, batches = 0;

  private:
    void residual(const double* x, double* F) const {
        for (int i = 0; i < m_; ++i) {
            const double* a = A_.data() + (size_t)i * n_;
            double acc = 0.0;
            for (int k = 0; k < n_; ++k) acc = std::fma(a[k], x[k], acc);
            F[i] = acc - y_[i];
        }
    }
    std::vector<double> A_, y_;
    int n_, m_, threads_;
};

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
        return 2;
    }
    FILE* in = std::fopen(argv[1], "rb");
    if (!in) return 2;
    int hdr[3];
    double prm[5];
    if (std::fread(hdr, sizeof(int), 3, in) != 3 || std::fread(prm, sizeof(double), 5, in) != 5) return 2;
    const int m = hdr[0], n = hdr[1], threads = hdr[2];
    std::vector<double> A((size_t)m * n), y(m), X(n);
    if (std::fread(A.data(), sizeof(double), A.size(), in) != A.size() ||
        std::fread(y.data(), sizeof(double), y.size(), in) != y.size() ||
        std::fread(X.data(), sizeof(double), X.size(), in) != X.size())
        return 2;
    std::fclose(in);

    DenseResidual obj(A, y, n, threads);
    LevMarq lm;   // LevenbergMarquardt.hpp:41 -- the reference's setParams order
    lm.setParams(prm[0], prm[1], prm[2], prm[3], prm[4], -1);
    lm.setObjPtr(obj);
    std::vector<double> F0(m, 0.0), FOpt(m, 0.0);   // pre-sized: m = F0.size() (LevenbergMarquardt.cpp:19)
    lm.findMin(X, F0, FOpt);

    double c0 = 0, c1 = 0;
    for (int i = 0; i < m; ++i) { c0 += F0[i] * F0[i]; c1 += FOpt[i] * FOpt[i]; }
    FILE* out = std::fopen(argv[2], "wb");
    if (!out) return 2;
    std::fwrite(X.data(), sizeof(double), n, out);
    std::fwrite(&c0, sizeof(double), 1, out);
    std::fwrite(&c1, sizeof(double), 1, out);
    long long counts[2] = {obj.evals, obj.batches};
    std::fwrite(counts, sizeof(long long), 2, out);
    std::fclose(out);
    return 0;
}
