// drivers.cpp -- C ABI entry points that run the C++ drop-in classes end to end on a
// built-in device objective (used by the parity tests and bench.py through ctypes), plus a
// callback-objective FD entry point for the host path of the FD engine.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <stdexcept>
#include <vector>

#include "BFGS_bnd_linesearch.hpp"
#include "BFGS_bnd_linesearch_MPI_SW.hpp"
#include "BFGS_with_bnd_linesearch_MPI.hpp"
#include "BFGS_with_linesearch.hpp"
#include "BFGS_with_linesearch_MPI.hpp"
#include "GeneticAlgorithm.hpp"
#include "GeneticAlgorithmMPI.hpp"
#include "LevenbergMarquardt.hpp"
#include "LevenbergMarquardtMPI.hpp"
#include "device_util.hpp"
#include "scalar_host.hpp"
#include "../pnol_internal.hpp"

using namespace pnol;

namespace {

std::vector<double> download_param(pnol_dobj* d, const double* p, size_t len) {
    std::vector<double> h(len);
    if (len && p) check(pnol_memcpy_d2h(d->ctx, h.data(), p, sizeof(double) * len), "d2h(params)");
    return h;
}

// scalar objective around a pnol_dobj: FD batches on the device; single points and line-search
// batches evaluated with the objective's host formula (identical arithmetic to the device batch)
class DriverScalar : public Objective {
  public:
    DriverScalar(pnol_dobj* d, bool host_only) : d_(d), host_only_(host_only) {
        p0_ = download_param(d, d->p0, d->len0);
        p1_ = download_param(d, d->p1, d->len1);
    }
    double objEval(vector<double>& X) override {
        evals++;
        const double* xp = X.data();
        double f;
        scalar_chains<1>(terms((int)X.size()), &xp, &f);
        return f;
    }
    // Trial points / pools: the host formula by default -- an O(n) sequential sum is a chain of n
    // dependent adds, which a host core runs faster than a GPU lane (tools/eval_probe.py: 36-44 us
    // per point at n = 4096 on the device plus the PCIe round trip, vs ~3.5 us on the host), and
    // the points of a batch run as interleaved chains.  PNOL_DEVICE_POINTS=1 sends every batch to
    // the device (pnol_dobj_eval_batch, the same bits) -- how the tests exercise that path.
    void objEvalBatch(const double* Xs, int nPts, int n, double* f) override {
        if (!host_only_ && device_points() && n == d_->n) {
            evals += nPts;
            check(pnol_dobj_eval_batch(d_->ctx, d_, Xs, nPts, f), "dobj_eval_batch");
            return;
        }
        evals += nPts;
        scalar_batch(terms(n), Xs, nPts, n, f);
    }
    pnol_dobj* deviceObjective(int n) override { return (host_only_ || n != d_->n) ? nullptr : d_; }
    void countEvals(long k) override { evals += k; }
    long evals = 0;

  private:
    ScalarTerms terms(int n) const {
        if (d_->kind != PNOL_OBJ_ROSENBROCK && d_->kind != PNOL_OBJ_POWER && d_->kind != PNOL_OBJ_QUADRATIC)
            throw std::runtime_error("DriverScalar: not a scalar objective");
        if (d_->kind == PNOL_OBJ_QUADRATIC && (p0_.size() < (size_t)n || p1_.size() < (size_t)n))
            throw std::runtime_error("DriverScalar: point longer than the objective's data");
        return ScalarTerms{d_->kind, n, d_->power, p0_.data(), p1_.data()};
    }
    static bool device_points() {
        const char* e = std::getenv("PNOL_DEVICE_POINTS");   // read per call (tests flip it)
        return e && std::atoi(e) != 0;
    }
    pnol_dobj* d_;
    bool host_only_;
    std::vector<double> p0_, p1_;
};

class DriverMulti : public MultiObjective {
  public:
    DriverMulti(pnol_dobj* d, bool host_only) : d_(d), host_only_(host_only) {
        if (host_only) {
            p0_ = download_param(d, d->p0, d->len0);
            p1_ = download_param(d, d->p1, d->len1);
        }
        x_.reset(d->ctx, d->n);
        F_.reset(d->ctx, d->m);
    }
    void objEval(vector<double>& X, vector<double>& F) override {
        evals++;
        if (!host_only_) {
            x_.upload(X);
            check(pnol_dobj_eval_d(d_->ctx, d_, x_.get(), F_.get()), "dobj_eval");
            F_.download(F);
            return;
        }
        const int m = d_->m, n = d_->n;
        switch (d_->kind) {
            case PNOL_OBJ_EXPCURVE:
                for (int k = 0; k < m; ++k) F[k] = p1_[k] - (X[0] * std::exp(X[1] * p0_[k]) + X[2]);
                return;
            case PNOL_OBJ_CUBIC:
                for (int k = 0; k < m; ++k) {
                    const double x = p0_[k];
                    F[k] = p1_[k] - (X[0] * std::pow(x, 3.0) + X[1] * (x * x) + X[2] * x + X[3]);
                }
                return;
            case PNOL_OBJ_LINRES:
                for (int i = 0; i < m; ++i) {
                    double acc = 0.0;
                    for (int k = 0; k < n; ++k) acc = std::fma(p0_[(size_t)i * n + k], X[k], acc);
                    F[i] = acc - p1_[i];
                }
                return;
            default:
                throw std::runtime_error("DriverMulti: not a residual objective");
        }
    }
    pnol_dobj* deviceObjective() override { return host_only_ ? nullptr : d_; }
    void countEvals(long k) override { evals += k; }
    long evals = 0;

  private:
    pnol_dobj* d_;
    bool host_only_;
    std::vector<double> p0_, p1_;
    DevVec x_, F_;
};

class CallbackMulti : public MultiObjective {
  public:
    CallbackMulti(pnol_host_multi_fn fn, void* user, int m) : fn_(fn), user_(user), m_(m) {}
    void objEval(vector<double>& X, vector<double>& F) override { fn_(X.data(), (int)X.size(), F.data(), m_, user_); }

  private:
    pnol_host_multi_fn fn_;
    void* user_;
    int m_;
};

class CallbackScalar : public Objective {
  public:
    CallbackScalar(pnol_host_scalar_fn fn, void* user) : fn_(fn), user_(user) {}
    double objEval(vector<double>& X) override {
        evals++;
        return fn_(X.data(), (int)X.size(), user_);
    }
    long evals = 0;

  private:
    pnol_host_scalar_fn fn_;
    void* user_;
};

template <class F>
int guarded(F&& body) {
    try {
        body();
        return PNOL_OK;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "[pnol_amd] %s\n", e.what());
        return PNOL_ERR_HIP;
    }
}

}  // namespace

extern "C" {

int pnol_run_bfgs(int which, pnol_dobj* obj, int host_eval, const double* p, int np, double* X, int n,
                  const double* Xlb, const double* Xub, pnol_result* res) {
    return pnol_run_bfgs_ex(which, obj, host_eval, p, np, X, n, Xlb, Xub, res, nullptr, 0, nullptr, nullptr);
}

int pnol_run_bfgs_ex(int which, pnol_dobj* obj, int host_eval, const double* p, int np, double* X, int n,
                     const double* Xlb, const double* Xub, pnol_result* res, double* ftrace, int trace_cap,
                     int* ntrace, double* profile) {
    if (profile)
        for (int k = 0; k < 8; ++k) profile[k] = 0.0;
    if (!obj || !p || !X || n <= 0 || !res || trace_cap < 0 || (trace_cap > 0 && !ftrace)) return PNOL_ERR_ARG;
    if (ntrace) *ntrace = 0;
    return guarded([&] {
        std::vector<double> trace;
        int iters = 0;
        DriverScalar o(obj, host_eval != 0);
        std::vector<double> x(X, X + n);
        double f0 = 0, fopt = 0;
        if (which == 0) {
            if (np < 12) throw std::runtime_error("BFGS needs 12 params");
            BFGS b;
            b.setParams(p[0], p[1], p[2], p[3], (int)p[4], p[5], p[6], p[7], p[8], p[9], p[10] != 0, p[11] != 0);
            if (np > 12) b.setUpdateMode((int)p[12]);
            b.setObjPtr(o);
            b.setProfile(profile);
            b.findMin(x, f0, fopt);
            if (profile) iters = (int)profile[0];
        } else if (which == 1) {
            if (np < 12) throw std::runtime_error("BFGS_MPI needs 12 params");
            BFGS_MPI b;
            b.setParams(p[0], p[1], p[2], p[3], (int)p[4], p[5], p[6], p[7], p[8], p[9], p[10] != 0, p[11] != 0);
            if (np > 12) b.setPoolSize((int)p[12]);
            if (np > 13) b.setFixZeroPool(p[13] != 0);
            if (np > 14) b.setUpdateMode((int)p[14]);
            b.setObjPtr(o);
            b.findMin(x, f0, fopt);
        } else if (which == 2) {
            if (np < 15 || !Xlb || !Xub) throw std::runtime_error("BFGS_Bnd needs 15 params and bounds");
            BFGS_Bnd b;
            b.setParams(p[0], p[1], p[2], p[3], p[4], p[5], (int)p[6], p[7], p[8], p[9], p[10], p[11], p[12],
                        p[13] != 0, (int)p[14]);
            if (np > 15) b.setUpdateMode((int)p[15]);
            b.setObjPtr(o);
            if (ftrace || ntrace) b.setFTrace(&trace);
            b.setProfile(profile);
            std::vector<double> lb(Xlb, Xlb + n), ub(Xub, Xub + n);
            b.findMinBnd(x, lb, ub, f0, fopt);
            iters = b.getTotalIter();
        } else if (which == 3) {
            if (np < 14 || !Xlb || !Xub) throw std::runtime_error("BFGSBnd_MPI needs 14 params and bounds");
            BFGSBnd_MPI b;
            b.setParams(p[0], p[1], p[2], p[3], p[4], (int)p[5], p[6], p[7], p[8], p[9], p[10], p[11], p[12] != 0,
                        p[13] != 0);
            if (np > 14) b.setPoolSize((int)p[14]);
            if (np > 15) b.setUpdateMode((int)p[15]);
            b.setObjPtr(o);
            std::vector<double> lb(Xlb, Xlb + n), ub(Xub, Xub + n);
            b.findMinBnd(x, lb, ub, f0, fopt);
        } else if (which == 4) {
            if (np < 15 || !Xlb || !Xub) throw std::runtime_error("BFGS_Bnd_MPI_SW needs 15 params and bounds");
            BFGS_Bnd_MPI_SW b;
            b.setParams(p[0], p[1], p[2], p[3], p[4], p[5], (int)p[6], p[7], p[8], p[9], p[10], p[11], p[12],
                        p[13] != 0, (int)p[14]);
            if (np > 15) b.setPoolSize((int)p[15]);
            if (np > 16) b.setUpdateMode((int)p[16]);
            b.setObjPtr(o);
            std::vector<double> lb(Xlb, Xlb + n), ub(Xub, Xub + n);
            b.findMinBnd(x, lb, ub, f0, fopt);
        } else {
            throw std::runtime_error("unknown BFGS variant");
        }
        for (int i = 0; i < n; ++i) X[i] = x[i];
        res->iters = iters;
        res->evals = o.evals;
        res->f0 = f0;
        res->fopt = fopt;
        for (int k = 0; k < (int)trace.size() && k < trace_cap; ++k) ftrace[k] = trace[k];
        if (ntrace) *ntrace = (int)trace.size();
    });
}

}  // extern "C"

namespace {
// GeneticAlgorithm / GeneticAlgorithmMPI on any Objective; evals: the objective's count
template <class Obj>
void run_ga_on(Obj& o, int which, const double* p, unsigned long long seed, double* X, int n, const double* Xlb,
           const double* Xub, pnol_result* res) {
    std::vector<double> x(X, X + n), lb(Xlb, Xlb + n), ub(Xub, Xub + n);
    double f0 = 0, fopt = 0;
    int gens = 0;
    if (which == 0) {
        GeneticAlgorithm g;
        g.setGAParams((int)p[0], (int)p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9] != 0, false);
        g.setSeed(seed);
        g.setObjPtr(o);
        g.findMinBnd(x, lb, ub, f0, fopt);
        gens = g.getGenerations();
    } else if (which == 1) {
        GeneticAlgorithmMPI g;
        g.setGAParams((int)p[0], (int)p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9] != 0);
        g.setSeed(seed);
        g.setObjPtr(o);
        g.findMinBnd(x, lb, ub, f0, fopt);
        gens = g.getGenerations();
    } else {
        throw std::runtime_error("unknown GA variant");
    }
    for (int i = 0; i < n; ++i) X[i] = x[i];
    res->iters = gens;
    res->evals = o.evals;
    res->f0 = f0;
    res->fopt = fopt;
}
}  // namespace

extern "C" {

int pnol_run_ga(int which, pnol_dobj* obj, int host_eval, const double* p, int np, unsigned long long seed, double* X,
                int n, const double* Xlb, const double* Xub, pnol_result* res) {
    if (!obj || !p || np < 10 || !X || n <= 0 || !Xlb || !Xub || !res) return PNOL_ERR_ARG;
    return guarded([&] {
        DriverScalar o(obj, host_eval != 0);
        run_ga_on(o, which, p, seed, X, n, Xlb, Xub, res);
    });
}

int pnol_host_run_ga(int which, pnol_host_scalar_fn fn, void* user, const double* p, int np, unsigned long long seed,
                     double* X, int n, const double* Xlb, const double* Xub, pnol_result* res) {
    if (!fn || !p || np < 10 || !X || n <= 0 || !Xlb || !Xub || !res) return PNOL_ERR_ARG;
    return guarded([&] {
        CallbackScalar o(fn, user);
        run_ga_on(o, which, p, seed, X, n, Xlb, Xub, res);
    });
}

int pnol_run_levmarq(int which, pnol_dobj* obj, int host_eval, const double* p, double* X, int n, double* F0,
                     double* FOpt, int m, pnol_result* res) {
    return pnol_run_levmarq_ex(which, obj, host_eval, p, X, n, F0, FOpt, m, res, nullptr);
}

int pnol_run_levmarq_ex(int which, pnol_dobj* obj, int host_eval, const double* p, double* X, int n, double* F0,
                        double* FOpt, int m, pnol_result* res, int* steps) {
    if (!obj || !p || !X || !F0 || !FOpt || n <= 0 || m <= 0 || !res) return PNOL_ERR_ARG;
    return guarded([&] {
        DriverMulti o(obj, host_eval != 0);
        std::vector<double> x(X, X + n), f0(m, 0.0), fopt(m, 0.0);
        if (which == 0) {
            LevMarq lm;
            lm.setParams(p[0], p[1], p[2], p[3], p[4], (int)p[5]);
            lm.setObjPtr(o);
            lm.findMin(x, f0, fopt);
            if (steps) { steps[0] = lm.getAcceptedSteps(); steps[1] = lm.getRejectedSteps(); }
        } else {
            LevMarqMPI lm;
            lm.setParams(p[0], p[1], p[2], p[3], p[4], (int)p[5]);
            lm.setObjPtr(o);
            lm.findMin(x, f0, fopt);
            if (steps) { steps[0] = lm.getAcceptedSteps(); steps[1] = lm.getRejectedSteps(); }
        }
        for (int i = 0; i < n; ++i) X[i] = x[i];
        for (int i = 0; i < m; ++i) { F0[i] = f0[i]; FOpt[i] = fopt[i]; }
        res->iters = 0;
        res->evals = o.evals;
        double c0 = 0, c1 = 0;
        for (int i = 0; i < m; ++i) { c0 = c0 + f0[i] * f0[i]; c1 = c1 + fopt[i] * fopt[i]; }
        res->f0 = c0;
        res->fopt = c1;
    });
}

int pnol_host_fd_hessian(pnol_host_scalar_fn fn, void* user, const double* x, const double* h, int n, double* B) {
    if (!fn || !x || !h || !B || n <= 0) return PNOL_ERR_ARG;
    return guarded([&] {
        CallbackScalar o(fn, user);
        std::vector<double> X(x, x + n), dX(h, h + n);
        std::vector<std::vector<double>> Bv;
        o.hessianApproximation(X, dX, Bv);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) B[(size_t)i * n + j] = Bv[i][j];
    });
}

int pnol_host_fd_jacobian(pnol_host_multi_fn fn, void* user, const double* x, const double* h, int n, int m,
                          int sharded, double* J) {
    if (!fn || !x || !h || !J || n <= 0 || m <= 0) return PNOL_ERR_ARG;
    return guarded([&] {
        CallbackMulti o(fn, user, m);
        std::vector<double> X(x, x + n), dX(h, h + n);
        std::vector<std::vector<double>> Jv(m, std::vector<double>(n));
        if (sharded) o.gradientApproximationMPI(X, dX, Jv);
        else o.gradientApproximation(X, dX, Jv);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < n; ++j) J[(size_t)i * n + j] = Jv[i][j];
    });
}

}  // extern "C"
