/*
 * ExampleObjectives.hpp  (MI355X-native PNOL drop-in)
 *
 * The reference's example objectives (Source/ExampleObjectives.hpp) plus the survey's
 * synthetic benchmark objectives.  Host objEval follows the reference
 * arithmetic; squares are written x*x, which is what GCC folds the reference's pow(x,2) to.
 *
 * Every class with a device counterpart evaluates its finite-difference batches on the GPU
 * by default (deviceObjective() != nullptr); useDevice(false) restores pure host
 * evaluation, which is how the parity tests check the device batch against the reference
 * loop.  The device batch of RosenbrockObject, PowerObject(2), QuadraticObjective,
 * CubicObjective and LinearResidualObjective is bitwise equal to the host loop;
 * ExpCurveObjective differs only by the device exp() (<= 1 ulp per term).
 */
#ifndef PNOL_AMD_EXAMPLEOBJECTIVES_HPP_
#define PNOL_AMD_EXAMPLEOBJECTIVES_HPP_

#include <cmath>
#include <stdexcept>
#include <vector>

#include "PNOL_Objective.hpp"

namespace pnol_examples {

// linspace(a, b, N, v) of the reference's utility library: v_i = a + i (b - a) / (N - 1)
inline void linspace(double a, double b, int N, std::vector<double>& v) {
    v.resize(N);
    for (int i = 0; i < N; ++i) v[i] = a + i * (b - a) / (N - 1);
}

// Owns (or borrows) the pnol_dobj behind a device-capable objective.
class DeviceHandle {
  public:
    ~DeviceHandle() { drop(); }
    bool enabled = true;
    pnol_dobj* get(int kind, int n, int m, const std::vector<double>& p0, const std::vector<double>& p1,
                   double power) {
        if (!enabled) return nullptr;
        if (obj_ && n_ == n) return obj_;
        drop();
        pnol_ctx* ctx = nullptr;
        if (pnol_default_ctx(&ctx) != PNOL_OK)
            throw std::runtime_error("pnol_amd: no gfx950 (MI355X) device visible; call useDevice(false) for host evaluation");
        int st = pnol_dobj_create(ctx, kind, n, m, p0.empty() ? nullptr : p0.data(), p0.size(),
                                  p1.empty() ? nullptr : p1.data(), p1.size(), power, &obj_);
        if (st != PNOL_OK) throw std::runtime_error(std::string("pnol_amd: pnol_dobj_create: ") + pnol_status_string(st));
        owned_ = true;
        n_ = n;
        return obj_;
    }
    void attach(pnol_dobj* o) {
        drop();
        obj_ = o;
        owned_ = false;
        if (o) pnol_dobj_info(o, nullptr, &n_, nullptr);
    }
    void drop() {
        if (obj_ && owned_) pnol_dobj_destroy(obj_);
        obj_ = nullptr;
        owned_ = false;
    }
    pnol_dobj* current() const { return enabled ? obj_ : nullptr; }

  private:
    pnol_dobj* obj_ = nullptr;
    bool owned_ = false;
    int n_ = 0;
};

}  // namespace pnol_examples

// ---- scalar objectives -----------------------------------------------------------------

class GoldsteinFunction : public Objective {
  private:
    int evals;

  public:
    double objEval(vector<double>& X) {   // ExampleObjectives.hpp:27-39
        evals++;
        const double x = X[0], y = X[1];
        const double a = x + y + 1, b = 2 * x - 3 * y;
        return (1 + (a * a) * (19 - 14 * x + 3 * (x * x) - 14 * y + 6 * x * y + 3 * (y * y))) *
               (30 + (b * b) * (18 - 32 * x + 12 * (x * x) + 48 * y - 36 * x * y + 27 * (y * y)));
    }
    GoldsteinFunction() : evals(0) {}
    double getEvals() { return evals; }
};

class BoothFunction : public Objective {
  private:
    int evals;

  public:
    double objEval(vector<double>& X) {   // :58-69
        evals++;
        const double a = X[0] + 2 * X[1] - 7, b = 2 * X[0] + X[1] - 5;
        return a * a + b * b;
    }
    BoothFunction() : evals(0) {}
    double getEvals() { return evals; }
};

class RosenbrockObject : public Objective {
  private:
    int evals;
    pnol_examples::DeviceHandle dev;

  public:
    double objEval(vector<double>& X) {   // :87-103
        evals++;
        double value = 0;
        for (size_t k = 0; k + 1 < X.size(); k++) {
            const double t = X[k + 1] - X[k] * X[k];
            const double u = 1 - X[k];
            value = value + (100.0 * (t * t) + u * u);
        }
        return value;
    }
    pnol_dobj* deviceObjective(int n) { return dev.enabled ? dev.get(PNOL_OBJ_ROSENBROCK, n, 0, {}, {}, 2.0) : nullptr; }
    void countEvals(long k) { evals += (int)k; }
    void useDevice(bool on) { dev.enabled = on; }
    RosenbrockObject() : evals(0) {}
    double getEvals() { return evals; }
};

class PowerObject : public Objective {
  private:
    int power;
    pnol_examples::DeviceHandle dev;

  public:
    double objEval(vector<double>& X) {   // :214-224
        double value = 0;
        for (size_t k = 0; k < X.size(); k++) value = value + (power == 2 ? X[k] * X[k] : std::pow(X[k], power));
        return value;
    }
    pnol_dobj* deviceObjective(int n) { return dev.enabled ? dev.get(PNOL_OBJ_POWER, n, 0, {}, {}, (double)power) : nullptr; }
    void countEvals(long k) { (void)k; }
    void useDevice(bool on) { dev.enabled = on; }
    void setPower(int p) { power = p; dev.drop(); }
    int getPower() { return power; }
    PowerObject() : power(2) {}
    ~PowerObject() {}
};

class PowerObjectSlow : public Objective {   // :238-271 (host only: the slowness is its point)
  private:
    int power;

  public:
    double objEval(vector<double>& X) {
        volatile double temp = 0;
        for (int k = 0; k < 100000; k++) temp = std::pow(std::sin(k * 2.3), 1.1);
        (void)temp;
        double value = 0;
        for (size_t k = 0; k < X.size(); k++) value = value + (power == 2 ? X[k] * X[k] : std::pow(X[k], power));
        return value;
    }
    void setPower(int p) { power = p; }
    int getPower() { return power; }
    PowerObjectSlow() : power(2) {}
};

class ExpCurveObjectiveSingle : public Objective {   // :277-320
  private:
    vector<double> xData, yData;

  public:
    double objEval(vector<double>& X) {
        double Fnorm = 0;
        for (size_t k = 0; k < xData.size(); k++) {
            const double func = X[0] * std::exp(X[1] * xData[k]) + X[2];
            const double r = yData[k] - func;
            Fnorm = Fnorm + r * r;
        }
        return Fnorm;
    }
    int getDataSize() { return (int)xData.size(); }
    ExpCurveObjectiveSingle() {
        pnol_examples::linspace(0, 5, 100, xData);
        yData.resize(xData.size());
        for (size_t k = 0; k < xData.size(); k++) yData[k] = 10.2 * std::exp(0.4 * xData[k]) + 0.1;
    }
};

// Synthetic convex quadratic of SURVEY 8(d) cfg 2 / 5 (d_i = 1 + 3u, b_i = 2u - 1, splitmix64):
//   f = sum_i ( (0.5 d_i x_i) x_i - b_i x_i + [i+1<n] (0.25 x_i) x_{i+1} ), i ascending.
class QuadraticObjective : public Objective {
  private:
    vector<double> d, b;
    long evals = 0;
    pnol_examples::DeviceHandle dev;

  public:
    QuadraticObjective(const vector<double>& dIn, const vector<double>& bIn) : d(dIn), b(bIn) {}
    // device-only construction around an existing (e.g. device-generated) objective
    explicit QuadraticObjective(pnol_dobj* o) { dev.attach(o); }
    double objEval(vector<double>& X) {
        if (d.empty()) {   // device-only instance: one-point batch on the device
            double f = 0;
            objEvalBatch(X.data(), 1, (int)X.size(), &f);
            return f;
        }
        evals++;
        const size_t n = X.size();
        double f = 0.0;
        for (size_t i = 0; i < n; ++i) {
            double t = (0.5 * d[i] * X[i]) * X[i] - b[i] * X[i];
            if (i + 1 < n) t = t + (0.25 * X[i]) * X[i + 1];
            f = f + t;
        }
        return f;
    }
    // line-search points and pools of a device-only instance run on the device in one batch
    // (context scratch, one upload and one download: no allocation per call)
    void objEvalBatch(const double* Xs, int nPts, int n, double* f) {
        if (!d.empty()) return Objective::objEvalBatch(Xs, nPts, n, f);
        pnol_ctx* ctx = nullptr;
        if (pnol_default_ctx(&ctx) != PNOL_OK) throw std::runtime_error("pnol_amd: no device");
        evals += nPts;
        if (pnol_dobj_eval_batch(ctx, dev.current(), Xs, nPts, f) != PNOL_OK)
            throw std::runtime_error("pnol_amd: device objective eval failed");
    }
    pnol_dobj* deviceObjective(int n) {
        (void)n;
        if (!dev.enabled) return nullptr;
        if (dev.current()) return dev.current();
        return dev.get(PNOL_OBJ_QUADRATIC, (int)d.size(), 0, d, b, 2.0);
    }
    void countEvals(long k) { evals += k; }
    void useDevice(bool on) { dev.enabled = on; }
    long getEvals() { return evals; }
};

// ---- residual objectives -----------------------------------------------------------------

class ExpCurveObjective : public MultiObjective {   // :113-154
  private:
    vector<double> xData, yData;
    pnol_examples::DeviceHandle dev;

  public:
    void objEval(vector<double>& X, vector<double>& F) {
        for (size_t k = 0; k < xData.size(); k++) {
            const double func = X[0] * std::exp(X[1] * xData[k]) + X[2];
            F[k] = yData[k] - func;
        }
    }
    pnol_dobj* deviceObjective() {
        return dev.enabled ? dev.get(PNOL_OBJ_EXPCURVE, 3, (int)xData.size(), xData, yData, 2.0) : nullptr;
    }
    void useDevice(bool on) { dev.enabled = on; }
    int getDataSize() { return (int)xData.size(); }
    ExpCurveObjective() {
        pnol_examples::linspace(0, 5, 100, xData);
        yData.resize(xData.size());
        for (size_t k = 0; k < xData.size(); k++) yData[k] = 10.2 * std::exp(0.4 * xData[k]) + 0.1;
    }
};

class CubicObjective : public MultiObjective {   // :160-201
  private:
    vector<double> xData, yData;
    pnol_examples::DeviceHandle dev;

  public:
    void objEval(vector<double>& X, vector<double>& F) {
        for (size_t k = 0; k < xData.size(); k++) {
            const double x = xData[k];
            const double func = X[0] * std::pow(x, 3.0) + X[1] * (x * x) + X[2] * x + X[3];
            F[k] = yData[k] - func;
        }
    }
    pnol_dobj* deviceObjective() {
        return dev.enabled ? dev.get(PNOL_OBJ_CUBIC, 4, (int)xData.size(), xData, yData, 2.0) : nullptr;
    }
    void useDevice(bool on) { dev.enabled = on; }
    int getDataSize() { return (int)xData.size(); }
    CubicObjective() {
        pnol_examples::linspace(-5, 5, 100, xData);
        yData.resize(xData.size());
        for (size_t k = 0; k < xData.size(); k++) {
            const double x = xData[k];
            yData[k] = 0.3 * std::pow(x, 3.0) + 1.1 * (x * x) - 4.3 * x + 7.3;
        }
    }
};

// Synthetic dense residual of SURVEY 8(d) cfg 3 / 4: r(x) = A x - y, an fma chain over k.
class LinearResidualObjective : public MultiObjective {
  private:
    vector<double> A, y;   // A row-major m x n
    int n, m;
    pnol_examples::DeviceHandle dev;

  public:
    LinearResidualObjective(const vector<double>& Ain, const vector<double>& yIn, int nIn)
        : A(Ain), y(yIn), n(nIn), m((int)yIn.size()) {}
    // device-only construction around an existing (e.g. synthetic, device-generated) objective
    LinearResidualObjective(pnol_dobj* o, int nIn, int mIn) : n(nIn), m(mIn) { dev.attach(o); }
    void objEval(vector<double>& X, vector<double>& F) {
        if (A.empty()) throw std::runtime_error("LinearResidualObjective: host data not present (device-only instance)");
        for (int i = 0; i < m; ++i) {
            const double* a = A.data() + (size_t)i * n;
            double acc = 0.0;
            for (int k = 0; k < n; ++k) acc = std::fma(a[k], X[k], acc);
            F[i] = acc - y[i];
        }
    }
    pnol_dobj* deviceObjective() {
        if (!dev.enabled) return nullptr;
        if (dev.current()) return dev.current();
        return dev.get(PNOL_OBJ_LINRES, n, m, A, y, 2.0);
    }
    void useDevice(bool on) { dev.enabled = on; }
    int getDataSize() { return m; }
};

#endif /* PNOL_AMD_EXAMPLEOBJECTIVES_HPP_ */
