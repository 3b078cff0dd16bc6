// dense_hessian.cpp -- see dense_hessian.hpp.
#include "dense_hessian.hpp"

#include <cmath>

#include "PNOL_Objective.hpp"

namespace pnol {

DenseInverseHessian::DenseInverseHessian(pnol_ctx* ctx, int n, int mode)
    : ctx_(ctx), n_(n), ld_(even_ld(n)), exact_(mode == 1 || (mode == 0 && n <= PNOL_SEQ_MAX)) {
    D_.reset(ctx, (size_t)n * ld_);
    y_.reset(ctx, n); s_.reset(ctx, n); g_.reset(ctx, n);
    u_.reset(ctx, n); w_.reset(ctx, n); v_.reset(ctx, n);
    if (!exact_) { ps_.reset(ctx, n); pa_.reset(ctx, n); pb_.reset(ctx, n); }
}

void DenseInverseHessian::setIdentity(const std::vector<double>* diagScale) {
    if (diagScale) {
        g_.upload(diagScale->data(), (size_t)n_);
        check(pnol_set_identity_d(ctx_, D_.get(), ld_, n_, g_.get()), "set_identity");
    } else {
        check(pnol_set_identity_d(ctx_, D_.get(), ld_, n_, nullptr), "set_identity");
    }
    pending_ = false;
}

void DenseInverseHessian::setMatrix(const std::vector<std::vector<double>>& D) {
    std::vector<double> h((size_t)n_ * ld_, 0.0);
    for (int i = 0; i < n_; ++i)
        for (int j = 0; j < n_; ++j) h[(size_t)i * ld_ + j] = D[i][j];
    D_.upload(h.data(), h.size());
    pending_ = false;
}

void DenseInverseHessian::setSubmatrixOf(DenseInverseHessian& src, const std::vector<int>& idx) {
    if ((int)idx.size() != n_) throw std::runtime_error("setSubmatrixOf: index count != n");
    src.materialize();
    DevVec di(ctx_, (idx.size() + 1) / 2);   // ints in a double-sized device buffer
    check(pnol_memcpy_h2d(ctx_, di.get(), idx.data(), sizeof(int) * idx.size()), "h2d");
    check(pnol_gather_submatrix_d(ctx_, src.D_.get(), src.ld_, src.n_, reinterpret_cast<const int*>(di.get()), n_,
                                  D_.get(), ld_),
          "gather_submatrix");
    pending_ = false;
}

void DenseInverseHessian::materialize() {
    if (!pending_) return;
    check(pnol_bfgs_pass_d(ctx_, D_.get(), ld_, n_, ps_.get(), pa_.get(), pb_.get(), 1, nullptr, nullptr, u_.get(),
                           w_.get(), v_.get()),
          "bfgs_pass(materialize)");
    pending_ = false;
}

void DenseInverseHessian::getMatrix(std::vector<std::vector<double>>& D) {
    materialize();
    std::vector<double> h((size_t)n_ * ld_);
    D_.download(h.data(), h.size());
    D.assign(n_, std::vector<double>(n_));
    for (int i = 0; i < n_; ++i)
        for (int j = 0; j < n_; ++j) D[i][j] = h[(size_t)i * ld_ + j];
}

void DenseInverseHessian::direction(const std::vector<double>& g, std::vector<double>& p) {
    p.resize(n_);
    g_.upload(g);
    if (!pending_) {
        check(pnol_hg_d(ctx_, D_.get(), ld_, g_.get(), v_.get(), n_), "hg");
        v_.download(p);   // v = -D g
        return;
    }
    // read-only pass over the stored D, then fold the pending correction in algebraically:
    // (D + s a^T + b s^T) g = D g + s (a.g) + b (s.g)
    check(pnol_bfgs_pass_d(ctx_, D_.get(), ld_, n_, nullptr, nullptr, nullptr, 0, nullptr, g_.get(), u_.get(),
                           w_.get(), v_.get()),
          "bfgs_pass(direction)");
    std::vector<double> v(n_);
    v_.download(v);
    const double ag = seq_dot(ha_, g), sg = seq_dot(hs_, g);
    for (int i = 0; i < n_; ++i) p[i] = -(v[i] + hs_[i] * ag + hb_[i] * sg);
}

void DenseInverseHessian::update(const std::vector<double>& y, const std::vector<double>& s,
                                 const std::vector<double>* gnext, std::vector<double>* pnext) {
    if (exact_) {
        y_.upload(y);
        s_.upload(s);
        check(pnol_bfgs_update_exact_d(ctx_, D_.get(), ld_, y_.get(), s_.get(), n_), "bfgs_update_exact");
        if (gnext && pnext) direction(*gnext, *pnext);
        return;
    }
    y_.upload(y);
    if (gnext) g_.upload(*gnext);
    // one pass: fold the pending correction in (write-back) and form D y, D^T y, D g_next
    check(pnol_bfgs_pass_d(ctx_, D_.get(), ld_, n_, pending_ ? ps_.get() : nullptr, pending_ ? pa_.get() : nullptr,
                           pending_ ? pb_.get() : nullptr, pending_ ? 1 : 0, y_.get(), gnext ? g_.get() : nullptr,
                           u_.get(), w_.get(), v_.get()),
          "bfgs_pass(update)");
    std::vector<double> u(n_), w(n_), v;
    u_.download(u);
    w_.download(w);
    if (gnext) { v.resize(n_); v_.download(v); }
    const double rho = 1 / seq_dot(y, s);
    const double beta = seq_dot(y, u);
    const double c = rho * rho * beta + rho;
    hs_ = s;
    ha_.resize(n_);
    hb_.resize(n_);
    for (int j = 0; j < n_; ++j) ha_[j] = c * s[j] - rho * w[j];
    for (int i = 0; i < n_; ++i) hb_[i] = -rho * u[i];
    ps_.upload(hs_);
    pa_.upload(ha_);
    pb_.upload(hb_);
    pending_ = true;
    if (gnext && pnext) {
        const double ag = seq_dot(ha_, *gnext), sg = seq_dot(hs_, *gnext);
        pnext->resize(n_);
        for (int i = 0; i < n_; ++i) (*pnext)[i] = -(v[i] + hs_[i] * ag + hb_[i] * sg);
    }
}

// D0 = inverse of the FD Hessian (initHessFD), column by column on the device
void init_from_fd_hessian(Objective* obj, std::vector<double>& X, double dXHess, DenseInverseHessian& D) {
    const int n = (int)X.size();
    std::vector<double> dXH(n, dXHess);
    std::vector<std::vector<double>> B;
    obj->hessianApproximation(X, dXH, B);
    pnol_ctx* ctx = require_ctx();
    const int ld = even_ld(n);
    std::vector<double> hB((size_t)n * ld, 0.0);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) hB[(size_t)i * ld + j] = B[i][j];
    DevVec dA(ctx, hB.size()), de(ctx, n), dc(ctx, n);
    std::vector<std::vector<double>> Dinv(n, std::vector<double>(n));
    std::vector<double> e(n, 0.0), c(n);
    for (int j = 0; j < n; ++j) {
        // matrixInverse via per-column solves; the solve consumes its matrix
        dA.upload(hB);
        e[j] = 1.0;
        de.upload(e);
        int info = 0;
        check(pnol_solve_d(ctx, dA.get(), ld, de.get(), dc.get(), n, 2, &info), "solve(initHessFD)");
        dc.download(c);
        for (int i = 0; i < n; ++i) Dinv[i][j] = c[i];
        e[j] = 0.0;
    }
    D.setMatrix(Dinv);
}


}  // namespace pnol
