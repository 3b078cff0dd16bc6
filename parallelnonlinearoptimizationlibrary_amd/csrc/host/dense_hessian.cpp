// dense_hessian.cpp -- see dense_hessian.hpp.
#include "dense_hessian.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "PNOL_Objective.hpp"

namespace pnol {

static bool shard_enabled() {
    const char* e = std::getenv("PNOL_BFGS_SHARD");
    return !e || std::atoi(e) != 0;
}

void DenseInverseHessian::init(int mode, bool shard) {
    exact_ = mode == 1 || (mode == 0 && n_ <= PNOL_SEQ_MAX);
    rb_ = 0;
    rc_ = n_;
    if (shard && !exact_ && comm_size() > 1 && shard_enabled()) {
        sharded_ = true;
        check(pnol_bfgs_rows(n_, comm_size(), comm_rank(), &rb_, &rc_), "bfgs_rows");
    }
}

DenseInverseHessian::DenseInverseHessian(pnol_ctx* ctx, int n, int mode, bool shard)
    : ctx_(ctx), n_(n), ld_(even_ld(n)) {
    init(mode, shard);
    cap_ = (size_t)(rc_ > 0 ? rc_ : 1) * ld_;
    D_.reset(ctx, cap_);
    Dp_ = D_.get();
    io_.reset(ctx_, (size_t)kSlots * n_);
    iop_ = io_.get();
    dev_ok_ = false;   // contents undefined until setIdentity / setMatrix
}

DenseInverseHessian::DenseInverseHessian(DenseInverseHessian& parent, int n, int mode, bool shard)
    : ctx_(parent.ctx_), n_(n), ld_(even_ld(n)) {
    init(mode, shard);
    const size_t need = (size_t)(rc_ > 0 ? rc_ : 1) * ld_;
    if (need <= parent.cap_ && parent.Dp_) {
        Dp_ = parent.Dp_;
        cap_ = parent.cap_;
        parent.clobbered_ = true;
    } else {
        cap_ = need;
        D_.reset(ctx_, cap_);
        Dp_ = D_.get();
    }
    if (n_ <= parent.n_ && parent.iop_) {
        iop_ = parent.iop_;
    } else {
        io_.reset(ctx_, (size_t)kSlots * n_);
        iop_ = io_.get();
    }
    dev_ok_ = false;
    // the parent's host state is forfeit too: release its pending correction while the
    // reduced problem runs (each recursion level would otherwise hold three n-vectors)
    parent.clobbered_ = true;
    parent.pending_ = parent.pend_dev_ = false;
    parent.ident_ = parent.dev_ok_ = false;
    for (std::vector<double>* v : {&parent.hs_, &parent.ha_, &parent.hb_, &parent.hscale_})
        std::vector<double>().swap(*v);
}

const double* DenseInverseHessian::deviceScale() {
    if (hscale_.empty()) return nullptr;
    if (!dscale_ok_) {
        if (dscale_.size() < (size_t)n_) dscale_.reset(ctx_, n_);
        dscale_.upload(hscale_.data(), (size_t)n_);
        dscale_ok_ = true;
    }
    return dscale_.get();
}

void DenseInverseHessian::setIdentity(const std::vector<double>* diagScale) {
    // lazy: nothing is written until something has to read D itself (ensureDevice)
    if (diagScale) hscale_.assign(diagScale->begin(), diagScale->begin() + n_);
    else hscale_.clear();
    dscale_ok_ = false;
    ident_ = true;
    dev_ok_ = false;
    pending_ = false;
    clobbered_ = false;
}

void DenseInverseHessian::ensureDevice() {
    if (clobbered_) throw std::runtime_error("DenseInverseHessian: D used while lent to a reduced problem");
    if (dev_ok_) return;
    if (!ident_) throw std::runtime_error("DenseInverseHessian: D used before it was set");
    const double* scale = deviceScale();
    if (sharded_) check(pnol_set_identity_rows_d(ctx_, Dp_, ld_, n_, scale), "set_identity");
    else check(pnol_set_identity_d(ctx_, Dp_, ld_, n_, scale), "set_identity");
    dev_ok_ = true;
}

// the diagonal shortcut is exact only for finite operands (0 * inf poisons a device row sum)
bool DenseInverseHessian::identFinite(const std::vector<double>* a, const std::vector<double>* b) const {
    for (const std::vector<double>* v : {a, b})
        if (v)
            for (int i = 0; i < n_; ++i)
                if (!std::isfinite((*v)[i])) return false;
    for (double x : hscale_)
        if (!std::isfinite(x)) return false;
    return true;
}

void DenseInverseHessian::setMatrix(const std::vector<std::vector<double>>& D) {
    std::vector<double> h((size_t)(rc_ > 0 ? rc_ : 1) * ld_, 0.0);
    for (int i = 0; i < rc_; ++i)
        for (int j = 0; j < n_; ++j) h[(size_t)i * ld_ + j] = D[rb_ + i][j];
    check(pnol_memcpy_h2d(ctx_, Dp_, h.data(), sizeof(double) * h.size()), "h2d");
    pending_ = false;
    ident_ = false;
    dev_ok_ = true;
    clobbered_ = false;
}

void DenseInverseHessian::setSubmatrixOf(DenseInverseHessian& src, const std::vector<int>& idx) {
    if ((int)idx.size() != n_) throw std::runtime_error("setSubmatrixOf: index count != n");
    if (src.ident_ && !src.pending_) {
        // a diagonal D's free-free block is the diagonal of the kept coordinates
        if (src.hscale_.empty()) {
            setIdentity();
        } else {
            std::vector<double> sub(n_);
            for (int a = 0; a < n_; ++a) sub[a] = src.hscale_[idx[a]];
            setIdentity(&sub);
        }
        return;
    }
    if (sharded_ && src.sharded_) {
        // the boundary recursion of the row-sharded variants: kept rows move to their new
        // owners device to device
        src.materialize();
        src.ensureDevice();
        check(pnol_gather_submatrix_mpi_d(ctx_, src.Dp_, src.ld_, src.n_, idx.data(), n_, Dp_, ld_),
              "gather_submatrix_mpi");
        pending_ = false;
        ident_ = false;
        dev_ok_ = true;
        clobbered_ = false;
        return;
    }
    if (sharded_ || src.sharded_) {
        // mixed sharding (not used by the drop-ins): through the host
        std::vector<std::vector<double>> full, sub(n_, std::vector<double>(n_));
        src.getMatrix(full);
        for (int a = 0; a < n_; ++a)
            for (int b = 0; b < n_; ++b) sub[a][b] = full[idx[a]][idx[b]];
        setMatrix(sub);
        return;
    }
    src.materialize();
    src.ensureDevice();
    DevVec di(ctx_, (idx.size() + 1) / 2);   // ints in a double-sized device buffer
    check(pnol_memcpy_h2d(ctx_, di.get(), idx.data(), sizeof(int) * idx.size()), "h2d");
    check(pnol_gather_submatrix_d(ctx_, src.Dp_, src.ld_, src.n_, reinterpret_cast<const int*>(di.get()), n_, Dp_,
                                  ld_),
          "gather_submatrix");
    pending_ = false;
    ident_ = false;
    dev_ok_ = true;
    clobbered_ = false;
}

void DenseInverseHessian::uploadPending() {
    if (!pending_ || pend_dev_) return;
    std::vector<double> sab(3 * (size_t)n_);   // s_p | a_p | b_p in one copy
    std::copy(hs_.begin(), hs_.end(), sab.begin());
    std::copy(ha_.begin(), ha_.end(), sab.begin() + n_);
    std::copy(hb_.begin(), hb_.end(), sab.begin() + 2 * n_);
    up(kPS, sab.data(), sab.size());
    pend_dev_ = true;
}

int DenseInverseHessian::pass(const double* sp, const double* ap, const double* bp, int wb, const double* y,
                              const double* g, double* u, double* w, double* v) {
    if (sp) uploadPending();
    ensureDevice();
    if (sharded_) return pnol_bfgs_pass_mpi_d(ctx_, Dp_, ld_, n_, sp, ap, bp, wb, y, g, u, w, v);
    return pnol_bfgs_pass_d(ctx_, Dp_, ld_, n_, sp, ap, bp, wb, y, g, u, w, v);
}

// fold the pending correction into a stored diagonal without reading it
int DenseInverseHessian::passIdent(const double* y, const double* g, double* u, double* w, double* v) {
    if (clobbered_) throw std::runtime_error("DenseInverseHessian: D used while lent to a reduced problem");
    uploadPending();
    const double* scale = deviceScale();
    int st = sharded_ ? pnol_bfgs_pass_ident_mpi_d(ctx_, Dp_, ld_, n_, scale, slot(kPS), slot(kPA), slot(kPB), y, g, u, w, v)
                      : pnol_bfgs_pass_ident_d(ctx_, Dp_, ld_, n_, scale, slot(kPS), slot(kPA), slot(kPB), y, g, u, w, v);
    ident_ = false;
    dev_ok_ = true;
    return st;
}

void DenseInverseHessian::materialize() {
    if (!pending_) return;
    if (ident_) check(passIdent(nullptr, nullptr, slot(kU), slot(kW), slot(kV)), "bfgs_pass(materialize)");
    else
        check(pass(slot(kPS), slot(kPA), slot(kPB), 1, nullptr, nullptr, slot(kU), slot(kW), slot(kV)),
              "bfgs_pass(materialize)");
    pending_ = false;
}

void DenseInverseHessian::getMatrix(std::vector<std::vector<double>>& D) {
    materialize();
    ensureDevice();
    D.assign(n_, std::vector<double>(n_));
    if (!sharded_) {
        std::vector<double> h((size_t)n_ * ld_);
        check(pnol_memcpy_d2h(ctx_, h.data(), Dp_, sizeof(double) * h.size()), "d2h");
        for (int i = 0; i < n_; ++i)
            for (int j = 0; j < n_; ++j) D[i][j] = h[(size_t)i * ld_ + j];
        return;
    }
    // every rank's rows, padded to the shard size, through the host allgather
    int b0 = 0, per = 0;
    check(pnol_bfgs_rows(n_, comm_size(), 0, &b0, &per), "bfgs_rows");
    std::vector<double> mine((size_t)per * ld_, 0.0), all((size_t)per * ld_ * comm_size());
    if (rc_ > 0) check(pnol_memcpy_d2h(ctx_, mine.data(), Dp_, sizeof(double) * (size_t)rc_ * ld_), "d2h");
    check(comm_allgather_host(ctx_, mine.data(), all.data(), mine.size()), "allgather(D)");
    for (int i = 0; i < n_; ++i)
        for (int j = 0; j < n_; ++j) D[i][j] = all[(size_t)i * ld_ + j];   // rank r's rows start at r * per
}

void DenseInverseHessian::direction(const std::vector<double>& g, std::vector<double>& p) {
    p.resize(n_);
    if (ident_ && !pending_ && identFinite(nullptr, nullptr)) {
        // a stored diagonal, nothing pending: p_i = -(0.0 + d_i g_i) in one pass (a non-finite
        // g_i sends the whole direction to the device path below, which rewrites p)
        const double* gp = g.data();
        const double* scp = hscale_.empty() ? nullptr : hscale_.data();
        double* pp = p.data();
        bool fin = true;
        for (int i = 0; i < n_; ++i) {
            fin = fin && std::isfinite(gp[i]);
            pp[i] = -(0.0 + (scp ? scp[i] : 1.0) * gp[i]);
        }
        if (fin) return;
    }
    if (ident_ && identFinite(&g, nullptr)) {
        // D g for a stored diagonal: the one nonzero term of each row sum, 0.0 + d_i g_i (the
        // device sums start from +0, so an exact zero product comes out +0)
        std::vector<double> v(n_);
        for (int i = 0; i < n_; ++i) v[i] = 0.0 + sc(i) * g[i];
        if (!pending_) {
            for (int i = 0; i < n_; ++i) p[i] = -v[i];
            return;
        }
        double ag, sg;
        seq_dot2(ha_, g, hs_, g, ag, sg);
        for (int i = 0; i < n_; ++i) p[i] = -(v[i] + hs_[i] * ag + hb_[i] * sg);
        return;
    }
    up(kG, g.data(), (size_t)n_);
    if (!pending_) {
        ensureDevice();
        if (sharded_) check(pnol_hg_mpi_d(ctx_, Dp_, ld_, slot(kG), slot(kV), n_), "hg");
        else check(pnol_hg_d(ctx_, Dp_, ld_, slot(kG), slot(kV), n_), "hg");
        down(kV, p.data(), (size_t)n_);   // v = -D g
        return;
    }
    // read-only pass over the stored D, then fold the pending correction in algebraically:
    // (D + s a^T + b s^T) g = D g + s (a.g) + b (s.g)
    check(pass(nullptr, nullptr, nullptr, 0, nullptr, slot(kG), slot(kU), slot(kW), slot(kV)),
          "bfgs_pass(direction)");
    std::vector<double> v(n_);
    down(kV, v.data(), (size_t)n_);
    double ag, sg;
    seq_dot2(ha_, g, hs_, g, ag, sg);
    for (int i = 0; i < n_; ++i) p[i] = -(v[i] + hs_[i] * ag + hb_[i] * sg);
}

void DenseInverseHessian::update(const std::vector<double>& y, const std::vector<double>& s,
                                 const std::vector<double>* gnext, std::vector<double>* pnext) {
    if (exact_) {
        ensureDevice();
        std::vector<double> ys(2 * (size_t)n_);
        std::copy(y.begin(), y.end(), ys.begin());
        std::copy(s.begin(), s.end(), ys.begin() + n_);
        up(kY, ys.data(), ys.size());   // y | s
        check(pnol_bfgs_update_exact_d(ctx_, Dp_, ld_, slot(kY), slot(kG), n_), "bfgs_update_exact");
        ident_ = false;
        if (gnext && pnext) direction(*gnext, *pnext);
        return;
    }
    if (ident_ && !pending_ && updateIdentFused(y, s, gnext, pnext)) return;
    std::vector<double> u(n_), w(n_), v;
    if (gnext) v.resize(n_);
    if (ident_ && !pending_ && identFinite(&y, gnext)) {
        // u = D y, w = D^T y, v = D g of a stored diagonal, exactly as the pass sums them
        for (int i = 0; i < n_; ++i) u[i] = w[i] = 0.0 + sc(i) * y[i];
        if (gnext)
            for (int i = 0; i < n_; ++i) v[i] = 0.0 + sc(i) * (*gnext)[i];
    } else {
        std::vector<double> yg((gnext ? 2 : 1) * (size_t)n_);
        std::copy(y.begin(), y.end(), yg.begin());
        if (gnext) std::copy(gnext->begin(), gnext->end(), yg.begin() + n_);
        up(kY, yg.data(), yg.size());   // y | g
        // one pass: fold the pending correction in (write-back) and form D y, D^T y, D g_next
        if (pending_ && ident_)
            check(passIdent(slot(kY), gnext ? slot(kG) : nullptr, slot(kU), slot(kW), slot(kV)), "bfgs_pass(update)");
        else
            check(pass(pending_ ? slot(kPS) : nullptr, pending_ ? slot(kPA) : nullptr, pending_ ? slot(kPB) : nullptr,
                       pending_ ? 1 : 0, slot(kY), gnext ? slot(kG) : nullptr, slot(kU), slot(kW), slot(kV)),
                  "bfgs_pass(update)");
        if (pending_) ident_ = false;
        std::vector<double> uwv((gnext ? 3 : 2) * (size_t)n_);
        down(kU, uwv.data(), uwv.size());   // u | w | v
        std::copy(uwv.begin(), uwv.begin() + n_, u.begin());
        std::copy(uwv.begin() + n_, uwv.begin() + 2 * n_, w.begin());
        if (gnext) std::copy(uwv.begin() + 2 * n_, uwv.end(), v.begin());
    }
    double ys, beta;
    seq_dot2(y, s, y, u, ys, beta);
    const double rho = 1 / ys;
    const double c = rho * rho * beta + rho;
    hs_ = s;
    ha_.resize(n_);
    hb_.resize(n_);
    for (int j = 0; j < n_; ++j) ha_[j] = c * s[j] - rho * w[j];
    for (int i = 0; i < n_; ++i) hb_[i] = -rho * u[i];
    pending_ = true;
    pend_dev_ = false;
    if (gnext && pnext) {
        double ag, sg;
        seq_dot2(ha_, *gnext, hs_, *gnext, ag, sg);
        pnext->resize(n_);
        for (int i = 0; i < n_; ++i) (*pnext)[i] = -(v[i] + hs_[i] * ag + hb_[i] * sg);
    }
}

// update() from a stored diagonal with no pending correction, in three passes over the
// vectors instead of one per quantity: (1) u = w = D y and v = D g_next (0.0 + d_i y_i, as the
// device sums give them) with the chains y.s and y.u; (2) the new pending correction
// (s, a = c s - rho w, b = -rho u) with the chains a.g and s.g; (3) p_next.  Every chain adds
// in index order from 0.0 exactly as seq_dot, so the bits are update()'s general path's.
// false (nothing changed) on a non-finite operand: the device path handles those.
bool DenseInverseHessian::updateIdentFused(const std::vector<double>& y, const std::vector<double>& s,
                                           const std::vector<double>* gnext, std::vector<double>* pnext) {
    const int n = n_;
    for (double x : hscale_)
        if (!std::isfinite(x)) return false;
    thread_local std::vector<double> ub, vb;
    if ((int)ub.size() < n) ub.resize(n);
    if (gnext && (int)vb.size() < n) vb.resize(n);
    double* u = ub.data();
    double* v = vb.data();
    const double* yp = y.data();
    const double* sp = s.data();
    const double* gp = gnext ? gnext->data() : nullptr;
    const double* scp = hscale_.empty() ? nullptr : hscale_.data();
    bool fin = true;
    double ys = 0.0, beta = 0.0;
    for (int i = 0; i < n; ++i) {
        const double di = scp ? scp[i] : 1.0, yi = yp[i];
        const double ui = 0.0 + di * yi;
        u[i] = ui;
        fin = fin && std::isfinite(yi);
        if (gp) {
            v[i] = 0.0 + di * gp[i];
            fin = fin && std::isfinite(gp[i]);
        }
        ys = ys + yi * sp[i];
        beta = beta + yi * ui;
    }
    if (!fin) return false;
    const double rho = 1 / ys;
    const double c = rho * rho * beta + rho;
    hs_.resize(n);
    ha_.resize(n);
    hb_.resize(n);
    double ag = 0.0, sg = 0.0;
    for (int i = 0; i < n; ++i) {
        const double si = sp[i], ai = c * si - rho * u[i];   // w = u for a diagonal D
        hs_[i] = si;
        ha_[i] = ai;
        hb_[i] = -rho * u[i];
        if (gp) {
            ag = ag + ai * gp[i];
            sg = sg + si * gp[i];
        }
    }
    pending_ = true;
    pend_dev_ = false;
    if (gnext && pnext) {
        pnext->resize(n);
        double* pn = pnext->data();
        for (int i = 0; i < n; ++i) pn[i] = -(v[i] + hs_[i] * ag + hb_[i] * sg);
    }
    return true;
}

void DenseInverseHessian::setInverseOf(const std::vector<std::vector<double>>& B) {
    // matrixInverse(B, D) (BFGS_with_linesearch.cpp:40): one device elimination of [B | I]
    // and per-column back substitution, bitwise the reference's per-column luSolve
    std::vector<double> hB((size_t)n_ * n_);
    for (int i = 0; i < n_; ++i)
        for (int j = 0; j < n_; ++j) hB[(size_t)i * n_ + j] = B[i][j];
    DevVec dB(ctx_, hB.size());
    dB.upload(hB);
    int info = 0;
    if (!sharded_) {
        if (clobbered_) throw std::runtime_error("DenseInverseHessian: D used while lent to a reduced problem");
        check(pnol_matrix_inverse_d(ctx_, dB.get(), n_, n_, Dp_, ld_, &info), "matrix_inverse(initHessFD)");
        pending_ = false;
        ident_ = false;
        dev_ok_ = true;
        return;
    }
    DevVec dI(ctx_, (size_t)n_ * n_);   // row-sharded D: the whole inverse, then this rank's rows
    check(pnol_matrix_inverse_d(ctx_, dB.get(), n_, n_, dI.get(), n_, &info), "matrix_inverse(initHessFD)");
    std::vector<double> h((size_t)n_ * n_);
    dI.download(h);
    std::vector<std::vector<double>> Dm(n_, std::vector<double>(n_));
    for (int i = 0; i < n_; ++i)
        for (int j = 0; j < n_; ++j) Dm[i][j] = h[(size_t)i * n_ + j];
    setMatrix(Dm);
}

// D0 = inverse of the FD Hessian (initHessFD): hessianApproximation (its points batched through
// objEvalBatch) + the device matrixInverse
void init_from_fd_hessian(Objective* obj, std::vector<double>& X, double dXHess, DenseInverseHessian& D) {
    const int n = (int)X.size();
    std::vector<double> dXH(n, dXHess);
    std::vector<std::vector<double>> B;
    obj->hessianApproximation(X, dXH, B);
    D.setInverseOf(B);
}


}  // namespace pnol
