// dense_hessian.hpp -- the BFGS inverse Hessian D as a device-resident matrix.
//
// Two execution modes (chosen per solve):
//  exact  updateHessianInv and p = -D g in the reference's operation order
//         (BFGS_with_linesearch.cpp:78-79, 389-432): bitwise equal to the CPU path.
//  fast   the rank-2 form, applied lazily: D is stored together with a pending correction
//         (s, a, b) meaning D + s a^T + b s^T.  update() runs ONE streaming pass that folds
//         the pending correction into D (write-back), and returns u = D y, w = D^T y and
//         v = D g_next, from which the next correction and the next direction follow with
//         O(n) vector algebra: 16 n^2 bytes of HBM traffic per BFGS iteration.
// Row-sharded (fast mode, shard requested, more than one rank): each rank keeps
// rows [rb, rb + rc) of D and the passes / H.g run on those rows only, the full n-vectors
// assembled by allgathers (pnol_*_mpi_d) -- bitwise the one-GPU results, 1/P of the HBM
// traffic per rank.
//
// Identity state.  setIdentity() (D = I or diag(scale): BFGS_with_linesearch.cpp:46-56,
// BFGS_bnd_linesearch.cpp:65-83, 607-616, 647) writes nothing: while D is a stored diagonal,
// D g, D y and D^T y are the single products 0.0 + scale_i v_i the device sums would give
// (every other term of each sum is an exact zero), formed on the host; the first fold of a
// pending correction synthesises the diagonal instead of reading it (16 n^2 bytes saved), and
// the identity is written out only when something must read D itself.  Non-finite inputs take
// the device path (0 * inf must poison the whole row as it does there).
//
// Storage lending.  BFGS_Bnd's active-set recursion discards the outer D while the reduced
// problem runs (it is reset to I on return, BFGS_bnd_linesearch.cpp:620, 647), so a reduced
// D borrows its parent's device buffer: the whole recursion -- up to one level per iteration
// at n = 16384 -- holds one n x n matrix (2.15 GB) instead of one per level.
#pragma once

#include <vector>

#include "device_util.hpp"

class Objective;

namespace pnol {

class DenseInverseHessian {
  public:
    // mode: 0 auto (exact for n <= PNOL_SEQ_MAX), 1 exact, 2 fast; shard: row-shard D over the
    // communicator when in fast mode with more than one rank (PNOL_BFGS_SHARD=0 disables)
    DenseInverseHessian(pnol_ctx* ctx, int n, int mode, bool shard = false);
    // a reduced D on the device buffer of `parent` (when it fits; else its own): the parent's
    // contents are forfeit until its next setIdentity / setMatrix
    DenseInverseHessian(DenseInverseHessian& parent, int n, int mode, bool shard = false);
    bool sharded() const { return sharded_; }
    int n() const { return n_; }
    bool exact() const { return exact_; }
    bool borrowed() const { return Dp_ != D_.get(); }

    void setIdentity(const std::vector<double>* diagScale = nullptr);
    void setMatrix(const std::vector<std::vector<double>>& D);
    // D = B^{-1}, the reference's matrixInverse (initHessFD), computed on the device
    void setInverseOf(const std::vector<std::vector<double>>& B);
    void getMatrix(std::vector<std::vector<double>>& D);
    // this = src[idx][idx] (idx ascending, size n()), gathered on the device
    void setSubmatrixOf(DenseInverseHessian& src, const std::vector<int>& idx);

    // p = -D g
    void direction(const std::vector<double>& g, std::vector<double>& p);
    // D <- (I - rho s y^T) D (I - rho y s^T) + rho s s^T; with gnext, pnext = -D_new gnext
    void update(const std::vector<double>& y, const std::vector<double>& s, const std::vector<double>* gnext,
                std::vector<double>* pnext);

  private:
    void init(int mode, bool shard);
    void materialize();   // fold a pending correction into D
    void ensureDevice();  // the stored D really in device memory (writes a lazy identity)
    const double* deviceScale();
    bool identFinite(const std::vector<double>* a, const std::vector<double>* b) const;
    bool updateIdentFused(const std::vector<double>& y, const std::vector<double>& s,
                          const std::vector<double>* gnext, std::vector<double>* pnext);
    double sc(int i) const { return hscale_.empty() ? 1.0 : hscale_[i]; }
    int pass(const double* sp, const double* ap, const double* bp, int wb, const double* y, const double* g, double* u,
             double* w, double* v);
    int passIdent(const double* y, const double* g, double* u, double* w, double* v);

    pnol_ctx* ctx_;
    int n_, ld_;
    bool exact_;
    bool sharded_ = false;
    int rb_ = 0, rc_ = 0;              // this rank's rows of D (all rows when not sharded)
    DevVec D_;                         // own storage (empty when borrowed)
    double* Dp_ = nullptr;             // the matrix: D_.get() or the lender's buffer
    size_t cap_ = 0;                   // doubles available at Dp_ (lent on to reduced problems)
    // staging vectors in one device block, so each group crosses PCIe in one copy:
    // [y | g | u | w | v | s_p | a_p | b_p] (exact mode: s in the g slot)
    // (lent down the recursion with D: the parent does not stage anything while it waits)
    DevVec io_;
    double* iop_ = nullptr;
    double* slot(int k) const { return iop_ + (size_t)k * n_; }
    void up(int k, const double* src, size_t count) {
        check(pnol_memcpy_h2d(ctx_, slot(k), src, sizeof(double) * count), "h2d");
    }
    void down(int k, double* dst, size_t count) const {
        check(pnol_memcpy_d2h(ctx_, dst, slot(k), sizeof(double) * count), "d2h");
    }
    enum { kY = 0, kG, kU, kW, kV, kPS, kPA, kPB, kSlots };
    DevVec dscale_;                    // device copy of the diagonal scale (lazy)
    bool pending_ = false;
    bool pend_dev_ = false;            // the pending correction is uploaded (lazily: most reduced
                                       // problems of the recursion never fold theirs)
    std::vector<double> hs_, ha_, hb_; // host copies of the pending correction
    void uploadPending();
    bool ident_ = false;               // stored D == diag(hscale_) (empty: I)
    bool dev_ok_ = true;               // device memory holds the stored D
    bool clobbered_ = false;           // buffer lent to a reduced problem since the last reset
    bool dscale_ok_ = false;
    std::vector<double> hscale_;
};

// D0 = inverse of the FD Hessian (initHessFD: hessianApproximation + matrixInverse,
// PNOL_Objective.cpp:38-85, BFGS_with_linesearch.cpp:34-41): one device LU factorisation,
// the n unit right-hand sides solved against it in the reference's per-column order
void init_from_fd_hessian(Objective* obj, std::vector<double>& X, double dXHess, DenseInverseHessian& D);

}  // namespace pnol
