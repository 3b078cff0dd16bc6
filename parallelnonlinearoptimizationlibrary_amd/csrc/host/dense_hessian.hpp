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
    bool sharded() const { return sharded_; }
    int n() const { return n_; }
    bool exact() const { return exact_; }

    void setIdentity(const std::vector<double>* diagScale = nullptr);
    void setMatrix(const std::vector<std::vector<double>>& D);
    void getMatrix(std::vector<std::vector<double>>& D);
    // this = src[idx][idx] (idx ascending, size n()), gathered on the device
    void setSubmatrixOf(DenseInverseHessian& src, const std::vector<int>& idx);

    // p = -D g
    void direction(const std::vector<double>& g, std::vector<double>& p);
    // D <- (I - rho s y^T) D (I - rho y s^T) + rho s s^T; with gnext, pnext = -D_new gnext
    void update(const std::vector<double>& y, const std::vector<double>& s, const std::vector<double>* gnext,
                std::vector<double>* pnext);

  private:
    void materialize();   // fold a pending correction into D
    int pass(const double* sp, const double* ap, const double* bp, int wb, const double* y, const double* g, double* u,
             double* w, double* v);

    pnol_ctx* ctx_;
    int n_, ld_;
    bool exact_;
    bool sharded_ = false;
    int rb_ = 0, rc_ = 0;              // this rank's rows of D (all rows when not sharded)
    DevVec D_;
    DevVec y_, s_, g_, u_, w_, v_;     // staging vectors
    DevVec ps_, pa_, pb_;              // pending correction (fast mode)
    bool pending_ = false;
    std::vector<double> hs_, ha_, hb_; // host copies of the pending correction
};

// D0 = inverse of the FD Hessian (initHessFD: hessianApproximation + matrixInverse,
// PNOL_Objective.cpp:38-85), column by column through the reference-order device LU
void init_from_fd_hessian(Objective* obj, std::vector<double>& X, double dXHess, DenseInverseHessian& D);

}  // namespace pnol
