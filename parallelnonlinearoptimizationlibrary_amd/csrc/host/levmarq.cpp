// levmarq.cpp -- LevMarq and LevMarqMPI (drop-in for Source/LevenbergMarquardt.cpp and
// Source/LevenbergMarquardtMPI.cpp).  Both share one device-resident loop; the MPI form
// shards the FD Jacobian columns over the communicator (cost-balanced tiles) and shares the
// rows of J^T between the ranks.
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <iostream>
#include <stdexcept>
#include <utility>

#include "../pnol_comm.hpp"
#include "../pnol_internal.hpp"
#include "LevenbergMarquardt.hpp"
#include "LevenbergMarquardtMPI.hpp"
#include "device_util.hpp"

using namespace pnol;

namespace {

struct LMParams {
    double lambda0, lambdaFactor, dXGrad, xMinDiff;
    int maxIter, verbose;
    int* steps;   // optional: [accepted, rejected] loop trips (LevMarq::getStepCounts)
};

double norm2(const std::vector<double>& v) { return std::sqrt(seq_dot(v, v)); }

void print_vec(const std::vector<double>& v) {
    for (double x : v) std::printf("%.17g ", x);
    std::printf("\n");
}

// Device state of one LM solve.  JT holds J column-major (one FD column per row, ld = ldjt,
// n rows in natural column order).  LevMarqMPI: each rank evaluates its cost-balanced FD
// tiles (fd_tiles_of) in place and comm_share_rows fills in the other ranks' rows.
class LMDevice {
  public:
    LMDevice(pnol_ctx* ctx, int n, int m, int nranks)
        : ctx_(ctx), n_(n), m_(m), ldjt_(even_ld(m)), lda_(even_ld(n)) {
        (void)nranks;
        JT_.reset(ctx, (size_t)n * ldjt_);
        A_.reset(ctx, (size_t)n * lda_);
        rhs_.reset(ctx, n); sigma_.reset(ctx, n); x_.reset(ctx, n); h_.reset(ctx, n);
        F_.reset(ctx, m); Fprev_.reset(ctx, m); F0_.reset(ctx, m);
    }

    // x_ / h_ hold copies of host vectors; skip the transfer when the host vector is unchanged
    // (the FD point after an accepted step is the point just evaluated; dX never changes)
    static bool same(const std::vector<double>& a, const std::vector<double>& b) {   // bitwise (+0 != -0)
        return a.size() == b.size() && std::memcmp(a.data(), b.data(), sizeof(double) * a.size()) == 0;
    }
    void uploadX(const std::vector<double>& X) {
        if (same(X, xh_)) return;
        x_.upload(X);
        xh_ = X;
        ckpt_valid_ = false;
    }
    void uploadH(const std::vector<double>& dX) {
        if (same(dX, hh_)) return;
        h_.upload(dX);
        hh_ = dX;
    }

    // residuals at X into host F and device F_
    void evalResiduals(MultiObjective* obj, std::vector<double>& X, std::vector<double>& F) {
        if (pnol_dobj* d = obj->deviceObjective()) {
            uploadX(X);
            // also keeps the base chain's checkpoints of x for the Jacobian of an accepted step
            check(pnol_dobj_eval_ckpt_d(ctx_, d, x_.get(), F_.get()), "objective eval");
            ckpt_valid_ = true;
            F_.download(F);
            obj->countEvals(1);
        } else {
            obj->objEval(X, F);
            F_.upload(F);
        }
    }

    // J^T at X (LevenbergMarquardt.cpp:55 / LevenbergMarquardtMPI.cpp:60)
    void jacobian(MultiObjective* obj, std::vector<double>& X, std::vector<double>& dX, bool sharded) {
        const int P = sharded ? comm_size() : 1, r = sharded ? comm_rank() : 0;
        std::vector<int> st, ct;
        fd_tiles_of(n_, P, r, st, ct);
        int cnt = 0;
        for (int c : ct) cnt += c;
        if (pnol_dobj* d = obj->deviceObjective()) {
            uploadX(X);
            uploadH(dX);
            check(pnol_fd_jacobian_tiles_d(ctx_, d, x_.get(), h_.get(), st.data(), ct.data(), (int)st.size(),
                                           F0_.get(), 1, JT_.get(), ldjt_),
                  "fd_jacobian");
            obj->countEvals(cnt + 1);
        } else {
            // host objective: the reference's column loop over this rank's tiles, each tile's
            // points handed to objEvalBatch at once, one upload per tile.  LevMarqMPI: the
            // reference sums the zero-padded values over the ranks, which turns -0.0 into +0.0
            // (PNOL_Objective.cpp:279-286) -- reproduced by the + 0.0 at P > 1
            const double pad = P > 1 ? 0.0 : -0.0;   // v + (-0.0) == v for every v
            std::vector<double> F0(m_), FdX((size_t)kFdTileCols * m_), pts((size_t)kFdTileCols * n_),
                blk((size_t)kFdTileCols * ldjt_, 0.0);
            obj->objEvalBatch(X.data(), 1, n_, F0.data(), m_);
            for (double& v : F0) v = v + pad;
            for (size_t t = 0; t < st.size(); ++t) {
                for (int q = 0; q < ct[t]; ++q) {
                    const int j = st[t] + q;
                    double* row = pts.data() + (size_t)q * n_;
                    std::memcpy(row, X.data(), sizeof(double) * n_);
                    row[j] = row[j] + dX[j];
                }
                obj->objEvalBatch(pts.data(), ct[t], n_, FdX.data(), m_);
                for (int q = 0; q < ct[t]; ++q) {
                    const int j = st[t] + q;
                    const double* Fj = FdX.data() + (size_t)q * m_;
                    for (int i = 0; i < m_; ++i) blk[(size_t)q * ldjt_ + i] = ((Fj[i] + pad) - F0[i]) / dX[j];
                }
                JT_.upload(blk.data(), (size_t)ct[t] * ldjt_, (size_t)st[t] * ldjt_);
            }
        }
        if (P > 1) check(comm_share_rows(ctx_, JT_.get(), ldjt_, n_), "share(J)");
    }

    // Single process, device objective: the FD Jacobian and A = J^T J + lambda diag(J^T J) in
    // one call, back to back (pnol_fd_jtj_d can also pipeline FD column chunks beside the J^T J
    // rows they complete; at cfg 3 that measured slower, so the loop does not use it); bitwise the
    // same J and A as jacobian() + the J^T J of step().
    bool jacobianAndNormal(MultiObjective* obj, std::vector<double>& X, std::vector<double>& dX, double lambda) {
        pnol_dobj* d = obj->deviceObjective();
        if (!d) return false;
        uploadX(X);
        uploadH(dX);
        // x_ still holds the point F_ was evaluated at: reuse F_ and its checkpoints
        const bool reuse = ckpt_valid_;
        check(pnol_fd_jtj_d(ctx_, d, x_.get(), h_.get(), reuse ? F_.get() : F0_.get(), reuse ? 3 : 1, JT_.get(),
                            ldjt_, lambda, A_.get(), lda_, nullptr, 1),
              "fd_jtj");
        obj->countEvals(n_ + 1);
        return true;
    }

    // sigma = (J^T J + lambda diag(J^T J))^{-1} (-J^T F)   (LevenbergMarquardt.cpp:59-83);
    // LevMarqMPI splits the J^T J tiles over the ranks (bitwise the same A).  have_A: A was
    // already formed by jacobianAndNormal.
    void step(double lambda, std::vector<double>& sigma, bool sharded, bool have_A = false) {
        if (have_A) {
        } else if (sharded && comm_size() > 1)
            check(pnol_jtj_mpi_d(ctx_, JT_.get(), ldjt_, m_, n_, lambda, A_.get(), lda_, nullptr), "jtj");
        else
            check(pnol_jtj_d(ctx_, JT_.get(), ldjt_, m_, n_, lambda, A_.get(), lda_, nullptr), "jtj");
        check(pnol_jtr_d(ctx_, JT_.get(), ldjt_, m_, n_, F_.get(), rhs_.get()), "jtr");
        int info = 0;
        check(pnol_solve_d(ctx_, A_.get(), lda_, rhs_.get(), sigma_.get(), n_, 0, &info), "solve");
        sigma_.download(sigma);
    }

    void saveF() { std::swap(F_, Fprev_); ckpt_valid_ = false; }   // Fprev <- F (the next eval overwrites F_)
    void restoreF() { std::swap(F_, Fprev_); ckpt_valid_ = false; }

  private:
    pnol_ctx* ctx_;
    int n_, m_, ldjt_, lda_;
    DevVec JT_, A_, rhs_, sigma_, x_, h_, F_, Fprev_, F0_;
    std::vector<double> xh_, hh_;   // host images of x_ and h_
    bool ckpt_valid_ = false;       // F_ = F(x_) and the context's checkpoints are x_'s
};

// The single-process LM loop on a device objective with one host wait per trip
// (n > PNOL_SEQ_MAX; PNOL_LM_ASYNC=0 selects the general loop below).  A trip is queued whole
// on the context stream: FD Jacobian + A at x_i, -J^T F_i, the Cholesky solve (no status
// readback in between), x_{i+1} = x_i + sigma_i and F(x_{i+1}) with its checkpoints on the
// device, then sigma_i, F(x_{i+1}) and the solve status into pinned memory behind one event.
// The host then replays the reference's decision (LevenbergMarquardt.cpp:87-160).  A
// non-positive Cholesky pivot is redone with the reference-order LU, as pnol_solve_d does; a
// Cholesky wait that ran past its cap is redone with the same Cholesky (never the LU).
// (Queueing trip i+1 before deciding step i was measured: a rejected step then costs a whole
// wasted trip, and the post-convergence steps of the bench are mostly rejections.  What is queued
// early instead is trip i+1's FD Jacobian alone, behind a gate kernel that the decision opens at
// the point it picks -- prequeue / release, PNOL_LM_GATE.)
//
// LevMarqMPI (sliced = true) runs the same loop with the Jacobian split over the ranks
// (pnol_lm_jacobian_mpi_d): each rank evaluates its FD column tiles for all rows, every m-slice
// of them sent to the slice's rank while its next tile computes (columns mode, the default), or
// every FD column on its own m-slices of residual rows with the trial point likewise on its own
// rows, shared point-to-point (rows mode, PNOL_LM_FD=rows; pnol_lm_eval_mpi_d); each rank forms its slices' share of J^T J and
// J^T F and one reduce-scatter + allgather assemble A and -J^T F on every rank
// (pnol_lm_normal_mpi_d).  The collectives are queued on the same stream, so the trip still
// has one host wait; A, rhs and hence the trajectory are bitwise the single-GPU ones.
class LMAsync {
  public:
    LMAsync(pnol_ctx* ctx, pnol_dobj* d, int n, int m, bool sliced)
        : ctx_(ctx), d_(d), n_(n), m_(m), ldjt_(even_ld(m)), lda_(even_ld(n)), sliced_(sliced) {
        size_t jt = (size_t)n * ldjt_;
        if (sliced) {
            check(pnol_lm_sliced_layout(m, n, nullptr, &jt), "sliced layout");
            // the FD decomposition, read once per solve (PNOL_LM_FD; a mode chosen through
            // pnol_lm_set_fd_mode stands) and the same on every rank: the two modes pair
            // different transfers, so ranks that disagreed would mismatch them
            if (!ctx->lm_fd_mode_set) ctx->lm_fd_mode = lm_fd_mode_env();
            std::vector<int> all;
            check(comm_allgather_int(ctx, ctx->lm_fd_mode, all), "allgather(fd mode)");
            for (int v : all)
                if (v != ctx->lm_fd_mode) throw std::runtime_error("LevMarqMPI: ranks disagree on PNOL_LM_FD");
            // the columns mode's phasing likewise: a phased rank posts one exchange per tile phase
            // on a second stream, an unphased one a single exchange
            ctx->lm_phased = lm_phased_env();
            check(comm_allgather_int(ctx, ctx->lm_phased, all), "allgather(phased)");
            for (int v : all)
                if (v != ctx->lm_phased) throw std::runtime_error("LevMarqMPI: ranks disagree on PNOL_LM_PHASED");
        }
        // The trip without forming A (default; PNOL_LM_TRIP=0 keeps the two calls, read once per
        // solve): one GPU, pnol_lm_trip_d -- the reduce launch writes A straight into the
        // Cholesky's padded matrix; LevMarqMPI, pnol_lm_normal_solve_mpi_d -- the persistent
        // Cholesky's first tasks sum the allgathered tiles (33.5 MB) into it.  (With one rank the
        // reduce tasks would stream the 285 MB of split-K partials in front of the chain's first
        // steps: 5 of 5 alternating same-box pairs slower than the two calls, 317-321 vs
        // 324-328.5 LM iters/s, profiles/r05_trip_ab.txt; PNOL_LM_REDUCE=tasks keeps that form.)
        {
            const char* e = std::getenv("PNOL_LM_TRIP");
            trip_fused_ = !e || std::atoi(e) != 0;
            const char* z = std::getenv("PNOL_LM_ZEROCOPY");
            zero_copy_ = trip_fused_ && !sliced && (!z || std::atoi(z) != 0);
            // the next trip's Jacobian queued behind a gate while the host decides (PNOL_LM_GATE=0:
            // queued after the decision, as the rest of the trip)
            const char* g = std::getenv("PNOL_LM_GATE");
            gate_ok_ = zero_copy_ && (!g || std::atoi(g) != 0);
            // how long a gate waits for the decision (ticks of 100 MHz; default 1 s; a test sets 0
            // to exercise the repeat of a trip whose gate gave up)
            const char* c = std::getenv("PNOL_LM_GATE_CAP");
            gate_cap_ = c ? std::strtoull(c, nullptr, 10) : 100000000ull;
        }
        // several ranks: every trip's solve status is agreed over the ranks before the host acts
        // on it (pnol_lm_agree_status_d), so all replicas take the same branch
        agree_ = sliced && comm_size() > 1;
        JT_.reset(ctx, jt);
        A_.reset(ctx, (size_t)n * lda_);
        rhs_.reset(ctx, n);
        h_.reset(ctx, n);
        // trip s's results side by side -- sigma_s | F(x_s + sigma_s) | solve status -- so one
        // copy brings them to the host; F(x_[s]) is trip s^1's middle part
        np_ = even_ld(n);
        mp_ = even_ld(m);
        for (int s = 0; s < 2; ++s) {
            x_[s].reset(ctx, n);
            trip_[s].reset(ctx, (size_t)np_ + mp_ + 2);
            check(pnol_host_alloc(&pin_[s], sizeof(double) * ((size_t)np_ + mp_ + 2)), "host_alloc");
            check(pnol_event_create(ctx, &ev_[s]), "event_create");
        }
        if (gate_ok_) {
            void* g = nullptr;
            check(pnol_host_alloc(&g, sizeof(int) * 4), "host_alloc");
            gate_h_ = static_cast<int*>(g);
            gate_h_[0] = gate_h_[1] = gate_h_[2] = gate_h_[3] = 0;
            gsel_.reset(ctx, 1);
        }
    }
    ~LMAsync() {
        if (gate_pending_) release(-1);   // a queued Jacobian returns at once
        (void)pnol_ctx_synchronize(ctx_);
        if (gate_h_) (void)pnol_host_free(gate_h_);
        for (int s = 0; s < 2; ++s) {
            (void)pnol_host_free(pin_[s]);
            (void)pnol_event_destroy(ev_[s]);
        }
    }
    double* x(int s) { return x_[s].get(); }
    double* F(int s) { return trip_[s ^ 1].get() + np_; }   // F(x_[s])
    double* sig(int s) { return trip_[s].get(); }
    int* info(int s) { return reinterpret_cast<int*>(trip_[s].get() + np_ + mp_); }
    const double* sigma_h(int s) const { return static_cast<const double*>(pin_[s]); }
    double* pin_sigma(int s) { return static_cast<double*>(pin_[s]); }
    const double* Fnext_h(int s) const { return static_cast<const double*>(pin_[s]) + np_; }
    int info_h(int s) const { return *reinterpret_cast<const int*>(static_cast<const double*>(pin_[s]) + np_ + mp_); }
    void uploadH(const std::vector<double>& dX) { h_.upload(dX); }

    // The next trip's FD Jacobian queued now, behind a gate the host opens with its decision
    // (release): at x_[s] if trip s's step is rejected, at x_[s^1] if accepted.  Between the
    // trial point's evaluation and the next Jacobian the GPU then waits only for the host's
    // decision, not for it to queue the launch as well.  False: nothing queued.
    bool prequeue(int s) {
        if (!gate_ok_) return false;
        ++gate_seq_;
        const int st = lm_prequeue_fd(ctx_, d_, x_[s].get(), F(s), x_[s ^ 1].get(), F(s ^ 1), h_.get(), JT_.get(),
                                      ldjt_, gate_h_, gate_seq_, reinterpret_cast<int*>(gsel_.get()),
                                      gate_h_ + 2, gate_cap_);
        if (st == PNOL_ERR_UNSUPPORTED) return false;
        check(st, "fd_jacobian (queued)");
        gate_pending_ = true;
        return true;
    }
    // the decision for the queued Jacobian: 0 at x_[s], 1 at x_[s^1], -1 none (it returns at once)
    void release(int choice) {
        __atomic_store_n(&gate_h_[1], choice, __ATOMIC_RELAXED);
        __atomic_store_n(&gate_h_[0], gate_seq_, __ATOMIC_RELEASE);
        gate_pending_ = false;
        rel_seq_ = gate_seq_;
        rel_choice_ = choice;
    }
    // after the trip that used the queued Jacobian: its gate passed the released choice on (a gate
    // that timed out -- the host answered after its cap -- made the Jacobian launch return)
    bool gate_passed() const {
        return __atomic_load_n(&gate_h_[3], __ATOMIC_ACQUIRE) == rel_seq_ &&
               __atomic_load_n(&gate_h_[2], __ATOMIC_RELAXED) == rel_choice_;
    }

    // trip at x_[s] (F_[s] = F(x_[s]); ckpt: its checkpoints are current) -> sigma, x_[s^1], F_[s^1]
    // queued: its FD Jacobian is queued already (prequeue, released)
    void enqueue(int s, double lambda, bool ckpt, bool queued = false) {
        if (sliced_) {
            check(pnol_lm_jacobian_mpi_d(ctx_, d_, x_[s].get(), h_.get(), F(s), ckpt ? 3 : 1, JT_.get()),
                  "fd_jacobian");
            if (trip_fused_) {
                lambda_[s] = lambda;
                check(pnol_lm_normal_solve_mpi_d(ctx_, JT_.get(), m_, n_, lambda, F(s), rhs_.get(), sig(s), info(s),
                                                 x_[s].get(), x_[s ^ 1].get()),
                      "normal equations + solve");
                agree(s);
                finish(s, false);
                return;
            }
            check(pnol_lm_normal_mpi_d(ctx_, JT_.get(), m_, n_, lambda, F(s), A_.get(), lda_, rhs_.get(),
                                       nullptr),
                  "normal equations");
        } else if (trip_fused_) {
            // FD Jacobian, the J^T J / -J^T F partials, the Cholesky that reduces them itself,
            // the backward solve forming the trial point; the backward solve and the trial point's
            // evaluation also write sigma, F(x + sigma) and the status straight into the pinned
            // block (pnol_ctx::TripMirror), so no copy follows the trip (PNOL_LM_ZEROCOPY=0: the copy)
            lambda_[s] = lambda;
            if (zero_copy_) ctx_->trip_mirror.sigma = pin_sigma(s);
            const int st = queued ? launch_fd_normal_solve(ctx_, d_, x_[s].get(), h_.get(), F(s), 3, JT_.get(), ldjt_,
                                                           lambda, rhs_.get(), sig(s), info(s), x_[s ^ 1].get(), true)
                                  : pnol_lm_trip_d(ctx_, d_, x_[s].get(), h_.get(), F(s), ckpt ? 3 : 1, JT_.get(),
                                                   ldjt_, lambda, rhs_.get(), sig(s), info(s), x_[s ^ 1].get());
            ctx_->trip_mirror = {};
            check(st, "lm trip");
            finish(s, false, zero_copy_);
            return;
        } else {
            // FD Jacobian, A and -J^T F in one queue (the GEMV in the J^T J's tail)
            check(pnol_fd_normal_d(ctx_, d_, x_[s].get(), h_.get(), F(s), ckpt ? 3 : 1, JT_.get(), ldjt_, lambda,
                                   A_.get(), lda_, nullptr, rhs_.get()),
                  "fd_normal");
        }
        // the solve's last launch also forms the trial point x_[s] + sigma
        check(pnol_solve_step_d(ctx_, A_.get(), lda_, rhs_.get(), sig(s), n_, info(s), x_[s].get(), x_[s ^ 1].get()),
              "solve");
        agree(s);
        finish(s, false);
    }
    // LevMarqMPI on several ranks: info(s)[1] = the trip's solve status code agreed over the ranks
    // (queued in stream order before the trial point, so it rides in the trip's one result copy)
    void agree(int s) {
        if (agree_) check(pnol_lm_agree_status_d(ctx_, info(s)), "agree(solve status)");
    }
    // what the host does about trip s's solve: 0 nothing, 1 relaunch the Cholesky (a wait ran past
    // its cap), 2 the reference-order LU (a non-positive pivot) -- the same on every rank
    int action_h(int s) const {
        const int* w = reinterpret_cast<const int*>(static_cast<const double*>(pin_[s]) + np_ + mp_);
        return agree_ ? w[1] : solve_status_code(w[0]);
    }
    // the rest of a trip once sigma_[s] is known: trial point (unless the solve formed it), its
    // residuals, copies back
    // zero_copy: the evaluation writes F(x + sigma) and the status word into the pinned block
    // itself (the backward solve wrote sigma there), instead of the copy of the three
    void finish(int s, bool add = true, bool zero_copy = false) {
        if (add) check(pnol_add_d(ctx_, x_[s].get(), sig(s), x_[s ^ 1].get(), n_), "add");
        // LevMarqMPI: each rank's rows, then all rows everywhere (rows mode)
        if (sliced_) {
            check(pnol_lm_eval_mpi_d(ctx_, d_, x_[s ^ 1].get(), F(s ^ 1)), "objective eval");
        } else {
            if (zero_copy) {
                double* pin = static_cast<double*>(pin_[s]);
                ctx_->trip_mirror.F = pin + np_;
                ctx_->trip_mirror.info_d = info(s);
                ctx_->trip_mirror.info_h = reinterpret_cast<int*>(pin + np_ + mp_);
            }
            const int st = pnol_dobj_eval_ckpt_d(ctx_, d_, x_[s ^ 1].get(), F(s ^ 1));
            ctx_->trip_mirror = {};
            check(st, "objective eval");
        }
        if (!zero_copy)
            check(pnol_memcpy_d2h_async(ctx_, pin_[s], trip_[s].get(), sizeof(double) * ((size_t)np_ + mp_ + 1)),
                  "d2h");
        check(pnol_event_record(ctx_, ev_[s]), "event");
    }
    void wait(int s) { check(pnol_event_wait(ev_[s]), "event wait"); }
    // trip s's solve again, on every rank alike (action_h): A from the trip's tiles, then the
    // reference-order LU after a non-positive pivot (action 2), or the same Cholesky relaunched
    // after a timed-out wait (action 1; pnol_solve_d method 0 retries a timeout itself, and a
    // pivot it finds non-positive goes to the LU there -- A is the same on every rank, so that
    // outcome is too).  Then the trial point and its residuals again: in rows mode that is the
    // same F exchange on every rank.
    void redo(int s, int action) {
        check(pnol_ctx_synchronize(ctx_), "sync");
        if (trip_fused_ && sliced_) {
            check(pnol_lm_normal_unpack_mpi_d(ctx_, m_, n_, lambda_[s], A_.get(), lda_), "normal equations");
        } else if (trip_fused_) {
            check(pnol_lm_trip_normal_d(ctx_, m_, n_, lambda_[s], A_.get(), lda_), "normal equations");
            // -J^T F again (the reducing Cholesky's first task wrote it; bitwise pnol_jtr_d's)
            check(pnol_jtr_d(ctx_, JT_.get(), ldjt_, m_, n_, F(s), rhs_.get()), "jtr");
        }
        int info = 0;
        if (action == 1) ctx_->chol_order0 = true;   // a timed-out wait: step-order claims from now on
        const int st = pnol_solve_d(ctx_, A_.get(), lda_, rhs_.get(), sig(s), n_, action == 2 ? 2 : 0, &info);
        if (agree_) {
            // a relaunch budget exhausted on one rank only must fail every rank alike: its peers
            // would otherwise go on into the next trip's collectives and wait for it forever
            std::vector<int> all;
            check(comm_allgather_int(ctx_, st, all), "allgather(redo status)");
            for (int v : all)
                if (v != PNOL_OK) check(st != PNOL_OK ? st : v, "solve (redo, agreed over the ranks)");
        }
        check(st, "solve");
        finish(s);
        wait(s);
    }

  private:
    pnol_ctx* ctx_;
    pnol_dobj* d_;
    int n_, m_, ldjt_, lda_;
    bool sliced_;
    bool trip_fused_ = false;
    bool zero_copy_ = false;   // the one-GPU fused trip's results written into pin_ by its kernels
    bool gate_ok_ = false;     // prequeue in use (one GPU, zero-copy trip)
    bool gate_pending_ = false;
    unsigned long long gate_cap_ = 0;
    int gate_seq_ = 0;                 // the last gate queued
    int rel_seq_ = 0, rel_choice_ = 0; // the last gate released and its choice
    int* gate_h_ = nullptr;    // pinned {seq, choice} (host -> gate), {choice, seq} (gate -> host)
    DevVec gsel_;
    bool agree_ = false;
    double lambda_[2] = {0, 0};   // trip s's lambda (the fused trip's LU fallback forms A)
    int np_ = 0, mp_ = 0;
    DevVec JT_, A_, rhs_, h_, x_[2], trip_[2];
    void* pin_[2] = {nullptr, nullptr};
    pnol_event* ev_[2] = {nullptr, nullptr};
};

bool lm_async_enabled() {
    const char* e = std::getenv("PNOL_LM_ASYNC");   // read per solve (tests compare both loops)
    return !e || std::atoi(e) != 0;
}

// The sliced LevMarqMPI form: linear-residual device objectives, up to PNOL_LM_SLICES ranks
// (PNOL_LM_SLICED=0 keeps the column-sharded general loop)
bool lm_sliced_ok(pnol_dobj* d) {
    const char* e = std::getenv("PNOL_LM_SLICED");
    if (e && std::atoi(e) == 0) return false;
    int kind = 0, n = 0, m = 0;
    return pnol_dobj_info(d, &kind, &n, &m) == PNOL_OK && kind == PNOL_OBJ_LINRES && comm_size() <= PNOL_LM_SLICES;
}

void lm_solve_async(MultiObjective* obj, pnol_dobj* d, const LMParams& P, bool sharded, bool sliced,
                    std::vector<double>& X, std::vector<double>& F0, std::vector<double>& FOpt) {
    const int n = (int)X.size();
    const int m = (int)F0.size();
    const bool loud = !sharded || comm_rank() == ROOT_ID;
    pnol_ctx* ctx = require_ctx();
    LMAsync dev(ctx, d, n, m, sliced);
    int own_cols = n;   // FD columns this rank evaluates per Jacobian (LevMarqMPI: its tiles)
    if (sharded) {
        std::vector<int> st, ct;
        fd_tiles_of(n, comm_size(), comm_rank(), st, ct);
        own_cols = 0;
        for (int c : ct) own_cols += c;
    }
    double lambda = P.lambda0;
    std::vector<double> dX(n, P.dXGrad), F(m);
    dev.uploadH(dX);
    int s = 0;
    check(pnol_memcpy_h2d(ctx, dev.x(s), X.data(), sizeof(double) * n), "h2d");
    check(pnol_dobj_eval_ckpt_d(ctx, d, dev.x(s), dev.F(s)), "objective eval");
    check(pnol_memcpy_d2h(ctx, F0.data(), dev.F(s), sizeof(double) * m), "d2h");
    obj->countEvals(1);
    F = F0;
    double nrm = norm2(F);
    double chiSq = nrm * nrm;
    int iter = 0;
    double xdiff2Norm = P.xMinDiff * 2;
    bool ckpt = true;   // the checkpoints in the context are those of x_[s]
    // PNOL_LM_HOSTPROF=1: the host's share of a trip (decision, enqueue) to stderr at the end
    const bool hprof = std::getenv("PNOL_LM_HOSTPROF") != nullptr;
    double h_dec = 0, h_enq = 0;
    auto hnow = [] { return std::chrono::steady_clock::now(); };
    auto t_dec = hnow();
    bool queued = false;   // trip s's Jacobian was queued behind the last trip (prequeue) and released
    while (iter < P.maxIter) {
        auto t0 = hnow();
        if (hprof && iter > 0) h_dec += std::chrono::duration<double, std::micro>(t0 - t_dec).count();
        dev.enqueue(s, lambda, ckpt, queued);
        // the next trip's Jacobian, behind a gate that the decision below opens (not after the
        // last trip; PNOL_LM_GATE=0: never)
        bool pre = iter + 1 < P.maxIter && dev.prequeue(s);
        if (hprof) h_enq += std::chrono::duration<double, std::micro>(hnow() - t0).count();
        dev.wait(s);
        if (hprof) t_dec = hnow();
        if (queued && !dev.gate_passed()) {
            // the gate gave up before the host answered (its 1 s cap): trip s ran without its
            // Jacobian -- run it again whole
            std::cerr << "[pnol] LM trip " << iter << ": queued Jacobian gate timed out; trip repeated" << std::endl;
            if (pre) dev.release(-1);
            dev.enqueue(s, lambda, ckpt, false);
            pre = iter + 1 < P.maxIter && dev.prequeue(s);
            dev.wait(s);
        }
        queued = false;
        if (const int action = dev.action_h(s)) {
            // the redo queues behind the gate: open it with no Jacobian first
            if (pre) dev.release(-1);
            pre = false;
            // the same action on every rank (agreed in the trip); a timed-out wait is never mapped
            // to the LU, and is always reported (PNOL_LM_DEBUG: the LU redos too)
            if (action == 1 || std::getenv("PNOL_LM_DEBUG"))
                std::cerr << "[pnol] LM trip " << iter << ": solve status " << dev.info_h(s) << " (agreed action "
                      << action << "): " << (action == 2 ? "reference-order LU" : "Cholesky relaunched") << std::endl;
            dev.redo(s, action);
        }
        obj->countEvals(own_cols + 1); // the trip's Jacobian
        obj->countEvals(1);            // its trial point
        // chi^2 straight from the pinned copy (no host copy of F: the accepted F stays on the
        // device and is downloaded once at the end)
        const double* sig_h = dev.sigma_h(s);
        const double* Fn = dev.Fnext_h(s);
        const double chiSqPrev = chiSq;
        nrm = std::sqrt(seq_dot(Fn, Fn, (size_t)m));
        chiSq = nrm * nrm;
        if (chiSq >= chiSqPrev || chiSq != chiSq) {
            // the reference prints lambda / lambdaFactor --> lambda before the multiply
            // (LevenbergMarquardt.cpp:107-111, LevenbergMarquardtMPI.cpp:112-116)
            if (sharded ? (P.verbose >= 1 && loud) : (P.verbose > 1))
                std::cout << "Step " << iter << " failed with chiSq = " << chiSq << ", chiSqPrev = " << chiSqPrev
                          << ",  increasing lambda: " << lambda / P.lambdaFactor << " --> " << lambda << std::endl;
            chiSq = chiSqPrev;
            lambda = lambda * P.lambdaFactor;
            if (P.steps) P.steps[1]++;
            ckpt = true;               // x_[s], F_[s] stand, and so do x_[s]'s checkpoints (the
                                       // trial point's went to the other slot)
            if (pre) dev.release(0);   // the queued Jacobian at x_[s]
        } else {
            lambda = lambda / P.lambdaFactor;
            if (P.steps) P.steps[0]++;
            xdiff2Norm = std::sqrt(seq_dot(sig_h, sig_h, (size_t)n));
            const bool done = xdiff2Norm < P.xMinDiff;
            if (pre) dev.release(done ? -1 : 1);   // the queued Jacobian at x_[s^1], or none
            for (int i = 0; i < n; ++i) X[i] = X[i] + sig_h[i];   // == x_[s^1] (same IEEE add)
            s ^= 1;
            ckpt = true;
            if (done) break;
        }
        queued = pre;
        if ((sharded ? (P.verbose >= 1 && loud) : (P.verbose > 0)) && iter % 10 == 0) {
            std::cout << "At iter = " << iter << " the xdiff 2Norm = " << xdiff2Norm << ", chi^2 = " << chiSq
                      << ", and params: ";
            print_vec(X);
        }
        iter++;
    }
    if (hprof && iter > 0)
        std::cerr << "[pnol] LM host per trip: decision " << h_dec / iter << " us, enqueue " << h_enq / (iter + 1)
                  << " us" << std::endl;
    FOpt.resize(m);
    check(pnol_memcpy_d2h(ctx, FOpt.data(), dev.F(s), sizeof(double) * m), "d2h");   // F(x_[s]) = F(X)
    if (P.verbose >= 0 && loud) {
        std::cout << std::endl << "-----------------------------------------------------------------------------------" << std::endl;
        std::cout << "Completed Levenberg Marquardt." << std::endl;
        std::cout << "At iter = " << iter << " the xdiff 2Norm = " << xdiff2Norm << ", chi^2 = " << chiSq
                  << ", and  optimal params: " << std::endl;
        print_vec(X);
        std::cout << "-----------------------------------------------------------------------------------" << std::endl << std::endl;
    }
}

void lm_solve(MultiObjective* obj, const LMParams& P, bool sharded, std::vector<double>& X, std::vector<double>& F0,
              std::vector<double>& FOpt) {
    const int n = (int)X.size();
    const int m = (int)F0.size();
    const int rank = sharded ? comm_rank() : 0;
    const bool loud = rank == ROOT_ID;
    if (n > PNOL_SEQ_MAX && lm_async_enabled())
        if (pnol_dobj* d = obj->deviceObjective())
            if (!sharded || lm_sliced_ok(d)) {
                // LevMarq keeps the row-major J^T (measured 0.7% faster on one GPU than the
                // sliced layout; bitwise the same trajectory)
                return lm_solve_async(obj, d, P, sharded, sharded, X, F0, FOpt);
            }
    pnol_ctx* ctx = require_ctx();
    LMDevice dev(ctx, n, m, sharded ? comm_size() : 1);

    double lambda = P.lambda0;
    std::vector<double> dX(n, P.dXGrad), F(m), Fprev(m), sigma(n), Xprev(n);
    dev.evalResiduals(obj, X, F0);
    F = F0;
    Fprev = F;
    Xprev = X;
    double nrm = norm2(F);
    double chiSq = nrm * nrm;   // pow(vector2Norm(F), 2)
    int iter = 0;
    double xdiff2Norm = P.xMinDiff * 2;
    while (iter < P.maxIter) {
        const bool have_A = !sharded && dev.jacobianAndNormal(obj, X, dX, lambda);
        if (!have_A) dev.jacobian(obj, X, dX, sharded);
        dev.step(lambda, sigma, sharded, have_A);
        Xprev = X;
        Fprev = F;
        dev.saveF();
        for (int i = 0; i < n; ++i) X[i] = X[i] + sigma[i];
        dev.evalResiduals(obj, X, F);
        const double chiSqPrev = chiSq;
        nrm = norm2(F);
        chiSq = nrm * nrm;
        if (chiSq >= chiSqPrev || chiSq != chiSq) {
            const bool talk = sharded ? (P.verbose >= 1 && loud) : (P.verbose > 1);
            if (talk)
                std::cout << "Step " << iter << " failed with chiSq = " << chiSq << ", chiSqPrev = " << chiSqPrev
                          << ",  increasing lambda: " << lambda / P.lambdaFactor << " --> " << lambda << std::endl;
            chiSq = chiSqPrev;
            X = Xprev;
            F = Fprev;
            dev.restoreF();
            lambda = lambda * P.lambdaFactor;
            if (P.steps) P.steps[1]++;
        } else {
            lambda = lambda / P.lambdaFactor;
            if (P.steps) P.steps[0]++;
            xdiff2Norm = norm2(sigma);
            if (xdiff2Norm < P.xMinDiff) break;
        }
        const bool talk = sharded ? (P.verbose >= 1 && loud) : (P.verbose > 0);
        if (talk && iter % 10 == 0) {
            std::cout << "At iter = " << iter << " the xdiff 2Norm = " << xdiff2Norm << ", chi^2 = " << chiSq
                      << ", and params: ";
            print_vec(X);
        }
        iter++;
    }
    FOpt = F;
    if (P.verbose >= 0 && loud) {
        std::cout << std::endl << "-----------------------------------------------------------------------------------" << std::endl;
        std::cout << "Completed Levenberg Marquardt." << std::endl;
        std::cout << "At iter = " << iter << " the xdiff 2Norm = " << xdiff2Norm << ", chi^2 = " << chiSq
                  << ", and  optimal params: " << std::endl;
        print_vec(X);
        std::cout << "-----------------------------------------------------------------------------------" << std::endl << std::endl;
    }
}

}  // namespace

void LevMarq::findMin(vector<double>& X, vector<double>& F0, vector<double>& FOpt) {
    stepCounts[0] = stepCounts[1] = 0;
    LMParams P{lambda0, lambdaFactor, dXGrad, xMinDiff, maxIter, verbose, stepCounts};
    lm_solve(mObjPtr, P, false, X, F0, FOpt);
}

void LevMarqMPI::findMin(vector<double>& X, vector<double>& F0, vector<double>& FOpt) {
    require_comm("LevMarqMPI::findMin");   // LevenbergMarquardtMPI.cpp:16-17
    stepCounts[0] = stepCounts[1] = 0;
    LMParams P{lambda0, lambdaFactor, dXGrad, xMinDiff, maxIter, verbose, stepCounts};
    lm_solve(mObjPtr, P, true, X, F0, FOpt);
}
