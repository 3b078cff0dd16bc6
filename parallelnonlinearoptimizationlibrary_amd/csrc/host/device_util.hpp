// device_util.hpp -- small RAII helpers the C++ drop-in classes use on top of the C ABI.
#pragma once

#include <chrono>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "../pnol_comm.hpp"
#include "pnol_amd.h"

namespace pnol {

// The drop-in classes have no error return (as in the reference); a failed device call is
// fatal for the solve and surfaces as an exception naming the call.
inline void check(int status, const char* what) {
    if (status != PNOL_OK)
        throw std::runtime_error(std::string("pnol_amd: ") + what + ": " + pnol_status_string(status));
}

// Every *_MPI entry point: the communicator of the MPI launch (pnol_comm_bind_launcher), or an
// error rather than a silent single-rank run of a multi-rank job.
inline void require_comm(const char* who) {
    if (comm_bind_launcher() != PNOL_OK)
        throw std::runtime_error(std::string("pnol_amd: ") + who +
                                 ": started by an MPI launcher with several ranks but no communicator is bound "
                                 "(MPI_Init + <mpi.h> on the include path, or pnol_comm_init_rccl)");
}

inline pnol_ctx* require_ctx() {
    pnol_ctx* c = default_ctx_or_null();
    if (!c) throw std::runtime_error("pnol_amd: no gfx950 (MI355X) device visible; the HIP path has no CPU fallback");
    return c;
}

// device array of doubles
class DevVec {
  public:
    DevVec() = default;
    DevVec(pnol_ctx* ctx, size_t count) { reset(ctx, count); }
    ~DevVec() { release(); }
    DevVec(const DevVec&) = delete;
    DevVec& operator=(const DevVec&) = delete;
    DevVec(DevVec&& o) noexcept : ctx_(o.ctx_), p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
    DevVec& operator=(DevVec&& o) noexcept {
        if (this != &o) { release(); ctx_ = o.ctx_; p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
        return *this;
    }

    void reset(pnol_ctx* ctx, size_t count) {
        release();
        ctx_ = ctx;
        n_ = count;
        void* p = nullptr;
        check(pnol_malloc(ctx, sizeof(double) * (count ? count : 1), &p), "pnol_malloc");
        p_ = static_cast<double*>(p);
    }
    void release() {
        if (p_ && ctx_) pnol_free(ctx_, p_);
        p_ = nullptr;
        n_ = 0;
    }
    double* get() const { return p_; }
    size_t size() const { return n_; }
    void upload(const double* src, size_t count, size_t offset = 0) {
        check(pnol_memcpy_h2d(ctx_, p_ + offset, src, sizeof(double) * count), "h2d");
    }
    void upload(const std::vector<double>& v) { upload(v.data(), v.size()); }
    void download(double* dst, size_t count, size_t offset = 0) const {
        check(pnol_memcpy_d2h(ctx_, dst, p_ + offset, sizeof(double) * count), "d2h");
    }
    void download(std::vector<double>& v) const { download(v.data(), v.size()); }

  private:
    pnol_ctx* ctx_ = nullptr;
    double* p_ = nullptr;
    size_t n_ = 0;
};

inline int even_ld(int n) { return (n + 1) & ~1; }

// Per-phase wall-clock accounting of a solve (extension diagnostics, pnol_run_bfgs_ex): adds
// the seconds of its scope to *acc when acc is set.  Every timed phase ends with its results
// on the host, so host time is the phase's time.
class PhaseClock {
  public:
    explicit PhaseClock(double* acc) : acc_(acc) {
        if (acc_) t0_ = std::chrono::steady_clock::now();
    }
    ~PhaseClock() { stop(); }
    // end the phase early (the destructor then adds nothing)
    void stop() {
        if (acc_) *acc_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0_).count();
        acc_ = nullptr;
    }

  private:
    double* acc_;
    std::chrono::steady_clock::time_point t0_;
};

// PNOL_BND_DETAIL=1: where the host time of the device Recur FD gradient goes (diagnostics):
// the full point / step build, the same-point check, the device call (copies + kernels), the
// host re-evaluations of a reuse, and the gather / cache bookkeeping
enum RecurDetail { kRdBuild = 0, kRdCheck, kRdDevice, kRdRedo, kRdGather, kRdCount };
inline double* recur_detail(int k) {
    static const bool on = [] {
        const char* e = std::getenv("PNOL_BND_DETAIL");
        return e && std::atoi(e) != 0;
    }();
    thread_local double slots[kRdCount];
    return on ? &slots[k] : nullptr;
}

// slots of a solve profile (8 doubles)
enum ProfileSlot { kProfIters = 0, kProfTotal, kProfGrad, kProfLineSearch, kProfUpdate, kProfPoints, kProfGradCalls,
                   kProfDepth };
inline double* prof_slot(double* prof, int k) { return prof ? prof + k : nullptr; }

// reference utility restatements used by the host-side control logic (sequential order,
// identical to the CPU oracle's)
inline double seq_dot(const double* a, const double* b, size_t n) {
    double s = 0.0;
    for (size_t i = 0; i < n; ++i) s = s + a[i] * b[i];
    return s;
}
inline double seq_dot(const std::vector<double>& a, const std::vector<double>& b) {
    return seq_dot(a.data(), b.data(), a.size());
}
// two independent sequential dot products in one loop: each chain is exactly seq_dot's, the two
// dependent add chains just overlap (a host core's add latency, not its throughput, bounds one)
inline void seq_dot2(const std::vector<double>& a1, const std::vector<double>& b1, const std::vector<double>& a2,
                     const std::vector<double>& b2, double& s1, double& s2) {
    const size_t n = a1.size();
    const double *p1 = a1.data(), *q1 = b1.data(), *p2 = a2.data(), *q2 = b2.data();
    double x = 0.0, y = 0.0;
    for (size_t i = 0; i < n; ++i) {
        x = x + p1[i] * q1[i];
        y = y + p2[i] * q2[i];
    }
    s1 = x;
    s2 = y;
}

}  // namespace pnol
