// objective.cpp -- the finite-difference engine of the drop-in Objective / MultiObjective.
//
// Host objectives follow the reference loops (PNOL_Objective.cpp) point by point, handed to
// objEvalBatch in batches of independent points (the default batch is the objEval loop in the
// reference's order); device objectives evaluate every point of a block in one launch.  The
// *MPI forms shard the columns in contiguous ceil(n/P) blocks and assemble with one allgather
// (RCCL over xGMI on GPU ranks) -- the reference's zero-padded Allreduce(SUM) of the function
// values is an allgather in disguise: x + 0 = x for every x but -0.0, which the sum turns into
// +0.0 at P > 1.  Host objectives' values get that same + 0.0 at P > 1 (zero_pad_sum) before
// the differences are formed; the built-in device objectives never produce -0.0 (their sums
// start from +0.0), so the result is the reference's bit for bit at every rank count.
#include <algorithm>
#include <climits>
#include <cstring>

#include "../pnol_comm.hpp"
#include "../pnol_internal.hpp"
#include "PNOL_Objective.hpp"
#include "recur_simd.hpp"
#include "device_util.hpp"
#include "scalar_host.hpp"

using namespace pnol;

namespace {

// points per objEvalBatch call: about 32 MiB of point and result data
int batch_points(int n, int per_out) {
    const size_t per = sizeof(double) * ((size_t)n + (size_t)per_out);
    const size_t cap = ((size_t)32 << 20) / (per ? per : 1);
    return (int)std::max<size_t>(1, std::min<size_t>(cap, INT_MAX / 2));
}

// f(point_k) for k in [0, total) through objEvalBatch, the points formed by make(k, row)
template <class Make>
void batched_eval(Objective* o, int n, int total, Make&& make, double* out) {
    const int chunk = std::min(total, batch_points(n, 1));
    if (total <= 0) return;
    std::vector<double> buf((size_t)chunk * n);
    for (int k = 0; k < total; k += chunk) {
        const int np = std::min(chunk, total - k);
        for (int q = 0; q < np; ++q) make(k + q, buf.data() + (size_t)q * n);
        o->objEvalBatch(buf.data(), np, n, out + k);
    }
}

// the reference's FD points: k == 0 and base -> X; else X + h_i e_i, i = b + k - base
void host_points(Objective* o, const std::vector<double>& X, const std::vector<double>& dX, int b, int cnt, bool base,
                 double* out) {
    const int n = (int)X.size();
    batched_eval(o, n, cnt + (base ? 1 : 0), [&](int k, double* row) {
        std::memcpy(row, X.data(), sizeof(double) * n);
        if (base && k == 0) return;
        const int i = b + k - (base ? 1 : 0);
        row[i] = row[i] + dX[i];   // XdX[i] = XdX[i] + dX[i]
    }, out);
}

// device FD gradient for coordinates [b, b+cnt) (one upload, one launch pair, one download)
void device_gradient(pnol_dobj* d, const std::vector<double>& X, const std::vector<double>& h, int b, int cnt,
                     double* f0, double* g) {
    check(pnol_fd_gradient(require_ctx(), d, X.data(), h.data(), b, cnt, f0, g), "fd_gradient");
}

// scatter a reduced vector into the full one (objEvalRecur's mapping, PNOL_Objective.cpp:311-323)
std::vector<double> scatter_full(const std::vector<double>& Xr, const std::vector<double>& cX,
                                 const std::vector<bool>& cI) {
    std::vector<double> X(cX.size());
    if (recur::free_count(cI) == Xr.size() && !Xr.empty()) {
        recur::scatter(X.data(), Xr, nullptr, 0.0, cX, cI);
        return X;
    }
    size_t ir = 0;
    for (size_t i = 0; i < cX.size(); ++i) X[i] = cI[i] ? cX[i] : Xr[ir++];
    return X;
}

// full index of every free (reduced) coordinate
std::vector<int> free_map(const std::vector<bool>& cI) {
    std::vector<int> map;
    for (size_t i = 0; i < cI.size(); ++i)
        if (!cI[i]) map.push_back((int)i);
    return map;
}

// Recur FD values on the host: objEvalRecur(X) (base) and objEvalRecur(X + dX_i e_i) for the
// reduced coordinates [b, b+cnt), as full points (scatter(X + dX_i e_i) == scatter(X) with
// entry map[i] replaced by X_i + dX_i) through objEvalBatch
void host_points_recur(Objective* o, const std::vector<double>& X, const std::vector<double>& dX, int b, int cnt,
                       const std::vector<double>& cX, const std::vector<bool>& cI, double* out) {
    const std::vector<double> Xf = scatter_full(X, cX, cI);
    const std::vector<int> map = free_map(cI);
    const int nf = (int)Xf.size();
    batched_eval(o, nf, cnt + 1, [&](int k, double* row) {
        std::memcpy(row, Xf.data(), sizeof(double) * nf);
        if (k == 0) return;
        const int i = b + k - 1;
        row[map[i]] = X[i] + dX[i];
    }, out);
}

// the last device Recur gradient: its full point, steps, per-coordinate values and F(x)
struct RecurCache {
    unsigned long long oid = 0;   // pnol_dobj::id (never reused)
    std::vector<double> Xf, hf, gf, pts, fv;
    std::vector<double> p0h, p1h;   // host copies of the objective's data (oid's)
    std::vector<int> redo;
    double F = 0.0;
};
RecurCache& recur_cache() {
    thread_local RecurCache c;
    return c;
}
// above this many changed steps the whole gradient goes to the device again
constexpr size_t kRecurRedoMax = 32;

// what the reference's zero-padded MPI_Allreduce(SUM) returns for a value one rank owns:
// v + 0.0 + ... + 0.0 = v, except -0.0 -> +0.0 (PNOL_Objective.cpp:147-148, 279-286); one rank: v
inline double zero_pad_sum(double v, int P) { return P > 1 ? v + 0.0 : v; }

}  // namespace

// ---- Objective -------------------------------------------------------------------------------

void Objective::objEvalBatch(const double* Xs, int nPts, int n, double* f) {
    std::vector<double> X(n);
    for (int k = 0; k < nPts; ++k) {
        X.assign(Xs + (size_t)k * n, Xs + (size_t)(k + 1) * n);
        f[k] = objEval(X);
    }
}

void Objective::gradientApproximation(vector<double>& X, vector<double>& dX, vector<double>& dFdX) {
    const int N = (int)X.size();
    dFdX.resize(N);
    if (pnol_dobj* d = deviceObjective(N)) {
        double F = 0;
        device_gradient(d, X, dX, 0, N, &F, dFdX.data());
        countEvals(N + 1);
        return;
    }
    std::vector<double> v(N + 1);   // F (base, evaluated first as the reference does), then FdX_i
    host_points(this, X, dX, 0, N, true, v.data());
    const double F = v[0];
    for (int i = 0; i < N; ++i) dFdX[i] = (v[i + 1] - F) / dX[i];
}

void Objective::hessianApproximation(vector<double>& X, vector<double>& dX, vector<vector<double>>& B) {
    // PNOL_Objective.cpp:38-85: F, then per upper-triangle pair (i <= j) the points
    // X + h_i e_i, X + h_j e_j, X + h_i e_i + h_j e_j in that order (the triples batched)
    const int N = (int)X.size();
    B.assign(N, vector<double>(N, 0.0));
    double F = 0;
    {
        std::vector<double> Xc = X;
        objEvalBatch(Xc.data(), 1, N, &F);
    }
    std::vector<std::pair<int, int>> pairs;
    pairs.reserve((size_t)N * (N + 1) / 2);
    for (int i = 0; i < N; ++i)
        for (int j = i; j < N; ++j) pairs.push_back({i, j});
    const int npairs = (int)pairs.size();
    const int chunk = std::max(1, batch_points(N, 1) / 3);
    std::vector<double> pts, f;
    for (int p0 = 0; p0 < npairs; p0 += chunk) {
        const int np = std::min(chunk, npairs - p0);
        pts.assign((size_t)3 * np * N, 0.0);
        f.assign((size_t)3 * np, 0.0);
        for (int q = 0; q < np; ++q) {
            const int i = pairs[p0 + q].first, j = pairs[p0 + q].second;
            double* xi = pts.data() + (size_t)(3 * q) * N;
            double* xj = xi + N;
            double* xij = xj + N;
            std::memcpy(xi, X.data(), sizeof(double) * N);
            std::memcpy(xj, X.data(), sizeof(double) * N);
            std::memcpy(xij, X.data(), sizeof(double) * N);
            xi[i] = xi[i] + dX[i];
            xj[j] = xj[j] + dX[j];
            xij[i] = xij[i] + dX[i];
            xij[j] = xij[j] + dX[j];
        }
        objEvalBatch(pts.data(), 3 * np, N, f.data());
        for (int q = 0; q < np; ++q) {
            const int i = pairs[p0 + q].first, j = pairs[p0 + q].second;
            const double Fi = f[3 * q], Fj = f[3 * q + 1], Fij = f[3 * q + 2];
            B[i][j] = (Fij - Fi - Fj + F) / (dX[i] * dX[j]);
        }
    }
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < i; ++j) B[i][j] = B[j][i];
}

void Objective::gradientApproximationMPI(vector<double>& X, vector<double>& dX, vector<double>& dFdX) {
    require_comm("Objective::gradientApproximationMPI");   // PNOL_Objective.cpp:102-103
    const int N = (int)X.size();
    const int P = comm_size(), r = comm_rank();
    int b = 0, cnt = 0;
    block_range(N, P, r, &b, &cnt);
    const int per = (N + P - 1) / P;
    std::vector<double> mine(per > 0 ? per : 1, 0.0), all((size_t)P * (per > 0 ? per : 1), 0.0);
    if (pnol_dobj* d = deviceObjective(N)) {
        double F = 0;
        device_gradient(d, X, dX, b, cnt, &F, mine.data());
        countEvals(cnt + 1);
    } else {
        // the base point redundantly on every rank (deterministic), then this rank's block
        std::vector<double> v(cnt + 1);
        host_points(this, X, dX, b, cnt, true, v.data());
        const double F = zero_pad_sum(v[0], P);
        for (int q = 0; q < cnt; ++q) mine[q] = (zero_pad_sum(v[q + 1], P) - F) / dX[b + q];
    }
    check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)(per > 0 ? per : 1)), "allgather(gradient)");
    dFdX.resize(N);
    for (int i = 0; i < N; ++i) dFdX[i] = all[i];   // ceil blocks: rank-major == coordinate order
}

double Objective::objEvalRecur(vector<double>& Xrecur, vector<double>& constantX, vector<bool>& constantIndicator) {
    std::vector<double> X = scatter_full(Xrecur, constantX, constantIndicator);
    return objEval(X);
}

void Objective::gradientApproximationRecur(vector<double>& X, vector<double>& dX, vector<double>& dFdX,
                                           vector<double>& constantX, vector<bool>& constantIndicator) {
    const int N = (int)X.size();
    dFdX.resize(N);
    if (pnol_dobj* d = deviceObjective((int)constantX.size())) {
        // full-length point and step: the free coordinate i maps to full index i_f; the
        // perturbed point equals the reference's scatter(X + dX_i e_i) bit for bit.  One pass
        // builds both (frozen coordinates: their constant and a dummy step 1.0), in buffers kept
        // across calls (the bounded solvers call this twice per iteration at full length).
        // recur_simd.hpp: eight entries per AVX-512 expand (the frozen pattern follows the active
        // set, which looks random to a branch predictor; the scalar fallback is branch-free).
        const size_t nf = constantX.size();
        PhaseClock t_build(recur_detail(kRdBuild));
        thread_local std::vector<double> Xf, hf, gf, gr;
        Xf.resize(nf);
        hf.resize(nf);
        gf.resize(nf);
        gr.resize(nf + 1);
        recur::scatter(Xf.data(), X, nullptr, 0.0, constantX, constantIndicator);
        recur::scatter_steps(hf.data(), dX, constantIndicator);
        // Same-point reuse: the bounded solvers' recursion unwinds through one level per frozen
        // coordinate, and every level asks for the gradient at the SAME full point (its free
        // coordinates are a superset of the level below's; BFGS_bnd_linesearch.cpp:620-650).
        // Every value f(x + h_i e_i) is a pure function of the full point and h_i, so a value
        // computed for the same full point and the same h_i by the previous call is the one this
        // call would compute, bit for bit; only coordinates whose step changed (those that were
        // frozen, with the dummy step, in the previous call) are evaluated -- on the host by the
        // library's own copy of the device formula (scalar_host.hpp, the device kernel's bits),
        // never through the overridable objEvalBatch (a user override, or a header objective
        // built with contraction on, could differ in the last place, and 1/h amplifies that).
        // Only kinds whose host formula is bitwise the device's (host_bitwise_kind: PowerObject
        // with power != 2 calls pow, which may not be); the evaluation count is the reference's
        // N + 1.
        t_build.stop();
        PhaseClock t_check(recur_detail(kRdCheck));
        RecurCache& rc = recur_cache();
        const bool pure = host_bitwise_kind(d->kind, d->power);
        std::vector<int>& redo = rc.redo;
        redo.clear();
        bool reuse = pure && rc.oid == d->id && rc.Xf.size() == nf &&
                     std::memcmp(rc.Xf.data(), Xf.data(), sizeof(double) * nf) == 0;
        if (reuse) {
            recur::free_diffs(rc.hf.data(), hf.data(), constantIndicator, kRecurRedoMax, redo);
            reuse = redo.size() <= kRecurRedoMax;
        }
        t_check.stop();
        const double* gsrc = gf.data();   // this call's per-coordinate values
        if (reuse) {
            PhaseClock t_redo(recur_detail(kRdRedo));
            gsrc = rc.gf.data();
            const int k = (int)redo.size();
            if (k > 0) {
                std::vector<double>& pts = rc.pts;
                pts.resize((size_t)k * nf);
                for (int q = 0; q < k; ++q) {
                    double* row = pts.data() + (size_t)q * nf;
                    std::memcpy(row, Xf.data(), sizeof(double) * nf);
                    const int i = redo[q];
                    row[i] = Xf[i] + hf[i];
                }
                rc.fv.resize(k);
                const ScalarTerms st{d->kind, (int)nf, d->power, rc.p0h.data(), rc.p1h.data()};
                scalar_batch(st, pts.data(), k, (int)nf, rc.fv.data());
                for (int q = 0; q < k; ++q) {
                    const int i = redo[q];
                    rc.gf[i] = (rc.fv[q] - rc.F) / hf[i];
                    rc.hf[i] = hf[i];
                }
            }
            countEvals(N + 1);
        } else {
            PhaseClock t_dev(recur_detail(kRdDevice));
            double F = 0;
            device_gradient(d, Xf, hf, 0, (int)nf, &F, gf.data());
            t_dev.stop();
            PhaseClock t_keep(recur_detail(kRdGather));
            countEvals(N + 1);
            if (pure) {
                if (rc.oid != d->id) {   // the objective's data, once per objective
                    rc.p0h.assign(d->len0, 0.0);
                    rc.p1h.assign(d->len1, 0.0);
                    pnol_ctx* c = d->ctx;
                    if (d->len0) check(pnol_memcpy_d2h(c, rc.p0h.data(), d->p0, sizeof(double) * d->len0), "d2h(p0)");
                    if (d->len1) check(pnol_memcpy_d2h(c, rc.p1h.data(), d->p1, sizeof(double) * d->len1), "d2h(p1)");
                }
                rc.oid = d->id;
                // the cache takes the buffers (no 3 x 8n-byte copies per call); the next call
                // refills the thread-local ones
                std::swap(rc.Xf, Xf);
                std::swap(rc.hf, hf);
                std::swap(rc.gf, gf);
                gsrc = rc.gf.data();
                rc.F = F;
                // the quadratic's formula reads d[i], b[i] for every i < n
                if (d->kind == PNOL_OBJ_QUADRATIC && (rc.p0h.size() < nf || rc.p1h.size() < nf)) rc.oid = 0;
            }
        }
        PhaseClock t_gather(recur_detail(kRdGather));
        if (recur::free_count(constantIndicator) == (size_t)N) {
            recur::gather(dFdX.data(), gsrc, constantIndicator);
        } else {   // a fallback walk's mismatched lengths: the scalar gather, slot for slot
            size_t ir = 0;
            for (size_t i = 0; i < nf; ++i) {
                gr[ir] = gsrc[i];
                ir += !constantIndicator[i];
            }
            std::copy(gr.begin(), gr.begin() + N, dFdX.begin());
        }
        return;
    }
    std::vector<double> v(N + 1);
    host_points_recur(this, X, dX, 0, N, constantX, constantIndicator, v.data());
    for (int i = 0; i < N; ++i) dFdX[i] = (v[i + 1] - v[0]) / dX[i];
}

void Objective::gradientApproximationMPIRecur(vector<double>& X, vector<double>& dX, vector<double>& dFdX,
                                              vector<double>& constantX, vector<bool>& constantIndicator) {
    // PNOL_Objective.cpp:366-459: same values as the serial Recur gradient, points sharded
    require_comm("Objective::gradientApproximationMPIRecur");
    const int N = (int)X.size();
    const int P = comm_size(), r = comm_rank();
    int b = 0, cnt = 0;
    block_range(N, P, r, &b, &cnt);
    const int per = (N + P - 1) / P > 0 ? (N + P - 1) / P : 1;
    std::vector<double> mine(per, 0.0), all((size_t)P * per, 0.0);
    if (pnol_dobj* d = deviceObjective((int)constantX.size())) {
        // the rank's free coordinates [b, b+cnt) span full indices [map[b], map[b+cnt-1]]: one
        // batched launch over that span (frozen coordinates inside it are evaluated and dropped)
        std::vector<double> Xf = scatter_full(X, constantX, constantIndicator);
        std::vector<double> hf(Xf.size(), 1.0);
        const std::vector<int> map = free_map(constantIndicator);
        for (int i = 0; i < N; ++i) hf[map[i]] = dX[i];
        if (cnt > 0) {
            const int f0i = map[b], span = map[b + cnt - 1] - f0i + 1;
            std::vector<double> gs(span);
            double F = 0;
            device_gradient(d, Xf, hf, f0i, span, &F, gs.data());
            for (int q = 0; q < cnt; ++q) mine[q] = gs[map[b + q] - f0i];
        }
        countEvals(cnt + 1);
    } else {
        std::vector<double> v(cnt + 1);
        host_points_recur(this, X, dX, b, cnt, constantX, constantIndicator, v.data());
        const double F = zero_pad_sum(v[0], P);
        for (int q = 0; q < cnt; ++q) mine[q] = (zero_pad_sum(v[q + 1], P) - F) / dX[b + q];
    }
    check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)per), "allgather(gradient recur)");
    dFdX.resize(N);
    for (int i = 0; i < N; ++i) dFdX[i] = all[i];
}

// ---- MultiObjective --------------------------------------------------------------------------

void MultiObjective::objEvalBatch(const double* Xs, int nPts, int n, double* F, int m) {
    std::vector<double> X(n), Fk(m);
    for (int k = 0; k < nPts; ++k) {
        X.assign(Xs + (size_t)k * n, Xs + (size_t)(k + 1) * n);
        objEval(X, Fk);
        std::memcpy(F + (size_t)k * m, Fk.data(), sizeof(double) * m);
    }
}

namespace {

// JT block rows [b, b+cnt) (ld = m) of a host multi-objective; F0 the base residuals.  The
// columns go to objEvalBatch in batches.
void host_jacobian_block(MultiObjective* o, std::vector<double>& X, std::vector<double>& dX, int m, int b, int cnt,
                         const std::vector<double>& F0, double* JT, int P = 1) {
    const int n = (int)X.size();
    const int chunk = std::max(1, std::min(cnt, batch_points(n, m)));
    std::vector<double> pts((size_t)chunk * n), FdX((size_t)chunk * m);
    for (int q0 = 0; q0 < cnt; q0 += chunk) {
        const int np = std::min(chunk, cnt - q0);
        for (int q = 0; q < np; ++q) {
            double* row = pts.data() + (size_t)q * n;
            std::memcpy(row, X.data(), sizeof(double) * n);
            const int j = b + q0 + q;
            row[j] = row[j] + dX[j];
        }
        o->objEvalBatch(pts.data(), np, n, FdX.data(), m);
        for (int q = 0; q < np; ++q) {
            const int j = b + q0 + q;
            const double* Fj = FdX.data() + (size_t)q * m;
            double* dst = JT + (size_t)(q0 + q) * m;
            for (int i = 0; i < m; ++i) dst[i] = (zero_pad_sum(Fj[i], P) - zero_pad_sum(F0[i], P)) / dX[j];
        }
    }
}

void base_residuals(MultiObjective* o, std::vector<double>& X, std::vector<double>& F) {
    o->objEvalBatch(X.data(), 1, (int)X.size(), F.data(), (int)F.size());
}

void device_jacobian(pnol_dobj* d, const std::vector<double>& X, const std::vector<double>& h, int m, bool sharded,
                     std::vector<double>& JT /* n x m */) {
    pnol_ctx* ctx = require_ctx();
    const int n = (int)X.size();
    const int P = sharded ? comm_size() : 1, r = sharded ? comm_rank() : 0;
    int b = 0, cnt = 0;
    block_range(n, P, r, &b, &cnt);
    const int per = (n + P - 1) / P;
    DevVec dx(ctx, n), dh(ctx, n), dF0(ctx, m), dJT(ctx, (size_t)P * per * m);
    dx.upload(X);
    dh.upload(h);
    check(pnol_fd_jacobian_d(ctx, d, dx.get(), dh.get(), b, cnt, dF0.get(), 1, dJT.get() + (size_t)b * m, m),
          "fd_jacobian");
    if (P > 1)
        check(comm_allgather_device(ctx, dJT.get() + (size_t)r * per * m, dJT.get(), (size_t)per * m),
              "allgather(jacobian)");
    JT.resize((size_t)n * m);
    dJT.download(JT.data(), JT.size());
}

}  // namespace

void MultiObjective::gradientApproximation(vector<double>& X, vector<double>& dX, vector<vector<double>>& J) {
    const int n = (int)X.size();
    const int m = (int)J.size();
    std::vector<double> JT((size_t)n * m);
    if (pnol_dobj* d = deviceObjective()) {
        device_jacobian(d, X, dX, m, false, JT);
        countEvals(n + 1);
    } else {
        std::vector<double> F(m);
        base_residuals(this, X, F);
        host_jacobian_block(this, X, dX, m, 0, n, F, JT.data());
    }
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) J[i][j] = JT[(size_t)j * m + i];
}

void MultiObjective::gradientApproximationMPI(vector<double>& X, vector<double>& dX, vector<vector<double>>& J) {
    require_comm("MultiObjective::gradientApproximationMPI");   // PNOL_Objective.cpp:227-228
    const int n = (int)X.size();
    const int m = (int)J.size();
    std::vector<double> JT((size_t)n * m);
    if (pnol_dobj* d = deviceObjective()) {
        device_jacobian(d, X, dX, m, true, JT);
        int b = 0, cnt = 0;
        block_range(n, comm_size(), comm_rank(), &b, &cnt);
        countEvals(cnt + 1);
    } else {
        const int P = comm_size(), r = comm_rank();
        int b = 0, cnt = 0;
        block_range(n, P, r, &b, &cnt);
        const int per = (n + P - 1) / P > 0 ? (n + P - 1) / P : 1;
        std::vector<double> F(m), mine((size_t)per * m, 0.0), all((size_t)P * per * m, 0.0);
        base_residuals(this, X, F);   // base residuals, redundantly per rank
        host_jacobian_block(this, X, dX, m, b, cnt, F, mine.data(), P);
        check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)per * m), "allgather(jacobian)");
        std::memcpy(JT.data(), all.data(), sizeof(double) * JT.size());
    }
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) J[i][j] = JT[(size_t)j * m + i];
}
