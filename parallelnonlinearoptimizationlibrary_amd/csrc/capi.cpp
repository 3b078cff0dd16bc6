// capi.cpp -- extern "C" kernel-level entry points of libpnol_amd.so (see include/pnol_amd.h).
// Argument checking happens here and in the launchers; every function returns a status.
#include <cmath>
#include <cstring>
#include <vector>

#include <algorithm>

#include "pnol_comm.hpp"
#include "pnol_internal.hpp"

using namespace pnol;

namespace {

int set_device(pnol_ctx* ctx) {
    if (!ctx) return PNOL_ERR_ARG;
    PNOL_HIP(hipSetDevice(ctx->device));
    return PNOL_OK;
}

}  // namespace

extern "C" {

int pnol_hg_d(pnol_ctx* ctx, const double* D, int ldd, const double* g, double* p, int n) {
    PNOL_CHECK(set_device(ctx));
    ScopedTimer tm(ctx, "hg");
    if (n <= PNOL_SEQ_MAX) return launch_gemv_neg_seq(ctx, D, ldd, n, n, g, p);
    return launch_gemv_neg(ctx, D, ldd, n, n, g, p);
}

int pnol_gemv_neg_d(pnol_ctx* ctx, const double* A, int lda, int rows, int cols, const double* x, double* y) {
    PNOL_CHECK(set_device(ctx));
    return launch_gemv_neg(ctx, A, lda, rows, cols, x, y);
}

int pnol_bfgs_update_exact_d(pnol_ctx* ctx, double* D, int ldd, const double* y, const double* s, int n) {
    PNOL_CHECK(set_device(ctx));
    return launch_bfgs_update_exact(ctx, D, ldd, y, s, n);
}

int pnol_bfgs_pass_d(pnol_ctx* ctx, double* D, int ldd, int n, const double* s_p, const double* a_p,
                     const double* b_p, int write_back, const double* y, const double* g, double* u, double* w,
                     double* v) {
    PNOL_CHECK(set_device(ctx));
    ScopedTimer tm(ctx, "bfgs_pass");
    return launch_bfgs_pass(ctx, D, ldd, n, s_p, a_p, b_p, write_back, y, g, u, w, v);
}

int pnol_bfgs_pass_ident_d(pnol_ctx* ctx, double* D, int ldd, int n, const double* scale, const double* s_p,
                           const double* a_p, const double* b_p, const double* y, const double* g, double* u, double* w,
                           double* v) {
    PNOL_CHECK(set_device(ctx));
    if (!s_p || !a_p || !b_p) return PNOL_ERR_ARG;
    ScopedTimer tm(ctx, "bfgs_pass");
    return launch_bfgs_pass(ctx, D, ldd, n, s_p, a_p, b_p, 1, y, g, u, w, v, 0, -1, nullptr, 1, scale);
}

int pnol_set_identity_d(pnol_ctx* ctx, double* D, int ldd, int n, const double* scale) {
    PNOL_CHECK(set_device(ctx));
    return launch_set_identity(ctx, D, ldd, n, scale);
}

int pnol_matrix_inverse_d(pnol_ctx* ctx, const double* B, int ldb, int n, double* Binv, int ldi, int* info) {
    PNOL_CHECK(set_device(ctx));
    ScopedTimer tm(ctx, "matrix_inverse");
    return launch_matrix_inverse(ctx, B, ldb, n, Binv, ldi, info);
}

int pnol_add_d(pnol_ctx* ctx, const double* x, const double* y, double* z, int n) {
    PNOL_CHECK(set_device(ctx));
    return launch_add(ctx, x, y, z, n);
}

int pnol_solve_async_d(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo) {
    PNOL_CHECK(set_device(ctx));
    if (!A || !rhs || !sigma || !dinfo || n <= 0 || lda < n) return PNOL_ERR_ARG;
    ScopedTimer tm(ctx, "solve");
    return launch_chol_solve(ctx, A, lda, rhs, sigma, n, dinfo);
}

int pnol_solve_step_d(pnol_ctx* ctx, const double* A, int lda, const double* rhs, double* sigma, int n, int* dinfo,
                      const double* x, double* xnext) {
    PNOL_CHECK(set_device(ctx));
    if (!A || !rhs || !sigma || !dinfo || !x || !xnext || n <= 0 || lda < n) return PNOL_ERR_ARG;
    ScopedTimer tm(ctx, "solve");
    return launch_chol_solve(ctx, A, lda, rhs, sigma, n, dinfo, x, xnext);
}

int pnol_gather_submatrix_d(pnol_ctx* ctx, const double* D, int ldd, int n, const int* idx, int nsub,
                            double* Dsub, int lds) {
    PNOL_CHECK(set_device(ctx));
    return launch_gather_sub(ctx, D, ldd, n, idx, nsub, Dsub, lds);
}

int pnol_jtj_d(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
               double* jtj_diag) {
    PNOL_CHECK(set_device(ctx));
    return launch_jtj(ctx, JT, ldjt, m, n, lambda, A, lda, jtj_diag);
}

// ---- BFGS D row-sharded over the communicator ----------------------------
static int bfgs_rows_per(int n, int P) {
    const int per = (n + P - 1) / P;
    return (per + 255) / 256 * 256;   // whole fused-pass row tiles (bfgs_pass_rows divides 256)
}

}  // extern "C" (reopened below)

extern "C" int pnol_bfgs_rows(int n, int nranks, int rank, int* begin, int* count) {
    if (n <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || !begin || !count) return PNOL_ERR_ARG;
    const int per = bfgs_rows_per(n, nranks);
    *begin = std::min(n, rank * per);
    *count = std::min(n, *begin + per) - *begin;
    return PNOL_OK;
}

extern "C" int pnol_bfgs_pass_part_tiles(int n, int nranks) {
    if (n <= 0 || nranks <= 0) return 0;
    const int prows = bfgs_pass_rows(n);
    const int whole = (n + prows - 1) / prows;
    const int gathered = nranks * (bfgs_rows_per(n, nranks) / prows);
    return std::max(whole, gathered);
}

namespace {

// part_w of the fused pass: every rank's row tiles, in place (rank r's tiles at r * tiles_per)
int pass_w_allgather(pnol_ctx* ctx, double* part_w, int n, int nrowt) {
    (void)nrowt;
    const int P = comm_size(), r = comm_rank();
    const size_t cnt = (size_t)(bfgs_rows_per(n, P) / bfgs_pass_rows(n)) * n;
    return comm_allgather_device(ctx, part_w + (size_t)r * cnt, part_w, cnt);
}

// full n-vector from per-rank row shards written in place at global offsets of buf
// (buf holds P * rows_per doubles), then copied to out
int rows_allgather(pnol_ctx* ctx, double* buf, int n, double* out) {
    const int P = comm_size(), r = comm_rank();
    const size_t per = (size_t)bfgs_rows_per(n, P);
    PNOL_CHECK(comm_allgather_device(ctx, buf + (size_t)r * per, buf, per));
    if (out) PNOL_HIP(hipMemcpyAsync(out, buf, sizeof(double) * n, hipMemcpyDeviceToDevice, ctx->stream));
    return PNOL_OK;
}

}  // namespace

extern "C" {

int pnol_set_identity_rows_d(pnol_ctx* ctx, double* Dsh, int ldd, int n, const double* scale) {
    PNOL_CHECK(set_device(ctx));
    int b = 0, c = 0;
    PNOL_CHECK(pnol_bfgs_rows(n, comm_size(), comm_rank(), &b, &c));
    return launch_set_identity(ctx, Dsh, ldd, n, scale, b, b + c);
}

int pnol_gather_submatrix_mpi_d(pnol_ctx* ctx, const double* D, int ldd, int n, const int* idx, int nsub,
                                double* Dsub, int lds) {
    PNOL_CHECK(set_device(ctx));
    if (!idx || nsub <= 0 || nsub > n || lds < nsub || ldd < n) return PNOL_ERR_ARG;
    for (int a = 0; a < nsub; ++a)
        if (idx[a] < 0 || idx[a] >= n || (a > 0 && idx[a] <= idx[a - 1])) return PNOL_ERR_ARG;
    const int P = comm_size(), me = comm_rank();
    // kept rows of old shard q: the new indices [a0[q], a1[q]) (contiguous: idx is ascending)
    std::vector<int> a0(P), a1(P), nb(P), nc(P);
    for (int q = 0; q < P; ++q) {
        int ob = 0, oc = 0;
        PNOL_CHECK(pnol_bfgs_rows(n, P, q, &ob, &oc));
        a0[q] = (int)(std::lower_bound(idx, idx + nsub, ob) - idx);
        a1[q] = (int)(std::lower_bound(idx, idx + nsub, ob + oc) - idx);
        PNOL_CHECK(pnol_bfgs_rows(nsub, P, q, &nb[q], &nc[q]));
    }
    int ob = 0, oc = 0;
    PNOL_CHECK(pnol_bfgs_rows(n, P, me, &ob, &oc));
    if (a1[me] > a0[me] && !D) return PNOL_ERR_ARG;
    if (nc[me] > 0 && !Dsub) return PNOL_ERR_ARG;
    void *di = nullptr, *pk = nullptr;
    PNOL_CHECK(ws_get(ctx, "subm_idx", sizeof(int) * (size_t)nsub, &di));
    PNOL_CHECK(pnol_memcpy_h2d(ctx, di, idx, sizeof(int) * (size_t)nsub));
    const int mine = a1[me] - a0[me];
    PNOL_CHECK(ws_get(ctx, "subm_pack", sizeof(double) * (size_t)std::max(mine, 1) * lds, &pk));
    double* pack = (double*)pk;
    PNOL_CHECK(launch_gather_rows(ctx, D, ldd, (const int*)di + a0[me], mine, ob, (const int*)di, nsub, pack, lds));
    // rows this rank keeps for itself
    const int slo = std::max(a0[me], nb[me]), shi = std::min(a1[me], nb[me] + nc[me]);
    if (shi > slo)
        PNOL_HIP(hipMemcpyAsync(Dsub + (size_t)(slo - nb[me]) * lds, pack + (size_t)(slo - a0[me]) * lds,
                                sizeof(double) * (size_t)(shi - slo) * lds, hipMemcpyDeviceToDevice, ctx->stream));
    if (P == 1) return PNOL_OK;
    return comm_exchange(ctx, pack, Dsub, [&](int q, int d, std::vector<XBlock>& bl) {
        bl.clear();
        const int lo = std::max(a0[q], nb[d]), hi = std::min(a1[q], nb[d] + nc[d]);
        if (hi > lo)
            bl.push_back({(size_t)(lo - a0[q]) * lds, (size_t)(lo - nb[d]) * lds, (size_t)(hi - lo) * lds});
    });
}

int pnol_hg_mpi_d(pnol_ctx* ctx, const double* Dsh, int ldd, const double* g, double* p, int n) {
    PNOL_CHECK(set_device(ctx));
    if (!Dsh || !g || !p || n <= 0 || ldd < n) return PNOL_ERR_ARG;
    const int P = comm_size();
    int b = 0, c = 0;
    PNOL_CHECK(pnol_bfgs_rows(n, P, comm_rank(), &b, &c));
    ScopedTimer tm(ctx, "hg");
    void* buf = nullptr;
    PNOL_CHECK(ws_get(ctx, "hg_rows", sizeof(double) * (size_t)P * bfgs_rows_per(n, P), &buf));
    double* pb = (double*)buf;
    if (c > 0) PNOL_CHECK(launch_gemv_neg(ctx, Dsh, ldd, c, n, g, pb + b));   // row i: the whole-matrix order
    return rows_allgather(ctx, pb, n, p);
}

int pnol_bfgs_pass_mpi_d(pnol_ctx* ctx, double* Dsh, int ldd, int n, const double* s_p, const double* a_p,
                         const double* b_p, int write_back, const double* y, const double* g, double* u, double* w,
                         double* v) {
    PNOL_CHECK(set_device(ctx));
    const int P = comm_size();
    int b = 0, c = 0;
    PNOL_CHECK(pnol_bfgs_rows(n, P, comm_rank(), &b, &c));
    ScopedTimer tm(ctx, "bfgs_pass");
    const size_t span = (size_t)P * bfgs_rows_per(n, P);
    void *ub = nullptr, *vb = nullptr;
    PNOL_CHECK(ws_get(ctx, "pass_rows_u", sizeof(double) * span, &ub));
    PNOL_CHECK(ws_get(ctx, "pass_rows_v", sizeof(double) * span, &vb));
    PNOL_CHECK(launch_bfgs_pass(ctx, Dsh, ldd, n, s_p, a_p, b_p, write_back, y, g, u ? (double*)ub : nullptr, w,
                                v ? (double*)vb : nullptr, b, b + c, P > 1 ? pass_w_allgather : nullptr));
    if (u) PNOL_CHECK(rows_allgather(ctx, (double*)ub, n, u));
    if (v) PNOL_CHECK(rows_allgather(ctx, (double*)vb, n, v));
    return PNOL_OK;
}

int pnol_bfgs_pass_ident_mpi_d(pnol_ctx* ctx, double* Dsh, int ldd, int n, const double* scale, const double* s_p,
                               const double* a_p, const double* b_p, const double* y, const double* g, double* u,
                               double* w, double* v) {
    PNOL_CHECK(set_device(ctx));
    if (!s_p || !a_p || !b_p) return PNOL_ERR_ARG;
    const int P = comm_size();
    int b = 0, c = 0;
    PNOL_CHECK(pnol_bfgs_rows(n, P, comm_rank(), &b, &c));
    ScopedTimer tm(ctx, "bfgs_pass");
    const size_t span = (size_t)P * bfgs_rows_per(n, P);
    void *ub = nullptr, *vb = nullptr;
    PNOL_CHECK(ws_get(ctx, "pass_rows_u", sizeof(double) * span, &ub));
    PNOL_CHECK(ws_get(ctx, "pass_rows_v", sizeof(double) * span, &vb));
    PNOL_CHECK(launch_bfgs_pass(ctx, Dsh, ldd, n, s_p, a_p, b_p, 1, y, g, u ? (double*)ub : nullptr, w,
                                v ? (double*)vb : nullptr, b, b + c, P > 1 ? pass_w_allgather : nullptr, 1, scale));
    if (u) PNOL_CHECK(rows_allgather(ctx, (double*)ub, n, u));
    if (v) PNOL_CHECK(rows_allgather(ctx, (double*)vb, n, v));
    return PNOL_OK;
}

int pnol_jtj_mpi_d(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, double lambda, double* A, int lda,
                   double* jtj_diag) {
    PNOL_CHECK(set_device(ctx));
    return launch_jtj_sharded(ctx, JT, ldjt, m, n, lambda, A, lda, jtj_diag);
}

int pnol_lm_sliced_layout(int m, int n, int* slice_rows, size_t* jt_elems) {
    static_assert(PNOL_LM_SLICES == kLmSlices, "slice count");
    if (m <= 0 || n <= 0) return PNOL_ERR_ARG;
    const int mS = lm_slice_rows(m);
    if (slice_rows) *slice_rows = mS;
    if (jt_elems) *jt_elems = (size_t)kLmSlices * n * mS;
    return PNOL_OK;
}

int pnol_lm_jacobian_mpi_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0,
                           int compute_f0, double* JTs) {
    PNOL_CHECK(set_device(ctx));
    if (!obj || !x || !h || !F0 || !JTs || compute_f0 < 0 || compute_f0 > 3) return PNOL_ERR_ARG;
    return launch_lm_jacobian(ctx, obj, x, h, F0, compute_f0, JTs);
}

int pnol_lm_set_fd_mode(pnol_ctx* ctx, int mode) {
    if (!ctx || mode < -1 || mode > 1) return PNOL_ERR_ARG;
    ctx->lm_fd_mode = mode < 0 ? lm_fd_mode_env() : mode;
    ctx->lm_fd_mode_set = mode >= 0;
    return PNOL_OK;
}

int pnol_lm_fd_mode(pnol_ctx* ctx, int* mode) {
    if (!ctx || !mode) return PNOL_ERR_ARG;
    *mode = lm_rows_mode(ctx) ? 1 : 0;
    return PNOL_OK;
}

int pnol_lm_rank_rows(int m, int nranks, int rank, int* r0, int* r1) {
    if (m <= 0 || nranks < 1 || nranks > kLmSlices || rank < 0 || rank >= nranks || !r0 || !r1) return PNOL_ERR_ARG;
    const int mS = lm_slice_rows(m);
    int s0 = 0, s1 = 0;
    lm_rank_slices(nranks, rank, &s0, &s1);
    *r0 = std::min(m, s0 * mS);
    *r1 = std::min(m, s1 * mS);
    return PNOL_OK;
}

int pnol_lm_eval_mpi_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, double* F) {
    PNOL_CHECK(set_device(ctx));
    if (!obj || !x || !F) return PNOL_ERR_ARG;
    return launch_lm_eval(ctx, obj, x, F);
}

int pnol_lm_normal_mpi_d(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F, double* A,
                         int lda, double* rhs, double* jtj_diag) {
    PNOL_CHECK(set_device(ctx));
    return launch_lm_normal(ctx, JTs, m, n, lambda, F, A, lda, rhs, jtj_diag);
}

int pnol_lm_normal_solve_mpi_d(pnol_ctx* ctx, const double* JTs, int m, int n, double lambda, const double* F,
                               double* rhs, double* sigma, int* dinfo, const double* x, double* xnext) {
    PNOL_CHECK(set_device(ctx));
    if (!JTs || !F || !rhs || !x || m <= 0) return PNOL_ERR_ARG;
    return launch_lm_normal_solve(ctx, JTs, m, n, lambda, F, rhs, sigma, dinfo, x, xnext);
}

int pnol_lm_normal_unpack_mpi_d(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda) {
    PNOL_CHECK(set_device(ctx));
    return launch_lm_normal_unpack(ctx, m, n, lambda, A, lda);
}

int pnol_lm_agree_status_d(pnol_ctx* ctx, int* dinfo) {
    PNOL_CHECK(set_device(ctx));
    if (!dinfo) return PNOL_ERR_ARG;
    return launch_status_agree(ctx, dinfo);
}

int pnol_jtr_d(pnol_ctx* ctx, const double* JT, int ldjt, int m, int n, const double* F, double* rhs) {
    PNOL_CHECK(set_device(ctx));
    if (!JT || !F || !rhs || m <= 0 || n <= 0 || ldjt < m) return PNOL_ERR_ARG;
    ScopedTimer tm(ctx, "jtr");
    return launch_jtr(ctx, JT, ldjt, m, n, F, rhs);
}

int pnol_solve_d(pnol_ctx* ctx, double* A, int lda, const double* rhs, double* sigma, int n, int method, int* info) {
    PNOL_CHECK(set_device(ctx));
    if (method < 0 || method > 5) return PNOL_ERR_ARG;
    ScopedTimer tm(ctx, "solve");
    return launch_solve(ctx, A, lda, rhs, sigma, n, method, info);
}

int pnol_dobj_create(pnol_ctx* ctx, int kind, int n, int m, const double* host_p0, size_t len0,
                     const double* host_p1, size_t len1, double power, pnol_dobj** out) {
    PNOL_CHECK(set_device(ctx));
    if (!out || n <= 0) return PNOL_ERR_ARG;
    *out = nullptr;
    switch (kind) {
        case PNOL_OBJ_ROSENBROCK: case PNOL_OBJ_POWER: break;
        case PNOL_OBJ_QUADRATIC:
            if (!host_p0 || !host_p1 || len0 < (size_t)n || len1 < (size_t)n) return PNOL_ERR_ARG;
            break;
        case PNOL_OBJ_EXPCURVE: case PNOL_OBJ_CUBIC:
            if (m <= 0 || !host_p0 || !host_p1 || len0 < (size_t)m || len1 < (size_t)m) return PNOL_ERR_ARG;
            if ((kind == PNOL_OBJ_EXPCURVE && n != 3) || (kind == PNOL_OBJ_CUBIC && n != 4)) return PNOL_ERR_ARG;
            break;
        case PNOL_OBJ_LINRES:
            if (m <= 0 || !host_p0 || !host_p1 || len0 < (size_t)m * n || len1 < (size_t)m) return PNOL_ERR_ARG;
            break;
        default:
            return PNOL_ERR_UNSUPPORTED;
    }
    auto* o = new pnol_dobj();
    o->kind = kind; o->n = n; o->m = m; o->power = power; o->ctx = ctx; o->device = ctx->device;
    o->len0 = len0; o->len1 = len1;
    auto upload = [&](const double* src, size_t len, double** dst) -> int {
        if (!src || !len) return PNOL_OK;
        if (hipMalloc(dst, sizeof(double) * len) != hipSuccess) return PNOL_ERR_NOMEM;
        PNOL_HIP(hipMemcpy(*dst, src, sizeof(double) * len, hipMemcpyHostToDevice));
        return PNOL_OK;
    };
    int st = upload(host_p0, len0, &o->p0);
    if (st == PNOL_OK) st = upload(host_p1, len1, &o->p1);
    if (st == PNOL_OK && kind == PNOL_OBJ_CUBIC) {
        // CubicObjective evaluates pow(xData[k],3) every call (ExampleObjectives.hpp:175); it only
        // depends on the data, so tabulate it once with the host libm the reference uses.
        std::vector<double> p3(m);
        for (int k = 0; k < m; ++k) p3[k] = std::pow(host_p0[k], 3.0);
        st = upload(p3.data(), (size_t)m, &o->p2);
    }
    if (st != PNOL_OK) {
        pnol_dobj_destroy(o);
        return st;
    }
    *out = o;
    return PNOL_OK;
}

int pnol_dobj_create_synthetic(pnol_ctx* ctx, int kind, int n, int m, unsigned long long seed, double bscale,
                               double* xstar_out, pnol_dobj** out) {
    PNOL_CHECK(set_device(ctx));
    if (!out || n <= 0) return PNOL_ERR_ARG;
    *out = nullptr;
    auto* o = new pnol_dobj();
    o->kind = kind; o->n = n; o->m = m; o->ctx = ctx; o->device = ctx->device;
    int st = PNOL_OK;
    if (kind == PNOL_OBJ_QUADRATIC) {
        if (hipMalloc(&o->p0, sizeof(double) * n) != hipSuccess || hipMalloc(&o->p1, sizeof(double) * n) != hipSuccess)
            st = PNOL_ERR_NOMEM;
        o->len0 = o->len1 = (size_t)n;
        if (st == PNOL_OK) st = launch_synthetic_quadratic(ctx, seed, n, bscale, o->p0, o->p1);
    } else if (kind == PNOL_OBJ_LINRES) {
        if (m <= 0) st = PNOL_ERR_ARG;
        double* xs = nullptr;
        if (st == PNOL_OK &&
            (hipMalloc(&o->p0, sizeof(double) * (size_t)m * n) != hipSuccess ||
             hipMalloc(&o->p1, sizeof(double) * (size_t)m) != hipSuccess || hipMalloc(&xs, sizeof(double) * n) != hipSuccess))
            st = PNOL_ERR_NOMEM;
        o->len0 = (size_t)m * n; o->len1 = (size_t)m;
        if (st == PNOL_OK) st = launch_synthetic_linres(ctx, seed, m, n, o->p0, xs, o->p1);
        if (st == PNOL_OK && xstar_out) {
            if (hipMemcpyAsync(xstar_out, xs, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
                st = PNOL_ERR_HIP;
        }
        if (const int w = stream_wait(ctx->stream)) st = w;
        if (xs) (void)hipFree(xs);
    } else {
        st = PNOL_ERR_UNSUPPORTED;
    }
    if (st == PNOL_OK) st = stream_wait(ctx->stream);
    if (st != PNOL_OK) {
        pnol_dobj_destroy(o);
        return st;
    }
    *out = o;
    return PNOL_OK;
}

int pnol_dobj_destroy(pnol_dobj* o) {
    if (!o) return PNOL_ERR_ARG;
    (void)hipSetDevice(o->device);
    if (o->p0) (void)hipFree(o->p0);
    if (o->p1) (void)hipFree(o->p1);
    if (o->p2) (void)hipFree(o->p2);
    if (o->at) (void)hipFree(o->at);
    (void)hipGetLastError();   // a failed clean-up call must not surface at the next launch check
    delete o;
    return PNOL_OK;
}

int pnol_dobj_info(pnol_dobj* o, int* kind, int* n, int* m) {
    if (!o) return PNOL_ERR_ARG;
    if (kind) *kind = o->kind;
    if (n) *n = o->n;
    if (m) *m = o->m;
    return PNOL_OK;
}

int pnol_dobj_eval_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, double* out) {
    PNOL_CHECK(set_device(ctx));
    return launch_dobj_eval(ctx, obj, x, out);
}

int pnol_dobj_eval_ckpt_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, double* out) {
    PNOL_CHECK(set_device(ctx));
    return launch_dobj_eval_ckpt(ctx, obj, x, out);
}

int pnol_fd_gradient_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, int i0, int cnt,
                       double* f0, double* g) {
    PNOL_CHECK(set_device(ctx));
    ScopedTimer tm(ctx, "fd_gradient");
    return launch_fd_gradient(ctx, obj, x, h, i0, cnt, f0, g);
}

// Host-pointer forms for the C++ classes' per-iteration calls: the context's scratch and
// pinned staging, one upload and one download per call (no allocation, one stream sync).
int pnol_fd_gradient(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, int i0, int cnt, double* f0,
                     double* g) {
    PNOL_CHECK(set_device(ctx));
    if (!obj || !x || !h || !f0 || (cnt > 0 && !g) || cnt < 0 || i0 < 0 || i0 + cnt > obj->n) return PNOL_ERR_ARG;
    // device block [x | h | g | f0] and its pinned image [x | h | g | f0]: the kernels read x from
    // the pinned image and write g and f0 into it (zero-copy); h goes up only when it changed.
    // Sized by n alone (cnt <= n), so a span that changes between calls does not regrow it
    const size_t n = (size_t)obj->n, io = 3 * n + 1;
    void* dv = nullptr;
    bool fresh = false;
    PNOL_CHECK(ws_get(ctx, "fdg_io", sizeof(double) * io, &dv, &fresh));
    if (fresh) ctx->fdg_h_dev = nullptr;   // the device copy of h is gone
    double* dx = (double*)dv;
    double *dh = dx + n, *dg = dx + 2 * n, *df = dg + cnt;
    double* st = (double*)pinned_stage(ctx, sizeof(double) * io);
    if (!st) {
        // larger than the pinned staging block: pageable copies straight from / to the caller
        ctx->fdg_h_dev = nullptr;
        PNOL_HIP(hipMemcpyAsync(dx, x, sizeof(double) * n, hipMemcpyHostToDevice, ctx->stream));
        PNOL_HIP(hipMemcpyAsync(dh, h, sizeof(double) * n, hipMemcpyHostToDevice, ctx->stream));
        {
            ScopedTimer tm(ctx, "fd_gradient");
            PNOL_CHECK(launch_fd_gradient(ctx, obj, dx, dh, i0, cnt, df, dg));
        }
        if (cnt > 0) PNOL_HIP(hipMemcpyAsync(g, dg, sizeof(double) * cnt, hipMemcpyDeviceToHost, ctx->stream));
        PNOL_HIP(hipMemcpyAsync(f0, df, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        PNOL_CHECK(stream_wait(ctx->stream));
        return PNOL_OK;
    }
    std::memcpy(st, x, sizeof(double) * n);
    // the step vector rarely changes between calls (a solver's dX): it is staged and sent only
    // when its content differs from the device's copy (one memcmp of the whole vector)
    bool same = ctx->fdg_h_dev == dh && ctx->fdg_h_host.size() == n &&
                std::memcmp(h, ctx->fdg_h_host.data(), sizeof(double) * n) == 0;
    if (!same) {   // the steps changed: the terms kernel brings them up with x (no copy command)
        std::memcpy(st + n, h, sizeof(double) * n);
        ctx->fdg_h_dev = nullptr;   // until the launch below has been queued
    }
    {
        // zero-copy: the terms kernel reads x (and a changed h) from the pinned block and copies
        // them to dx / dh for the chain, the finish writes g and f0 straight into it -- no copy
        // commands, no copy gaps (the bounded solvers' step vector changes with the active set,
        // i.e. on nearly every cfg-5 iteration)
        ScopedTimer tm(ctx, "fd_gradient");
        PNOL_CHECK(launch_fd_gradient(ctx, obj, st, dh, i0, cnt, st + 2 * n + cnt, st + 2 * n, dx,
                                      same ? nullptr : st + n));
    }
    if (!same) {
        ctx->fdg_h_host.assign(h, h + n);
        ctx->fdg_h_dev = dh;
    }
    PNOL_CHECK(stream_wait(ctx->stream));
    if (cnt > 0) std::memcpy(g, st + 2 * n, sizeof(double) * cnt);
    *f0 = st[2 * n + cnt];
    return PNOL_OK;
}

int pnol_dobj_eval_batch(pnol_ctx* ctx, pnol_dobj* obj, const double* Xs, int npts, double* out) {
    PNOL_CHECK(set_device(ctx));
    if (!obj || npts < 0 || (npts > 0 && (!Xs || !out))) return PNOL_ERR_ARG;
    if (npts == 0) return PNOL_OK;
    const size_t n = (size_t)obj->n, per = obj->m > 0 ? (size_t)obj->m : 1;
    const size_t nin = n * npts, nout = per * npts;
    void* dv = nullptr;
    PNOL_CHECK(ws_get(ctx, "batch_io", sizeof(double) * (nin + nout), &dv));
    double *dX = (double*)dv, *dF = dX + nin;
    double* st = (double*)pinned_stage(ctx, sizeof(double) * std::max(nin, nout));
    if (st) {
        std::memcpy(st, Xs, sizeof(double) * nin);
        PNOL_HIP(hipMemcpyAsync(dX, st, sizeof(double) * nin, hipMemcpyHostToDevice, ctx->stream));
    } else {
        PNOL_HIP(hipMemcpyAsync(dX, Xs, sizeof(double) * nin, hipMemcpyHostToDevice, ctx->stream));
    }
    PNOL_CHECK(launch_eval_batch(ctx, obj, dX, npts, dF));
    PNOL_HIP(hipMemcpyAsync(st ? st : out, dF, sizeof(double) * nout, hipMemcpyDeviceToHost, ctx->stream));
    PNOL_CHECK(stream_wait(ctx->stream));
    if (st) std::memcpy(out, st, sizeof(double) * nout);
    return PNOL_OK;
}

int pnol_fd_jacobian_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, int j0, int cnt, double* F0,
                       int compute_f0, double* JT, int ldjt) {
    PNOL_CHECK(set_device(ctx));
    return launch_fd_jacobian(ctx, obj, x, h, j0, cnt, F0, compute_f0, JT, ldjt);
}

int pnol_fd_jtj_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0, int compute_f0,
                  double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, int nchunks) {
    PNOL_CHECK(set_device(ctx));
    if (!obj || !x || !h || !F0 || !JT || !A || ldjt < obj->m || lda < obj->n) return PNOL_ERR_ARG;
    if (compute_f0 < 0 || compute_f0 > 3) return PNOL_ERR_ARG;
    return launch_fd_jtj(ctx, obj, x, h, F0, compute_f0, JT, ldjt, lambda, A, lda, jtj_diag, nchunks);
}

int pnol_fd_normal_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0, int compute_f0,
                     double* JT, int ldjt, double lambda, double* A, int lda, double* jtj_diag, double* rhs) {
    PNOL_CHECK(set_device(ctx));
    if (!obj || !x || !h || !F0 || !JT || !A || !rhs || ldjt < obj->m || lda < obj->n) return PNOL_ERR_ARG;
    if (compute_f0 < 0 || compute_f0 > 3) return PNOL_ERR_ARG;
    return launch_fd_jtj(ctx, obj, x, h, F0, compute_f0, JT, ldjt, lambda, A, lda, jtj_diag, 1, rhs);
}

int pnol_lm_trip_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, double* F0, int compute_f0,
                   double* JT, int ldjt, double lambda, double* rhs, double* sigma, int* dinfo, double* xnext) {
    PNOL_CHECK(set_device(ctx));
    if (compute_f0 < 0 || compute_f0 > 3) return PNOL_ERR_ARG;
    return launch_fd_normal_solve(ctx, obj, x, h, F0, compute_f0, JT, ldjt, lambda, rhs, sigma, dinfo, xnext);
}

int pnol_lm_trip_normal_d(pnol_ctx* ctx, int m, int n, double lambda, double* A, int lda) {
    PNOL_CHECK(set_device(ctx));
    return launch_jtj_from_partials(ctx, m, n, lambda, A, lda);
}

int pnol_fd_jacobian_tiles_d(pnol_ctx* ctx, pnol_dobj* obj, const double* x, const double* h, const int* start,
                             const int* count, int ntiles, double* F0, int compute_f0, double* JT, int ldjt) {
    PNOL_CHECK(set_device(ctx));
    if (ntiles < 0 || (ntiles > 0 && (!start || !count)) || compute_f0 < 0 || compute_f0 > 3) return PNOL_ERR_ARG;
    return launch_fd_jacobian_tiles(ctx, obj, x, h, start, count, ntiles, F0, compute_f0, JT, 0, ldjt);
}

}  // extern "C"
