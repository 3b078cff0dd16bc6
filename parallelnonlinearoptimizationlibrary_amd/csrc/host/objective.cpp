// objective.cpp -- the finite-difference engine of the drop-in Objective / MultiObjective.
//
// Host objectives follow the reference loops (PNOL_Objective.cpp) point by point; device
// objectives evaluate every point of a block in one launch.  The *MPI forms shard the
// columns in contiguous ceil(n/P) blocks and assemble with one allgather (RCCL over xGMI
// on GPU ranks) -- the reference's zero-padded Allreduce(SUM) is an allgather in disguise
// (x + 0 = x), so the assembled result is bitwise the serial one for any rank count.
#include <cstring>

#include "../pnol_comm.hpp"
#include "PNOL_Objective.hpp"
#include "device_util.hpp"

using namespace pnol;

namespace {

// f at x + h_i e_i for i in [b, b+cnt) into out[0..cnt), host objective
void host_points(Objective* o, std::vector<double>& X, std::vector<double>& dX, int b, int cnt, double* out) {
    std::vector<double> XdX(X.size());
    for (int q = 0; q < cnt; ++q) {
        const int i = b + q;
        XdX = X;
        XdX[i] = XdX[i] + dX[i];
        out[q] = o->objEval(XdX);
    }
}

// device FD gradient for coordinates [b, b+cnt); returns f0 and g[0..cnt)
void device_gradient(pnol_dobj* d, const std::vector<double>& X, const std::vector<double>& h, int b, int cnt,
                     double* f0, double* g) {
    pnol_ctx* ctx = require_ctx();
    const int n = (int)X.size();
    DevVec dx(ctx, n), dh(ctx, n), dg(ctx, cnt > 0 ? cnt : 1), df(ctx, 1);
    dx.upload(X);
    dh.upload(h);
    check(pnol_fd_gradient_d(ctx, d, dx.get(), dh.get(), b, cnt, df.get(), dg.get()), "fd_gradient");
    if (cnt > 0) dg.download(g, (size_t)cnt);
    df.download(f0, 1);
}

// scatter a reduced vector into the full one (objEvalRecur's mapping, PNOL_Objective.cpp:311-323)
std::vector<double> scatter_full(const std::vector<double>& Xr, const std::vector<double>& cX,
                                 const std::vector<bool>& cI) {
    std::vector<double> X(cX.size());
    size_t ir = 0;
    for (size_t i = 0; i < cX.size(); ++i) X[i] = cI[i] ? cX[i] : Xr[ir++];
    return X;
}

}  // namespace

// ---- Objective -------------------------------------------------------------------------------

void Objective::gradientApproximation(vector<double>& X, vector<double>& dX, vector<double>& dFdX) {
    const int N = (int)X.size();
    dFdX.resize(N);
    if (pnol_dobj* d = deviceObjective(N)) {
        double F = 0;
        device_gradient(d, X, dX, 0, N, &F, dFdX.data());
        countEvals(N + 1);
        return;
    }
    const double F = objEval(X);
    std::vector<double> FdX(N);
    host_points(this, X, dX, 0, N, FdX.data());
    for (int i = 0; i < N; ++i) dFdX[i] = (FdX[i] - F) / dX[i];
}

void Objective::hessianApproximation(vector<double>& X, vector<double>& dX, vector<vector<double>>& B) {
    // PNOL_Objective.cpp:38-85 (3 evaluations per upper-triangle pair, mirrored)
    const int N = (int)X.size();
    B.assign(N, vector<double>(N, 0.0));
    const double F = objEval(X);
    vector<double> Xi(N), Xj(N), Xij(N);
    for (int i = 0; i < N; ++i)
        for (int j = i; j < N; ++j) {
            Xi = X; Xj = X; Xij = X;
            Xi[i] = Xi[i] + dX[i];
            Xj[j] = Xj[j] + dX[j];
            Xij[i] = Xij[i] + dX[i];
            Xij[j] = Xij[j] + dX[j];
            const double Fi = objEval(Xi), Fj = objEval(Xj), Fij = objEval(Xij);
            B[i][j] = (Fij - Fi - Fj + F) / (dX[i] * dX[j]);
        }
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < i; ++j) B[i][j] = B[j][i];
}

void Objective::gradientApproximationMPI(vector<double>& X, vector<double>& dX, vector<double>& dFdX) {
    const int N = (int)X.size();
    const int P = comm_size(), r = comm_rank();
    int b = 0, cnt = 0;
    block_range(N, P, r, &b, &cnt);
    const int per = (N + P - 1) / P;
    std::vector<double> mine(per > 0 ? per : 1, 0.0), all((size_t)P * (per > 0 ? per : 1), 0.0);
    double F = 0;
    if (pnol_dobj* d = deviceObjective(N)) {
        device_gradient(d, X, dX, b, cnt, &F, mine.data());
        countEvals(cnt + 1);
    } else {
        F = objEval(X);   // the base point, redundantly on every rank (deterministic)
        std::vector<double> FdX(cnt > 0 ? cnt : 1);
        host_points(this, X, dX, b, cnt, FdX.data());
        for (int q = 0; q < cnt; ++q) mine[q] = (FdX[q] - F) / dX[b + q];
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
        // full-length point and step: the free coordinate i maps to full index map[i]; the
        // perturbed point equals the reference's scatter(X + dX_i e_i) bit for bit
        std::vector<double> Xf = scatter_full(X, constantX, constantIndicator);
        std::vector<double> hf(Xf.size(), 1.0);
        std::vector<int> map;
        for (size_t i = 0, ir = 0; i < constantX.size(); ++i)
            if (!constantIndicator[i]) { map.push_back((int)i); hf[i] = dX[ir++]; }
        std::vector<double> gf(Xf.size());
        double F = 0;
        device_gradient(d, Xf, hf, 0, (int)Xf.size(), &F, gf.data());
        countEvals(N + 1);
        for (int i = 0; i < N; ++i) dFdX[i] = gf[map[i]];
        return;
    }
    const double F = objEvalRecur(X, constantX, constantIndicator);
    std::vector<double> XdX(N);
    for (int i = 0; i < N; ++i) {
        XdX = X;
        XdX[i] = XdX[i] + dX[i];
        const double FdX = objEvalRecur(XdX, constantX, constantIndicator);
        dFdX[i] = (FdX - F) / dX[i];
    }
}

void Objective::gradientApproximationMPIRecur(vector<double>& X, vector<double>& dX, vector<double>& dFdX,
                                              vector<double>& constantX, vector<bool>& constantIndicator) {
    // PNOL_Objective.cpp:366-459: same values as the serial Recur gradient, points sharded
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
        std::vector<int> map;
        for (size_t i = 0, ir = 0; i < constantX.size(); ++i)
            if (!constantIndicator[i]) { map.push_back((int)i); hf[i] = dX[ir++]; }
        if (cnt > 0) {
            const int f0i = map[b], span = map[b + cnt - 1] - f0i + 1;
            std::vector<double> gs(span);
            double F = 0;
            device_gradient(d, Xf, hf, f0i, span, &F, gs.data());
            for (int q = 0; q < cnt; ++q) mine[q] = gs[map[b + q] - f0i];
        }
        countEvals(cnt + 1);
    } else {
        const double F = objEvalRecur(X, constantX, constantIndicator);
        std::vector<double> XdX(N);
        for (int q = 0; q < cnt; ++q) {
            const int i = b + q;
            XdX = X;
            XdX[i] = XdX[i] + dX[i];
            mine[q] = (objEvalRecur(XdX, constantX, constantIndicator) - F) / dX[i];
        }
    }
    check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)per), "allgather(gradient recur)");
    dFdX.resize(N);
    for (int i = 0; i < N; ++i) dFdX[i] = all[i];
}

// ---- MultiObjective --------------------------------------------------------------------------

namespace {

// JT block rows [b, b+cnt) (ld = m) of a host multi-objective; F0 the base residuals
void host_jacobian_block(MultiObjective* o, std::vector<double>& X, std::vector<double>& dX, int m, int b, int cnt,
                         const std::vector<double>& F0, double* JT) {
    std::vector<double> XdX(X.size()), FdX(m);
    for (int q = 0; q < cnt; ++q) {
        const int j = b + q;
        XdX = X;
        XdX[j] = XdX[j] + dX[j];
        o->objEval(XdX, FdX);
        for (int i = 0; i < m; ++i) JT[(size_t)q * m + i] = (FdX[i] - F0[i]) / dX[j];
    }
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
        objEval(X, F);
        host_jacobian_block(this, X, dX, m, 0, n, F, JT.data());
    }
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) J[i][j] = JT[(size_t)j * m + i];
}

void MultiObjective::gradientApproximationMPI(vector<double>& X, vector<double>& dX, vector<vector<double>>& J) {
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
        objEval(X, F);   // base residuals, redundantly per rank
        host_jacobian_block(this, X, dX, m, b, cnt, F, mine.data());
        check(comm_allgather_host(nullptr, mine.data(), all.data(), (size_t)per * m), "allgather(jacobian)");
        std::memcpy(JT.data(), all.data(), sizeof(double) * JT.size());
    }
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) J[i][j] = JT[(size_t)j * m + i];
}
