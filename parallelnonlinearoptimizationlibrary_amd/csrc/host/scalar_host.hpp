// scalar_host.hpp -- the built-in scalar device objectives' own formulas on the host.
//
// The term i of RosenbrockObject / PowerObject / the synthetic quadratic (ExampleObjectives.hpp
// :79-111, :206-234; SURVEY 8(d) cfg 2/5) in the device kernels' operation order, summed
// sequentially (f = f + t_i in index order).  Compiled into the library with
// -ffp-contract=off, so these are the device batch's bits -- for every kind except PowerObject
// with power != 2, whose std::pow may differ from the device pow in the last place
// (host_bitwise_kind).  Used where the library itself needs a value with the device's bits
// (drivers' line-search batches, the Recur gradient's same-point reuse), never through the
// user-overridable objEvalBatch.
#pragma once

#include <algorithm>
#include <cmath>
#include <vector>

#include "pnol_amd.h"

namespace pnol {

struct ScalarTerms {
    int kind, n;
    double power;
    const double *p0, *p1;
};

template <int KIND>
inline double scalar_term(const ScalarTerms& st, const double* X, int i) {
    if (KIND == PNOL_OBJ_ROSENBROCK) {
        const double t = X[i + 1] - X[i] * X[i], u = 1.0 - X[i];
        return 100.0 * (t * t) + u * u;
    } else if (KIND == PNOL_OBJ_POWER) {
        return st.power == 2.0 ? X[i] * X[i] : std::pow(X[i], st.power);
    } else {
        double t = (0.5 * st.p0[i] * X[i]) * X[i] - st.p1[i] * X[i];
        if (i + 1 < st.n) t = t + (0.25 * X[i]) * X[i + 1];
        return t;
    }
}

// f(X_c) for C points at once.  Each point is the objective's sequential sum f = f + t_i in
// index order (the host objEval's bits); a lone chain is bound by one dependent add per term,
// C interleaved chains let the core overlap their add latencies.
template <int KIND, int C>
inline void scalar_chains_k(const ScalarTerms& st, const double* const* X, double* out) {
    double f[C];
    for (int c = 0; c < C; ++c) f[c] = 0.0;
    const int nt = KIND == PNOL_OBJ_ROSENBROCK ? std::max(st.n - 1, 0) : st.n;
    for (int i = 0; i < nt; ++i)
        for (int c = 0; c < C; ++c) f[c] = f[c] + scalar_term<KIND>(st, X[c], i);
    for (int c = 0; c < C; ++c) out[c] = f[c];
}

template <int C>
inline void scalar_chains(const ScalarTerms& st, const double* const* X, double* out) {
    if (st.kind == PNOL_OBJ_ROSENBROCK) scalar_chains_k<PNOL_OBJ_ROSENBROCK, C>(st, X, out);
    else if (st.kind == PNOL_OBJ_POWER) scalar_chains_k<PNOL_OBJ_POWER, C>(st, X, out);
    else scalar_chains_k<PNOL_OBJ_QUADRATIC, C>(st, X, out);
}

// f of nPts points (rows of Xs, n each), four / two / one interleaved chains at a time
inline void scalar_batch(const ScalarTerms& st, const double* Xs, int nPts, int n, double* f) {
    int k = 0;
    for (; k + 4 <= nPts; k += 4) {
        const double* xp[4] = {Xs + (size_t)k * n, Xs + (size_t)(k + 1) * n, Xs + (size_t)(k + 2) * n,
                               Xs + (size_t)(k + 3) * n};
        scalar_chains<4>(st, xp, f + k);
    }
    if (nPts - k >= 2) {
        const double* xp[2] = {Xs + (size_t)k * n, Xs + (size_t)(k + 1) * n};
        scalar_chains<2>(st, xp, f + k);
        k += 2;
    }
    if (k < nPts) {
        const double* xp = Xs + (size_t)k * n;
        scalar_chains<1>(st, &xp, f + k);
    }
}

// the kinds whose host formula is the device kernels' bits (no transcendental call)
inline bool host_bitwise_kind(int kind, double power) {
    return kind == PNOL_OBJ_ROSENBROCK || kind == PNOL_OBJ_QUADRATIC || (kind == PNOL_OBJ_POWER && power == 2.0);
}

}  // namespace pnol
