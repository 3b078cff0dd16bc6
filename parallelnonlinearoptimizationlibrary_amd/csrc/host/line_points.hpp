// line_points.hpp -- line-search trial points through Objective::objEvalBatch.
//
// Every line search of the reference evaluates f at X + alpha p for a handful of step sizes
// that are known together: the Wolfe search's phi(alpha) and its forward-difference partner
// phi(alpha + dalpha) (BFGS_with_linesearch.cpp:144-174, BFGS_bnd_linesearch.cpp:465-496), and
// the MPI classes' pools (BFGS_with_linesearch_MPI.cpp:163-223, BFGS_with_bnd_linsearch_MPI.cpp:
// 246-354, BFGS_bnd_linesearch_MPI_SW.cpp:599-699).  They go to objEvalBatch as one batch, in
// the reference's evaluation order.  Each point is formed exactly as the reference forms it:
// Xa_i = X_i + alpha * p_i, with alpha the already-rounded step (alpha + dalpha included).
#pragma once

#include <cstring>
#include <vector>

#include "PNOL_Objective.hpp"
#include "recur_simd.hpp"

namespace pnol {

// f[k] = objEval(X + alphas[k] p)
inline void eval_line_points(Objective* o, const std::vector<double>& X, const std::vector<double>& p,
                             const double* alphas, int na, double* f) {
    if (na <= 0) return;
    const int n = (int)X.size();
    thread_local std::vector<double> pts;   // kept across calls (one batch per line-search step)
    pts.resize((size_t)na * n);
    for (int k = 0; k < na; ++k) {
        double* row = pts.data() + (size_t)k * n;
        const double a = alphas[k];
        for (int i = 0; i < n; ++i) row[i] = X[i] + a * p[i];
    }
    o->objEvalBatch(pts.data(), na, n, f);
}

// f[k] = objEvalRecur(X + alphas[k] p, cX, cI) = objEval(scatter(X + alphas[k] p))
// (PNOL_Objective.cpp:303-333: frozen coordinates from cX, the free ones in order)
inline void eval_line_points_recur(Objective* o, const std::vector<double>& X, const std::vector<double>& p,
                                   const double* alphas, int na, const std::vector<double>& cX,
                                   const std::vector<bool>& cI, double* f) {
    if (na <= 0) return;
    const int nf = (int)cX.size();
    thread_local std::vector<double> pts;   // kept across calls (two per bounded BFGS iteration)
    pts.resize((size_t)na * nf);
    // recur::scatter: AVX-512 expand where the host has it, else the branch-free walk (the
    // frozen pattern follows the active set: unpredictable) with the clamped free index
    for (int k = 0; k < na; ++k) recur::scatter(pts.data() + (size_t)k * nf, X, p.data(), alphas[k], cX, cI);
    o->objEvalBatch(pts.data(), na, nf, f);
}

}  // namespace pnol
