// CPU check of csrc/host/recur_simd.hpp (the bounded solvers' frozen-coordinate scatter / gather):
// the AVX-512 paths against the scalar walks they replace, bitwise, over random indicator
// patterns and lengths (tail blocks, all-frozen / all-free words, empty reduced vectors).
// Built and run by tests/test_host_fd.py::test_recur_simd_matches_scalar_walks.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "recur_simd.hpp"

using namespace pnol;

static void ref_scatter(double* out, const std::vector<double>& x, const double* p, double a,
                        const std::vector<double>& cX, const std::vector<bool>& cI) {
    const size_t nf = cX.size(), nr = x.size(), last = nr > 0 ? nr - 1 : 0;
    size_t r = 0;
    for (size_t i = 0; i < nf; ++i) {
        const bool c = cI[i];
        const size_t q = r < last ? r : last;
        const double v = nr > 0 ? (p ? x[q] + a * p[q] : x[q]) : 0.0;
        out[i] = c ? cX[i] : v;
        r += !c;
    }
}

static bool same(const double* a, const double* b, size_t n) { return std::memcmp(a, b, n * sizeof(double)) == 0; }

int main() {
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    int fails = 0, cases = 0;
    const size_t sizes[] = {1, 7, 8, 9, 63, 64, 65, 127, 200, 513, 16384};
    const double dens[] = {0.0, 0.05, 0.5, 0.7, 0.95, 1.0};
    for (size_t nf : sizes)
        for (double dfz : dens)
            for (int rep = 0; rep < 3; ++rep) {
                std::bernoulli_distribution bz(dfz);
                std::vector<bool> cI(nf);
                std::vector<double> cX(nf);
                for (size_t i = 0; i < nf; ++i) {
                    cI[i] = bz(g);
                    cX[i] = u(g);
                }
                const size_t nfree = recur::free_count(cI);
                size_t cnt = 0;
                for (size_t i = 0; i < nf; ++i) cnt += !cI[i];
                if (cnt != nfree) ++fails;
                for (int mism = 0; mism < 2; ++mism) {   // matching reduced length, then a mismatch
                    const size_t nr = mism ? nfree + 3 : nfree;
                    std::vector<double> x(nr), p(nr), h(nr);
                    for (size_t r = 0; r < nr; ++r) {
                        x[r] = u(g);
                        p[r] = u(g);
                        h[r] = 1e-6 * (1 + u(g));
                    }
                    const double a = u(g);
                    std::vector<double> o1(nf), o2(nf);
                    recur::scatter(o1.data(), x, nullptr, 0.0, cX, cI);
                    ref_scatter(o2.data(), x, nullptr, 0.0, cX, cI);
                    fails += !same(o1.data(), o2.data(), nf);
                    recur::scatter(o1.data(), x, p.data(), a, cX, cI);
                    ref_scatter(o2.data(), x, p.data(), a, cX, cI);
                    fails += !same(o1.data(), o2.data(), nf);
                    recur::scatter_steps(o1.data(), h, cI);
                    std::vector<double> ones(nf, 1.0);
                    ref_scatter(o2.data(), h, nullptr, 0.0, ones, cI);
                    if (nr == 0) std::fill(o2.begin(), o2.end(), 1.0);
                    fails += !same(o1.data(), o2.data(), nf);
                    cases += 3;
                }
                std::vector<double> full(nf), g1(nfree + 1, -7.0), g2(nfree + 1, -7.0);
                for (auto& v : full) v = u(g);
                recur::gather(g1.data(), full.data(), cI);
                size_t r = 0;
                for (size_t i = 0; i < nf; ++i)
                    if (!cI[i]) g2[r++] = full[i];
                fails += !same(g1.data(), g2.data(), nfree + 1);
                std::vector<double> b = full;
                std::vector<int> want, got;
                for (size_t i = 0; i < nf; i += 1 + (i % 37)) {
                    b[i] = b[i] + 1.0;
                    if (!cI[i]) want.push_back((int)i);
                }
                recur::free_diffs(full.data(), b.data(), cI, 1u << 30, got);
                fails += got != want;
                recur::free_diffs(full.data(), b.data(), cI, 2, got);
                const size_t k = want.size() < 3 ? want.size() : 3;
                fails += got.size() != k || !std::equal(got.begin(), got.end(), want.begin());
                cases += 3;
            }
    // alpha_bnd / bound_hits against the reference loops (bounds hit exactly, p = 0, +-0)
    for (size_t n : sizes)
        for (int rep = 0; rep < 4; ++rep) {
            std::vector<double> X(n), lb(n), ub(n), p(n), gr(n);
            for (size_t i = 0; i < n; ++i) {
                lb[i] = -0.5;
                ub[i] = 0.5;
                const int c = (int)(g() % 6);
                X[i] = c == 0 ? lb[i] : (c == 1 ? ub[i] : 0.49 * u(g));
                p[i] = c == 2 ? 0.0 : (c == 3 ? -0.0 : u(g));
                gr[i] = (g() % 5 == 0) ? 0.0 : u(g);
            }
            double bnd = 0;
            for (size_t i = 0; i < n; ++i) {
                const double a1 = (ub[i] - X[i]) / p[i], a2 = (lb[i] - X[i]) / p[i];
                double ai;
                if (a1 > 0) ai = a1;
                else if (a2 > 0) ai = a2;
                else ai = 0;
                if (i == 0) bnd = ai;
                if (bnd > ai) bnd = ai;
            }
            const double b2 = recur::alpha_bnd(X.data(), lb.data(), ub.data(), p.data(), n);
            fails += std::memcmp(&bnd, &b2, sizeof(double)) != 0;
            std::vector<int> want, got;
            const double tol = 1e-9;
            for (size_t k = 0; k < n; ++k) {
                const bool lo = (std::fabs(X[k] - lb[k]) < tol) & ((p[k] < 0) | (gr[k] > 0));
                const bool hi = (std::fabs(X[k] - ub[k]) < tol) & ((p[k] > 0) | (gr[k] < 0));
                if (lo | hi) want.push_back((int)k);
            }
            recur::bound_hits(X.data(), lb.data(), ub.data(), p.data(), gr.data(), n, tol, got);
            fails += got != want;
            cases += 2;
        }
    std::printf("recur_simd: avx512=%d cases=%d fails=%d\n", (int)recur::has_avx512(), cases, fails);
    return fails ? 1 : 0;
}
