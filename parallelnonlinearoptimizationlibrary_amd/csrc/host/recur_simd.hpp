// recur_simd.hpp -- the frozen-coordinate scatter / gather of the bounded solvers' Recur calls
// (PNOL_Objective.cpp:303-360, BFGS_bnd_linesearch.cpp:465-496) at full length, with AVX-512
// expand / compress where the host has it.
//
// A Recur call maps the reduced point (the free coordinates in order) to the full one: frozen
// coordinate i reads constantX[i], the r-th free one the r-th reduced entry.  At cfg 5 (n =
// 16384, ~9.4k recursion levels) every iteration walks the 16384-entry indicator several times
// (the FD gradient's point and steps, its result, the line search's trial points); one entry
// per step with a loop-carried free index costs ~25 us per walk.  With AVX-512 eight entries
// go per instruction: vexpandpd places the next free values into the lanes whose indicator bit
// is clear (the frozen lanes keep constantX), vcompresspd packs the free lanes back.  Pure data
// movement, plus X + a p formed as the scalar loop forms it (one rounding for the product, one
// for the sum; nothing contracted) -- every result is bitwise the scalar walk's, which stays as
// the fallback (no AVX-512, or a free count that does not match the reduced length).
#pragma once

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#define PNOL_RECUR_X86 1
#else
#define PNOL_RECUR_X86 0
#endif

namespace pnol {
namespace recur {

// the indicator's 64-bit words (libstdc++ stores vector<bool> as whole words from bit 0)
inline const uint64_t* words(const std::vector<bool>& v) {
#if defined(__GLIBCXX__)
    static_assert(sizeof(*v.begin()._M_p) == sizeof(uint64_t), "64-bit vector<bool> words");
    return reinterpret_cast<const uint64_t*>(v.begin()._M_p);
#else
    (void)v;
    return nullptr;
#endif
}

inline bool has_avx512() {
#if PNOL_RECUR_X86
    // PNOL_NO_AVX512=1 keeps the scalar walks (tests run both)
    static const bool ok = __builtin_cpu_supports("avx512f") != 0 && !std::getenv("PNOL_NO_AVX512");
    return ok;
#else
    return false;
#endif
}

// frozen bits of entries [i, i + 8) (i a multiple of 8)
inline unsigned frozen8(const uint64_t* w, size_t i) { return (unsigned)(w[i >> 6] >> (i & 63)) & 0xFFu; }

inline size_t free_count(const std::vector<bool>& cI) {
    size_t c = 0;
    if (const uint64_t* w = words(cI)) {
        const size_t n = cI.size(), nw = n / 64;
        for (size_t q = 0; q < nw; ++q) c += 64 - (size_t)__builtin_popcountll(w[q]);
        for (size_t i = nw * 64; i < n; ++i) c += !cI[i];
        return c;
    }
    for (size_t i = 0; i < cI.size(); ++i) c += !cI[i];
    return c;
}

#if PNOL_RECUR_X86
// out[i] = frozen ? base[i] (or the constant `fill` when base is null) : src[r++]
__attribute__((target("avx512f"))) inline void expand_avx512(double* out, const double* base, double fill,
                                                            const double* src, const uint64_t* w, size_t nf) {
    size_t r = 0;
    const __m512d fv = _mm512_set1_pd(fill);
    size_t i = 0;
    for (; i + 8 <= nf; i += 8) {
        const __mmask8 fm = (__mmask8)(~frozen8(w, i) & 0xFFu);
        const __m512d b = base ? _mm512_loadu_pd(base + i) : fv;
        _mm512_storeu_pd(out + i, _mm512_mask_expandloadu_pd(b, fm, src + r));
        r += (size_t)__builtin_popcount((unsigned)fm);
    }
    if (i < nf) {
        const __mmask8 tail = (__mmask8)((1u << (nf - i)) - 1u);
        const __mmask8 fm = (__mmask8)(~frozen8(w, i) & tail);
        const __m512d b = base ? _mm512_maskz_loadu_pd(tail, base + i) : fv;
        _mm512_mask_storeu_pd(out + i, tail, _mm512_mask_expandloadu_pd(b, fm, src + r));
    }
}

// out[r++] = full[i] for the free entries i
__attribute__((target("avx512f"))) inline void compress_avx512(double* out, const double* full, const uint64_t* w,
                                                              size_t nf) {
    size_t r = 0, i = 0;
    for (; i + 8 <= nf; i += 8) {
        const __mmask8 fm = (__mmask8)(~frozen8(w, i) & 0xFFu);
        _mm512_mask_compressstoreu_pd(out + r, fm, _mm512_loadu_pd(full + i));
        r += (size_t)__builtin_popcount((unsigned)fm);
    }
    if (i < nf) {
        const __mmask8 tail = (__mmask8)((1u << (nf - i)) - 1u);
        const __mmask8 fm = (__mmask8)(~frozen8(w, i) & tail);
        _mm512_mask_compressstoreu_pd(out + r, fm, _mm512_maskz_loadu_pd(tail, full + i));
    }
}
#endif

// thread-local scratch for X + a p over the reduced coordinates
inline double* scratch(size_t n) {
    thread_local std::vector<double> s;
    if (s.size() < n) s.resize(n);
    return s.data();
}

// Full point of the reduced x (or of x + a p when p is given): frozen i -> cX[i], the r-th free
// -> x[r] (+ a p[r]).  Scalar walk: the free index is clamped to the last reduced entry and an
// empty x reads 0.0 -- the bounded solvers' fallback walks may pass a reduced vector whose
// length differs from the free count; the vector path runs only when they agree.
inline void scatter(double* out, const std::vector<double>& x, const double* p, double a,
                    const std::vector<double>& cX, const std::vector<bool>& cI) {
    const size_t nf = cX.size(), nr = x.size();
#if PNOL_RECUR_X86
    if (has_avx512() && nr > 0)
        if (const uint64_t* w = words(cI))
            if (free_count(cI) == nr) {
                const double* src = x.data();
                if (p) {
                    double* t = scratch(nr);
                    for (size_t r = 0; r < nr; ++r) t[r] = x[r] + a * p[r];
                    src = t;
                }
                expand_avx512(out, cX.data(), 0.0, src, w, nf);
                return;
            }
#endif
    const size_t last = nr > 0 ? nr - 1 : 0;
    size_t r = 0;
    for (size_t i = 0; i < nf; ++i) {
        const bool c = cI[i];
        const size_t q = r < last ? r : last;
        const double v = nr > 0 ? (p ? x[q] + a * p[q] : x[q]) : 0.0;
        out[i] = c ? cX[i] : v;
        r += !c;
    }
}

// Full steps: frozen i -> 1.0 (a dummy step), the r-th free -> h[r] (clamped / 1.0 as above)
inline void scatter_steps(double* out, const std::vector<double>& h, const std::vector<bool>& cI) {
    const size_t nf = cI.size(), nr = h.size();
#if PNOL_RECUR_X86
    if (has_avx512() && nr > 0)
        if (const uint64_t* w = words(cI))
            if (free_count(cI) == nr) {
                expand_avx512(out, nullptr, 1.0, h.data(), w, nf);
                return;
            }
#endif
    const size_t last = nr > 0 ? nr - 1 : 0;
    size_t r = 0;
    for (size_t i = 0; i < nf; ++i) {
        const bool c = cI[i];
        const size_t q = r < last ? r : last;
        out[i] = c ? 1.0 : (nr > 0 ? h[q] : 1.0);
        r += !c;
    }
}

// out[0, free count) = full[i] for the free entries i, in order
inline void gather(double* out, const double* full, const std::vector<bool>& cI) {
    const size_t nf = cI.size();
#if PNOL_RECUR_X86
    if (has_avx512())
        if (const uint64_t* w = words(cI)) {
            compress_avx512(out, full, w, nf);
            return;
        }
#endif
    size_t r = 0;
    for (size_t i = 0; i < nf; ++i)
        if (!cI[i]) out[r++] = full[i];
}

// the free entries i whose 8 bytes differ between a and b, ascending, stopping past `cap` hits
inline void free_diffs(const double* a, const double* b, const std::vector<bool>& cI, size_t cap,
                       std::vector<int>& hits) {
    hits.clear();
    const size_t nf = cI.size();
    const uint64_t* w = words(cI);
    for (size_t i = 0; i < nf; i += 64) {
        const size_t e = i + 64 < nf ? i + 64 : nf;
        if (std::memcmp(a + i, b + i, sizeof(double) * (e - i)) == 0) continue;   // the common case
        const uint64_t fw = w ? w[i >> 6] : 0;
        for (size_t j = i; j < e; ++j) {
            const bool frozen = w ? ((fw >> (j & 63)) & 1u) != 0 : (bool)cI[j];
            if (!frozen && std::memcmp(a + j, b + j, sizeof(double)) != 0) {
                hits.push_back((int)j);
                if (hits.size() > cap) return;
            }
        }
    }
}

// ---- the bounded solvers' other full-length loops ---------------------------------------

#if PNOL_RECUR_X86
__attribute__((target("avx512f"))) inline double alpha_bnd_avx512(const double* X, const double* lb, const double* ub,
                                                                  const double* p, size_t n) {
    const __m512d zero = _mm512_setzero_pd();
    __m512d m = _mm512_set1_pd(__builtin_inf());
    size_t i = 0;
    for (; i < n; i += 8) {
        const __mmask8 live = n - i >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << (n - i)) - 1u);
        const __m512d x = _mm512_maskz_loadu_pd(live, X + i), pv = _mm512_mask_loadu_pd(_mm512_set1_pd(1.0), live, p + i);
        const __m512d a1 = _mm512_div_pd(_mm512_sub_pd(_mm512_maskz_loadu_pd(live, ub + i), x), pv);
        const __m512d a2 = _mm512_div_pd(_mm512_sub_pd(_mm512_maskz_loadu_pd(live, lb + i), x), pv);
        const __mmask8 g1 = _mm512_cmp_pd_mask(a1, zero, _CMP_GT_OQ), g2 = _mm512_cmp_pd_mask(a2, zero, _CMP_GT_OQ);
        // ai = a1 > 0 ? a1 : (a2 > 0 ? a2 : 0)
        const __m512d ai = _mm512_mask_mov_pd(_mm512_maskz_mov_pd(g2, a2), g1, a1);
        m = _mm512_mask_min_pd(m, live, m, ai);
    }
    return _mm512_reduce_min_pd(m);
}
#endif

// computeAlphaBnd's value (Box_boundary_functions.cpp:11-40): min over i of a_i, a_i the first
// positive of (ub_i - x_i) / p_i and (lb_i - x_i) / p_i, else 0.  Every a_i is +0 or positive
// (never NaN or -0), so the minimum does not depend on the order it is taken in.
inline double alpha_bnd(const double* X, const double* lb, const double* ub, const double* p, size_t n) {
#if PNOL_RECUR_X86
    if (n > 0 && has_avx512()) return alpha_bnd_avx512(X, lb, ub, p, n);
#endif
    double bnd = 0;
    for (size_t i = 0; i < n; ++i) {
        const double a1 = (ub[i] - X[i]) / p[i];
        const double a2 = (lb[i] - X[i]) / p[i];
        double ai;
        if (a1 > 0) ai = a1;
        else if (a2 > 0) ai = a2;
        else ai = 0;
        if (i == 0) bnd = ai;
        if (bnd > ai) bnd = ai;
    }
    return bnd;
}

#if PNOL_RECUR_X86
__attribute__((target("avx512f"))) inline void bound_hits_avx512(const double* X, const double* lb, const double* ub,
                                                                const double* p, const double* g, size_t n, double tol,
                                                                std::vector<int>& hits) {
    const __m512d zero = _mm512_setzero_pd(), tv = _mm512_set1_pd(tol);
    const __m512i absm = _mm512_set1_epi64(0x7FFFFFFFFFFFFFFFLL);
    for (size_t i = 0; i < n; i += 8) {
        const __mmask8 live = n - i >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << (n - i)) - 1u);
        const __m512d x = _mm512_maskz_loadu_pd(live, X + i), pv = _mm512_maskz_loadu_pd(live, p + i),
                      gv = _mm512_maskz_loadu_pd(live, g + i);
        const __m512d dl = _mm512_castsi512_pd(
            _mm512_and_si512(_mm512_castpd_si512(_mm512_sub_pd(x, _mm512_maskz_loadu_pd(live, lb + i))), absm));
        const __m512d du = _mm512_castsi512_pd(
            _mm512_and_si512(_mm512_castpd_si512(_mm512_sub_pd(x, _mm512_maskz_loadu_pd(live, ub + i))), absm));
        const __mmask8 pn = _mm512_cmp_pd_mask(pv, zero, _CMP_LT_OQ), pp = _mm512_cmp_pd_mask(pv, zero, _CMP_GT_OQ);
        const __mmask8 gp = _mm512_cmp_pd_mask(gv, zero, _CMP_GT_OQ), gn = _mm512_cmp_pd_mask(gv, zero, _CMP_LT_OQ);
        const __mmask8 lo = _mm512_cmp_pd_mask(dl, tv, _CMP_LT_OQ) & (pn | gp);
        const __mmask8 hi = _mm512_cmp_pd_mask(du, tv, _CMP_LT_OQ) & (pp | gn);
        unsigned m = (unsigned)((lo | hi) & live);
        while (m) {
            hits.push_back((int)(i + (size_t)__builtin_ctz(m)));
            m &= m - 1;
        }
    }
}
#endif

// positions k (ascending) where x_k sits within tol of a bound and the direction or the
// gradient points out of the box there (BFGS_bnd_linesearch.cpp:518-560):
//   lo: |x_k - lb_k| < tol and (p_k < 0 or g_k > 0);  hi: |x_k - ub_k| < tol and (p_k > 0 or g_k < 0)
inline void bound_hits(const double* X, const double* lb, const double* ub, const double* p, const double* g, size_t n,
                       double tol, std::vector<int>& hits) {
    hits.clear();
#if PNOL_RECUR_X86
    if (has_avx512()) {
        bound_hits_avx512(X, lb, ub, p, g, n, tol, hits);
        return;
    }
#endif
    for (size_t k = 0; k < n; ++k) {
        const double xk = X[k], pk = p[k], gk = g[k];
        const bool lo = (__builtin_fabs(xk - lb[k]) < tol) & ((pk < 0) | (gk > 0));
        const bool hi = (__builtin_fabs(xk - ub[k]) < tol) & ((pk > 0) | (gk < 0));
        if (lo | hi) hits.push_back((int)k);
    }
}

}  // namespace recur
}  // namespace pnol
