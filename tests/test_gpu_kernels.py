"""Kernel-level parity of the HIP path against the CPU oracle (and numpy fp64 where the
reference order is not the contract).  Run on an MI355X: pytest -m gpu.

Tolerances: 'bitwise' where the kernel follows the reference operation order (n <=
PNOL_SEQ_MAX paths, FD batches of transcendental-free objectives, the exact BFGS update,
the reference-order LU); otherwise |err| <= 8 eps * sum|a_i b_i| per reduced entry (a
reordered fp64 sum), written out per test.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps


@pytest.fixture(scope="module")
def ctx():
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context
    if L.device_count() < 1:
        pytest.fail("no gfx950 device visible for a -m gpu run")
    return Context(0)


def _reorder_tol(A, x):
    return 8 * EPS * (np.abs(A) @ np.abs(x)) + 1e-300


def _np(t):
    return t.cpu().numpy()


# ---- H.g ---------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 2, 5, 64])
def test_hg_small_bitwise(ctx, oracle, n):
    rng = np.random.default_rng(n)
    D = rng.standard_normal((n, n)); g = rng.standard_normal(n)
    p = _np(ctx.hg(ctx.tensor(D), ctx.tensor(g)))
    assert np.array_equal(p, -oracle.matvec(D, g))


@pytest.mark.parametrize("n", [65, 300, 1023, 4099, 8192])
def test_hg_large(ctx, n):
    rng = np.random.default_rng(n)
    D = rng.standard_normal((n, n)); g = rng.standard_normal(n)
    p = _np(ctx.hg(ctx.tensor(D), ctx.tensor(g)))
    assert np.all(np.abs(p + D @ g) <= _reorder_tol(D, g))


def test_hg_padded_leading_dimension(ctx):
    rng = np.random.default_rng(3)
    n, ld = 301, 320
    big = rng.standard_normal((n, ld))
    Dt = ctx.tensor(big)[:, :n]
    g = rng.standard_normal(n)
    p = _np(ctx.hg(Dt, ctx.tensor(g)))
    D = big[:, :n]
    assert np.all(np.abs(p + D @ g) <= _reorder_tol(D, g))


@pytest.mark.parametrize("rows,cols", [(2048, 16384), (7, 1001), (4096, 33), (9000, 256)])
def test_gemv_neg_rectangular(ctx, rows, cols):
    rng = np.random.default_rng(rows + cols)
    A = rng.standard_normal((rows, cols)); x = rng.standard_normal(cols)
    y = _np(ctx.gemv_neg(ctx.tensor(A), ctx.tensor(x)))
    assert np.all(np.abs(y + A @ x) <= _reorder_tol(A, x))


# ---- BFGS update ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 3, 8, 64, 100])
def test_bfgs_update_exact_bitwise(ctx, oracle, n):
    rng = np.random.default_rng(10 + n)
    D = np.eye(n) + 0.1 * rng.standard_normal((n, n))
    y = rng.standard_normal(n); s = rng.standard_normal(n)
    Dt = ctx.tensor(D)
    ctx.bfgs_update_exact(Dt, ctx.tensor(y), ctx.tensor(s))
    assert np.array_equal(_np(Dt), oracle.update_hessian_inv(D, y, s))


@pytest.mark.parametrize("n", [1, 7, 300, 513, 1030])
@pytest.mark.parametrize("pending,wb", [(False, False), (True, True), (True, False)])
def test_bfgs_pass(ctx, n, pending, wb):
    rng = np.random.default_rng(n * 7 + pending + 2 * wb)
    D = rng.standard_normal((n, n)); y = rng.standard_normal(n); g = rng.standard_normal(n)
    sp, ap, bp = rng.standard_normal(n), rng.standard_normal(n), rng.standard_normal(n)
    Dt = ctx.tensor(D)
    pend = (ctx.tensor(sp), ctx.tensor(ap), ctx.tensor(bp)) if pending else None
    u, w, v = (_np(t) for t in ctx.bfgs_pass(Dt, ctx.tensor(y), ctx.tensor(g), pend, wb))
    Dc = D + np.outer(sp, ap) + np.outer(bp, sp) if pending else D
    assert np.all(np.abs(u - Dc @ y) <= _reorder_tol(Dc, y) + 4 * EPS * np.abs(Dc).max() * np.abs(y).sum())
    assert np.all(np.abs(v - Dc @ g) <= _reorder_tol(Dc, g) + 4 * EPS * np.abs(Dc).max() * np.abs(g).sum())
    assert np.all(np.abs(w - Dc.T @ y) <= _reorder_tol(Dc.T, y) + 4 * EPS * np.abs(Dc).max() * np.abs(y).sum())
    Dafter = _np(Dt)
    if wb:
        assert np.allclose(Dafter, Dc, rtol=4 * EPS, atol=4 * EPS * np.abs(Dc).max())
    else:
        assert np.array_equal(Dafter, D)


def test_fused_update_sequence_matches_reference_form(ctx, oracle):
    """Three lazy rank-2 updates (the fast mode's algebra) vs the reference O(n^3) form."""
    rng = np.random.default_rng(5)
    n = 257
    Dref = np.eye(n)
    Dt = ctx.tensor(np.eye(n))
    pend = None
    for it in range(3):
        y = rng.standard_normal(n); s = rng.standard_normal(n) + 0.5 * y
        u, w, _ = (_np(t) for t in ctx.bfgs_pass(Dt, ctx.tensor(y), None, pend, pend is not None))
        rho = 1 / np.dot(y, s); beta = np.dot(y, u); c = rho * rho * beta + rho
        a = c * s - rho * w; b = -rho * u
        pend = (ctx.tensor(s), ctx.tensor(a), ctx.tensor(b))
        Dref = oracle.update_hessian_inv(Dref, y, s)
    ctx.bfgs_pass(Dt, None, None, pend, True)
    assert np.allclose(_np(Dt), Dref, rtol=1e-11, atol=1e-11 * np.abs(Dref).max())


@pytest.mark.parametrize("n", [7, 300, 1030, 4097])
@pytest.mark.parametrize("scaled", [False, True])
def test_bfgs_pass_ident_equals_pass_on_identity(ctx, n, scaled):
    """pnol_bfgs_pass_ident_d (the stored diagonal synthesised, not read) is bitwise the
    write-back pass over a real identity / diag(scale): u, w, v and the written D."""
    import ctypes as C
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import _ptr
    rng = np.random.default_rng(n + 11 * scaled)
    y, g = rng.standard_normal(n), rng.standard_normal(n)
    sp, ap, bp = rng.standard_normal(n), rng.standard_normal(n), rng.standard_normal(n)
    scale = rng.uniform(0.5, 2.0, n) if scaled else None
    ld = n + (n & 1)
    Dref = ctx.empty(n, ld)
    ctx.set_identity(Dref[:, :n], ctx.tensor(scale) if scaled else None)
    pend = (ctx.tensor(sp), ctx.tensor(ap), ctx.tensor(bp))
    yt, gt = ctx.tensor(y), ctx.tensor(g)
    u0, w0, v0 = (_np(t) for t in ctx.bfgs_pass(Dref[:, :n], yt, gt, pend, True))
    Dids = ctx.tensor(np.full((n, ld), np.nan))   # never read: NaN garbage must not leak in
    u1, w1, v1 = ctx.empty(n), ctx.empty(n), ctx.empty(n)
    st = ctx.tensor(scale) if scaled else None
    L.check(L.lib().pnol_bfgs_pass_ident_d(ctx.h, _ptr(Dids), ld, n, _ptr(st), _ptr(pend[0]), _ptr(pend[1]),
                                           _ptr(pend[2]), _ptr(yt), _ptr(gt), _ptr(u1), _ptr(w1), _ptr(v1)),
            "pnol_bfgs_pass_ident_d")
    assert np.array_equal(_np(u1), u0) and np.array_equal(_np(w1), w0) and np.array_equal(_np(v1), v0)
    assert np.array_equal(_np(Dids)[:, :n], _np(Dref)[:, :n])


@pytest.mark.parametrize("n", [4096, 8192])
def test_fused_pass_vs_oracle_rank2_form_large(ctx, oracle, n):
    """Two BFGS updates through the fused pass (lazy pending correction, folded with
    write-back) vs the oracle's rank-2 restatement of updateHessianInv at the cfg-2 / north-star
    sizes (the O(n^3) reference form is checked against the rank-2 one at n <= 257 above).
    Tolerance: both sum the same terms in different orders -- 1e-12 of max|D| per entry."""
    rng = np.random.default_rng(n)
    D0 = np.eye(n) + 1e-3 * rng.standard_normal((n, n))
    Dt = ctx.tensor(D0)
    Dref = D0.copy()
    pend = None
    for it in range(2):
        y = rng.standard_normal(n); s = rng.standard_normal(n) + 0.5 * y
        u, w, _ = (_np(t) for t in ctx.bfgs_pass(Dt, ctx.tensor(y), None, pend, pend is not None))
        rho = 1 / oracle.lib().orc_util_dot(oracle.ptr(y), oracle.ptr(s), n)
        beta = np.dot(y, u); c = rho * rho * beta + rho
        a = c * s - rho * w; b = -rho * u
        pend = (ctx.tensor(s), ctx.tensor(a), ctx.tensor(b))
        Dref = oracle.update_hessian_inv_rank2(Dref, y, s)
    ctx.bfgs_pass(Dt, None, None, pend, True)
    got = _np(Dt)
    err = np.abs(got - Dref).max() / np.abs(Dref).max()
    assert err <= 1e-12, err


def test_set_identity(ctx):
    Dt = ctx.tensor(np.full((9, 9), 3.0))
    ctx.set_identity(Dt)
    assert np.array_equal(_np(Dt), np.eye(9))
    scale = np.arange(1.0, 10.0)
    ctx.set_identity(Dt, ctx.tensor(scale))
    assert np.array_equal(_np(Dt), np.diag(scale))


# ---- LM linear algebra ---------------------------------------------------------------------
@pytest.mark.parametrize("m,n", [(100, 3), (100, 4), (4096, 64)])
def test_jtj_small_bitwise(ctx, oracle, m, n):
    rng = np.random.default_rng(m + n)
    J = rng.standard_normal((m, n)); F = rng.standard_normal(m); lam = 0.01
    JTJ, A, rhs, _ = oracle.lm_step(J, F, lam)
    JT = ctx.tensor(J.T.copy())
    Ad, diag = ctx.jtj(JT, lam, want_diag=True)
    assert np.array_equal(_np(Ad), A)
    assert np.array_equal(_np(diag), np.diag(JTJ))
    assert np.array_equal(_np(ctx.jtr(JT, ctx.tensor(F))), rhs)


@pytest.mark.parametrize("m,n", [(1000, 65), (2000, 130), (3001, 300), (16384, 2048), (513, 1000)])
def test_jtj_mfma(ctx, m, n):
    rng = np.random.default_rng(m * 3 + n)
    J = rng.standard_normal((m, n)) / np.sqrt(n)
    lam = 1e-3
    Ad, diag = ctx.jtj(ctx.tensor(J.T.copy()), lam, want_diag=True)
    A = _np(Ad)
    ref = J.T @ J
    tol = 8 * EPS * (np.abs(J).T @ np.abs(J)) * max(1, np.log2(m))
    off = ~np.eye(n, dtype=bool)
    assert np.all(np.abs(A - ref)[off] <= tol[off])
    assert np.all(np.abs(np.diag(A) - (1 + lam) * np.diag(ref)) <= 2 * np.diag(tol))
    assert np.array_equal(A, A.T)   # mirrored: exactly symmetric, like the reference's JT J
    assert np.all(np.abs(_np(diag) - np.diag(ref)) <= np.diag(tol))


def test_jtj_mfma_layout_asymmetric(ctx):
    """Integer-valued J: the MFMA result is exact, so any row/col slip in the C/D layout shows."""
    rng = np.random.default_rng(11)
    m, n = 256, 160
    J = rng.integers(-3, 4, size=(m, n)).astype(np.float64)
    A = _np(ctx.jtj(ctx.tensor(J.T.copy()), 0.0))
    assert np.array_equal(A, J.T @ J)


@pytest.mark.parametrize("method", [4, 5])
@pytest.mark.parametrize("n", [65, 100, 129, 777, 1000, 2048, 3001])
def test_cholesky_solve(ctx, n, method):
    """method 4: lookahead tile Cholesky with diagonal-tile inverses and the forward solve folded
    in, one launch per panel step; method 5 (the default): the same as one persistent launch."""
    rng = np.random.default_rng(n)
    J = rng.standard_normal((2 * n, n))
    A = J.T @ J + np.eye(n)
    b = rng.standard_normal(n)
    sigma, info = ctx.solve(ctx.tensor(A), ctx.tensor(b), method=method)
    assert info == 1
    x = np.linalg.solve(A, b)
    assert np.linalg.norm(_np(sigma) - x) <= 1e-10 * np.linalg.norm(x) * np.linalg.cond(A)


@pytest.mark.parametrize("method", [4, 5])
def test_cholesky_odd_leading_dimension(ctx, method):
    """Odd lda: scalar staging paths (no 16-byte loads)."""
    rng = np.random.default_rng(77)
    n = 300
    J = rng.standard_normal((400, n))
    A = J.T @ J + np.eye(n)
    b = rng.standard_normal(n)
    Ap = ctx.empty(n, n + 1)
    Ap[:, :n] = ctx.tensor(A)
    sigma, info = ctx.solve(Ap[:, :n], ctx.tensor(b), method=method)
    assert info == 1
    x = np.linalg.solve(A, b)
    assert np.linalg.norm(_np(sigma) - x) <= 1e-10 * np.linalg.norm(x) * np.linalg.cond(A)


@pytest.mark.parametrize("method", [4, 5])
def test_cholesky_repeated_solves_reuse_ready_flags(ctx, method):
    """The flag-chained solves tag each call with a new epoch; sizes that grow and shrink (the
    flag buffer is reallocated) and back-to-back calls must all be exact."""
    rng = np.random.default_rng(5)
    for n in (300, 300, 1500, 64 * 70, 200, 1500):
        J = rng.standard_normal((n + 50, n))
        A = J.T @ J + n * np.eye(n)
        b = rng.standard_normal(n)
        sigma, info = ctx.solve(ctx.tensor(A), ctx.tensor(b), method=method)
        assert info == 1, n
        x = np.linalg.solve(A, b)
        assert np.linalg.norm(_np(sigma) - x) <= 1e-12 * np.linalg.norm(x) * np.linalg.cond(A), n


@pytest.mark.parametrize("n", [3, 4, 50, 100])
def test_lu_reference_order_bitwise(ctx, oracle, n):
    rng = np.random.default_rng(n + 100)
    A = rng.standard_normal((n, n)); b = rng.standard_normal(n)
    sigma, info = ctx.solve(ctx.tensor(A), ctx.tensor(b), method=2)
    assert info == 2
    assert np.array_equal(_np(sigma), oracle.lusolve(A, b))


def test_lu_multi_launch_bitwise(ctx, oracle):
    n = 300   # > 256: the per-column multi-launch form
    rng = np.random.default_rng(42)
    A = rng.standard_normal((n, n)); b = rng.standard_normal(n)
    sigma, info = ctx.solve(ctx.tensor(A), ctx.tensor(b), method=2)
    assert np.array_equal(_np(sigma), oracle.lusolve(A, b))


def test_cholesky_m4_keeps_A_and_matches_lu(ctx):
    """Method 4 factors a padded copy (A is left intact) and agrees with the reference-order LU;
    the removed methods 1 and 3 are refused."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    rng = np.random.default_rng(3)
    n = 1000
    J = rng.standard_normal((1200, n))
    A = J.T @ J + 0.5 * np.eye(n)
    b = rng.standard_normal(n)
    At = ctx.tensor(A)
    s4, i4 = ctx.solve(At, ctx.tensor(b), method=4)
    assert i4 == 1
    assert np.array_equal(_np(At), A)
    s2, i2 = ctx.solve(ctx.tensor(A), ctx.tensor(b), method=2)
    assert i2 == 2
    x = np.linalg.solve(A, b)
    c = np.linalg.cond(A)
    for s in (s4, s2):
        assert np.linalg.norm(_np(s) - x) <= 1e-12 * np.linalg.norm(x) * c
    for m in (1, 3):
        with pytest.raises(RuntimeError):
            ctx.solve(ctx.tensor(A), ctx.tensor(b), method=m)


@pytest.mark.parametrize("method", [4, 5])
def test_cholesky_m4_bitwise_under_contention(ctx, method):
    """Methods 4 and 5 hand tiles between workgroups through flags (5: the whole factorisation
    in one launch, tasks from a queue); the result must not depend on scheduling.  Large GEMMs
    on a second stream perturb which workgroups run when; every solve must equal the solo
    solve bitwise, and both forms give the same bits."""
    import torch
    rng = np.random.default_rng(21)
    n = 1500
    J = rng.standard_normal((1700, n))
    A = J.T @ J + 0.1 * np.eye(n)
    b = rng.standard_normal(n)
    At, bt = ctx.tensor(A), ctx.tensor(b)
    ref, info = ctx.solve(At, bt, method=4)
    ref = _np(ref)
    assert info == 1
    side = torch.cuda.Stream()
    X = torch.randn(4096, 4096, device="cuda", dtype=torch.float64)
    for rep in range(6):
        with torch.cuda.stream(side):
            for _ in range(3):
                X = (X @ X) * 1e-3
        sigma, info = ctx.solve(At, bt, method=method)
        assert info == 1
        assert np.array_equal(_np(sigma), ref), rep
    torch.cuda.synchronize()


@pytest.mark.parametrize("n", [65, 128, 300, 1000, 2048, 2111])
def test_cholesky_persistent_equals_per_step_launches(ctx, n):
    """Method 5 (one persistent launch: the diagonal chain in one workgroup, panels and updates
    from an ordered task queue) performs every tile operation of method 4 in the same order:
    sigma is bitwise equal, A is left intact, and method 0 (auto) uses it by default."""
    rng = np.random.default_rng(n)
    J = rng.standard_normal((n + 40, n))
    A = J.T @ J + 0.5 * np.eye(n)
    b = rng.standard_normal(n)
    At, bt = ctx.tensor(A), ctx.tensor(b)
    s4, i4 = ctx.solve(At, bt, method=4)
    s5, i5 = ctx.solve(At, bt, method=5)
    s0, i0 = ctx.solve(At, bt, method=0)
    assert i4 == i5 == i0 == 1
    assert np.array_equal(_np(At), A)
    assert np.array_equal(_np(s5), _np(s4))
    assert np.array_equal(_np(s0), _np(s4))
    x = np.linalg.solve(A, b)
    assert np.linalg.norm(_np(s5) - x) <= 1e-10 * np.linalg.norm(x) * np.linalg.cond(A)


@pytest.mark.parametrize("n", [130, 1000, 2048])
def test_cholesky_step_order_claims_bitwise(ctx, monkeypatch, n):
    """The persistent Cholesky's workers in step order (order 0: what a shared GPU and a context
    that saw a timed-out wait use) perform the same tile operations as the default order 1, with
    the critical update tasks forming their own L panels (PNOL_CHOL_SELFL=1, default) as one task
    per tile or as two half-tile tasks (PNOL_CHOL_SPLIT=1, default), or waiting for the panel
    tasks' (SELFL 0), each step's other updates claimed by tile row (PNOL_CHOL_ROWMAJOR=1,
    default) or by column: sigma bitwise equal in all of them, and equal to method 4's."""
    rng = np.random.default_rng(n + 7)
    J = rng.standard_normal((n + 40, n))
    A = J.T @ J + 0.5 * np.eye(n)
    b = rng.standard_normal(n)
    At, bt = ctx.tensor(A), ctx.tensor(b)
    s4, _ = ctx.solve(At, bt, method=4)
    for selfl, split, rowmajor in (("1", "1", "1"), ("1", "1", "0"), ("1", "0", "1"), ("0", "1", "1")):
        monkeypatch.setenv("PNOL_CHOL_SELFL", selfl)
        monkeypatch.setenv("PNOL_CHOL_SPLIT", split)
        monkeypatch.setenv("PNOL_CHOL_ROWMAJOR", rowmajor)
        monkeypatch.setenv("PNOL_CHOL_ORDER", "0")
        s_0, i_0 = ctx.solve(At, bt, method=5)
        monkeypatch.setenv("PNOL_CHOL_ORDER", "1")
        s_1, i_1 = ctx.solve(At, bt, method=5)
        assert i_0 == i_1 == 1
        assert np.array_equal(_np(s_0), _np(s4)) and np.array_equal(_np(s_1), _np(s4)), (selfl, split, rowmajor)


@pytest.mark.parametrize("n", [130, 700, 2048, 2111])
def test_cholesky_lookahead_equals_plain_chain(ctx, monkeypatch, n):
    """Method 5's diagonal chain starts the next tile's products inside the current factor
    (waves 2 / 3: the left half of L and K blocks 0, 1 of A_dd - L L^T), the rest after it.
    Every accumulator takes the same MFMAs in the same order: sigma is bitwise the chain without
    the look-ahead (PNOL_CHOL_LOOKAHEAD=0) and method 4's; so is a step whose tiles came too
    late for the products and were only staged (the next prepare reads them from LDS)."""
    rng = np.random.default_rng(n + 7)
    J = rng.standard_normal((n + 64, n))
    A = J.T @ J + 0.25 * np.eye(n)
    b = rng.standard_normal(n)
    At, bt = ctx.tensor(A), ctx.tensor(b)
    monkeypatch.setenv("PNOL_CHOL_LOOKAHEAD", "0")
    s_off, i_off = ctx.solve(At, bt, method=5)
    monkeypatch.setenv("PNOL_CHOL_LOOKAHEAD", "52")   # gives up when late: mixed steps
    s_mix, i_mix = ctx.solve(At, bt, method=5)
    monkeypatch.setenv("PNOL_CHOL_LOOKAHEAD", "1000")   # waits for the tiles: every step
    s_on, i_on = ctx.solve(At, bt, method=5)
    monkeypatch.setenv("PNOL_CHOL_LOOKAHEAD", "1")   # late tiles staged only, prepared from LDS
    s_stg, i_stg = ctx.solve(At, bt, method=5)
    monkeypatch.delenv("PNOL_CHOL_LOOKAHEAD")           # default (48)
    s_def, i_def = ctx.solve(At, bt, method=5)
    s4, i4 = ctx.solve(At, bt, method=4)
    assert i_off == i_mix == i_on == i_stg == i_def == i4 == 1
    assert np.array_equal(_np(s_on), _np(s_off))
    assert np.array_equal(_np(s_stg), _np(s_off))
    assert np.array_equal(_np(s_mix), _np(s_off))
    assert np.array_equal(_np(s_def), _np(s_off))
    assert np.array_equal(_np(s_on), _np(s4))


def test_cholesky_bwd_granules_equal_flag_form(ctx, monkeypatch):
    """The backward solve's granule hand-off (x_w[t] with its epoch in one 16-byte sc1 store,
    polled by the consumers) assumes an aligned 16-byte store is seen whole.  A torn read (new
    epoch, old x) would pass the epoch test and corrupt sigma.  Many solves of varying size,
    back to back (epochs advancing, the granule buffer reused), each bitwise the flag form's
    (PNOL_BWD_GRANULE=0)."""
    rng = np.random.default_rng(1234)
    for k in range(40):
        n = int(rng.integers(65, 1400))
        J = rng.standard_normal((n + 16, n))
        A = J.T @ J + 0.5 * np.eye(n)
        b = rng.standard_normal(n)
        At, bt = ctx.tensor(A), ctx.tensor(b)
        monkeypatch.setenv("PNOL_BWD_GRANULE", "0")
        s_flag, i_flag = ctx.solve(At, bt, method=5)
        monkeypatch.delenv("PNOL_BWD_GRANULE")
        outs = [ctx.solve(At, bt, method=5) for _ in range(3)]
        assert i_flag == 1 and all(i == 1 for _, i in outs)
        for s, _ in outs:
            assert np.array_equal(_np(s), _np(s_flag)), (k, n)


@pytest.mark.parametrize("n", [200, 1000])
def test_cholesky_falls_back_to_lu_on_indefinite(ctx, oracle, n):
    rng = np.random.default_rng(9)
    A = rng.standard_normal((n, n)); A = A + A.T   # symmetric indefinite
    b = rng.standard_normal(n)
    sigma, info = ctx.solve(ctx.tensor(A), ctx.tensor(b), method=0)
    assert info == 2
    assert np.array_equal(_np(sigma), oracle.lusolve(A, b))


# ---- FD engine -------------------------------------------------------------------------
@pytest.mark.parametrize("n", [2, 5, 1000, 4097])
def test_fd_gradient_rosenbrock_bitwise(ctx, oracle, n):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    rng = np.random.default_rng(n)
    x = rng.uniform(-2, 2, n); h = np.full(n, 1e-7)
    d = DeviceObjective(ctx, L.OBJ_ROSENBROCK, n)
    f0, g = d.fd_gradient(ctx.tensor(x), ctx.tensor(h))
    o = oracle.rosenbrock(n)
    assert np.array_equal(_np(g), oracle.fd_gradient(o, x, h))
    assert _np(f0)[0] == oracle.obj_eval(o, x)
    # a column block of the same gradient (the sharded path)
    i0, cnt = n // 3, max(1, n // 2)
    _, gb = d.fd_gradient(ctx.tensor(x), ctx.tensor(h), i0, cnt)
    assert np.array_equal(_np(gb), oracle.fd_gradient(o, x, h)[i0:i0 + cnt])


@pytest.mark.parametrize("kind", ["rosenbrock", "quadratic", "power2"])
@pytest.mark.parametrize("n,i0,cnt", [(1, 0, 1), (2, 1, 1), (63, 0, 63), (64, 0, 64), (65, 1, 64), (130, 3, 127),
                                      (1000, 511, 200), (16384, 0, 16384), (16384, 8000, 100)])
def test_fd_gradient_term_form_windows_bitwise(ctx, oracle, kind, n, i0, cnt):
    """The term-form FD gradient (base terms once, per-wave perturbation windows, uniform adds
    elsewhere) against the oracle's point-by-point evaluation, for blocks whose waves straddle
    the start, the end and the middle of the coordinate range (the sharded and Recur paths
    launch such blocks)."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    rng = np.random.default_rng(n + i0)
    x = rng.uniform(-1.5, 1.5, n); h = rng.uniform(1e-7, 1e-6, n)
    if kind == "rosenbrock":
        d, o = DeviceObjective(ctx, L.OBJ_ROSENBROCK, n), oracle.rosenbrock(n)
    elif kind == "quadratic":
        dd, bb = oracle.quadratic_data(n, bscale=4.0)
        d, o = DeviceObjective(ctx, L.OBJ_QUADRATIC, n, 0, dd, bb), oracle.Obj(oracle.QUADRATIC, n, 0, dd, bb)
    else:   # (power 3 goes through the device pow(): ulp-close, tested by tolerance elsewhere)
        d, o = DeviceObjective(ctx, L.OBJ_POWER, n, power=2.0), oracle.power(n, 2)
    f0, g = d.fd_gradient(ctx.tensor(x), ctx.tensor(h), i0, cnt)
    ref = oracle.fd_gradient(o, x, h)[i0:i0 + cnt]
    assert np.array_equal(_np(g), ref)
    assert _np(f0)[0] == oracle.obj_eval(o, x)


@pytest.mark.parametrize("n", [3, 4096])
def test_fd_gradient_quadratic_and_power_bitwise(ctx, oracle, n):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    dd, bb = oracle.quadratic_data(n)
    x = np.linspace(-1, 1, n); h = np.full(n, 1e-6)
    q = DeviceObjective(ctx, L.OBJ_QUADRATIC, n, 0, dd, bb)
    _, g = q.fd_gradient(ctx.tensor(x), ctx.tensor(h))
    assert np.array_equal(_np(g), oracle.fd_gradient(oracle.Obj(oracle.QUADRATIC, n, 0, dd, bb), x, h))
    p2 = DeviceObjective(ctx, L.OBJ_POWER, n, power=2.0)
    _, g2 = p2.fd_gradient(ctx.tensor(x), ctx.tensor(h))
    assert np.array_equal(_np(g2), oracle.fd_gradient(oracle.power(n, 2), x, h))


def test_fd_gradient_power3_known_answer(ctx):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    d = DeviceObjective(ctx, L.OBJ_POWER, 5, power=3.0)   # testGradientEvaluation, Examples.cpp:512-540
    _, g = d.fd_gradient(ctx.tensor(np.full(5, 3.0)), ctx.tensor(np.full(5, 1e-6)))
    np.testing.assert_allclose(_np(g), 27.0, rtol=1e-5)


def test_fd_jacobian_cubic_bitwise_expcurve_close(ctx, oracle):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    oc = oracle.cubic()
    c = DeviceObjective(ctx, L.OBJ_CUBIC, 4, 100, oc.p0, oc.p1)
    x = np.full(4, 0.1); h = np.full(4, 1e-6)
    F0, JT = c.fd_jacobian(ctx.tensor(x), ctx.tensor(h))
    assert np.array_equal(_np(JT).T, oracle.fd_jacobian(oc, x, h))
    assert np.array_equal(_np(F0), oracle.obj_eval_multi(oc, x))
    oe = oracle.expcurve()
    e = DeviceObjective(ctx, L.OBJ_EXPCURVE, 3, 100, oe.p0, oe.p1)
    x = np.full(3, 0.1)
    _, JT = e.fd_jacobian(ctx.tensor(x), ctx.tensor(h[:3]))
    ref = oracle.fd_jacobian(oe, x, h[:3])
    # device exp vs glibc exp differ by <= 1 ulp per term; the FD quotient amplifies by |F|/h
    assert np.all(np.abs(_np(JT).T - ref) <= 4 * EPS * (1 + np.abs(oracle.obj_eval_multi(oe, x)))[:, None] / 1e-6 * 10)


@pytest.mark.parametrize("m,n,j0,cnt", [(300, 70, 0, 70), (300, 70, 13, 29), (1000, 129, 64, 65), (257, 33, 32, 1),
                                       (700, 300, 0, 300), (700, 300, 37, 200), (130, 16, 0, 16), (130, 17, 16, 1),
                                       (1500, 1000, 0, 1000), (513, 2048, 100, 700), (257, 400, 250, 150)])
def test_fd_jacobian_linres_bitwise(ctx, oracle, m, n, j0, cnt):
    """Prefix-shared chains (tiles start from the base chain's 16-column checkpoints) are
    the same fma sequence as full-length evaluation: bitwise equal to the oracle's n+1 evals."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    A, xs, y = oracle.linres_data(m, n)
    d = DeviceObjective(ctx, L.OBJ_LINRES, n, m, A, y)
    x = np.linspace(-0.5, 0.5, n); h = np.full(n, 1e-7)
    F0, JT = d.fd_jacobian(ctx.tensor(x), ctx.tensor(h), j0, cnt)
    o = oracle.Obj(oracle.LINRES, n, m, A, y)
    ref = oracle.fd_jacobian(o, x, h)
    assert np.array_equal(_np(JT), ref.T[j0:j0 + cnt])
    assert np.array_equal(_np(F0), oracle.obj_eval_multi(o, x))
    assert np.array_equal(_np(d.eval(ctx.tensor(x))), oracle.obj_eval_multi(o, x))
    # caller-provided F0 (compute_f0 = 0, the LM path): same Jacobian, F0 untouched
    F0b = ctx.tensor(oracle.obj_eval_multi(o, x))
    _, JT2 = d.fd_jacobian(ctx.tensor(x), ctx.tensor(h), j0, cnt, F0=F0b, compute_f0=False)
    assert np.array_equal(_np(JT2), ref.T[j0:j0 + cnt])
    assert np.array_equal(_np(F0b), oracle.obj_eval_multi(o, x))


@pytest.mark.parametrize("m,n,P", [(513, 700, 3), (300, 1000, 4), (257, 2048, 8), (130, 129, 2)])
def test_fd_jacobian_tiles_bitwise(ctx, oracle, m, n, P):
    """LevMarqMPI's cost-balanced tile sets (pnol_fd_tiles), each rank's tiles evaluated in
    place: the union is bitwise the oracle's FD Jacobian and untouched rows stay untouched."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L, fd_tiles
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    A, xs, y = oracle.linres_data(m, n)
    d = DeviceObjective(ctx, L.OBJ_LINRES, n, m, A, y)
    x = np.linspace(-0.5, 0.5, n); h = np.full(n, 1e-7)
    o = oracle.Obj(oracle.LINRES, n, m, A, y)
    ref = oracle.fd_jacobian(o, x, h).T
    full = np.zeros((n, m))
    for r in range(P):
        tiles = fd_tiles(n, P, r)
        JT = ctx.tensor(np.full((n, m), 7.0))
        F0, JT = d.fd_jacobian_tiles(ctx.tensor(x), ctx.tensor(h), tiles, JT)
        got = _np(JT)
        mine = np.zeros(n, dtype=bool)
        for s0, c in tiles:
            mine[s0:s0 + c] = True
        assert np.array_equal(got[mine], ref[mine]), r
        assert np.all(got[~mine] == 7.0)
        assert np.array_equal(_np(F0), oracle.obj_eval_multi(o, x))
        full[mine] = got[mine]
    assert np.array_equal(full, ref)


@pytest.mark.parametrize("m,n", [(513, 700), (300, 129), (1000, 2048)])
def test_fd_checkpoint_reuse_bitwise(ctx, oracle, m, n):
    """pnol_dobj_eval_ckpt_d then an FD call with compute_f0 = 2 (the LM accepted-step path)
    skips the base-chain pass and stays bitwise; checkpoints of another x are not reused."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L, fd_tiles
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    A, xs, y = oracle.linres_data(m, n)
    d = DeviceObjective(ctx, L.OBJ_LINRES, n, m, A, y)
    o = oracle.Obj(oracle.LINRES, n, m, A, y)
    x = np.linspace(-0.5, 0.5, n); h = np.full(n, 1e-7)
    x2 = np.linspace(0.3, -0.2, n)
    ref = oracle.fd_jacobian(o, x, h).T
    tiles = fd_tiles(n, 1, 0)
    dx, dx2, dh = ctx.tensor(x), ctx.tensor(x2), ctx.tensor(h)
    F = d.eval_ckpt(dx)
    assert np.array_equal(_np(F), oracle.obj_eval_multi(o, x))
    _, JT = d.fd_jacobian_tiles(dx, dh, tiles, ctx.empty(n, m), F0=F, compute_f0=2)
    assert np.array_equal(_np(JT), ref)
    # checkpoints now belong to x2: an FD call at x with compute_f0 = 2 must recompute them
    d.eval_ckpt(dx2)
    _, JT = d.fd_jacobian_tiles(dx, dh, tiles, ctx.empty(n, m), F0=F, compute_f0=2)
    assert np.array_equal(_np(JT), ref)


@pytest.mark.parametrize("m,n", [(1000, 300), (4096, 2048)])
def test_fd_checkpoint_reuse_is_content_keyed(ctx, oracle, m, n):
    """compute_f0 = 2 after x was updated IN PLACE (same device pointer): the device check of
    x against the slot's recorded content fails, so F0 and the checkpoints are recomputed --
    the Jacobian and F0 are x's new ones, bitwise.  A new objective at a recycled address never
    matches an old slot (slots are tagged by creation id).  compute_f0 = 3 (the LM loop's
    trusted reuse) on an unchanged x stays bitwise."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L, fd_tiles
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    A, xs, y = oracle.linres_data(m, n)
    o = oracle.Obj(oracle.LINRES, n, m, A, y)
    x = np.linspace(-0.5, 0.5, n); x2 = np.linspace(0.3, -0.2, n); h = np.full(n, 1e-7)
    tiles = fd_tiles(n, 1, 0)
    d = DeviceObjective(ctx, L.OBJ_LINRES, n, m, A, y)
    dx, dh = ctx.tensor(x), ctx.tensor(h)
    F = d.eval_ckpt(dx)
    dx.copy_(ctx.tensor(x2))                       # in place: same pointer, new content
    _, JT = d.fd_jacobian_tiles(dx, dh, tiles, ctx.empty(n, m), F0=F, compute_f0=2)
    assert np.array_equal(_np(JT), oracle.fd_jacobian(o, x2, h).T)
    assert np.array_equal(_np(F), oracle.obj_eval_multi(o, x2))
    # unchanged x: trusted reuse (3) and checked reuse (2) agree bitwise with a fresh call (1)
    F2 = d.eval_ckpt(dx)
    _, J3 = d.fd_jacobian_tiles(dx, dh, tiles, ctx.empty(n, m), F0=F2, compute_f0=3)
    _, J1 = d.fd_jacobian_tiles(dx, dh, tiles, ctx.empty(n, m), F0=ctx.empty(m), compute_f0=1)
    assert np.array_equal(_np(J3), _np(J1))
    # a different objective (other data) created after this one is destroyed
    d.close()
    A2 = A[::-1].copy()
    d2 = DeviceObjective(ctx, L.OBJ_LINRES, n, m, A2, y)
    o2 = oracle.Obj(oracle.LINRES, n, m, A2, y)
    Fz = ctx.tensor(oracle.obj_eval_multi(o2, x2))
    _, J2 = d2.fd_jacobian_tiles(dx, dh, tiles, ctx.empty(n, m), F0=Fz, compute_f0=2)
    assert np.array_equal(_np(J2), oracle.fd_jacobian(o2, x2, h).T)


@pytest.mark.parametrize("m,n,t64", [(2000, 300, "0"), (5000, 1000, "0"), (777, 129, "0"), (16384, 2048, "0"),
                                     (5000, 1000, "1"), (777, 129, "1"), (16384, 2048, "1"), (300, 100, "0"),
                                     (300, 100, "1"), (4100, 65, "1")])
def test_lm_sliced_jacobian_and_normal_bitwise(ctx, m, n, t64, monkeypatch):
    """One rank of the m-sliced LevMarqMPI path: pnol_lm_jacobian_mpi_d writes the same J values
    into the sliced layout, and pnol_lm_normal_mpi_d gives A, diag(J^T J) and -J^T F bitwise
    equal to pnol_fd_jacobian_d + pnol_jtj_d + pnol_jtr_d (one summation tree on both paths).
    t64 = "1": the 64 x 64-tile SYRK the ranks of an 8-GPU run use (same per-element sums)."""
    monkeypatch.setenv("PNOL_SYRK_T64", t64)
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective, lm_sliced_layout
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.linspace(-0.5, 0.5, n)); h = ctx.tensor(np.full(n, 1e-7))
    F0a, JTa = d.fd_jacobian(x, h, 0, n)
    Aa, da = ctx.jtj(JTa, 0.37, want_diag=True)
    ra = ctx.jtr(JTa, F0a)
    mS, tot = lm_sliced_layout(m, n)
    assert mS % 64 == 0 and L.LM_SLICES * mS >= m and tot == L.LM_SLICES * n * mS
    F0b, JTs = d.lm_jacobian_mpi(x, h)
    Ab, rb, db = ctx.lm_normal_mpi(JTs, m, n, 0.37, F0b, want_diag=True)
    ctx.synchronize()
    assert np.array_equal(_np(F0b), _np(F0a))
    js = _np(JTs).reshape(L.LM_SLICES, n, mS)
    ja = _np(JTa)
    for s in range(L.LM_SLICES):
        w = min(mS, max(0, m - s * mS))
        assert np.array_equal(js[s, :, :w], ja[:, s * mS:s * mS + w]), s
    assert np.array_equal(_np(Ab), _np(Aa))
    assert np.array_equal(_np(db), _np(da))
    assert np.array_equal(_np(rb), _np(ra))
    # and the tree sums are the sums: fp64 torch reference
    import torch
    J = JTa.double()
    ref = J @ J.T
    assert float((torch.diagonal(Ab) / 1.37 - torch.diagonal(ref)).abs().max() / ref.abs().max()) < 1e-12
    rr = -(J @ F0a)
    assert float((rb - rr).abs().max() / rr.abs().max()) < 1e-12


@pytest.mark.parametrize("m,n", [(16384, 2048), (5000, 1000), (777, 129)])
def test_lm_normal_solve_mpi_one_rank_bitwise(ctx, m, n):
    """One rank of pnol_lm_normal_solve_mpi_d (the split-K partials of its slices summed by the
    Cholesky's first tasks): rhs, sigma, x + sigma and the status bitwise pnol_lm_normal_mpi_d +
    pnol_solve_step_d; pnol_lm_normal_unpack_mpi_d forms the same A."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.linspace(-0.5, 0.5, n)); h = ctx.tensor(np.full(n, 1e-7))
    F0, JTs = d.lm_jacobian_mpi(x, h)
    for lam in (0.37, 1e-3):
        Aa, ra = ctx.lm_normal_mpi(JTs, m, n, lam, F0)
        sa, xa, ia = ctx.solve_step(Aa, ra, x)
        rb, sb, xb, ib = ctx.lm_normal_solve_mpi(JTs, m, n, lam, F0, x)
        ctx.synchronize()
        assert ia == 0 and ib == 0
        assert np.array_equal(_np(rb), _np(ra)) and np.array_equal(_np(sb), _np(sa)) and np.array_equal(_np(xb), _np(xa))
        Ab = ctx.lm_normal_unpack_mpi(m, n, lam)
        ctx.synchronize()
        assert np.array_equal(_np(Ab), _np(Aa))


@pytest.mark.parametrize("m,n,chunks", [(2000, 700, 4), (1500, 1000, 3), (513, 2048, 8), (300, 129, 2), (400, 300, 1)])
def test_fd_jtj_pipelined_bitwise(ctx, m, n, chunks):
    """The pipelined FD Jacobian + J^T J (two streams, chunked) equals the two separate calls
    bitwise: JT, F0, A (with the Marquardt diagonal) and diag(J^T J)."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.linspace(-0.5, 0.5, n)); h = ctx.tensor(np.full(n, 1e-7))
    F0a, JTa = d.fd_jacobian(x, h, 0, n)
    Aa, da = ctx.jtj(JTa, 0.37, want_diag=True)
    JTb, Ab = ctx.empty(n, m), ctx.empty(n, n)
    for _ in range(2):   # repeated: events / aux stream reuse
        F0b, JTb, Ab, db = d.fd_jtj(x, h, 0.37, JTb, Ab, nchunks=chunks, want_diag=True)
    ctx.synchronize()
    assert np.array_equal(_np(JTb), _np(JTa))
    assert np.array_equal(_np(F0b), _np(F0a))
    assert np.array_equal(_np(Ab), _np(Aa))
    assert np.array_equal(_np(db), _np(da))


@pytest.mark.parametrize("m,n", [(16384, 2048), (5000, 1000), (777, 129), (300, 40)])
def test_fd_normal_bitwise(ctx, m, n):
    """pnol_fd_normal_d (FD Jacobian + A + -J^T F in one queue, the -J^T F tree in the J^T J reduce
    launch) equals pnol_fd_jacobian_d + pnol_jtj_d + pnol_jtr_d bitwise, over repeated calls (the
    second call's JT is a new point's)."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    h = ctx.tensor(np.full(n, 1e-7))
    JTb, Ab, rb = ctx.empty(n, m), ctx.empty(n, n), ctx.empty(n)
    for rep, lo in enumerate((-0.5, -0.25)):
        x = ctx.tensor(np.linspace(lo, 0.5, n))
        F0a, JTa = d.fd_jacobian(x, h, 0, n)
        Aa = ctx.jtj(JTa, 0.37)
        ra = ctx.jtr(JTa, F0a)
        F0b, JTb, Ab, rb = d.fd_normal(x, h, 0.37, JTb, Ab, rb)
        ctx.synchronize()
        assert np.array_equal(_np(JTb), _np(JTa)), rep
        assert np.array_equal(_np(F0b), _np(F0a)), rep
        assert np.array_equal(_np(Ab), _np(Aa)), rep
        assert np.array_equal(_np(rb), _np(ra)), rep


@pytest.mark.parametrize("reduce", ["launch", "tasks", "tail", "tail_sc1", "tail_rowsorder"])
@pytest.mark.parametrize("m,n", [(16384, 2048), (5000, 1000), (777, 129), (3000, 257), (2000, 700), (512, 96)])
def test_lm_trip_bitwise(ctx, monkeypatch, m, n, reduce):
    """The LM trip without A (pnol_lm_trip_d: the reduce launch writes the J^T J split-K partials'
    sums straight into the persistent Cholesky's padded matrix and -J^T F into b -- or, reduce =
    tasks, the persistent launch's first tasks do that reduce; tail, the reduce workgroups ride in
    the SYRK's own launch behind an in-launch split-K hand-off, _sc1 with write-through partials)
    gives JT, F0, rhs, sigma, x + sigma
    and the solve status bitwise those of pnol_fd_normal_d + pnol_solve_step_d, over repeated trips
    at new points and lambdas; the A the LU fallback forms from the trip's partials
    (pnol_lm_trip_normal_d) is bitwise pnol_fd_normal_d's A."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    monkeypatch.setenv("PNOL_LM_REDUCE", reduce.split("_")[0])
    monkeypatch.setenv("PNOL_SYRK_RED_SC1", "1" if reduce.endswith("_sc1") else "0")
    monkeypatch.setenv("PNOL_SYRK_DLAST", "0" if reduce.endswith("_rowsorder") else "1")
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    h = ctx.tensor(np.full(n, 1e-7))
    JTa, Aa, ra, JTb = ctx.empty(n, m), ctx.empty(n, n), ctx.empty(n), ctx.empty(n, m)
    for rep, (lo, lam) in enumerate(((-0.5, 0.37), (-0.25, 1e-3), (0.1, 20.0))):
        x = ctx.tensor(np.linspace(lo, 0.5, n))
        F0a, JTa, Aa, ra = d.fd_normal(x, h, lam, JTa, Aa, ra)
        sa, xa, ia = ctx.solve_step(Aa, ra, x)
        F0b, JTb, rb, sb, xb, ib = d.lm_trip(x, h, lam, JTb)
        ctx.synchronize()
        assert ia == 0 and ib == 0, (rep, ia, ib)
        assert np.array_equal(_np(JTb), _np(JTa)), rep
        assert np.array_equal(_np(F0b), _np(F0a)), rep
        assert np.array_equal(_np(rb), _np(ra)), rep
        assert np.array_equal(_np(sb), _np(sa)), rep
        assert np.array_equal(_np(xb), _np(xa)), rep
        Ab = ctx.lm_trip_normal(m, n, lam)
        ctx.synchronize()
        assert np.array_equal(_np(Ab), _np(Aa)), rep


def test_lm_trip_reports_non_spd(ctx):
    """A non-positive pivot met by the fused trip's Cholesky is reported in the status word (the
    LM loop then forms A from the partials and redoes the solve with the LU), and the next trip
    on the same context is sound again."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    n = 300
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, 200)   # 200 residuals: J^T J singular
    x, h = ctx.tensor(np.linspace(-0.5, 0.5, n)), ctx.tensor(np.full(n, 1e-7))
    *_, info = d.lm_trip(x, h, 0.0, ctx.empty(n, 200))
    assert info != 0
    d2 = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, 1000)
    JTa, Aa, ra = ctx.empty(n, 1000), ctx.empty(n, n), ctx.empty(n)
    F0a, JTa, Aa, ra = d2.fd_normal(x, h, 0.5, JTa, Aa, ra)
    sa, _, ia = ctx.solve_step(Aa, ra, x)
    *_, sb, _, ib = d2.lm_trip(x, h, 0.5, ctx.empty(n, 1000))
    assert ia == 0 and ib == 0
    assert np.array_equal(_np(sb), _np(sa))


def test_lm_agree_status_codes_one_rank(ctx):
    """pnol_lm_agree_status_d with one rank: dinfo[1] = the action code of dinfo[0] -- 0 none, 1 a
    timed-out Cholesky wait (kCholTimeout = -7: relaunch the Cholesky), 2 any other nonzero status
    (a non-positive / NaN pivot: the reference-order LU)."""
    import ctypes as C
    import torch
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    for v, code in ((0, 0), (-7, 1), (5, 2), (-1, 2), (2049, 2)):
        t = torch.tensor([v, 99], dtype=torch.int32, device=f"cuda:{ctx.device}")
        L.check(L.lib().pnol_lm_agree_status_d(ctx.h, C.c_void_p(t.data_ptr())), "agree")
        ctx.synchronize()
        assert t.cpu().tolist() == [v, code], (v, t.cpu().tolist())


def test_lm_trip_normal_refuses_stale_partials(ctx):
    """pnol_lm_trip_normal_d forms A only from the partials of the last pnol_lm_trip_d of the same
    (m, n): after another J^T J call overwrote them, or for another shape, it refuses
    (PNOL_ERR_ARG) instead of returning a wrong A."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    m, n = 1000, 300
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x, h = ctx.tensor(np.linspace(-0.5, 0.5, n)), ctx.tensor(np.full(n, 1e-7))
    JT = ctx.empty(n, m)
    d.lm_trip(x, h, 0.5, JT)
    ctx.synchronize()
    ctx.lm_trip_normal(m, n, 0.5)                          # the trip's own partials: fine
    with pytest.raises(L.PnolError) as e:
        ctx.lm_trip_normal(m + 64, n, 0.5)                 # another shape
    assert e.value.status == L.PNOL_ERR_ARG
    ctx.jtj(JT, 0.5)                                       # overwrites the partials
    ctx.synchronize()
    with pytest.raises(L.PnolError) as e:
        ctx.lm_trip_normal(m, n, 0.5)
    assert e.value.status == L.PNOL_ERR_ARG


def test_synthetic_data_matches_oracle_stream(ctx, oracle):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective
    m, n = 200, 50
    d = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    A, xs, y = oracle.linres_data(m, n)
    assert np.array_equal(d.xstar, xs)
    x = np.zeros(n)
    F = _np(d.eval(ctx.tensor(x)))          # r(0) = -y
    assert np.array_equal(F, -y)
    q = DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, 64, bscale=4.0)
    dd, bb = oracle.quadratic_data(64, bscale=4.0)
    _, g = q.fd_gradient(ctx.tensor(np.zeros(64)), ctx.tensor(np.full(64, 1e-6)))
    assert np.array_equal(_np(g), oracle.fd_gradient(oracle.Obj(oracle.QUADRATIC, 64, 0, dd, bb), np.zeros(64),
                                                      np.full(64, 1e-6)))
