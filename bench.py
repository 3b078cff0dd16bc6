"""bench.py -- MI355X PNOL hot path: LM iterations/s at m=16384, n=2048 (+ BFGS H.g GB/s).

A "step" is one LevenbergMarquardt loop trip of the C++ drop-in (LevMarq at N=1, LevMarqMPI
at N>1, one process per GPU, FD columns sharded with an RCCL allgather): the batched
finite-difference Jacobian of the synthetic dense residual r(x) = A x - y (SURVEY 8(d)
cfg 3/4, splitmix64 seed 0x5EED2018, data generated in HBM), J^T J on fp64 MFMA with the
Marquardt diagonal, -J^T F, the damped Cholesky solve, F(x + sigma) and the accept/reject
test.  Every trip recomputes the whole Jacobian (all n perturbed evaluations), J^T J, -J^T F
and the solve, also after a rejected step, as the reference does.  F(x) and its prefix
checkpoints depend on x alone and are kept from the evaluation that made them (the trial
point's, or the trip before a rejection); the evaluation counter still counts F(x) per trip.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Per-kernel durations come from HIP events recorded on the
solver's own stream during the timed steps (pnol_ctx_timer); `cpu_baseline` times the
oracle (oracle/, the CPU restatement of the reference) on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

M_RES, N_PAR = 16384, 2048          # BASELINE.json metric: LM at m=16384, n=2048
HG_N = 8192                         # north-star H.g size (>= 60% of HBM roofline target)
HBM_PEAK_GBS = 8000.0               # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6             # fp64 matrix == fp64 vector peak on MI355X


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hg", action="store_true")
    ap.add_argument("--no-timers", action="store_true", help="no per-kernel HIP events in the timed region")
    # (not --m / --n: torch.distributed.run would take those for abbreviations of its own options)
    ap.add_argument("--residuals", type=int, default=M_RES, help="m, residual rows (default: the metric's 16384)")
    ap.add_argument("--params", type=int, default=N_PAR, help="n, parameters (default: the metric's 2048)")
    ap.add_argument("--host-comm", action="store_true",
                    help="rehearsal on one GPU: gloo + the library's host communicator instead of RCCL")
    ap.add_argument("--no-bfgs", action="store_true", help="skip the BFGS cfg-2 / BFGS_Bnd cfg-5 solve blocks")
    return ap.parse_args()


def _red_dev():
    """Device for collective scratch tensors: cuda under nccl (RCCL), cpu under gloo."""
    import torch.distributed as dist
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def _timer(L, ctx_h, name):
    ms, cnt = C.c_double(), C.c_int()
    L.check(L.lib().pnol_ctx_timer(ctx_h, name.encode(), C.byref(ms), C.byref(cnt)), "pnol_ctx_timer")
    return ms.value, cnt.value


def pmc_traffic():
    """Per-launch L2<->fabric bytes of the hot kernels from the newest committed PMC summary
    (profiles/r*_pmc_traffic.json, made by tools/pmc_traffic.py from separate rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE passes of this bench), or {} if none is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return {}
    try:
        return json.load(open(files[-1])).get("kernels", {})
    except (OSError, ValueError):
        return {}


def fd_flop_executed(m, n, tiles, bk=16, pw=32):
    """fp64 flops the FD GEMM runs for the (start, count) point tiles: each wave's 32 points
    continue the base chain from the checkpoint at ks = 16*floor(c0 / 16) (c0 = the wave's first
    column) to k = n-1 (k_linres_fdP<true>, the default kernel)."""
    tot = 0
    for s0, cnt in tiles:
        for p0 in range(0, cnt, pw):
            c0 = s0 + p0
            tot += min(pw, cnt - p0) * (n - (c0 // bk) * bk)
    return 2.0 * m * tot


def fd_flop_minimal(m, tiles, n):
    """The flops no bitwise FD evaluation of the sequential fma chain can avoid: point j must
    run its own chain from k = j (its first differing term) to n-1."""
    return 2.0 * m * sum(n - j for s0, cnt in tiles for j in range(s0, s0 + cnt))


def pmc_valu(kind="fd_valu"):
    """VALU- (or MFMA-) busy fractions of the hot kernels from the newest committed PMC summary
    (profiles/r*_pmc_fd_valu.json / r*_pmc_syrk_mfma.json, tools/pmc_valu.py), or {}."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{kind}.json")))
    if not files:
        return {}
    try:
        return json.load(open(files[-1])).get("kernels", {})
    except (OSError, ValueError):
        return {}


def bench_hg(ctx, n, reps=20):
    """Standalone p = -D g at n (8 n^2 + 16 n bytes per launch) and the fused BFGS pass
    (16 n^2 bytes with write-back), timed with HIP events on the context stream."""
    import torch
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    g = torch.randn(n, dtype=torch.float64, device="cuda")
    D = torch.randn(n, n, dtype=torch.float64, device="cuda")
    flush = torch.empty(512 * 1024 * 1024 // 8, dtype=torch.float64, device="cuda")   # > 256 MiB MALL
    L.check(L.lib().pnol_ctx_enable_timers(ctx.h, 1), "timers")
    L.check(L.lib().pnol_ctx_reset_timers(ctx.h), "reset")
    for _ in range(3):
        ctx.hg(D, g)
    ctx.synchronize()
    L.check(L.lib().pnol_ctx_reset_timers(ctx.h), "reset")
    for _ in range(reps):
        flush.fill_(1.0)      # cold Infinity Cache before every launch
        ctx.hg(D, g)
    ctx.synchronize()
    ms, cnt = _timer(L, ctx.h, "hg")
    t_hg = ms / cnt * 1e-3
    hg_bytes = 8.0 * n * n + 16.0 * n
    # fused pass with write-back and a pending correction (the fast-mode BFGS iteration)
    y = torch.randn(n, dtype=torch.float64, device="cuda")
    s, a, b = (torch.randn(n, dtype=torch.float64, device="cuda") * 1e-3 for _ in range(3))
    ctx.bfgs_pass(D, y, g, (s, a, b), True)
    ctx.synchronize()
    L.check(L.lib().pnol_ctx_reset_timers(ctx.h), "reset")
    for _ in range(reps):
        flush.fill_(1.0)
        ctx.bfgs_pass(D, y, g, (s, a, b), True)
    ctx.synchronize()
    ms2, cnt2 = _timer(L, ctx.h, "bfgs_pass")
    t_pass = ms2 / cnt2 * 1e-3
    del D, flush
    torch.cuda.empty_cache()
    return {
        "n": n, "hg_us": t_hg * 1e6, "hg_GBps": hg_bytes / t_hg / 1e9,
        "hg_frac_of_hbm": hg_bytes / t_hg / 1e9 / HBM_PEAK_GBS,
        "fused_pass_us": t_pass * 1e6, "fused_pass_GBps": 16.0 * n * n / t_pass / 1e9,
        "fused_pass_frac_of_hbm": 16.0 * n * n / t_pass / 1e9 / HBM_PEAK_GBS,
        "cold_cache": True,
    }


def bench_hg_sharded(h, n, world, rank, reps=20):
    """BFGS D row-sharded over the ranks (pnol_hg_mpi_d, collective): each rank streams its
    rows of D and the row shards of p are allgathered.  Returns the whole-job rate
    (8 n^2 + 16 n bytes / max-over-ranks time, allgather included)."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    rb, rc = C.c_int(), C.c_int()
    L.check(L.lib().pnol_bfgs_rows(n, world, rank, C.byref(rb), C.byref(rc)), "bfgs_rows")
    D = torch.randn(max(rc.value, 1), n, dtype=torch.float64, device="cuda")
    g = torch.randn(n, dtype=torch.float64, device="cuda")
    p = torch.empty(n, dtype=torch.float64, device="cuda")

    def once():
        L.check(L.lib().pnol_hg_mpi_d(h, D.data_ptr(), n, g.data_ptr(), p.data_ptr(), n), "hg_mpi")

    for _ in range(3):
        once()
    L.check(L.lib().pnol_ctx_synchronize(h), "sync")
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    L.check(L.lib().pnol_ctx_synchronize(h), "sync")
    t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=_red_dev())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t = float(t.item())
    del D
    torch.cuda.empty_cache()
    byts = 8.0 * n * n + 16.0 * n
    return {"n": n, "ranks": world, "rows_per_rank": rc.value, "hg_us": t * 1e6, "hg_GBps_whole_job": byts / t / 1e9,
            "note": "host-timed (allgather included), warm cache; per-rank HBM share 1/P of D"}


CFG2_P = [1e-4, 0.9, 1e-6, 1, 1000, 1e-6, 1e-3, 200, 1e-9, 1e-6, 0, 0]      # BFGS setParams order (tests)
CFG5_P = [1e-4, 0.8, 1e-6, 1, 1e-10, 2, 50, 1e-5, 1e-6, 1e-3, 200, 1e-5, 1e-5, 0, -1]   # testBFGSBnd, Examples.cpp:75


def _box_qp_solution(d, b, lb, ub, sweeps=400):
    """KKT point of the cfg-5 box QP (tridiagonal diag(d) + 0.25 off-diagonals): projected
    red-black Gauss-Seidel, contraction <= 0.5 per sweep (a check of the solve, not timed)."""
    n = len(d)
    x = np.zeros(n)
    for _ in range(sweeps):
        for par in (0, 1):
            i = np.arange(par, n, 2)
            nb = np.where(i + 1 < n, x[np.minimum(i + 1, n - 1)], 0.0) + np.where(i >= 1, x[np.maximum(i - 1, 0)], 0.0)
            x[i] = np.clip((b[i] - 0.25 * nb) / d[i], lb[i], ub[i])
    return x


def bench_bfgs_solve(ctx, which, n, bscale, params, bounds=None):
    """One whole BFGS (which=0, cfg 2) or BFGS_Bnd (which=2, cfg 5) solve of the synthetic
    quadratic generated in HBM, with the per-phase host profile and the device kernel timers."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective, run_bfgs
    obj = DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, n, 0, bscale=bscale)
    dctx = C.c_void_p()
    L.check(L.lib().pnol_default_ctx(C.byref(dctx)), "pnol_default_ctx")
    L.check(L.lib().pnol_ctx_enable_timers(dctx, 1), "timers")
    L.check(L.lib().pnol_ctx_reset_timers(dctx), "timers")
    prof = {}
    lb, ub = bounds if bounds else (None, None)
    t0 = time.perf_counter()
    out = run_bfgs(obj, np.zeros(n), params, which=which, lb=lb, ub=ub, profile=prof,
                   trace_cap=(1 << 20) if which == 2 else 0)
    wall = time.perf_counter() - t0
    X, res = out[0], out[1]
    kern = {k: _timer(L, dctx, k) for k in ("fd_gradient", "bfgs_pass", "hg")}
    L.check(L.lib().pnol_ctx_enable_timers(dctx, 0), "timers")
    it = max(int(prof.get("iterations", 0)), 1)
    blk = {"n": n, "iterations": int(prof.get("iterations", 0)), "evals": int(res.evals), "seconds": wall,
           "ms_per_iteration": wall / it * 1e3, "iterations_per_s": it / wall, "f0": res.f0, "fopt": res.fopt,
           "phases_ms_per_iteration": {k: prof[k] / it * 1e3 for k in ("fd_gradient_s", "line_search_s", "update_s")},
           "other_ms_per_iteration": (prof["total_s"] - prof["fd_gradient_s"] - prof["line_search_s"]
                                      - prof["update_s"]) / it * 1e3,
           "line_search_points": int(prof["line_search_points"]), "gradient_calls": int(prof["gradient_calls"]),
           "kernel_ms_total": {k: v[0] for k, v in kern.items()}, "kernel_launches": {k: v[1] for k, v in kern.items()}}
    kern_ms = sum(v[0] for v in kern.values())
    blk["kernel_ms_per_iteration"] = kern_ms / it
    blk["iteration_over_kernel_sum"] = (wall * 1e3 / it) / (kern_ms / it) if kern_ms > 0 else None
    if which == 2:
        import oracle as O   # test infrastructure: only the splitmix64 data stream, for the KKT check
        d, b = O.quadratic_data(n, bscale=bscale)
        xs = _box_qp_solution(d, b, lb, ub)
        tr = out[2]
        blk.update({"max_recursion_depth": int(prof["max_recursion_depth"]),
                    "inside_box": bool(np.all(X >= lb) and np.all(X <= ub)),
                    "f_trace_nonincreasing": bool(np.all(np.diff(tr) <= 0)),
                    "active_bounds": int(np.sum(np.abs(X - lb) < 1e-5) + np.sum(np.abs(X - ub) < 1e-5)),
                    "max_abs_err_vs_kkt_point": float(np.max(np.abs(X - xs)))})
    obj.close()
    return blk


def _median_time(fn, reps):
    """Median wall time of `reps` calls of fn() (and every sample, for the spread)."""
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo, as lscpu prints it) and its logical CPU count."""
    name = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                name = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return name, os.cpu_count()


def cpu_lm_trip(O, objs, x, h, ex, P):
    """One whole LevMarq loop trip of the reference CPU path at the oracle's (m, n), timed end to
    end once on P threads (LevenbergMarquardt.cpp:55-103 at the rank count P of
    LevenbergMarquardtMPI): F(x); the FD Jacobian with its columns dealt round-robin over the P
    threads (PNOL_Objective.cpp:228-246); J^T J by the reference's matrixMultiply, its rows split
    over the threads (the reference replicates the whole product on every rank -- splitting it
    is generous to the CPU); rhs = -J^T F (matrixVectorMultiply); luSolve; F(x + sigma).  Returns
    (seconds, sigma)."""
    o0 = objs[0]
    m, n = o0.s.m, len(x)
    t0 = time.perf_counter()
    F = O.obj_eval_multi(o0, x)
    J = np.empty((m, n))

    def cols(q):
        for j in range(q, n, P):                 # owner(j) = j mod P
            xj = x.copy()
            xj[j] = xj[j] + h[j]
            J[:, j] = (O.obj_eval_multi(objs[q], xj) - F) / h[j]
    list(ex.map(cols, range(P)))
    JT = np.ascontiguousarray(J.T)
    blk = (n + P - 1) // P
    parts = list(ex.map(lambda q: O.matmul(JT[q * blk:min(n, (q + 1) * blk)], J) if q * blk < n else None, range(P)))
    A = np.vstack([p for p in parts if p is not None])
    A[np.diag_indices(n)] *= 1.0 + 0.001
    rhs = -O.matvec(JT, F)
    sigma = O.lusolve(A, rhs)
    O.obj_eval_multi(o0, x + sigma)
    return time.perf_counter() - t0, sigma


def cpu_baseline(m, n, budget_s=20.0):
    """The reference path on the host cores: the oracle (the CPU restatement of the reference,
    loop for loop) built -O3 -march=x86-64-v3 -ffp-contract=off (liboracle_fast.so), timed on a
    bounded sample of one LM loop trip at (m, n) and extrapolated to the whole trip.  Every leg
    is the median of >= 3 timings (the samples are reported beside it):
      - residual evaluations (the n + 2 of a trip), 1 thread and P threads -- the reference's
        MPI FD sharding (PNOL_Objective.cpp:202-299) as P concurrent evaluators;
      - rows of J^T J with the reference's matrixMultiply, 1 and P threads;
      - the reference LU (luSolve) at n = 1024, scaled by (n / 1024)^3.
    value = LM trips per second with P threads (P = the host cores this process may use, at
    most 16, the box's per-GPU CPU share), from one whole trip timed end to end (cpu_lm_trip);
    the sampled legs above extrapolate the 1-thread trip and cross-check it.  Also,
    single-threaded: cfg 1 (BFGS on the 2-D
    Rosenbrock, the whole solve), cfg 2 (BFGS at n = 4096: whole solve with the rank-2 update
    form, and per iteration with the reference's O(n^3) update extrapolated from n = 512), and
    the BFGS kernels' CPU counterparts (p = -D g at n = 8192, the rank-2 update at n = 4096)."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    O.use_fast()
    P = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1))
    A, xs, y = O.linres_data(m, n)
    o = O.Obj(O.LINRES, n, m, A, y)
    x = np.zeros(n)
    O.obj_eval_multi(o, x)                                                  # warm
    t_eval, s_eval = _median_time(lambda: O.obj_eval_multi(o, x), 5)
    # P concurrent evaluators (ctypes releases the GIL inside the C call): per evaluation, amortised
    objs = [O.Obj(O.LINRES, n, m, A, y) for _ in range(P)]
    with ThreadPoolExecutor(P) as ex:
        list(ex.map(lambda q: O.obj_eval_multi(objs[q], x), range(P)))   # warm
        t_ep, s_ep = _median_time(lambda: list(ex.map(lambda q: O.obj_eval_multi(objs[q % P], x), range(2 * P))), 3)
        t_eval_par = t_ep / (2 * P)
    J = np.ascontiguousarray(A)                    # any m x n data: cost is data-independent
    JT = np.ascontiguousarray(J.T)
    t_row, s_row = _median_time(lambda: O.matmul(JT[0:1], J), 3)
    with ThreadPoolExecutor(P) as ex:
        t_rp, s_rp = _median_time(lambda: list(ex.map(lambda q: O.matmul(JT[q:q + 1], J), range(P))), 3)
        t_row_par = t_rp / P
    nl = min(n, 1024)
    Al = JT[:nl, :nl] @ JT[:nl, :nl].T + np.eye(nl)
    t_lu_s, s_lu = _median_time(lambda: O.lusolve(Al, np.ones(nl)), 3)
    t_lu = t_lu_s * (n / nl) ** 3
    t_trip1 = t_eval * (n + 2) + t_row * n + t_lu
    t_tripP_sampled = t_eval_par * (n + 2) + t_row_par * n + t_lu
    # the whole trip timed twice (a one-shot timing of a multi-second threaded trip is exposed to
    # noise; it sets the baseline): value from their median, both samples in the line
    with ThreadPoolExecutor(P) as ex:
        s_trip = [cpu_lm_trip(O, objs, np.zeros(n), np.full(n, 1e-7), ex, P)[0] for _ in range(2)]
    t_trip_whole = float(np.median(s_trip))
    t_tripP = t_trip_whole
    # cfg 1: the whole BFGS solve on the 2-D Rosenbrock (the reference's CPU example)
    g1 = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_survey.json")))["bfgs_rosenbrock2_m12_1"]
    t_cfg1, _ = _median_time(lambda: O.bfgs_findmin(O.rosenbrock(2), g1["x0"], g1["params"]), 5)
    # cfg 2: BFGS n = 4096 (the bench's own parameters): whole solve with the rank-2 update form
    dd, bb = O.quadratic_data(4096)
    runs = []

    def cfg2():
        runs.append(O.bfgs_findmin(O.Obj(O.QUADRATIC, 4096, 0, dd, bb), np.zeros(4096), CFG2_P, rank2=True))
    t_cfg2, s_cfg2 = _median_time(cfg2, 3)
    it2 = max(runs[-1][1].iters, 1)
    # BFGS counterparts (single thread, the reference's sequential loops)
    rng = np.random.default_rng(0)
    hg = {}
    for nh in (4096, 8192, 16384):
        D = rng.standard_normal((nh, nh)); g = rng.standard_normal(nh)
        O.matvec(D, g)
        t, smp = _median_time(lambda: O.matvec(D, g), 5)
        hg[nh] = (t, smp)
        del D
    t_hg, s_hg = hg[8192]
    nu = 4096
    D = np.eye(nu) + 1e-3 * rng.standard_normal((nu, nu)); yv = rng.standard_normal(nu); sv = yv + 0.1
    t_r2, s_r2 = _median_time(lambda: O.update_hessian_inv_rank2(D, yv, sv), 3)
    del D
    n3 = 512
    D = np.eye(n3); y3 = rng.standard_normal(n3); s3 = y3 + 0.1
    t_n3, s_n3 = _median_time(lambda: O.update_hessian_inv(D, y3, s3), 3)
    scale3 = (4096 / n3) ** 3
    ref_iter = t_cfg2 / it2 - t_r2 + t_n3 * scale3
    model, ncpu = cpu_model()
    return {
        "value": 1.0 / t_tripP, "unit": "LM iters/sec", "cores": P, "kind": "port",
        "cpu_model": model, "host_logical_cpus": ncpu,
        "sample": (f"oracle (C restatement, gcc -O3 -march=x86-64-v3 -ffp-contract=off) at m={m}, n={n}: one whole LM "
                   f"trip timed end to end on {P} threads, median of 2 ({t_trip_whole:.1f} s: F(x), the FD Jacobian's columns "
                   f"round-robin over the threads, J^T J rows by the reference matrixMultiply split over the threads, "
                   f"-J^T F, luSolve, F(x + sigma)) on a {model}; the 1-thread trip extrapolated from medians of "
                   f"sampled legs: residual eval {t_eval*1e3:.1f} ms x{n + 2}, a J^T J row {t_row*1e3:.1f} ms x{n}, LU "
                   f"at n={nl} {t_lu_s:.2f} s scaled by (n/{nl})^3 = {t_trip1:.1f} s (the same legs on {P} threads: "
                   f"{t_tripP_sampled:.1f} s)"),
        "seconds_per_trip": t_tripP, "seconds_per_trip_whole_timed": t_trip_whole,
        "seconds_per_trip_whole_samples": s_trip,
        "whole_over_sampled_P_threads": t_trip_whole / t_tripP_sampled,
        "seconds_per_trip_sampled_P_threads": t_tripP_sampled,
        "seconds_per_trip_1_thread": t_trip1, "iters_per_s_1_thread": 1.0 / t_trip1,
        "threads": P,
        "samples_s": {"eval_1t": s_eval, "eval_Pt_2P_evals": s_ep, "jtj_row_1t": s_row, "jtj_rows_Pt_P_rows": s_rp,
                      "lu_n1024": s_lu},
        "cfg1_bfgs_rosenbrock2_solve_s": t_cfg1,
        "cfg2_bfgs_n4096": {"solve_s_rank2_update": t_cfg2, "solve_samples_s": s_cfg2, "iterations": it2,
                            "s_per_iteration_rank2_update": t_cfg2 / it2,
                            "s_per_iteration_reference_update_extrapolated": ref_iter,
                            "note": "reference O(n^3) updateHessianInv per iteration = its n=512 time x (4096/512)^3"},
        "bfgs_cpu_1_thread": {
            "hg_n8192_s": t_hg, "hg_n8192_GBps": 8.0 * 8192 * 8192 / t_hg / 1e9, "hg_samples_s": s_hg,
            "hg_GBps": {str(k): (8.0 * k * k + 16.0 * k) / v[0] / 1e9 for k, v in hg.items()},
            "hg_s": {str(k): v[0] for k, v in hg.items()},
            "rank2_update_n4096_s": t_r2, "rank2_samples_s": s_r2,
            "reference_update_n512_s": t_n3, "reference_update_n512_samples_s": s_n3,
            "reference_update_n4096_s_extrapolated": t_n3 * scale3,
            "reference_update_n4096_s_extrapolated_range": [min(s_n3) * scale3, max(s_n3) * scale3],
        },
    }


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, base_env, port):
    """The environment of each of the n ranks bench.py starts itself (one process per GPU, as
    torch.distributed.run would set it up on one node, rendezvous on 127.0.0.1)."""
    envs = []
    for r in range(n):
        e = dict(base_env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def launch_ranks(argv, n, timeout_s=None, python=None, script=None):
    """`bench.py --gpus N` without a launcher: start N child processes of this script, one per
    GPU, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set; relay rank 0's
    stdout (its one JSON line) and return non-zero if any rank fails.  This process never touches
    the GPU (it runs before `import torch`).  When one rank fails the others are stopped (they
    would wait in a collective for it)."""
    import subprocess
    py = python or sys.executable
    envs = rank_envs(n, os.environ, _free_port())
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen([py, script or os.path.abspath(__file__)] + list(argv), env=envs[r],
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = []
    import threading
    rd = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    rd.start()
    t0 = time.monotonic()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or (timeout_s is not None and time.monotonic() - t0 > timeout_s):
            rc = bad[0] if bad else 124
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        if all(c == 0 for c in codes):
            break
        time.sleep(0.05)
    rd.join(timeout=30)
    data = out0[0] if out0 else b""
    if data:
        sys.stdout.buffer.write(data)
        sys.stdout.flush()
    if rc:
        print(f"[bench] a rank exited with status {rc}; {n} ranks stopped", file=sys.stderr, flush=True)
    return rc


def main():
    args = _args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start the ranks here, before anything touches the GPU
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to measure a different "
              f"job size than the one asked for", file=sys.stderr, flush=True)
        sys.exit(2)
    # the ONE JSON line goes to the real stdout; everything else written to fd 1 -- the drop-in
    # solvers' console messages (BFGS_Bnd prints one per boundary recursion, as the reference
    # does), library logs -- goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
    from parallelnonlinearoptimizationlibrary_amd.dist import env_rank_world, init_rccl

    rank, world, local = env_rank_world()
    if args.host_comm:   # ranks may share the box's GPUs in the rehearsal
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    os.environ["PNOL_DEVICE"] = str(local)
    if world > 1 and args.host_comm:
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    elif world > 1:
        dist.init_process_group("nccl", init_method="env://", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))

    m, n = args.residuals, args.params
    # LevMarqMPI's Jacobian decomposition (csrc/kernels/fd.hip launch_lm_jacobian): columns mode,
    # the reference's (cost-balanced FD column tiles per rank, each tile's m-slices exchanged
    # while the next computes), is the headline; rows mode (every FD column on the rank's own
    # m-slices, no J exchange; linear residuals only) is timed beside it at N > 1 as an extra
    os.environ.pop("PNOL_LM_FD", None)
    rows_mode = False
    ctx = Context(local)
    # the C++ drop-in classes run on the process default context: bind its timers
    dctx = C.c_void_p()
    L.check(L.lib().pnol_default_ctx(C.byref(dctx)), "pnol_default_ctx")
    host_comm = None
    comm_backend = "none"
    if world > 1 and args.host_comm:
        from parallelnonlinearoptimizationlibrary_amd.dist import HostComm
        host_comm = HostComm(rank, world)
        comm_backend = "host-gloo"
    elif world > 1:
        class _Ctx:  # RCCL communicator on the solver's context
            h = dctx
        init_rccl(_Ctx, rank, world)
        comm_backend = "rccl"
        # the RCCL transport first runs here: a small LevMarqMPI must reproduce the one-process
        # LevMarq bit for bit, or the measurement falls back to the host communicator over a
        # gloo group (labelled as such in "comm")
        from parallelnonlinearoptimizationlibrary_amd.dist import HostComm, rccl_selfcheck
        ok, why = rccl_selfcheck(ctx, world)
        if rank == 0:
            print(f"[bench] RCCL self-check: {why}", file=sys.stderr, flush=True)
        if not ok:
            L.lib().pnol_comm_finalize()
            host_comm = HostComm(rank, world, group=dist.new_group(backend="gloo"))
            comm_backend = f"host-gloo (RCCL self-check failed: {why[:160]})"

    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)   # A, y generated in HBM
    x0 = np.zeros(n)
    which = 1 if world > 1 else 0

    trips = [0, 0]

    def run(iters):
        X = x0.copy()
        p = np.array([0.001, 10.0, 1e-7, float(iters), 0.0, -1.0])  # xMinDiff 0: every trip runs
        F0, FO = np.zeros(m), np.zeros(m)
        res = L.Result()
        steps = (C.c_int * 2)()
        dp = C.POINTER(C.c_double)
        L.check(L.lib().pnol_run_levmarq_ex(which, obj.h, 0, p.ctypes.data_as(dp), X.ctypes.data_as(dp), n,
                                            F0.ctypes.data_as(dp), FO.ctypes.data_as(dp), m, C.byref(res), steps),
                "pnol_run_levmarq")
        trips[:] = [steps[0], steps[1]]
        return X

    # warmup with every per-kernel timer on: the full breakdown (untimed); the timed region
    # keeps only the timers of the kernels priced below (each timer adds two event records
    # between launches, ~1.5% of a trip with all of them on)
    names = ("fd_jtj", "fd_jacobian", "fd_ckpt", "linres_eval", "syrk", "syrk_rows", "syrk_reduce", "jtr", "solve",
             "allgather", "exchange_J", "exchange_J_busy", "exchange_A", "exchange_F")

    def timed_lm():
        """W warmup trips (all timers: the breakdown), then K timed trips between barriers +
        synchronize, max over ranks; per-step kernel times of this rank and max over ranks."""
        L.check(L.lib().pnol_ctx_enable_timers(dctx, 0 if args.no_timers else 1), "timers")
        L.check(L.lib().pnol_ctx_reset_timers(dctx), "timers")
        run(args.warmup)
        torch.cuda.synchronize()
        bd = {k: _timer(L, dctx, k) for k in names}
        bd = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in bd.items()}
        L.check(L.lib().pnol_ctx_enable_timers(dctx, 0 if args.no_timers else 2), "timers")
        L.check(L.lib().pnol_ctx_reset_timers(dctx), "timers")
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Xr = run(args.steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=_red_dev())
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        timers = {k: _timer(L, dctx, k) for k in names}
        # per-step kernel times, max over ranks (the slowest rank sets the pace)
        pl = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in timers.items()}
        # the checkpoint pass runs only when no slot holds x's checkpoints (the first trip; the
        # trial-point evaluation and the two slots cover accepted and rejected steps): per trip
        pl["fd_ckpt_per_step"] = timers["fd_ckpt"][0] / max(args.steps, 1)
        if world > 1:
            keys = sorted(pl)
            tv = torch.tensor([pl[k] for k in keys], dtype=torch.float64, device=_red_dev())
            dist.all_reduce(tv, op=dist.ReduceOp.MAX)
            pm = dict(zip(keys, tv.tolist()))
        else:
            pm = dict(pl)
        L.check(L.lib().pnol_ctx_enable_timers(dctx, 0), "timers")
        return el, Xr, bd, pl, pm, list(trips)

    elapsed, X, breakdown, per_local, per_max, trips_main = timed_lm()
    err = float(np.max(np.abs(X - obj.xstar)) / np.max(np.abs(obj.xstar)))
    rows_extra = None
    if world > 1:
        # rows mode beside the headline (labelled extra; linear residuals only): every rank the
        # same environment, LevMarqMPI reads it once per solve and checks that the ranks agree
        os.environ["PNOL_LM_FD"] = "rows"
        el_r, X_r, _, pl_r, pm_r, tr_r = timed_lm()
        os.environ.pop("PNOL_LM_FD", None)
        rows_extra = {
            "value": args.steps / el_r, "unit": "iters/s", "ms_per_step": el_r / args.steps * 1e3,
            "fd_jacobian_ms_max_over_ranks": pm_r["fd_jacobian"] + pm_r["fd_ckpt_per_step"],
            "exchange_F_ms_max_over_ranks": pm_r["exchange_F"],
            "kernel_ms_per_step_max_over_ranks": pm_r, "trips_accepted": tr_r[0], "trips_rejected": tr_r[1],
            "X_bitwise_equal_columns_mode": bool(np.array_equal(X_r, X)),
            "note": ("LevMarqMPI rows mode (PNOL_LM_FD=rows): every FD column on the rank's own m-slices of "
                     "residual rows, no J exchange; valid for the linear residual only (not the reference's "
                     "decomposition) -- an extra, not the headline"),
        }
    trips[:] = trips_main

    hg_sharded = None
    if world > 1 and not args.no_hg:
        hg_sharded = bench_hg_sharded(dctx, HG_N, world, rank)
    hg = None
    if rank == 0 and not args.no_hg:
        hg = bench_hg(ctx, HG_N)
        hg4096 = bench_hg(ctx, 4096)
        hg16384 = bench_hg(ctx, 16384)      # cfg 5: D = 2.15 GB
    bfgs2 = bnd5 = None
    if rank == 0 and not args.no_bfgs:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        bfgs2 = bench_bfgs_solve(ctx, 0, 4096, 1.0, CFG2_P)
        n5 = 16384
        bnd5 = bench_bfgs_solve(ctx, 2, n5, 4.0, CFG5_P, bounds=(np.full(n5, -0.5), np.full(n5, 0.5)))
    if rank == 0:
        per = per_local
        syrk_ms = per["syrk"]
        # J^T J flops of the SYRK this rank ran: all m rows on one GPU; at N > 1 (LevMarqMPI on
        # m-slices) only the rows of its own slices (unique entries of the symmetric result)
        if world > 1:
            mS = C.c_int()
            L.check(L.lib().pnol_lm_sliced_layout(m, n, C.byref(mS), None), "pnol_lm_sliced_layout")
            s0, s1 = rank * L.LM_SLICES // world, (rank + 1) * L.LM_SLICES // world
            jtj_rows = max(0, min(m, s1 * mS.value) - s0 * mS.value)
        else:
            jtj_rows = m
        jtj_flop = float(jtj_rows) * n * (n + 1)
        from parallelnonlinearoptimizationlibrary_amd import fd_tiles
        if world > 1 and rows_mode:
            my_tiles = fd_tiles(n, 1, 0)                     # rows mode: every FD column ...
            fd_rows = jtj_rows                               # ... on this rank's own m-slices
        else:
            my_tiles = fd_tiles(n, world, rank)              # this rank's cost-balanced FD tiles, all rows
            fd_rows = m
        my_cols = sum(c for _, c in my_tiles)
        fd_flop_nominal = 2.0 * fd_rows * n * my_cols        # full-length chains for this rank's points
        fd_flop = fd_flop_executed(fd_rows, n, my_tiles)     # prefix-shared chains actually run
        pmc = pmc_traffic()
        one_gpu = world == 1
        roofline = {
            "kernel": (("k_syrk_red<2> (J^T J split-K partials on fp64 MFMA v_mfma_f64_16x16x4_f64, 8 waves per "
                        "128 x 128 tile, with their reduce into the Cholesky's matrix in the same launch)"
                        if os.environ.get("PNOL_LM_REDUCE", "tail") == "tail" else
                        "k_syrk_tile<0,128,8 waves> (J^T J, fp64 MFMA v_mfma_f64_16x16x4_f64)") if one_gpu else
                       "k_syrk_tile<4,64> on this rank's m-slices (J^T J share, fp64 MFMA v_mfma_f64_16x16x4_f64)"),
            "bound": "mfma", "achieved": jtj_flop / (syrk_ms * 1e-3) / 1e12 if syrk_ms else None,
            "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "flop_per_launch": jtj_flop, "rows": jtj_rows,
            # one GPU: the PMC passes of this bench; N > 1: the PMC passes of the sliced kernel over
            # all 8 m-slices in one process (tools/syrk_sliced_probe.py, the metric's m and n), times
            # this rank's rows / m; other sizes have no committed pass (null)
            "traffic": ((pmc.get("k_syrk_red", {}) or pmc.get("k_syrk_tile<0, 128>", {})).get("traffic_bytes_per_launch")
                        if one_gpu else
                        (pmc["k_syrk_tile<4, 64>"]["traffic_bytes_per_launch"] * jtj_rows / m
                         if (m, n) == (M_RES, N_PAR) and "traffic_bytes_per_launch" in pmc.get("k_syrk_tile<4, 64>", {})
                         else None)),
            "mfma_busy_pmc": next((v.get("mfma_busy_frac") for k, v in pmc_valu("syrk_mfma").items()
                                   if "k_syrk_red" in k or "k_syrk_tile" in k), None) if one_gpu else None,
        }
        roofline["frac"] = roofline["achieved"] / FP64_PEAK_TFLOPS if roofline["achieved"] else None
        fd_ms = per["fd_jacobian"]
        rooflines = {
            "fd_jacobian": {"kernel": "k_linres_fdP<true> (batched FD evaluation, row per lane, fp64 VALU fma with "
                                      "the x_k operand in SGPRs, prefix-shared chains)",
                            "bound": "valu_fp64", "ms": fd_ms,
                            "achieved": fd_flop / (fd_ms * 1e-3) / 1e12 if fd_ms else None,
                            "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "flop_executed": fd_flop,
                            "flop_minimal": fd_flop_minimal(fd_rows, my_tiles, n), "rows": fd_rows,
                            "flop_nominal_full_chains": fd_flop_nominal,
                            "valu_busy_pmc": next((v.get("valu_busy_frac") for k, v in pmc_valu().items()
                                                   if "k_linres_fdP" in k), None),
                            "ckpt_ms_per_call": per["fd_ckpt"], "ckpt_ms_per_step": per["fd_ckpt_per_step"]},
            "jtj": dict(roofline, ms=syrk_ms),
        }
        if hg:
            rooflines["hg"] = {"kernel": "k_gemv_neg_wg<2,NT> (p = -D g, non-temporal 16-B loads)", "bound": "hbm",
                               "achieved": hg["hg_GBps"],
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hg["hg_frac_of_hbm"],
                               "algorithmic_bytes": 8.0 * HG_N * HG_N + 16.0 * HG_N,
                               # the launch at this n: (n / 2) workgroups of 256 lanes (launch_gemv_neg);
                               # the bench also runs H.g at n = 4096 and 16384, so key by grid
                               "traffic": pmc.get(f"k_gemv_neg_wg<2, true>@grid{HG_N // 2 * 256}",
                                                  {}).get("traffic_bytes_per_launch"),
                               "n": HG_N}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(m, n)
        ms_per_step = elapsed / args.steps * 1e3
        if world > 1:
            transport = ("host communicator over gloo: one-GPU rehearsal" if args.host_comm else
                         "RCCL p2p" if comm_backend == "rccl" else comm_backend)
            workload = (f"LevenbergMarquardtMPI m={m} n={n}, FD columns in cost-balanced tiles over {world} GPUs, "
                        f"each tile's J rows exchanged by m-slice behind its launch ({transport}), "
                        f"J^T J + J^T F by m-slice + reduce-scatter/allgather")
        else:
            workload = f"LevenbergMarquardt m={m} n={n}, FD columns on 1 GPU"
        line = {
            "metric": f"LM iters/sec at m={m},n={n}",
            "value": args.steps / elapsed,
            "unit": "iters/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 seed 0x5EED2018, r(x)=Ax-y generated in HBM)",
            "config": {"workload": workload, "m": m, "n": n, "parallelism": f"fd-columns+m-slices x{world}" if world > 1 else "single"},
            "roofline": roofline,
            "rooflines": rooflines,
            "kernel_ms_per_step": per,   # timed region: the priced kernels only
            "kernel_ms_per_call_warmup_breakdown": breakdown,   # every timer, warmup trips (untimed)
            "kernel_ms_per_step_max_over_ranks": per_max,
            # the north star's strong-scaling quantity: the sharded FD Jacobian + its exchange
            # (columns mode: the m-slice point-to-point exchange left after the FD launches end --
            # exchange_J, the exposed part; exchange_J_busy is its whole span on the comm stream)
            "fd_jacobian_ms_max_over_ranks": per_max["fd_jacobian"] + per_max["fd_ckpt_per_step"] + (
                per_max["exchange_J"] if per_max["exchange_J_busy"] > 0 else per_max["allgather"]),
            "exchange_J_ms_max_over_ranks": {"exposed": per_max["exchange_J"], "busy": per_max["exchange_J_busy"]}
            if world > 1 else None,
            "lm_fd_mode": ("rows" if rows_mode else "columns") if world > 1 else "single",
            "rows_mode_extra": rows_extra,
            "converged_rel_err_vs_xstar": err,
            # the timed trips' outcomes: every trip recomputes J, J^T J and the solve either way
            "trips_accepted": trips[0], "trips_rejected": trips[1],
            "bfgs_hg": hg, "bfgs_hg_n4096": hg4096 if hg else None, "bfgs_hg_n16384": hg16384 if hg else None,
            "bfgs_hg_row_sharded": hg_sharded,
            "bfgs_cfg2_solve": bfgs2, "bfgs_bnd_cfg5_solve": bnd5,
            "comm": {"backend": comm_backend, "ranks": world},
            "cpu_baseline": cpu,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
