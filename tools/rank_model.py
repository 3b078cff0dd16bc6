"""Per-rank LM step model for LevMarqMPI at N = 1/2/4/8 GPUs (cfg 4), measured on ONE
MI355X: each piece of rank r's trip timed on its own, then combined with the transfer volumes of
the exchange steps at a stated xGMI rate (the 8-GPU run itself is the driver's).

  FD_r(P)      rank r's cost-balanced FD column tiles (pnol_fd_tiles snake order) for all m rows,
               launched as the columns mode launches them: one launch per tile, cheapest first,
               the last tile cut into S column groups (PNOL_LM_SUBPHASES); timed as the span of
               the launch sequence on the stream (launch gaps included), max over r, for S = 1, 2, 4
               and for the single tile-list launch (no phasing)
  exposed(P,S) the last phase's transfer, which nothing hides: each rank sends the last column
               group's rows of every other rank's m-slices, over one link per peer in parallel:
               cols_last * (m / P) * 8 bytes / LINK_GBPS + PHASE_LATENCY_US
  fd_jacobian_ms_max_over_ranks(P, S) = max_r FD_r(P, S) + exposed(P, S) -- the north star's
               strong-scaling quantity (>= 6x at P = 8: <= T1 / 6)
  SYRK(P)      J^T J over m / P residual rows (a rank's m-slices), with the reduce
  solve        the persistent tile Cholesky + backward solve at n (replicated on every rank)
  eval         F(x + sigma) (columns mode: all rows on every rank)
  exchanges    + the J^T J node reduce-scatter and the tile allgather (~8 n^2 bytes over the ranks)
  device-initiated (a design, NOT built): the FD kernel's epilogue stores each m-slice row block of
               its tiles straight into the slice owner's buffer over xGMI (IPC-mapped peer memory)
               and bumps a completion word there, so the transfer runs under the FD launch itself:
               max_r FD_r(P) (one tile-list launch) + max(0, per-link bytes / LINK_GBPS - FD_r(P))
               + FLAG_LATENCY_US -- assuming the remote stores do not slow the VALU-bound FD

    python tools/rank_model.py [--out profiles/r06_rank_model.json]
    python tools/rank_model.py --derive profiles/r06_rank_model.json   (recompute the modelled fields
                                                                       of a measured file, no GPU)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINK_GBPS = 64.0          # assumed effective one-direction rate of one xGMI peer link (GB/s)
PHASE_LATENCY_US = 10.0   # assumed fixed cost of one grouped RCCL send/recv phase (launch + handshake)
FLAG_LATENCY_US = 5.0     # assumed cost of the device-initiated design's cross-GPU completion word


def device_initiated(d, P, m, n, t1):
    """the device-initiated exchange design's prediction from a rank's measured one-launch FD"""
    fd = d["fd_ms_max_one_launch"]
    cols = -(-n // P)                       # a rank's FD columns (cost-balanced tiles, ~n / P)
    rows_out = m - -(-m // P)               # the rows of its columns that other ranks hold
    per_link = cols * rows_out * 8.0 / (P - 1)
    link_ms = per_link / (LINK_GBPS * 1e9) * 1e3
    total = fd + max(0.0, link_ms - fd) + FLAG_LATENCY_US / 1e3
    return {"fd_ms_max_one_launch": fd, "bytes_per_link": per_link, "link_ms": link_ms,
            "flag_latency_us_assumed": FLAG_LATENCY_US, "fd_jacobian_ms_max_over_ranks": total,
            "speedup_vs_one_gpu": t1 / total, "built": False}


def phase_tiles(tiles, sub):
    """the columns mode's launch order (fd.hip lm_phase_tiles): cheapest first, last tile cut in sub"""
    t = sorted(tiles, key=lambda x: -x[0])
    if sub < 2 or not t:
        return t
    s0, c = t.pop()
    w = max(16, (c // sub + 15) // 16 * 16)
    for a in range(0, c, w):
        t.append((s0 + a, min(w, c - a)))
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="")
    ap.add_argument("--derive", default="", help="recompute the modelled fields of a measured file")
    args = ap.parse_args()
    if args.derive:
        out = json.load(open(args.derive))
        for P, d in out["per_P"].items():
            if int(P) > 1:
                d["fd_jacobian_model_device_initiated"] = device_initiated(d, int(P), out["m"], out["n"],
                                                                           out["fd_ms_one_gpu"])
        out["flag_latency_us_assumed"] = FLAG_LATENCY_US
        with open(args.derive, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps({P: d.get("fd_jacobian_model_device_initiated") for P, d in out["per_P"].items()}, indent=1))
        return
    import numpy as np
    import torch
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective
    m, n = args.m, args.n
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    x = ctx.tensor(np.linspace(-0.5, 0.5, n))
    h = ctx.tensor(np.full(n, 1e-7))
    JT = ctx.empty(n, m)

    def timed(fn):
        fn()
        ctx.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    F0 = obj.eval_ckpt(x)   # F0 and the prefix checkpoints of x, reused by every FD call (the trip's compute_f0 = 3)

    def fd_span(seq):
        """GPU span of one launch per entry of seq (each a tile list), back to back: the stream is
        held by a spin kernel while the host enqueues the whole sequence, so host call overhead
        (Python here, C++ in the library's phased loop) does not open gaps between the launches"""
        ts = []
        for it in range(args.reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(4_000_000)
            a.record()
            for tl in seq:
                obj.fd_jacobian_tiles(x, h, tl, JT, F0=F0, compute_f0=3)
            b.record()
            b.synchronize()
            if it:
                ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    out = {"m": m, "n": n, "link_GBps_assumed": LINK_GBPS, "phase_latency_us_assumed": PHASE_LATENCY_US,
           "flag_latency_us_assumed": FLAG_LATENCY_US, "reps": args.reps, "per_P": {}}
    full = L.fd_tiles(n, 1, 0)
    t1 = fd_span([full])
    out["fd_ms_one_gpu"] = t1
    subs = (1, 2, 4)
    for P in (1, 2, 4, 8):
        d = {"fd_ms_one_launch_per_rank": [], "fd_ms_phased_per_rank": {str(s): [] for s in subs}}
        for r in range(P):
            tiles = L.fd_tiles(n, P, r)
            d["fd_ms_one_launch_per_rank"].append(fd_span([tiles]) if tiles else 0.0)
            if P > 1:
                for s in subs:
                    seq = [[t] for t in phase_tiles(tiles, s)]
                    d["fd_ms_phased_per_rank"][str(s)].append(fd_span(seq) if seq else 0.0)
        d["fd_ms_max_one_launch"] = max(d["fd_ms_one_launch_per_rank"])
        if P > 1:
            mS = -(-m // P)
            fdj = {}
            for s in subs:
                last_cols = phase_tiles(L.fd_tiles(n, P, 0), s)[-1][1]
                exposed = last_cols * mS * 8.0 / (LINK_GBPS * 1e9) * 1e3 + PHASE_LATENCY_US / 1e3
                fmax = max(d["fd_ms_phased_per_rank"][str(s)])
                fdj[str(s)] = {"fd_ms_max": fmax, "last_phase_cols": last_cols, "exposed_ms": exposed,
                               "fd_jacobian_ms_max_over_ranks": fmax + exposed,
                               "speedup_vs_one_gpu": t1 / (fmax + exposed),
                               "launch_overhead_vs_one_launch": fmax / d["fd_ms_max_one_launch"] - 1.0}
            d["fd_jacobian_model"] = fdj
            d["fd_jacobian_model_device_initiated"] = device_initiated(d, P, m, n, t1)
        mp = m // P
        JTs = torch.randn(n, mp, dtype=torch.float64, device=f"cuda:{ctx.device}")
        d["syrk_reduce_ms"] = timed(lambda: ctx.jtj(JTs, 0.01))
        del JTs
        if P == 1:
            d.pop("fd_ms_phased_per_rank")
        out["per_P"][P] = d
    # the replicated pieces at n: solve (Cholesky + backward), F(x + sigma)
    rng = np.random.default_rng(0)
    B = rng.standard_normal((n, n))
    A = ctx.tensor(B @ B.T / n + np.eye(n))
    rhs = ctx.tensor(rng.standard_normal(n))
    t_solve = timed(lambda: ctx.solve_step(A, rhs, x))
    t_eval = timed(lambda: obj.eval(x))
    out["solve_ms"] = t_solve
    out["eval_ms"] = t_eval
    S = 1   # kLmSubphases, the library default
    for P, d in out["per_P"].items():
        if P == 1:
            fdj, exch = d["fd_ms_max_one_launch"], 0.0
        else:
            fdj = d["fd_jacobian_model"][str(S)]["fd_jacobian_ms_max_over_ranks"]
            # the node reduce-scatter + allgather of ~8 n^2 bytes split over P ranks, P-1 links at once
            tiles_bytes = 8.0 * n * n
            exch = (tiles_bytes / P / LINK_GBPS / 1e6) * 2
        d["exchange_A_ms_model"] = exch
        d["step_ms_model"] = fdj + d["syrk_reduce_ms"] + exch + t_solve + t_eval
        d["lm_iters_per_s_model"] = 1e3 / d["step_ms_model"]
    s1 = out["per_P"][1]["step_ms_model"]
    for P, d in out["per_P"].items():
        d["speedup_model_vs_1"] = s1 / d["step_ms_model"]
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
