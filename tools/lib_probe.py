"""Library yardsticks for the LM trip's dense kernels on one MI355X (fp64):
J^T J as torch.mm (rocBLAS / hipBLASLt dgemm) on the cfg-3 shape, and the damped solve as
torch.linalg.cholesky + cholesky_solve (rocSOLVER) at n = 2048.  Not product code: it tells
how the hand-written SYRK and tile Cholesky compare with the vendor libraries."""
import json
import sys

import torch


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    m, n = 16384, 2048
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    JT = torch.randn(n, m, dtype=torch.float64, device=dev, generator=g)
    out = {}
    ms = timeit(lambda: torch.mm(JT, JT.t()))
    out["dgemm_JT_JTt_ms"] = ms
    out["dgemm_TFs_full"] = 2.0 * n * n * m / ms / 1e9
    out["dgemm_TFs_syrk_equiv"] = m * n * (n + 1) / ms / 1e9
    A = torch.mm(JT, JT.t())
    A.diagonal().mul_(1.001)
    b = torch.randn(n, 1, dtype=torch.float64, device=dev, generator=g)

    def chol():
        L = torch.linalg.cholesky(A)
        return torch.cholesky_solve(b, L)

    out["potrf_potrs_ms"] = timeit(chol, reps=10)
    out["potrf_ms"] = timeit(lambda: torch.linalg.cholesky(A), reps=10)
    out["lu_solve_ms"] = timeit(lambda: torch.linalg.solve(A, b), reps=10)
    print(json.dumps(out))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
