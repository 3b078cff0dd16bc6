"""Worker for tests/test_gpu_mpi.py: one rank of LevMarqMPI on the (shared) GPU with the
host communicator backend (torch.distributed gloo allgather).  Writes its results to
<out>/rank<r>.npz.  Started as a child process by the test (never exec'd in place)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, m, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    what = sys.argv[4] if len(sys.argv) > 4 else ""
    lm_only = what in ("lm", "lmonly")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_bfgs, run_levmarq
    from parallelnonlinearoptimizationlibrary_amd.dist import HostComm
    comm = HostComm(rank, world)
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X, F0, FO, res = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=1)
    if what == "lmonly":   # the LevMarqMPI solve alone (full-size cfg 4), with the mode it ran in
        dctx = C.c_void_p()
        L.check(L.lib().pnol_default_ctx(C.byref(dctx)), "pnol_default_ctx")
        mode = C.c_int()
        L.check(L.lib().pnol_lm_fd_mode(dctx, C.byref(mode)), "pnol_lm_fd_mode")
        np.savez(os.path.join(out, f"rank{rank}.npz"), X=X, F0=F0, FO=FO, mode=np.array([mode.value]))
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    # the sharded J^T J kernel on its own, on a random JT
    rng = np.random.default_rng(11)
    JT = ctx.tensor(rng.standard_normal((n, m)))
    A = ctx.empty(n, n)
    diag = ctx.empty(n)
    L.check(L.lib().pnol_jtj_mpi_d(ctx.h, JT.data_ptr(), m, m, n, 0.25, A.data_ptr(), n, diag.data_ptr()),
            "pnol_jtj_mpi_d")
    ctx.synchronize()
    # the m-sliced normal equations (pnol_lm_normal_mpi_d) on the same JT and a random F:
    # every rank uploads the whole sliced layout and reads only its own slices
    from parallelnonlinearoptimizationlibrary_amd.device import lm_sliced_layout, to_sliced
    mS, _ = lm_sliced_layout(m, n)
    JTs = ctx.tensor(to_sliced(JT.cpu().numpy(), mS).reshape(-1))
    Fr = ctx.tensor(np.random.default_rng(12).standard_normal(m))
    As, rs, ds = ctx.lm_normal_mpi(JTs, m, n, 0.25, Fr, want_diag=True)
    ctx.synchronize()
    res = dict(X=X, F0=F0, FO=FO, A=A.cpu().numpy(), diag=diag.cpu().numpy(), As=As.cpu().numpy(),
               rs=rs.cpu().numpy(), ds=ds.cpu().numpy())
    if lm_only:
        np.savez(os.path.join(out, f"rank{rank}.npz"), **res)
        comm.close()
        dist.barrier()
        dist.destroy_process_group()
        return
    # BFGSBnd_MPI, testBFGSBnd_MPI start (Examples.cpp:90-120): Npool = world, pool entries
    # round-robin over the ranks, FD gradients sharded
    nb = 10
    x0 = np.full(nb, 3.0); x0[0] = -0.5
    lb = np.full(nb, -5.0); lb[0] = -1.0
    Pb = [1e-4, 0.1, 1e-16, 4, 1, 1000, 1e-7, 1e-3, 200, 1e-5, 1e-5, 1e-5, 0, 0]
    Xb, resb = run_bfgs(DeviceObjective(ctx, L.OBJ_ROSENBROCK, nb), x0, Pb, which=3, lb=lb, ub=np.full(nb, 5.0))
    # BFGS_Bnd_MPI_SW, testBFGSBndMPISW (Examples.cpp:12-45): pools of world + 1 / world + 2
    Psw = [1e-4, 0.8, 1e-6, 1, 1e-10, 2, 50, 1e-5, 1e-6, 1e-3, 200, 1e-5, 1e-5, 0, -1]
    Xs, ress = run_bfgs(DeviceObjective(ctx, L.OBJ_ROSENBROCK, 3), [-1.0, 2.0, 2.0], Psw, which=4, lb=[-1.0] * 3,
                        ub=[5.0] * 3)
    # BFGS D row-sharded: this rank's rows through the collective pass / H.g
    nD = 700
    rng = np.random.default_rng(3)
    Dfull = rng.standard_normal((nD, nD))
    g, yv, sv, av, bv = (rng.standard_normal(nD) for _ in range(5))
    rb, rc = C.c_int(), C.c_int()
    L.check(L.lib().pnol_bfgs_rows(nD, world, rank, C.byref(rb), C.byref(rc)), "bfgs_rows")
    rb, rc = rb.value, rc.value
    Dsh = ctx.tensor(Dfull[rb:rb + rc] if rc > 0 else np.zeros((1, nD)))
    dg, dy, ds, da, db = (ctx.tensor(a) for a in (g, yv, sv, av, bv))
    p = ctx.empty(nD)
    L.check(L.lib().pnol_hg_mpi_d(ctx.h, Dsh.data_ptr(), nD, dg.data_ptr(), p.data_ptr(), nD), "hg_mpi")
    u, w, v = ctx.empty(nD), ctx.empty(nD), ctx.empty(nD)
    L.check(L.lib().pnol_bfgs_pass_mpi_d(ctx.h, Dsh.data_ptr(), nD, nD, ds.data_ptr(), da.data_ptr(), db.data_ptr(), 1,
                                         dy.data_ptr(), dg.data_ptr(), u.data_ptr(), w.data_ptr(), v.data_ptr()),
            "pass_mpi")
    ctx.synchronize()
    # the boundary recursion's free-free block of the row-sharded D (pnol_gather_submatrix_mpi_d):
    # kept rows to their new owners, device to device
    keep = np.sort(np.random.default_rng(4).choice(nD, 411, replace=False)).astype(np.int32)
    Dsh2 = ctx.tensor(Dfull[rb:rb + rc] if rc > 0 else np.zeros((1, nD)))
    sb, sc = C.c_int(), C.c_int()
    L.check(L.lib().pnol_bfgs_rows(len(keep), world, rank, C.byref(sb), C.byref(sc)), "bfgs_rows")
    sb, sc = sb.value, sc.value
    Dsub = ctx.empty(max(sc, 1), len(keep))
    L.check(L.lib().pnol_gather_submatrix_mpi_d(ctx.h, Dsh2.data_ptr(), nD, nD,
                                                keep.ctypes.data_as(C.POINTER(C.c_int)), len(keep),
                                                Dsub.data_ptr(), len(keep)), "gather_submatrix_mpi")
    ctx.synchronize()
    # BFGS_MPI, fast mode (fused passes) on the synthetic quadratic with D row-sharded; pool 4
    nq = 300
    Pq = [1e-4, 0.9, 4, 1, 1000, 1e-6, 1e-3, 40, 1e-9, 1e-6, 0, 0, 4, 1, 2]
    Xq, resq = run_bfgs(DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, nq), np.zeros(nq), Pq, which=1)
    # GeneticAlgorithmMPI: the population dealt round-robin over the ranks, one device batch each
    from parallelnonlinearoptimizationlibrary_amd.device import run_ga
    Pga = [40, 200, 0.1, 0.3, 0.2, 0.5, 0.01, 0.5, 20, 0]
    Xga, resga = run_ga(DeviceObjective(ctx, L.OBJ_ROSENBROCK, 4), np.full(4, -1.0), np.full(4, -2.0),
                        np.full(4, 2.0), Pga, 12345, which=1)
    # BFGSBnd_MPI in fast mode at n = 600 (D row-sharded over the ranks; active bounds, so the
    # reduced problems start from the sharded free-free block)
    Pf = [1e-4, 0.1, 1e-16, 4, 1, 200, 1e-6, 1e-3, 100, 1e-9, 1e-6, 1e-9, 0, 0, 4]
    Xf, resf = run_bfgs(DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, 600, 0, bscale=4.0), np.zeros(600), Pf,
                        which=3, lb=np.full(600, -0.25), ub=np.full(600, 0.25))
    np.savez(os.path.join(out, f"rank{rank}.npz"), **res, Xb=Xb, Xf=Xf, ff=np.array([resf.fopt]), Xga=Xga,
             ga=np.array([resga.f0, resga.fopt, resga.iters, resga.evals]),
             fb=np.array([resb.fopt]), Xs=Xs, fs=np.array([ress.fopt]), hg=p.cpu().numpy(), u=u.cpu().numpy(),
             w=w.cpu().numpy(), v=v.cpu().numpy(), Drows=Dsh.cpu().numpy()[:rc], rows=np.array([rb, rc]), Xq=Xq,
             fq=np.array([resq.fopt]), Dsub=Dsub.cpu().numpy()[:sc], subrows=np.array([sb, sc]), keep=keep)
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
