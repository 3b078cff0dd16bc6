"""RCCL rehearsal on one GPU: WORLD_SIZE processes (torch.distributed.run) share device 0 and
bind the library's RCCL communicator (gloo only carries the unique id).  Runs LevMarqMPI (the
m-sliced path: point-to-point slice exchange, tree-order reduce-scatter, in-place allgather)
and the tile-split J^T J, and checks them bitwise against the single-process LevMarq / pnol_jtj_d.
RCCL may refuse two ranks on one device; the probe then reports that and exits 3.
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_probe.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    from parallelnonlinearoptimizationlibrary_amd.dist import env_rank_world, init_rccl
    rank, world, _ = env_rank_world()
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dctx = C.c_void_p()
    L.check(L.lib().pnol_default_ctx(C.byref(dctx)), "default ctx")

    class _Ctx:
        h = dctx
    try:
        init_rccl(_Ctx, rank, world)
    except Exception as e:   # noqa: BLE001
        print(f"rank {rank}: RCCL init refused: {e}", flush=True)
        sys.exit(3)
    ctx = Context(0)
    m, n = 3000, 600
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    Xm, *_ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 6, 0.0, -1), which=1)
    rng = np.random.default_rng(5)
    JT = ctx.tensor(rng.standard_normal((n, m)))
    Am = ctx.empty(n, n)
    L.check(L.lib().pnol_jtj_mpi_d(dctx, JT.data_ptr(), m, m, n, 0.25, Am.data_ptr(), n, None), "jtj_mpi")
    torch.cuda.synchronize()
    ok = True
    if rank == 0:
        L.lib().pnol_comm_finalize()
        X1, *_ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 6, 0.0, -1), which=0)
        A1 = ctx.jtj(JT, 0.25)
        ok = np.array_equal(Xm, X1) and torch.equal(Am, A1)
        print(f"LevMarqMPI over RCCL x{world}: X bitwise {np.array_equal(Xm, X1)}, "
              f"tile-split J^T J bitwise {torch.equal(Am, A1)}, |X - x*| {np.max(np.abs(Xm - obj.xstar)):.3g}",
              flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
