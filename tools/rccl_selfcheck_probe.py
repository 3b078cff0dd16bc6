"""The bench's N > 1 RCCL self-check (dist.rccl_selfcheck) on whatever ranks are launched: with
one rank on a one-GPU box it runs the RCCL communicator of size 1 (ncclCommInitRank, the
LevMarqMPI path's calls with P = 1) and the bitwise comparison; RCCL refuses two ranks on one
device, so larger worlds need one GPU per rank.
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/rccl_selfcheck_probe.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context
    from parallelnonlinearoptimizationlibrary_amd.dist import env_rank_world, init_rccl, rccl_selfcheck
    rank, world, local = env_rank_world()
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", init_method="env://", rank=rank, world_size=world,
                            device_id=torch.device("cuda", local))
    dctx = C.c_void_p()
    L.check(L.lib().pnol_default_ctx(C.byref(dctx)), "default ctx")

    class _Ctx:
        h = dctx
    init_rccl(_Ctx, rank, world)
    ctx = Context(local)
    ok, why = rccl_selfcheck(ctx, world)
    print(f"rank {rank}/{world}: RCCL self-check ok={ok} ({why})", flush=True)
    # the bench's fallback after a failed check: the RCCL communicator dropped, the host
    # communicator over a gloo group beside the NCCL default group, LevMarqMPI through it
    import numpy as np
    from parallelnonlinearoptimizationlibrary_amd.device import DeviceObjective, run_levmarq
    from parallelnonlinearoptimizationlibrary_amd.dist import HostComm
    L.lib().pnol_comm_finalize()
    hc = HostComm(rank, world, group=dist.new_group(backend="gloo"))
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, 300, 1500)
    params = (0.001, 10.0, 1e-7, 6, 0.0, -1)
    x_mpi, *_ = run_levmarq(obj, np.zeros(300), params, which=1)
    x_one, *_ = run_levmarq(obj, np.zeros(300), params, which=0)
    fb = bool(np.array_equal(x_mpi, x_one))
    print(f"rank {rank}/{world}: host-communicator fallback ok={fb}", flush=True)
    hc.close()
    dist.destroy_process_group()
    sys.exit(0 if (ok and fb) else 1)


if __name__ == "__main__":
    main()
