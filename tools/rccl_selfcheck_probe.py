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
    ok, why = rccl_selfcheck(Context(local), world)
    print(f"rank {rank}/{world}: RCCL self-check ok={ok} ({why})", flush=True)
    L.lib().pnol_comm_finalize()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
