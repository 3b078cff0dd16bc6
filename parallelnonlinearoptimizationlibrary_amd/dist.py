"""RCCL communicator bootstrap for the *_MPI drop-ins: one process per GPU.

torch.distributed (launched by torch.distributed.run) only carries the 128-byte RCCL unique
id from rank 0 to the others; every data-path collective afterwards is the library's own
ncclAllGather on its stream.  For CPU tests the host backend takes a Python allgather
(torch.distributed over gloo) instead.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _lib as L


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init_rccl(ctx, rank: int, world: int):
    """Create the library's RCCL communicator; torch.distributed must be initialised."""
    import torch
    import torch.distributed as dist
    buf = C.create_string_buffer(128)
    if rank == 0:
        L.check(L.lib().pnol_comm_unique_id(buf), "pnol_comm_unique_id")
    t = torch.tensor(list(buf.raw), dtype=torch.uint8)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.broadcast(t, src=0)
    raw = bytes(t.cpu().tolist())
    L.check(L.lib().pnol_comm_init_rccl(ctx.h, world, rank, raw), "pnol_comm_init_rccl")
    n, r = C.c_int(), C.c_int()
    L.check(L.lib().pnol_comm_size(C.byref(n), C.byref(r)), "pnol_comm_size")
    if rank == 0:
        import sys
        print(f"[pnol_amd] RCCL communicator: {n.value} ranks", file=sys.stderr, flush=True)
    return n.value


def rccl_selfcheck(ctx, world: int, timeout_s: float = 300.0):
    """Before an N > 1 measurement: one small LevMarqMPI run through the library's RCCL
    communicator (m-slice exchange, tree-order reduce-scatter, allgather) must give bitwise the
    single-process LevMarq's X on every rank.  Returns (ok, reason), agreed by all ranks.

    A rank whose run raises may leave the others blocked inside an RCCL collective, where no
    agreement all_reduce can reach them: such a rank exits the process (status 3) so the launcher
    stops the job, and a watchdog exits any rank still inside the check after `timeout_s`
    (status 124).  Only a completed run whose X differs is reported as (False, reason)."""
    import sys
    import threading
    import numpy as np
    import torch
    import torch.distributed as dist
    from .device import DeviceObjective, run_levmarq

    def _expire():
        print(f"[pnol_amd] RCCL self-check still running after {timeout_s:.0f} s: exiting", file=sys.stderr,
              flush=True)
        os._exit(124)

    dog = threading.Timer(timeout_s, _expire)
    dog.daemon = True
    dog.start()
    ok, why = True, "ok"
    try:
        m, n = 1500, 300
        obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
        params = (0.001, 10.0, 1e-7, 6, 0.0, -1)
        x_mpi, *_ = run_levmarq(obj, np.zeros(n), params, which=1)
        x_one, *_ = run_levmarq(obj, np.zeros(n), params, which=0)
        if not np.array_equal(x_mpi, x_one):
            ok, why = False, f"LevMarqMPI X differs from LevMarq (max |dx| {np.abs(x_mpi - x_one).max():.3e})"
    except Exception as e:  # noqa: BLE001 -- the other ranks may be stuck in a collective
        print(f"[pnol_amd] RCCL self-check raised {type(e).__name__}: {e}; exiting", file=sys.stderr, flush=True)
        os._exit(3)
    flag = torch.tensor([0.0 if ok else 1.0], device="cuda")
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    dog.cancel()
    if flag.item() != 0.0 and ok:
        ok, why = False, "the self-check failed on another rank"
    return ok, why


class HostComm:
    """Host-backend communicator: allgather of raw bytes through torch.distributed (gloo);
    `group`: a gloo process group when the default group is NCCL."""

    def __init__(self, rank: int, world: int, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.world = torch, dist, world

        def _allgather(send, recv, nbytes, user):
            try:
                src = (C.c_uint8 * nbytes).from_address(send)
                t = torch.frombuffer(bytearray(src), dtype=torch.uint8)
                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(outs, t, group=group)
                C.memmove(recv, bytes(torch.cat(outs).numpy()), nbytes * world)
                return 0
            except Exception:  # pragma: no cover - surfaces as PNOL_ERR_COMM
                return 1

        self._cb = L.ALLGATHER_FN(_allgather)
        L.check(L.lib().pnol_comm_init_host(world, rank, self._cb, None), "pnol_comm_init_host")

    def close(self):
        L.lib().pnol_comm_finalize()
