"""World-size-2 CPU test of the sharded FD path (the *_MPI drop-ins' only exchange): two gloo
ranks run MultiObjective::gradientApproximationMPI in the C++ library with the host
communicator backend; the assembled Jacobian must equal the serial one bit for bit
(the reference's zero-padded Allreduce semantics, PNOL_Objective.cpp:279-288)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import ctypes as C
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.dist import HostComm
    comm = HostComm(rank, world)
    nr, rr = C.c_int(), C.c_int()
    L.lib().pnol_comm_size(C.byref(nr), C.byref(rr))
    assert (nr.value, rr.value) == (world, rank)
    # a 9-parameter residual (odd count: ragged last block) built from the linear residual
    m, n = 37, 9
    A, xs, y = O.linres_data(m, n)
    obj = O.Obj(O.LINRES, n, m, A, y)
    evals = []

    def fn(x, nn, F, mm, user):
        xv = np.ctypeslib.as_array(x, shape=(nn,)).copy()
        evals.append(1)
        out = O.obj_eval_multi(obj, xv)
        C.memmove(F, out.ctypes.data, 8 * mm)
    cb = L.HOST_MULTI_FN(fn)
    x = np.linspace(-0.3, 0.4, n); h = np.full(n, 1e-7)
    J = np.zeros((m, n))
    dp = C.POINTER(C.c_double)
    L.check(L.lib().pnol_host_fd_jacobian(cb, None, x.ctypes.data_as(dp), h.ctypes.data_as(dp), n, m, 1,
                                          J.ctypes.data_as(dp)), "sharded host fd")
    np.save(os.path.join(out_dir, f"J{rank}.npy"), J)
    np.save(os.path.join(out_dir, f"evals{rank}.npy"), np.array([len(evals)]))
    comm.close()
    dist.destroy_process_group()


def test_sharded_fd_jacobian_world2(tmp_path, oracle):
    world = 2
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    m, n = 37, 9
    A, xs, y = oracle.linres_data(m, n)
    ref = oracle.fd_jacobian(oracle.Obj(oracle.LINRES, n, m, A, y), np.linspace(-0.3, 0.4, n), np.full(n, 1e-7))
    J0 = np.load(tmp_path / "J0.npy"); J1 = np.load(tmp_path / "J1.npy")
    assert np.array_equal(J0, ref) and np.array_equal(J1, ref)
    # each rank evaluated its ceil(9/2) = 5 / 4 columns plus the base point
    assert int(np.load(tmp_path / "evals0.npy")[0]) == 6
    assert int(np.load(tmp_path / "evals1.npy")[0]) == 5
