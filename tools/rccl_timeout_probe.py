"""The library's bounded RCCL wait (runtime.cpp stream_wait / event_wait), on one GPU: a one-rank
RCCL communicator is bound, the context stream is blocked by a stream-wait packet on a pinned
word nobody sets, and pnol_ctx_synchronize must come back with PNOL_ERR_COMM after
PNOL_COMM_TIMEOUT_S (here 1 s) instead of hanging; the communicator is then aborted, so the
next collective fails too.  The word is released before exit so the stream drains.
Run as a child process (tests/test_gpu_mpi.py::test_rccl_stuck_wait_is_bounded)."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PNOL_COMM_TIMEOUT_S"] = "1"
from parallelnonlinearoptimizationlibrary_amd import _lib as L  # noqa: E402

lib = L.lib()
hip = C.CDLL("libamdhip64.so")
ctx = C.c_void_p()
L.check(lib.pnol_ctx_create(0, C.byref(ctx)), "ctx_create")
uid = C.create_string_buffer(128)
L.check(lib.pnol_comm_unique_id(uid), "unique_id")
L.check(lib.pnol_comm_init_rccl(ctx, 1, 0, uid.raw), "init_rccl")
word = C.c_void_p()
L.check(lib.pnol_host_alloc(C.byref(word), 64), "host_alloc")
flag = C.cast(word, C.POINTER(C.c_uint32))
flag[0] = 0
stream = C.c_void_p()
L.check(lib.pnol_ctx_get_stream(ctx, C.byref(stream)), "get_stream")
hip.hipStreamWaitValue32.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint, C.c_uint32]
rc_wait = hip.hipStreamWaitValue32(stream, word, 1, 0, 0xFFFFFFFF)   # 0 = hipStreamWaitValueGte
assert rc_wait == 0, f"hipStreamWaitValue32 -> {rc_wait}"
# The stream-wait packet stands in for an RCCL kernel waiting on a peer that never comes.  A real
# one exits when ncclCommAbort raises the communicator's abort flag; a wait packet does not, and
# the abort's own device synchronisation waits for the stream -- so a timer thread releases the
# word 3 s in (after the 1 s deadline has fired), which lets the abort complete.
import threading  # noqa: E402
rel = threading.Timer(3.0, lambda: flag.__setitem__(0, 1))
rel.start()
try:
    t0 = time.time()
    st = lib.pnol_ctx_synchronize(ctx)
    dt = time.time() - t0
finally:
    rel.join()
    flag[0] = 1   # release the stream whatever happened
rc_after = lib.pnol_ctx_synchronize(ctx)
dev = C.c_void_p()
L.check(lib.pnol_malloc(ctx, 64, C.byref(dev)), "malloc")
rc_coll = lib.pnol_comm_allgather_d(ctx, dev, dev, C.c_size_t(1))
lib.pnol_free(ctx, dev)
lib.pnol_comm_finalize()
lib.pnol_host_free(word)
lib.pnol_ctx_destroy(ctx)
print(f"bounded wait: status={st} after {dt:.2f}s; drained status={rc_after}; collective after abort={rc_coll}")
ok = st == L.PNOL_ERR_COMM and 0.9 <= dt < 30 and rc_after == 0 and rc_coll == L.PNOL_ERR_COMM
print("RCCL bounded wait ok=" + str(ok))
sys.exit(0 if ok else 1)
