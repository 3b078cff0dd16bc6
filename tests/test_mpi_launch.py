"""The *_MPI drop-ins under the reference's own launch model, `mpiexec -n P ./app`.

The reference's MPI classes take P and the rank from MPI_COMM_WORLD
(LevenbergMarquardtMPI.cpp:16-17, PNOL_Objective.cpp:102-103 / 227-228,
BFGS_with_linesearch_MPI.cpp:231-235).  examples/mpi/reference_style_mpi.cpp is a program of
the reference's shape -- MPI_Init, the *_MPI classes, MPI_Finalize, no communicator bootstrap
-- built against the drop-in headers with <mpi.h> on the include path; include/pnol_mpi_bind.hpp
binds MPI_COMM_WORLD at the first *_MPI call.  The `_nobind` build keeps the binding out, and
the library must then refuse the 2-rank job rather than run it as one rank.

MPICH 3.3 under /opt/conda is the launcher; the tests skip with that reason when it is absent.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = os.environ.get("PNOL_MPIEXEC", "/opt/conda/bin/mpiexec")
APP = os.path.join(ROOT, "examples", "mpi", "reference_style_mpi")
APP_NOBIND = APP + "_nobind"

needs_mpi = pytest.mark.skipif(not os.path.exists(MPIEXEC), reason=f"no MPI launcher at {MPIEXEC} (nothing installed)")


def _apps():
    if not (os.path.exists(APP) and os.path.exists(APP_NOBIND)):   # normally built by build()
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples", "mpi")], check=True, timeout=300)


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "PNOL_DEVICE"):   # nothing but the MPI launcher
        env.pop(k, None)
    env.setdefault("HYDRA_LAUNCHER", "fork")
    return env


def _run(nprocs, case, out, app=APP, timeout=240):
    cmd = ([MPIEXEC, "-n", str(nprocs)] if nprocs else []) + [app, case, str(out)]
    return subprocess.run(cmd, capture_output=True, timeout=timeout, env=_env(), cwd=str(out.parent))


def _parse(path):
    res = {}
    for line in open(path):
        k, *v = line.split()
        res[k] = v
    return res


def _hex(v):
    return np.array([float.fromhex(x) for x in v])


@needs_mpi
@pytest.mark.parametrize("nprocs", [2, 3])
def test_reference_program_binds_mpi_comm_world(tmp_path, nprocs):
    """testGradientApproxMultMPI's shape on the program's own host MultiObjective: the library's
    communicator is MPI_COMM_WORLD (size = nprocs), the MPI Jacobian is bitwise the serial one,
    and each rank evaluated the base point plus its own contiguous column block
    (PNOL_Objective.cpp:202-299)."""
    _apps()
    out = tmp_path / "grad.txt"
    r = _run(nprocs, "grad", out)
    assert r.returncode == 0, (r.stdout + r.stderr).decode()[-3000:]
    res = _parse(out)
    assert int(res["nprocs"][0]) == nprocs and int(res["nprocs"][2]) == nprocs   # pnol_comm_size
    n = 4
    assert int(res["nprocs"][4]) == n + 1
    J, Jm = _hex(res["J"]), _hex(res["Jmpi"])
    assert J.size == 50 * n and np.array_equal(J.view(np.uint64), Jm.view(np.uint64))
    per = -(-n // nprocs)
    want = [1 + max(0, min(n, (r_ + 1) * per) - min(n, r_ * per)) for r_ in range(nprocs)]
    assert [int(e) for e in res["rank_evals"]] == want


@needs_mpi
def test_multi_rank_launch_without_binding_is_refused(tmp_path):
    """A 2-rank launch whose program carries no binding (-DPNOL_AMD_NO_MPI_BIND) is refused by
    the first *_MPI call; it never runs as P = 1."""
    _apps()
    r = _run(2, "grad", tmp_path / "nobind.txt", app=APP_NOBIND)
    assert r.returncode != 0
    err = (r.stdout + r.stderr).decode()
    assert "no communicator is bound" in err, err[-2000:]


def test_singleton_program_runs_as_one_rank(tmp_path):
    """The same binary started without a launcher (MPI singleton): one rank, serial == MPI."""
    if not os.path.exists("/opt/conda/lib/libmpi.so"):
        pytest.skip("no MPI library under /opt/conda")
    _apps()
    out = tmp_path / "single.txt"
    r = _run(0, "grad", out)
    assert r.returncode == 0, (r.stdout + r.stderr).decode()[-3000:]
    res = _parse(out)
    assert int(res["nprocs"][2]) == 1
    assert np.array_equal(_hex(res["J"]), _hex(res["Jmpi"]))
    assert [int(e) for e in res["rank_evals"]] == [5]


def test_launcher_world_size_reads_launcher_env():
    """pnol_launcher_world_size: PMI_SIZE (MPICH / Intel MPI), OMPI_COMM_WORLD_SIZE (Open MPI),
    MV2_COMM_WORLD_SIZE (MVAPICH); 1 without a launcher.  Run in a child so the env is clean."""
    import sys
    code = ("import ctypes,sys; sys.path.insert(0, %r);"
            "from parallelnonlinearoptimizationlibrary_amd import _lib as L; print(L.lib().pnol_launcher_world_size())"
            % ROOT)
    for env_k, v, want in ((None, None, 1), ("PMI_SIZE", "4", 4), ("OMPI_COMM_WORLD_SIZE", "3", 3),
                           ("MV2_COMM_WORLD_SIZE", "2", 2)):
        env = _env()
        for k in ("PMI_SIZE", "OMPI_COMM_WORLD_SIZE", "MV2_COMM_WORLD_SIZE"):
            env.pop(k, None)
        if env_k:
            env[env_k] = v
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, env=env, timeout=120)
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        assert int(r.stdout.decode().split()[-1]) == want


@pytest.mark.parametrize("n", [12289, 13825, 16384, 20000, 4096, 8192, 100])
def test_bfgs_pass_part_tiles_cover_any_rank_count(n):
    """The fused pass's w-partial workspace holds every rank's row tiles of the allgathered
    layout (rank r's at r * tiles per shard) for any rank count, 32-row tiles included."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    lib = L.lib()
    prows = 32 if n >= 12288 else (256 if n >= 8192 else 128)
    whole = -(-n // prows)
    for P in range(1, 17):
        per = (-(-n // P) + 255) // 256 * 256
        assert lib.pnol_bfgs_pass_part_tiles(n, P) >= max(whole, P * (per // prows)), (n, P)


@pytest.mark.gpu
@needs_mpi
def test_bfgs_mpi_under_mpiexec_matches_oracle(tmp_path, oracle):
    """testBFGS_MPI (Examples.cpp:163-188) under `mpiexec -n 2`, no code change: Npool = 2 from
    MPI_COMM_WORLD (BFGS_with_linesearch_MPI.cpp:231-235), X and fOpt bitwise the oracle's
    BFGS_MPI at np = 2.  On a one-GPU box both ranks share the GPU over the host backend."""
    _apps()
    out = tmp_path / "bfgs.txt"
    r = _run(2, "bfgs_mpi", out)
    assert r.returncode == 0, (r.stdout + r.stderr).decode()[-3000:]
    res = _parse(out)
    X = _hex(res["X"])
    P = [1e-4, 0.1, 4, 1, 1000, 1e-7, 1e-3, 200, 1e-5, 1e-5, 0, 0]
    Xo, reso = oracle.bfgs_mpi_findmin(oracle.rosenbrock(10), [10.0] * 10, P, 2)
    assert np.array_equal(X, Xo)
    assert _hex(res["fopt"])[0] == reso.fopt


@pytest.mark.gpu
@needs_mpi
def test_lm_mpi_under_mpiexec_matches_reference_output(tmp_path):
    """testLMExpMPI (Examples.cpp:128-158) under `mpiexec -n 2`: X within 1e-10 of the
    reference's recorded output (the same at np = 1, 2, 4, 8; tests/golden/reference_survey.json;
    the device exp() is the only difference from the host loop)."""
    import json
    _apps()
    out = tmp_path / "lm.txt"
    r = _run(2, "lm_mpi", out)
    assert r.returncode == 0, (r.stdout + r.stderr).decode()[-3000:]
    X = _hex(_parse(out)["X"])
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_survey.json")))["testLMExp"]["X"]
    assert np.max(np.abs(X - np.array(gold)) / np.abs(np.array(gold))) <= 1e-10
