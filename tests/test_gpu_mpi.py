"""LevMarqMPI, BFGSBnd_MPI and BFGS_Bnd_MPI_SW on the device with more than one rank: two processes share the box's one GPU and
exchange through the host communicator backend (gloo allgather callback).  The sharded FD
Jacobian (column blocks + allgather) and the tile-sharded J^T J (pnol_jtj_mpi_d) must give
results bitwise equal to the single-rank device run -- the reference's MPI results are
likewise independent of the rank count."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_workers(tmp_path, world, m, n, *extra, rank_env=None):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", PNOL_DEVICE="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update((rank_env or {}).get(r, {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_mpi_worker.py"), str(tmp_path),
                                       str(m), str(n), *extra], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode(errors="replace"))
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-3000:] for o in outs)


def _check_levmarq_and_normal(tmp_path, world, m, n):
    """LevMarqMPI X, the tile-split J^T J and the m-sliced normal equations of every rank equal
    the single-GPU LevMarq / pnol_jtj_d / pnol_jtr_d bitwise."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X1, *_ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=0)
    rng = np.random.default_rng(11)
    JT = ctx.tensor(rng.standard_normal((n, m)))
    A1, d1 = ctx.jtj(JT, 0.25, want_diag=True)
    r1 = ctx.jtr(JT, ctx.tensor(np.random.default_rng(12).standard_normal(m)))
    A1, d1, r1 = A1.cpu().numpy(), d1.cpu().numpy(), r1.cpu().numpy()
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["X"], X1), r
        assert np.array_equal(z["A"], A1), r
        assert np.array_equal(z["diag"], d1), r
        assert np.array_equal(z["As"], A1), r
        assert np.array_equal(z["ds"], d1), r
        assert np.array_equal(z["rs"], r1), r


@pytest.mark.parametrize("world,m,n", [(4, 1500, 200), (5, 1500, 200), (8, 1500, 200), (8, 600, 130), (6, 700, 129)])
def test_levmarq_mpi_m_sliced_more_ranks(tmp_path, world, m, n):
    """The m-sliced LevMarqMPI path at 4 to 8 ranks (one slice per rank at 8; uneven dyadic
    slice covers at 5 and 6; m = 600 leaves slices 5-7 empty, so three ranks own no rows; ranks
    without FD tiles or without J^T J tiles), bitwise the single-GPU results."""
    _run_workers(tmp_path, world, m, n, "lm")
    _check_levmarq_and_normal(tmp_path, world, m, n)


def _set_mode(monkeypatch, mode):
    if mode == "rows":
        monkeypatch.setenv("PNOL_LM_FD", "rows")
    else:
        monkeypatch.delenv("PNOL_LM_FD", raising=False)


@pytest.mark.parametrize("mode", ["rows", "columns"])
@pytest.mark.parametrize("world,m,n", [(2, 1500, 200), (4, 2000, 300), (8, 600, 130), (3, 1000, 700)])
def test_levmarq_mpi_fd_modes_bitwise(tmp_path, monkeypatch, mode, world, m, n):
    """LevMarqMPI's two Jacobian decompositions: columns mode (default, the reference's:
    cost-balanced FD column tiles per rank, each tile's m-slices exchanged behind its launch) and
    rows mode (PNOL_LM_FD=rows: every FD column on the rank's own m-slices, trial residuals
    shared point-to-point -- no Jacobian exchange).  X, F0 and FOpt on every rank are bitwise the
    single-GPU LevMarq's either way (m = 600 at 8 ranks: three ranks own no rows; n = 700 at 3
    ranks: unequal tile counts, so rank 2 sits out the last exchange phase)."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    _set_mode(monkeypatch, mode)
    _run_workers(tmp_path, world, m, n, "lm")
    monkeypatch.delenv("PNOL_LM_FD", raising=False)
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X1, F01, FO1, _ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=0)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["X"], X1), (mode, r)
        assert np.array_equal(z["F0"], F01) and np.array_equal(z["FO"], FO1), (mode, r)


@pytest.mark.parametrize("trip,force", [("1", "0"), ("0", "0"), ("1", "1")])
@pytest.mark.parametrize("world", [2, 4])
def test_levmarq_mpi_trip_forms_bitwise(tmp_path, monkeypatch, trip, force, world):
    """LevMarqMPI's normal equations + solve without forming A (pnol_lm_normal_solve_mpi_d: the
    allgathered tiles go straight into the Cholesky's matrix; the default), the two calls
    (PNOL_LM_TRIP=0), and the LU fallback forced on every trip (A formed from the same tiles,
    pnol_lm_normal_unpack_mpi_d): X, F0 and FOpt on every rank bitwise the one-GPU LevMarq's
    under the same settings."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    m, n = 2000, 300
    monkeypatch.setenv("PNOL_LM_TRIP", trip)
    monkeypatch.setenv("PNOL_CHOL_FORCE_FALLBACK", force)
    _run_workers(tmp_path, world, m, n, "lm")
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X1, F01, FO1, _ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=0)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["X"], X1), (trip, force, r)
        assert np.array_equal(z["F0"], F01) and np.array_equal(z["FO"], FO1), (trip, force, r)


@pytest.mark.parametrize("world", [2, 3])
def test_levmarq_mpi_columns_unphased_bitwise(tmp_path, monkeypatch, world):
    """Columns mode with the Jacobian's slice exchange in one step after the FD launch
    (PNOL_LM_PHASED=0: no second stream, no per-tile events) gives the same X, F0 and FOpt as
    one GPU -- the same blocks reach the same ranks, only the overlap differs."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    m, n = 1000, 700
    _set_mode(monkeypatch, "columns")
    monkeypatch.setenv("PNOL_LM_PHASED", "0")
    _run_workers(tmp_path, world, m, n, "lmonly")
    monkeypatch.delenv("PNOL_LM_PHASED")
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X1, F01, FO1, _ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=0)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["X"], X1), r
        assert np.array_equal(z["F0"], F01) and np.array_equal(z["FO"], FO1), r


@pytest.mark.parametrize("status", ["1", "-7"])
@pytest.mark.parametrize("mode", ["columns", "rows"])
@pytest.mark.parametrize("world", [2, 3])
def test_levmarq_mpi_one_rank_solve_status(tmp_path, monkeypatch, status, mode, world):
    """One rank's trip solve reports a status its peers do not see (PNOL_CHOL_FORCE_FALLBACK on
    the last rank only, every trip): a non-positive pivot (1) or a timed-out wait (-7).  The
    reference's replicas never branch per rank -- each runs the same luSolve on the same A
    (LevenbergMarquardtMPI.cpp:88) -- so the status is agreed over the ranks inside the trip
    (pnol_lm_agree_status_d) and every rank takes the same action: the reference-order LU for a
    pivot, the same Cholesky relaunched for a timeout.  In both FD modes (rows mode exchanges the
    trial residuals, so a rank-local redo would desync the collectives) X, F0 and FOpt on every
    rank are bitwise the one-GPU LevMarq's with the LU on every trip (status 1) or unforced (-7)."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    m, n = 1000, 700
    _set_mode(monkeypatch, mode)
    monkeypatch.delenv("PNOL_CHOL_FORCE_FALLBACK", raising=False)
    _run_workers(tmp_path, world, m, n, "lmonly", rank_env={world - 1: {"PNOL_CHOL_FORCE_FALLBACK": status}})
    monkeypatch.delenv("PNOL_LM_FD", raising=False)
    if status == "1":
        monkeypatch.setenv("PNOL_CHOL_FORCE_FALLBACK", "1")
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X1, F01, FO1, _ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=0)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["X"], X1), (status, mode, r)
        assert np.array_equal(z["F0"], F01) and np.array_equal(z["FO"], FO1), (status, mode, r)


@pytest.mark.parametrize("mode", ["columns", "rows"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_levmarq_mpi_cfg4_full_size_bitwise(tmp_path, monkeypatch, mode, world):
    """cfg 4 at the headline size (m = 16384, n = 2048; LevenbergMarquardtMPI.cpp:12-172 with the
    FD Jacobian of PNOL_Objective.cpp:202-299): columns mode (the reference's decomposition, the
    bench's headline: FD column tiles per rank + the phased m-slice exchange) and rows mode over
    2, 4 and 8 ranks (sharing the box's GPU, host communicator) give X, F0 and FOpt after 5 trips
    bitwise equal to the one-GPU LevMarq, which test_lm_cfg3_full_size_matches_oracle_trips holds
    to the oracle's trips."""
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_levmarq
    m, n = 16384, 2048
    _set_mode(monkeypatch, mode)
    _run_workers(tmp_path, world, m, n, "lmonly")
    monkeypatch.delenv("PNOL_LM_FD", raising=False)
    ctx = Context(0)
    obj = DeviceObjective.synthetic(ctx, L.OBJ_LINRES, n, m)
    X1, F01, FO1, _ = run_levmarq(obj, np.zeros(n), (0.001, 10.0, 1e-7, 5, 0.0, -1), which=0)
    obj.close()
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert int(z["mode"][0]) == (1 if mode == "rows" else 0), r
        assert np.array_equal(z["X"], X1), r
        assert np.array_equal(z["F0"], F01) and np.array_equal(z["FO"], FO1), r


def test_levmarq_mpi_mode_disagreement_is_refused(tmp_path):
    """The FD decomposition is read once per LevMarqMPI solve and must be the same on every rank
    (the two modes pair different transfers): ranks started with different PNOL_LM_FD stop with
    an error instead of mismatching their exchanges."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", PNOL_DEVICE="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.pop("PNOL_LM_FD", None)
        if r == 1:
            env["PNOL_LM_FD"] = "rows"
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_mpi_worker.py"), str(tmp_path),
                                       "600", "130", "lmonly"], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode(errors="replace"))
    assert all(p.returncode != 0 for p in procs), "\n".join(o[-2000:] for o in outs)
    assert any("disagree on PNOL_LM_FD" in o for o in outs)


@pytest.mark.parametrize("world", [2, 3])
def test_levmarq_mpi_ranks_bitwise_equal_single(tmp_path, world, oracle):
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    from parallelnonlinearoptimizationlibrary_amd.device import Context, DeviceObjective, run_bfgs
    m, n = 2000, 300     # 6 J^T J tiles: uneven tile ranges at world = 3 / 4
    _run_workers(tmp_path, world, m, n)
    _check_levmarq_and_normal(tmp_path, world, m, n)
    ctx = Context(0)
    # BFGSBnd_MPI across the ranks equals the reference at np = world
    nb = 10
    x0 = np.full(nb, 3.0); x0[0] = -0.5
    lb = np.full(nb, -5.0); lb[0] = -1.0
    Pb = [1e-4, 0.1, 1e-16, 4, 1, 1000, 1e-7, 1e-3, 200, 1e-5, 1e-5, 1e-5, 0, 0]
    Xo, reso, st = oracle.bfgs_bnd_mpi_findmin(oracle.rosenbrock(nb), x0, lb, np.full(nb, 5.0), Pb, world)
    assert st == 0
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["Xb"], Xo), r
        assert z["fb"][0] == reso.fopt, r
    # BFGS_Bnd_MPI_SW across the ranks equals the reference at np = world
    Psw = [1e-4, 0.8, 1e-6, 1, 1e-10, 2, 50, 1e-5, 1e-6, 1e-3, 200, 1e-5, 1e-5, 0, -1]
    Xo, reso = oracle.bfgs_bnd_mpi_sw_findmin(oracle.rosenbrock(3), [-1.0, 2.0, 2.0], [-1.0] * 3, [5.0] * 3, Psw,
                                              world)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["Xs"], Xo), r
        assert z["fs"][0] == reso.fopt, r
    # GeneticAlgorithmMPI across the ranks equals the restatement at np = world (row f4); the
    # evaluation count is the whole job's, split over the ranks
    Xgo, rgo, st = oracle.ga_findmin(oracle.rosenbrock(4), np.full(4, -1.0), np.full(4, -2.0), np.full(4, 2.0),
                                     [40, 200, 0.1, 0.3, 0.2, 0.5, 0.01, 0.5, 20], 12345, world)
    assert st == 0
    evals = 0
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["Xga"], Xgo), r
        assert z["ga"][0] == rgo.f0 and z["ga"][1] == rgo.fopt and z["ga"][2] == rgo.iters, r
        evals += int(z["ga"][3])
    assert evals == rgo.evals
    # BFGS D row-sharded: the collective H.g / fused pass equal the whole-matrix kernels bitwise,
    # and BFGS_MPI in fast mode gives the single-rank trajectory bitwise
    import torch
    nD = 700
    rng = np.random.default_rng(3)
    Dfull = rng.standard_normal((nD, nD))
    g, yv, sv, av, bv = (rng.standard_normal(nD) for _ in range(5))
    dD = ctx.tensor(Dfull)
    hg = ctx.hg(dD, ctx.tensor(g)).cpu().numpy()
    u, w, v = (t.cpu().numpy() for t in ctx.bfgs_pass(dD, ctx.tensor(yv), ctx.tensor(g),
                                                       pending=(ctx.tensor(sv), ctx.tensor(av), ctx.tensor(bv)),
                                                       write_back=True))
    Dafter = dD.cpu().numpy()
    covered = 0
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["hg"], hg), r
        assert np.array_equal(z["u"], u) and np.array_equal(z["w"], w) and np.array_equal(z["v"], v), r
        rb, rc = z["rows"]
        assert np.array_equal(z["Drows"], Dafter[rb:rb + rc]), r
        covered += rc
    assert covered == nD
    # the sharded free-free block: every rank's new rows equal the whole-matrix gather
    covered = 0
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        keep = z["keep"]
        sub = Dfull[np.ix_(keep, keep)]
        sb, sc = z["subrows"]
        assert np.array_equal(z["Dsub"], sub[sb:sb + sc]), r
        covered += sc
    assert covered == len(keep)
    from parallelnonlinearoptimizationlibrary_amd.device import run_bfgs
    # BFGSBnd_MPI fast mode with the sharded D and its sharded boundary recursion: the ranks'
    # trajectory equals the single-rank one bitwise
    Pf = [1e-4, 0.1, 1e-16, 4, 1, 200, 1e-6, 1e-3, 100, 1e-9, 1e-6, 1e-9, 0, 0, 4]
    Xf1, resf1 = run_bfgs(DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, 600, 0, bscale=4.0), np.zeros(600), Pf,
                          which=3, lb=np.full(600, -0.25), ub=np.full(600, 0.25))
    assert np.any(np.abs(Xf1) == 0.25)   # bounds active: the recursion ran
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["Xf"], Xf1), r
        assert z["ff"][0] == resf1.fopt, r
    Pq = [1e-4, 0.9, 4, 1, 1000, 1e-6, 1e-3, 40, 1e-9, 1e-6, 0, 0, 4, 1, 2]
    Xq1, resq1 = run_bfgs(DeviceObjective.synthetic(ctx, L.OBJ_QUADRATIC, 300), np.zeros(300), Pq, which=1)
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        assert np.array_equal(z["Xq"], Xq1), r
        assert z["fq"][0] == resq1.fopt, r


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_multi_rank_line_is_valid(tmp_path, world):
    """bench.py's N > 1 line, rehearsed with `world` ranks on the box's one GPU over the host
    communicator: the roofline prices the SYRK each rank actually ran -- its own m-slices' rows
    (LevenbergMarquardtMPI.cpp:64-78 split by slice) -- so achieved = rows n (n + 1) / syrk time
    and frac <= 1; the line names the communicator and its size, and carries the FD-Jacobian
    strong-scaling quantity."""
    import json
    port = _free_port()
    m, n = 8192, 1024
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(os.path.dirname(HERE), "bench.py"),
           "--gpus", str(world), "--host-comm", "--steps", "3", "--warmup", "1", "--residuals", str(m), "--params", str(n),
           "--no-cpu-baseline", "--no-hg", "--no-bfgs"]
    r = subprocess.run(cmd, capture_output=True, timeout=300, env=dict(os.environ, PNOL_DEVICE="0"))
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-3000:]
    line = json.loads([l for l in r.stdout.decode().splitlines() if l.startswith("{")][-1])
    rf = line["roofline"]
    mS = ((m + 7) // 8 + 63) // 64 * 64          # lm_slice_rows: 8 m-slices, 64-row multiples
    rows = min(m, (8 // world) * mS)              # rank 0 holds slices [0, 8 / world)
    assert rf["rows"] == rows and rf["flop_per_launch"] == float(rows) * n * (n + 1)
    syrk_ms = line["kernel_ms_per_step"]["syrk"]
    assert abs(rf["achieved"] - rf["flop_per_launch"] / (syrk_ms * 1e-3) / 1e12) <= 1e-9 * rf["achieved"]
    assert 0 < rf["frac"] <= 1.0
    assert rf["traffic"] is None   # no committed PMC pass at this (m, n); the metric's size has one
    assert line["comm"] == {"backend": "host-gloo", "ranks": world} and line["n_gpus"] == world
    assert line["fd_jacobian_ms_max_over_ranks"] > 0
    assert "host communicator" in line["config"]["workload"]


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` without a launcher starts its own two ranks (one process per
    GPU; here both share the box's GPU over the host communicator) and the relayed line reports
    the job it measured: n_gpus = communicator size = 2."""
    import json
    m, n = 4096, 512
    cmd = [sys.executable, os.path.join(os.path.dirname(HERE), "bench.py"), "--gpus", "2", "--host-comm",
           "--steps", "2", "--warmup", "1", "--residuals", str(m), "--params", str(n),
           "--no-bfgs", "--no-hg", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-3000:]
    lines = [l for l in r.stdout.decode().splitlines() if l.strip()]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["comm"] == {"backend": "host-gloo", "ranks": 2}
    assert 0 < line["roofline"]["frac"] <= 1.0
    assert line["value"] > 0


def test_rccl_selfcheck_world1():
    """The bench's N > 1 guard (dist.rccl_selfcheck): the library's RCCL communicator (one rank on
    the box's one GPU -- RCCL refuses two ranks on one device) carries a small LevMarqMPI whose X
    must equal the one-process LevMarq bit for bit; the probe exits 0 only when it does."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", f"--master-port={port}", os.path.join(os.path.dirname(HERE), "tools", "rccl_selfcheck_probe.py")]
    r = subprocess.run(cmd, capture_output=True, timeout=240)
    out = r.stdout.decode(errors="replace") + r.stderr.decode(errors="replace")
    assert r.returncode == 0, out[-3000:]
    assert "RCCL self-check ok=True" in out
    assert "host-communicator fallback ok=True" in out


def test_rccl_stuck_wait_is_bounded():
    """A device wait with an RCCL communicator bound is bounded: a stream blocked past
    PNOL_COMM_TIMEOUT_S returns PNOL_ERR_COMM after ncclCommAbort, and later collectives fail
    with PNOL_ERR_COMM -- a stuck exchange on a multi-GPU node ends in an error, not a hang
    (tools/rccl_timeout_probe.py, one rank on the box's GPU)."""
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), "tools", "rccl_timeout_probe.py")],
                       capture_output=True, timeout=180)
    out = r.stdout.decode(errors="replace") + r.stderr.decode(errors="replace")
    assert r.returncode == 0, out[-3000:]
    assert "RCCL bounded wait ok=True" in out
