"""The C-ABI library builds, loads without a GPU, and exports every symbol include/pnol_amd.h declares."""
import re
import os

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "pnol_amd.h")).read()
    return sorted(set(re.findall(r"^(?:int|void|const char\*)\s+(pnol_[a-z0-9_]+)\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    lib = L.lib()
    declared = _declared()
    assert len(declared) >= 35
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    # the ctypes binding covers exactly the declared surface
    assert sorted(L.declared_symbols()) == declared


def test_version_and_status_strings():
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    assert L.lib().pnol_version() == 100
    assert L.status_string(0) == "ok"
    assert "gfx950" in L.status_string(L.PNOL_ERR_NODEVICE)


def test_no_device_fails_loudly_on_cpu_host():
    from parallelnonlinearoptimizationlibrary_amd import _lib as L
    if L.device_count() > 0:
        pytest.skip("a GPU is visible")
    import ctypes as C
    h = C.c_void_p()
    assert L.lib().pnol_ctx_create(0, C.byref(h)) == L.PNOL_ERR_NODEVICE
    assert L.lib().pnol_default_ctx(C.byref(h)) == L.PNOL_ERR_NODEVICE


@pytest.mark.parametrize("n,P", [(2048, 8), (2048, 3), (5, 8), (7, 2), (1, 1), (16, 16)])
def test_block_range_partitions_columns(n, P):
    from parallelnonlinearoptimizationlibrary_amd import block_range
    seen = []
    per = -(-n // P)
    for r in range(P):
        b, c = block_range(n, P, r)
        assert c >= 0 and (c == 0 or b == r * per)
        seen.extend(range(b, b + c))
    assert seen == list(range(n))


@pytest.mark.parametrize("n,P", [(2048, 8), (2048, 4), (2048, 2), (2048, 3), (2000, 8), (100, 4), (1, 1), (4096, 8)])
def test_fd_tiles_partition_and_balance(n, P):
    """LevMarqMPI's FD split: every column exactly once, tiles of PNOL_FD_TILE columns, and with
    prefix sharing (column j costs ~ n - 16 floor(j0 / 16) for its tile start j0) the per-rank
    cost within a few percent of the mean whenever every rank holds an even tile count."""
    from parallelnonlinearoptimizationlibrary_amd import fd_tiles
    cols, cost = [], []
    for r in range(P):
        tl = fd_tiles(n, P, r)
        c = 0
        for s0, cnt in tl:
            assert s0 % 128 == 0 and 0 < cnt <= 128
            cols.extend(range(s0, s0 + cnt))
            c += cnt * (n - s0)
        cost.append(c)
    assert sorted(cols) == list(range(n))
    nt = -(-n // 128)
    if nt % (2 * P) == 0:
        assert max(cost) <= 1.05 * (sum(cost) / P)
