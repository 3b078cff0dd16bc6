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
