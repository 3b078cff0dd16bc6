"""MI355X-native PNOL hot path: BFGS / Levenberg-Marquardt inner loops on gfx950.

The product is libpnol_amd.so (HIP kernels, the C ABI of include/pnol_amd.h and the C++
drop-in classes of include/*.hpp).  This package only loads and drives it:
  _lib      ctypes binding of every C-ABI entry point
  device    torch-tensor wrappers (Context, DeviceObjective, run_bfgs, run_levmarq)
  dist      RCCL communicator bootstrap over torch.distributed (one process per GPU)
  build     hipcc build of the library (used by __graft_entry__.build())
"""
from ._lib import (PNOL_OK, PNOL_SEQ_MAX, OBJ_CUBIC, OBJ_EXPCURVE, OBJ_LINRES, OBJ_POWER, OBJ_QUADRATIC,
                   OBJ_ROSENBROCK, PnolError, block_range, device_count, fd_tiles, lib)

__all__ = ["lib", "device_count", "block_range", "fd_tiles", "PnolError", "PNOL_OK", "PNOL_SEQ_MAX", "OBJ_ROSENBROCK",
           "OBJ_POWER", "OBJ_QUADRATIC", "OBJ_EXPCURVE", "OBJ_CUBIC", "OBJ_LINRES"]
