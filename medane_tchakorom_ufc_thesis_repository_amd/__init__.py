"""MI355X-native GMRES inner-solve path of the multisplitting solvers of
craftman22/medane_tchakorom_ufc_thesis_repository.

Layers:
  include/msplit.h            C ABI (the drop-in boundary; PETSc Mat/Vec/KSP roles)
  csrc/                       HIP kernels for gfx950 + the KSPGMRES host logic in C
  _lib.py / petsc.py          ctypes binding and PETSc-style host objects
  utils.py                    the reference's glue (assembly, split, inner_solver, ...)
  comm.py / multisplitting.py block exchange (RCCL via torch.distributed) and the SM driver
"""
from ._lib import LIB_PATH, MsplitError, load  # noqa: F401

__all__ = ["load", "LIB_PATH", "MsplitError"]
