"""MI355X-native GMRES inner-solve path of the multisplitting solvers of
craftman22/medane_tchakorom_ufc_thesis_repository.

Layers:
  include/msplit.h            C ABI (the drop-in boundary; PETSc Mat/Vec/KSP roles)
  csrc/                       HIP kernels for gfx950 + the KSPGMRES host logic in C
  _lib.py / petsc.py          ctypes binding and PETSc-style host objects
  utils.py                    the reference's glue (assembly, split, inner_solver, ...)
  comm.py                     one library communicator per rank (LibComm: RCCL send/recv and all-gathers
                              on the context's stream; torch.distributed only broadcasts the id)
  multisplitting.py           the synchronous drivers (SM, SMSM-global/-local/-semi-local)
  asynchronous.py             the asynchronous drivers (AM, AMAM-*) over HBM mailboxes
"""
from ._lib import LIB_PATH, MsplitError, load  # noqa: F401

__all__ = ["load", "LIB_PATH", "MsplitError"]
