"""ctypes binding of libmsplit_hip.so (include/msplit.h).

The product path has exactly one implementation: the HIP library.  Loading it
fails loudly when the .so is missing, and every call raises MsplitError with
the library's message when the C ABI returns a nonzero (PETSc-numbered) code.
There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# MSPLIT_LIB: another build of the same library (same-box A/B of two builds, tools/ab_build.sh)
LIB_PATH = os.environ.get("MSPLIT_LIB") or os.path.join(HERE, "libmsplit_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "msplit.h")

KERNEL_CLASSES = {"spmv": 0, "mdot": 1, "maxpy": 2, "norm": 3, "scale": 4, "other": 5,
                  "spmm": 6, "dgemv": 7, "dgemvt": 8, "spmvdot": 9}

REASONS = {
    0: "CONVERGED_ITERATING", 1: "CONVERGED_RTOL_NORMAL", 2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL",
    4: "CONVERGED_ITS", 9: "CONVERGED_ATOL_NORMAL",
    -2: "DIVERGED_NULL", -3: "DIVERGED_ITS", -4: "DIVERGED_DTOL",
    -5: "DIVERGED_BREAKDOWN", -9: "DIVERGED_NANORINF",
}


class MsplitError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


class KspOpts(C.Structure):
    _fields_ = [("restart", C.c_int32), ("max_it", C.c_int32), ("rtol", C.c_double),
                ("abstol", C.c_double), ("divtol", C.c_double), ("haptol", C.c_double),
                ("breakdowntol", C.c_double), ("uirnorm", C.c_int32), ("guess_nonzero", C.c_int32)]


class LsqrOpts(C.Structure):
    _fields_ = [("max_it", C.c_int32), ("rtol", C.c_double), ("abstol", C.c_double), ("divtol", C.c_double),
                ("exact_norm", C.c_int32), ("conv_test", C.c_int32)]


LSQR_CONV = {"default": 0, "lsqr": 1, "skip": 2}
COMM_ID_BYTES = 128
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64)

_lib = None

_P = C.POINTER
_vp = C.c_void_p
_i32p = _P(C.c_int32)
_dp = _P(C.c_double)

# name -> argtypes (restype is int for all but msp_get_last_error)
_SIGS = {
    "msp_ctx_create": [C.c_int, _vp, _P(_vp)],
    "msp_ctx_destroy": [_P(_vp)],
    "msp_ctx_synchronize": [_vp],
    "msp_get_device_count": [_P(C.c_int)],
    "msp_ctx_set_timing": [_vp, C.c_int],
    "msp_ctx_set_reduction": [_vp, C.c_int],
    "msp_ctx_get_reduction": [_vp, _P(C.c_int)],
    "msp_ctx_reset_kernel_stats": [_vp],
    "msp_ctx_get_kernel_stats": [_vp, C.c_int, _P(C.c_int64), _dp, _dp],
    "msp_mat_create_csr": [_vp, C.c_int32, C.c_int32, _i32p, _i32p, _dp, _P(_vp)],
    "msp_mat_create_csr_rows": [_vp, C.c_int32, C.c_int32, C.c_int32, _i32p, _i32p, _i32p, _dp, _P(_vp)],
    "msp_mat_create_box_stencil": [_vp, C.c_int, C.c_int32, C.c_int32, C.c_int32, _P(_vp)],
    "msp_mat_destroy": [_P(_vp)],
    "msp_mat_get_info": [_vp, _i32p, _i32p, _P(C.c_int64)],
    "msp_mat_get_csr": [_vp, _i32p, _i32p, _dp],
    "msp_mat_mult": [_vp, _vp, _vp],
    "msp_mat_residual": [_vp, _vp, _vp, _vp],
    "msp_mat_residual_listed": [_vp, _vp, _vp, _vp],
    "msp_vec_create": [_vp, C.c_int64, _P(_vp)],
    "msp_vec_create_with_array": [_vp, C.c_int64, _vp, _P(_vp)],
    "msp_vec_destroy": [_P(_vp)],
    "msp_vec_get_size": [_vp, _P(C.c_int64)],
    "msp_vec_get_array": [_vp, _P(_vp)],
    "msp_vec_set_values": [_vp, C.c_int64, C.c_int64, _dp],
    "msp_vec_get_values": [_vp, C.c_int64, C.c_int64, _dp],
    "msp_vec_copy_range": [_vp, C.c_int64, _vp, C.c_int64, C.c_int64],
    "msp_vec_set": [_vp, C.c_double],
    "msp_vec_copy": [_vp, _vp],
    "msp_vec_scale": [_vp, C.c_double],
    "msp_vec_axpy": [_vp, C.c_double, _vp],
    "msp_vec_aypx": [_vp, C.c_double, _vp],
    "msp_vec_waxpy": [_vp, C.c_double, _vp, _vp],
    "msp_vec_dot": [_vp, _vp, _dp],
    "msp_vec_norm": [_vp, _dp],
    "msp_vec_normalize": [_vp, _dp],
    "msp_vec_mdot": [_vp, C.c_int, _P(_vp), _dp],
    "msp_vec_maxpy": [_vp, C.c_int, _dp, _P(_vp)],
    "msp_ksp_get_default_opts": [_P(KspOpts)],
    "msp_ksp_create": [_vp, _P(_vp)],
    "msp_ksp_destroy": [_P(_vp)],
    "msp_ksp_set_operators": [_vp, _vp],
    "msp_ksp_set_opts": [_vp, _P(KspOpts)],
    "msp_ksp_get_opts": [_vp, _P(KspOpts)],
    "msp_ksp_set_up": [_vp],
    "msp_ksp_solve": [_vp, _vp, _vp],
    "msp_ksp_get_iteration_number": [_vp, _i32p],
    "msp_ksp_get_residual_norm": [_vp, _dp],
    "msp_ksp_get_converged_reason": [_vp, _i32p],
    "msp_ksp_get_residual_history": [_vp, _P(_dp), _i32p],
    "msp_mat_create_box_stencil_ext": [_vp, C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                       _P(_vp)],
    "msp_mat_create_box_matfree": [_vp, C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _dp,
                                   _P(_vp)],
    "msp_mat_create_box_convdiff": [_vp, C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _dp,
                                    _P(_vp)],
    "msp_mat_set_storage": [_vp, C.c_int],
    "msp_mat_get_storage": [_vp, _i32p, _i32p],
    "msp_mat_release_csr": [_vp],
    "msp_mat_get_spmv_kernel": [_vp, _P(C.c_char_p)],
    "msp_dense_create": [_vp, C.c_int64, C.c_int32, _P(_vp)],
    "msp_dense_destroy": [_P(_vp)],
    "msp_dense_get_info": [_vp, _P(C.c_int64), _i32p, _P(C.c_int64)],
    "msp_dense_get_array": [_vp, _P(_vp)],
    "msp_dense_zero_entries": [_vp],
    "msp_dense_set_values": [_vp, _dp, C.c_int64],
    "msp_dense_get_values": [_vp, _dp, C.c_int64],
    "msp_dense_set_column": [_vp, C.c_int32, C.c_int64, _vp, C.c_int64, C.c_int64],
    "msp_dense_mult": [_vp, _vp, C.c_int64, C.c_int64, _vp, C.c_int64],
    "msp_dense_mult_transpose": [_vp, _vp, _vp],
    "msp_dense_gram": [_vp, _vp, _vp],
    "msp_dense_sum": [C.c_int32, _P(_vp), _vp],
    "msp_dense_create_view": [_vp, C.c_int32, C.c_int32, _P(_vp)],
    "msp_mat_matmult_dense": [_vp, _vp, _vp],
    "msp_comm_get_unique_id": [_P(C.c_uint8)],
    "msp_comm_rccl_available": [_i32p],
    "msp_comm_create_rccl": [_vp, C.c_int32, C.c_int32, _P(C.c_uint8), _P(_vp)],
    "msp_comm_create_host": [_vp, C.c_int32, C.c_int32, ALLGATHER_FN, _vp, _P(_vp)],
    "msp_comm_destroy": [_P(_vp)],
    "msp_comm_get_size": [_vp, _i32p, _i32p],
    "msp_comm_allgather": [_vp, _vp, _vp, C.c_int64],
    "msp_lsqr_get_default_opts": [_P(LsqrOpts)],
    "msp_lsqr_create": [_vp, _P(_vp)],
    "msp_lsqr_destroy": [_P(_vp)],
    "msp_lsqr_set_opts": [_vp, _P(LsqrOpts)],
    "msp_lsqr_get_opts": [_vp, _P(LsqrOpts)],
    "msp_lsqr_set_operators": [_vp, C.c_int32, _P(_vp)],
    "msp_lsqr_set_comm": [_vp, _vp],
    "msp_lsqr_solve": [_vp, _P(_vp), _vp],
    "msp_lsqr_get_iteration_number": [_vp, _i32p],
    "msp_lsqr_get_residual_norm": [_vp, _dp],
    "msp_lsqr_get_converged_reason": [_vp, _i32p],
    "msp_lsqr_get_norms": [_vp, _dp, _dp],
    "msp_lsqr_get_residual_history": [_vp, _P(_dp), _i32p],
    "msp_amsg_create": [C.c_char_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32, _P(_vp)],
    "msp_amsg_destroy": [_P(_vp)],
    "msp_amsg_attached": [_vp, _i32p],
    "msp_amsg_send": [_vp, C.c_int32, C.c_int32, _i32p, C.c_int32, _dp, C.c_int64],
    "msp_amsg_recv": [_vp, C.c_int32, C.c_int32, _i32p, C.c_int32, _dp, C.c_int64, _P(C.c_int64), _i32p],
    "msp_amsg_send_vec": [_vp, C.c_int32, _i32p, C.c_int32, _vp, C.c_int64, C.c_int64],
    "msp_amsg_recv_vec": [_vp, C.c_int32, _i32p, C.c_int32, _vp, C.c_int64, C.c_int64, _P(C.c_int64), _i32p],
    "msp_comm_exchange_neighbors": [_vp, _vp, C.c_int64, C.c_int64, _vp, C.c_int64, C.c_int64, C.c_int64],
    "msp_comm_sum_ordered": [_vp, _dp, _dp, C.c_int32],
    "msp_comm_agree": [_vp, C.c_int64, C.POINTER(C.c_int32)],
    "msp_amsg_enable_device": [_vp, _vp],
    "msp_amsg_close_peers": [_vp],
    "msp_amsg_get_stats": [_vp, _P(C.c_int64), _P(C.c_int64)],
    "msp_amsg_discard_pending": [_vp, _P(C.c_int64), _P(C.c_int64)],
    "msp_amsg_get_link_info": [_vp, C.c_int32, _P(C.c_int64), C.c_int32],
    "msp_abcast_discard_pending": [_vp, _P(C.c_int64), _P(C.c_int64)],
    "msp_abcast_enable_device": [_vp, _vp, C.c_int32],
    "msp_abcast_get_nbuf": [_vp, _i32p],
    "msp_abcast_get_stats": [_vp, _P(C.c_int64), _P(C.c_int64)],
    "msp_abcast_close_peers": [_vp],
    "msp_abcast_create": [C.c_char_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32, _P(_vp)],
    "msp_abcast_destroy": [_P(_vp)],
    "msp_abcast_publish": [_vp, _dp, C.c_int64, C.c_int32, C.c_int64, _i32p],
    "msp_abcast_fetch": [_vp, C.c_int32, _dp, C.c_int64, C.c_int32, C.c_int64, _i32p],
    "msp_abcast_publish_dense": [_vp, _vp, _i32p],
    "msp_abcast_fetch_dense": [_vp, C.c_int32, _vp, _i32p],
    "msp_cvd_create": [_vp, C.c_int32, C.c_int32, _i32p, C.c_int32, _i32p, C.c_int32, _P(_vp)],
    "msp_cvd_destroy": [_P(_vp)],
    "msp_cvd_data_received": [_vp, C.c_int32, C.c_int32, C.c_int32, _i32p],
    "msp_cvd_step": [_vp, C.c_int32],
    "msp_cvd_get_state": [_vp, _i32p, _i32p],
    "msp_cvd_get_info": [_vp, _i32p, C.c_int32],
}


def header_symbols() -> list[str]:
    """Every function declared in include/msplit.h."""
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(msp_[a-z0-9_]+)\s*\(", txt)))


def load() -> C.CDLL:
    """Load the HIP library.  Import torch first when it is used in the same
    process, so that one HIP runtime (same soname) serves both."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C medane_tchakorom_ufc_thesis_repository_amd/csrc` (hipcc, gfx950). "
            "There is no CPU fallback for the MI355X path.")
    L = C.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = C.c_int
    L.msp_get_last_error.argtypes = []
    L.msp_get_last_error.restype = C.c_char_p
    L.msp_build_source_digest.argtypes = []
    L.msp_build_source_digest.restype = C.c_char_p
    _lib = L
    return L


def source_digest() -> str:
    """SHA-256 of the library sources in this tree, hashed as csrc/Makefile does (DIGEST_SRCS: *.hip *.c *.h
    *.hpp, Makefile and include/msplit.h, in sorted path order, concatenated)."""
    import glob
    import hashlib
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    names = [os.path.basename(f) for pat in ("*.hip", "*.c", "*.h", "*.hpp") for f in glob.glob(os.path.join(csrc, pat))]
    names += ["Makefile", "../../include/msplit.h"]
    h = hashlib.sha256()
    for n in sorted(set(names)):
        with open(os.path.join(csrc, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build_digest() -> str:
    """The digest libmsplit_hip.so was built with (msp_build_source_digest)."""
    return load().msp_build_source_digest().decode()


def check(rc: int):
    if rc:
        msg = load().msp_get_last_error().decode(errors="replace")
        raise MsplitError(rc, msg)


def call(name: str, *args):
    check(getattr(load(), name)(*args))
