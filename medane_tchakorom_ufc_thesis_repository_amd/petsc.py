"""PETSc-style host objects over the HIP C ABI (include/msplit.h).

This mirrors the slice of PETSc 3.22.1's Mat/Vec/KSP/options API that the
reference's drivers and glue use on the inner-solve path
(src/utils/utils.c:139-168, :512-541, :943-970; drivers' PetscOptionsGet*):
same object roles, same option keys and prefixes, same error behaviour
(nonzero PETSc error numbers raise).  Every numeric operation runs in
libmsplit_hip.so on the GPU; nothing here computes on vector data.
"""
from __future__ import annotations

import ctypes as C
import shlex
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import KspOpts, LsqrOpts, MsplitError, call

PETSC_ERR_SUP = 56
PETSC_ERR_ARG_WRONG = 62


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


# --------------------------------------------------------------------- options
class Options:
    """The PETSc options database (PetscOptionsGetInt/Real/String/Bool)."""

    def __init__(self, args: Iterable[str] | str | None = None):
        self._db: dict[str, str | None] = {}
        if args is None:
            return
        toks = shlex.split(args) if isinstance(args, str) else list(args)
        i = 0
        while i < len(toks):
            t = toks[i]
            if not t.startswith("-") or _is_number(t):
                raise MsplitError(PETSC_ERR_ARG_WRONG, f"stray option value {t!r}")
            key = t.lstrip("-")
            if i + 1 < len(toks) and (not toks[i + 1].startswith("-") or _is_number(toks[i + 1])):
                self._db[key] = toks[i + 1]
                i += 2
            else:
                self._db[key] = None
                i += 1

    def set(self, key: str, value=None):
        self._db[key.lstrip("-")] = None if value is None else str(value)

    def has(self, key: str, prefix: str | None = None) -> bool:
        return ((prefix or "") + key) in self._db

    def get_string(self, key, default=None, prefix=None):
        k = (prefix or "") + key
        if k not in self._db:
            return default
        v = self._db[k]
        return default if v is None else v

    def get_int(self, key, default=None, prefix=None):
        v = self.get_string(key, None, prefix)
        return default if v is None else int(float(v)) if "e" in v.lower() else int(v)

    def get_real(self, key, default=None, prefix=None):
        v = self.get_string(key, None, prefix)
        return default if v is None else float(v)

    def get_bool(self, key, default=False, prefix=None):
        k = (prefix or "") + key
        if k not in self._db:
            return default
        v = self._db[k]
        if v is None:
            return True
        return v.lower() in ("1", "true", "yes", "on")

    def keys(self):
        return list(self._db)


def _is_number(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


# --------------------------------------------------------------------- context
class Context:
    """One GPU: device id + the HIP stream every object's work is ordered on."""

    def __init__(self, device: int = 0, stream: int | None = None, timing: bool = False):
        L = _lib.load()
        h = C.c_void_p()
        call("msp_ctx_create", device, C.c_void_p(stream) if stream else None, C.byref(h))
        self.h = h
        self.device = device
        self._L = L
        if timing:
            self.set_timing(True)

    def synchronize(self):
        call("msp_ctx_synchronize", self.h)

    REDUCTIONS = {"dbr": 0, "seq": 1}

    def set_reduction(self, mode: str):
        """Reduction order of every dot/norm/MDot on this context: "dbr" (default, the
        deterministic blocked reduction) or "seq" (PETSc's sequential order, a parity mode;
        include/msplit.h MSP_REDUCE_SEQ)."""
        call("msp_ctx_set_reduction", self.h, self.REDUCTIONS[mode])

    def get_reduction(self) -> str:
        m = C.c_int()
        call("msp_ctx_get_reduction", self.h, C.byref(m))
        return {v: k for k, v in self.REDUCTIONS.items()}[m.value]

    def set_timing(self, on: bool, every: int = 1):
        """HIP-event timing of each kernel class; every > 1 brackets one launch in `every` per class."""
        call("msp_ctx_set_timing", self.h, max(1, int(every)) if on else 0)

    def reset_kernel_stats(self):
        call("msp_ctx_reset_kernel_stats", self.h)

    def kernel_stats(self) -> dict:
        out = {}
        for name, cls in _lib.KERNEL_CLASSES.items():
            n = C.c_int64()
            ms = C.c_double()
            by = C.c_double()
            call("msp_ctx_get_kernel_stats", self.h, cls, C.byref(n), C.byref(ms), C.byref(by))
            out[name] = {"launches": n.value, "ms": ms.value, "bytes": by.value}
        return out

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_ctx_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def device_count() -> int:
    n = C.c_int()
    call("msp_get_device_count", C.byref(n))
    return n.value


# ------------------------------------------------------------------------- Vec
class Vec:
    """A device vector (VecCreate + VecSetSizes, utils.c:157-168)."""

    def __init__(self, ctx: Context, n: int, device_ptr: int | None = None):
        self.ctx = ctx
        h = C.c_void_p()
        if device_ptr is None:
            call("msp_vec_create", ctx.h, int(n), C.byref(h))
        else:
            call("msp_vec_create_with_array", ctx.h, int(n), C.c_void_p(device_ptr), C.byref(h))
        self.h = h
        self.n = int(n)

    @classmethod
    def from_array(cls, ctx: Context, a) -> "Vec":
        a = np.ascontiguousarray(a, np.float64)
        v = cls(ctx, a.size)
        v.set_values(a)
        return v

    def duplicate(self) -> "Vec":                                  # VecDuplicate
        return Vec(self.ctx, self.n)

    def get_size(self) -> int:
        return self.n

    def device_ptr(self) -> int:
        p = C.c_void_p()
        call("msp_vec_get_array", self.h, C.byref(p))
        return p.value or 0

    def set_values(self, a, offset: int = 0):                      # VecSetValues (contiguous)
        a = np.ascontiguousarray(a, np.float64)
        call("msp_vec_set_values", self.h, int(offset), a.size, _dp(a))

    def get_array(self, offset: int = 0, n: int | None = None) -> np.ndarray:  # VecGetArrayRead (copy)
        n = self.n - offset if n is None else n
        out = np.empty(n)
        call("msp_vec_get_values", self.h, int(offset), int(n), _dp(out))
        return out

    def copy_range_to(self, src_off: int, dst: "Vec", dst_off: int, n: int):
        call("msp_vec_copy_range", self.h, int(src_off), dst.h, int(dst_off), int(n))

    def set(self, alpha: float):                                   # VecSet
        call("msp_vec_set", self.h, float(alpha))

    def copy(self, y: "Vec"):                                      # VecCopy(self, y)
        call("msp_vec_copy", self.h, y.h)

    def scale(self, alpha: float):                                 # VecScale
        call("msp_vec_scale", self.h, float(alpha))

    def axpy(self, alpha: float, x: "Vec"):                        # VecAXPY(self, alpha, x)
        call("msp_vec_axpy", self.h, float(alpha), x.h)

    def aypx(self, beta: float, x: "Vec"):                         # VecAYPX(self, beta, x)
        call("msp_vec_aypx", self.h, float(beta), x.h)

    def waxpy(self, alpha: float, x: "Vec", y: "Vec"):             # VecWAXPY(self, alpha, x, y)
        call("msp_vec_waxpy", self.h, float(alpha), x.h, y.h)

    def dot(self, y: "Vec") -> float:                              # VecDot
        v = C.c_double()
        call("msp_vec_dot", self.h, y.h, C.byref(v))
        return v.value

    def norm(self) -> float:                                       # VecNorm(NORM_2)
        v = C.c_double()
        call("msp_vec_norm", self.h, C.byref(v))
        return v.value

    def normalize(self) -> float:                                  # VecNormalize
        v = C.c_double()
        call("msp_vec_normalize", self.h, C.byref(v))
        return v.value

    def mdot(self, ys: Sequence["Vec"]) -> np.ndarray:             # VecMDot
        out = np.zeros(len(ys))
        arr = (C.c_void_p * max(len(ys), 1))(*[y.h.value for y in ys])
        call("msp_vec_mdot", self.h, len(ys), arr, _dp(out))
        return out

    def maxpy(self, alpha, xs: Sequence["Vec"]):                   # VecMAXPY
        a = np.ascontiguousarray(alpha, np.float64)
        if a.size != len(xs):
            raise MsplitError(60, "VecMAXPY: len(alpha) != len(x)")
        arr = (C.c_void_p * max(len(xs), 1))(*[x.h.value for x in xs])
        call("msp_vec_maxpy", self.h, len(xs), _dp(a), arr)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_vec_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------------------- Mat
class Mat:
    """A device AIJ (CSR) matrix."""

    def __init__(self, ctx: Context, h: C.c_void_p, keep=None):
        self.ctx = ctx
        self.h = h
        self._keep = keep
        nr, nc, nnz = C.c_int32(), C.c_int32(), C.c_int64()
        call("msp_mat_get_info", h, C.byref(nr), C.byref(nc), C.byref(nnz))
        self.shape = (nr.value, nc.value)
        self.nnz = nnz.value

    @classmethod
    def from_csr(cls, ctx: Context, nrows: int, ncols: int, rowptr, col, val) -> "Mat":
        rp = np.ascontiguousarray(rowptr, np.int32)
        cl = np.ascontiguousarray(col, np.int32)
        vl = np.ascontiguousarray(val, np.float64)
        if rp.size != nrows + 1:
            raise MsplitError(60, f"rowptr has {rp.size} entries, expected {nrows + 1}")
        h = C.c_void_p()
        call("msp_mat_create_csr", ctx.h, int(nrows), int(ncols), _ip(rp), _ip(cl), _dp(vl), C.byref(h))
        return cls(ctx, h)

    @classmethod
    def from_csr_rows(cls, ctx: Context, nrows: int, ncols: int, row_ids, rowptr, col, val) -> "Mat":
        ri = np.ascontiguousarray(row_ids, np.int32)
        rp = np.ascontiguousarray(rowptr, np.int32) if len(row_ids) else np.zeros(1, np.int32)
        cl = np.ascontiguousarray(col, np.int32) if len(col) else np.zeros(1, np.int32)
        vl = np.ascontiguousarray(val, np.float64) if len(val) else np.zeros(1)
        h = C.c_void_p()
        call("msp_mat_create_csr_rows", ctx.h, int(nrows), int(ncols), int(ri.size), _ip(ri), _ip(rp), _ip(cl),
             _dp(vl), C.byref(h))
        return cls(ctx, h)

    @classmethod
    def box_stencil(cls, ctx: Context, dim: int, nx: int, ny: int, nz: int = 1) -> "Mat":
        h = C.c_void_p()
        call("msp_mat_create_box_stencil", ctx.h, int(dim), int(nx), int(ny), int(nz), C.byref(h))
        return cls(ctx, h)

    @classmethod
    def box_stencil_ext(cls, ctx: Context, dim: int, nx: int, ny: int, nz: int, lo: bool, hi: bool) -> "Mat":
        """Block rows with their coupling to the neighbour plane below/above kept as
        extra columns ([plane below | own | plane above]): the operator of R = A S."""
        h = C.c_void_p()
        call("msp_mat_create_box_stencil_ext", ctx.h, int(dim), int(nx), int(ny), int(nz), 1 if lo else 0,
             1 if hi else 0, C.byref(h))
        return cls(ctx, h)

    @classmethod
    def box_convdiff(cls, ctx: Context, dim: int, nx: int, ny: int, nz: int, lo: bool, hi: bool, peclet) -> "Mat":
        """The upwind convection-diffusion stencil (msp_mat_create_box_convdiff): BASELINE configs[4]'s operator."""
        pe = np.ascontiguousarray(peclet, np.float64)
        h = C.c_void_p()
        call("msp_mat_create_box_convdiff", ctx.h, int(dim), int(nx), int(ny), int(nz), 1 if lo else 0,
             1 if hi else 0, _dp(pe), C.byref(h))
        return cls(ctx, h)

    @classmethod
    def box_matfree(cls, ctx: Context, dim: int, nx: int, ny: int, nz: int, lo: bool = False, hi: bool = False,
                    peclet=None) -> "Mat":
        """The box operator without storage (msp_mat_create_box_matfree): bitwise the assembled one's products."""
        pe = np.ascontiguousarray(peclet if peclet is not None else (0.0, 0.0, 0.0), np.float64)
        h = C.c_void_p()
        call("msp_mat_create_box_matfree", ctx.h, int(dim), int(nx), int(ny), int(nz), 1 if lo else 0,
             1 if hi else 0, _dp(pe), C.byref(h))
        return cls(ctx, h)

    def mat_mult_dense(self, S: "DenseMat", R: "DenseMat"):        # MatMatMult(A, S, MAT_REUSE_MATRIX, &R)
        call("msp_mat_matmult_dense", self.h, S.h, R.h)

    def get_csr(self):
        rp = np.empty(self.shape[0] + 1, np.int32)
        cl = np.empty(max(self.nnz, 1), np.int32)
        vl = np.empty(max(self.nnz, 1))
        call("msp_mat_get_csr", self.h, _ip(rp), _ip(cl), _dp(vl))
        return rp, cl[: self.nnz], vl[: self.nnz]

    STORAGE = {"none": -1, "csr": 0, "dv": 1, "stencil": 2}

    def set_storage(self, storage: str):
        """Entry storage in HBM (msp_mat_set_storage): 'csr', 'dv' (one byte per entry) or 'stencil' (a box
        stencil's presence byte and per-row values); same products."""
        call("msp_mat_set_storage", self.h, self.STORAGE[storage])

    def get_storage(self) -> str:
        st = C.c_int32()
        nd = C.c_int32()
        call("msp_mat_get_storage", self.h, C.byref(st), C.byref(nd))
        return {v: k for k, v in self.STORAGE.items()}[st.value]

    def spmv_kernel(self) -> str:
        """The kernel family MatMult / MatResidual / the GMRES products launch (msp_mat_get_spmv_kernel)."""
        name = C.c_char_p()
        call("msp_mat_get_spmv_kernel", self.h, C.byref(name))
        return name.value.decode()

    def release_csr(self):
        """Free the CSR arrays of a matrix in DV storage (msp_mat_release_csr); products keep working."""
        call("msp_mat_release_csr", self.h)

    def create_vecs(self):                                          # MatCreateVecs
        return Vec(self.ctx, self.shape[1]), Vec(self.ctx, self.shape[0])

    def mult(self, x: Vec, y: Vec):                                 # MatMult
        call("msp_mat_mult", self.h, x.h, y.h)

    def residual(self, b: Vec, x: Vec, r: Vec):                     # MatResidual
        call("msp_mat_residual", self.h, b.h, x.h, r.h)

    def residual_listed(self, b: Vec, x: Vec, r: Vec):
        """MatResidual over the rows a row-compressed matrix lists; r's other rows are left as they are
        (msp_mat_residual_listed: bitwise MatResidual when they already hold b)."""
        call("msp_mat_residual_listed", self.h, b.h, x.h, r.h)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_mat_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ----------------------------------------------------------------------- dense
class DenseMat:
    """Rows of a MATDENSE matrix in HBM, column-major (create_matrix_dense,
    utils.c:123-137, + MatZeroEntries)."""

    def __init__(self, ctx: Context, nrows: int, ncols: int):
        self.ctx = ctx
        h = C.c_void_p()
        call("msp_dense_create", ctx.h, int(nrows), int(ncols), C.byref(h))
        self.h = h
        self.shape = (int(nrows), int(ncols))
        lda = C.c_int64()
        call("msp_dense_get_info", h, None, None, C.byref(lda))
        self.lda = lda.value

    @classmethod
    def from_array(cls, ctx: Context, a) -> "DenseMat":
        a = np.asfortranarray(a, np.float64)
        M = cls(ctx, a.shape[0], a.shape[1])
        M.set_values(a)
        return M

    def set_values(self, a):
        a = np.asfortranarray(a, np.float64)
        if a.shape != self.shape:
            raise MsplitError(60, f"dense values of shape {a.shape}, expected {self.shape}")
        call("msp_dense_set_values", self.h, _dp(a), max(self.shape[0], 1))

    def get_values(self) -> np.ndarray:
        a = np.zeros(self.shape, order="F")
        call("msp_dense_get_values", self.h, _dp(a), max(self.shape[0], 1))
        return a

    def zero_entries(self):                                          # MatZeroEntries
        call("msp_dense_zero_entries", self.h)

    def set_column(self, j: int, row0: int, x: Vec, xoff: int = 0, n: int | None = None):
        """MatSetValuesLocal(S, n rows from row0, 1, &j, x[xoff:xoff+n])."""
        n = x.n - xoff if n is None else n
        call("msp_dense_set_column", self.h, int(j), int(row0), x.h, int(xoff), int(n))

    def mult(self, alpha: Vec, y: Vec, row0: int = 0, n: int | None = None, yoff: int = 0):   # MatMult
        n = self.shape[0] - row0 if n is None else n
        call("msp_dense_mult", self.h, alpha.h, int(row0), int(n), y.h, int(yoff))

    def mult_transpose(self, u: Vec, out: Vec):                      # MatMultTranspose (local rows)
        call("msp_dense_mult_transpose", self.h, u.h, out.h)

    def gram(self, b: Vec, out: "DenseMat"):
        """out = [R^T R | R^T b] over this block's rows (msp_dense_gram; MatTransposeMatMult + MatMultTranspose
        of outer_solver, utils.c:978-979); out is s x (s+1)."""
        call("msp_dense_gram", self.h, b.h, out.h)

    def view(self, col0: int, ncols: int) -> "DenseMat":
        """Columns [col0, col0+ncols) sharing this block's storage (msp_dense_create_view)."""
        V = DenseMat.__new__(DenseMat)
        h = C.c_void_p()
        call("msp_dense_create_view", self.h, int(col0), int(ncols), C.byref(h))
        V.ctx, V.h, V.shape, V.lda = self.ctx, h, (self.shape[0], int(ncols)), self.lda
        V._base = self                                              # keep the storage alive
        return V

    def column_vec(self, j: int) -> "Vec":
        """Column j as a Vec over this block's storage (msp_vec_create_with_array)."""
        v = Vec(self.ctx, self.shape[0], device_ptr=self.device_ptr() + 8 * self.lda * int(j))
        v._base = self
        return v

    def device_ptr(self) -> int:
        p = C.c_void_p()
        call("msp_dense_get_array", self.h, C.byref(p))
        return p.value

    @staticmethod
    def sum(parts, out: "DenseMat"):
        """out = sum of parts in order, elementwise from 0.0 (msp_dense_sum)."""
        arr = (C.c_void_p * len(parts))(*[p.h.value for p in parts])
        call("msp_dense_sum", len(parts), arr, out.h)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_dense_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------------------ comm
class Comm:
    """Cross-process all-gather used by the distributed LSQR (msp_comm)."""

    def __init__(self, h: C.c_void_p, keep=None, ctx: Context | None = None):
        self.h = h
        self._keep = keep
        self._ctx = ctx          # msp_comm synchronises the context's stream on destroy: keep it alive
        n, r = C.c_int32(), C.c_int32()
        call("msp_comm_get_size", h, C.byref(n), C.byref(r))
        self.size, self.rank = n.value, r.value

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES)()
        call("msp_comm_get_unique_id", buf)
        return bytes(buf)

    @staticmethod
    def rccl_available() -> bool:
        """librccl loads (no bootstrap thread started: the readiness test of the ranks other than 0)."""
        ok = C.c_int32(0)
        call("msp_comm_rccl_available", C.byref(ok))
        return bool(ok.value)

    @classmethod
    def rccl(cls, ctx: Context, nranks: int, rank: int, uid: bytes) -> "Comm":
        buf = (C.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        call("msp_comm_create_rccl", ctx.h, int(nranks), int(rank), buf, C.byref(h))
        return cls(h, ctx=ctx)

    @classmethod
    def host(cls, ctx: Context, nranks: int, rank: int, allgather) -> "Comm":
        """allgather(send: np.ndarray) -> np.ndarray of nranks*len(send) values."""
        def cb(_user, send, recv, count):
            try:
                a = np.ctypeslib.as_array(send, shape=(count,)).copy()
                out = np.asarray(allgather(a), np.float64).reshape(-1)
                np.ctypeslib.as_array(recv, shape=(count * nranks,))[:] = out
                return 0
            except Exception:  # reported through the C error path
                return 1
        fn = _lib.ALLGATHER_FN(cb)
        h = C.c_void_p()
        call("msp_comm_create_host", ctx.h, int(nranks), int(rank), fn, None, C.byref(h))
        return cls(h, keep=fn, ctx=ctx)

    def allgather(self, send: Vec, recv: Vec, count: int):
        call("msp_comm_allgather", self.h, send.h, recv.h, int(count))

    def exchange_neighbors(self, src: Vec, lo_src: int, hi_src: int, dst: Vec, lo_dst: int, hi_dst: int,
                           count: int):
        """comm_sync_send_and_receive for chain neighbours: planes to rank-1 / rank+1 and back."""
        call("msp_comm_exchange_neighbors", self.h, src.h, int(lo_src), int(hi_src), dst.h, int(lo_dst),
             int(hi_dst), int(count))

    def sum_ordered(self, values) -> np.ndarray:
        """Sum over ranks, in rank order (the outer-residual Allreduce)."""
        a = np.ascontiguousarray(values, np.float64).reshape(-1)
        out = np.zeros_like(a)
        call("msp_comm_sum_ordered", self.h, _dp(a), _dp(out), a.size)
        return out

    def agree(self, token: int) -> bool:
        """msp_comm_agree: every rank holds the same token (raises, on every rank, when they do not)."""
        ok = C.c_int32(0)
        call("msp_comm_agree", self.h, int(token), C.byref(ok))
        return bool(ok.value)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_comm_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------------------ LSQR
class LSQR:
    """KSPLSQR with PCNONE over row blocks of a dense operator (the reference's
    outer solver, outer_solver_norm_equation utils.c:1061-1078; options
    running_bulk_test_g5k:247-248)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        call("msp_lsqr_create", ctx.h, C.byref(h))
        self.h = h
        self.prefix = ""
        self._R = []
        self._comm = None

    def get_opts(self) -> LsqrOpts:
        o = LsqrOpts()
        call("msp_lsqr_get_opts", self.h, C.byref(o))
        return o

    def _set(self, **kw):
        o = self.get_opts()
        for k, v in kw.items():
            setattr(o, k, v)
        call("msp_lsqr_set_opts", self.h, C.byref(o))

    def set_options_prefix(self, prefix: str | None):
        self.prefix = prefix or ""

    def set_tolerances(self, rtol=None, abstol=None, divtol=None, max_it=None):
        kw = {}
        if rtol is not None:
            kw["rtol"] = float(rtol)
        if abstol is not None:
            kw["abstol"] = float(abstol)
        if divtol is not None:
            kw["divtol"] = float(divtol)
        if max_it is not None:
            kw["max_it"] = int(max_it)
        self._set(**kw)

    def set_from_options(self, opts: Options):                      # KSPSetFromOptions
        p = self.prefix
        kt = opts.get_string("ksp_type", "lsqr", p)
        if kt.lower() != "lsqr":
            raise MsplitError(PETSC_ERR_SUP, f"-{p}ksp_type {kt}: the outer solver on the MI355X path is lsqr")
        pt = opts.get_string("pc_type", "none", p)
        if pt.lower() != "none":
            raise MsplitError(PETSC_ERR_SUP, f"-{p}pc_type {pt}: only none is implemented on the MI355X path")
        nt = opts.get_string("ksp_norm_type", "unpreconditioned", p).lower()
        if nt not in ("unpreconditioned", "none"):
            raise MsplitError(PETSC_ERR_SUP, f"-{p}ksp_norm_type {nt} not supported by LSQR")
        o = self.get_opts()
        o.max_it = opts.get_int("ksp_max_it", o.max_it, p)
        o.rtol = opts.get_real("ksp_rtol", o.rtol, p)
        o.abstol = opts.get_real("ksp_atol", o.abstol, p)
        o.divtol = opts.get_real("ksp_divtol", o.divtol, p)
        if opts.has("ksp_lsqr_exact_mat_norm", p):
            o.exact_norm = 1 if opts.get_bool("ksp_lsqr_exact_mat_norm", True, p) else 0
        ct = opts.get_string("ksp_convergence_test", None, p)
        if ct is not None:
            if ct.lower() not in _lib.LSQR_CONV:
                raise MsplitError(PETSC_ERR_ARG_WRONG, f"-{p}ksp_convergence_test {ct}")
            o.conv_test = _lib.LSQR_CONV[ct.lower()]
        call("msp_lsqr_set_opts", self.h, C.byref(o))

    def set_operators(self, R: Sequence[DenseMat]):                 # KSPSetOperators(outer_ksp, R, R)
        self._R = list(R)
        arr = (C.c_void_p * len(self._R))(*[M.h.value for M in self._R])
        call("msp_lsqr_set_operators", self.h, len(self._R), arr)

    def set_comm(self, comm: Comm | None):
        self._comm = comm
        call("msp_lsqr_set_comm", self.h, comm.h if comm else None)

    def solve(self, b: Sequence[Vec], x: Vec):                      # KSPSolve(outer_ksp, b, alpha)
        arr = (C.c_void_p * len(b))(*[v.h.value for v in b])
        call("msp_lsqr_solve", self.h, arr, x.h)

    def get_iteration_number(self) -> int:
        v = C.c_int32()
        call("msp_lsqr_get_iteration_number", self.h, C.byref(v))
        return v.value

    def get_residual_norm(self) -> float:
        v = C.c_double()
        call("msp_lsqr_get_residual_norm", self.h, C.byref(v))
        return v.value

    def get_converged_reason(self) -> int:
        v = C.c_int32()
        call("msp_lsqr_get_converged_reason", self.h, C.byref(v))
        return v.value

    def get_norms(self):                                            # KSPLSQRGetNorms
        a, b = C.c_double(), C.c_double()
        call("msp_lsqr_get_norms", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def get_residual_history(self) -> np.ndarray:
        p = C.POINTER(C.c_double)()
        n = C.c_int32()
        call("msp_lsqr_get_residual_history", self.h, C.byref(p), C.byref(n))
        return np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_lsqr_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------------------- KSP
class KSP:
    """KSPGMRES with PCNONE (the reference's canonical inner solver,
    running_bulk_test_g5k:64-70; initializeKSP, utils.c:512-541)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        call("msp_ksp_create", ctx.h, C.byref(h))
        self.h = h
        self.prefix = ""
        self.A: Mat | None = None

    # -- configuration
    def get_opts(self) -> KspOpts:
        o = KspOpts()
        call("msp_ksp_get_opts", self.h, C.byref(o))
        return o

    def _set(self, **kw):
        o = self.get_opts()
        for k, v in kw.items():
            setattr(o, k, v)
        call("msp_ksp_set_opts", self.h, C.byref(o))

    def set_operators(self, A: Mat):                                # KSPSetOperators
        self.A = A
        call("msp_ksp_set_operators", self.h, A.h)

    def set_options_prefix(self, prefix: str | None):                # KSPSetOptionsPrefix
        self.prefix = prefix or ""

    def set_initial_guess_nonzero(self, flag: bool):                # KSPSetInitialGuessNonzero
        self._set(guess_nonzero=1 if flag else 0)

    def converged_default_set_uirnorm(self):                        # KSPConvergedDefaultSetUIRNorm
        self._set(uirnorm=1)

    def set_tolerances(self, rtol=None, abstol=None, divtol=None, max_it=None):   # KSPSetTolerances
        kw = {}
        if rtol is not None:
            kw["rtol"] = float(rtol)
        if abstol is not None:
            kw["abstol"] = float(abstol)
        if divtol is not None:
            kw["divtol"] = float(divtol)
        if max_it is not None:
            kw["max_it"] = int(max_it)
        self._set(**kw)

    def gmres_set_restart(self, m: int):                            # KSPGMRESSetRestart
        self._set(restart=int(m))

    def set_from_options(self, opts: Options):                      # KSPSetFromOptions
        p = self.prefix
        kt = opts.get_string("ksp_type", "gmres", p)
        if kt.lower() != "gmres":
            raise MsplitError(PETSC_ERR_SUP, f"-{p}ksp_type {kt}: only gmres is implemented on the MI355X path")
        pt = opts.get_string("pc_type", "none", p)
        if pt.lower() != "none":
            raise MsplitError(PETSC_ERR_SUP, f"-{p}pc_type {pt}: only none is implemented on the MI355X path")
        if opts.has("ksp_gmres_modifiedgramschmidt", p):
            raise MsplitError(PETSC_ERR_SUP, "modified Gram-Schmidt is not implemented (CGS only)")
        rt = opts.get_string("ksp_gmres_cgs_refinement_type", "refine_never", p)
        if rt.lower() != "refine_never":
            raise MsplitError(PETSC_ERR_SUP, f"CGS refinement {rt} not implemented (REFINE_NEVER only)")
        nt = opts.get_string("ksp_norm_type", "preconditioned", p).lower()
        if nt not in ("preconditioned", "unpreconditioned"):
            raise MsplitError(PETSC_ERR_SUP, f"-{p}ksp_norm_type {nt} not supported by GMRES")
        o = self.get_opts()
        o.restart = opts.get_int("ksp_gmres_restart", o.restart, p)
        o.max_it = opts.get_int("ksp_max_it", o.max_it, p)
        o.rtol = opts.get_real("ksp_rtol", o.rtol, p)
        o.abstol = opts.get_real("ksp_atol", o.abstol, p)
        o.divtol = opts.get_real("ksp_divtol", o.divtol, p)
        o.haptol = opts.get_real("ksp_gmres_haptol", o.haptol, p)
        o.breakdowntol = opts.get_real("ksp_gmres_breakdown_tolerance", o.breakdowntol, p)
        if opts.get_bool("ksp_converged_use_initial_residual_norm", False, p):
            o.uirnorm = 1
        if opts.has("ksp_initial_guess_nonzero", p):
            o.guess_nonzero = 1 if opts.get_bool("ksp_initial_guess_nonzero", False, p) else 0
        call("msp_ksp_set_opts", self.h, C.byref(o))

    def set_up(self):
        call("msp_ksp_set_up", self.h)

    # -- solve
    def solve(self, b: Vec, x: Vec):                                # KSPSolve
        call("msp_ksp_solve", self.h, b.h, x.h)

    def get_iteration_number(self) -> int:
        v = C.c_int32()
        call("msp_ksp_get_iteration_number", self.h, C.byref(v))
        return v.value

    def get_residual_norm(self) -> float:
        v = C.c_double()
        call("msp_ksp_get_residual_norm", self.h, C.byref(v))
        return v.value

    def get_converged_reason(self) -> int:
        v = C.c_int32()
        call("msp_ksp_get_converged_reason", self.h, C.byref(v))
        return v.value

    def get_residual_history(self) -> np.ndarray:
        p = C.POINTER(C.c_double)()
        n = C.c_int32()
        call("msp_ksp_get_residual_history", self.h, C.byref(p), C.byref(n))
        return np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_ksp_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------ async messages
class AsyncMessages:
    """Newest-value message slots in shared memory between the blocks of an
    asynchronous run (msp_amsg): the reference's MPI Isend / Iprobe-drain layer
    (comm.c:455-554, conv_detection_prime.c)."""

    DATA, PARTIAL_CV, VERIFICATION, RESPONSE, VERDICT = range(5)

    def __init__(self, name: str, nranks: int, rank: int, data_cap: int, owner: bool):
        h = C.c_void_p()
        call("msp_amsg_create", name.encode(), int(nranks), int(rank), int(data_cap), 1 if owner else 0, C.byref(h))
        self.h = h
        self.rank = rank
        self.nranks = nranks

    def attached(self) -> int:
        n = C.c_int32()
        call("msp_amsg_attached", self.h, C.byref(n))
        return n.value

    def send(self, dst: int, kind: int, ints, data=None):
        iv = np.ascontiguousarray(ints, np.int32)
        if data is None:
            call("msp_amsg_send", self.h, int(dst), int(kind), _ip(iv), iv.size, None, 0)
        else:
            d = np.ascontiguousarray(data, np.float64)
            call("msp_amsg_send", self.h, int(dst), int(kind), _ip(iv), iv.size, _dp(d), d.size)

    def recv(self, src: int, kind: int, nints: int, cap: int = 0):
        """(got, ints, data): the newest message of (src, kind) not taken yet."""
        iv = np.zeros(max(nints, 1), np.int32)
        d = np.zeros(max(cap, 1))
        n = C.c_int64()
        got = C.c_int32()
        call("msp_amsg_recv", self.h, int(src), int(kind), _ip(iv), int(nints), _dp(d), int(cap), C.byref(n),
             C.byref(got))
        return bool(got.value), iv[:nints].tolist(), d[:n.value] if got.value else None

    def send_vec(self, dst: int, ints, v: Vec, off: int, n: int):
        iv = np.ascontiguousarray(ints, np.int32)
        call("msp_amsg_send_vec", self.h, int(dst), _ip(iv), iv.size, v.h, int(off), int(n))

    def enable_device(self, ctx: Context):
        """Device slots: planes stay in the sender's HBM (HIP IPC), received by peer copy over xGMI."""
        call("msp_amsg_enable_device", self.h, ctx.h)
        self._ctx = ctx

    def close_peers(self):
        call("msp_amsg_close_peers", self.h)

    def stats(self) -> tuple:
        """(sends posted, sends skipped) on the device slots: a send is skipped while its previous copy is not yet
        published or the receiver still reads the free buffer (comm_async_test_and_send_prime's MPI_Test)."""
        a, b = C.c_int64(), C.c_int64()
        call("msp_amsg_get_stats", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def discard_pending(self) -> tuple:
        """comm_discard_pending_messages + the MPI_Cancel of pending sends at the end of a run
        (AMAM-global_prime.c:522-572): (messages discarded unread, own sends still in flight, completed)."""
        a, b = C.c_int64(), C.c_int64()
        call("msp_amsg_discard_pending", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def link_info(self, src: int) -> list:
        """Diagnostics: [data pub, data claim, data seen, partial-CV seq, partial-CV seen, verdict seq, src's slots
        opened, ranks attached] of the link src -> this rank."""
        v = np.zeros(8, np.int64)
        call("msp_amsg_get_link_info", self.h, int(src), v.ctypes.data_as(C.POINTER(C.c_int64)), 8)
        return v.tolist()

    def recv_vec(self, src: int, nints: int, v: Vec, off: int, cap: int):
        iv = np.zeros(max(nints, 1), np.int32)
        n = C.c_int64()
        got = C.c_int32()
        call("msp_amsg_recv_vec", self.h, int(src), _ip(iv), int(nints), v.h, int(off), int(cap), C.byref(n),
             C.byref(got))
        return bool(got.value), iv[:nints].tolist(), n.value

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_amsg_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class AsyncBroadcast:
    """Newest-value broadcast of each block's rows of R in shared memory
    (msp_abcast): comm_async_test_and_send_min / comm_async_probe_and_receive_min
    (comm.c:288-351) as AMAM-global uses them."""

    def __init__(self, name: str, nranks: int, rank: int, cap: int, owner: bool):
        h = C.c_void_p()
        call("msp_abcast_create", name.encode(), int(nranks), int(rank), int(cap), 1 if owner else 0, C.byref(h))
        self.h = h
        self.rank = rank
        self.nranks = nranks

    def publish(self, data: np.ndarray) -> bool:
        """Host block (nrows x ncols, column-major); False = the previous send is still being read."""
        d = np.asfortranarray(data, np.float64)
        nrows, ncols = d.shape
        ok = C.c_int32()
        call("msp_abcast_publish", self.h, _dp(d), int(nrows), int(ncols), int(max(nrows, 1)), C.byref(ok))
        return bool(ok.value)

    def fetch(self, src: int, out: np.ndarray) -> bool:
        """Copy src's newest block into out (Fortran-ordered float64) if it is newer than the last one taken."""
        if not (out.flags.f_contiguous and out.dtype == np.float64):
            raise ValueError("out must be a Fortran-ordered float64 array")
        nrows, ncols = out.shape
        got = C.c_int32()
        call("msp_abcast_fetch", self.h, int(src), _dp(out), int(nrows), int(ncols), int(max(nrows, 1)),
             C.byref(got))
        return bool(got.value)

    def enable_device(self, ctx: Context, nbuf: int = 0) -> int:
        """Device buffers: published blocks stay in the sender's HBM (HIP IPC); nbuf 1 halves their HBM, 0 lets
        the library choose (two while a quarter of the HBM stays free after them).  Returns the count in use."""
        call("msp_abcast_enable_device", self.h, ctx.h, int(nbuf))
        self._ctx = ctx
        n = C.c_int32()
        call("msp_abcast_get_nbuf", self.h, C.byref(n))
        return n.value

    def close_peers(self):
        call("msp_abcast_close_peers", self.h)

    def stats(self) -> tuple:
        """(device publishes enqueued, skipped: previous copy unpublished or the buffer still read)."""
        a, b = C.c_int64(), C.c_int64()
        call("msp_abcast_get_stats", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def discard_pending(self) -> tuple:
        """(newer R blocks discarded unread, own publish still in flight, completed) at the end of a run."""
        a, b = C.c_int64(), C.c_int64()
        call("msp_abcast_discard_pending", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def publish_dense(self, D: "DenseMat") -> bool:
        ok = C.c_int32()
        call("msp_abcast_publish_dense", self.h, D.h, C.byref(ok))
        return bool(ok.value)

    def fetch_dense(self, src: int, D: "DenseMat") -> bool:
        got = C.c_int32()
        call("msp_abcast_fetch_dense", self.h, int(src), D.h, C.byref(got))
        return bool(got.value)

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_abcast_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class ConvDetection:
    """The reference's decentralised convergence detection (msp_cvd,
    conv_detection_prime.c) for one block root."""

    NORMAL, WAIT4VERIFICATION, VERIFICATION, FINISHED = range(4)

    def __init__(self, am: AsyncMessages, rank: int, neighbors, dependencies, strict: bool = False):
        nb = np.ascontiguousarray(neighbors, np.int32)
        dp = np.ascontiguousarray(dependencies, np.int32)
        h = C.c_void_p()
        call("msp_cvd_create", am.h, int(rank), nb.size, _ip(nb) if nb.size else None, dp.size,
             _ip(dp) if dp.size else None, 1 if strict else 0, C.byref(h))
        self.h = h
        self._am = am

    def data_received(self, d: int, tag: int, iteration: int) -> bool:
        acc = C.c_int32()
        call("msp_cvd_data_received", self.h, int(d), int(tag), int(iteration), C.byref(acc))
        return bool(acc.value)

    def step(self, under_threshold: bool):
        call("msp_cvd_step", self.h, 1 if under_threshold else 0)

    def state(self):
        s, t = C.c_int32(), C.c_int32()
        call("msp_cvd_get_state", self.h, C.byref(s), C.byref(t))
        return s.value, t.value

    def info(self) -> dict:
        v = np.zeros(8, np.int32)
        call("msp_cvd_get_info", self.h, _ip(v), 8)
        keys = ("state", "phase_tag", "elected", "local_cv", "pp_begin", "pp_end", "nb_not_recvd", "partial_cv_sent")
        return dict(zip(keys, v.tolist()))

    def destroy(self):
        if getattr(self, "h", None) and self.h.value:
            call("msp_cvd_destroy", C.byref(self.h))

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
