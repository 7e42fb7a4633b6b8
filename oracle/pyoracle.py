"""ctypes view of the CPU oracle (oracle/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  The functions
mirror oracle/oracle.h; see that header for the reference file:line each one
restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborc.so")

REDUCE_SEQ = 0
REDUCE_DBR = 1
REDUCE_MT = 2      # PETSc's MPI dot order, one rank per thread (CPU-baseline timing)
DBR_CHUNK = 256 * 2 * 8

REASONS = {
    0: "CONVERGED_ITERATING", 1: "CONVERGED_RTOL_NORMAL", 2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL",
    4: "CONVERGED_ITS", 9: "CONVERGED_ATOL_NORMAL",
    7: "CONVERGED_HAPPY_BREAKDOWN", -2: "DIVERGED_NULL", -3: "DIVERGED_ITS",
    -4: "DIVERGED_DTOL", -5: "DIVERGED_BREAKDOWN", -9: "DIVERGED_NANORINF",
}


class CSR(C.Structure):
    _fields_ = [("nrows", C.c_int32), ("ncols", C.c_int32), ("nnz", C.c_int64),
                ("rowptr", C.POINTER(C.c_int32)), ("col", C.POINTER(C.c_int32)),
                ("val", C.POINTER(C.c_double))]


class GmresOpts(C.Structure):
    _fields_ = [("restart", C.c_int), ("max_it", C.c_int), ("rtol", C.c_double),
                ("abstol", C.c_double), ("divtol", C.c_double), ("haptol", C.c_double),
                ("breakdowntol", C.c_double), ("uirnorm", C.c_int), ("guess_nonzero", C.c_int),
                ("reduce_mode", C.c_int)]


class GmresResult(C.Structure):
    _fields_ = [("its", C.c_int), ("reason", C.c_int), ("rnorm", C.c_double), ("nhist", C.c_int)]


class SMProblem(C.Structure):
    _fields_ = [("dim", C.c_int), ("nx", C.c_int), ("ny", C.c_int), ("nz", C.c_int), ("nb", C.c_int),
                ("rtol", C.c_double), ("atol", C.c_double), ("max_outer", C.c_int),
                ("peclet", C.c_double * 3)]


class SMResult(C.Structure):
    _fields_ = [("outer_its", C.c_int), ("norm0", C.c_double), ("final_norm", C.c_double),
                ("error", C.c_double), ("total_inner_its", C.c_int64)]


class LsqrOpts(C.Structure):
    _fields_ = [("max_it", C.c_int), ("rtol", C.c_double), ("abstol", C.c_double), ("divtol", C.c_double),
                ("exact_norm", C.c_int), ("conv_test", C.c_int), ("reduce_mode", C.c_int), ("onepass", C.c_int)]


class LsqrResult(C.Structure):
    _fields_ = [("its", C.c_int), ("reason", C.c_int), ("rnorm", C.c_double), ("arnorm", C.c_double),
                ("anorm", C.c_double), ("nhist", C.c_int)]


class SMSMProblem(C.Structure):
    _fields_ = [("dim", C.c_int), ("nx", C.c_int), ("ny", C.c_int), ("nz", C.c_int), ("nb", C.c_int),
                ("s", C.c_int), ("rtol", C.c_double), ("atol", C.c_double), ("max_outer", C.c_int),
                ("peclet", C.c_double * 3), ("lean", C.c_int)]


CONV_DEFAULT, CONV_LSQR, CONV_SKIP = 0, 1, 2

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        dp = P(C.c_double)
        L.orc_csr_free.argtypes = [P(CSR)]
        for name in ("orc_poisson3d_rows",):
            getattr(L, name).argtypes = [C.c_int] * 5 + [P(CSR)]
        L.orc_poisson2d_rows.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int64, P(CSR)]
        L.orc_poisson2d_complete.argtypes = [C.c_int, C.c_int, P(CSR)]
        L.orc_convdiff_rows.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int64, dp, P(CSR)]
        L.orc_split.argtypes = [P(CSR), C.c_int64, C.c_int64, P(CSR), P(CSR)]
        L.orc_spmv.argtypes = [P(CSR), dp, dp]
        L.orc_residual.argtypes = [P(CSR), dp, dp, dp]
        L.orc_dot.argtypes = [C.c_int, C.c_int64, dp, dp]
        L.orc_dot.restype = C.c_double
        L.orc_norm2.argtypes = [C.c_int, C.c_int64, dp]
        L.orc_norm2.restype = C.c_double
        L.orc_mdot.argtypes = [C.c_int, C.c_int64, C.c_int, dp, P(dp), dp]
        L.orc_maxpy.argtypes = [C.c_int64, C.c_int, dp, P(dp), dp]
        L.orc_gmres_default_opts.argtypes = [P(GmresOpts)]
        L.orc_gmres_solve.argtypes = [P(CSR), dp, dp, P(GmresOpts), P(GmresResult), dp, C.c_int]
        L.orc_final_residual_norm.argtypes = [C.c_int, C.c_int, P(P(CSR)), dp, P(dp)]
        L.orc_final_residual_norm.restype = C.c_double
        L.orc_sm_solve.argtypes = [P(SMProblem), P(GmresOpts), P(SMResult), dp, C.c_int, P(C.c_int), dp]
        L.orc_lsqr_default_opts.argtypes = [P(LsqrOpts)]
        L.orc_lsqr_solve.argtypes = [C.c_int, P(C.c_int64), C.c_int, P(dp), P(C.c_int64), P(dp), dp,
                                     P(LsqrOpts), P(LsqrResult), dp, C.c_int]
        L.orc_dense_mult.argtypes = [C.c_int64, C.c_int, dp, C.c_int64, dp, dp]
        L.orc_dense_gram.argtypes = [C.c_int, C.c_int64, C.c_int, dp, C.c_int64, dp, dp, C.c_int64]
        L.orc_smsm_solve.argtypes = [P(SMSMProblem), P(GmresOpts), P(LsqrOpts), P(SMResult), dp, C.c_int,
                                     P(C.c_int), P(C.c_int), P(C.c_int), dp]
        _lib = L
    return _lib


def set_threads(threads: int):
    """OpenMP threads of the element-wise loops and of REDUCE_MT dots (CPU baseline)."""
    lib().orc_set_threads(int(threads))


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Mat:
    """A CSR matrix owned by the oracle library, with numpy views."""

    def __init__(self, csr: CSR):
        self.csr = csr

    @classmethod
    def from_arrays(cls, nrows, ncols, rowptr, col, val):
        m = cls.__new__(cls)
        m._keep = (np.ascontiguousarray(rowptr, np.int32), np.ascontiguousarray(col, np.int32),
                   np.ascontiguousarray(val, np.float64))
        c = CSR()
        c.nrows, c.ncols, c.nnz = nrows, ncols, len(m._keep[1])
        c.rowptr = m._keep[0].ctypes.data_as(C.POINTER(C.c_int32))
        c.col = m._keep[1].ctypes.data_as(C.POINTER(C.c_int32))
        c.val = m._keep[2].ctypes.data_as(C.POINTER(C.c_double))
        m.csr = c
        return m

    def __del__(self):
        if getattr(self, "_keep", None) is None and getattr(self, "csr", None) is not None and _lib is not None:
            _lib.orc_csr_free(C.byref(self.csr))
            self.csr = None

    @property
    def shape(self):
        return (self.csr.nrows, self.csr.ncols)

    @property
    def nnz(self):
        return self.csr.nnz

    def arrays(self):
        n, nnz = self.csr.nrows, self.csr.nnz
        rp = np.ctypeslib.as_array(self.csr.rowptr, shape=(n + 1,)).copy()
        col = np.ctypeslib.as_array(self.csr.col, shape=(max(nnz, 1),))[:nnz].copy()
        val = np.ctypeslib.as_array(self.csr.val, shape=(max(nnz, 1),))[:nnz].copy()
        return rp, col, val

    def dense(self):
        rp, col, val = self.arrays()
        D = np.zeros(self.shape)
        for r in range(self.shape[0]):
            for k in range(rp[r], rp[r + 1]):
                D[r, col[k]] = val[k]
        return D

    def mult(self, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty(self.shape[0])
        lib().orc_spmv(C.byref(self.csr), _dp(x), _dp(y))
        return y

    def residual(self, b, x):
        b = np.ascontiguousarray(b, np.float64)
        x = np.ascontiguousarray(x, np.float64)
        r = np.empty(self.shape[0])
        lib().orc_residual(C.byref(self.csr), _dp(b), _dp(x), _dp(r))
        return r


def _check(rc, what):
    if rc:
        raise RuntimeError(f"{what} failed with code {rc}")


def poisson3d_rows(nx, ny, nz, z0, z1) -> Mat:
    c = CSR()
    _check(lib().orc_poisson3d_rows(nx, ny, nz, z0, z1, C.byref(c)), "orc_poisson3d_rows")
    return Mat(c)


def poisson2d_rows(m, n, row0, row1) -> Mat:
    c = CSR()
    _check(lib().orc_poisson2d_rows(m, n, row0, row1, C.byref(c)), "orc_poisson2d_rows")
    return Mat(c)


def poisson2d_complete(m, n) -> Mat:
    c = CSR()
    _check(lib().orc_poisson2d_complete(m, n, C.byref(c)), "orc_poisson2d_complete")
    return Mat(c)


def convdiff_rows(dim, nx, ny, nz, row0, row1, peclet) -> Mat:
    """Rows [row0,row1) of the upwind convection-diffusion operator (see oracle.h)."""
    csr = CSR()
    pe = np.ascontiguousarray(peclet, np.float64)
    _check(lib().orc_convdiff_rows(dim, nx, ny, nz if dim == 3 else 1, row0, row1, _dp(pe), C.byref(csr)),
           "orc_convdiff_rows")
    return Mat(csr)


def split(A: Mat, c0: int, c1: int):
    a, o = CSR(), CSR()
    _check(lib().orc_split(C.byref(A.csr), c0, c1, C.byref(a), C.byref(o)), "orc_split")
    return Mat(a), Mat(o)


def dot(x, y, mode=REDUCE_SEQ) -> float:
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    return lib().orc_dot(mode, len(x), _dp(x), _dp(y))


def norm2(x, mode=REDUCE_SEQ) -> float:
    x = np.ascontiguousarray(x, np.float64)
    return lib().orc_norm2(mode, len(x), _dp(x))


def mdot(w, V, mode=REDUCE_SEQ) -> np.ndarray:
    w = np.ascontiguousarray(w, np.float64)
    Vs = [np.ascontiguousarray(v, np.float64) for v in V]
    arr = (C.POINTER(C.c_double) * max(len(Vs), 1))(*[_dp(v) for v in Vs])
    out = np.zeros(len(Vs))
    lib().orc_mdot(mode, len(w), len(Vs), _dp(w), arr, _dp(out))
    return out


def maxpy(w, alpha, V) -> np.ndarray:
    w = np.array(w, np.float64, copy=True)
    Vs = [np.ascontiguousarray(v, np.float64) for v in V]
    a = np.ascontiguousarray(alpha, np.float64)
    arr = (C.POINTER(C.c_double) * max(len(Vs), 1))(*[_dp(v) for v in Vs])
    lib().orc_maxpy(len(w), len(Vs), _dp(a), arr, _dp(w))
    return w


def gmres_opts(**kw) -> GmresOpts:
    o = GmresOpts()
    lib().orc_gmres_default_opts(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise KeyError(k)
        setattr(o, k, v)
    return o


def gmres(A: Mat, b, x0=None, hist_cap=None, **opts):
    """KSPSolve with KSPGMRES semantics.  Returns (x, result-dict)."""
    o = gmres_opts(**opts)
    b = np.ascontiguousarray(b, np.float64)
    x = np.zeros(A.shape[0]) if x0 is None else np.array(x0, np.float64, copy=True)
    cap = hist_cap if hist_cap is not None else o.max_it + 2
    hist = np.zeros(max(cap, 1))
    r = GmresResult()
    _check(lib().orc_gmres_solve(C.byref(A.csr), _dp(b), _dp(x), C.byref(o), C.byref(r), _dp(hist), cap),
           "orc_gmres_solve")
    return x, {"its": r.its, "reason": r.reason, "rnorm": r.rnorm, "hist": hist[:min(r.nhist, cap)].copy()}


def final_residual_norm(Ablocks, x, bblocks, mode=REDUCE_SEQ) -> float:
    P = C.POINTER
    x = np.ascontiguousarray(x, np.float64)
    bs = [np.ascontiguousarray(b, np.float64) for b in bblocks]
    Aarr = (P(CSR) * len(Ablocks))(*[C.pointer(A.csr) for A in Ablocks])
    barr = (P(C.c_double) * len(bs))(*[_dp(b) for b in bs])
    return lib().orc_final_residual_norm(mode, len(Ablocks), Aarr, _dp(x), barr)


def sm_solve(dim, nx, ny, nz, nb, rtol, inner: dict, atol=1e-100, max_outer=10000, peclet=(0.0, 0.0, 0.0)):
    """Synchronous multisplitting over nb blocks (see oracle.h).  Returns a dict."""
    p = SMProblem(dim, nx, ny, nz if dim == 3 else 1, nb, rtol, atol, max_outer, (C.c_double * 3)(*peclet))
    o = gmres_opts(**inner)
    res = SMResult()
    cap = max_outer
    hist = np.zeros(cap)
    its = np.zeros(cap * nb, np.int32)
    N = nx * ny * (nz if dim == 3 else 1)
    x = np.zeros(N)
    _check(lib().orc_sm_solve(C.byref(p), C.byref(o), C.byref(res), _dp(hist), cap,
                              its.ctypes.data_as(C.POINTER(C.c_int)), _dp(x)), "orc_sm_solve")
    n = res.outer_its
    return {"outer_its": n, "norm0": res.norm0, "final_norm": res.final_norm, "error": res.error,
            "total_inner_its": res.total_inner_its, "hist": hist[:min(n, cap)].copy(),
            "inner_its": its[:min(n, cap) * nb].reshape(-1, nb).copy(), "x": x}


def lsqr_opts(**kw) -> LsqrOpts:
    o = LsqrOpts()
    lib().orc_lsqr_default_opts(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise KeyError(k)
        setattr(o, k, v)
    return o


def lsqr(R_blocks, b_blocks, hist_cap=None, **opts):
    """KSPSolve with KSPLSQR semantics (zero guess, PCNONE) over a dense operator
    given as row blocks (each an (n_b, s) array).  Returns (x, result-dict)."""
    o = lsqr_opts(**opts)
    P = C.POINTER
    Rs = [np.asfortranarray(R, np.float64) for R in R_blocks]
    bs = [np.ascontiguousarray(b, np.float64) for b in b_blocks]
    s = Rs[0].shape[1]
    nb = len(Rs)
    nrows = (C.c_int64 * nb)(*[R.shape[0] for R in Rs])
    lda = (C.c_int64 * nb)(*[max(R.shape[0], 1) for R in Rs])
    Rarr = (P(C.c_double) * nb)(*[_dp(R) for R in Rs])
    barr = (P(C.c_double) * nb)(*[_dp(b) for b in bs])
    x = np.zeros(s)
    cap = hist_cap if hist_cap is not None else o.max_it + 2
    hist = np.zeros(max(cap, 1))
    r = LsqrResult()
    _check(lib().orc_lsqr_solve(nb, nrows, s, Rarr, lda, barr, _dp(x), C.byref(o), C.byref(r), _dp(hist), cap),
           "orc_lsqr_solve")
    return x, {"its": r.its, "reason": r.reason, "rnorm": r.rnorm, "arnorm": r.arnorm, "anorm": r.anorm,
               "hist": hist[:min(r.nhist, cap)].copy()}


def dense_gram(R, b, mode=REDUCE_SEQ) -> np.ndarray:
    """[R^T R | R^T b] (s x (s+1)) over one block's rows (orc_dense_gram; outer_solver, utils.c:978-979)."""
    R = np.asfortranarray(R, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    n, s = R.shape
    G = np.zeros((s, s + 1), order="F")
    lib().orc_dense_gram(mode, n, s, _dp(R), max(n, 1), _dp(b), _dp(G), s)
    return G


def dense_mult(S, alpha) -> np.ndarray:
    S = np.asfortranarray(S, np.float64)
    a = np.ascontiguousarray(alpha, np.float64)
    y = np.zeros(S.shape[0])
    lib().orc_dense_mult(S.shape[0], S.shape[1], _dp(S), max(S.shape[0], 1), _dp(a), _dp(y))
    return y


def smsm_solve(dim, nx, ny, nz, nb, s, rtol, inner: dict, outer: dict, atol=1e-100, max_outer=1000,
               peclet=(0.0, 0.0, 0.0), lean=False):
    """SMSM with global minimization over nb blocks (see oracle.h).  Returns a dict.  lean (dim 3): the same
    record without assembled matrices or a stored R (the 512^3 records)."""
    p = SMSMProblem(dim, nx, ny, nz if dim == 3 else 1, nb, s, rtol, atol, max_outer, (C.c_double * 3)(*peclet),
                    1 if lean else 0)
    io = gmres_opts(**inner)
    oo = lsqr_opts(**outer)
    res = SMResult()
    cap = max_outer
    hist = np.zeros(cap)
    lits = np.zeros(cap, np.int32)
    lreason = np.zeros(cap, np.int32)
    its = np.zeros(cap * s * nb, np.int32)
    N = nx * ny * (nz if dim == 3 else 1)
    x = np.zeros(N)
    ip = C.POINTER(C.c_int)
    _check(lib().orc_smsm_solve(C.byref(p), C.byref(io), C.byref(oo), C.byref(res), _dp(hist), cap,
                                lits.ctypes.data_as(ip), lreason.ctypes.data_as(ip), its.ctypes.data_as(ip),
                                _dp(x)), "orc_smsm_solve")
    n = min(res.outer_its, cap)
    return {"outer_its": res.outer_its, "norm0": res.norm0, "final_norm": res.final_norm, "error": res.error,
            "total_inner_its": res.total_inner_its, "hist": hist[:n].copy(), "lsqr_its": lits[:n].copy(),
            "lsqr_reason": lreason[:n].copy(), "inner_its": its[:n * s * nb].reshape(n, s, nb).copy(), "x": x}
