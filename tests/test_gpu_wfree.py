"""The W-free GMRES step for box stencils (KSPGMRESCycle's MatMult + CGS block, gmres.c:143-156 in PETSc 3.22.1,
driven by the reference's inner_solver, utils.c:512-541).

The fused MatMult+MDot (k_box_spmv_mdot_march) no longer stores W = A (sc VV(it)); the CGS VecMAXPY after it
(k_box_maxpy_march) recomputes W for its rows on the same chunk tiles and takes VV(it) -- the basis' last vector --
from its march registers.  Every result must be bitwise the stored-W step's (msk_set_gm_wfree(0)) and the DBR
oracle's: the iteration count, every residual-history entry and the solution, over every MAXPY grouping
(nv & 3 leading vectors, then groups of four; nv <= 3 in one group), ragged and single-plane z tiles, both
workgroup orders, eager and captured cycles, Poisson and convection-diffusion.
"""
import ctypes
from contextlib import contextmanager

import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd import _lib
from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Mat, Options, Vec

pytestmark = pytest.mark.gpu

SEED = 20261017


def _L():
    L = _lib.load()
    L.msk_set_gm_wfree.argtypes = [ctypes.c_int]
    L.msk_set_gm_wfree.restype = None
    L.msk_get_gm_wfree.restype = ctypes.c_int
    L.msk_box_wfree_fits.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    L.msk_box_wfree_fits.restype = ctypes.c_int
    return L


@contextmanager
def wfree(on):
    L = _L()
    old = L.msk_get_gm_wfree()
    L.msk_set_gm_wfree(on)
    try:
        yield
    finally:
        L.msk_set_gm_wfree(old)


def _solve(ctx, A, b, restart, max_it):
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                 f"-ksp_gmres_restart {restart} -ksp_max_it {max_it} -ksp_rtol 1e-30"))
    x = Vec(ctx, A.shape[0])
    ksp.solve(Vec.from_array(ctx, b), x)
    return ksp.get_iteration_number(), ksp.get_residual_history(), x.get_array()


def _check(ctx, oracle, A, b, restart, max_it, timing=False):
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    ctx.set_timing(timing)
    try:
        with wfree(1):
            its1, h1, x1 = _solve(ctx, A, b, restart, max_it)
        with wfree(0):
            its0, h0, x0 = _solve(ctx, A, b, restart, max_it)
    finally:
        ctx.set_timing(False)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, restart=restart, max_it=max_it,
                          rtol=1e-30)
    assert its1 == its0 == ro["its"]
    assert np.array_equal(h1, ro["hist"]) and np.array_equal(h0, ro["hist"])
    assert np.array_equal(x1, xo) and np.array_equal(x0, xo)


@pytest.mark.parametrize("shape", [(64, 64, 33), (256, 16, 7), (128, 32, 5), (2048, 2, 3), (64, 64, 1),
                                   (512, 8, 2), (256, 256, 2)])
@pytest.mark.parametrize("peclet", [None, (0.5, -0.25, 0.3)])
def test_wfree_gmres_bitwise(ctx, oracle, shape, peclet):
    """GMRES(30) over 45 iterations (a full cycle of every nv 1..30, then a second one): the W-free step is
    taken (msk_box_wfree_fits) and equals the stored-W step and the oracle bit for bit."""
    nx, ny, nz = shape
    A = Mat.box_stencil(ctx, 3, nx, ny, nz) if peclet is None else Mat.box_convdiff(ctx, 3, nx, ny, nz, False,
                                                                                    False, peclet)
    n = A.shape[0]
    assert _L().msk_box_wfree_fits(nx, nx * ny, n, 0) == 1
    b = np.random.default_rng(SEED).uniform(-1, 1, n)
    _check(ctx, oracle, A, b, 30, 45)


@pytest.mark.parametrize("restart", [1, 2, 3, 4, 5, 6, 7, 8, 9, 13, 32, 33])
def test_wfree_every_group_shape(ctx, oracle, restart):
    """Restarts 1..9 and 13 give every leading-group size (nv & 3 = 0..3) with and without groups of four, and
    nv <= 3 where x is in the leading group; 32 is the largest the fused kernels take, 33 falls back to the
    separate kernels (W stored) -- all bitwise the oracle."""
    A = Mat.box_stencil(ctx, 3, 64, 64, 9)
    b = np.random.default_rng(SEED + restart).uniform(-1, 1, A.shape[0])
    _check(ctx, oracle, A, b, restart, 3 * restart + 2)


@pytest.mark.parametrize("timing", [False, True])
def test_wfree_eager_and_captured(ctx, oracle, timing):
    """Per-kernel timing on: eager launches; off: the cycle is captured once and replayed as a HIP graph.  The
    switch re-keys the captured cycles (msk_set_gm_wfree bumps the shape epoch), so both settings run their own
    kernels in one process."""
    A = Mat.box_stencil(ctx, 3, 128, 64, 6)
    b = np.random.default_rng(SEED).uniform(-1, 1, A.shape[0])
    _check(ctx, oracle, A, b, 30, 70, timing=timing)


@pytest.mark.parametrize("shape", [(100, 30, 9), (37, 11, 9), (256, 40, 7), (2, 3, 50), (300, 7, 5), (2048, 3, 2),
                                   (256, 64, 0), (100, 37, 0), (33, 7, 0), (512, 40, 0), (300, 1, 0)])
@pytest.mark.parametrize("peclet", [None, (0.5, -0.25, 0.3)])
def test_wfree_unmarched_forms(ctx, oracle, shape, peclet):
    """Where the fused kernel does not march -- planes that do not hold whole 4096-row chunks, a ragged last chunk
    (n % 4096 != 0, incl. a single ragged chunk), and 2D boxes (nz = 0 here: nx x ny, marched as nx x 1 x ny) --
    the W-free MAXPY takes one chunk per workgroup (k_box_maxpy) and still equals the stored-W step and the oracle
    bit for bit."""
    nx, ny, nz = shape
    dim = 2 if nz == 0 else 3
    if peclet is not None and dim == 2:
        peclet = (peclet[0], peclet[1], 0.0)
    if dim == 3:
        A = Mat.box_stencil(ctx, 3, nx, ny, nz) if peclet is None else Mat.box_convdiff(ctx, 3, nx, ny, nz, False,
                                                                                        False, peclet)
    else:
        A = Mat.box_stencil(ctx, 2, nx, ny) if peclet is None else Mat.box_convdiff(ctx, 2, nx, ny, 1, False, False,
                                                                                    peclet)
    n = A.shape[0]
    assert _L().msk_box_wfree_fits(nx, nx * (ny if dim == 3 else 1), n, 1 if dim == 2 else 0) == 1
    _check(ctx, oracle, A, np.random.default_rng(SEED).uniform(-1, 1, n), 12, 30)


def test_wfree_not_taken(ctx, oracle):
    """Boxes the fused kernel does not take (nx > 2048, or one-wide lines) keep the stored-W path; with the
    switch off no box takes it."""
    L = _L()
    assert L.msk_box_wfree_fits(4096, 4096 * 2, 4096 * 2 * 3, 0) == 0
    assert L.msk_box_wfree_fits(1, 50, 50 * 7, 0) == 0
    with wfree(0):
        assert L.msk_box_wfree_fits(256, 256 * 16, 256 * 16 * 4, 0) == 0
    A = Mat.box_stencil(ctx, 3, 1, 30, 20)
    _check(ctx, oracle, A, np.random.default_rng(SEED).uniform(-1, 1, A.shape[0]), 30, 40)


def test_wfree_maxpy_class_bytes(ctx):
    """With timing on, the MAXPY class counts the W-free kernel's bytes (presence byte, x once, nv - 1 basis
    vectors, wout) and the fused class no W store: 8 n (nv + 1) + n and 8 n nv (x from the march, nv - 1 streamed
    basis vectors, no W) + n per Arnoldi step."""
    A = Mat.box_stencil(ctx, 3, 64, 64, 8)
    n = A.shape[0]
    b = Vec.from_array(ctx, np.random.default_rng(SEED).uniform(-1, 1, n))
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options("-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                 "-ksp_gmres_restart 10 -ksp_max_it 10 -ksp_rtol 1e-30"))
    x = Vec(ctx, n)
    ctx.reset_kernel_stats()
    ctx.set_timing(True)
    try:
        with wfree(1):
            ksp.solve(b, x)
    finally:
        ctx.set_timing(False)
    st = ctx.kernel_stats()
    # Arnoldi steps nv = 1..10; the MAXPY class also holds BuildSoln (8 n (10 + 2))
    maxpy = sum(8.0 * n * (nv + 1) + n for nv in range(1, 11)) + 8.0 * n * 12
    spmvdot = sum(8.0 * n * nv + n for nv in range(1, 11))
    assert st["maxpy"]["bytes"] == pytest.approx(maxpy, rel=1e-12)
    assert st["spmvdot"]["bytes"] == pytest.approx(spmvdot, rel=1e-12)


@pytest.mark.parametrize("alt", ["1", "0"])
@pytest.mark.parametrize("shape", [(64, 64, 33), (128, 32, 5), (256, 16, 7), (64, 64, 8)])
def test_fused_march_direction_bitwise(ctx, oracle, shape, alt, monkeypatch):
    """Round 6: odd plane groups of the fused MatMult+MDot march down (MSPLIT_BOXMDOT_ALT, default on), so that the
    boundary planes two groups share are read by both at the same moment (the second time from the L2).  Both
    orders give the stored-W step's and the oracle's bits: the march order changes no chunk's arithmetic."""
    monkeypatch.setenv("MSPLIT_BOXMDOT_ALT", alt)  # 1: alternating, 0: up only
    nx, ny, nz = shape
    A = Mat.box_stencil(ctx, 3, nx, ny, nz)
    b = np.random.default_rng(SEED + nz).uniform(-1, 1, A.shape[0])
    _check(ctx, oracle, A, b, 30, 45)
