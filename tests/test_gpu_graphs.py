"""HIP-graph replay of GMRES restart cycles (ksp_gmres.c run_cycle).

A captured cycle must give exactly the eager enqueue's results, across
repeated solves, different x vectors and cycle lengths, and after the
operator's storage changes (the cache key holds the matrix version)."""
import os

import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Mat, Options, Vec

pytestmark = pytest.mark.gpu


def _solve(ctx, A, b, x, opts):
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options(opts + " -pc_type none"))
    ksp.solve(b, x)
    return ksp


def _run(ctx, graphs: bool):
    os.environ["MSPLIT_GRAPHS"] = "1" if graphs else "0"
    try:
        A = Mat.box_stencil(ctx, 3, 18, 14, 10)
        n = A.shape[0]
        ones, b = Vec(ctx, n), Vec(ctx, n)
        ones.set(1.0)
        A.mult(ones, b)
        out = []
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options("-ksp_gmres_restart 30 -ksp_max_it 75 -ksp_rtol 1e-14 -pc_type none"))
        xs = [Vec(ctx, n), Vec(ctx, n)]
        for rep in range(3):                      # cycles of 30, 30, 15; two x vectors; a storage switch
            x = xs[rep % 2]
            if rep == 2:
                A.set_storage("csr")
            ksp.solve(b, x)
            out.append((ksp.get_iteration_number(), ksp.get_residual_history().copy(), x.get_array()))
        A.set_storage("dv")
        ksp.set_initial_guess_nonzero(True)       # warm start from the last x: KSPInitialResidual path
        ksp.solve(b, xs[0])
        out.append((ksp.get_iteration_number(), ksp.get_residual_history().copy(), xs[0].get_array()))
        return out
    finally:
        os.environ.pop("MSPLIT_GRAPHS", None)


def test_graph_cycles_equal_eager(ctx, oracle):
    eager = _run(ctx, False)
    graph = _run(ctx, True)
    for (ie, he, xe), (ig, hg, xg) in zip(eager, graph):
        assert ie == ig
        assert np.array_equal(he, hg)
        assert np.array_equal(xe, xg)
    # and the first solve is the oracle's
    Ao = oracle.poisson3d_rows(18, 14, 10, 0, 10)
    bo = Ao.mult(np.ones(18 * 14 * 10))
    xo, ro = oracle.gmres(Ao, bo, restart=30, max_it=75, rtol=1e-14, reduce_mode=oracle.REDUCE_DBR)
    assert graph[0][0] == ro["its"]
    assert np.array_equal(graph[0][1], ro["hist"])
    assert np.array_equal(graph[0][2], xo)


def test_graphs_off_under_timing(ctx):
    """Per-kernel timing needs eager launches: with timing on the solve still runs (eagerly) and the
    kernel statistics see every Arnoldi step."""
    A = Mat.box_stencil(ctx, 3, 12, 12, 12)
    n = A.shape[0]
    ones, b, x = Vec(ctx, n), Vec(ctx, n), Vec(ctx, n)
    ones.set(1.0)
    A.mult(ones, b)
    ctx.set_timing(True)
    ctx.reset_kernel_stats()
    try:
        ksp = _solve(ctx, A, b, x, "-ksp_gmres_restart 10 -ksp_max_it 20 -ksp_rtol 1e-30")
        st = ctx.kernel_stats()
    finally:
        ctx.set_timing(False)
    assert ksp.get_iteration_number() == 20
    # VecMDot runs alone or fused with the MatMult before it (box stencils: k_box_spmv_mdot[_march])
    assert st["mdot"]["launches"] + st["spmvdot"]["launches"] >= 20 and st["maxpy"]["launches"] >= 20


def test_graph_recaptured_after_partial_buffer_grows(ctx):
    """A captured cycle points at the context's DBR partial buffer; work on a larger vector reallocates it,
    and the next solve must capture again (not replay into the freed buffer)."""
    def solve_twice(graphs):
        os.environ["MSPLIT_GRAPHS"] = "1" if graphs else "0"
        try:
            A = Mat.box_stencil(ctx, 3, 16, 16, 16)
            n = A.shape[0]
            ones, b, x = Vec(ctx, n), Vec(ctx, n), Vec(ctx, n)
            ones.set(1.0)
            A.mult(ones, b)
            ksp = _solve(ctx, A, b, x, "-ksp_gmres_restart 20 -ksp_max_it 40 -ksp_rtol 1e-30")
            big = Vec(ctx, 64 * n)                  # its norm needs a larger partial buffer
            big.set(0.5)
            big.norm()
            ksp.solve(b, x)
            return ksp.get_residual_history().copy(), x.get_array()
        finally:
            os.environ.pop("MSPLIT_GRAPHS", None)
    he, xe = solve_twice(False)
    hg, xg = solve_twice(True)
    assert np.array_equal(he, hg) and np.array_equal(xe, xg)


@pytest.mark.parametrize("restart,max_it", [(30, 75), (7, 40)])
def test_gmres_with_matmult_in_cgs_kernels_bitwise(ctx, oracle, restart, max_it):
    """MSK_TUNE_GM_OPFUSE (65536): W = A (sc VV(it)) computed inside MDot and MAXPY from the DV codes
    instead of a MatMult kernel writing it: the oracle's histories and solution, bit for bit."""
    import ctypes
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    L = _lib.load()
    L.msk_set_tuning.argtypes = [ctypes.c_int]
    L.msk_set_tuning.restype = None
    A = Mat.box_convdiff(ctx, 3, 20, 17, 13, False, False, (0.3, -0.2, 0.1))
    rp, col, val = A.get_csr()
    n = A.shape[0]
    ones, b, x = Vec(ctx, n), Vec(ctx, n), Vec(ctx, n)
    ones.set(1.0)
    A.mult(ones, b)
    try:
        L.msk_set_tuning(65536)
        ksp = _solve(ctx, A, b, x, f"-ksp_gmres_restart {restart} -ksp_max_it {max_it} -ksp_rtol 1e-13")
    finally:
        L.msk_set_tuning(0)
    Ao = oracle.Mat.from_arrays(n, n, rp, col, val)
    xo, ro = oracle.gmres(Ao, b.get_array(), restart=restart, max_it=max_it, rtol=1e-13,
                          reduce_mode=oracle.REDUCE_DBR)
    assert ksp.get_iteration_number() == ro["its"]
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(x.get_array(), xo)
