"""Object lifetimes across the C ABI: every object made on a context holds a reference to it
(msp_ctx_destroy drops the caller's), so objects may be destroyed after their context, in any order --
as Python's garbage collector does with the objects of a reference cycle."""
import gc

import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, LSQR, Context, DenseMat, Mat, Options, Vec

pytestmark = pytest.mark.gpu


def test_objects_outlive_their_context(ctx, oracle):
    c = Context(0)
    A = Mat.box_stencil(c, 3, 12, 10, 8)
    n = A.shape[0]
    b = Vec.from_array(c, np.ones(n))
    x = Vec(c, n)
    ksp = KSP(c)
    ksp.set_operators(A)
    ksp.set_from_options(Options("-ksp_type gmres -pc_type none -ksp_gmres_restart 10 -ksp_max_it 20 -ksp_rtol 1e-30"))
    D = DenseMat(c, n, 3)
    l = LSQR(c)
    c.destroy()                      # the caller's reference only: the objects keep the context alive
    ksp.solve(b, x)                  # still usable, on the same stream
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(n, n, rp, col, val)
    xo, ro = oracle.gmres(O, np.ones(n), restart=10, max_it=20, rtol=1e-30, reduce_mode=oracle.REDUCE_DBR)
    assert np.array_equal(x.get_array(), xo)
    for o in (x, A, l, ksp, D, b):   # the last one frees the context
        o.destroy()


def test_reference_cycle_with_context_collected(ctx):
    """A cycle holding a context and its objects: the collector finalises them in an arbitrary order."""
    class Holder:
        pass
    for _ in range(3):
        h = Holder()
        h.c = Context(0)
        h.v = [Vec.from_array(h.c, np.arange(1000.0)) for _ in range(4)]
        h.A = Mat.box_stencil(h.c, 3, 8, 8, 8)
        h.self = h                   # the cycle
        del h
        gc.collect()
    v = Vec.from_array(ctx, np.ones(10))
    assert v.norm() == np.sqrt(10.0)
