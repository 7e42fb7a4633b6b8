"""The convection-diffusion operator (BASELINE configs[4]) on the GPU against the
oracle: on-device assembly bit for bit, then the SM and SMSM-global drivers on
the non-symmetric system bit for bit (DBR order)."""
import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd import utils
from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks, make_smsm, sm_solve, smsm_solve
from medane_tchakorom_ufc_thesis_repository_amd.petsc import Mat, Options

pytestmark = pytest.mark.gpu

PE = [(0.5, 0.25, -0.3), (-1.5, 2.0, 0.75), (0.0, 0.0, 0.0)]


@pytest.mark.parametrize("P", PE)
@pytest.mark.parametrize("dim,nx,ny,nz,nb", [(3, 6, 5, 8, 2), (3, 7, 4, 9, 3), (2, 12, 10, 1, 3)])
def test_device_assembly_is_the_oracle_operator(ctx, oracle, dim, nx, ny, nz, nb, P):
    """A_ext (block rows, [plane below | own | plane above] columns) and A_ii from
    the device assembly kernel == the oracle's rows, CSR for CSR."""
    for b in range(nb):
        L = utils.block_layout(dim, nx, ny, nz, nb, b, P)
        lo = L.plane if b > 0 else 0
        hi = L.plane if b < nb - 1 else 0
        rp, c, v = oracle.convdiff_rows(dim, nx, ny, nz, L.r0, L.r1, P).arrays()
        A = Mat.box_convdiff(ctx, *L.box, lo > 0, hi > 0, P)
        assert A.shape == (L.nrows, lo + L.nrows + hi)
        grp, gc, gv = A.get_csr()
        assert np.array_equal(grp, rp) and np.array_equal(gc, c - (L.r0 - lo)) and np.array_equal(gv, v)
        Aii = Mat.box_convdiff(ctx, *L.box, False, False, P)
        brp, bc, bv = oracle.split(oracle.convdiff_rows(dim, nx, ny, nz, L.r0, L.r1, P), L.r0, L.r1)[0].arrays()
        grp, gc, gv = Aii.get_csr()
        assert np.array_equal(grp, brp) and np.array_equal(gc, bc) and np.array_equal(gv, bv)


def test_large_device_assembly_properties(ctx):
    """A 128^3 block: row sums = the boundary defect, nnz = 7 n - 2 (faces)."""
    P = (0.5, 0.25, -0.3)
    n = 128
    A = Mat.box_convdiff(ctx, 3, n, n, n, False, False, P)
    rp, c, v = A.get_csr()
    assert rp[-1] == 7 * n ** 3 - 6 * n * n
    cf = utils.convdiff_coefs(3, P)
    assert np.count_nonzero(v == cf[3]) == n ** 3
    rows = np.repeat(np.arange(n ** 3), np.diff(rp))
    assert np.all(np.diff(c)[np.diff(rows) == 0] > 0)


@pytest.mark.parametrize("P", PE[:2])
@pytest.mark.parametrize("dim,nx,ny,nz,nb", [(3, 12, 10, 8, 1), (3, 10, 10, 12, 4), (2, 32, 32, 1, 2)])
def test_sm_convdiff_bitwise_vs_oracle(ctx, oracle, dim, nx, ny, nz, nb, P):
    inner = dict(restart=30, max_it=20, rtol=1e-20)
    rtol = 1e-7
    opts = Options(" ".join(f"-inner{b + 1}_ksp_max_it 20 -inner{b + 1}_ksp_rtol 1e-20 -inner{b + 1}_pc_type none"
                            for b in range(nb)))
    comm = LocalComm()
    blocks = make_blocks(ctx, dim, nx, ny, nz, nb, range(nb), opts, comm, P)
    res = sm_solve(blocks, comm, rtol=rtol, max_outer=200)
    ro = oracle.sm_solve(dim, nx, ny, nz, nb, rtol, dict(inner, reduce_mode=oracle.REDUCE_DBR), max_outer=200,
                         peclet=P)
    assert res.outer_its == ro["outer_its"]
    assert res.norm0 == ro["norm0"]
    assert np.array_equal(np.array(res.hist), ro["hist"])
    assert np.array_equal(np.array(res.inner_its), ro["inner_its"])
    x = np.concatenate([blk.x.get_array() for blk in blocks])
    assert np.array_equal(x, ro["x"])


def _smsm_opts(nb):
    inner = " ".join(f"-inner{b + 1}_ksp_max_it 10 -inner{b + 1}_ksp_rtol 1e-20 -inner{b + 1}_pc_type none "
                     f"-inner{b + 1}_ksp_gmres_restart 30 -inner{b + 1}_ksp_atol 1e-100" for b in range(nb))
    outer = " ".join(f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default "
                     f"-outer{b + 1}_ksp_lsqr_exact_mat_norm -outer{b + 1}_ksp_atol 1e-100 "
                     f"-outer{b + 1}_ksp_max_it 70 -outer{b + 1}_ksp_rtol 1e-15 -outer{b + 1}_pc_type none"
                     for b in range(nb))
    return Options(inner + " " + outer)


@pytest.mark.parametrize("dim,nx,ny,nz,nb,s", [(3, 8, 8, 8, 2, 4), (2, 24, 20, 1, 3, 5), (3, 64, 64, 12, 3, 4)])
def test_smsm_convdiff_bitwise_vs_oracle(ctx, oracle, dim, nx, ny, nz, nb, s):
    """SMSM-global on convection-diffusion blocks, bitwise the oracle; 64 x 64 planes (whole DBR chunks): the
    blocks' A_ext with coupling planes take the chunk-tile march for R = A S and the global residual."""
    P = (0.5, 0.25, -0.3)
    rtol = 1e-8
    comm = LocalComm()
    blocks, mini = make_smsm(ctx, dim, nx, ny, nz, nb, range(nb), s, _smsm_opts(nb), comm, P)
    res = smsm_solve(blocks, comm, s, mini, rtol=rtol, max_outer=100)
    ro = oracle.smsm_solve(dim, nx, ny, nz, nb, s, rtol,
                           dict(restart=30, max_it=10, rtol=1e-20, abstol=1e-100, reduce_mode=oracle.REDUCE_DBR),
                           dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0,
                                reduce_mode=oracle.REDUCE_DBR), max_outer=100, peclet=P)
    assert res.outer_its == ro["outer_its"]
    assert res.norm0 == ro["norm0"]
    assert np.array_equal(np.array(res.hist), ro["hist"])
    assert np.array_equal(np.array(res.lsqr_its), ro["lsqr_its"])
    x = np.concatenate([blk.x.get_array() for blk in blocks])
    assert np.array_equal(x, ro["x"])
    assert res.final_norm == ro["final_norm"]
