"""The HIP path on the reference's own known-answer tests (src/tests/utils_test.c).

* poisson2DMatrix on the 2 x 2 mesh in 2 blocks (utils_test.c:183-220) and
  poisson3DMatrix on the 2 x 2 x 2 mesh in 2 blocks (:76-169): each block's rows
  assembled on the device (k_box_stencil, the block's rows in the column space
  [plane below | own | plane above], which for two blocks of these meshes is the
  global column space) equal the reference rows exactly.
* computeFinalResidualNorm (utils.c:575-595; KAT utils_test.c:225-228 with the
  inputs of :285-317): MatResidual + VecNorm on the device per block, the squared
  local norms summed in block order (the MPI_Allreduce of two values), sqrt --
  2.54567588 to Unity's float tolerance.

The values come from tests/golden/reference_kats.json (data copied from the
reference test, tests/golden/make_golden.py), so nothing here reads
/root/reference at run time.
"""
import json
import math
import os

import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd import utils
from medane_tchakorom_ufc_thesis_repository_amd.petsc import Mat, Vec

pytestmark = pytest.mark.gpu

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def _block_dense(ctx, dim, nx, ny, nz, b, storage):
    L = utils.block_layout(dim, nx, ny, nz, 2, b)
    A = Mat.box_stencil_ext(ctx, *L.box, b > 0, b < 1)
    A.set_storage(storage)
    rp, col, val = A.get_csr()
    D = np.zeros(A.shape)
    for r in range(A.shape[0]):
        D[r, col[rp[r]:rp[r + 1]]] = val[rp[r]:rp[r + 1]]
    return A, D


@pytest.mark.parametrize("storage", ["csr", "dv"])
def test_kat_poisson2DMatrix_device(ctx, storage):
    # 2 x 2 mesh (n_mesh_lines = n_mesh_columns = 2), two blocks of one mesh line
    for b in (0, 1):
        A, D = _block_dense(ctx, 2, 2, 2, 1, b, storage)
        assert A.shape == (2, 4)
        assert np.array_equal(D, np.array(KATS["poisson2d_2x2"][str(b)], float))


@pytest.mark.parametrize("storage", ["csr", "dv"])
def test_kat_poisson3DMatrix_device(ctx, storage):
    for b in (0, 1):
        A, D = _block_dense(ctx, 3, 2, 2, 2, b, storage)
        assert A.shape == (4, 8)
        assert np.array_equal(D, np.array(KATS["poisson3d_2x2x2"][str(b)], float))


@pytest.mark.parametrize("storage", ["csr", "dv"])
def test_kat_computeFinalResidualNorm_device(ctx, oracle, storage):
    inp = KATS["residual_inputs"]
    total = 0.0
    for b in (0, 1):
        A, _ = _block_dense(ctx, 2, 2, 2, 1, b, storage)
        x = Vec.from_array(ctx, np.array(inp["x"][str(b)]))       # each block's own x (utils_test.c:285-317)
        bb = Vec.from_array(ctx, np.array(inp["b"][str(b)]))
        r = Vec(ctx, 2)
        A.residual(bb, x, r)                                      # MatResidual
        ln = r.norm()                                             # VecNorm(NORM_2)
        # the same block on the CPU oracle, bit for bit
        Ao = oracle.poisson2d_rows(2, 2, 2 * b, 2 * b + 2)
        assert ln == oracle.final_residual_norm([Ao], np.array(inp["x"][str(b)]), [np.array(inp["b"][str(b)])],
                                             oracle.REDUCE_DBR)
        total += ln * ln                                          # local_norm^2, Allreduce(SUM) in block order
    got = math.sqrt(total)
    golden = KATS["residual_norm_golden"]
    assert abs(got - golden) <= 1e-5 * golden                    # TEST_ASSERT_EQUAL_FLOAT
    assert f"{got:.8f}" == "2.54567588"
