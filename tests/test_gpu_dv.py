"""DV storage (one byte per matrix entry, include/msplit.h MSP_STORAGE_DV).

The products over DV storage must equal the CSR kernel's and the oracle's
MatMult_SeqAIJ order bit for bit (the storage changes, the sequence of
products and sums does not); matrices that do not fit keep CSR storage.
"""
import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd.petsc import KSP, Mat, Options, Vec

pytestmark = pytest.mark.gpu

SEED = 20251121


def _products(ctx, A, O, r):
    nr, nc = O.shape
    x = r.uniform(-1, 1, nc)
    b = r.uniform(-1, 1, nr)
    xv, bv, yv = Vec.from_array(ctx, x), Vec.from_array(ctx, b), Vec(ctx, nr)
    A.mult(xv, yv)
    y = yv.get_array()
    A.residual(bv, xv, yv)
    res = yv.get_array()
    assert np.array_equal(y, O.mult(x))
    assert np.array_equal(res, O.residual(b, x))
    return y, res


def _both_storages(ctx, A, O):
    assert A.get_storage() == "dv"
    yd, rd = _products(ctx, A, O, np.random.default_rng(SEED))
    A.set_storage("csr")
    assert A.get_storage() == "csr"
    yc, rc = _products(ctx, A, O, np.random.default_rng(SEED))
    A.set_storage("dv")
    assert np.array_equal(yd, yc) and np.array_equal(rd, rc)


@pytest.mark.parametrize("dim,nx,ny,nz,lo,hi", [(3, 37, 11, 9, 0, 0), (3, 16, 16, 8, 1, 1), (3, 16, 16, 8, 1, 0),
                                                (3, 1, 1, 9, 0, 1), (2, 64, 50, 1, 0, 0), (2, 33, 7, 1, 1, 1),
                                                (3, 64, 64, 64, 0, 0)])
def test_box_operators_take_dv_and_match_csr(ctx, oracle, dim, nx, ny, nz, lo, hi):
    A = Mat.box_stencil_ext(ctx, dim, nx, ny, nz, bool(lo), bool(hi))
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    _both_storages(ctx, A, O)


@pytest.mark.parametrize("peclet", [(0.5, 0.25, -0.3), (-2.0, 0.0, 1.5)])
def test_convdiff_takes_dv(ctx, oracle, peclet):
    A = Mat.box_convdiff(ctx, 3, 24, 20, 12, True, True, peclet)
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    _both_storages(ctx, A, O)


def _banded(n, offsets, values, r, drop=0.2):
    """Rows with entries at r + offsets (inside [0, n)), each value drawn from a small set, some dropped."""
    rows, cols, vals = [], [], []
    rp = [0]
    for i in range(n):
        cs = [i + d for d in offsets if 0 <= i + d < n and r.random() > drop]
        cols += sorted(cs)
        vals += list(r.choice(values, size=len(cs)))
        rp.append(len(cols))
    return np.array(rp, np.int32), np.array(cols, np.int32), np.array(vals, np.float64)


@pytest.mark.parametrize("n", [1, 255, 256, 257, 4099, 20000])
def test_host_csr_with_few_pairs_takes_dv(ctx, oracle, n):
    r = np.random.default_rng(SEED + n)
    rp, col, val = _banded(n, [-300, -17, -1, 0, 1, 5, 17, 299], [-1.0, 2.5, 6.0, -0.0], r)
    O = oracle.Mat.from_arrays(n, n, rp, col, val)
    A = Mat.from_csr(ctx, n, n, rp, col, val)
    if len(val) == 0:
        assert A.get_storage() == "csr"
        return
    _both_storages(ctx, A, O)


def test_exactly_256_pairs_fit_and_257_do_not(ctx, oracle):
    n = 600
    for npairs, want in ((256, "dv"), (257, "csr")):
        rp = np.arange(n + 1, dtype=np.int32)
        col = np.arange(n, dtype=np.int32)
        val = np.array([float(i % npairs) + 0.5 for i in range(n)])  # diagonal, npairs distinct values
        A = Mat.from_csr(ctx, n, n, rp, col, val)
        assert A.get_storage() == want
        O = oracle.Mat.from_arrays(n, n, rp, col, val)
        _products(ctx, A, O, np.random.default_rng(SEED))


def test_signed_zero_and_nan_bits_are_distinct_pairs(ctx, oracle):
    # -0.0 and 0.0 are different pairs: the dictionary compares bits
    n = 300
    rp = np.arange(n + 1, dtype=np.int32)
    col = np.arange(n, dtype=np.int32)
    val = np.where(np.arange(n) % 2 == 0, 0.0, -0.0)
    A = Mat.from_csr(ctx, n, n, rp, col, val)
    assert A.get_storage() == "dv"
    x = np.full(n, -1.0)
    xv, yv = Vec.from_array(ctx, x), Vec(ctx, n)
    A.mult(xv, yv)
    y = yv.get_array()
    O = oracle.Mat.from_arrays(n, n, rp, col, val)
    assert np.array_equal(np.signbit(y), np.signbit(O.mult(x)))


def test_unfit_matrices_keep_csr(ctx, oracle):
    r = np.random.default_rng(SEED)
    n = 2000
    # random values: thousands of distinct pairs
    rp, col, val = _banded(n, [-3, 0, 3], [0.0], r)
    val = r.standard_normal(len(val))
    A = Mat.from_csr(ctx, n, n, rp, col, val)
    assert A.get_storage() == "csr"
    with pytest.raises(Exception):
        A.set_storage("dv")
    # one row longer than 255 entries
    lens = np.full(n, 1)
    lens[7] = 300
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.concatenate([np.arange(l) if l > 1 else [i] for i, l in enumerate(lens)]).astype(np.int32)
    val = np.ones(rp[-1])
    A = Mat.from_csr(ctx, n, n, rp, col, val)
    assert A.get_storage() == "csr"
    O = oracle.Mat.from_arrays(n, n, rp, col, val)
    _products(ctx, A, O, r)


def test_matfree_reports_no_storage(ctx):
    A = Mat.box_matfree(ctx, 3, 8, 8, 8)
    assert A.get_storage() == "none"


@pytest.mark.parametrize("dim,nx,ny,nz,restart,max_it,rtol", [(3, 24, 20, 16, 30, 90, 1e-12),
                                                             (2, 96, 64, 1, 7, 60, 1e-10)])
def test_gmres_on_dv_equals_csr_and_oracle(ctx, oracle, dim, nx, ny, nz, restart, max_it, rtol):
    """The whole GMRES solve (scaled MatMult inside the Arnoldi step, MatResidual at restarts) on DV storage
    is bitwise the CSR solve and the DBR oracle's."""
    out = {}
    for st in ("dv", "csr"):
        A = Mat.box_stencil(ctx, dim, nx, ny, nz)
        A.set_storage(st)
        n = A.shape[0]
        ones, b, x = Vec(ctx, n), Vec(ctx, n), Vec(ctx, n)
        ones.set(1.0)
        A.mult(ones, b)
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(f"-ksp_gmres_restart {restart} -ksp_max_it {max_it} -ksp_rtol {rtol!r} "
                                     "-pc_type none"))
        ksp.solve(b, x)
        out[st] = (ksp.get_iteration_number(), ksp.get_residual_history(), x.get_array(), b.get_array())
    assert out["dv"][0] == out["csr"][0]
    for a, c in zip(out["dv"][1:], out["csr"][1:]):
        assert np.array_equal(a, c)
    if dim == 3:
        Ao = oracle.poisson3d_rows(nx, ny, nz, 0, nz)
    else:
        Ao = oracle.poisson2d_rows(ny, nx, 0, nx * ny)
    xo, ro = oracle.gmres(Ao, out["dv"][3], restart=restart, max_it=max_it, rtol=rtol,
                          reduce_mode=oracle.REDUCE_DBR)
    assert out["dv"][0] == ro["its"]
    assert np.array_equal(out["dv"][1], ro["hist"])
    assert np.array_equal(out["dv"][2], xo)


@pytest.mark.parametrize("assembly,product", [(0, 8192), (0, 16384), (0, 0),            # ELL: 1, 2, 4 rows per lane
                                              (32768, 32768 | 8192), (32768, 32768 | 16384),
                                              (32768, 32768)])                         # CSR-order codes
@pytest.mark.parametrize("case", ["box", "banded", "ragged-tail", "w4", "w16", "long-rows"])
def test_layout_and_rows_per_lane_variants_bitwise(ctx, oracle, assembly, product, case):
    """Each DV layout (ELL of 4/8/16 codes per row, or CSR-order codes with row lengths) and each
    rows-per-lane variant against the oracle."""
    import ctypes
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    L = _lib.load()
    L.msk_set_tuning.argtypes = [ctypes.c_int]
    L.msk_set_tuning.restype = None
    r = np.random.default_rng(SEED)
    offsets = {"banded": [-40, -1, 0, 2, 33], "ragged-tail": [-40, -1, 0, 2, 33], "w4": [-7, 0, 1],
               "w16": [-900, -64, -9, -8, -3, -2, -1, 0, 1, 2, 3, 8, 64, 900],
               "long-rows": list(range(-20, 21))}
    try:
        L.msk_set_tuning(assembly)
        if case == "box":
            A = Mat.box_stencil_ext(ctx, 3, 20, 13, 11, True, True)
            rp, col, val = A.get_csr()
            nr, nc = A.shape
        else:
            nr = nc = 1024 * 3 + (517 if case == "ragged-tail" else 0)
            rp, col, val = _banded(nr, offsets[case], [-1.0, 4.0, 0.5], r,
                                   drop=0.9 if case == "ragged-tail" else 0.3)
            A = Mat.from_csr(ctx, nr, nc, rp, col, val)
        assert A.get_storage() == "dv"
        O = oracle.Mat.from_arrays(nr, nc, rp, col, val)
        L.msk_set_tuning(product)
        _products(ctx, A, O, r)
    finally:
        L.msk_set_tuning(0)


@pytest.mark.parametrize("s", [1, 7, 20, 33])
@pytest.mark.parametrize("peclet", [None, (0.5, -0.25, 1.0)])
def test_matmult_dense_on_dv_equals_csr_and_oracle(ctx, oracle, s, peclet):
    """MatMatMult R = A_ext S (SMSM's R, SMSM-global.c:325-327) on DV storage: the CSR kernel's and the
    oracle's row sums bit for bit."""
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import DenseMat
    A = Mat.box_convdiff(ctx, 3, 12, 9, 7, True, True, peclet or (0.0, 0.0, 0.0))
    rp, col, val = A.get_csr()
    nr, nc = A.shape
    S = np.random.default_rng(SEED + s).standard_normal((nc, s))
    out = {}
    for st in ("dv", "csr"):
        A.set_storage(st)
        Rd = DenseMat(ctx, nr, s)
        A.mat_mult_dense(DenseMat.from_array(ctx, S), Rd)
        out[st] = Rd.get_values()
    O = oracle.Mat.from_arrays(nr, nc, rp, col, val)
    ref = np.stack([O.mult(S[:, j]) for j in range(s)], axis=1)
    assert np.array_equal(out["dv"], ref)
    assert np.array_equal(out["csr"], ref)


def test_release_csr(ctx, oracle):
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import DenseMat
    A = Mat.box_stencil_ext(ctx, 3, 16, 12, 10, True, False)
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    A.release_csr()
    A.release_csr()                          # idempotent
    assert A.get_storage() == "dv"
    with pytest.raises(Exception):
        A.get_csr()
    with pytest.raises(Exception):
        A.set_storage("csr")
    _products(ctx, A, O, np.random.default_rng(SEED))
    S = np.random.default_rng(SEED).standard_normal((A.shape[1], 5))
    Rd = DenseMat(ctx, A.shape[0], 5)
    A.mat_mult_dense(DenseMat.from_array(ctx, S), Rd)
    assert np.array_equal(Rd.get_values(), np.stack([O.mult(S[:, j]) for j in range(5)], axis=1))
    # a matrix in CSR storage cannot drop its CSR
    B = Mat.box_stencil(ctx, 3, 8, 8, 8)
    B.set_storage("csr")
    with pytest.raises(Exception):
        B.release_csr()


def test_gmres_after_release_csr(ctx, oracle):
    A = Mat.box_stencil(ctx, 3, 20, 16, 12)
    A.release_csr()
    n = A.shape[0]
    ones, b, x = Vec(ctx, n), Vec(ctx, n), Vec(ctx, n)
    ones.set(1.0)
    A.mult(ones, b)
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options("-ksp_gmres_restart 30 -ksp_max_it 70 -ksp_rtol 1e-12 -pc_type none"))
    ksp.solve(b, x)
    Ao = oracle.poisson3d_rows(20, 16, 12, 0, 12)
    xo, ro = oracle.gmres(Ao, b.get_array(), restart=30, max_it=70, rtol=1e-12, reduce_mode=oracle.REDUCE_DBR)
    assert ksp.get_iteration_number() == ro["its"]
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(x.get_array(), xo)


def test_tall_matrix_dv(ctx, oracle):
    """More rows than columns (each row reads x at row - offset inside [0, ncols))."""
    r = np.random.default_rng(SEED)
    nr, nc = 3000, 1100
    rows_c, rows_v, rp = [], [], [0]
    for i in range(nr):
        cs = sorted({c for c in (i - 1900, i - 1000, i - 7) if 0 <= c < nc and r.random() > 0.2})
        rows_c += cs
        rows_v += list(r.choice([2.0, -1.5], size=len(cs)))
        rp.append(len(rows_c))
    rp, col, val = np.array(rp, np.int32), np.array(rows_c, np.int32), np.array(rows_v)
    A = Mat.from_csr(ctx, nr, nc, rp, col, val)
    O = oracle.Mat.from_arrays(nr, nc, rp, col, val)
    _both_storages(ctx, A, O)


@pytest.mark.parametrize("flags", [67108864, 67108864 | 8192, 67108864 | 16384, 134217728])
@pytest.mark.parametrize("nz", [40, 64, 1])
def test_ell_xcd_block_order_bitwise(ctx, oracle, flags, nz):
    """The XCD-contiguous block order of the ELL SpMV (MSK_TUNE_ELL_XCD_ON, forced here on a small plane; the
    default turns it on from 2^18 rows per plane) over full windows of 64 blocks and a ragged tail, and the
    identity order forced off: MatMult, MatResidual and the scaled GMRES form equal the oracle."""
    from test_gpu_kernels import tuning
    A = Mat.box_stencil_ext(ctx, 3, 64, 64, nz, nz > 1, False)
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    assert A.get_storage() == "dv"
    with tuning(flags):
        _products(ctx, A, O, np.random.default_rng(SEED))



MARCH_OFF, MARCH_NOXCD, BOX_SEPARATE, BOX_FLAT, BOX_NOXCD = 268435456, 536870912, 1073741824, 32, 524288


@pytest.mark.parametrize("flags", [0, MARCH_NOXCD, MARCH_OFF, BOX_SEPARATE, BOX_FLAT, BOX_NOXCD])
@pytest.mark.parametrize("shape", [(256, 16, 40), (512, 3, 17), (256, 1, 1), (256, 5, 16), (768, 2, 33),
                                   (256, 40, 7), (256, 100, 40), (37, 11, 9), (64, 64, 64), (100, 30, 20),
                                   (300, 7, 5), (1, 1, 9), (16, 16, 1), (2, 3, 50), (129, 2, 3),
                                   (256, 16, 7), (1024, 4, 9), (2048, 2, 5), (64, 128, 6), (256, 512, 5)])
@pytest.mark.parametrize("peclet", [None, (0.5, -0.25, 0.3)])
def test_box_march_bitwise(ctx, oracle, flags, shape, peclet):
    """The z-march SpMV of box stencils (the default for 3D boxes; MSK_TUNE_ELL_MARCH_NOXCD: identity workgroup
    order; MSK_TUNE_ELL_MARCH_OFF: the row-parallel ELL kernel): whole and ragged z tiles (16 planes per workgroup),
    one and several y lines, one and several 256-wide x segments, segments spanning several lines (nx < 256 or not
    a multiple of 256) and a ragged last segment per plane, full XCD runs of 32 workgroups and a ragged tail.  MatMult and MatResidual equal the oracle; GMRES -- the scaled MatMult with its stop flag -- equals
    the oracle's DBR GMRES bit for bit."""
    from test_gpu_kernels import tuning
    nx, ny, nz = shape
    A = Mat.box_stencil(ctx, 3, nx, ny, nz) if peclet is None else Mat.box_convdiff(ctx, 3, nx, ny, nz, False,
                                                                                    False, peclet)
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    assert A.get_storage() == "dv"
    n = A.shape[0]
    b = O.mult(np.random.default_rng(SEED).uniform(-1, 1, n))
    o = dict(restart=12, max_it=40, rtol=1e-30)
    with tuning(flags):
        _products(ctx, A, O, np.random.default_rng(SEED))
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                     f"-ksp_gmres_restart {o['restart']} -ksp_max_it {o['max_it']} "
                                     f"-ksp_rtol {o['rtol']}"))
        xv = Vec(ctx, n)
        ksp.solve(Vec.from_array(ctx, b), xv)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, **o)
    assert ksp.get_iteration_number() == ro["its"]
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(xv.get_array(), xo)


def test_box_march_large_plane(ctx, oracle):
    """512 x 512 planes: the z-march kernel equals the row-parallel ELL kernel (MSK_TUNE_ELL_MARCH_OFF, XCD order
    at this plane size) and the oracle bit for bit.  A flag combination with no kernel is an error."""
    from test_gpu_kernels import tuning
    from medane_tchakorom_ufc_thesis_repository_amd import MsplitError
    A = Mat.box_stencil(ctx, 3, 512, 512, 5)
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    y0, r0 = _products(ctx, A, O, np.random.default_rng(SEED))
    with tuning(MARCH_OFF):
        y1, r1 = _products(ctx, A, O, np.random.default_rng(SEED))
    assert np.array_equal(y0, y1) and np.array_equal(r0, r1)
    x = Vec.from_array(ctx, np.ones(A.shape[0]))
    y = Vec(ctx, A.shape[0])
    with tuning(MARCH_OFF | MARCH_NOXCD):
        with pytest.raises(MsplitError):
            A.mult(x, y)


@pytest.mark.parametrize("lines", [1, 4])
@pytest.mark.parametrize("zt", [0, 3])
@pytest.mark.parametrize("shape", [(256, 16, 40), (512, 3, 17), (256, 1, 1), (256, 5, 16), (768, 2, 33),
                                   (256, 9, 7), (512, 8, 2)])
@pytest.mark.parametrize("mode", ["products", "gmres"])
def test_box_march_lines_bitwise(ctx, oracle, lines, zt, shape, mode):
    """Both march tiles forced (msk_set_march_lines: 1 = 256 plane rows, 4 = four whole y lines, the default for
    nx % 256 == 0 from 1024 workgroups) with the automatic or a ragged 3-plane depth (msk_set_march_z): full and
    ragged line tiles (ny % 4 != 0), one line, several x segments.  MatMult / MatResidual, and GMRES with the scaled
    form, equal the oracle bit for bit."""
    import ctypes
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    L = _lib.load()
    L.msk_set_march_lines.argtypes = [ctypes.c_int]
    L.msk_set_march_z.argtypes = [ctypes.c_int]
    nx, ny, nz = shape
    A = Mat.box_convdiff(ctx, 3, nx, ny, nz, False, False, (0.5, -0.25, 0.3))
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    n = A.shape[0]
    L.msk_set_march_lines(lines)
    L.msk_set_march_z(zt)
    try:
        if mode == "products":
            _products(ctx, A, O, np.random.default_rng(SEED))
            return
        b = O.mult(np.random.default_rng(SEED).uniform(-1, 1, n))
        o = dict(restart=8, max_it=20, rtol=1e-30)
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                     f"-ksp_gmres_restart {o['restart']} -ksp_max_it {o['max_it']} "
                                     f"-ksp_rtol {o['rtol']}"))
        xv = Vec(ctx, n)
        ksp.solve(Vec.from_array(ctx, b), xv)
    finally:
        L.msk_set_march_lines(0)
        L.msk_set_march_z(0)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, **o)
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(xv.get_array(), xo)


@pytest.mark.parametrize("flags", [0, MARCH_NOXCD, MARCH_OFF, BOX_SEPARATE])
@pytest.mark.parametrize("shape", [(256, 64), (100, 37), (1024, 9), (33, 7), (1, 50), (300, 1), (512, 40)])
@pytest.mark.parametrize("peclet", [None, (0.5, -0.25, 0.0)])
def test_box_march_2d_bitwise(ctx, oracle, flags, shape, peclet):
    """2D box stencils take the march too, as an nx x 1 x ny box (five codes -nx, -1, 0, +1, +nx mapped onto the
    3D neighbours): MatMult, MatResidual and GMRES equal the oracle bit for bit, as do the identity order and the
    row-parallel kernel."""
    from test_gpu_kernels import tuning
    nx, ny = shape
    A = Mat.box_stencil(ctx, 2, nx, ny) if peclet is None else Mat.box_convdiff(ctx, 2, nx, ny, 1, False, False,
                                                                                peclet)
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    assert A.get_storage() == "dv"
    n = A.shape[0]
    b = O.mult(np.random.default_rng(SEED).uniform(-1, 1, n))
    o = dict(restart=10, max_it=30, rtol=1e-30)
    with tuning(flags):
        _products(ctx, A, O, np.random.default_rng(SEED))
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                     f"-ksp_gmres_restart {o['restart']} -ksp_max_it {o['max_it']} "
                                     f"-ksp_rtol {o['rtol']}"))
        xv = Vec(ctx, n)
        ksp.solve(Vec.from_array(ctx, b), xv)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, **o)
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(xv.get_array(), xo)


@pytest.mark.parametrize("shape", [(64, 1, 64), (1, 30, 20), (2, 1, 40), (1, 1, 33), (300, 1, 17)])
@pytest.mark.parametrize("peclet", [None, (0.5, 0.25, 0.25), (0.0, 0.7, 0.7)])
def test_box_march_degenerate_lines(ctx, oracle, shape, peclet):
    """3D boxes with one y line (ny == 1) or one x column (nx == 1): two stencil deltas coincide (+nx = +P, or
    -1 = -nx), so the encoder would name the +z coupling +nx when the two values are equal (py = pz >= 0, and the
    Poisson operator) and the march would drop it.  Such boxes keep the row-parallel ELL kernel; products and
    GMRES equal the oracle bit for bit."""
    nx, ny, nz = shape
    A = Mat.box_stencil(ctx, 3, nx, ny, nz) if peclet is None else Mat.box_convdiff(ctx, 3, nx, ny, nz, False,
                                                                                    False, peclet)
    assert A.spmv_kernel() != "k_spmv_box_march"
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    n = A.shape[0]
    _products(ctx, A, O, np.random.default_rng(SEED))
    b = O.mult(np.random.default_rng(SEED).uniform(-1, 1, n))
    o = dict(restart=8, max_it=24, rtol=1e-30)
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                 f"-ksp_gmres_restart {o['restart']} -ksp_max_it {o['max_it']} -ksp_rtol {o['rtol']}"))
    xv = Vec(ctx, n)
    ksp.solve(Vec.from_array(ctx, b), xv)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, **o)
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(xv.get_array(), xo)


def _gmres_vs_oracle(ctx, oracle, A, O, b, restart=30, max_it=30):
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                 f"-ksp_gmres_restart {restart} -ksp_max_it {max_it} -ksp_rtol 1e-30"))
    xv = Vec(ctx, A.shape[0])
    ksp.solve(Vec.from_array(ctx, b), xv)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, restart=restart, max_it=max_it,
                          rtol=1e-30)
    assert ksp.get_iteration_number() == ro["its"]
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(xv.get_array(), xo)


@pytest.mark.parametrize("flags", [0, BOX_SEPARATE, BOX_FLAT])
@pytest.mark.parametrize("case", ["3d_256", "3d_ragged", "2d_configs0_block", "3d_convdiff", "3d_dropped"])
def test_assembled_box_takes_the_march(ctx, oracle, case, flags):
    """An operator the caller assembles (the reference's poisson3DMatrix / poisson2DMatrix rows cut to a block by
    MatCreateSubMatrix, utils.c:30-121, :247-293, :450-478) handed to msp_mat_create_csr -- the path the PETSc
    plugin's MatAssemblyEnd takes -- is recognised as a box stencil and runs the z-march SpMV: MatMult, MatResidual
    and GMRES(30) equal the oracle bit for bit.  3d_256 is configs[1]'s operator; 2d_configs0_block one of
    configs[0]'s two diagonal blocks; 3d_dropped a box with random entries left out (the presence bytes, not the
    geometry, say which neighbours a row holds)."""
    r = np.random.default_rng(SEED)
    if case == "3d_256":
        O = oracle.poisson3d_rows(256, 256, 256, 0, 256)
    elif case == "3d_ragged":
        O = oracle.poisson3d_rows(37, 11, 9, 0, 9)
    elif case == "2d_configs0_block":
        Ab = oracle.poisson2d_rows(256, 256, 256 * 128, 256 * 256)     # block 1 of configs[0]
        O, _ = oracle.split(Ab, 256 * 128, 256 * 256)
    elif case == "3d_convdiff":
        O = oracle.convdiff_rows(3, 64, 48, 40, 0, 64 * 48 * 40, (0.5, -0.25, 0.3))
    else:
        B = oracle.poisson3d_rows(48, 40, 24, 0, 24)
        rp0, c0, v0 = B.arrays()
        keep = (r.random(len(c0)) > 0.15) | (np.repeat(np.arange(B.shape[0]), np.diff(rp0)) == c0)
        rows = np.repeat(np.arange(B.shape[0]), np.diff(rp0))[keep]
        rp = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=B.shape[0]))]).astype(np.int32)
        O = oracle.Mat.from_arrays(B.shape[0], B.shape[1], rp, c0[keep], v0[keep])
    rp, col, val = O.arrays()
    n = O.shape[0]
    A = Mat.from_csr(ctx, n, n, rp, col, val)
    assert A.get_storage() == "dv"
    assert A.spmv_kernel() == "k_spmv_box_march"
    _products(ctx, A, O, np.random.default_rng(SEED))
    b = O.mult(np.ones(n)) if case == "3d_256" else O.mult(r.uniform(-1, 1, n))
    from test_gpu_kernels import tuning
    with tuning(flags):     # 0: the GMRES MatMult fused with the VecMDot (k_box_spmv_mdot); BOX_SEPARATE: two kernels
        _gmres_vs_oracle(ctx, oracle, A, O, b, max_it=30 if case == "3d_256" else 45)


@pytest.mark.parametrize("wrap", ["x_minus", "x_plus", "y_minus", "y_plus", "x_minus_2d"])
def test_assembled_box_with_wrapped_entry_keeps_ell(ctx, oracle, wrap):
    """The same dictionary, but one row holds a neighbour across a line or plane edge (a -1 entry at i = 0, ...):
    the march would read it as 0.0, so the device check keeps the row-parallel ELL kernel, whose products and GMRES
    still equal the oracle bit for bit."""
    nx, ny, nz = (20, 12, 10) if wrap != "x_minus_2d" else (30, 16, 1)
    O0 = oracle.poisson3d_rows(nx, ny, nz, 0, nz) if nz > 1 else oracle.poisson2d_rows(ny, nx, 0, nx * ny)
    rp, col, val = (a.copy() for a in O0.arrays())
    n = O0.shape[0]
    P = nx * ny
    row, delta = {"x_minus": (5 * P + 3 * nx, -1), "x_plus": (5 * P + 3 * nx + nx - 1, 1),
                  "y_minus": (4 * P + 7, -nx), "y_plus": (4 * P + (ny - 1) * nx + 7, nx),
                  "x_minus_2d": (3 * nx, -1)}[wrap]
    rows = [list(zip(col[rp[i]:rp[i + 1]], val[rp[i]:rp[i + 1]])) for i in range(n)]
    assert all(c != row + delta for c, _ in rows[row])
    rows[row] = sorted(rows[row] + [(row + delta, -1.0)])
    rp = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int32)
    col = np.array([c for x in rows for c, _ in x], np.int32)
    val = np.array([v for x in rows for _, v in x])
    O = oracle.Mat.from_arrays(n, n, rp, col, val)
    A = Mat.from_csr(ctx, n, n, rp, col, val)
    assert A.get_storage() == "dv"
    assert A.spmv_kernel() == "k_spmv_ell"
    _products(ctx, A, O, np.random.default_rng(SEED))
    _gmres_vs_oracle(ctx, oracle, A, O, O.mult(np.random.default_rng(SEED).uniform(-1, 1, n)), max_it=40)


@pytest.mark.parametrize("defect", ["duplicate_diagonal", "duplicate_neighbour", "unsorted_row"])
def test_assembled_box_with_duplicate_or_unsorted_row_is_refused(ctx, oracle, defect):
    """A box-stencil dictionary whose one row repeats a column (which the march would add once, not twice) or lists
    its columns out of order (which the march would sum in another order than the row's): msp_mat_create_csr
    refuses both with PETSC_ERR_ARG_WRONG before any storage -- march, ELL or CSR -- is chosen, as an assembled
    PETSc AIJ never holds either (MatAssemblyEnd merges duplicates and sorts each row)."""
    from medane_tchakorom_ufc_thesis_repository_amd import MsplitError
    nx, ny, nz = 16, 12, 8
    O = oracle.poisson3d_rows(nx, ny, nz, 0, nz)
    rp, col, val = (a.copy() for a in O.arrays())
    n = O.shape[0]
    row = 3 * nx * ny + 5 * nx + 7                       # an interior row: 7 entries, columns ascending
    rows = [list(zip(col[rp[i]:rp[i + 1]], val[rp[i]:rp[i + 1]])) for i in range(n)]
    if defect == "duplicate_diagonal":
        rows[row] = sorted(rows[row] + [(row, 0.5)])
    elif defect == "duplicate_neighbour":
        rows[row] = sorted(rows[row] + [(row + nx, -1.0)])
    else:
        rows[row][2], rows[row][3] = rows[row][3], rows[row][2]
    rp = np.concatenate([[0], np.cumsum([len(x) for x in rows])]).astype(np.int32)
    col = np.array([c for x in rows for c, _ in x], np.int32)
    val = np.array([v for x in rows for _, v in x])
    with pytest.raises(MsplitError) as e:
        Mat.from_csr(ctx, n, n, rp, col, val)
    assert e.value.code == 62 and "ascending" in str(e.value)


_SELF_SCRIPT = r"""
import hashlib, json, sys
import numpy as np
from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, KSP, Mat, Options, Vec
ctx = Context(0)
A = Mat.box_stencil(ctx, 3, 64, 64, 32)
n = A.shape[0]
b = Vec.from_array(ctx, np.random.default_rng(7).uniform(-1, 1, n))
ksp = KSP(ctx)
ksp.set_operators(A)
ksp.set_from_options(Options("-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned -ksp_gmres_restart 30 "
                             "-ksp_max_it 75 -ksp_rtol 1e-30"))
x = Vec(ctx, n)
ctx.set_timing(True)
ksp.solve(b, x)
ctx.set_timing(False)
print(json.dumps({"hist": [float(h).hex() for h in ksp.get_residual_history()],
                  "x": hashlib.sha256(x.get_array().tobytes()).hexdigest(),
                  "spmvdot": ctx.kernel_stats()["spmvdot"]["launches"]}))
"""


def test_box_mdot_self_dot_from_registers_is_bitwise():
    """GMRES's basis ends with the vector the MatMult reads (VV(it)); the fused z-march kernel takes that dot from the
    x rows it holds in registers instead of re-reading the vector.  The same GMRES(30) run with the dot streamed from
    HBM (MSPLIT_BOXMDOT_SELF=0, read once per process, hence two processes) gives the same history and x bits."""
    import json
    import os
    import subprocess
    import sys
    outs = []
    for self_env in ("1", "0"):
        env = dict(os.environ, MSPLIT_BOXMDOT_SELF=self_env)
        r = subprocess.run([sys.executable, "-c", _SELF_SCRIPT], env=env, capture_output=True, text=True, timeout=240,
                           cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert outs[0]["spmvdot"] > 0 and outs[1]["spmvdot"] > 0
    assert len(outs[0]["hist"]) > 75
    assert outs[0]["hist"] == outs[1]["hist"] and outs[0]["x"] == outs[1]["x"]


@pytest.mark.parametrize("zt", [0, 3])
@pytest.mark.parametrize("shape", [(256, 16, 40), (512, 8, 2), (64, 64, 33), (2048, 2, 7), (128, 32, 5),
                                   (256, 256, 3), (64, 64, 1), (4096 // 2, 2, 1)])
@pytest.mark.parametrize("mode", ["products", "gmres"])
def test_box_march_chunk_bitwise(ctx, oracle, zt, shape, mode):
    """The march over DBR chunk tiles (k_box_march_chunk: planes of whole 4096-row chunks, nx even <= 2048; the
    default for such boxes), forced with msk_set_march_lines(16), with its 2-plane or a ragged 3-plane depth:
    MatMult and MatResidual, and GMRES with the MatMult kept apart from the VecMDot (the scaled form with the
    VecScale output), equal the oracle bit for bit.  XCD-contiguous tiles from 32 tiles per plane (2048 x 2,
    256 x 256 with 16 tiles per plane: plane order)."""
    import ctypes
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from test_gpu_kernels import tuning
    L = _lib.load()
    L.msk_set_march_lines.argtypes = [ctypes.c_int]
    L.msk_set_march_z.argtypes = [ctypes.c_int]
    nx, ny, nz = shape
    A = Mat.box_convdiff(ctx, 3, nx, ny, nz, False, False, (0.5, -0.25, 0.3))
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    n = A.shape[0]
    L.msk_set_march_lines(16)
    L.msk_set_march_z(zt)
    try:
        if mode == "products":
            _products(ctx, A, O, np.random.default_rng(SEED))
            return
        b = O.mult(np.random.default_rng(SEED).uniform(-1, 1, n))
        o = dict(restart=8, max_it=20, rtol=1e-30)
        ksp = KSP(ctx)
        ksp.set_operators(A)
        ksp.set_from_options(Options(f"-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned "
                                     f"-ksp_gmres_restart {o['restart']} -ksp_max_it {o['max_it']} "
                                     f"-ksp_rtol {o['rtol']}"))
        xv = Vec(ctx, n)
        with tuning(BOX_SEPARATE):
            ksp.solve(Vec.from_array(ctx, b), xv)
    finally:
        L.msk_set_march_lines(0)
        L.msk_set_march_z(0)
    xo, ro = oracle.gmres(O, b, reduce_mode=oracle.REDUCE_DBR, guess_nonzero=0, **o)
    assert np.array_equal(ksp.get_residual_history(), ro["hist"])
    assert np.array_equal(xv.get_array(), xo)


def test_box_march_chunk_refused_where_it_does_not_fit(ctx):
    """msk_set_march_lines(16) on a box whose planes are not whole DBR chunks is an error, not another kernel."""
    import ctypes
    from medane_tchakorom_ufc_thesis_repository_amd import _lib
    from medane_tchakorom_ufc_thesis_repository_amd import MsplitError
    L = _lib.load()
    L.msk_set_march_lines.argtypes = [ctypes.c_int]
    A = Mat.box_convdiff(ctx, 3, 48, 40, 6, False, False, (0.0, 0.0, 0.0))
    x, y = Vec(ctx, A.shape[0]), Vec(ctx, A.shape[0])
    x.set(1.0)
    L.msk_set_march_lines(16)
    try:
        with pytest.raises(MsplitError):
            A.mult(x, y)
    finally:
        L.msk_set_march_lines(0)


@pytest.mark.parametrize("halo", [1, 2, 3])
@pytest.mark.parametrize("shape", [(64, 64, 9), (256, 16, 5), (128, 32, 3), (64, 64, 1), (512, 8, 2)])
def test_box_with_coupling_planes_takes_the_chunk_march(ctx, oracle, halo, shape):
    """A block's rows of the block-Jacobi operator with its coupling columns (A_ext: the plane below and / or
    above the block in the column space, utils.c:891-921) marches over chunk tiles when its planes hold whole DBR
    chunks: MatMult, MatResidual and R = A S (MatMatMult, column by column) equal the CSR operator's products
    bit for bit -- the ±P neighbours of the first / last plane read from the coupling planes."""
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import DenseMat
    nx, ny, nz = shape
    lo, hi = bool(halo & 1), bool(halo & 2)
    A = Mat.box_convdiff(ctx, 3, nx, ny, nz, lo, hi, (0.5, -0.25, 0.3))
    assert A.get_storage() == "dv" and A.spmv_kernel() == "k_spmv_box_march"
    rp, col, val = A.get_csr()
    O = oracle.Mat.from_arrays(A.shape[0], A.shape[1], rp, col, val)
    _products(ctx, A, O, np.random.default_rng(SEED))
    s = 5
    S = np.random.default_rng(SEED + 1).uniform(-1, 1, (A.shape[1], s))
    Sd = DenseMat.from_array(ctx, S)
    Rd = DenseMat(ctx, A.shape[0], s)
    A.mat_mult_dense(Sd, Rd)
    R = Rd.get_values()
    for q in range(s):
        assert np.array_equal(R[:, q], O.mult(np.ascontiguousarray(S[:, q])))


@pytest.mark.parametrize("flags", [0, 2048])
@pytest.mark.parametrize("n", [24, 48])
def test_non_stencil_aij_keeps_csr_and_equals_oracle(ctx, oracle, n, flags):
    """bench.py's non_stencil_aij operator (utils.heterogeneous_poisson3d: a per-cell kappa, so almost every row
    holds its own values and no dictionary fits) on boxes whose planes do not hold whole 4096-row chunks keeps CSR
    storage, and MatMult, MatResidual and GMRES(30) through msp_mat_create_csr equal the oracle bit for bit, with
    the default step (k_spmv_lds8 + the CGS kernels) and with the MatMult fused with the VecMDot (MSPLIT_TUNING
    2048, k_spmv_mdot)."""
    from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d
    from test_gpu_kernels import tuning
    rp, col, val = heterogeneous_poisson3d(n)
    N = n ** 3
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    assert A.get_storage() == "csr"
    O = oracle.Mat.from_arrays(N, N, rp, col, val)
    _products(ctx, A, O, np.random.default_rng(SEED))
    with tuning(flags):
        _gmres_vs_oracle(ctx, oracle, A, O, O.mult(np.ones(N)), max_it=75)


def _unsymmetric(rp, col, val, seed=SEED):
    """The same operator with a few upper entries scaled: no longer symmetric, so it keeps the seven legs."""
    val = val.copy()
    rows = np.repeat(np.arange(rp.size - 1), np.diff(rp))
    upper = np.flatnonzero(col > rows)
    pick = np.random.default_rng(seed).choice(upper, size=max(1, upper.size // 1000), replace=False)
    val[pick] *= 1.5
    return val


@pytest.mark.parametrize("layout", ["sym", "sym-one", "blocked", "soa", "blocked-unsym"])
@pytest.mark.parametrize("flags", [0, BOX_SEPARATE])
@pytest.mark.parametrize("shape", [(64, 64, 16), (128, 32, 9), (64, 64, 2), (2048, 2, 3), (1024, 4, 5)])
def test_variable_coefficient_box_takes_the_stencil_storage(ctx, oracle, shape, flags, layout, monkeypatch):
    """A box stencil with variable coefficients (utils.heterogeneous_poisson3d) whose planes hold whole 4096-row
    chunks: no dictionary fits, so msp_mat_create_csr gives it the STENCIL storage (a presence byte and the row's
    seven values per row, k_box_march_chunk_rv; in GMRES the MatMult fused with the VecMDot, W stored).  MatMult,
    MatResidual and GMRES(30) over 3 restart cycles equal the oracle bit for bit -- with the fused step (0) and
    with the separate MatMult (BOX_SEPARATE), in both value layouts -- and switching to CSR gives the same
    products."""
    from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d
    from test_gpu_kernels import tuning
    nx, ny, nz = shape
    rp, col, val = heterogeneous_poisson3d(nx, ny, nz)
    N = nx * ny * nz
    # the value layout chosen at assembly: symmetric (the diagonal and upper legs; the default for a symmetric
    # operator with planes up to 1024 wide), chunk-blocked seven legs (MSPLIT_RV_SYM=0, or an unsymmetric operator),
    # or per-leg arrays (MSPLIT_RV_LAYOUT=soa)
    # sym: the fused step with two threads per DBR lane where nx <= 512 (k_box_spmv_mdot_march_sym2); sym-one: the
    # one-thread form (MSPLIT_RV_SYM2=0)
    monkeypatch.setenv("MSPLIT_RV_LAYOUT", "soa" if layout == "soa" else "blocked")
    monkeypatch.setenv("MSPLIT_RV_SYM", "0" if layout == "blocked" else "1")
    monkeypatch.setenv("MSPLIT_RV_SYM2", "0" if layout == "sym-one" else "1")
    if layout == "blocked-unsym":
        val = _unsymmetric(rp, col, val)
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    sym = layout.startswith("sym") and nx <= 1024
    assert A.get_storage() == "stencil"
    assert A.spmv_kernel() == ("k_box_march_chunk_rv_sym" if sym else "k_box_march_chunk_rv")
    O = oracle.Mat.from_arrays(N, N, rp, col, val)
    y, res = _products(ctx, A, O, np.random.default_rng(SEED))
    with tuning(flags):
        _gmres_vs_oracle(ctx, oracle, A, O, O.mult(np.ones(N)), max_it=75)
    A.set_storage("csr")
    yc, rc = _products(ctx, A, O, np.random.default_rng(SEED))
    assert np.array_equal(y, yc) and np.array_equal(res, rc)
    A.set_storage("stencil")
    assert A.get_storage() == "stencil"


@pytest.mark.parametrize("defect", ["dropped", "wrapped", "eighth_offset", "odd_nx"])
def test_stencil_storage_edge_cases(ctx, oracle, defect):
    """Entries left out of some rows still take the STENCIL storage (the presence bytes say which neighbours a row
    holds) and equal the oracle; a row holding a neighbour across a line edge (x-1 at i = 0), an eighth column
    offset, or a box whose plane rows the chunk march cannot tile (odd nx) keep CSR, still bitwise the oracle."""
    from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d
    nx, ny, nz = (64, 64, 6) if defect != "odd_nx" else (3, 4096, 2)
    rp, col, val = heterogeneous_poisson3d(nx, ny, nz)
    N = nx * ny * nz
    rows = np.repeat(np.arange(N), np.diff(rp))
    if defect == "dropped":
        keep = (np.random.default_rng(SEED).random(col.size) > 0.2) | (rows == col)
        rows, col, val = rows[keep], col[keep], val[keep]
    elif defect in ("wrapped", "eighth_offset"):
        r0 = 3 * nx * ny + 5 * nx                          # i = 0 of an interior line
        c_new = r0 - 1 if defect == "wrapped" else r0 + 2
        rows, col, val = np.append(rows, r0), np.append(col, c_new), np.append(val, -0.25)
        order = np.lexsort((col, rows))
        rows, col, val = rows[order], col[order], val[order]
    rp = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=N))]).astype(np.int32)
    col = col.astype(np.int32)
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    O = oracle.Mat.from_arrays(N, N, rp, col, val)
    assert A.get_storage() == ("stencil" if defect == "dropped" else "csr")
    _products(ctx, A, O, np.random.default_rng(SEED))
    _gmres_vs_oracle(ctx, oracle, A, O, O.mult(np.random.default_rng(SEED).uniform(-1, 1, N)), max_it=40)


def test_stencil_storage_selectable_under_csr_default(ctx, oracle, monkeypatch):
    """MSPLIT_MAT_STORAGE=csr keeps the products in CSR at assembly, but the STENCIL storage is still built (as the
    DV storage is), so msp_mat_set_storage can switch to it later -- bitwise the same products; a
    symmetric operator is sized for its four legs."""
    from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d
    nx, ny, nz = 64, 64, 8
    rp, col, val = heterogeneous_poisson3d(nx, ny, nz)
    N = nx * ny * nz
    monkeypatch.setenv("MSPLIT_MAT_STORAGE", "csr")
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    assert A.get_storage() == "csr"
    O = oracle.Mat.from_arrays(N, N, rp, col, val)
    y, res = _products(ctx, A, O, np.random.default_rng(SEED))
    A.set_storage("stencil")
    assert A.get_storage() == "stencil" and A.spmv_kernel() == "k_box_march_chunk_rv_sym"
    ys, rs = _products(ctx, A, O, np.random.default_rng(SEED))
    assert np.array_equal(y, ys) and np.array_equal(res, rs)


@pytest.mark.parametrize("alt", ["1", "0"])
@pytest.mark.parametrize("layout", ["sym", "sym-one", "blocked-unsym"])
@pytest.mark.parametrize("shape", [(64, 64, 16), (128, 32, 9), (256, 16, 13)])
def test_stencil_fused_march_direction_bitwise(ctx, oracle, shape, layout, alt, monkeypatch):
    """The STENCIL storage's fused MatMult+MDot with odd plane groups marching down (MSPLIT_BOXMDOT_ALT; the
    symmetric two-thread kernel then loads the z+1 legs of the plane below with its x, and carries the plane's own
    upward): GMRES(30) over 75 iterations bitwise the oracle in both march orders."""
    from medane_tchakorom_ufc_thesis_repository_amd.utils import heterogeneous_poisson3d
    monkeypatch.setenv("MSPLIT_BOXMDOT_ALT", alt)  # 1: alternating, 0: up only
    monkeypatch.setenv("MSPLIT_RV_LAYOUT", "blocked")
    monkeypatch.setenv("MSPLIT_RV_SYM", "1")
    monkeypatch.setenv("MSPLIT_RV_SYM2", "0" if layout == "sym-one" else "1")
    nx, ny, nz = shape
    rp, col, val = heterogeneous_poisson3d(nx, ny, nz)
    if layout == "blocked-unsym":
        val = _unsymmetric(rp, col, val)
    N = nx * ny * nz
    A = Mat.from_csr(ctx, N, N, rp, col, val)
    assert A.get_storage() == "stencil"
    O = oracle.Mat.from_arrays(N, N, rp, col, val)
    _gmres_vs_oracle(ctx, oracle, A, O, O.mult(np.ones(N)), max_it=75)
