"""Host glue of the reference's inner-solve path, restated over the HIP objects.

Names follow the reference (src/utils/utils.c) so that a reader can put the
two side by side.  Assembly here is vectorised numpy producing the same CSR
(ascending columns per row, PETSc AIJ) the reference's MatSetValues loops
produce; large operators are assembled on the device instead
(petsc.Mat.box_stencil).  Blocks are generalised from the reference's 2 to nb
(z-slabs in 3D, whole mesh lines in 2D), one block per GPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .petsc import KSP, LSQR, Context, Mat, Options, Vec


# ------------------------------------------------------------------ dimensions
def computeDimensionRelatedVariables(nprocs, nprocs_per_jacobi_block, proc_global_rank, n_mesh_lines, n_mesh_columns):
    """utils.c:652-666 -> (njacobi_blocks, rank_jacobi_block, proc_local_rank,
    n_mesh_points, jacobi_block_size).  2D as in the reference (utils.c:662)."""
    njacobi_blocks = nprocs // nprocs_per_jacobi_block
    rank_jacobi_block = proc_global_rank // nprocs_per_jacobi_block
    proc_local_rank = proc_global_rank % nprocs_per_jacobi_block
    n_mesh_points = n_mesh_lines * n_mesh_columns
    jacobi_block_size = n_mesh_points // njacobi_blocks
    return njacobi_blocks, rank_jacobi_block, proc_local_rank, n_mesh_points, jacobi_block_size


# -------------------------------------------------------------------- assembly
def _csr_from_entries(nrows, rows, cols, vals):
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    rowptr = np.zeros(nrows + 1, np.int64)
    np.add.at(rowptr, rows + 1, 1)
    rowptr = np.cumsum(rowptr)
    return rowptr.astype(np.int32), cols.astype(np.int32), vals.astype(np.float64)


def poisson3DMatrix_rows(nx, ny, nz, z0, z1):
    """Rows of planes [z0,z1) of poisson3DMatrix (utils.c:30-121), global
    columns; local row = global row - z0*nx*ny.  Returns (rowptr, col, val, ncols)."""
    nxny = nx * ny
    k, j, i = np.meshgrid(np.arange(z0, z1), np.arange(ny), np.arange(nx), indexing="ij")
    i, j, k = i.ravel(), j.ravel(), k.ravel()
    g = (i + j * nx + k * nxny).astype(np.int64)
    lr = g - z0 * nxny
    parts = [(lr, g, np.full(g.size, 6.0))]
    for mask, off in ((k > 0, -nxny), (j > 0, -nx), (i > 0, -1), (i < nx - 1, 1), (j < ny - 1, nx),
                      (k < nz - 1, nxny)):
        parts.append((lr[mask], g[mask] + off, np.full(int(mask.sum()), -1.0)))
    rows = np.concatenate([p[0] for p in parts])
    cols = np.concatenate([p[1] for p in parts])
    vals = np.concatenate([p[2] for p in parts])
    rp, c, v = _csr_from_entries(int(g.size), rows, cols, vals)
    return rp, c, v, nxny * nz


def _splitmix64(x):
    z = x + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def heterogeneous_poisson3d(nx: int, ny: int | None = None, nz: int | None = None, seed: int = 20251121):
    """An assembled AIJ operator with variable coefficients: -div(kappa grad u) on the nx x ny x nz grid (ny, nz
    default to nx), 7 points, in the reference's numbering (x fastest, as poisson3DMatrix, utils.c:30-121).
    kappa per cell is 1 + (h mod 1000) / 1000, h a splitmix64 hash of (cell index + seed); the face between two
    cells weighs 2 ka kb / (ka + kb), a boundary face the cell's own kappa (Dirichlet), the diagonal is the sum
    of the six face weights in the order z-, y-, x-, x+, y+, z+, the neighbours -weight.  Only IEEE + - * / (no
    libm), so the arrays are the same bits on every machine.  Almost every row holds its own values, so no
    (column - row, value) dictionary fits: the library stores it as the box stencil it is (MSP_STORAGE_STENCIL,
    per-row values) when its planes hold whole 4096-row chunks, else as CSR -- the general AIJ a PETSc user
    assembles (bench.py non_stencil_aij).  Returns (rowptr int32, col int32, val float64), columns ascending."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    P = nx * ny
    N = P * nz
    with np.errstate(over="ignore"):
        h = _splitmix64(np.arange(N, dtype=np.uint64) + np.uint64(seed))
    kap = (1.0 + (h % np.uint64(1000)).astype(np.float64) * 0.001).reshape(nz, ny, nx)   # [k, j, i]

    def face(axis, side):
        nb = np.roll(kap, -side, axis=axis)
        w = 2.0 * kap * nb / (kap + nb)
        edge = [slice(None)] * 3
        edge[axis] = -1 if side > 0 else 0
        w[tuple(edge)] = kap[tuple(edge)]                # boundary face: Dirichlet, the cell's own kappa
        return w.ravel()
    wzm, wym, wxm = face(0, -1), face(1, -1), face(2, -1)
    wxp, wyp, wzp = face(2, 1), face(1, 1), face(0, 1)
    diag = ((((wzm + wym) + wxm) + wxp) + wyp) + wzp
    g = np.arange(N, dtype=np.int64)
    i, j, k = g % nx, (g // nx) % ny, g // P
    cols = np.stack([g - P, g - nx, g - 1, g, g + 1, g + nx, g + P], axis=1)
    vals = np.stack([-wzm, -wym, -wxm, diag, -wxp, -wyp, -wzp], axis=1)
    keep = np.stack([k > 0, j > 0, i > 0, np.ones(N, bool), i < nx - 1, j < ny - 1, k < nz - 1], axis=1)
    rowptr = np.concatenate([[0], np.cumsum(keep.sum(axis=1))]).astype(np.int32)
    return rowptr, cols[keep].astype(np.int32), vals[keep]


def poisson2DMatrix_rows(m, n, row0, row1):
    """Rows [row0,row1) of poisson2DMatrix (utils.c:247-293): i = Ii / n,
    j = Ii - i*n, diagonal 4.  Returns (rowptr, col, val, ncols)."""
    Ii = np.arange(row0, row1, dtype=np.int64)
    i = Ii // n
    j = Ii - i * n
    lr = Ii - row0
    parts = [(lr, Ii, np.full(Ii.size, 4.0))]
    for mask, off in ((i > 0, -n), (i < m - 1, n), (j > 0, -1), (j < n - 1, 1)):
        parts.append((lr[mask], Ii[mask] + off, np.full(int(mask.sum()), -1.0)))
    rows = np.concatenate([p[0] for p in parts])
    cols = np.concatenate([p[1] for p in parts])
    vals = np.concatenate([p[2] for p in parts])
    rp, c, v = _csr_from_entries(int(Ii.size), rows, cols, vals)
    return rp, c, v, m * n


def poisson2DMatrix_complete(m, n):
    """poisson2DMatrix_complete (utils.c:383-445): square mesh, Ii = i*m + j."""
    if m != n:
        raise ValueError("poisson2DMatrix_complete assumes a square mesh (utils.c:390)")
    return poisson2DMatrix_rows(m, n, 0, m * n)


def split_columns(rowptr, col, val, c0, c1):
    """divideSubDomainIntoBlockMatrices (utils.c:450-478): own columns [c0,c1)
    -> A_ii (local columns), the rest -> coupling rows (global columns)."""
    nrows = rowptr.size - 1
    rows = np.repeat(np.arange(nrows), np.diff(rowptr))
    own = (col >= c0) & (col < c1)
    rp_i, c_i, v_i = _csr_from_entries(nrows, rows[own], col[own] - c0, val[own])
    rp_o, c_o, v_o = _csr_from_entries(nrows, rows[~own], col[~own], val[~own])
    return (rp_i, c_i, v_i), (rp_o, c_o, v_o)


# -------------------------------------------------------------- block layout
@dataclass
class BlockLayout:
    """One multisplitting block (one GPU): rows [r0,r1) of the global operator,
    its halo (entries of neighbouring blocks its coupling rows read), what it
    sends to each neighbour, and the coupling block in halo numbering."""
    dim: int
    nx: int
    ny: int
    nz: int
    nb: int
    b: int
    r0: int
    r1: int
    plane: int                                  # entries per coupling plane / line
    recv: list = field(default_factory=list)   # (nbr, halo_off, count, nbr_local_off)
    send: list = field(default_factory=list)   # (nbr, local_off, count)
    halo_size: int = 0
    coupling: tuple = ()                        # (row_ids, rowptr, col(halo idx), val)
    peclet: tuple = (0.0, 0.0, 0.0)             # operator: Poisson (0) or upwind convection-diffusion

    @property
    def nrows(self):
        return self.r1 - self.r0

    @property
    def box(self):
        """(dim, nx, ny, nz) of the box stencil equal to this block's A_ii."""
        if self.dim == 3:
            return 3, self.nx, self.ny, self.nrows // (self.nx * self.ny)
        return 2, self.ny, self.nrows // self.ny, 1


def convdiff_coefs(dim, peclet=None):
    """The 7 stencil values (slow-, y-, x-, diagonal, x+, y+, slow+) of the upwind
    convection-diffusion operator h^2(-Lap u + beta.grad u) in cell Peclet numbers
    P_d = beta_d h / 2 (x fastest; 2D: x and the line direction).  P = 0 is the
    reference's Poisson stencil exactly (msplit.h, msp_mat_create_box_convdiff)."""
    px, py, pz = (tuple(float(v) for v in peclet) + (0.0, 0.0, 0.0))[:3] if peclet is not None else (0.0, 0.0, 0.0)
    if dim == 2:
        pz = 0.0
    cm = lambda p: -1.0 - 2.0 * max(p, 0.0)
    cp = lambda p: -1.0 + 2.0 * min(p, 0.0)
    if dim == 3:
        return [cm(pz), cm(py), cm(px), ((6.0 + 2.0 * abs(px)) + 2.0 * abs(py)) + 2.0 * abs(pz),
                cp(px), cp(py), cp(pz)]
    return [cm(py), 0.0, cm(px), (4.0 + 2.0 * abs(px)) + 2.0 * abs(py), cp(px), 0.0, cp(py)]


def block_layout(dim, nx, ny, nz, nb, b, peclet=None) -> BlockLayout:
    """Slab partition of the reference's stencil into nb blocks.
    dim 3: nx x ny x nz grid, block b = planes [b*nz/nb, (b+1)*nz/nb).
    dim 2: m = nx mesh lines x n = ny mesh columns (poisson2DMatrix numbering),
    block b = rows [b*N/nb, (b+1)*N/nb), whole mesh lines only.
    peclet: the convection-diffusion operator's coupling values instead of -1."""
    if dim == 3:
        if nz % nb:
            raise ValueError(f"nz={nz} must be divisible by the number of blocks {nb}")
        plane = nx * ny
        ppb = nz // nb
        r0, r1 = b * ppb * plane, (b + 1) * ppb * plane
    elif dim == 2:
        N = nx * ny
        if N % nb or (N // nb) % ny:
            raise ValueError("2D blocks must hold whole mesh lines (N/nb a multiple of n_grid_columns)")
        plane = ny
        r0, r1 = b * (N // nb), (b + 1) * (N // nb)
    else:
        raise ValueError("dim must be 2 or 3")
    L = BlockLayout(dim, nx, ny, nz if dim == 3 else 1, nb, b, r0, r1, plane)
    nloc = r1 - r0
    off = 0
    rows_lo = rows_hi = np.zeros(0, np.int64)
    if b > 0:
        L.recv.append((b - 1, off, plane, nloc - plane))     # neighbour's last plane
        L.send.append((b - 1, 0, plane))                     # my first plane
        rows_lo = np.arange(plane, dtype=np.int64)           # local rows coupling down
        lo_off = off
        off += plane
    if b < nb - 1:
        L.recv.append((b + 1, off, plane, 0))                # neighbour's first plane
        L.send.append((b + 1, nloc - plane, plane))          # my last plane
        rows_hi = np.arange(nloc - plane, nloc, dtype=np.int64)
        hi_off = off
        off += plane
    L.halo_size = off
    L.peclet = tuple(peclet) if peclet is not None else (0.0, 0.0, 0.0)
    cf = convdiff_coefs(dim, peclet)
    # coupling rows: row l couples to halo lo_off + l (below) and/or hi_off + (l - (nloc-plane)) (above);
    # halo numbering is ascending in global column, so per-row column order is PETSc's.
    ent_r, ent_c, ent_v = [], [], []
    if rows_lo.size:
        ent_r.append(rows_lo)
        ent_c.append(lo_off + rows_lo)
        ent_v.append(np.full(rows_lo.size, cf[0]))
    if rows_hi.size:
        ent_r.append(rows_hi)
        ent_c.append(hi_off + (rows_hi - (nloc - plane)))
        ent_v.append(np.full(rows_hi.size, cf[6]))
    if ent_r:
        r = np.concatenate(ent_r)
        c = np.concatenate(ent_c)
        v = np.concatenate(ent_v)
        order = np.lexsort((c, r))
        r, c, v = r[order], c[order], v[order]
        row_ids, counts = np.unique(r, return_counts=True)
        rowptr = np.concatenate([[0], np.cumsum(counts)])
        L.coupling = (row_ids.astype(np.int32), rowptr.astype(np.int32), c.astype(np.int32), v)
    else:
        L.coupling = (np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0))
    return L


# --------------------------------------------------------------- solver glue
def initializeKSP(ctx: Context, A: Mat, zero_initial_guess: bool, ksp_prefix: str | None,
                  opts: Options | None) -> KSP:
    """utils.c:512-541: KSPCreate; SetOperators; SetOptionsPrefix;
    SetInitialGuessNonzero(!zero); SetFromOptions."""
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_options_prefix(ksp_prefix)
    ksp.set_initial_guess_nonzero(not zero_initial_guess)
    ksp.set_from_options(opts or Options())
    return ksp


def initializeOuterKSP(ctx: Context, ksp_prefix: str | None, opts: Options | None) -> LSQR:
    """initializeKSP(comm, &outer_ksp, NULL, .., PETSC_TRUE, "outer1_"/"outer2_", ..)
    (SMSM-global.c:219): the outer least-squares solver, zero initial guess,
    configured from the options database (-outer1_ksp_type lsqr ...)."""
    ksp = LSQR(ctx)
    ksp.set_options_prefix(ksp_prefix)
    ksp.set_from_options(opts or Options())
    return ksp


def inner_solver(ksp: KSP, rhs: Vec, x: Vec) -> int:
    """utils.c:950-970: UIRNorm convergence, nonzero initial guess, KSPSolve;
    returns the iteration count."""
    ksp.converged_default_set_uirnorm()
    ksp.set_initial_guess_nonzero(True)
    ksp.solve(rhs, x)
    return ksp.get_iteration_number()


def updateLocalRHS(A_off: Mat, halo: Vec, b_block: Vec, rhs: Vec, rhs_holds_b: bool = False):
    """utils.c:943-948: rhs = b_i - A_ij x_j (MatResidual), x_j = the halo.  rhs_holds_b: rhs already equals
    b_i in the rows A_off lists no entry for (b_i - 0 = b_i), so only the coupled rows are recomputed -- the same
    bits without the 16 B/row copy of b."""
    if rhs_holds_b:
        A_off.residual_listed(b_block, halo, rhs)
    else:
        A_off.residual(b_block, halo, rhs)
