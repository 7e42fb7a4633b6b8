"""Synchronous multisplitting drivers over the GPU inner solve.

sm_solve mirrors src/synchronous-multisplitting/synchronous-multisplitting.c:
setup (:101-164), the outer loop (:170-206) and the final report (:208-229);
smsm_solve mirrors the global-minimization variant,
src/synchronous-multisplitting-synchronous-minimization-global/
synchronous-multisplitting-synchronous-minimization-global.c (setup :134-284,
loop :288-363).  Both are generalised from 2 blocks to nb z-slab (3D) or
mesh-line (2D) blocks, one per GPU.  Each block's inner solve is GMRES on its diagonal block A_ii
(inner_solver, utils.c:950-970) running entirely in that GPU's HBM; the only
traffic between blocks is the boundary-plane exchange and one scalar per block
per outer iteration (comm.py).

The driver itself is backend-agnostic: it calls the block operations below,
which GpuBlock implements with the HIP library.  (tests/ drive the same loop
with a CPU test double to cover the multi-rank logic on gloo.)
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

from .petsc import Context, DenseMat, Mat, Options, Vec
from .utils import BlockLayout, block_layout, initializeKSP, initializeOuterKSP, inner_solver, updateLocalRHS


class GpuBlock:
    """One multisplitting block in HBM: A_ii (assembled on the device), the
    coupling rows A_ij, b_i, x_i, the local right-hand side, the halo and the
    inner KSP (prefix inner{b+1}_, synchronous-multisplitting.c:129-143)."""

    async_transport = "device"   # asynchronous.py: planes and R rows through HBM slots (xGMI peer copies)

    def __init__(self, ctx: Context, layout: BlockLayout, opts: Options | None, comm, prefix: str | None = None):
        self.ctx = ctx
        self.layout = layout
        n = layout.nrows
        dim, bx, by, bz = layout.box
        self.peclet = tuple(getattr(layout, "peclet", (0.0, 0.0, 0.0)))
        # -msplit_operator matfree: A_ii applied without storage (bitwise the assembled products)
        if opts is not None and opts.get_string("msplit_operator", "csr") == "matfree":
            self.A = Mat.box_matfree(ctx, dim, bx, by, bz, False, False, self.peclet)
        else:
            self.A = Mat.box_convdiff(ctx, dim, bx, by, bz, False, False, self.peclet)
        # DV storage holds the operator in ~1 byte per entry; its CSR copy is freed unless -msplit_keep_csr
        self._release_csr = not (opts is not None and opts.get_bool("msplit_keep_csr", False))
        self._maybe_release_csr(self.A)
        row_ids, rowptr, col, val = layout.coupling
        self.A_off = Mat.from_csr_rows(ctx, n, layout.halo_size, row_ids, rowptr, col, val)
        self.halo, self.halo_t = comm.alloc(ctx, layout.halo_size)
        self.send_bufs = {nbr: comm.alloc(ctx, cnt) for nbr, _, cnt in layout.send}
        self._send_spec = {nbr: (off, cnt) for nbr, off, cnt in layout.send}
        self._recv_spec = {nbr: (hoff, cnt) for nbr, hoff, cnt, _ in layout.recv}
        self._device_bufs = getattr(comm, "device_buffers", True)
        self.b = Vec(ctx, n)
        self.x = Vec(ctx, n)
        self.rhs = Vec(ctx, n)
        self._rhs_holds_b = False
        self.r = Vec(ctx, n)
        # computeTheRightHandSideWithInitialGuess (utils.c:623-650): b_i = A_block u, u = 1,
        # over the block's full rows in ascending-column order (MatMult_SeqAIJ)
        self._ensure_ext()
        ones = Vec(ctx, self.lo_rows + n + self.hi_rows)
        ones.set(1.0)
        self.A_ext.mult(ones, self.b)
        del ones
        self.prefix = prefix if prefix is not None else f"inner{layout.b + 1}_"
        self.opts = opts
        self.ksp = initializeKSP(ctx, self.A, False, self.prefix, opts)
        self.last_its = 0

    # -- exchange hooks (comm.py)
    def pack_send(self, nbr):
        """The plane(s) neighbour nbr's coupling rows read, as a torch tensor."""
        off, cnt = self._send_spec[nbr]
        vec, t = self.send_bufs[nbr]
        if self._device_bufs:                       # HBM buffer shared with torch (RCCL)
            self.x.copy_range_to(off, vec, 0, cnt)
            self.ctx.synchronize()
            return t[:cnt]
        import torch
        t[:cnt] = torch.from_numpy(self.x.get_array(off, cnt))
        return t[:cnt]

    def recv_buffer(self, nbr):
        hoff, cnt = self._recv_spec[nbr]
        return self.halo_t[hoff:hoff + cnt]

    def unpack_recv(self):
        if not self._device_bufs and self.layout.halo_size:
            self.halo.set_values(self.halo_t[:self.layout.halo_size].numpy())

    def copy_halo_from(self, by_id):
        """LocalComm: neighbour blocks in this process, device-to-device."""
        for nbr, hoff, cnt, nbr_off in self.layout.recv:
            by_id[nbr].x.copy_range_to(nbr_off, self.halo, hoff, cnt)

    # -- block operations used by the driver
    def reset_halo(self):
        """x_j = 0 before the first exchange (vectors are zero-initialised)."""
        self.halo.set(0.0)

    def norm0_sq(self) -> float:
        """computeFinalResidualNorm at x = 0 (utils.c:575-595): ||b_i - A 0||^2 = ||b_i||^2."""
        ln = self.b.norm()
        return ln * ln

    def update_rhs(self):
        # the first update writes every row (rhs = b - A_off halo); rhs is written nowhere else and b is fixed
        # at construction, so later updates recompute the coupled rows only (bitwise the full MatResidual)
        updateLocalRHS(self.A_off, self.halo, self.b, self.rhs,
                       rhs_holds_b=self._rhs_holds_b and os.environ.get("MSPLIT_RHS_FULL", "0") == "0")
        self._rhs_holds_b = True                         # A_off is row-compressed (Mat.from_csr_rows)

    def solve(self) -> int:
        self.last_its = inner_solver(self.ksp, self.rhs, self.x)
        return self.last_its

    def local_residual_sq(self) -> float:
        """MatResidual(A_ii, rhs, x) + VecNorm, squared (synchronous-multisplitting.c:187-191)."""
        self.A.residual(self.rhs, self.x, self.r)
        ln = self.r.norm()
        return ln * ln

    # -- global minimization (SMSM-global) hooks
    def setup_minimization(self, s: int):
        """S (the s latest iterates, with the neighbour planes R = A S reads) and
        R = A S in HBM, and A_ext = this block's rows of A_block_jacobi with the
        coupling columns (create_redistributed_A_block_jacobi, utils.c:891-921)."""
        L = self.layout
        self.s = int(s)
        self._ensure_ext()
        self.S = DenseMat(self.ctx, self.lo_rows + L.nrows + self.hi_rows, self.s)
        self.R = DenseMat(self.ctx, L.nrows, self.s)

    def _ensure_ext(self):
        """A_ext: the block's full rows of A_block_jacobi, coupling columns kept."""
        if getattr(self, "A_ext", None) is not None:
            return
        L = self.layout
        self.lo_rows = L.plane if any(nbr < L.b for nbr, *_ in L.recv) else 0
        self.hi_rows = L.plane if any(nbr > L.b for nbr, *_ in L.recv) else 0
        dim, bx, by, bz = L.box
        self.A_ext = Mat.box_convdiff(self.ctx, dim, bx, by, bz, self.lo_rows > 0, self.hi_rows > 0,
                                      getattr(self, "peclet", (0.0, 0.0, 0.0)))
        self._maybe_release_csr(self.A_ext)

    def _maybe_release_csr(self, M):
        if getattr(self, "_release_csr", False) and M.get_storage() == "dv":
            M.release_csr()

    # -- local minimization (SMSM-local, AMAM-local) hooks
    def setup_local_minimization(self, s: int, opts: Options | None, prefix: str | None = None):
        """S_i (the block's own s latest iterates), R_i = A_ii S_i and a one-block
        LSQR (create_matrix_dense of N/nb x s, SMSM-local.c / AMAM-local_prime.c:246-253;
        outer KSP prefix outer{b+1}_)."""
        self.s = int(s)
        n = self.layout.nrows
        self.S_loc = DenseMat(self.ctx, n, self.s)
        self.R_loc = DenseMat(self.ctx, n, self.s)
        self.alpha_loc = Vec(self.ctx, self.s)
        self.lsqr_loc = initializeOuterKSP(self.ctx, prefix if prefix is not None else f"outer{self.layout.b + 1}_",
                                           opts)
        self.lsqr_loc.set_operators([self.R_loc])

    def store_local_column(self, k: int):
        """S_i(:, k) = x_i (MatSetValues(S, .., k, x_i))."""
        self.S_loc.set_column(k, 0, self.x)

    def local_minimize(self):
        """R_i = A_ii S_i, rhs_i = b_i - A_ij x_j, alpha = LSQR(R_i, rhs_i), x_i = S_i alpha
        (SMSM-local.c / AMAM-local_prime.c:400-404)."""
        self.A.mat_mult_dense(self.S_loc, self.R_loc)
        self.update_rhs()
        self.lsqr_loc.solve([self.rhs], self.alpha_loc)
        self.S_loc.mult(self.alpha_loc, self.x)
        return (self.lsqr_loc.get_residual_norm(), self.lsqr_loc.get_iteration_number(),
                self.lsqr_loc.get_converged_reason())

    # -- semi-local minimization (SMSM-semi-local, AMAM-semi-local)
    def semi_local_minimize(self, apply: bool = True):
        """R_i = A_block S_i (own rows of the global R), alpha_i = LSQR(R_i, b_i)
        (outer_solver_norm_equation_modify, utils.c:1080-1103), x_minimized = S_i alpha_i
        over the block's rows and neighbour planes; apply: x_i and the halo take it
        (SMSM-semi-local.c:332-335; the asynchronous variant never applies it)."""
        if getattr(self, "lsqr_semi", None) is None:
            self.lsqr_semi = initializeOuterKSP(self.ctx, f"outer{self.layout.b + 1}_", self.opts)
            self.lsqr_semi.set_operators([self.R])
            self.alpha_semi = Vec(self.ctx, self.s)
        self.form_R()
        self.lsqr_semi.solve([self.b], self.alpha_semi)
        if apply:
            self.apply_alpha(self.alpha_semi)
        else:                                                  # computed and dropped, as the reference does
            if getattr(self, "xmin_scratch", None) is None:
                self.xmin_scratch = Vec(self.ctx, self.lo_rows + self.layout.nrows + self.hi_rows)
            self.S.mult(self.alpha_semi, self.xmin_scratch)
        return (self.lsqr_semi.get_residual_norm(), self.lsqr_semi.get_iteration_number(),
                self.lsqr_semi.get_converged_reason())

    # -- global asynchronous minimization (AMAM-global)
    MINIMIZATIONS = ("lsqr", "rtr")

    def setup_global_async_minimization(self, s: int, opts: Options | None = None, prefix: str | None = None,
                                        minimization: str | None = None):
        """AMAM-global_prime.c:238-330: S over the block's rows and neighbour planes,
        this block's rows of R, the replicated R -- every block's rows, zero until
        that block's first message arrives (MatZeroEntries(R)) --, the global b and
        the outer LSQR over the nb row blocks in block order.

        minimization "rtr" (-msplit_minimization rtr) is the reference's outer_solver
        (utils.c:972-996) instead of outer_solver_norm_equation: each block forms
        G_b = R_b^T R_b and c_b = R_b^T b_b in one pass over its rows (msp_dense_gram) and
        publishes those s(s+1) doubles newest-value; every block sums the newest parts in
        block order (zeros before a block's first message: R_j = 0 gives G_j = 0) and runs
        the outer KSP (lsqr, the same options) on G alpha = c.  No replicated R or b: a
        block holds its own rows only, whatever the block count."""
        L = self.layout
        self.setup_minimization(s)
        if minimization is None:
            o = opts if opts is not None else self.opts
            minimization = o.get_string("msplit_minimization", "lsqr").lower() if o is not None else "lsqr"
        if minimization not in self.MINIMIZATIONS:
            raise ValueError(f"-msplit_minimization {minimization}: expected one of {self.MINIMIZATIONS}")
        self.minimization = minimization
        pfx = prefix if prefix is not None else f"outer{L.b + 1}_"
        if minimization == "rtr":
            self.Gc = DenseMat(self.ctx, self.s, self.s + 1)              # [R_b^T R_b | R_b^T b_b]
            self.Gc_rep = []
            for j in range(L.nb):                                         # newest part of every block
                if j == L.b:
                    self.Gc_rep.append(self.Gc)
                else:
                    G = DenseMat(self.ctx, self.s, self.s + 1)
                    G.zero_entries()
                    self.Gc_rep.append(G)
            self.Gsum = DenseMat(self.ctx, self.s, self.s + 1)
            self.G_op = self.Gsum.view(0, self.s)                         # R_transpose_R
            self.c_rhs = self.Gsum.column_vec(self.s)                     # vec_R_transpose_b_block_jacobi
            self.lsqr_glob = initializeOuterKSP(self.ctx, pfx, opts if opts is not None else self.opts)
            self.lsqr_glob.set_operators([self.G_op])
            self.alpha_glob = Vec(self.ctx, self.s)
            return
        self.R_rep, self.b_all = [], []
        for j in range(L.nb):
            if j == L.b:
                self.R_rep.append(self.R)
                self.b_all.append(self.b)
                continue
            Lj = block_layout(L.dim, L.nx, L.ny, L.nz, L.nb, j, L.peclet)
            R = DenseMat(self.ctx, Lj.nrows, self.s)
            R.zero_entries()
            self.R_rep.append(R)
            lo = any(nbr < j for nbr, *_ in Lj.recv)
            hi = any(nbr > j for nbr, *_ in Lj.recv)
            A = Mat.box_convdiff(self.ctx, *Lj.box, lo, hi, L.peclet)   # b_j = A_block_j 1 (utils.c:623-650)
            ones = Vec(self.ctx, (Lj.plane if lo else 0) + Lj.nrows + (Lj.plane if hi else 0))
            ones.set(1.0)
            bj = Vec(self.ctx, Lj.nrows)
            A.mult(ones, bj)
            self.b_all.append(bj)
            del A, ones
        self.lsqr_glob = initializeOuterKSP(self.ctx, pfx, opts if opts is not None else self.opts)
        self.lsqr_glob.set_operators(self.R_rep)
        self.alpha_glob = Vec(self.ctx, self.s)

    def bcast_cap(self) -> int:
        """Doubles one block publishes per minimization: its rows of R, or its Gram part."""
        if getattr(self, "minimization", "lsqr") == "rtr":
            return self.s * (self.s + 1)
        return self.R.shape[0] * self.R.shape[1]

    def global_async_minimize(self, bcast):
        """AMAM-global_prime.c:415-440: R_i = A_block S, send it (comm_async_test_and_send_min),
        take the newest rows of every other block (comm_async_probe_and_receive_min),
        alpha = LSQR(R, b) over the replicated R (outer_solver_norm_equation,
        utils.c:1061-1078), x_minimized = S alpha into x_i and the neighbour planes."""
        self.form_R()
        if self.minimization == "rtr":                 # outer_solver, utils.c:972-996
            self.R.gram(self.b, self.Gc)               # MatTransposeMatMult + MatMultTranspose (:978-979)
            bcast.publish_dense(self.Gc)
            for j, G in enumerate(self.Gc_rep):
                if j != self.layout.b:
                    bcast.fetch_dense(j, G)
            DenseMat.sum(self.Gc_rep, self.Gsum)       # block order
            self.lsqr_glob.solve([self.c_rhs], self.alpha_glob)   # KSPSolve(outer_ksp, R^T b, alpha) (:982)
            self.apply_alpha(self.alpha_glob)          # MatMult(S, alpha, x_minimized) (:993)
            return (self.lsqr_glob.get_residual_norm(), self.lsqr_glob.get_iteration_number(),
                    self.lsqr_glob.get_converged_reason())
        bcast.publish_dense(self.R)
        for j, R in enumerate(self.R_rep):
            if j != self.layout.b:
                bcast.fetch_dense(j, R)
        self.lsqr_glob.solve(self.b_all, self.alpha_glob)
        self.apply_alpha(self.alpha_glob)
        return (self.lsqr_glob.get_residual_norm(), self.lsqr_glob.get_iteration_number(),
                self.lsqr_glob.get_converged_reason())

    # -- asynchronous (AM) hooks: asynchronous.py
    def async_recv(self, am, nbr, hoff, cnt):
        """The newest plane of neighbour nbr, into a staging copy of the halo
        (comm_async_probe_and_receive_prime receives into a temporary buffer)."""
        if getattr(self, "halo_stage", None) is None:
            self.halo_stage = Vec(self.ctx, max(self.layout.halo_size, 1))
        got, ints, _ = am.recv_vec(nbr, 2, self.halo_stage, hoff, cnt)
        return got, (ints[0], ints[1])

    def async_accept(self, hoff, cnt):
        """receive_data_dependency accepted it: copy into x_j's plane."""
        self.halo_stage.copy_range_to(hoff, self.halo, hoff, cnt)

    def async_send(self, am, nbr, off, cnt, tag, it):
        """comm_async_test_and_send_prime: the plane nbr reads, stamped (PhaseTag, iteration)."""
        am.send_vec(nbr, [tag, it], self.x, off, cnt)

    def store_column(self, k: int):
        """S(:, k) = x after the k-th inner solve and exchange (MatSetValuesLocal,
        SMSM-global.c:314-316): own rows and the received neighbour planes."""
        n = self.layout.nrows
        self.S.set_column(k, self.lo_rows, self.x)
        if self.lo_rows:
            self.S.set_column(k, 0, self.halo, 0, self.lo_rows)
        if self.hi_rows:
            self.S.set_column(k, self.lo_rows + n, self.halo, self.lo_rows, self.hi_rows)

    def form_R(self):
        """R = A S (MatMatMult, SMSM-global.c:325-327)."""
        self.A_ext.mat_mult_dense(self.S, self.R)

    def apply_alpha(self, alpha: Vec):
        """x_minimized = S alpha, scattered back into x_i and the neighbour planes
        (SMSM-global.c:349-352 and utils.c:1076): the planes are computed from
        the stored neighbour values with the neighbour's own row arithmetic, so
        they equal what the neighbour computes for those rows."""
        n = self.layout.nrows
        self.S.mult(alpha, self.x, row0=self.lo_rows, n=n)
        if self.lo_rows:
            self.S.mult(alpha, self.halo, row0=0, n=self.lo_rows, yoff=0)
        if self.hi_rows:
            self.S.mult(alpha, self.halo, row0=self.lo_rows + n, n=self.hi_rows, yoff=self.lo_rows)

    def block_residual_sq(self) -> float:
        """||b_i - A_block x||^2 over the block's full rows (computeFinalResidualNorm,
        utils.c:575-595): A_ext applied to [plane below | x_i | plane above]."""
        self._ensure_ext()
        n = self.layout.nrows
        xe = Vec(self.ctx, self.lo_rows + n + self.hi_rows)
        self.x.copy_range_to(0, xe, self.lo_rows, n)
        if self.lo_rows:
            self.halo.copy_range_to(0, xe, 0, self.lo_rows)
        if self.hi_rows:
            self.halo.copy_range_to(self.lo_rows, xe, self.lo_rows + n, self.hi_rows)
        self.A_ext.residual(self.b, xe, self.r)
        ln = self.r.norm()
        return ln * ln

    def error_sq(self) -> float:
        """||x_i - 1||^2 (computeError, utils.c:1045-1059, on this block's rows)."""
        ones = Vec(self.ctx, self.layout.nrows)
        ones.set(1.0)
        d = Vec(self.ctx, self.layout.nrows)
        d.waxpy(-1.0, ones, self.x)
        e = d.norm()
        return e * e


@dataclass
class SMResult:
    outer_its: int = 0
    norm0: float = 0.0
    hist: list = field(default_factory=list)          # outer residual norms
    inner_its: list = field(default_factory=list)     # per outer: [its of each local block]
    error: float = float("nan")
    elapsed: float = 0.0


def fault_stop_rank() -> int:
    """MSPLIT_FAULT_STOP_RANK (the tests' fault injection), read once when a solve sets up; -1: none."""
    v = os.environ.get("MSPLIT_FAULT_STOP_RANK")
    return int(v) if v else -1


def agree_on_stop(comm, outer_its: int, stop: bool, fault: int = -1) -> bool:
    """Every rank must take the same stop decision at the same outer iteration, or the next collective of the
    rank that goes on waits forever for the one that stopped (synchronous-multisplitting.c:187-206 assumes
    agreement).  One all-gather of (outer_its, stop) per outer iteration (comm.agree, msp_comm_agree) turns a
    disagreement -- e.g. from a transport fault -- into an error on every rank.  MSPLIT_FAULT_STOP_RANK=r flips
    rank r's decision at the first outer iteration: the fault injection the tests use."""
    if fault == comm.rank and outer_its == 1:
        stop = not stop
    if comm.world > 1:
        comm.agree(outer_its * 2 + int(stop))
    return stop


def sm_solve(blocks, comm, rtol: float, atol: float = 1e-100, max_outer: int = 10000,
             monitor=None) -> SMResult:
    """The synchronous multisplitting outer loop (synchronous-multisplitting.c:155-206)."""
    res = SMResult()
    fault = fault_stop_rank()
    # global_norm_0 (:162): sqrt of the block-ordered sum of squared local norms
    res.norm0 = math.sqrt(comm.ordered_sum(blocks, [blk.norm0_sq() for blk in blocks]))
    for blk in blocks:                                      # updateLocalRHS before the loop (:164)
        blk.reset_halo()
        blk.update_rhs()
    comm.barrier()
    t0 = time.perf_counter()
    while True:
        its = [blk.solve() for blk in blocks]               # inner_solver (:176)
        comm.exchange(blocks)                               # comm_sync_send_and_receive (:185)
        sq = []
        for blk in blocks:
            blk.update_rhs()                                # updateLocalRHS (:186)
            sq.append(blk.local_residual_sq())              # MatResidual + VecNorm (:187-188)
        norm = math.sqrt(comm.ordered_sum(blocks, sq))      # Allreduce(SUM) on the roots (:192-193)
        res.hist.append(norm)
        res.inner_its.append(its)
        res.outer_its += 1
        if monitor:
            monitor(res.outer_its, norm, its)
        # (:198) and the outer cap, agreed by every rank
        if agree_on_stop(comm, res.outer_its, norm <= max(atol, rtol * res.norm0) or res.outer_its >= max_outer,
                         fault):
            break
    comm.barrier()
    res.elapsed = time.perf_counter() - t0
    res.error = math.sqrt(comm.ordered_sum(blocks, [blk.error_sq() for blk in blocks]))
    return res


class GpuMinimizer:
    """The outer least-squares step of SMSM-global on the GPUs: one KSPLSQR over
    R = A S, row-distributed (each rank its blocks' rows; block partials
    all-gathered, msp_comm), alpha replicated, then x = S alpha on every block
    (outer_solver_norm_equation, utils.c:1061-1078).  prefix: the reference's
    outer{b+1}_ options prefix of the lowest local block."""

    def __init__(self, ctx: Context, blocks, comm, opts: Options | None, prefix: str | None = None):
        self.ctx = ctx
        self.blocks = blocks
        b0 = min(blk.layout.b for blk in blocks)
        self.lsqr = initializeOuterKSP(ctx, prefix if prefix is not None else f"outer{b0 + 1}_", opts)
        self.lsqr.set_operators([blk.R for blk in blocks])
        self.comm = comm.lsqr_comm(ctx) if hasattr(comm, "lsqr_comm") else None
        self._own_comm = getattr(comm, "lsqr_comm_owned", True)   # LibComm shares its communicator
        self.lsqr.set_comm(self.comm)
        self.alpha = Vec(ctx, blocks[0].s)

    def close(self):
        """Release the cross-rank communicator while the process group still runs
        (ncclCommDestroy is collective-free, but must precede the runtime's teardown)."""
        self.ctx.synchronize()
        if self.comm is not None:
            self.lsqr.set_comm(None)
            if self._own_comm:
                self.comm.destroy()
            self.comm = None

    def solve(self, blocks):
        self.lsqr.solve([blk.b for blk in blocks], self.alpha)
        for blk in blocks:
            blk.apply_alpha(self.alpha)
        return (self.lsqr.get_residual_norm(), self.lsqr.get_iteration_number(),
                self.lsqr.get_converged_reason())


@dataclass
class SMSMResult:
    outer_its: int = 0
    norm0: float = 0.0
    hist: list = field(default_factory=list)          # outer LSQR residual norms (the stop test's norm)
    lsqr_its: list = field(default_factory=list)
    lsqr_reason: list = field(default_factory=list)
    inner_its: list = field(default_factory=list)     # per outer: s lists of [its of each local block]
    final_norm: float = float("nan")
    error: float = float("nan")
    elapsed: float = 0.0


def smsm_solve(blocks, comm, s: int, minimizer, rtol: float, atol: float = 1e-100, max_outer: int = 10000,
               monitor=None) -> SMSMResult:
    """SMSM with global minimization (SMSM-global.c:288-363), nb blocks:
    s times {rhs_i = b_i - A_ij x_j; inner GMRES; exchange; S(:,k) = x},
    R = A S, alpha = LSQR(R, b), x = S alpha; stop on the LSQR residual norm."""
    res = SMSMResult()
    fault = fault_stop_rank()
    # global_norm_0 = computeFinalResidualNorm at x = 0 (:280)
    res.norm0 = math.sqrt(comm.ordered_sum(blocks, [blk.norm0_sq() for blk in blocks]))
    for blk in blocks:
        blk.reset_halo()
    comm.barrier()
    t0 = time.perf_counter()
    while True:
        its_outer = []
        for k in range(s):
            for blk in blocks:
                blk.update_rhs()                             # updateLocalRHS (:297)
            its_outer.append([blk.solve() for blk in blocks])  # inner_solver (:299)
            comm.exchange(blocks)                            # comm_sync_send_and_receive (:301)
            for blk in blocks:
                blk.store_column(k)                          # MatSetValuesLocal(S, .., k, x) (:314-316)
        for blk in blocks:
            blk.form_R()                                     # R = A S (:325-327)
        norm, lits, lreason = minimizer.solve(blocks)        # LSQR + x = S alpha (:331-352)
        res.hist.append(norm)
        res.lsqr_its.append(lits)
        res.lsqr_reason.append(lreason)
        res.inner_its.append(its_outer)
        res.outer_its += 1
        if monitor:
            monitor(res.outer_its, norm, its_outer, lits)
        # (:342) and the outer cap, agreed by every rank
        if agree_on_stop(comm, res.outer_its, norm <= max(atol, rtol * res.norm0) or res.outer_its >= max_outer,
                         fault):
            break
    comm.barrier()
    res.elapsed = time.perf_counter() - t0
    res.final_norm = math.sqrt(comm.ordered_sum(blocks, [blk.block_residual_sq() for blk in blocks]))
    res.error = math.sqrt(comm.ordered_sum(blocks, [blk.error_sq() for blk in blocks]))
    return res


def make_blocks(ctx: Context, dim, nx, ny, nz, nb, block_ids, opts: Options | None, comm, peclet=None):
    """GpuBlocks of the Poisson operator, or (peclet) the upwind convection-diffusion one."""
    return [GpuBlock(ctx, block_layout(dim, nx, ny, nz, nb, b, peclet), opts, comm) for b in block_ids]


@dataclass
class LocalMinResult:
    outer_its: int = 0
    norm0: float = 0.0
    hist: list = field(default_factory=list)          # per outer: [local norm of each local block]
    lsqr_its: list = field(default_factory=list)      # per outer: [LSQR its of each local block]
    inner_its: list = field(default_factory=list)     # per outer: s lists of [its of each local block]
    final_norm: float = float("nan")
    error: float = float("nan")
    elapsed: float = 0.0


def smsm_local_solve(blocks, comm, s: int, rtol: float, atol: float = 1e-100, max_outer: int = 10000,
                     monitor=None) -> LocalMinResult:
    """SMSM with local minimization (synchronous-multisplitting-synchronous-minimization-local.c):
    s times {rhs_i; inner GMRES; exchange; S_i(:,k) = x_i}, then R_i = A_ii S_i,
    rhs_i, x_i = S_i LSQR(R_i, rhs_i); stop when every block's ||rhs_i - A_ii x_i||
    <= max(atol, rtol/sqrt(nb) ||b||) (comm_sync_convergence_detection, comm.c:235-250)."""
    res = LocalMinResult()
    res.norm0 = math.sqrt(comm.ordered_sum(blocks, [blk.norm0_sq() for blk in blocks]))
    nb = blocks[0].layout.nb
    thr = max(atol, rtol / math.sqrt(nb) * res.norm0)
    for blk in blocks:
        blk.reset_halo()
    comm.barrier()
    t0 = time.perf_counter()
    while True:
        its_outer = []
        for k in range(s):
            for blk in blocks:
                blk.update_rhs()
            its_outer.append([blk.solve() for blk in blocks])
            comm.exchange(blocks)
            for blk in blocks:
                blk.store_local_column(k)
        norms, lits = [], []
        for blk in blocks:
            _, li, _ = blk.local_minimize()
            lits.append(li)
            norms.append(math.sqrt(blk.local_residual_sq()))      # MatResidual(A_ii, rhs_i, x_i)
        res.hist.append(norms)
        res.lsqr_its.append(lits)
        res.inner_its.append(its_outer)
        res.outer_its += 1
        if monitor:
            monitor(res.outer_its, norms, its_outer, lits)
        conv = [1.0 if n <= thr else 0.0 for n in norms]
        if comm.ordered_sum(blocks, conv) == float(nb):           # every block converged
            break
        if res.outer_its >= max_outer:
            break
    comm.barrier()
    res.elapsed = time.perf_counter() - t0
    comm.exchange(blocks)                                        # comm_sync_send_and_receive_final
    res.final_norm = math.sqrt(comm.ordered_sum(blocks, [blk.block_residual_sq() for blk in blocks]))
    res.error = math.sqrt(comm.ordered_sum(blocks, [blk.error_sq() for blk in blocks]))
    return res


def smsm_semi_local_solve(blocks, comm, s: int, rtol: float, atol: float = 1e-100, max_outer: int = 10000,
                          monitor=None) -> LocalMinResult:
    """SMSM with semi-local minimization (synchronous-multisplitting-synchronous-minimization-
    semi-local.c:288-345): s times {rhs_i; inner GMRES; exchange; S_i(:,k) = x over the
    block's rows and neighbour planes}, R_i = A_block S_i, alpha_i = LSQR(R_i, b_i); the
    local test on the last inner iterate; x_i and the block's view of its neighbours
    <- S_i alpha_i; stop when every block passes (comm_sync_convergence_detection)."""
    res = LocalMinResult()
    res.norm0 = math.sqrt(comm.ordered_sum(blocks, [blk.norm0_sq() for blk in blocks]))
    nb = blocks[0].layout.nb
    thr = max(atol, rtol / math.sqrt(nb) * res.norm0)
    for blk in blocks:
        blk.reset_halo()
    comm.barrier()
    t0 = time.perf_counter()
    while True:
        its_outer = []
        for k in range(s):
            for blk in blocks:
                blk.update_rhs()
            its_outer.append([blk.solve() for blk in blocks])
            comm.exchange(blocks)
            for blk in blocks:
                blk.store_column(k)
        norms, lits = [], []
        for blk in blocks:
            norms.append(math.sqrt(blk.local_residual_sq()))      # last inner iterate (:336-337)
        for blk in blocks:
            _, li, _ = blk.semi_local_minimize(apply=True)
            lits.append(li)
        res.hist.append(norms)
        res.lsqr_its.append(lits)
        res.inner_its.append(its_outer)
        res.outer_its += 1
        if monitor:
            monitor(res.outer_its, norms, its_outer, lits)
        conv = [1.0 if n <= thr else 0.0 for n in norms]
        if comm.ordered_sum(blocks, conv) == float(nb):
            break
        if res.outer_its >= max_outer:
            break
    comm.barrier()
    res.elapsed = time.perf_counter() - t0
    comm.exchange(blocks)
    res.final_norm = math.sqrt(comm.ordered_sum(blocks, [blk.block_residual_sq() for blk in blocks]))
    res.error = math.sqrt(comm.ordered_sum(blocks, [blk.error_sq() for blk in blocks]))
    return res


def make_smsm(ctx: Context, dim, nx, ny, nz, nb, block_ids, s: int, opts: Options | None, comm, peclet=None):
    """GpuBlocks with the minimization storage, and the GpuMinimizer over them."""
    blocks = make_blocks(ctx, dim, nx, ny, nz, nb, block_ids, opts, comm, peclet)
    for blk in blocks:
        blk.setup_minimization(s)
    return blocks, GpuMinimizer(ctx, blocks, comm, opts)
