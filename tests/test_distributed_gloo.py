"""The N > 1 path on CPU: world_size-2 gloo runs of the product's SM driver
(multisplitting.sm_solve) and exchange layer (comm.TorchComm).

The GPU block is replaced by a CPU test double whose arithmetic is the
oracle's (DBR order), so the distributed run must reproduce the single-process
oracle SM solve bit for bit: same outer iterations, same residual history,
same iterate.  What is under test is the product's driver loop, block layout,
halo exchange pattern and block-ordered norm reduction.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

INNER = dict(restart=30, max_it=20, rtol=1e-20)


class OracleBlock:
    """CPU test double of multisplitting.GpuBlock (same hooks, oracle arithmetic)."""

    def __init__(self, layout, po):
        self.po = po
        self.layout = L = layout
        if L.dim == 3:
            ppb = L.nz // L.nb
            Ab = po.poisson3d_rows(L.nx, L.ny, L.nz, L.b * ppb, (L.b + 1) * ppb)
        else:
            Ab = po.poisson2d_rows(L.nx, L.ny, L.r0, L.r1)
        self.A, _ = po.split(Ab, L.r0, L.r1)
        row_ids, crp, cc, cv = L.coupling
        rp = np.zeros(L.nrows + 1, np.int64)
        rp[row_ids + 1] = np.diff(crp)
        rp = np.cumsum(rp)
        self.A_off = po.Mat.from_arrays(L.nrows, max(L.halo_size, 1), rp, cc, cv)
        self.b = Ab.mult(np.ones(Ab.shape[1]))          # A_block u, u = 1
        self.x = np.zeros(L.nrows)
        self.halo = np.zeros(L.halo_size)
        self.halo_t = torch.zeros(max(L.halo_size, 2), dtype=torch.float64)
        self.rhs = self.b.copy()
        self._send = {nbr: (off, cnt) for nbr, off, cnt in L.send}
        self._recv = {nbr: (hoff, cnt) for nbr, hoff, cnt, _ in L.recv}

    def pack_send(self, nbr):
        off, cnt = self._send[nbr]
        return torch.from_numpy(self.x[off:off + cnt].copy())

    def recv_buffer(self, nbr):
        hoff, cnt = self._recv[nbr]
        return self.halo_t[hoff:hoff + cnt]

    def unpack_recv(self):
        self.halo = self.halo_t[:self.layout.halo_size].numpy().copy()

    def reset_halo(self):
        self.halo[:] = 0.0

    def norm0_sq(self):
        ln = self.po.norm2(self.b, self.po.REDUCE_DBR)
        return ln * ln

    def update_rhs(self):
        h = self.halo if self.layout.halo_size else np.zeros(1)
        self.rhs = self.A_off.residual(self.b, h)

    def solve(self):
        self.x, r = self.po.gmres(self.A, self.rhs, x0=self.x, guess_nonzero=1, uirnorm=1,
                                  reduce_mode=self.po.REDUCE_DBR, **INNER)
        return r["its"]

    def local_residual_sq(self):
        ln = self.po.norm2(self.A.residual(self.rhs, self.x), self.po.REDUCE_DBR)
        return ln * ln

    # -- SMSM-global hooks (same arithmetic as oracle.smsm_solve)
    def setup_minimization(self, s):
        L = self.layout
        self.s = s
        self.lo = L.plane if L.b > 0 else 0
        self.hi = L.plane if L.b < L.nb - 1 else 0
        if L.dim == 3:
            ppb = L.nz // L.nb
            Ab = self.po.poisson3d_rows(L.nx, L.ny, L.nz, L.b * ppb, (L.b + 1) * ppb)
        else:
            Ab = self.po.poisson2d_rows(L.nx, L.ny, L.r0, L.r1)
        rp, c, v = Ab.arrays()
        ne = self.lo + L.nrows + self.hi
        self.A_ext = self.po.Mat.from_arrays(L.nrows, ne, rp, c - (L.r0 - self.lo), v)
        self.S = np.zeros((ne, s), order="F")
        self.R = np.zeros((L.nrows, s), order="F")

    def store_column(self, k):
        n = self.layout.nrows
        self.S[self.lo:self.lo + n, k] = self.x
        self.S[:self.lo, k] = self.halo[:self.lo]
        self.S[self.lo + n:, k] = self.halo[self.lo:self.lo + self.hi]

    def form_R(self):
        for k in range(self.s):
            self.R[:, k] = self.A_ext.mult(np.ascontiguousarray(self.S[:, k]))

    def apply_alpha(self, alpha):
        n = self.layout.nrows
        xe = self.po.dense_mult(self.S, alpha)
        self.x = xe[self.lo:self.lo + n].copy()
        self.halo = np.concatenate([xe[:self.lo], xe[self.lo + n:]])

    def block_residual_sq(self):
        n = self.layout.nrows
        xe = np.concatenate([self.halo[:self.lo], self.x, self.halo[self.lo:]])
        ln = self.po.norm2(self.A_ext.residual(self.b, xe), self.po.REDUCE_DBR)
        return ln * ln

    def error_sq(self):
        e = self.po.norm2(self.x - 1.0, self.po.REDUCE_DBR)
        return e * e


class OracleMinimizer:
    """Test double of multisplitting.GpuMinimizer: every rank gathers all
    blocks' rows of R and b and runs the oracle's block-ordered LSQR."""

    def __init__(self, po, outer):
        self.po = po
        self.outer = outer

    def solve(self, blocks):
        (blk,) = blocks
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, (blk.R, blk.b))
        alpha, r = self.po.lsqr([p[0] for p in parts], [p[1] for p in parts], reduce_mode=self.po.REDUCE_DBR,
                                **self.outer)
        blk.apply_alpha(alpha)
        return r["rnorm"], r["its"], r["reason"]


OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)


def _smsm_worker(rank, world, port, problem, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from medane_tchakorom_ufc_thesis_repository_amd.comm import TorchComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import smsm_solve
    from medane_tchakorom_ufc_thesis_repository_amd.utils import block_layout
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dim, nx, ny, nz, s, rtol = problem
        blk = OracleBlock(block_layout(dim, nx, ny, nz, world, rank), po)
        blk.setup_minimization(s)
        comm = TorchComm()
        res = smsm_solve([blk], comm, s, OracleMinimizer(po, OUTER), rtol=rtol, max_outer=100)
        q.put((rank, res.outer_its, res.norm0, list(res.hist), [[k[0] for k in o] for o in res.inner_its],
               list(res.lsqr_its), res.final_norm, blk.x))
    finally:
        dist.destroy_process_group()


def _worker(rank, world, port, problem, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from medane_tchakorom_ufc_thesis_repository_amd.comm import TorchComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import sm_solve
    from medane_tchakorom_ufc_thesis_repository_amd.utils import block_layout
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dim, nx, ny, nz, rtol = problem
        blk = OracleBlock(block_layout(dim, nx, ny, nz, world, rank), po)
        comm = TorchComm()
        res = sm_solve([blk], comm, rtol=rtol, max_outer=300)
        q.put((rank, res.outer_its, res.norm0, list(res.hist), [i[0] for i in res.inner_its], blk.x))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, problem, target=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target or _worker, args=(r, world, port, problem, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize("problem", [(3, 10, 9, 8, 1e-6), (2, 24, 20, 1, 1e-5)])
def test_sm_two_ranks_gloo_matches_oracle(oracle, problem):
    dim, nx, ny, nz, rtol = problem
    out = _run(2, problem)
    ref = oracle.sm_solve(dim, nx, ny, nz, 2, rtol, dict(INNER, reduce_mode=oracle.REDUCE_DBR), max_outer=300)
    for rank, outer, norm0, hist, its, x in out:
        assert outer == ref["outer_its"]
        assert norm0 == ref["norm0"]
        assert np.array_equal(np.array(hist), ref["hist"])
        assert np.array_equal(np.array(its), ref["inner_its"][:, rank])
    x = np.concatenate([o[5] for o in out])
    assert np.array_equal(x, ref["x"])


def test_sm_four_ranks_gloo_matches_oracle(oracle):
    problem = (3, 8, 8, 8, 1e-6)
    out = _run(4, problem)
    ref = oracle.sm_solve(3, 8, 8, 8, 4, 1e-6, dict(INNER, reduce_mode=oracle.REDUCE_DBR), max_outer=300)
    assert all(o[1] == ref["outer_its"] for o in out)
    assert np.array_equal(np.array(out[0][3]), ref["hist"])
    assert np.array_equal(np.concatenate([o[5] for o in out]), ref["x"])


@pytest.mark.parametrize("world,problem", [(2, (2, 32, 32, 1, 4, 1e-6)), (2, (3, 8, 8, 8, 4, 1e-6)),
                                           (4, (3, 6, 6, 8, 3, 1e-6))])
def test_smsm_gloo_matches_oracle(oracle, world, problem):
    dim, nx, ny, nz, s, rtol = problem
    out = _run(world, problem, _smsm_worker)
    ref = oracle.smsm_solve(dim, nx, ny, nz, world, s, rtol, dict(INNER, reduce_mode=oracle.REDUCE_DBR),
                            dict(OUTER, reduce_mode=oracle.REDUCE_DBR), max_outer=100)
    for rank, outer, norm0, hist, its, lits, fnorm, x in out:
        assert outer == ref["outer_its"]
        assert norm0 == ref["norm0"]
        assert np.array_equal(np.array(hist), ref["hist"])
        assert np.array_equal(np.array(its), ref["inner_its"][:, :, rank])
        assert np.array_equal(np.array(lits), ref["lsqr_its"])
        assert fnorm == ref["final_norm"]
    assert np.array_equal(np.concatenate([o[7] for o in out]), ref["x"])


def _fault_worker(rank, world, port, problem, q):
    """sm_solve with rank 1's stop decision flipped at the first outer iteration (MSPLIT_FAULT_STOP_RANK)."""
    os.environ["MSPLIT_FAULT_STOP_RANK"] = "1"
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from medane_tchakorom_ufc_thesis_repository_amd.comm import TorchComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import sm_solve
    from medane_tchakorom_ufc_thesis_repository_amd.utils import block_layout
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dim, nx, ny, nz, rtol = problem
        blk = OracleBlock(block_layout(dim, nx, ny, nz, world, rank), po)
        try:
            sm_solve([blk], TorchComm(), rtol=rtol, max_outer=300)
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_stop_disagreement_is_an_error_on_every_rank_not_a_hang():
    """The ranks agree on (outer iteration, stop) once per outer iteration (multisplitting.agree_on_stop,
    msp_comm_agree).  One rank injected to stop alone at the first outer iteration: every rank raises, naming
    the disagreement, instead of the others blocking in their next collective (round 4's pre-fix hang)."""
    out = _run(3, (3, 8, 8, 9, 1e-6), _fault_worker)
    assert [r for r, _ in out] == [0, 1, 2]
    assert all("disagree" in msg for _, msg in out), out


def test_smsm_eight_ranks_gloo_matches_oracle(oracle):
    """nb = 8 (the driver's scaling world size), one rank per block over gloo, bitwise the oracle."""
    problem = (3, 6, 6, 16, 3, 1e-6)
    out = _run(8, problem, _smsm_worker)
    ref = oracle.smsm_solve(3, 6, 6, 16, 8, 3, 1e-6, dict(INNER, reduce_mode=oracle.REDUCE_DBR),
                            dict(OUTER, reduce_mode=oracle.REDUCE_DBR), max_outer=100)
    for rank, outer, norm0, hist, its, lits, fnorm, x in out:
        assert outer == ref["outer_its"] and norm0 == ref["norm0"]
        assert np.array_equal(np.array(hist), ref["hist"])
        assert np.array_equal(np.array(lits), ref["lsqr_its"])
        assert fnorm == ref["final_norm"]
    assert np.array_equal(np.concatenate([o[7] for o in out]), ref["x"])
