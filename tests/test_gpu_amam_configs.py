"""AMAM-global -- the algorithm of BASELINE configs[3] (3D Poisson 1024^3, 8 blocks) and configs[4]
(3D convection-diffusion 512^3, 8 blocks) -- at its real per-GPU block size on the one MI355X: two blocks of
the per-GPU geometry (1024 x 1024 x 128; 512 x 512 x 64) round-robin on this GPU (LocalComm, HBM
mailboxes), s = 20 inner GMRES(30) solves of max_it 20 per outer iteration, outer LSQR max_it 70
(running_bulk_test_g5k:296-317), both minimizations: the replicated-R LSQR (outer_solver_norm_equation,
utils.c:1061-1078) and the reference's normal equations (outer_solver, utils.c:972-996,
-msplit_minimization rtr).  Checked: two outer iterations per block, a bitwise rerun (every local norm of
the trace, the blocks' ||x||, the final residual), the local residual decreasing, and a clean termination
of the detection protocol (every block FINISHED in the same phase) at a tolerance the blocks reach.
Asynchronous runs have no reference history: parity is the residual."""
import gc

import numpy as np
import pytest

from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
from medane_tchakorom_ufc_thesis_repository_amd.comm import LocalComm
from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks
from medane_tchakorom_ufc_thesis_repository_amd.petsc import ConvDetection, Options

pytestmark = pytest.mark.gpu

S, INNER_MAX_IT = 20, 20


def _opts(minimization):
    return Options(" ".join(
        f"-inner{b}_ksp_type gmres -inner{b}_ksp_gmres_restart 30 -inner{b}_ksp_max_it {INNER_MAX_IT} "
        f"-inner{b}_ksp_rtol 1e-20 -inner{b}_ksp_atol 1e-100 -inner{b}_pc_type none "
        f"-outer{b}_ksp_type lsqr -outer{b}_ksp_convergence_test default -outer{b}_ksp_lsqr_exact_mat_norm "
        f"-outer{b}_ksp_atol 1e-100 -outer{b}_ksp_max_it 70 -outer{b}_ksp_rtol 1e-15 -outer{b}_pc_type none"
        for b in (1, 2)) + f" -s {S} -msplit_minimization {minimization}")


def _reset(blocks):
    """x = 0 and the newest-value minimization state back to MatZeroEntries (a fresh run on the same blocks)."""
    for blk in blocks:
        blk.x.set(0.0)
        for D in (blk.Gc_rep if blk.minimization == "rtr" else blk.R_rep):
            D.zero_entries()


def _fingerprint(res, blocks):
    return ([(b, it, float(ln).hex()) for b, it, ln, _, _ in res.trace],
            [float(blk.x.norm()).hex() for blk in blocks], float(res.final_norm).hex())


@pytest.mark.parametrize("config", ["configs3", "configs4"])
@pytest.mark.parametrize("minimization", ["lsqr", "rtr"])
def test_amam_global_per_gpu_block_pair(ctx, config, minimization, monkeypatch):
    # one R broadcast buffer per block for the replicated-R LSQR: two blocks' replicated R and their buffers
    # otherwise take 288 of the 309 GB (tools/amam_configs.py pair, profiles/r03/amam/)
    monkeypatch.setenv("MSPLIT_ABCAST_NBUF", "1")
    n, planes, peclet = (1024, 128, None) if config == "configs3" else (512, 64, (0.5, 0.25, -0.3))
    comm = LocalComm()
    blocks = make_blocks(ctx, 3, n, n, 2 * planes, 2, [0, 1], _opts(minimization), comm, peclet)
    try:
        for blk in blocks:
            blk.setup_global_async_minimization(S)
            assert blk.minimization == minimization
        runs = []
        for _ in range(2):                                   # two outer iterations per block, then a rerun
            _reset(blocks)
            res = am_solve(blocks, comm, rtol=1e-30, record=True, variant="amam_global", s=S, max_iterations=2,
                           stop_at_limit=True)
            assert res.iterations == [2, 2] and res.inner_its == [2 * S * INNER_MAX_IT] * 2
            assert res.transport == "device"
            runs.append(_fingerprint(res, blocks))
        assert runs[0] == runs[1]                            # bitwise rerun
        trace = {(b, it): float.fromhex(h) for b, it, h in runs[0][0]}
        for b in (0, 1):
            assert trace[(b, 2)] < trace[(b, 1)] < res.norm0    # the local residual decreases
        assert res.final_norm < res.norm0
        # a clean termination: a tolerance the blocks pass after their first outer iteration
        rtol = 2.0 * np.sqrt(2.0) * max(trace[(0, 1)], trace[(1, 1)]) / res.norm0
        _reset(blocks)
        res = am_solve(blocks, comm, rtol=rtol, record=True, variant="amam_global", s=S, max_iterations=10)
        assert res.converged
        last = {b: st for b, _, _, st, _ in res.trace}
        assert last == {0: ConvDetection.FINISHED, 1: ConvDetection.FINISHED}
        assert len(set(res.phase_tags)) == 1
        assert np.isfinite(res.final_norm) and res.final_norm < res.norm0
    finally:
        del blocks
        gc.collect()
