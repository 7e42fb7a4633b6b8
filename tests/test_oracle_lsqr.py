"""The CPU oracle's outer least-squares solve (KSPLSQR) and SMSM-global loop.

KSPLSQR lives in un-vendored PETSc 3.22.1 and no reference test pins it, so
(as for GMRES) the C oracle and the independent pure-Python twin must agree
bit for bit, and both must agree with independent implementations of the same
mathematics: numpy's least-squares solution once LSQR has converged, and
scipy's LSQR (Paige & Saunders' algorithm, the one PETSc follows) iterate by
iterate while the Krylov space is still growing.
"""
import numpy as np
import pytest
import scipy.sparse.linalg as sla

import twin

RNG = np.random.default_rng(20251121)


def _problem(m, s, cond=1.0):
    Q1, _ = np.linalg.qr(RNG.standard_normal((m, s)))
    Q2, _ = np.linalg.qr(RNG.standard_normal((s, s)))
    sv = np.geomspace(1.0, 1.0 / cond, s)
    return (Q1 * sv) @ Q2.T, RNG.standard_normal(m)


@pytest.mark.parametrize("conv", ["default", "lsqr", "skip"])
@pytest.mark.parametrize("exact", [0, 1])
def test_lsqr_oracle_equals_twin(oracle, conv, exact):
    R, b = _problem(37, 5, cond=30.0)
    kw = dict(max_it=12, rtol=1e-9, abstol=1e-50, exact_norm=exact)
    x, r = oracle.lsqr([R], [b], conv_test={"default": 0, "lsqr": 1, "skip": 2}[conv], **kw)
    xt, its, reason, rnorm, hist = twin.lsqr(R.tolist(), b.tolist(), conv_test=conv, **kw)
    assert (r["its"], r["reason"]) == (its, reason)
    assert r["rnorm"] == rnorm
    assert np.array_equal(r["hist"], np.array(hist))
    assert np.array_equal(x, np.array(xt))


def test_lsqr_multiblock_seq_is_the_global_sequential_order(oracle):
    # SEQ mode with the rows split over blocks = one sequential sum over all rows
    R, b = _problem(60, 4, cond=10.0)
    kw = dict(max_it=20, rtol=1e-12, exact_norm=1)
    x1, r1 = oracle.lsqr([R], [b], **kw)
    x3, r3 = oracle.lsqr([R[:17], R[17:41], R[41:]], [b[:17], b[17:41], b[41:]], **kw)
    assert np.array_equal(x1, x3) and np.array_equal(r1["hist"], r3["hist"])
    assert (r1["its"], r1["reason"]) == (r3["its"], r3["reason"])


def test_lsqr_dbr_block_order(oracle):
    # DBR mode: per-block DBR partials added in block order from 0.0 -- block
    # sizes change the sums, yet the solution is the least-squares one
    R, b = _problem(9000, 6, cond=5.0)
    xs = np.linalg.lstsq(R, b, rcond=None)[0]
    for cuts in ([9000], [4096, 4904], [3000, 3000, 3000]):
        edges = np.cumsum([0] + cuts)
        Rb = [R[a:c] for a, c in zip(edges[:-1], edges[1:])]
        bb = [b[a:c] for a, c in zip(edges[:-1], edges[1:])]
        x, r = oracle.lsqr(Rb, bb, max_it=30, rtol=1e-14, exact_norm=1, conv_test=0, reduce_mode=oracle.REDUCE_DBR)
        assert np.allclose(x, xs, rtol=0, atol=1e-12 * np.abs(xs).max())
        assert abs(r["rnorm"] - np.linalg.norm(b - R @ xs)) < 1e-10 * np.linalg.norm(b)


def test_lsqr_matches_scipy_iterates(oracle):
    # before the Krylov space is exhausted (k < s), LSQR iterates agree with scipy's
    R, b = _problem(200, 8, cond=10.0)
    for k in (1, 3, 6):
        x, r = oracle.lsqr([R], [b], max_it=k, rtol=1e-30, abstol=0.0, conv_test=oracle.CONV_DEFAULT)
        xs = sla.lsqr(R, b, atol=0.0, btol=0.0, conlim=0.0, iter_lim=k)[0]
        assert r["its"] == k and r["reason"] == -3
        assert np.allclose(x, xs, rtol=1e-10, atol=1e-12)


def test_lsqr_converges_to_lstsq(oracle):
    R, b = _problem(300, 10, cond=1e3)
    xs = np.linalg.lstsq(R, b, rcond=None)[0]
    x, r = oracle.lsqr([R], [b], max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)
    assert r["reason"] == -3 and r["its"] == 70        # the campaign setting never meets rtol 1e-15
    assert np.allclose(x, xs, rtol=1e-8, atol=1e-8 * np.abs(xs).max())
    assert abs(r["rnorm"] - np.linalg.norm(b - R @ xs)) <= 1e-9 * np.linalg.norm(b)
    # the LSQR test proper stops on the normal-equation residual
    x2, r2 = oracle.lsqr([R], [b], max_it=70, rtol=1e-8, exact_norm=1, conv_test=oracle.CONV_LSQR)
    assert r2["reason"] == 1 and r2["its"] < 70
    assert np.linalg.norm(R.T @ (b - R @ x2)) <= 1e-6 * np.linalg.norm(R) * np.linalg.norm(b - R @ x2)


def test_lsqr_edge_cases(oracle):
    R, b = _problem(20, 3)
    # zero right-hand side: converged at n = 0 (rnorm = 0 < atol)
    x, r = oracle.lsqr([R], [np.zeros(20)], max_it=10)
    assert (r["its"], r["reason"], r["rnorm"]) == (0, 3, 0.0) and not x.any()
    # max_it = 0: the do-while still takes one step (KSPSolve_LSQR)
    x, r = oracle.lsqr([R], [b], max_it=0, rtol=1e-30, conv_test=oracle.CONV_DEFAULT)
    assert (r["its"], r["reason"]) == (1, -3)
    # a consistent system: b in range(R) -> phibar falls to the rtol test
    x, r = oracle.lsqr([R], [R @ np.array([1.0, -2.0, 0.5])], max_it=50, rtol=1e-10, conv_test=0)
    assert r["reason"] == 2 and np.allclose(x, [1.0, -2.0, 0.5], atol=1e-9)
    # skip: runs to max_it, reason CONVERGED_ITS
    x, r = oracle.lsqr([R], [b], max_it=7, conv_test=oracle.CONV_SKIP)
    assert (r["its"], r["reason"]) == (7, 4)


def test_dense_mult_order(oracle):
    S = RNG.standard_normal((50, 7))
    a = RNG.standard_normal(7)
    y = oracle.dense_mult(S, a)
    ref = np.zeros(50)
    for j in range(7):
        ref = ref + a[j] * S[:, j]
    assert np.array_equal(y, ref)


INNER = dict(restart=30, max_it=20, rtol=1e-20)
OUTER = dict(max_it=70, rtol=1e-15, abstol=1e-100, exact_norm=1, conv_test=0)   # running_bulk_test_g5k:247


@pytest.mark.parametrize("problem", [(2, 32, 32, 1, 2, 4), (3, 8, 8, 8, 2, 4), (3, 6, 6, 8, 4, 3)])
def test_smsm_oracle_converges(oracle, problem):
    dim, nx, ny, nz, nb, s = problem
    r = oracle.smsm_solve(dim, nx, ny, nz, nb, s, 1e-6, INNER, OUTER)
    assert r["norm0"] > 0 and r["outer_its"] < 50
    assert r["hist"][-1] <= 1e-6 * r["norm0"]
    assert r["inner_its"].shape == (r["outer_its"], s, nb)
    # the LSQR residual estimate is the true residual of the minimized iterate
    assert abs(r["final_norm"] - r["hist"][-1]) <= 1e-3 * r["hist"][-1]
    # the minimization pays: far fewer outer iterations x s than SM's outer count
    sm = oracle.sm_solve(dim, nx, ny, nz, nb, 1e-6, INNER, max_outer=5000)
    assert r["outer_its"] * s < sm["outer_its"]


def test_smsm_oracle_dbr_vs_seq(oracle):
    # same outer and inner counts; histories close (the LSQR steps past rank s
    # run on rounding noise, so the two orders drift apart -- see DESIGN.md)
    a = oracle.smsm_solve(2, 32, 32, 1, 2, 4, 1e-6, INNER, OUTER)
    b = oracle.smsm_solve(2, 32, 32, 1, 2, 4, 1e-6, dict(INNER, reduce_mode=1), dict(OUTER, reduce_mode=1))
    assert a["outer_its"] == b["outer_its"]
    assert np.array_equal(a["inner_its"], b["inner_its"])
    assert np.allclose(a["hist"][:3], b["hist"][:3], rtol=1e-9)
    assert np.allclose(a["hist"], b["hist"], rtol=0.1)
