"""KSPGMRES termination branches other than convergence by rtol (PETSc 3.22.1
KSPConvergedDefault / KSPGMRESCycle semantics, restated in oracle/oracle.c
gm_converged, gm_cycle, gm_update_hessenberg; option defaults at
/root/reference tmp/petscmpiexec_help:336-341 (divtol 1e4) and :603-606
(haptol 1e-30, breakdown tolerance 0.1)).

Each case is (operator arrays, b, x0 or None, PETSc option string, oracle
kwargs, expected KSPConvergedReason).  Shared by the oracle self-test
(test_oracle.py, CPU) and the device parity test (test_gpu_gmres.py).
"""
import numpy as np

DIVERGED_NULL, DIVERGED_DTOL, DIVERGED_BREAKDOWN, DIVERGED_NANORINF = -2, -4, -5, -9
CONVERGED_RTOL, CONVERGED_ATOL = 2, 3

BASE = "-ksp_type gmres -pc_type none -ksp_norm_type unpreconditioned"


def _poisson(oracle, nx, ny, nz):
    return oracle.poisson3d_rows(nx, ny, nz, 0, nz).arrays()


def cases(oracle):
    r = np.random.default_rng(20251121)
    out = {}
    # DIVERGED_DTOL: nonzero guess whose residual exceeds divtol * ||b|| at iteration 0
    rp, col, val = _poisson(oracle, 9, 8, 7)
    n = len(rp) - 1
    b = np.asarray(oracle.Mat.from_arrays(n, n, rp, col, val).mult(np.ones(n)))
    x0 = 100.0 * r.uniform(-1, 1, n)
    out["dtol"] = ((rp, col, val), b, x0,
                   f"{BASE} -ksp_gmres_restart 30 -ksp_max_it 50 -ksp_rtol 1e-8 -ksp_divtol 10 "
                   "-ksp_initial_guess_nonzero",
                   dict(restart=30, max_it=50, rtol=1e-8, divtol=10.0, guess_nonzero=1), DIVERGED_DTOL)
    # DIVERGED_NANORINF: a NaN in b (KSPCheckNorm on ||b||)
    bn = b.copy()
    bn[17] = np.nan
    out["nan_b"] = ((rp, col, val), bn, None, f"{BASE} -ksp_gmres_restart 30 -ksp_max_it 50 -ksp_rtol 1e-8",
                    dict(restart=30, max_it=50, rtol=1e-8), DIVERGED_NANORINF)
    # DIVERGED_NANORINF: an Inf in the initial guess
    xi = np.zeros(n)
    xi[5] = np.inf
    out["inf_x0"] = ((rp, col, val), b, xi,
                     f"{BASE} -ksp_gmres_restart 30 -ksp_max_it 50 -ksp_rtol 1e-8 -ksp_initial_guess_nonzero",
                     dict(restart=30, max_it=50, rtol=1e-8, guess_nonzero=1), DIVERGED_NANORINF)
    # DIVERGED_BREAKDOWN at a restart: the recomputed residual differs from the recurrence's estimate by
    # more than breakdowntol * ||r0|| of the cycle (KSPGMRESCycle's restart check)
    out["restart_breakdown"] = ((rp, col, val), b, None,
                                f"{BASE} -ksp_gmres_restart 3 -ksp_max_it 60 -ksp_rtol 1e-30 "
                                "-ksp_gmres_breakdown_tolerance 1e-300",
                                dict(restart=3, max_it=60, rtol=1e-30, breakdowntol=1e-300), DIVERGED_BREAKDOWN)
    # A v = 0 (a zero-valued operator) leaves a zero Hessenberg column: KSPGMRESUpdateHessenberg sets
    # DIVERGED_NULL, then KSPGMRESBuildSoln finds HH(0,0) == 0 and overwrites it with DIVERGED_BREAKDOWN
    # (PETSc 3.22.1 order; the final reason is BREAKDOWN after one iteration)
    out["null"] = ((rp, col, np.zeros_like(val)), b, None,
                   f"{BASE} -ksp_gmres_restart 30 -ksp_max_it 50 -ksp_rtol 1e-8",
                   dict(restart=30, max_it=50, rtol=1e-8), DIVERGED_BREAKDOWN)
    # happy breakdown mid-cycle: two distinct eigenvalues exhaust the Krylov space at the second step;
    # with -ksp_gmres_haptol 1e-8 the tiny new direction ends the cycle with res = 0 (CONVERGED_ATOL)
    m = 3000
    rpd = np.arange(m + 1, dtype=np.int32)
    cold = np.arange(m, dtype=np.int32)
    vald = np.where(np.arange(m) % 2 == 0, 2.0, 5.0)
    bd = 1e-3 * r.uniform(-1, 1, m)
    out["happy"] = ((rpd, cold, vald), bd, None,
                    f"{BASE} -ksp_gmres_restart 30 -ksp_max_it 50 -ksp_rtol 1e-30 -ksp_atol 1e-60 "
                    "-ksp_gmres_haptol 1e-8",
                    dict(restart=30, max_it=50, rtol=1e-30, abstol=1e-60, haptol=1e-8), CONVERGED_ATOL)
    # DIVERGED_DTOL after a restart is impossible (GMRES residuals never grow) -- not a case
    return out
