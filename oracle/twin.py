"""Pure-Python twin of the C oracle, for small cases only.

TEST INFRASTRUCTURE ONLY.  Written independently of oracle.c from the same
reference call sites, so that the two restatements check each other:
  * assembly inserts entries in the reference's own MatSetValues order
    (utils.c:57-112 for 3D, :261-287 for 2D) and then sorts each row, which is
    what PETSc AIJ storage does [PETSc-ext];
  * GMRES follows KSPSolve_GMRES/KSPGMRESCycle [PETSc-ext] with Python floats
    (IEEE binary64, no FMA), sequential reductions (ORC_REDUCE_SEQ).
"""
from __future__ import annotations

import math

import numpy as np


def _rows_to_csr(rows: list[dict], ncols: int):
    rowptr = [0]
    col, val = [], []
    for r in rows:
        for c in sorted(r):
            col.append(c)
            val.append(r[c])
        rowptr.append(len(col))
    return np.array(rowptr, np.int32), np.array(col, np.int32), np.array(val, np.float64), ncols


def poisson3d_block_reference_order(nx, ny, nz, rank_jacobi_block):
    """poisson3DMatrix (utils.c:30-121) for BLOCK_RANK_ZERO/ONE, literally:
    the z range uses n_grid_columns (ny) as the reference does (utils.c:45,51)."""
    if rank_jacobi_block == 0:
        z_start, z_end, prev = 0, ny // 2, 0
    else:
        z_start, z_end, prev = ny // 2, ny, (nx * ny * nz) // 2
    nrows = (nx * ny * nz) // 2
    rows = [dict() for _ in range(nrows)]
    for k in range(z_start, z_end):
        for j in range(ny):
            for i in range(nx):
                row = i + j * nx + k * nx * ny
                ent = [(row, 6.0)]
                if i > 0:
                    ent.append((row - 1, -1.0))
                if i < nx - 1:
                    ent.append((row + 1, -1.0))
                if j > 0:
                    ent.append((row - nx, -1.0))
                if j < ny - 1:
                    ent.append((row + nx, -1.0))
                if k > 0:
                    ent.append((row - nx * ny, -1.0))
                if k < nz - 1:
                    ent.append((row + nx * ny, -1.0))
                g = row - prev
                for c, v in ent:
                    rows[g][c] = v  # INSERT_VALUES
    return _rows_to_csr(rows, nx * ny * nz)


def poisson2d_block_reference_order(m, n, rank_jacobi_block, njacobi_blocks, idx_start=0, idx_end=None):
    """poisson2DMatrix (utils.c:247-293) for one block owned by one rank."""
    rbs = (m * n) // njacobi_blocks
    if idx_end is None:
        idx_end = rbs
    rows = [dict() for _ in range(rbs)]
    for Ii in range(rank_jacobi_block * rbs + idx_start, rank_jacobi_block * rbs + idx_end):
        i = Ii // n
        j = Ii - i * n
        new = Ii - rank_jacobi_block * rbs
        if i > 0:
            rows[new][Ii - n] = -1.0
        if i < m - 1:
            rows[new][Ii + n] = -1.0
        if j > 0:
            rows[new][Ii - 1] = -1.0
        if j < n - 1:
            rows[new][Ii + 1] = -1.0
        rows[new][Ii] = 4.0
    return _rows_to_csr(rows, m * n)


def spmv(rowptr, col, val, x):
    y = np.empty(len(rowptr) - 1)
    for r in range(len(rowptr) - 1):
        s = 0.0
        for k in range(rowptr[r], rowptr[r + 1]):
            s += float(val[k]) * float(x[col[k]])
        y[r] = s
    return y


def _dot(x, y):
    s = 0.0
    for a, b in zip(x, y):
        s += float(a) * float(b)
    return s


def _norm(x):
    return math.sqrt(_dot(x, x))


def _maxpy(w, a, V):
    k = len(V)
    jrem = k & 3
    out = np.array(w, dtype=np.float64, copy=True)
    for i in range(len(out)):
        u = float(out[i])
        if jrem == 3:
            u = u + ((a[0] * V[0][i] + a[1] * V[1][i]) + a[2] * V[2][i])
        elif jrem == 2:
            u = u + (a[0] * V[0][i] + a[1] * V[1][i])
        elif jrem == 1:
            u = a[0] * V[0][i] + u
        for j in range(jrem, k, 4):
            u = u + (((a[j] * V[j][i] + a[j + 1] * V[j + 1][i]) + a[j + 2] * V[j + 2][i]) + a[j + 3] * V[j + 3][i])
        out[i] = u
    return out


def gmres(rowptr, col, val, b, x0=None, restart=30, max_it=10000, rtol=1e-5, abstol=1e-50, divtol=1e4,
          haptol=1e-30, breakdowntol=0.1, uirnorm=False, guess_nonzero=False):
    """KSPSolve with KSPGMRES(restart), CGS REFINE_NEVER, PCNONE [PETSc-ext]."""
    n = len(rowptr) - 1
    b = [float(v) for v in b]
    guess_zero = not guess_nonzero
    x = [0.0] * n if (x0 is None or guess_zero) else [float(v) for v in x0]
    m = restart
    st = {"its": 0, "reason": 0, "rnorm": -1.0, "rnorm0": 0.0, "ttol": 0.0, "gm_rnorm0": 0.0}
    hist = []

    def converged(nn, rn):
        st["reason"] = 0
        if nn == 0:
            if not guess_zero and not uirnorm:
                sn = _norm(b)
                if sn == 0.0:
                    sn = rn
                st["rnorm0"] = sn
            else:
                st["rnorm0"] = rn
            st["ttol"] = max(rtol * st["rnorm0"], abstol)
        if math.isnan(rn) or math.isinf(rn):
            st["reason"] = -9
        elif rn <= st["ttol"]:
            st["reason"] = 3 if rn < abstol else 2
        elif rn >= divtol * st["rnorm0"]:
            st["reason"] = -4

    def normalize(v):
        t = _norm(v)
        if t != 0.0 and not (math.isnan(t) or math.isinf(t)):
            s = 1.0 / t
            for i in range(n):
                v[i] = v[i] * s
        return t

    itcount = 0
    while not st["reason"]:
        if not guess_zero:
            t1 = spmv(rowptr, col, val, x)
            VV = [[b[i] + (-1.0) * t1[i] for i in range(n)]]
        else:
            VV = [list(b)]
        HH = [[0.0] * (m + 1) for _ in range(m + 2)]  # HH[row][col]
        cc = [0.0] * (m + 2)
        ss = [0.0] * (m + 2)
        grs = [0.0] * (m + 2)
        it = 0
        hapend = False
        res = normalize(VV[0])
        cyc = 0
        if math.isnan(res) or math.isinf(res):
            st["reason"] = -9
        elif st["rnorm"] > 0.0 and abs(res - st["rnorm"]) > breakdowntol * st["gm_rnorm0"]:
            st["reason"] = -5
        else:
            grs[0] = st["gm_rnorm0"] = res
            st["rnorm"] = res
            hist.append(res)
            if res == 0.0:
                st["reason"] = 3
            else:
                converged(st["its"], res)
                early_return = False
                while not st["reason"] and it < m and st["its"] < max_it:
                    if it:
                        hist.append(res)
                    w = list(spmv(rowptr, col, val, VV[it]))
                    lhh = [_dot(w, VV[j]) for j in range(it + 1)]
                    bad = any(math.isnan(v) or math.isinf(v) for v in lhh)
                    if bad:
                        st["reason"] = -9
                        break
                    lhh = [-v for v in lhh]
                    w = list(_maxpy(w, lhh, VV[: it + 1]))
                    for j in range(it + 1):
                        HH[j][it] = 0.0 - lhh[j]
                    tt = normalize(w)
                    if math.isnan(tt) or math.isinf(tt):
                        st["reason"] = -9
                        early_return = True
                        break
                    VV.append(w)
                    HH[it + 1][it] = tt
                    hapbnd = abs(tt / grs[it])
                    if hapbnd > haptol:
                        hapbnd = haptol
                    if tt < hapbnd:
                        hapend = True
                    # UpdateHessenberg
                    for j in range(1, it + 1):
                        t0 = HH[j - 1][it]
                        HH[j - 1][it] = cc[j - 1] * t0 + ss[j - 1] * HH[j][it]
                        HH[j][it] = cc[j - 1] * HH[j][it] - (ss[j - 1] * t0)
                    if not hapend:
                        t2 = math.sqrt(HH[it][it] * HH[it][it] + HH[it + 1][it] * HH[it + 1][it])
                        if t2 == 0.0:
                            st["reason"] = -2
                        else:
                            cc[it] = HH[it][it] / t2
                            ss[it] = HH[it + 1][it] / t2
                            grs[it + 1] = -(ss[it] * grs[it])
                            grs[it] = cc[it] * grs[it]
                            HH[it][it] = cc[it] * HH[it][it] + ss[it] * HH[it + 1][it]
                            res = abs(grs[it + 1])
                    else:
                        res = 0.0
                    it += 1
                    st["its"] += 1
                    st["rnorm"] = res
                    if st["reason"]:
                        break
                    converged(st["its"], res)
                    if hapend and not st["reason"]:
                        st["reason"] = -5
                        break
                if not early_return:
                    if it and (st["reason"] or st["its"] >= max_it):
                        hist.append(res)
                    cyc = it
                    # BuildSoln(it-1), nrs aliases grs
                    k_it = it - 1
                    if k_it >= 0:
                        nrs = grs
                        ok = True
                        if HH[k_it][k_it] != 0.0:
                            nrs[k_it] = grs[k_it] / HH[k_it][k_it]
                        else:
                            st["reason"] = -5
                            ok = False
                        if ok:
                            for ii in range(1, k_it + 1):
                                k = k_it - ii
                                t3 = grs[k]
                                for j in range(k + 1, k_it + 1):
                                    t3 = t3 - HH[k][j] * nrs[j]
                                if HH[k][k] == 0.0:
                                    st["reason"] = -5
                                    ok = False
                                    break
                                nrs[k] = t3 / HH[k][k]
                        if ok:
                            tmp = _maxpy([0.0] * n, nrs[: k_it + 1], VV[: k_it + 1])
                            x = [x[i] + 1.0 * float(tmp[i]) for i in range(n)]
        itcount += cyc
        if itcount >= max_it:
            if not st["reason"]:
                st["reason"] = -3
            break
        guess_zero = False
    return np.array(x), {"its": st["its"], "reason": st["reason"], "rnorm": st["rnorm"], "hist": np.array(hist)}


def lsqr(R, b, max_it=10000, rtol=1e-5, abstol=1e-50, divtol=1e4, exact_norm=False, conv_test="lsqr"):
    """KSPSolve_LSQR [PETSc-ext], PCNONE, zero initial guess, sequential sums:
    R is a list of rows (each a list of s floats), b a list.  Returns (x, its,
    reason, rnorm, hist).  Plain Python floats, one statement per PETSc Vec op."""
    m, s = len(R), len(R[0])
    hist = []

    def gemv(v):                      # MatMult: per row, columns in order, from 0
        out = []
        for i in range(m):
            acc = 0.0
            for j in range(s):
                acc = acc + v[j] * R[i][j]
            out.append(acc)
        return out

    def gemvt(u):                     # MatMultTranspose: per column, rows in order
        out = []
        for j in range(s):
            acc = 0.0
            for i in range(m):
                acc += R[i][j] * u[i]
            out.append(acc)
        return out

    def nrm(v):
        acc = 0.0
        for a in v:
            acc += a * a
        return math.sqrt(acc)

    def scale(v, a):                  # VecScale special cases
        if a == 0.0:
            return [0.0] * len(v)
        return v if a == 1.0 else [t * a for t in v]

    def axpy(y, a, x):                # VecAXPY, returns early for a == 0
        return y if a == 0.0 else [yi + a * xi for yi, xi in zip(y, x)]

    def aypx(y, a, x):                # VecAYPX special cases
        if a == 0.0:
            return list(x)
        if a == 1.0:
            return [yi + xi for yi, xi in zip(y, x)]
        return [xi + a * yi for yi, xi in zip(y, x)]

    state = {"rnorm0": 0.0, "ttol": 0.0}

    def converged(n, rn, arnorm, anorm):
        if conv_test == "skip":
            return 4 if n >= max_it else 0
        if n == 0:
            state["rnorm0"] = rn
            state["ttol"] = max(rtol * rn, abstol)
        if math.isnan(rn) or math.isinf(rn):
            return -9
        if rn <= state["ttol"]:
            return 3 if rn < abstol else 2
        if rn >= divtol * state["rnorm0"]:
            return -4
        if conv_test != "lsqr" or n == 0:
            return 0
        if arnorm < abstol:
            return 9
        if arnorm < rtol * anorm * rn:
            return 1
        return 0

    x = [0.0] * s
    u = list(b)
    rnorm = nrm(u)
    if math.isnan(rnorm) or math.isinf(rnorm):
        return x, 0, -9, rnorm, hist
    hist.append(rnorm)
    reason = converged(0, rnorm, 0.0, 0.0)
    if reason:
        return x, 0, reason, rnorm, hist
    beta = rnorm
    u = scale(u, 1.0 / beta)
    v = gemvt(u)
    alpha = nrm(v)
    v = scale(v, 1.0 / alpha)
    w = list(v)
    if exact_norm:
        acc = 0.0
        for j in range(s):
            for i in range(m):
                acc += R[i][j] * R[i][j]
        anorm = math.sqrt(acc)
    else:
        anorm = 0.0
    arnorm = alpha * beta
    phibar, rhobar = beta, alpha
    its = 0
    i = 0
    while True:
        u1 = axpy(gemv(v), -alpha, u)
        beta = nrm(u1)
        if math.isnan(beta) or math.isinf(beta):
            reason = -9
            break
        if beta > 0.0:
            u1 = scale(u1, 1.0 / beta)
            if not exact_norm:
                anorm = math.sqrt(anorm * anorm + alpha * alpha + beta * beta)
        v1 = axpy(gemvt(u1), -beta, v)
        alpha = nrm(v1)
        if math.isnan(alpha) or math.isinf(alpha):
            reason = -9
            break
        v1 = scale(v1, 1.0 / alpha)
        rho = math.sqrt(rhobar * rhobar + beta * beta)
        c, sn = rhobar / rho, beta / rho
        theta = sn * alpha
        rhobar = -c * alpha
        phi = c * phibar
        phibar = sn * phibar
        tau = sn * phi
        x = axpy(x, phi / rho, w)
        w = aypx(w, -theta / rho, v1)
        arnorm = alpha * abs(tau)
        rnorm = phibar
        its += 1
        hist.append(rnorm)
        reason = converged(i + 1, rnorm, arnorm, anorm)
        if reason:
            break
        u, v = u1, v1
        i += 1
        if i >= max_it:
            break
    if i >= max_it and not reason:
        reason = -3
    return x, its, reason, rnorm, hist
