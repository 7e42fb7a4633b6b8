/*
 * ksp_gmres.c -- KSPGMRES host logic over device-resident Krylov vectors.
 *
 * Restates PETSc 3.22.1's KSPSolve_GMRES / KSPGMRESCycle / classical
 * Gram-Schmidt (REFINE_NEVER) / KSPGMRESUpdateHessenberg / KSPGMRESBuildSoln /
 * KSPConvergedDefault with PCNONE -- the inner solve the reference calls from
 * inner_solver() (src/utils/utils.c:950-970) and gmres_solution.c:70.
 *
 * Data layout: the m+1 basis vectors VV(0..m) are one HBM allocation,
 * (m+1) x stride doubles, stride = n rounded up to 512 (4 KiB aligned).
 * Per Arnoldi step the device runs SpMV, the fused MDot (DBR), MAXPY with the
 * MDot results read straight from HBM, and the squared norm; ONE synchronising
 * copy brings h(0..it) and ||w||^2 to the host, which updates the 31x30
 * Hessenberg/Givens state (negligible) exactly as PETSc does and launches the
 * scale.  The host never touches vector data.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "msplit.h"
#include "msplit_internal.h"

#define PMAX(a, b) ((a) < (b) ? (b) : (a)) /* PetscMax */

struct msp_ksp {
  msp_ctx *ctx;
  msp_mat *A;
  msp_ksp_opts o;
  int setup;
  int m_alloc;
  int64_t n, stride;
  double *basis;   /* device: (m+1) * stride */
  double **VV;     /* host array of device pointers */
  double *tmp;     /* device: BuildSoln temporary when it+1 > 32 */
  double *dh;      /* device: h(0..it), ||w||^2 */
  double *hbuf;    /* pinned host copy of dh */
  double *hh, *cc, *ss, *grs, *lhh; /* host Hessenberg state */
  double *hist;
  int hist_cap, nhist;
  /* KSP state of the current solve */
  int its, reason, guess_zero;
  double rnorm, rnorm0, ttol, gm_rnorm0;
  const double *b;
  double *x;
};

#define HH(k, a, b) ((k)->hh[(int64_t)(b) * ((k)->o.restart + 2) + (a)])

static int is_bad(double v) { return isnan(v) || isinf(v); }

int msp_ksp_get_default_opts(msp_ksp_opts *o) {
  if (!o) {
    mspi_set_error(MSP_ERR_ARG_NULL, "opts is NULL");
    return MSP_ERR_ARG_NULL;
  }
  o->restart = 30;
  o->max_it = 10000;
  o->rtol = 1e-5;
  o->abstol = 1e-50;
  o->divtol = 1e4;
  o->haptol = 1e-30;
  o->breakdowntol = 0.1;
  o->uirnorm = 0;
  o->guess_nonzero = 0;
  return MSP_SUCCESS;
}

int msp_ksp_create(msp_ctx *ctx, msp_ksp **out) {
  if (!ctx || !out) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  msp_ksp *k = (msp_ksp *)calloc(1, sizeof(msp_ksp));
  if (!k) {
    mspi_set_error(MSP_ERR_MEM, "KSP allocation failed");
    return MSP_ERR_MEM;
  }
  k->ctx = ctx;
  msp_ksp_get_default_opts(&k->o);
  *out = k;
  return MSP_SUCCESS;
}

static void ksp_free_work(msp_ksp *k) {
  if (k->basis) mspi_free(k->ctx, k->basis);
  if (k->tmp) mspi_free(k->ctx, k->tmp);
  if (k->dh) mspi_free(k->ctx, k->dh);
  if (k->hbuf) mspi_host_free(k->hbuf);
  free(k->VV);
  free(k->hh);
  free(k->cc);
  free(k->ss);
  free(k->grs);
  free(k->lhh);
  free(k->hist);
  k->basis = k->tmp = k->dh = k->hbuf = NULL;
  k->VV = NULL;
  k->hh = k->cc = k->ss = k->grs = k->lhh = k->hist = NULL;
  k->setup = 0;
}

int msp_ksp_destroy(msp_ksp **pk) {
  if (!pk || !*pk) return MSP_SUCCESS;
  msp_ctx_synchronize((*pk)->ctx);
  ksp_free_work(*pk);
  free(*pk);
  *pk = NULL;
  return MSP_SUCCESS;
}

int msp_ksp_set_operators(msp_ksp *k, msp_mat *A) {
  if (!k || !A) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  int32_t nr, nc;
  mspi_mat_dims(A, &nr, &nc);
  if (nr != nc) {
    mspi_set_error(MSP_ERR_ARG_SIZ, "KSP operator must be square, got %d x %d", nr, nc);
    return MSP_ERR_ARG_SIZ;
  }
  if (mspi_mat_ctx(A) != k->ctx) {
    mspi_set_error(MSP_ERR_ARG_WRONG, "operator belongs to another context");
    return MSP_ERR_ARG_WRONG;
  }
  if (k->A && k->n != nr) ksp_free_work(k);
  k->A = A;
  k->n = nr;
  return MSP_SUCCESS;
}

int msp_ksp_set_opts(msp_ksp *k, const msp_ksp_opts *o) {
  if (!k || !o) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  if (o->restart < 1 || o->max_it < 0 || o->rtol < 0 || o->abstol < 0 || o->divtol < 0) {
    mspi_set_error(MSP_ERR_ARG_OUTOFRANGE, "invalid KSP options (restart %d, max_it %d)", o->restart, o->max_it);
    return MSP_ERR_ARG_OUTOFRANGE;
  }
  if (k->setup && o->restart != k->o.restart) ksp_free_work(k);
  k->o = *o;
  return MSP_SUCCESS;
}

int msp_ksp_get_opts(const msp_ksp *k, msp_ksp_opts *o) {
  if (!k || !o) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  *o = k->o;
  return MSP_SUCCESS;
}

int msp_ksp_set_up(msp_ksp *k) {
  if (!k || !k->A) {
    mspi_set_error(MSP_ERR_ARG_WRONG, "KSPSetUp before KSPSetOperators");
    return MSP_ERR_ARG_WRONG;
  }
  if (k->setup) return MSP_SUCCESS;
  const int m = k->o.restart;
  /* an extra skew between basis vectors measured no gain in the solve
   * (same-box A/B, profiles/r01/README.md); kept as a tuning knob */
  int64_t skew = 0;
  const char *env = getenv("MSPLIT_BASIS_SKEW"); /* tuning knob, doubles, rounded to 512 */
  if (env) skew = (atoll(env) + 511) / 512 * 512;
  k->stride = (k->n + 511) / 512 * 512 + skew;
  int rc = mspi_malloc(k->ctx, (void **)&k->basis, (size_t)(m + 1) * (size_t)k->stride * sizeof(double) + 4096);
  if (!rc) rc = mspi_malloc(k->ctx, (void **)&k->dh, (size_t)(m + 2) * sizeof(double));
  if (!rc) rc = mspi_host_malloc((void **)&k->hbuf, (size_t)(m + 2) * sizeof(double));
  if (!rc && m + 1 > MSPI_MAX_GROUP) rc = mspi_malloc(k->ctx, (void **)&k->tmp, (size_t)k->stride * sizeof(double) + 4096);
  k->VV = (double **)calloc((size_t)m + 1, sizeof(double *));
  k->hh = (double *)calloc((size_t)(m + 2) * (size_t)(m + 1), sizeof(double));
  k->cc = (double *)calloc((size_t)m + 2, sizeof(double));
  k->ss = (double *)calloc((size_t)m + 2, sizeof(double));
  k->grs = (double *)calloc((size_t)m + 2, sizeof(double));
  k->lhh = (double *)calloc((size_t)m + 2, sizeof(double));
  k->hist_cap = 1024;
  k->hist = (double *)calloc((size_t)k->hist_cap, sizeof(double));
  if (!rc && (!k->VV || !k->hh || !k->cc || !k->ss || !k->grs || !k->lhh || !k->hist)) {
    mspi_set_error(MSP_ERR_MEM, "host allocation failed");
    rc = MSP_ERR_MEM;
  }
  if (rc) {
    ksp_free_work(k);
    return rc;
  }
  for (int j = 0; j <= m; ++j) k->VV[j] = k->basis + (int64_t)j * k->stride;
  k->m_alloc = m;
  k->setup = 1;
  return MSP_SUCCESS;
}

static void log_res(msp_ksp *k, double r) {
  if (k->nhist >= k->hist_cap) {
    int cap = k->hist_cap * 2;
    double *h = (double *)realloc(k->hist, (size_t)cap * sizeof(double));
    if (!h) return; /* history truncated; the solve itself is unaffected */
    k->hist = h;
    k->hist_cap = cap;
  }
  k->hist[k->nhist++] = r;
}

/* device squared norm -> host norm (VecNorm NORM_2: sqrt of the dot) */
static int dev_norm(msp_ksp *k, const double *v, double *out) {
  int rc = mspi_norm2sq(k->ctx, v, k->n, k->dh);
  if (!rc) rc = mspi_d2h_sync(k->ctx, k->hbuf, k->dh, sizeof(double));
  if (!rc) *out = sqrt(k->hbuf[0]);
  return rc;
}

/* VecNormalize */
static int dev_normalize(msp_ksp *k, double *v, double *out) {
  double t = 0.0;
  int rc = dev_norm(k, v, &t);
  if (rc) return rc;
  if (t != 0.0 && !is_bad(t)) {
    const double s = 1.0 / t;
    rc = mspi_scale(k->ctx, v, k->n, s);
  }
  *out = t;
  return rc;
}

/* KSPConvergedDefault [PETSc-ext] */
static int converged(msp_ksp *k, int n, double rnorm) {
  k->reason = MSP_CONVERGED_ITERATING;
  if (n == 0) {
    if (!k->guess_zero && !k->o.uirnorm) {
      double snorm = 0.0;
      int rc = dev_norm(k, k->b, &snorm);
      if (rc) return rc;
      if (snorm == 0.0) snorm = rnorm;
      k->rnorm0 = snorm;
    } else {
      k->rnorm0 = rnorm;
    }
    k->ttol = PMAX(k->o.rtol * k->rnorm0, k->o.abstol);
  }
  if (is_bad(rnorm)) k->reason = MSP_DIVERGED_NANORINF;
  else if (rnorm <= k->ttol) k->reason = (rnorm < k->o.abstol) ? MSP_CONVERGED_ATOL : MSP_CONVERGED_RTOL;
  else if (rnorm >= k->o.divtol * k->rnorm0) k->reason = MSP_DIVERGED_DTOL;
  return MSP_SUCCESS;
}

/* KSPGMRESUpdateHessenberg [PETSc-ext] */
static void update_hessenberg(msp_ksp *k, int it, int hapend, double *res) {
  double *hh = &HH(k, 0, it);
  for (int j = 1; j <= it; ++j) {
    const double tt = hh[j - 1];
    hh[j - 1] = k->cc[j - 1] * tt + k->ss[j - 1] * hh[j];
    hh[j] = k->cc[j - 1] * hh[j] - (k->ss[j - 1] * tt);
  }
  if (!hapend) {
    const double tt = sqrt(hh[it] * hh[it] + hh[it + 1] * hh[it + 1]);
    if (tt == 0.0) {
      k->reason = MSP_DIVERGED_NULL;
      return;
    }
    k->cc[it] = hh[it] / tt;
    k->ss[it] = hh[it + 1] / tt;
    k->grs[it + 1] = -(k->ss[it] * k->grs[it]);
    k->grs[it] = k->cc[it] * k->grs[it];
    hh[it] = k->cc[it] * hh[it] + k->ss[it] * hh[it + 1];
    *res = fabs(k->grs[it + 1]);
  } else {
    *res = 0.0;
  }
}

/* KSPGMRESBuildSoln(GRS(0), x, x, ksp, it) [PETSc-ext]: back-solve on the host,
 * then x += sum_j nrs_j VV(j) in one device pass (VecSet(T,0); VecMAXPY(T);
 * KSPUnwindPreconditioner (PCNONE); VecAXPY(x, 1, T)). */
static int build_soln(msp_ksp *k, int it) {
  if (it < 0) return MSP_SUCCESS;
  double *nrs = k->grs;
  if (HH(k, it, it) != 0.0) {
    nrs[it] = k->grs[it] / HH(k, it, it);
  } else {
    k->reason = MSP_DIVERGED_BREAKDOWN;
    return MSP_SUCCESS;
  }
  for (int ii = 1; ii <= it; ++ii) {
    const int kk = it - ii;
    double tt = k->grs[kk];
    for (int j = kk + 1; j <= it; ++j) tt = tt - HH(k, kk, j) * nrs[j];
    if (HH(k, kk, kk) == 0.0) {
      k->reason = MSP_DIVERGED_BREAKDOWN;
      return MSP_SUCCESS;
    }
    nrs[kk] = tt / HH(k, kk, kk);
  }
  if (it + 1 <= MSPI_MAX_GROUP)
    return mspi_maxpy(k->ctx, k->x, it + 1, (const double *const *)k->VV, k->n, nrs, NULL, 0, 1);
  int rc = mspi_set(k->ctx, k->tmp, k->n, 0.0);
  if (!rc) rc = mspi_maxpy(k->ctx, k->tmp, it + 1, (const double *const *)k->VV, k->n, nrs, NULL, 0, 0);
  if (!rc) {
    const double *one[1] = {k->tmp};
    const double a1 = 1.0;
    /* VecAXPY(x, 1.0, T): x + 1.0*T == x + T, a one-vector MAXPY */
    rc = mspi_maxpy(k->ctx, k->x, 1, one, k->n, &a1, NULL, 0, 0);
  }
  return rc;
}

/* KSPGMRESCycle [PETSc-ext] */
static int cycle(msp_ksp *k, int *itcount) {
  const int m = k->o.restart;
  int it = 0, hapend = 0, rc;
  double res = 0.0;
  *itcount = 0;
  if ((rc = dev_normalize(k, k->VV[0], &res))) return rc;
  if (is_bad(res)) { /* KSPCheckNorm */
    k->reason = MSP_DIVERGED_NANORINF;
    return MSP_SUCCESS;
  }
  if (k->rnorm > 0.0 && fabs(res - k->rnorm) > k->o.breakdowntol * k->gm_rnorm0) {
    k->reason = MSP_DIVERGED_BREAKDOWN;
    return MSP_SUCCESS;
  }
  k->grs[0] = k->gm_rnorm0 = res;
  k->rnorm = res;
  log_res(k, res);
  if (res == 0.0) {
    k->reason = MSP_CONVERGED_ATOL;
    return MSP_SUCCESS;
  }
  if ((rc = converged(k, k->its, res))) return rc;
  while (!k->reason && it < m && k->its < k->o.max_it) {
    if (it) log_res(k, res);
    double *w = k->VV[it + 1];
    /* KSP_PCApplyBAorAB (PCNONE): w = A VV(it) */
    if ((rc = mspi_spmv(k->A, k->VV[it], w))) return rc;
    /* CGS: h = VecMDot(w, VV(0..it)); VecMAXPY(w, -h, VV); then ||w||^2 -- one sync */
    if ((rc = mspi_mdot(k->ctx, w, it + 1, (const double *const *)k->VV, k->n, k->dh))) return rc;
    if ((rc = mspi_maxpy_norm(k->ctx, w, it + 1, (const double *const *)k->VV, k->n, k->dh, 1, k->dh + it + 1)))
      return rc;
    if ((rc = mspi_d2h_sync(k->ctx, k->hbuf, k->dh, (size_t)(it + 2) * sizeof(double)))) return rc;
    double *hh = &HH(k, 0, it);
    int bad = 0;
    for (int j = 0; j <= it; ++j) {
      hh[j] = 0.0;
      if (is_bad(k->hbuf[j])) bad = 1;
      k->lhh[j] = -k->hbuf[j];
    }
    if (bad) { /* KSPCheckDot in the orthogonalization */
      k->reason = MSP_DIVERGED_NANORINF;
      break;
    }
    for (int j = 0; j <= it; ++j) hh[j] -= k->lhh[j];
    /* VecNormalize(VV(it+1)) */
    const double tt = sqrt(k->hbuf[it + 1]);
    if (is_bad(tt)) { /* KSPCheckNorm: return without BuildSoln */
      k->reason = MSP_DIVERGED_NANORINF;
      return MSP_SUCCESS;
    }
    if (tt != 0.0) {
      const double s = 1.0 / tt;
      if ((rc = mspi_scale(k->ctx, w, k->n, s))) return rc;
    }
    HH(k, it + 1, it) = tt;
    double hapbnd = fabs(tt / k->grs[it]);
    if (hapbnd > k->o.haptol) hapbnd = k->o.haptol;
    if (tt < hapbnd) hapend = 1;
    update_hessenberg(k, it, hapend, &res);
    it++;
    k->its++;
    k->rnorm = res;
    if (k->reason) break;
    if ((rc = converged(k, k->its, res))) return rc;
    if (hapend && !k->reason) {
      k->reason = MSP_DIVERGED_BREAKDOWN;
      break;
    }
  }
  if (it && (k->reason || k->its >= k->o.max_it)) log_res(k, res);
  *itcount = it;
  return build_soln(k, it - 1);
}

int msp_ksp_solve(msp_ksp *k, const msp_vec *b, msp_vec *x) {
  if (!k || !b || !x) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  if (!k->A) {
    mspi_set_error(MSP_ERR_ARG_WRONG, "KSPSolve before KSPSetOperators");
    return MSP_ERR_ARG_WRONG;
  }
  if (b->n != k->n || x->n != k->n) {
    mspi_set_error(MSP_ERR_ARG_SIZ, "KSPSolve sizes: operator %lld, b %lld, x %lld", (long long)k->n,
                   (long long)b->n, (long long)x->n);
    return MSP_ERR_ARG_SIZ;
  }
  if (b->d == x->d) {
    mspi_set_error(MSP_ERR_ARG_WRONG, "b and x must be different vectors");
    return MSP_ERR_ARG_WRONG;
  }
  int rc = mspi_set_device(k->ctx);
  if (!rc) rc = msp_ksp_set_up(k);
  if (rc) return rc;
  k->b = b->d;
  k->x = x->d;
  k->nhist = 0;
  k->its = 0;
  k->reason = MSP_CONVERGED_ITERATING;
  k->rnorm = -1.0; /* special marker for KSPGMRESCycle() */
  k->guess_zero = !k->o.guess_nonzero;
  if (k->guess_zero && (rc = mspi_set(k->ctx, k->x, k->n, 0.0))) return rc;
  int itcount = 0;
  while (!k->reason) {
    /* KSPInitialResidual: VV(0) = b - A x, or b for a zero guess */
    if (!k->guess_zero) rc = mspi_residual(k->A, k->b, k->x, k->VV[0]);
    else rc = mspi_copy(k->ctx, k->VV[0], k->b, k->n);
    if (rc) return rc;
    int its = 0;
    if ((rc = cycle(k, &its))) return rc;
    itcount += its;
    if (itcount >= k->o.max_it) {
      if (!k->reason) k->reason = MSP_DIVERGED_ITS;
      break;
    }
    k->guess_zero = 0;
  }
  return msp_ctx_synchronize(k->ctx);
}

int msp_ksp_get_iteration_number(const msp_ksp *k, int32_t *its) {
  if (!k || !its) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  *its = k->its;
  return MSP_SUCCESS;
}

int msp_ksp_get_residual_norm(const msp_ksp *k, double *rnorm) {
  if (!k || !rnorm) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  *rnorm = k->rnorm;
  return MSP_SUCCESS;
}

int msp_ksp_get_converged_reason(const msp_ksp *k, int32_t *reason) {
  if (!k || !reason) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  *reason = k->reason;
  return MSP_SUCCESS;
}

int msp_ksp_get_residual_history(const msp_ksp *k, const double **hist, int32_t *n) {
  if (!k || !hist || !n) {
    mspi_set_error(MSP_ERR_ARG_NULL, "NULL argument");
    return MSP_ERR_ARG_NULL;
  }
  *hist = k->hist;
  *n = k->nhist < k->hist_cap ? k->nhist : k->hist_cap;
  return MSP_SUCCESS;
}
