/*
 * ksp_lsqr.c -- KSPLSQR host logic over a row-distributed dense operator.
 *
 * Restates PETSc 3.22.1's KSPSolve_LSQR with PCNONE and a zero initial guess
 * (plus KSPConvergedDefault / KSPLSQRConvergedDefault / KSPConvergedSkip) --
 * the outer least-squares solve of the minimization variants,
 * outer_solver_norm_equation (src/utils/utils.c:1061-1078), with the option
 * set of running_bulk_test_g5k:247-248.
 *
 * The reference holds all of R (N x s) on every block and runs the same LSQR
 * on each.  Here each GPU holds only its rows of R, b and the two N-length
 * work vectors U, U1; the s-length vectors and the scalar recurrence are
 * replicated (msplit_lsqr.hip).  One LSQR step is
 *   GEMV   U1 = R V - alpha U, ||U1||^2 partial   (one pass over R and U)
 *   gather block partials, beta (one lane)
 *   DOTS   U1 *= 1/beta, R^T U1 partials          (one pass over R and U1)
 *   gather block partials, the rest of the step (one lane)
 * so 2 x 8*n*(s+2) bytes of HBM traffic per block and step, and two
 * all-gathers of 1 and s doubles per block.  The host enqueues steps in
 * chunks and reads the state back once per chunk; steps past the end return
 * at once on the device's stop flag.
 *
 * The DBR default (round 5) takes both products in ONE pass over R:
 *   ONEPASS  U1 = R V - alpha U, ||U1||^2 and R^T U1 partials  (one pass over R and U)
 *   gather block partials (1 + s doubles), beta, V1 = (R^T U1) * (1/beta) - beta V, the rest (one lane)
 * 8*n*(s+3) bytes and one all-gather per block and step.  R^T U1 is taken from the unscaled U1 and
 * multiplied by 1/beta after the sum -- one rounding that differs from PETSc's order (VecScale first),
 * restated by the oracle's DBR mode (orc_lsqr_opts.onepass).  MSP_REDUCE_SEQ keeps PETSc's order;
 * MSPLIT_LSQR_ONEPASS=0 the two passes.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "msplit.h"
#include "msplit_internal.h"

#define LSQR_CHUNK 8

struct msp_lsqr {
  msp_ctx *ctx;
  msp_lsqr_opts o;
  int32_t nloc, s;
  msp_dense **R;          /* nloc local row blocks */
  msp_comm *comm;
  /* work, sized by setup() */
  int setup;
  int32_t nranks, nblk, hist_cap;
  int64_t maxn;
  double **U;             /* 2*nloc device vectors: U[k] (even steps) and U[nloc+k] */
  double *partial;        /* nchunks(maxn) * 32 */
  double *gloc, *gall;    /* nloc*s, nblk*s */
  double *floc, *fall;    /* Frobenius column sums: nloc*s, nblk*s */
  void *dblock;           /* state + V, V1, W + hist */
  mspi_lsqr_dev d;
  mspi_lsqr_state *hst;   /* pinned mirror */
  double *hist;           /* host copy */
  int nhist, its, reason;
  double rnorm, arnorm, anorm;
};

static int err(int code, const char *msg) {
  mspi_set_error(code, "%s", msg);
  return code;
}

int msp_lsqr_get_default_opts(msp_lsqr_opts *o) {
  if (!o) return err(MSP_ERR_ARG_NULL, "opts is NULL");
  o->max_it = 10000;
  o->rtol = 1e-5;
  o->abstol = 1e-50;
  o->divtol = 1e4;
  o->exact_norm = 0;
  o->conv_test = MSP_LSQR_CONV_LSQR; /* KSPCreate_LSQR installs KSPLSQRConvergedDefault */
  return MSP_SUCCESS;
}

int msp_lsqr_create(msp_ctx *ctx, msp_lsqr **out) {
  if (!ctx || !out) return err(MSP_ERR_ARG_NULL, "NULL argument");
  msp_lsqr *l = (msp_lsqr *)calloc(1, sizeof(msp_lsqr));
  if (!l) return err(MSP_ERR_MEM, "LSQR allocation failed");
  l->ctx = ctx;
  mspi_ctx_retain(ctx);
  msp_lsqr_get_default_opts(&l->o);
  *out = l;
  return MSP_SUCCESS;
}

static void lsqr_free_work(msp_lsqr *l) {
  if (l->U) {
    for (int k = 0; k < 2 * l->nloc; ++k) mspi_free(l->ctx, l->U[k]);
    free(l->U);
  }
  mspi_free(l->ctx, l->partial);
  if (l->gall != l->gloc) mspi_free(l->ctx, l->gall);
  if (l->fall != l->floc) mspi_free(l->ctx, l->fall);
  mspi_free(l->ctx, l->gloc);
  mspi_free(l->ctx, l->floc);
  mspi_free(l->ctx, l->dblock);
  if (l->hst) mspi_host_free(l->hst);
  free(l->hist);
  l->U = NULL;
  l->partial = l->gloc = l->gall = l->floc = l->fall = NULL;
  l->dblock = NULL;
  l->hst = NULL;
  l->hist = NULL;
  memset(&l->d, 0, sizeof(l->d));
  l->setup = 0;
}

int msp_lsqr_destroy(msp_lsqr **pl) {
  if (!pl || !*pl) return MSP_SUCCESS;
  msp_ctx *c = (*pl)->ctx;
  msp_ctx_synchronize(c);
  lsqr_free_work(*pl);
  free((*pl)->R);
  free(*pl);
  *pl = NULL;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

int msp_lsqr_set_opts(msp_lsqr *l, const msp_lsqr_opts *o) {
  if (!l || !o) return err(MSP_ERR_ARG_NULL, "NULL argument");
  if (o->max_it < 0 || o->rtol < 0 || o->abstol < 0) return err(MSP_ERR_ARG_OUTOFRANGE, "negative LSQR tolerance");
  if (o->conv_test < MSP_LSQR_CONV_DEFAULT || o->conv_test > MSP_LSQR_CONV_SKIP)
    return err(MSP_ERR_ARG_OUTOFRANGE, "unknown LSQR convergence test");
  if (o->max_it + 2 > l->hist_cap) lsqr_free_work(l);
  l->o = *o;
  return MSP_SUCCESS;
}

int msp_lsqr_get_opts(const msp_lsqr *l, msp_lsqr_opts *o) {
  if (!l || !o) return err(MSP_ERR_ARG_NULL, "NULL argument");
  *o = l->o;
  return MSP_SUCCESS;
}

int msp_lsqr_set_operators(msp_lsqr *l, int32_t nloc, msp_dense *const *R) {
  if (!l || !R || nloc < 1) return err(MSP_ERR_ARG_NULL, "NULL argument or no blocks");
  for (int k = 0; k < nloc; ++k) {
    if (!R[k]) return err(MSP_ERR_ARG_NULL, "R block is NULL");
    if (R[k]->ctx != l->ctx) return err(MSP_ERR_ARG_WRONG, "R block belongs to another context");
    if (R[k]->ncols != R[0]->ncols) return err(MSP_ERR_ARG_SIZ, "R blocks differ in column count");
  }
  lsqr_free_work(l);
  free(l->R);
  l->R = (msp_dense **)malloc((size_t)nloc * sizeof(msp_dense *));
  if (!l->R) return err(MSP_ERR_MEM, "allocation failed");
  memcpy(l->R, R, (size_t)nloc * sizeof(msp_dense *));
  l->nloc = nloc;
  l->s = R[0]->ncols;
  return MSP_SUCCESS;
}

int msp_lsqr_set_comm(msp_lsqr *l, msp_comm *comm) {
  if (!l) return err(MSP_ERR_ARG_NULL, "lsqr is NULL");
  lsqr_free_work(l);
  l->comm = comm;
  return MSP_SUCCESS;
}

static int64_t nchunks(int64_t n) { return (n + 4095) / 4096; }

static int lsqr_setup(msp_lsqr *l) {
  if (l->setup) return MSP_SUCCESS;
  int rc;
  int32_t rank;
  mspi_comm_size(l->comm, &l->nranks, &rank);
  l->nblk = l->nranks * l->nloc;
  l->hist_cap = l->o.max_it + 2;
  l->maxn = 0;
  for (int k = 0; k < l->nloc; ++k)
    if (l->R[k]->nrows > l->maxn) l->maxn = l->R[k]->nrows;
  const int s = l->s;
  l->U = (double **)calloc((size_t)l->nloc * 2u, sizeof(double *));
  if (!l->U) return err(MSP_ERR_MEM, "allocation failed");
  for (int k = 0; k < 2 * l->nloc; ++k) {
    const int64_t n = l->R[k % l->nloc]->nrows;
    if ((rc = mspi_malloc(l->ctx, (void **)&l->U[k], (size_t)((n + 511) / 512 * 512 + 512) * sizeof(double))))
      goto fail;
  }
  const int64_t nch = nchunks(l->maxn) > 0 ? nchunks(l->maxn) : 1;
  const int64_t pw = s + 1 > 32 ? s + 1 : 32; /* partials per chunk: the one-pass step's 1 + s */
  if ((rc = mspi_malloc(l->ctx, (void **)&l->partial, (size_t)nch * pw * sizeof(double)))) goto fail;
  if ((rc = mspi_malloc(l->ctx, (void **)&l->gloc, (size_t)l->nloc * (s + 1) * sizeof(double)))) goto fail;
  if ((rc = mspi_malloc(l->ctx, (void **)&l->floc, (size_t)l->nloc * s * sizeof(double)))) goto fail;
  if (l->comm) {
    if ((rc = mspi_malloc(l->ctx, (void **)&l->gall, (size_t)l->nblk * (s + 1) * sizeof(double)))) goto fail;
    if ((rc = mspi_malloc(l->ctx, (void **)&l->fall, (size_t)l->nblk * s * sizeof(double)))) goto fail;
  } else { /* every block is local: the local partials are the gathered ones */
    l->gall = l->gloc;
    l->fall = l->floc;
  }
  const size_t st_bytes = (sizeof(mspi_lsqr_state) + 255) / 256 * 256;
  const size_t bytes = st_bytes + (size_t)(3 * s + l->hist_cap) * sizeof(double);
  if ((rc = mspi_malloc(l->ctx, &l->dblock, bytes))) goto fail;
  if ((rc = mspi_host_malloc((void **)&l->hst, sizeof(mspi_lsqr_state)))) goto fail;
  l->hist = (double *)malloc((size_t)l->hist_cap * sizeof(double));
  if (!l->hist) {
    rc = err(MSP_ERR_MEM, "allocation failed");
    goto fail;
  }
  char *p = (char *)l->dblock;
  l->d.st = (mspi_lsqr_state *)p;
  l->d.V = (double *)(p + st_bytes);
  l->d.V1 = l->d.V + s;
  l->d.W = l->d.V1 + s;
  l->d.hist = l->d.W + s;
  l->d.g = l->gall;
  l->setup = 1;
  return MSP_SUCCESS;
fail:
  lsqr_free_work(l);
  return rc;
}

/* MSP_REDUCE_SEQ: overwrite the nloc block partials in loc (m per block, ncol used) with
 * one sequential sum chained across the blocks (the reference's LSQR runs on one rank
 * over all of R, SMSM-global.c:136), carried by the last block's slot.  x[k] + j*ldx
 * is column j of block k (ldx = 0 with ncol = 1: a vector); y[k] the vector it is
 * dotted with (y = x: a squared norm); frob: every column's squares in one sum. */
static int seq_chain(msp_lsqr *l, double *const *x, int64_t ldx_R, double *const *y, int ncol, int frob,
                     double *loc, int m) {
  mspi_seq_segs sg;
  memset(&sg, 0, sizeof(sg));
  sg.nseg = l->nloc;
  for (int k = 0; k < l->nloc; ++k) {
    sg.x[k] = x ? x[k] : l->R[k]->d;
    sg.ldx[k] = ldx_R ? l->R[k]->lda : 0;
    sg.y[k] = y ? y[k] : (x ? x[k] : NULL);
    sg.n[k] = l->R[k]->nrows;
  }
  return mspi_seq_chain(l->ctx, &sg, ncol, frob, loc, m, &l->d.st->stop);
}

/* all-gather nloc*m local partials into gall (block order over ranks) */
static int gather(msp_lsqr *l, const double *loc, double *all, int m) {
  if (!l->comm) return MSP_SUCCESS;
  return mspi_comm_allgather(l->comm, loc, all, (int64_t)l->nloc * m);
}

int msp_lsqr_solve(msp_lsqr *l, msp_vec *const *b, msp_vec *x) {
  if (!l || !b || !x) return err(MSP_ERR_ARG_NULL, "NULL argument");
  if (!l->R) return err(MSP_ERR_ARG_WRONG, "msp_lsqr_set_operators was not called");
  if (x->n != l->s) return err(MSP_ERR_ARG_SIZ, "x must have one entry per column of R");
  for (int k = 0; k < l->nloc; ++k) {
    if (!b[k]) return err(MSP_ERR_ARG_NULL, "b block is NULL");
    if (b[k]->n != l->R[k]->nrows) return err(MSP_ERR_ARG_SIZ, "b block and R block differ in rows");
  }
  int rc;
  if ((rc = mspi_set_device(l->ctx)) || (rc = lsqr_setup(l))) return rc;
  msp_ctx *c = l->ctx;
  const int seq = mspi_reduce_seq(c);
  if (seq && (l->nranks > 1 || l->nloc > MSPI_SEQ_MAXSEG))
    return err(MSP_ERR_SUP, "MSP_REDUCE_SEQ chains the LSQR sums across the row blocks of one process only");
  double *bd[MSPI_SEQ_MAXSEG];
  for (int k = 0; k < l->nloc && seq; ++k) bd[k] = b[k]->d;
  const int s = l->s, nloc = l->nloc;
  const int *stop = &l->d.st->stop;
  mspi_lsqr_dev d = l->d;
  d.X = x->d;

  mspi_lsqr_state *h = l->hst;
  memset(h, 0, sizeof(*h));
  h->max_it = l->o.max_it;
  h->conv_test = l->o.conv_test;
  h->exact_norm = l->o.exact_norm;
  h->hist_cap = l->hist_cap;
  h->s = s;
  h->nblk = l->nblk;
  h->rtol = l->o.rtol;
  h->abstol = l->o.abstol;
  h->divtol = l->o.divtol;
  if ((rc = mspi_h2d_async(c, d.st, h, sizeof(*h)))) return rc;

  /* u <- b; rnorm = ||u|| (n = 0 test); u *= 1/beta; V = R^T u */
  for (int k = 0; k < nloc; ++k)
    if ((rc = mspi_norm2sq(c, b[k]->d, b[k]->n, l->gloc + k))) return rc;
  if (seq && (rc = seq_chain(l, bd, 0, NULL, 1, 0, l->gloc, 1))) return rc;
  if ((rc = gather(l, l->gloc, l->gall, 1)) || (rc = mspi_ls_start(c, d))) return rc;
  if (l->o.exact_norm) {
    for (int k = 0; k < nloc; ++k)
      if ((rc = mspi_dense_colsumsq(c, l->R[k]->d, l->R[k]->lda, s, l->R[k]->nrows, l->partial, l->floc + k * s)))
        return rc;
    if (seq && (rc = seq_chain(l, NULL, 1, NULL, s, 1, l->floc, s))) return rc;
    if ((rc = gather(l, l->floc, l->fall, s))) return rc;
  }
  for (int k = 0; k < nloc; ++k)
    if ((rc = mspi_dense_scaled_dots(c, b[k]->d, l->U[k], &d.st->uscale, l->R[k]->d, l->R[k]->lda, s,
                                     l->R[k]->nrows, l->partial, l->gloc + k * s, stop)))
      return rc;
  if (seq && (rc = seq_chain(l, NULL, 1, l->U, s, 0, l->gloc, s))) return rc;
  if ((rc = gather(l, l->gloc, l->gall, s)) || (rc = mspi_ls_first(c, d, l->o.exact_norm ? l->fall : NULL)))
    return rc;

  /* Deferred VecScale (DBR order): U1 *= 1/beta is applied where U1 is read -- in the R^T U1 dots and, as U, in
   * the next step's R V - alpha U -- instead of being written back: the same roundings, one N-vector write per
   * step less (SEQ mode re-reads the scaled U1 for its sequential sums, so it keeps the write). */
  static int write_back = -1; /* MSPLIT_LSQR_SCALE_WRITE=1: the round-2 write-back (same-box A/B) */
  if (write_back < 0) {
    const char *e = getenv("MSPLIT_LSQR_SCALE_WRITE");
    write_back = e && e[0] == '1';
  }
  const int defer = !seq && !write_back;
  /* MSPLIT_LSQR_ONEPASS=0: the two passes, PETSc's operation order (same-box A/B; the oracle's onepass = 0);
   * read per solve, so a test can switch it */
  const char *ope = getenv("MSPLIT_LSQR_ONEPASS");
  const int onepass = defer && !(ope && ope[0] == '0');
  const int nsteps = l->o.max_it > 0 ? l->o.max_it : 1; /* the do-while runs at least once */
  for (int i = 0; i < nsteps; ++i) {
    double **U = l->U + (i & 1 ? nloc : 0);
    double **U1 = l->U + (i & 1 ? 0 : nloc);
    /* U of step 0 is the scaled b (written by the first dots); later it is the previous U1, stored unscaled,
     * whose scale 1/beta is still in st->uscale until this step's beta replaces it */
    const double *usc = defer && i > 0 ? &d.st->uscale : NULL;
    if (onepass) { /* one pass over R: U1, ||U1||^2 and R^T U1 (unscaled) per block, one gather, one lane */
      for (int k = 0; k < nloc; ++k)
        if ((rc = mspi_dense_lsqr_onepass(c, l->R[k]->d, l->R[k]->lda, s, l->R[k]->nrows, d.V, &d.st->nalpha, U[k],
                                          usc, U1[k], l->partial, l->gloc + k * (s + 1), stop)))
          return rc;
      if ((rc = gather(l, l->gloc, l->gall, s + 1)) || (rc = mspi_ls_onepass_step(c, d))) return rc;
      if ((i + 1) % LSQR_CHUNK == 0 || i + 1 == nsteps) {
        if ((rc = mspi_d2h_sync(c, h, d.st, sizeof(*h)))) return rc;
        if (h->stop) break;
      }
      continue;
    }
    for (int k = 0; k < nloc; ++k)
      if ((rc = mspi_dense_gemv(c, l->R[k]->d, l->R[k]->lda, s, l->R[k]->nrows, d.V, &d.st->nalpha, U[k], usc,
                                U1[k], l->partial, l->gloc + k, stop)))
        return rc;
    if (seq && (rc = seq_chain(l, U1, 0, NULL, 1, 0, l->gloc, 1))) return rc;
    if ((rc = gather(l, l->gloc, l->gall, 1)) || (rc = mspi_ls_beta(c, d))) return rc;
    for (int k = 0; k < nloc; ++k)
      if ((rc = mspi_dense_scaled_dots(c, U1[k], defer ? NULL : U1[k], &d.st->uscale, l->R[k]->d, l->R[k]->lda, s,
                                       l->R[k]->nrows, l->partial, l->gloc + k * s, stop)))
        return rc;
    if (seq && (rc = seq_chain(l, NULL, 1, U1, s, 0, l->gloc, s))) return rc;
    if ((rc = gather(l, l->gloc, l->gall, s)) || (rc = mspi_ls_step(c, d))) return rc;
    if ((i + 1) % LSQR_CHUNK == 0 || i + 1 == nsteps) {
      if ((rc = mspi_d2h_sync(c, h, d.st, sizeof(*h)))) return rc;
      if (h->stop) break;
    }
  }
  if ((rc = mspi_d2h_sync(c, h, d.st, sizeof(*h)))) return rc;
  l->its = h->its;
  l->reason = h->reason;
  l->rnorm = h->rnorm;
  l->arnorm = h->arnorm;
  l->anorm = h->anorm;
  l->nhist = h->nhist < l->hist_cap ? h->nhist : l->hist_cap;
  if (l->nhist > 0 && (rc = mspi_d2h_sync(c, l->hist, d.hist, (size_t)l->nhist * sizeof(double)))) return rc;
  return MSP_SUCCESS;
}

int msp_lsqr_get_iteration_number(const msp_lsqr *l, int32_t *its) {
  if (!l || !its) return err(MSP_ERR_ARG_NULL, "NULL argument");
  *its = l->its;
  return MSP_SUCCESS;
}

int msp_lsqr_get_residual_norm(const msp_lsqr *l, double *rnorm) {
  if (!l || !rnorm) return err(MSP_ERR_ARG_NULL, "NULL argument");
  *rnorm = l->rnorm;
  return MSP_SUCCESS;
}

int msp_lsqr_get_converged_reason(const msp_lsqr *l, int32_t *reason) {
  if (!l || !reason) return err(MSP_ERR_ARG_NULL, "NULL argument");
  *reason = l->reason;
  return MSP_SUCCESS;
}

int msp_lsqr_get_norms(const msp_lsqr *l, double *arnorm, double *anorm) {
  if (!l) return err(MSP_ERR_ARG_NULL, "lsqr is NULL");
  if (arnorm) *arnorm = l->arnorm;
  if (anorm) *anorm = l->anorm;
  return MSP_SUCCESS;
}

int msp_lsqr_get_residual_history(const msp_lsqr *l, const double **hist, int32_t *n) {
  if (!l || !hist || !n) return err(MSP_ERR_ARG_NULL, "NULL argument");
  *hist = l->hist;
  *n = l->nhist;
  return MSP_SUCCESS;
}
