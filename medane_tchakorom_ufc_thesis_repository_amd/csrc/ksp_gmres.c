/*
 * ksp_gmres.c -- KSPGMRES host logic over device-resident Krylov vectors.
 *
 * Restates PETSc 3.22.1's KSPSolve_GMRES / KSPGMRESCycle / classical
 * Gram-Schmidt (REFINE_NEVER) / KSPGMRESUpdateHessenberg / KSPGMRESBuildSoln /
 * KSPConvergedDefault with PCNONE -- the inner solve the reference calls from
 * inner_solver() (src/utils/utils.c:950-970) and gmres_solution.c:70.
 *
 * Division of labour.  This file owns the solve: options, the restart loop of
 * KSPSolve_GMRES, the order of every operation, and the decision to start
 * another cycle.  The per-iteration scalar steps of KSPGMRESCycle (Givens
 * update, happy-breakdown and convergence tests, residual history) run in
 * one-lane device kernels (msplit_gmres.hip) on a device-resident state, so a
 * whole restart cycle is enqueued without a host round trip; the host reads
 * the state back once per cycle.  Iterations past a convergence are enqueued
 * speculatively and return at once on the device's stop flag.
 *
 * Per Arnoldi step (VV = basis in HBM, sc = its scales on the device):
 *   SpMV      W = A (sc[it]*VV(it))                  (VecNormalize of the
 *             previous vector deferred: VV(it) stays as the MAXPY stored it and
 *             every reader multiplies by sc[it] = 1/||VV(it)||, which rounds each
 *             element exactly as VecScale would have stored it)
 *   MDot      h(0..it) = W . sc.VV(0..it)            (DBR order)
 *   MAXPY     VV(it+1) = W - sum h_j sc[j] VV(j), and ||VV(it+1)||^2   (one pass)
 *   update    the Hessenberg column, Givens rotation, tests, sc[it+1] (one lane)
 * W is PETSc's VEC_VV(it+1) before the orthogonalisation; keeping it in its own
 * vector makes the MAXPY write a different vector than it reads (an in-place
 * MAXPY measured 5 % slower, same box).
 *
 * Data layout: VV(0..min(m, max_it)) are one allocation, (min(m, max_it)+1) x stride doubles, stride =
 * n rounded up to 512 (4 KiB aligned); W is separate.  KSPInitialResidual
 * writes VV(0).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "msplit.h"
#include "msplit_internal.h"

/* Captured restart cycles (HIP graphs), keyed by everything the capture baked
 * in: the operator and the kernels its products launch, the context's DBR
 * partial buffer (its epoch), x, the cycle length K, the tuning flags and the launch-shape overrides.  The basis, W and the device state are fixed
 * between ksp_free_work calls, which drop the cache. */
#define KSP_NGRAPH 4
typedef struct {
  void *exec;
  const msp_mat *A;
  uint64_t aver, epoch;
  const double *x;
  int K, tuning, shape;
} ksp_graph;

struct msp_ksp {
  msp_ctx *ctx;
  ksp_graph graphs[KSP_NGRAPH];
  int gnext;
  int graphs_off; /* a capture failed on this KSP's stream (e.g. the legacy null stream): eager from then on */
  msp_mat *A;
  msp_ksp_opts o;
  int setup;
  int64_t n, stride;
  double *basis;            /* device: (m+1) * stride, stored unnormalised (scales in g.sc) */
  double *tmp;              /* device: W = A VV(it) before the orthogonalisation */
  mspi_gmres_dev g;         /* device-resident recurrence state and arrays */
  void *gblock;             /* the single device allocation behind g */
  mspi_gmres_state *hst;    /* pinned host mirror of *g.st */
  double *hist;             /* host copy of the residual history */
  int hist_cap, nhist;
  int its, reason;
  double rnorm;
};

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
  mspi_ctx_retain(ctx);
  msp_ksp_get_default_opts(&k->o);
  *out = k;
  return MSP_SUCCESS;
}

static void ksp_drop_graphs(msp_ksp *k) {
  for (int i = 0; i < KSP_NGRAPH; ++i) {
    mspi_graph_destroy(k->graphs[i].exec);
    memset(&k->graphs[i], 0, sizeof(k->graphs[i]));
  }
  k->gnext = 0;
}

static void ksp_free_work(msp_ksp *k) {
  ksp_drop_graphs(k);
  if (k->basis) mspi_free(k->ctx, k->basis);
  if (k->tmp) mspi_free(k->ctx, k->tmp);
  if (k->gblock) mspi_free(k->ctx, k->gblock);
  if (k->hst) mspi_host_free(k->hst);
  free(k->hist);
  k->basis = k->tmp = NULL;
  k->gblock = NULL;
  k->hst = NULL;
  k->hist = NULL;
  memset(&k->g, 0, sizeof(k->g));
  k->hist_cap = 0;
  k->setup = 0;
}

int msp_ksp_destroy(msp_ksp **pk) {
  if (!pk || !*pk) return MSP_SUCCESS;
  msp_ctx *c = (*pk)->ctx;
  msp_ctx_synchronize(c);
  ksp_free_work(*pk);
  free(*pk);
  *pk = NULL;
  mspi_ctx_release(c);
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
  ksp_drop_graphs(k); /* even for the same handle: a new matrix can reuse a destroyed one's address */
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
  if (k->setup && (o->restart != k->o.restart || o->max_it + 2 > k->hist_cap)) ksp_free_work(k);
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
  const int64_t m = k->o.restart;
  /* a cycle runs K <= min(restart, max_it) steps and touches VV(0..K): with max_it < restart (the campaign's
   * inner solves, max_it 20 under GMRES(30)) only max_it + 1 basis vectors are ever used -- 11 of 32 GB less
   * per configs[3] block.  A larger max_it frees the work (hist_cap, msp_ksp_set_opts). */
  const int64_t mv = (k->o.max_it < m ? k->o.max_it : m) + 1;
  int64_t skew = 0; /* an extra skew between basis vectors measured no gain (profiles/r01/skew_ab) */
  const char *env = getenv("MSPLIT_BASIS_SKEW");
  if (env) skew = (atoll(env) + 511) / 512 * 512;
  k->stride = (k->n + 511) / 512 * 512 + skew;
  k->hist_cap = k->o.max_it + 2;
  /* one device block for the recurrence: state, then hh, cc, ss, grs, h, sc, hist */
  const size_t nd = (size_t)((m + 2) * (m + 1) + 5 * (m + 2) + k->hist_cap);
  const size_t st_bytes = (sizeof(mspi_gmres_state) + 63) / 64 * 64;
  int rc = mspi_malloc(k->ctx, (void **)&k->basis, (size_t)mv * (size_t)k->stride * sizeof(double) + 4096);
  /* W (k->tmp) is allocated by the first cycle that stores it (ensure_w): the W-free step never does */
  if (!rc) rc = mspi_malloc(k->ctx, &k->gblock, st_bytes + nd * sizeof(double));
  if (!rc) rc = mspi_host_malloc((void **)&k->hst, sizeof(mspi_gmres_state));
  k->hist = (double *)calloc((size_t)k->hist_cap, sizeof(double));
  if (!rc && !k->hist) {
    mspi_set_error(MSP_ERR_MEM, "host allocation failed");
    rc = MSP_ERR_MEM;
  }
  if (rc) {
    ksp_free_work(k);
    return rc;
  }
  double *d = (double *)((char *)k->gblock + st_bytes);
  k->g.st = (mspi_gmres_state *)k->gblock;
  k->g.hh = d;
  d += (m + 2) * (m + 1);
  k->g.cc = d;
  d += m + 2;
  k->g.ss = d;
  d += m + 2;
  k->g.grs = d;
  d += m + 2;
  k->g.h = d;
  d += m + 2;
  k->g.sc = d;
  d += m + 2;
  k->g.hist = d;
  k->setup = 1;
  return MSP_SUCCESS;
}

static double *VV(const msp_ksp *k, int j) { return k->basis + (int64_t)j * k->stride; }

/* Which Arnoldi step a cycle runs: the operator computed inside MDot and MAXPY (opfuse), the W-free step on a box
 * stencil (wfree), or W stored between the MatMult and the CGS kernels (neither).  The W-free choice follows the
 * operator and msk_set_gm_wfree, so it is asked again before every solve. */
static void step_kind(const msp_ksp *k, int *opfuse, int *wfree) {
  *opfuse = mspi_op_fusable(k->A) && k->o.restart + 1 <= MSPI_MAX_GROUP;
  *wfree = !*opfuse && k->o.restart <= MSPI_MAX_GROUP && mspi_gm_wfree(k->A);
}

/* The stored-W step's n-vector, allocated the first time a cycle takes that step (before any graph capture: no
 * allocation inside a captured cycle) -- 134-537 MB per block that the default W-free step never touches. */
static int ensure_w(msp_ksp *k) {
  int opfuse, wfree;
  step_kind(k, &opfuse, &wfree);
  if (opfuse || wfree || k->tmp) return MSP_SUCCESS;
  return mspi_malloc(k->ctx, (void **)&k->tmp, (size_t)k->stride * sizeof(double) + 4096);
}

/* One KSPGMRESCycle from its initial residual in VV(0): VecNormalize (deferred),
 * up to K Arnoldi steps, BuildSoln(it-1) into x.  Enqueued, no host synchronisation. */
static int enqueue_cycle(msp_ksp *k, double *x, int K) {
  msp_ctx *c = k->ctx;
  const int *stop = &k->g.st->stop;
  const double *sc = k->g.sc;
  double *sumsq = &k->g.h[0];
  int rc = mspi_norm2sq(c, VV(k, 0), k->n, sumsq);
  if (!rc) rc = mspi_gm_cycle_start(c, k->g, sumsq);
  int opfuse, wfree;
  step_kind(k, &opfuse, &wfree);
  for (int it = 0; it < K && !rc && opfuse; ++it) {
    /* W = A (sc[it] VV(it)) never reaches HBM: MDot and MAXPY each compute their rows of it from the operator's
     * one-byte codes and VV(it) (which both stream anyway), bitwise the separate MatMult's W */
    rc = mspi_mdot_op(k->A, VV(k, it), sc + it, it + 1, k->basis, k->stride, sc, k->g.h, stop);
    if (!rc)
      rc = mspi_maxpy_norm_update_op(k->A, VV(k, it), sc + it, VV(k, it + 1), it + 1, k->basis, k->stride, sc, k->g,
                                     k->o.restart, stop);
  }
  /* box stencils: W is not stored; the MAXPY recomputes its rows from VV(it) (which it streams anyway) */
  for (int it = 0; it < K && !rc && wfree; ++it) {
    rc = mspi_spmv_mdot(k->A, VV(k, it), sc + it, NULL, it + 1, k->basis, k->stride, sc, k->g.h, stop);
    if (!rc)
      rc = mspi_maxpy_norm_update_march(k->A, VV(k, it), sc + it, VV(k, it + 1), it + 1, k->basis, k->stride, sc,
                                        k->g, k->o.restart, stop);
  }
  for (int it = 0; it < K && !rc && !opfuse && !wfree; ++it) {
    /* W = A (sc[it] VV(it))  (KSP_PCApplyBAorAB with PCNONE on the normalised VV(it)),
     * CGS: h = VecMDot(W, VV(0..it)) -- one fused launch where the operator allows */
    rc = mspi_spmv_mdot(k->A, VV(k, it), sc + it, k->tmp, it + 1, k->basis, k->stride, sc, k->g.h, stop);
    if (rc == MSP_ERR_SUP) {
      rc = mspi_spmv_scaled(k->A, VV(k, it), sc + it, NULL, k->tmp, stop);
      if (!rc) rc = mspi_mdot_basis(c, k->tmp, it + 1, k->basis, k->stride, sc, k->n, k->g.h, stop);
    }
    /* then VV(it+1) = W - sum h_j VV(j); ||VV(it+1)||^2 */
    /* then h(it+1) = ||VV(it+1)||^2, sc[it+1] and the Hessenberg column update */
    if (!rc)
      rc = mspi_maxpy_norm_update(c, k->tmp, VV(k, it + 1), it + 1, k->basis, k->stride, sc, k->n, k->g, it,
                                  k->o.restart, stop);
  }
  /* KSPGMRESBuildSoln: back-solve (one lane, H staged in LDS), then x += sum nrs_j VV(j) */
  if (!rc) rc = mspi_gm_build(c, k->g, (int)k->o.restart);
  if (!rc) rc = mspi_maxpy_accum_basis(c, x, &k->g.st->nbuild, k->basis, k->stride, sc, k->n, k->g.grs, K);
  return rc;
}

/* A cycle from the graph cache: captured the first time its key is seen, then
 * replayed with one hipGraphLaunch (the host enqueues ~5 launches per Arnoldi
 * step otherwise, which small systems feel).  Same kernels, same arguments,
 * same order: results are those of the eager enqueue. */
static int run_cycle(msp_ksp *k, double *x, int K) {
  msp_ctx *c = k->ctx;
  if (k->graphs_off || !mspi_graphs_enabled(c)) return enqueue_cycle(k, x, K);
  int rc = mspi_reserve_partial(c, k->n); /* before the lookup: it may reallocate (a new epoch) */
  if (rc) return rc;
  const uint64_t aver = mspi_mat_version(k->A), epoch = mspi_ctx_epoch(c);
  const int tuning = msk_get_tuning(), shape = msk_get_shape_epoch();
  for (int i = 0; i < KSP_NGRAPH; ++i) {
    const ksp_graph *g = &k->graphs[i];
    if (g->exec && g->A == k->A && g->aver == aver && g->epoch == epoch && g->x == x && g->K == K &&
        g->tuning == tuning && g->shape == shape)
      return mspi_graph_launch(c, g->exec);
  }
  if (mspi_capture_begin(c)) { /* stream cannot be captured: run it eagerly */
    k->graphs_off = 1;
    return enqueue_cycle(k, x, K);
  }
  rc = enqueue_cycle(k, x, K);
  void *exec = NULL;
  const int rc2 = mspi_capture_end(c, rc == 0, &exec);
  if (rc) return rc;
  if (rc2 || !exec) { /* nothing ran: the capture only recorded the cycle */
    k->graphs_off = 1;
    return enqueue_cycle(k, x, K);
  }
  ksp_graph *g = &k->graphs[k->gnext];
  k->gnext = (k->gnext + 1) % KSP_NGRAPH;
  mspi_graph_destroy(g->exec);
  g->exec = exec;
  g->A = k->A;
  g->aver = aver;
  g->epoch = epoch;
  g->x = x;
  g->K = K;
  g->tuning = tuning;
  g->shape = shape;
  return mspi_graph_launch(c, exec);
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
  if (!rc) rc = ensure_w(k);
  if (rc) return rc;
  msp_ctx *c = k->ctx;
  const int guess_zero = !k->o.guess_nonzero;

  /* KSPSolve_GMRES state, initialised on the host and pushed once */
  mspi_gmres_state *h = k->hst;
  memset(h, 0, sizeof(*h));
  h->rnorm = -1.0; /* special marker for KSPGMRESCycle() */
  h->guess_zero = guess_zero;
  h->m = k->o.restart;
  h->max_it = k->o.max_it;
  h->uirnorm = k->o.uirnorm;
  h->hist_cap = k->hist_cap;
  h->rtol = k->o.rtol;
  h->abstol = k->o.abstol;
  h->divtol = k->o.divtol;
  h->haptol = k->o.haptol;
  h->breakdowntol = k->o.breakdowntol;
  h->scale = 1.0;
  if (!guess_zero && !k->o.uirnorm) { /* KSPConvergedDefault at n == 0 needs ||b|| */
    double bb = 0.0;
    if ((rc = mspi_norm2sq(c, b->d, k->n, k->g.h))) return rc;
    if ((rc = mspi_d2h_sync(c, &bb, k->g.h, sizeof(double)))) return rc;
    h->bnorm = sqrt(bb);
  }
  if ((rc = mspi_h2d_async(c, k->g.st, h, sizeof(*h)))) return rc;
  if (guess_zero && (rc = mspi_set(c, x->d, k->n, 0.0))) return rc; /* KSPSolve zeroes x */

  int cycle_zero_guess = guess_zero, itcount = 0, its = 0, reason = 0;
  while (!reason) {
    /* KSPInitialResidual: VV(0) = b - A x (VecCopy + VecAXPY(-1)), or b for a zero guess */
    if (!cycle_zero_guess) rc = mspi_residual(k->A, b->d, x->d, VV(k, 0));
    else rc = mspi_copy(c, VV(k, 0), b->d, k->n);
    if (rc) return rc;
    int K = k->o.max_it - its;
    if (K > k->o.restart) K = k->o.restart;
    if (K < 0) K = 0;
    if ((rc = run_cycle(k, x->d, K))) return rc;
    if ((rc = mspi_d2h_sync(c, h, k->g.st, sizeof(*h)))) return rc; /* the one sync per cycle */
    its = h->its;
    reason = h->reason;
    itcount += h->it;
    if (itcount >= k->o.max_it) {
      if (!reason) reason = MSP_DIVERGED_ITS;
      break;
    }
    cycle_zero_guess = 0;
  }
  k->its = its;
  k->reason = reason;
  k->rnorm = h->rnorm;
  k->nhist = h->nhist < k->hist_cap ? h->nhist : k->hist_cap;
  if (k->nhist && (rc = mspi_d2h_sync(c, k->hist, k->g.hist, (size_t)k->nhist * sizeof(double)))) return rc;
  return MSP_SUCCESS;
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
  *n = k->nhist;
  return MSP_SUCCESS;
}
