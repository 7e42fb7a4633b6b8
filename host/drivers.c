/*
 * drivers.c -- the multisplitting drivers over the C ABI (see msplit_drivers.h).
 * Each function cites the reference lines and the Python host function it
 * mirrors; the library calls and their order are the same, so results match
 * the Python host (and through it the CPU oracle) bit for bit.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "msplit_drivers.h"

#define CK(call)                                                                     \
  do {                                                                               \
    int rc_ = (call);                                                                \
    if (rc_) {                                                                       \
      fprintf(stderr, "%s:%d %s failed (%d): %s\n", __FILE__, __LINE__, #call, rc_, \
              msp_get_last_error());                                                 \
      return rc_;                                                                    \
    }                                                                                \
  } while (0)

#define MSD_MAX_BLOCKS 64

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* ------------------------------------------------------------------ options */
struct msd_options {
  int n;
  char **key;
  char **val;
};

static int is_number(const char *s) {
  char *end = NULL;
  strtod(s, &end);
  return end && end != s && *end == '\0';
}

msd_options *msd_options_parse(int argc, char **argv) {
  msd_options *o = (msd_options *)calloc(1, sizeof(msd_options));
  o->key = (char **)calloc((size_t)argc + 1, sizeof(char *));
  o->val = (char **)calloc((size_t)argc + 1, sizeof(char *));
  for (int i = 1; i < argc; ++i) {
    const char *t = argv[i];
    if (t[0] != '-' || is_number(t)) continue; /* stray value: ignored, as PETSc warns */
    while (*t == '-') ++t;
    o->key[o->n] = strdup(t);
    if (i + 1 < argc && (argv[i + 1][0] != '-' || is_number(argv[i + 1]))) o->val[o->n] = strdup(argv[++i]);
    o->n++;
  }
  return o;
}

void msd_options_free(msd_options *o) {
  if (!o) return;
  for (int i = 0; i < o->n; ++i) {
    free(o->key[i]);
    free(o->val[i]);
  }
  free(o->key);
  free(o->val);
  free(o);
}

static int find(const msd_options *o, const char *prefix, const char *key) {
  char full[256];
  snprintf(full, sizeof(full), "%s%s", prefix ? prefix : "", key);
  for (int i = o->n - 1; i >= 0; --i) /* the last occurrence wins */
    if (!strcmp(o->key[i], full)) return i;
  return -1;
}

int msd_opt_has(const msd_options *o, const char *prefix, const char *key) { return find(o, prefix, key) >= 0; }

const char *msd_opt_str(const msd_options *o, const char *prefix, const char *key, const char *dflt) {
  const int i = find(o, prefix, key);
  return (i < 0 || !o->val[i]) ? dflt : o->val[i];
}

int64_t msd_opt_int(const msd_options *o, const char *prefix, const char *key, int64_t dflt) {
  const char *v = msd_opt_str(o, prefix, key, NULL);
  return v ? (int64_t)strtod(v, NULL) : dflt;
}

double msd_opt_real(const msd_options *o, const char *prefix, const char *key, double dflt) {
  const char *v = msd_opt_str(o, prefix, key, NULL);
  return v ? strtod(v, NULL) : dflt;
}

static int opt_bool(const msd_options *o, const char *prefix, const char *key, int dflt) {
  const int i = find(o, prefix, key);
  if (i < 0) return dflt;
  if (!o->val[i]) return 1;
  return !strcasecmp(o->val[i], "1") || !strcasecmp(o->val[i], "true") || !strcasecmp(o->val[i], "yes");
}

/* ------------------------------------------------------------------- layout */
/* utils.py block_layout: z-slabs (3D) or whole mesh lines (2D). */
int msd_layout_make(int dim, int32_t nx, int32_t ny, int32_t nz, int nb, int b, const double *peclet,
                    msd_layout *L) {
  memset(L, 0, sizeof(*L));
  if (nb < 1 || nb > MSD_MAX_BLOCKS || b < 0 || b >= nb) return MSP_ERR_ARG_OUTOFRANGE;
  L->dim = dim;
  L->nb = nb;
  L->b = b;
  L->nx = nx;
  L->ny = ny;
  L->nz = dim == 3 ? nz : 1;
  if (dim == 3) {
    if (nz % nb) return MSP_ERR_ARG_SIZ;
    L->plane = (int64_t)nx * ny;
    const int64_t ppb = nz / nb;
    L->r0 = (int64_t)b * ppb * L->plane;
    L->r1 = (int64_t)(b + 1) * ppb * L->plane;
  } else if (dim == 2) {
    const int64_t N = (int64_t)nx * ny;
    if (N % nb || (N / nb) % ny) return MSP_ERR_ARG_SIZ;
    L->plane = ny;
    L->r0 = (int64_t)b * (N / nb);
    L->r1 = (int64_t)(b + 1) * (N / nb);
  } else {
    return MSP_ERR_ARG_WRONG;
  }
  L->has_lo = b > 0;
  L->has_hi = b < nb - 1;
  L->halo_size = (L->has_lo ? L->plane : 0) + (L->has_hi ? L->plane : 0);
  const int64_t nloc = L->r1 - L->r0;
  L->box[0] = dim;
  if (dim == 3) {
    L->box[1] = nx;
    L->box[2] = ny;
    L->box[3] = (int32_t)(nloc / ((int64_t)nx * ny));
  } else {
    L->box[1] = ny;
    L->box[2] = (int32_t)(nloc / ny);
    L->box[3] = 1;
  }
  for (int d = 0; d < 3; ++d) L->peclet[d] = peclet ? peclet[d] : 0.0;
  return MSP_SUCCESS;
}

/* coupling values: the slow-direction lower / upper coefficients (utils.py convdiff_coefs) */
static void slow_coefs(const msd_layout *L, double *lo, double *hi) {
  const double p = L->dim == 3 ? L->peclet[2] : L->peclet[1];
  *lo = -1.0 - 2.0 * (p > 0.0 ? p : 0.0);
  *hi = -1.0 + 2.0 * (p < 0.0 ? p : 0.0);
}

/* -------------------------------------------------------------------- block */
typedef struct {
  msd_layout L;
  int64_t n, lo, hi; /* own rows; neighbour-plane rows of the ext column space */
  msp_mat *A, *A_off, *A_ext;
  msp_vec *halo, *b, *x, *rhs, *r, *xe, *ones, *d, *stage;
  msp_ksp *ksp;
  msp_ksp_opts ko;
  msp_dense *S, *R;
  /* asynchronous state */
  msp_amsg *am;
  msp_cvd *cvd;
  int it, inner, tag, state, steps;
  int rhs_holds_b; /* rhs = b in the rows A_off lists no entry for: later updates recompute the coupled rows only */
  double local_norm;
  /* AMAM-global: the replicated R (own rows = R), the global b, the block's own LSQR */
  msp_abcast *bc;
  msp_dense *Rrep[64];
  msp_vec *ball[64];
  msp_lsqr *lsqr;
  msp_vec *alpha;
  /* -msplit_minimization rtr (outer_solver, utils.c:972-996): Gram parts [R_j^T R_j | R_j^T b_j] (own = Gc),
   * their block-ordered sum Gsum, its R^T R view (the outer KSP's operator) and R^T b column */
  int rtr;
  msp_dense *Gc, *Gsum, *Gop;
  msp_vec *crhs;
} msd_block;

static int ksp_from_options(msp_ksp *k, const msd_options *o, const char *p, msp_ksp_opts *ko) {
  const char *kt = msd_opt_str(o, p, "ksp_type", "gmres"), *pt = msd_opt_str(o, p, "pc_type", "none");
  if (strcasecmp(kt, "gmres") || strcasecmp(pt, "none")) {
    fprintf(stderr, "-%sksp_type %s -%spc_type %s: the MI355X path is gmres with pc none\n", p, kt, p, pt);
    return MSP_ERR_SUP;
  }
  CK(msp_ksp_get_opts(k, ko));
  ko->restart = (int32_t)msd_opt_int(o, p, "ksp_gmres_restart", ko->restart);
  ko->max_it = (int32_t)msd_opt_int(o, p, "ksp_max_it", ko->max_it);
  ko->rtol = msd_opt_real(o, p, "ksp_rtol", ko->rtol);
  ko->abstol = msd_opt_real(o, p, "ksp_atol", ko->abstol);
  ko->divtol = msd_opt_real(o, p, "ksp_divtol", ko->divtol);
  ko->haptol = msd_opt_real(o, p, "ksp_gmres_haptol", ko->haptol);
  ko->breakdowntol = msd_opt_real(o, p, "ksp_gmres_breakdown_tolerance", ko->breakdowntol);
  if (opt_bool(o, p, "ksp_converged_use_initial_residual_norm", 0)) ko->uirnorm = 1;
  if (msd_opt_has(o, p, "ksp_initial_guess_nonzero")) ko->guess_nonzero = opt_bool(o, p, "ksp_initial_guess_nonzero", 0);
  CK(msp_ksp_set_opts(k, ko));
  return MSP_SUCCESS;
}

/* GpuBlock.__init__ (multisplitting.py): A_ii, A_ij, halo, b = A_block 1, the inner KSP */

/* A block's operators in DV storage (about one byte per entry) need no CSR copy:
 * free it (msp_mat_release_csr), so a 1024^3 / 8 block holds 1.1 GB per
 * operator instead of 11.7 GB. */
static int release_csr_if_dv(msp_mat *M) {
  int st = 0;
  int rc = msp_mat_get_storage(M, &st, NULL);
  if (rc || st != MSP_STORAGE_DV) return rc;
  return msp_mat_release_csr(M);
}

static int block_init(msp_ctx *ctx, const msd_problem *p, const msd_options *o, int b, msd_block *B) {
  memset(B, 0, sizeof(*B));
  CK(msd_layout_make(p->dim, p->nx, p->ny, p->nz, p->nb, b, p->peclet, &B->L));
  msd_layout *L = &B->L;
  B->n = L->r1 - L->r0;
  B->lo = L->has_lo ? L->plane : 0;
  B->hi = L->has_hi ? L->plane : 0;
  if (p->matfree) CK(msp_mat_create_box_matfree(ctx, L->box[0], L->box[1], L->box[2], L->box[3], 0, 0, L->peclet, &B->A));
  else CK(msp_mat_create_box_convdiff(ctx, L->box[0], L->box[1], L->box[2], L->box[3], 0, 0, L->peclet, &B->A));
  CK(release_csr_if_dv(B->A));
  /* coupling rows in halo numbering: row l < plane reads halo[l] (below), row l >= n-plane reads
   * halo[lo + l - (n-plane)] (above); ascending halo index = ascending global column */
  double clo, chi;
  slow_coefs(L, &clo, &chi);
  int32_t *rid = (int32_t *)malloc(sizeof(int32_t) * (size_t)(2 * L->plane + 1));
  int32_t *rp = (int32_t *)malloc(sizeof(int32_t) * (size_t)(2 * L->plane + 2));
  int32_t *cl = (int32_t *)malloc(sizeof(int32_t) * (size_t)(2 * L->plane + 1));
  double *vl = (double *)malloc(sizeof(double) * (size_t)(2 * L->plane + 1));
  if (!rid || !rp || !cl || !vl) return MSP_ERR_MEM;
  int32_t nl = 0, ne = 0;
  rp[0] = 0;
  for (int64_t l = 0; l < B->n; ++l) {
    const int dn = L->has_lo && l < L->plane, up = L->has_hi && l >= B->n - L->plane;
    if (!dn && !up) continue;
    if (dn) { cl[ne] = (int32_t)l; vl[ne++] = clo; }
    if (up) { cl[ne] = (int32_t)(B->lo + l - (B->n - L->plane)); vl[ne++] = chi; }
    rid[nl++] = (int32_t)l;
    rp[nl] = ne;
  }
  const int rc = msp_mat_create_csr_rows(ctx, (int32_t)B->n, (int32_t)L->halo_size, nl, rid, rp, cl, vl, &B->A_off);
  free(rid);
  free(rp);
  free(cl);
  free(vl);
  CK(rc);
  CK(msp_vec_create(ctx, L->halo_size, &B->halo));
  CK(msp_vec_create(ctx, L->halo_size > 0 ? L->halo_size : 1, &B->stage));
  CK(msp_vec_create(ctx, B->n, &B->b));
  CK(msp_vec_create(ctx, B->n, &B->x));
  CK(msp_vec_create(ctx, B->n, &B->rhs));
  CK(msp_vec_create(ctx, B->n, &B->r));
  CK(msp_vec_create(ctx, B->n, &B->ones));
  CK(msp_vec_create(ctx, B->n, &B->d));
  CK(msp_vec_create(ctx, B->lo + B->n + B->hi, &B->xe));
  /* computeTheRightHandSideWithInitialGuess (utils.c:623-650): b_i = A_block 1 */
  CK(msp_mat_create_box_convdiff(ctx, L->box[0], L->box[1], L->box[2], L->box[3], B->lo > 0, B->hi > 0, L->peclet,
                                 &B->A_ext));
  CK(release_csr_if_dv(B->A_ext));
  CK(msp_vec_set(B->xe, 1.0));
  CK(msp_mat_mult(B->A_ext, B->xe, B->b));
  CK(msp_vec_set(B->ones, 1.0));
  /* initializeKSP (utils.c:512-541), prefix inner{b+1}_, nonzero guess */
  char prefix[32];
  snprintf(prefix, sizeof(prefix), "inner%d_", b + 1);
  CK(msp_ksp_create(ctx, &B->ksp));
  CK(msp_ksp_set_operators(B->ksp, B->A));
  CK(ksp_from_options(B->ksp, o, prefix, &B->ko));
  return MSP_SUCCESS;
}

static void block_free(msd_block *B) {
  msp_ksp_destroy(&B->ksp);
  msp_dense_destroy(&B->S);
  msp_dense_destroy(&B->R);
  msp_mat_destroy(&B->A);
  msp_mat_destroy(&B->A_off);
  msp_mat_destroy(&B->A_ext);
  msp_vec *v[] = {B->halo, B->stage, B->b, B->x, B->rhs, B->r, B->ones, B->d, B->xe};
  for (size_t i = 0; i < sizeof(v) / sizeof(v[0]); ++i) msp_vec_destroy(&v[i]);
}

/* utils.c:943-948.  The first update writes every row; b is fixed and rhs written nowhere else, so later ones
 * recompute the coupled rows only (msp_mat_residual_listed: bitwise the full MatResidual). */
static int update_rhs(msd_block *B) {
  const int rc = B->rhs_holds_b ? msp_mat_residual_listed(B->A_off, B->b, B->halo, B->rhs)
                                 : msp_mat_residual(B->A_off, B->b, B->halo, B->rhs);
  if (!rc) B->rhs_holds_b = 1;
  return rc;
}

static int inner_solve(msd_block *B, int *its) { /* inner_solver, utils.c:950-970 */
  B->ko.uirnorm = 1;
  B->ko.guess_nonzero = 1;
  CK(msp_ksp_set_opts(B->ksp, &B->ko));
  CK(msp_ksp_solve(B->ksp, B->rhs, B->x));
  int32_t k;
  CK(msp_ksp_get_iteration_number(B->ksp, &k));
  *its = k;
  return MSP_SUCCESS;
}

static int norm_sq(const msp_vec *v, double *sq) {
  double ln;
  CK(msp_vec_norm(v, &ln));
  *sq = ln * ln;
  return MSP_SUCCESS;
}

static int local_residual_sq(msd_block *B, double *sq) { /* MatResidual(A_ii) + VecNorm */
  CK(msp_mat_residual(B->A, B->rhs, B->x, B->r));
  return norm_sq(B->r, sq);
}

static int block_residual_sq(msd_block *B, double *sq) { /* computeFinalResidualNorm, utils.c:575-595 */
  CK(msp_vec_copy_range(B->x, 0, B->xe, B->lo, B->n));
  if (B->lo) CK(msp_vec_copy_range(B->halo, 0, B->xe, 0, B->lo));
  if (B->hi) CK(msp_vec_copy_range(B->halo, B->lo, B->xe, B->lo + B->n, B->hi));
  CK(msp_mat_residual(B->A_ext, B->b, B->xe, B->r));
  return norm_sq(B->r, sq);
}

static int error_sq(msd_block *B, double *sq) { /* computeError, utils.c:1045-1059 */
  CK(msp_vec_waxpy(B->d, -1.0, B->ones, B->x));
  return norm_sq(B->d, sq);
}

/* ---------------------------------------------------------------- transport */
typedef struct {
  const msd_transport *t;
  msd_block *blk[MSD_MAX_BLOCKS];
  int nlocal;
  int fault_stop_rank; /* MSPLIT_FAULT_STOP_RANK, read once at setup (-1: none) */
} msd_run;

static int ordered_sum(msd_run *R, const double *v, double *out) { /* block order, from 0.0 */
  if (R->t->world == 1) {
    double acc = 0.0;
    for (int i = 0; i < R->nlocal; ++i) acc += v[i];
    *out = acc;
    return MSP_SUCCESS;
  }
  return msp_comm_sum_ordered(R->t->comm, v, out, 1);
}

static void barrier(msd_run *R) {
  if (R->t->world > 1 && R->t->barrier) R->t->barrier(R->t->user);
}

/* comm_sync_send_and_receive (comm.c:126-141): the neighbours' boundary planes into the halo */
static int exchange(msd_run *R) {
  if (R->t->world > 1) {
    msd_block *B = R->blk[0];
    return msp_comm_exchange_neighbors(R->t->comm, B->x, 0, B->n - B->L.plane, B->halo, 0, B->lo, B->L.plane);
  }
  for (int i = 0; i < R->nlocal; ++i) {
    msd_block *B = R->blk[i];
    if (B->L.has_lo) CK(msp_vec_copy_range(R->blk[i - 1]->x, R->blk[i - 1]->n - B->L.plane, B->halo, 0, B->L.plane));
    if (B->L.has_hi) CK(msp_vec_copy_range(R->blk[i + 1]->x, 0, B->halo, B->lo, B->L.plane));
  }
  return MSP_SUCCESS;
}

static int sum_over_blocks(msd_run *R, int (*f)(msd_block *, double *), double *out) {
  double v[MSD_MAX_BLOCKS];
  for (int i = 0; i < R->nlocal; ++i) CK(f(R->blk[i], &v[i]));
  CK(ordered_sum(R, v, out));
  *out = sqrt(*out);
  return MSP_SUCCESS;
}

/* Every rank takes the same stop decision at the same outer iteration (synchronous-multisplitting.c:187-206 assumes
 * it; a rank that stops alone leaves the others waiting in their next collective forever): one msp_comm_agree of
 * (outer_its, stop) per outer iteration, an error on every rank on a mismatch.  MSPLIT_FAULT_STOP_RANK=r flips rank
 * r's decision at the first outer iteration (the tests' fault injection; multisplitting.py agree_on_stop).  The
 * guard cannot ride on the residual sum's all-gather: the stop decision is taken from that sum's result, and a rank
 * that stopped alone would be missing from the next one.  Its price is one 8-byte all-gather per outer iteration
 * (an outer iteration is s inner GMRES solves: SMSM-global's per-GPU block, about 1 s). */
static int agree_on_stop(msd_run *R, int outer_its, int *stop) {
  if (R->fault_stop_rank == R->t->rank && outer_its == 1) *stop = !*stop;
  if (R->t->world == 1) return MSP_SUCCESS;
  int32_t ok = 0;
  const int rc = msp_comm_agree(R->t->comm, (int64_t)outer_its * 2 + (*stop ? 1 : 0), &ok);
  if (rc) fprintf(stderr, "msplit: rank %d: %s\n", R->t->rank, msp_get_last_error());
  return rc;
}

/* -msplit_dump_x <prefix>: each block's x as raw f64 to <prefix>.<block> (the tests hash it against the oracle's) */
static int dump_x(msd_run *R, const msd_options *o) {
  const char *pre = msd_opt_str(o, NULL, "msplit_dump_x", NULL);
  if (!pre) return MSP_SUCCESS;
  for (int i = 0; i < R->nlocal; ++i) {
    msd_block *B = R->blk[i];
    double *h = (double *)malloc((size_t)(B->n > 0 ? B->n : 1) * sizeof(double));
    if (!h) return MSP_ERR_MEM;
    int rc = msp_vec_get_values(B->x, 0, B->n, h);
    char path[4096];
    snprintf(path, sizeof(path), "%s.%d", pre, B->L.b);
    FILE *fp = rc ? NULL : fopen(path, "wb");
    if (!rc && (!fp || fwrite(h, sizeof(double), (size_t)B->n, fp) != (size_t)B->n)) rc = MSP_ERR_LIB;
    if (fp) fclose(fp);
    free(h);
    if (rc) return rc;
  }
  return MSP_SUCCESS;
}

static int norm0_sq(msd_block *B, double *sq) { return norm_sq(B->b, sq); }

static int setup_run(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t, msd_run *R,
                     msd_block *store) {
  memset(R, 0, sizeof(*R));
  R->t = t;
  const char *fault = getenv("MSPLIT_FAULT_STOP_RANK");
  R->fault_stop_rank = fault && *fault ? atoi(fault) : -1;
  if (t->world > 1) {
    if (p->nb != t->world) {
      fprintf(stderr, "one block per rank: %d blocks on %d ranks\n", p->nb, t->world);
      return MSP_ERR_ARG_WRONG;
    }
    R->nlocal = 1;
    R->blk[0] = &store[0];
    return block_init(ctx, p, o, t->rank, &store[0]);
  }
  if (p->nb > MSD_MAX_BLOCKS) return MSP_ERR_ARG_OUTOFRANGE;
  R->nlocal = p->nb;
  for (int b = 0; b < p->nb; ++b) {
    R->blk[b] = &store[b];
    CK(block_init(ctx, p, o, b, &store[b]));
  }
  return MSP_SUCCESS;
}

static void free_run(msd_run *R) {
  for (int i = 0; i < R->nlocal; ++i) block_free(R->blk[i]);
}

/* ------------------------------------------------------------------- SM */
/* synchronous-multisplitting.c:155-206; multisplitting.py sm_solve */
int msd_sm_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t, msd_result *res) {
  static msd_block store[MSD_MAX_BLOCKS];
  msd_run R;
  memset(res, 0, sizeof(*res));
  CK(setup_run(ctx, p, o, t, &R, store));
  CK(sum_over_blocks(&R, norm0_sq, &res->norm0));
  for (int i = 0; i < R.nlocal; ++i) {
    CK(msp_vec_set(R.blk[i]->halo, 0.0));
    CK(update_rhs(R.blk[i]));
  }
  barrier(&R);
  const double t0 = now_s();
  for (;;) {
    for (int i = 0; i < R.nlocal; ++i) {
      int its;
      CK(inner_solve(R.blk[i], &its));
    }
    CK(exchange(&R));
    double sq[MSD_MAX_BLOCKS], norm;
    for (int i = 0; i < R.nlocal; ++i) {
      CK(update_rhs(R.blk[i]));
      CK(local_residual_sq(R.blk[i], &sq[i]));
    }
    CK(ordered_sum(&R, sq, &norm));
    norm = sqrt(norm);
    if (res->outer_its < MSD_HIST_CAP) res->hist[res->outer_its] = norm;
    res->outer_its++;
    res->last_norm = norm;
    int stop = norm <= fmax(p->atol, p->rtol * res->norm0) || res->outer_its >= p->max_outer;
    CK(agree_on_stop(&R, res->outer_its, &stop));
    if (stop) break;
  }
  barrier(&R);
  res->elapsed = now_s() - t0;
  res->final_norm = res->last_norm;
  CK(sum_over_blocks(&R, error_sq, &res->error));
  CK(dump_x(&R, o));
  free_run(&R);
  return MSP_SUCCESS;
}

/* -------------------------------------------------------------- SMSM-global */
static int lsqr_from_options(msp_lsqr *l, const msd_options *o, const char *p) {
  msp_lsqr_opts lo;
  const char *kt = msd_opt_str(o, p, "ksp_type", "lsqr"), *pt = msd_opt_str(o, p, "pc_type", "none");
  if (strcasecmp(kt, "lsqr") || strcasecmp(pt, "none")) {
    fprintf(stderr, "-%sksp_type %s -%spc_type %s: the outer solver on the MI355X path is lsqr with pc none\n", p,
            kt, p, pt);
    return MSP_ERR_SUP;
  }
  CK(msp_lsqr_get_opts(l, &lo));
  lo.max_it = (int32_t)msd_opt_int(o, p, "ksp_max_it", lo.max_it);
  lo.rtol = msd_opt_real(o, p, "ksp_rtol", lo.rtol);
  lo.abstol = msd_opt_real(o, p, "ksp_atol", lo.abstol);
  lo.divtol = msd_opt_real(o, p, "ksp_divtol", lo.divtol);
  if (msd_opt_has(o, p, "ksp_lsqr_exact_mat_norm")) lo.exact_norm = opt_bool(o, p, "ksp_lsqr_exact_mat_norm", 1);
  const char *ct = msd_opt_str(o, p, "ksp_convergence_test", NULL);
  if (ct) {
    if (!strcasecmp(ct, "default")) lo.conv_test = MSP_LSQR_CONV_DEFAULT;
    else if (!strcasecmp(ct, "lsqr")) lo.conv_test = MSP_LSQR_CONV_LSQR;
    else if (!strcasecmp(ct, "skip")) lo.conv_test = MSP_LSQR_CONV_SKIP;
    else return MSP_ERR_ARG_WRONG;
  }
  CK(msp_lsqr_set_opts(l, &lo));
  return MSP_SUCCESS;
}

/* S (s latest iterates over own rows + neighbour planes), R = A_ext S, x = S alpha */
static int store_column(msd_block *B, int k) { /* MatSetValuesLocal(S, .., k, x), SMSM-global.c:314-316 */
  CK(msp_dense_set_column(B->S, k, B->lo, B->x, 0, B->n));
  if (B->lo) CK(msp_dense_set_column(B->S, k, 0, B->halo, 0, B->lo));
  if (B->hi) CK(msp_dense_set_column(B->S, k, B->lo + B->n, B->halo, B->lo, B->hi));
  return MSP_SUCCESS;
}

static int apply_alpha(msd_block *B, msp_vec *alpha) { /* x_minimized = S alpha into x_i and the planes */
  CK(msp_dense_mult(B->S, alpha, B->lo, B->n, B->x, 0));
  if (B->lo) CK(msp_dense_mult(B->S, alpha, 0, B->lo, B->halo, 0));
  if (B->hi) CK(msp_dense_mult(B->S, alpha, B->lo + B->n, B->hi, B->halo, B->lo));
  return MSP_SUCCESS;
}

/* SMSM-global.c:288-363; multisplitting.py smsm_solve + GpuMinimizer */
int msd_smsm_global_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t,
                          msd_result *res) {
  static msd_block store[MSD_MAX_BLOCKS];
  msd_run R;
  memset(res, 0, sizeof(*res));
  CK(setup_run(ctx, p, o, t, &R, store));
  msp_dense *Rs[MSD_MAX_BLOCKS];
  msp_vec *bs[MSD_MAX_BLOCKS];
  for (int i = 0; i < R.nlocal; ++i) {
    msd_block *B = R.blk[i];
    CK(msp_dense_create(ctx, B->lo + B->n + B->hi, p->s, &B->S));
    CK(msp_dense_create(ctx, B->n, p->s, &B->R));
    Rs[i] = B->R;
    bs[i] = B->b;
  }
  msp_lsqr *lsqr;
  msp_vec *alpha;
  char prefix[32];
  snprintf(prefix, sizeof(prefix), "outer%d_", R.blk[0]->L.b + 1);
  CK(msp_lsqr_create(ctx, &lsqr));
  CK(lsqr_from_options(lsqr, o, prefix));
  CK(msp_lsqr_set_operators(lsqr, R.nlocal, Rs));
  CK(msp_lsqr_set_comm(lsqr, t->world > 1 ? t->comm : NULL));
  CK(msp_vec_create(ctx, p->s, &alpha));
  CK(sum_over_blocks(&R, norm0_sq, &res->norm0));
  for (int i = 0; i < R.nlocal; ++i) CK(msp_vec_set(R.blk[i]->halo, 0.0));
  barrier(&R);
  const double t0 = now_s();
  for (;;) {
    for (int k = 0; k < p->s; ++k) {
      for (int i = 0; i < R.nlocal; ++i) CK(update_rhs(R.blk[i]));
      for (int i = 0; i < R.nlocal; ++i) {
        int its;
        CK(inner_solve(R.blk[i], &its));
      }
      CK(exchange(&R));
      for (int i = 0; i < R.nlocal; ++i) CK(store_column(R.blk[i], k));
    }
    for (int i = 0; i < R.nlocal; ++i) CK(msp_mat_matmult_dense(R.blk[i]->A_ext, R.blk[i]->S, R.blk[i]->R));
    CK(msp_lsqr_solve(lsqr, bs, alpha)); /* outer_solver_norm_equation, utils.c:1061-1078 */
    for (int i = 0; i < R.nlocal; ++i) CK(apply_alpha(R.blk[i], alpha));
    double norm;
    CK(msp_lsqr_get_residual_norm(lsqr, &norm)); /* KSPGetResidualNorm, SMSM-global.c:341 */
    if (res->outer_its < MSD_HIST_CAP) {
      int32_t lits = 0;
      CK(msp_lsqr_get_iteration_number(lsqr, &lits));
      res->hist[res->outer_its] = norm;
      res->lsqr_its[res->outer_its] = lits;
    }
    res->outer_its++;
    res->last_norm = norm;
    int stop = norm <= fmax(p->atol, p->rtol * res->norm0) || res->outer_its >= p->max_outer;
    CK(agree_on_stop(&R, res->outer_its, &stop));
    if (stop) break;
  }
  barrier(&R);
  res->elapsed = now_s() - t0;
  CK(sum_over_blocks(&R, block_residual_sq, &res->final_norm));
  CK(sum_over_blocks(&R, error_sq, &res->error));
  CK(dump_x(&R, o));
  msp_lsqr_destroy(&lsqr);
  msp_vec_destroy(&alpha);
  free_run(&R);
  return MSP_SUCCESS;
}

/* ------------------------------------------------------------------- AM */
/* asynchronous-multisplitting_prime.c:333-427; asynchronous.py am_solve (variant "am") */
static int am_receive(msd_block *B) { /* comm_async_probe_and_receive_prime */
  const msd_layout *L = &B->L;
  int d = 0;
  for (int side = 0; side < 2; ++side) {
    const int has = side == 0 ? L->has_lo : L->has_hi;
    if (!has) continue;
    const int nbr = L->b + (side == 0 ? -1 : 1);
    const int64_t hoff = side == 0 ? 0 : B->lo;
    int32_t ints[2] = {0, 0}, got = 0, accept = 0;
    int64_t n = 0;
    CK(msp_amsg_recv_vec(B->am, nbr, ints, 2, B->stage, hoff, L->plane, &n, &got));
    if (got) {
      CK(msp_cvd_data_received(B->cvd, d, ints[0], ints[1], &accept));
      if (accept) CK(msp_vec_copy_range(B->stage, hoff, B->halo, hoff, L->plane));
    }
    ++d;
  }
  return MSP_SUCCESS;
}

static int am_publish(msd_block *B, int stamp) { /* comm_async_test_and_send_prime */
  const msd_layout *L = &B->L;
  const int32_t ints[2] = {B->tag, stamp};
  if (L->has_lo) CK(msp_amsg_send_vec(B->am, L->b - 1, ints, 2, B->x, 0, L->plane));
  if (L->has_hi) CK(msp_amsg_send_vec(B->am, L->b + 1, ints, 2, B->x, B->n - L->plane, L->plane));
  return MSP_SUCCESS;
}

int msd_am_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t, msd_result *res) {
  static msd_block store[MSD_MAX_BLOCKS];
  msd_run R;
  memset(res, 0, sizeof(*res));
  CK(setup_run(ctx, p, o, t, &R, store));
  CK(sum_over_blocks(&R, norm0_sq, &res->norm0));
  /* the run's shared-memory region: named by rank 0, created by block 0's owner first */
  char name[128];
  snprintf(name, sizeof(name), "/msplit_cam_%d_%ld", (int)getpid(), (long)(now_s() * 1e6) % 1000000000L);
  if (t->world > 1 && t->bcast) t->bcast(t->user, name, (int)sizeof(name), 0);
  for (int pass = 0; pass < 2; ++pass) { /* the owner, then everyone else */
    for (int i = 0; i < R.nlocal; ++i) {
      msd_block *B = R.blk[i];
      const int owner = B->L.b == 0;
      if (owner != (pass == 0)) continue;
      CK(msp_amsg_create(name, p->nb, B->L.b, B->L.plane > 0 ? B->L.plane : 1, owner, &B->am));
      int32_t nbrs[2], nn = 0;
      if (B->L.has_lo) nbrs[nn++] = B->L.b - 1;
      if (B->L.has_hi) nbrs[nn++] = B->L.b + 1;
      CK(msp_cvd_create(B->am, B->L.b, nn, nbrs, nn, nbrs, 0, &B->cvd));
    }
    barrier(&R);
  }
  if (!p->async_host) { /* HBM slots, peer copies over xGMI */
    for (int i = 0; i < R.nlocal; ++i) CK(msp_amsg_enable_device(R.blk[i]->am, ctx));
    barrier(&R);
  }
  for (int i = 0; i < R.nlocal; ++i) {
    CK(msp_vec_set(R.blk[i]->halo, 0.0));
    CK(update_rhs(R.blk[i]));
  }
  barrier(&R);
  const double thr = fmax(p->atol, p->rtol / sqrt((double)p->nb) * res->norm0);
  const double t0 = now_s();
  int active[MSD_MAX_BLOCKS], na = R.nlocal, limited = 0;
  for (int i = 0; i < na; ++i) active[i] = i;
  while (na > 0) {
    for (int a = 0; a < na; ++a) {
      msd_block *B = R.blk[active[a]];
      int its;
      CK(am_receive(B));
      CK(update_rhs(B));
      CK(inner_solve(B, &its));
      B->inner += its;
      CK(am_publish(B, B->it));
      double sq;
      CK(local_residual_sq(B, &sq));
      B->local_norm = sqrt(sq);
      CK(msp_cvd_step(B->cvd, B->local_norm <= thr));
      B->it++;
      CK(msp_cvd_get_state(B->cvd, &B->state, &B->tag));
    }
    int keep = 0;
    for (int a = 0; a < na; ++a)
      if (R.blk[active[a]]->state != MSP_CVD_FINISHED) active[keep++] = active[a];
    na = keep;
    for (int a = 0; a < na; ++a)
      if (R.blk[active[a]]->it >= p->max_outer) limited = 1;
    if (limited) break;
  }
  barrier(&R);
  res->elapsed = now_s() - t0;
  CK(exchange(&R)); /* comm_sync_send_and_receive_final */
  CK(sum_over_blocks(&R, block_residual_sq, &res->final_norm));
  CK(sum_over_blocks(&R, error_sq, &res->error));
  res->nlocal = R.nlocal;
  for (int i = 0; i < R.nlocal; ++i) {
    res->iterations[i] = R.blk[i]->it;
    res->states[i] = R.blk[i]->state;
    res->tags[i] = R.blk[i]->tag;
  }
  res->last_norm = limited ? -1.0 : 0.0;
  barrier(&R);
  for (int i = 0; i < R.nlocal; ++i) /* drain and cancel, AM_prime.c's end of run (every rank is past its loop) */
    CK(msp_amsg_discard_pending(R.blk[i]->am, &res->discarded[i], &res->in_flight[i]));
  barrier(&R);
  for (int i = 0; i < R.nlocal; ++i) msp_amsg_close_peers(R.blk[i]->am);
  barrier(&R);
  for (int pass = 0; pass < 2; ++pass) { /* the owner unlinks the region last */
    for (int i = 0; i < R.nlocal; ++i) {
      msd_block *B = R.blk[i];
      if ((B->L.b == 0) != (pass == 1)) continue;
      msp_cvd_destroy(&B->cvd);
      msp_amsg_destroy(&B->am);
    }
    barrier(&R);
  }
  free_run(&R);
  return limited ? MSP_ERR_ARG_OUTOFRANGE : MSP_SUCCESS;
}

/* ---------------------------------------------------------- AMAM-global */
/* asynchronous-multisplitting-asynchronous-minimization-global_prime.c:238-481; asynchronous.py am_solve
 * (variant "amam_global") over multisplitting.py setup_global_async_minimization / global_async_minimize.
 * Every block holds the whole R (each block's rows as last received, zero before the first message, the
 * reference's MatZeroEntries(R)) and the global b, and solves its own LSQR over the nb row blocks in block
 * order; R rows travel newest-value through msp_abcast. */
static int amam_setup_block(msp_ctx *ctx, const msd_problem *p, const msd_options *o, msd_block *B) {
  const msd_layout *L = &B->L;
  CK(msp_dense_create(ctx, B->lo + B->n + B->hi, p->s, &B->S));
  CK(msp_dense_create(ctx, B->n, p->s, &B->R));
  char prefix[32];
  snprintf(prefix, sizeof(prefix), "outer%d_", L->b + 1);
  B->rtr = p->rtr;
  if (B->rtr) { /* no replicated R, no global b: Gram parts of s(s+1) doubles per block */
    for (int j = 0; j < p->nb; ++j) {
      CK(msp_dense_create(ctx, p->s, p->s + 1, &B->Rrep[j]));
      CK(msp_dense_zero_entries(B->Rrep[j]));
    }
    B->Gc = B->Rrep[L->b];
    CK(msp_dense_create(ctx, p->s, p->s + 1, &B->Gsum));
    CK(msp_dense_create_view(B->Gsum, 0, p->s, &B->Gop));
    double *gd;
    int64_t lda;
    CK(msp_dense_get_array(B->Gsum, &gd));
    CK(msp_dense_get_info(B->Gsum, NULL, NULL, &lda));
    CK(msp_vec_create_with_array(ctx, p->s, gd + (int64_t)p->s * lda, &B->crhs));
    CK(msp_lsqr_create(ctx, &B->lsqr));
    CK(lsqr_from_options(B->lsqr, o, prefix));
    CK(msp_lsqr_set_operators(B->lsqr, 1, &B->Gop));
    CK(msp_lsqr_set_comm(B->lsqr, NULL));
    CK(msp_vec_create(ctx, p->s, &B->alpha));
    return MSP_SUCCESS;
  }
  for (int j = 0; j < p->nb; ++j) {
    if (j == L->b) {
      B->Rrep[j] = B->R;
      B->ball[j] = B->b;
      continue;
    }
    msd_layout Lj;
    CK(msd_layout_make(p->dim, p->nx, p->ny, p->nz, p->nb, j, p->peclet, &Lj));
    const int64_t nj = Lj.r1 - Lj.r0, loj = Lj.has_lo ? Lj.plane : 0, hij = Lj.has_hi ? Lj.plane : 0;
    CK(msp_dense_create(ctx, nj, p->s, &B->Rrep[j]));
    CK(msp_dense_zero_entries(B->Rrep[j]));
    /* b_j = A_block_j 1 (utils.c:623-650) */
    msp_mat *Aj;
    msp_vec *ones, *bj;
    CK(msp_mat_create_box_convdiff(ctx, Lj.box[0], Lj.box[1], Lj.box[2], Lj.box[3], loj > 0, hij > 0, Lj.peclet,
                                   &Aj));
    CK(msp_vec_create(ctx, loj + nj + hij, &ones));
    CK(msp_vec_set(ones, 1.0));
    CK(msp_vec_create(ctx, nj, &bj));
    CK(msp_mat_mult(Aj, ones, bj));
    msp_vec_destroy(&ones);
    msp_mat_destroy(&Aj);
    B->ball[j] = bj;
  }
  CK(msp_lsqr_create(ctx, &B->lsqr));
  CK(lsqr_from_options(B->lsqr, o, prefix));
  CK(msp_lsqr_set_operators(B->lsqr, p->nb, B->Rrep));
  CK(msp_lsqr_set_comm(B->lsqr, NULL));
  CK(msp_vec_create(ctx, p->s, &B->alpha));
  return MSP_SUCCESS;
}

static void amam_free_block(msd_block *B, int nb) {
  for (int j = 0; j < nb; ++j) {
    if (j == B->L.b && !B->rtr) continue;
    msp_dense_destroy(&B->Rrep[j]);
    msp_vec_destroy(&B->ball[j]);
  }
  msp_vec_destroy(&B->crhs);
  msp_dense_destroy(&B->Gop);
  msp_dense_destroy(&B->Gsum);
  msp_lsqr_destroy(&B->lsqr);
  msp_vec_destroy(&B->alpha);
}

static int amam_minimize(msd_block *B, int nb) { /* global_async_minimize, AMAM-global_prime.c:415-440 */
  int32_t done;
  CK(msp_mat_matmult_dense(B->A_ext, B->S, B->R)); /* R_i = A_block S */
  if (B->rtr) {                                     /* outer_solver, utils.c:972-996 */
    CK(msp_dense_gram(B->R, B->b, B->Gc));          /* MatTransposeMatMult + MatMultTranspose (:978-979) */
    CK(msp_abcast_publish_dense(B->bc, B->Gc, &done));
    for (int j = 0; j < nb; ++j)
      if (j != B->L.b) CK(msp_abcast_fetch_dense(B->bc, j, B->Rrep[j], &done));
    CK(msp_dense_sum(nb, (const msp_dense *const *)B->Rrep, B->Gsum)); /* block order */
    CK(msp_lsqr_solve(B->lsqr, &B->crhs, B->alpha)); /* KSPSolve(outer_ksp, R^T b, alpha) (:982) */
    return apply_alpha(B, B->alpha);
  }
  CK(msp_abcast_publish_dense(B->bc, B->R, &done)); /* comm_async_test_and_send_min */
  for (int j = 0; j < nb; ++j)                      /* comm_async_probe_and_receive_min */
    if (j != B->L.b) CK(msp_abcast_fetch_dense(B->bc, j, B->Rrep[j], &done));
  CK(msp_lsqr_solve(B->lsqr, B->ball, B->alpha)); /* outer_solver_norm_equation, utils.c:1061-1078 */
  return apply_alpha(B, B->alpha);
}

static int amam_iterate(msd_block *B, const msd_problem *p, double thr) { /* AMAM-global_prime.c:378-447 */
  for (int k = 0; k < p->s; ++k) {
    int its;
    CK(am_receive(B));
    CK(update_rhs(B));
    CK(inner_solve(B, &its));
    B->inner += its;
    CK(am_publish(B, B->steps));
    CK(am_receive(B));
    CK(store_column(B, k));
    B->steps++;
  }
  CK(amam_minimize(B, p->nb));
  double sq;
  CK(block_residual_sq(B, &sq)); /* MatResidual(A_block, b_i, x_minimized) + VecNorm */
  B->local_norm = sqrt(sq);
  CK(msp_cvd_step(B->cvd, B->local_norm <= thr));
  B->it++;
  return msp_cvd_get_state(B->cvd, &B->state, &B->tag);
}

int msd_amam_global_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t,
                          msd_result *res) {
  static msd_block store[MSD_MAX_BLOCKS];
  msd_run R;
  memset(res, 0, sizeof(*res));
  CK(setup_run(ctx, p, o, t, &R, store));
  for (int i = 0; i < R.nlocal; ++i) CK(amam_setup_block(ctx, p, o, R.blk[i]));
  CK(sum_over_blocks(&R, norm0_sq, &res->norm0));
  /* the largest block of R any block broadcasts: block 0's replicated R (asynchronous.py) */
  int64_t cap = p->rtr ? (int64_t)p->s * (p->s + 1) : 0;
  for (int j = 0; j < p->nb && !p->rtr; ++j) {
    msd_layout Lj;
    CK(msd_layout_make(p->dim, p->nx, p->ny, p->nz, p->nb, j, p->peclet, &Lj));
    const int64_t c = (Lj.r1 - Lj.r0) * (int64_t)p->s;
    if (c > cap) cap = c;
  }
  char name[128], rname[136];
  snprintf(name, sizeof(name), "/msplit_camam_%d_%ld", (int)getpid(), (long)(now_s() * 1e6) % 1000000000L);
  if (t->world > 1 && t->bcast) t->bcast(t->user, name, (int)sizeof(name), 0);
  snprintf(rname, sizeof(rname), "%s_R", name);
  for (int pass = 0; pass < 2; ++pass) { /* the owner, then everyone else */
    for (int i = 0; i < R.nlocal; ++i) {
      msd_block *B = R.blk[i];
      const int owner = B->L.b == 0;
      if (owner != (pass == 0)) continue;
      CK(msp_amsg_create(name, p->nb, B->L.b, B->L.plane > 0 ? B->L.plane : 1, owner, &B->am));
      CK(msp_abcast_create(rname, p->nb, B->L.b, cap, owner, &B->bc));
      int32_t nbrs[2], nn = 0;
      if (B->L.has_lo) nbrs[nn++] = B->L.b - 1;
      if (B->L.has_hi) nbrs[nn++] = B->L.b + 1;
      CK(msp_cvd_create(B->am, B->L.b, nn, nbrs, nn, nbrs, 0, &B->cvd));
    }
    barrier(&R);
  }
  if (!p->async_host) { /* HBM slots and R buffers, peer copies over xGMI */
    /* MSPLIT_ABCAST_NBUF = 1 or 2 forces the R-buffer count; otherwise the library's rule (two while a quarter
     * of the HBM stays free after them) */
    const char *e = getenv("MSPLIT_ABCAST_NBUF");
    const int nbuf = e && (atoi(e) == 1 || atoi(e) == 2) ? atoi(e) : 0;
    for (int i = 0; i < R.nlocal; ++i) {
      CK(msp_amsg_enable_device(R.blk[i]->am, ctx));
      CK(msp_abcast_enable_device(R.blk[i]->bc, ctx, nbuf));
    }
    barrier(&R);
  }
  for (int i = 0; i < R.nlocal; ++i) {
    CK(msp_vec_set(R.blk[i]->halo, 0.0));
    CK(update_rhs(R.blk[i]));
  }
  barrier(&R);
  const double thr = fmax(p->atol, p->rtol / sqrt((double)p->nb) * res->norm0);
  const double t0 = now_s();
  int active[MSD_MAX_BLOCKS], na = R.nlocal, limited = 0;
  for (int i = 0; i < na; ++i) active[i] = i;
  while (na > 0) {
    for (int a = 0; a < na; ++a) CK(amam_iterate(R.blk[active[a]], p, thr)); /* round-robin */
    int keep = 0;
    for (int a = 0; a < na; ++a)
      if (R.blk[active[a]]->state != MSP_CVD_FINISHED) active[keep++] = active[a];
    na = keep;
    for (int a = 0; a < na; ++a)
      if (R.blk[active[a]]->it >= p->max_outer) limited = 1;
    if (limited) break;
  }
  barrier(&R);
  res->elapsed = now_s() - t0;
  CK(exchange(&R)); /* comm_sync_send_and_receive_final */
  CK(sum_over_blocks(&R, block_residual_sq, &res->final_norm));
  CK(sum_over_blocks(&R, error_sq, &res->error));
  res->nlocal = R.nlocal;
  for (int i = 0; i < R.nlocal; ++i) {
    res->iterations[i] = R.blk[i]->it;
    res->states[i] = R.blk[i]->state;
    res->tags[i] = R.blk[i]->tag;
  }
  res->last_norm = limited ? -1.0 : 0.0;
  barrier(&R);
  for (int i = 0; i < R.nlocal; ++i) { /* drain and cancel (AMAM-global_prime.c:522-572) */
    int64_t d, f;
    CK(msp_amsg_discard_pending(R.blk[i]->am, &res->discarded[i], &res->in_flight[i]));
    CK(msp_abcast_discard_pending(R.blk[i]->bc, &d, &f));
    res->discarded[i] += d;
    res->in_flight[i] += f;
  }
  barrier(&R);
  for (int i = 0; i < R.nlocal; ++i) {
    msp_amsg_close_peers(R.blk[i]->am);
    msp_abcast_close_peers(R.blk[i]->bc);
  }
  barrier(&R);
  for (int pass = 0; pass < 2; ++pass) { /* the owner unlinks the regions last */
    for (int i = 0; i < R.nlocal; ++i) {
      msd_block *B = R.blk[i];
      if ((B->L.b == 0) != (pass == 1)) continue;
      msp_cvd_destroy(&B->cvd);
      msp_amsg_destroy(&B->am);
      msp_abcast_destroy(&B->bc);
    }
    barrier(&R);
  }
  for (int i = 0; i < R.nlocal; ++i) amam_free_block(R.blk[i], p->nb);
  free_run(&R);
  return limited ? MSP_ERR_ARG_OUTOFRANGE : MSP_SUCCESS;
}
