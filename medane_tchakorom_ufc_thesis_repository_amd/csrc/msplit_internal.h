/*
 * msplit_internal.h -- what the C host side (ksp_gmres.c) needs from the HIP
 * side (msplit_runtime.hip / msplit_kernels.hip).  Raw device pointers, all
 * work stream-ordered on the context's stream.
 */
#ifndef MSPLIT_INTERNAL_H
#define MSPLIT_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "msplit.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Largest number of vectors one MDot / MAXPY launch handles; more are split
 * into groups (the per-vector arithmetic does not depend on the grouping). */
#define MSPI_MAX_GROUP 32

struct msp_vec {
  msp_ctx *ctx;
  int64_t n;
  double *d;
  int owned;
};

void mspi_set_error(int code, const char *fmt, ...);

/* scratch: device doubles (>= 2*MSPI_MAX_GROUP+8) and pinned host doubles (same) */
double *mspi_dev_scratch(msp_ctx *ctx);
double *mspi_host_scratch(msp_ctx *ctx);
int mspi_malloc(msp_ctx *ctx, void **p, size_t bytes);
int mspi_free(msp_ctx *ctx, void *p);
/* pinned host memory (for per-iteration scalars) */
int mspi_host_malloc(void **p, size_t bytes);
int mspi_host_free(void *p);
int mspi_set_device(msp_ctx *ctx);
/* async device->host copy followed by a stream synchronise */
int mspi_d2h_sync(msp_ctx *ctx, void *host, const void *dev, size_t bytes);

int mspi_mat_dims(const msp_mat *A, int32_t *nrows, int32_t *ncols);
msp_ctx *mspi_mat_ctx(const msp_mat *A);

/* y = A x ; r = b - A x */
int mspi_spmv(msp_mat *A, const double *x, double *y);
int mspi_residual(msp_mat *A, const double *b, const double *x, double *r);
/* out_dev[j] = w . V[j] (DBR order), j < nv; any nv (grouped internally) */
int mspi_mdot(msp_ctx *ctx, const double *w, int nv, const double *const *V, int64_t n, double *out_dev);
/* out_dev[0] = x . x (DBR order) */
int mspi_norm2sq(msp_ctx *ctx, const double *x, int64_t n, double *out_dev);
/* w = w + sum_j a_j V[j] (PETSc 4-grouping), a_j = (negate ? -1 : 1) * alpha[j];
 * alpha is a host array (alpha_host) or a device array (alpha_dev).
 * accumulate_into_x: w_out = w + (0 + sum) instead (BuildSoln's VecSet(T,0);
 * VecMAXPY(T); VecAXPY(x,1,T) in one pass). */
int mspi_maxpy(msp_ctx *ctx, double *w, int nv, const double *const *V, int64_t n, const double *alpha_host,
               const double *alpha_dev, int negate, int accumulate_into_x);
int mspi_scale(msp_ctx *ctx, double *x, int64_t n, double alpha);
int mspi_copy(msp_ctx *ctx, double *dst, const double *src, int64_t n);
int mspi_set(msp_ctx *ctx, double *x, int64_t n, double alpha);

/* ---- device-resident KSPGMRES state (msplit_gmres.hip) ---- */
typedef struct {
  int32_t stop;        /* cycle over: later kernels of this cycle return at once */
  int32_t skip_build;  /* cycle returned before BuildSoln (PETSc's early PetscFunctionReturn) */
  int32_t it;          /* iterations done in this cycle */
  int32_t its;         /* ksp->its */
  int32_t reason;      /* KSPConvergedReason */
  int32_t nhist;       /* residual history entries written */
  int32_t nbuild;      /* vectors BuildSoln combines (it of BuildSoln + 1, or 0) */
  int32_t guess_zero;  /* the solve's original zero-guess flag (KSPConvergedDefault n == 0) */
  int32_t m, max_it, uirnorm, hist_cap;
  double res, rnorm, rnorm0, ttol, gm_rnorm0;
  double scale;        /* VecNormalize factor still to apply to the newest vector (fused into SpMV) */
  double bnorm;        /* ||b|| for the n == 0 test with a nonzero guess and no UIRNorm */
  double rtol, abstol, divtol, haptol, breakdowntol;
} mspi_gmres_state;

typedef struct {
  mspi_gmres_state *st; /* device */
  double *hh;           /* (m+2) x (m+1), HH(a,b) = hh[b*(m+2)+a] */
  double *cc, *ss, *grs; /* m+2 each */
  double *h;            /* m+2: MDot results h(0..it), then ||w||^2 at h(it+1) */
  double *hist;         /* hist_cap */
} mspi_gmres_dev;

/* one-lane kernels of the GMRES recurrence */
int mspi_gm_cycle_start(msp_ctx *ctx, mspi_gmres_dev g, const double *sumsq_dev);
int mspi_gm_iter_update(msp_ctx *ctx, mspi_gmres_dev g);
int mspi_gm_build(msp_ctx *ctx, mspi_gmres_dev g);
/* data-path pieces with a stop flag; basis = VV(j) at base + j*stride */
int mspi_spmv_scaled(msp_mat *A, const double *x, const double *sdev, double *vout, double *y, const int *stop);
int mspi_mdot_basis(msp_ctx *ctx, const double *w, int nv, const double *base, int64_t stride, int64_t n,
                    double *out_dev, const int *stop);
int mspi_maxpy_norm_basis(msp_ctx *ctx, const double *win, double *wout, int nv, const double *base, int64_t stride,
                          int64_t n, const double *alpha_dev, double *sumsq_dev, const int *stop);
int mspi_maxpy_accum_basis(msp_ctx *ctx, double *x, const int *nvdev, const double *base, int64_t stride, int64_t n,
                           const double *coef_dev, int nv_expected);
int mspi_h2d_async(msp_ctx *ctx, void *dev, const void *host, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif
