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
/* CGS update fused with VecNorm: w += sum_j (-h_j) V[j] (h on the device),
 * then out_dev[0] = ||w||^2 in DBR order, in one pass over the vectors. */
int mspi_maxpy_norm(msp_ctx *ctx, double *w, int nv, const double *const *V, int64_t n, const double *alpha_dev,
                    int negate, double *out_dev);
int mspi_scale(msp_ctx *ctx, double *x, int64_t n, double alpha);
int mspi_copy(msp_ctx *ctx, double *dst, const double *src, int64_t n);
int mspi_set(msp_ctx *ctx, double *x, int64_t n, double alpha);

#ifdef __cplusplus
}
#endif
#endif
