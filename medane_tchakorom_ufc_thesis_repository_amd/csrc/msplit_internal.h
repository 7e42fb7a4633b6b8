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
/* hipMalloc of a large buffer, physically contiguous from 64 MiB where the driver can (MSPLIT_ALLOC_CONTIGUOUS=0: plain) */
int mspi_big_alloc(void **p, size_t bytes); /* 0 = hipSuccess */
int mspi_free(msp_ctx *ctx, void *p);
/* pinned host memory (for per-iteration scalars) */
int mspi_host_malloc(void **p, size_t bytes);
int mspi_host_free(void *p);
int mspi_set_device(msp_ctx *ctx);
/* reference counting of the context by the objects made on it (msp_ctx_destroy releases the caller's) */
void mspi_ctx_retain(msp_ctx *ctx);
void mspi_ctx_release(msp_ctx *ctx);
/* async device->host copy followed by a stream synchronise */
int mspi_d2h_sync(msp_ctx *ctx, void *host, const void *dev, size_t bytes);

int mspi_mat_dims(const msp_mat *A, int32_t *nrows, int32_t *ncols);
msp_ctx *mspi_mat_ctx(const msp_mat *A);
typedef struct {
  const int32_t *rowptr, *col;
  const double *val;
  int64_t nnz;
  int compressed;
  int32_t lds_cap; /* LDS entries per 256-row block for the staged kernels (0: rows too long) */
} mspi_csr_view;
mspi_csr_view mspi_mat_csr(const msp_mat *A);
/* R = A S over DV storage (ELL layout); MSP_ERR_SUP when A is not in it */
int mspi_mat_spmm_dv(msp_mat *A, const double *S, int64_t lds, int nc, int64_t srows, double *R, int64_t ldr);

/* dense row block, column-major, lda a multiple of 512 */
struct msp_dense {
  msp_ctx *ctx;
  int64_t nrows;
  int32_t ncols;
  int64_t lda;
  double *d;
  int view; /* msp_dense_create_view: columns of another block, storage not freed */
};

/* y = A[:, 0:nc] coef (+ (*nal_dev) U when U != NULL, skipped when *nal_dev == 0); usc_dev != NULL: U is
 * stored unscaled and its value is U * (*usc_dev) (a deferred VecScale, rounded as the scale would have been);
 * sumsq_dev != NULL: also ||y||^2 (DBR; partial holds nchunks doubles). */
int mspi_dense_gemv(msp_ctx *ctx, const double *A, int64_t lda, int nc, int64_t n, const double *coef_dev,
                    const double *nal_dev, const double *U, const double *usc_dev, double *y, double *partial,
                    double *sumsq_dev, const int *stop);
/* sc_dev != NULL: w = win * (*sc_dev) first, stored to wout unless wout == NULL (deferred: the next reader
 * scales); out_dev[j] = column_j . w (DBR), j < nc.
 * partial holds nchunks*32 doubles. */
int mspi_dense_scaled_dots(msp_ctx *ctx, const double *win, double *wout, const double *sc_dev, const double *A,
                           int64_t lda, int nc, int64_t n, double *partial, double *out_dev, const int *stop);
/* one LSQR step's U1 = A coef + nal (U usc) (unscaled) with out[0] = ||U1||^2, out[1 + v] = A_v . U1 (DBR),
 * in one pass over A where it can (msplit_dense.hip); partial: nchunks * (nc + 1) doubles */
int mspi_dense_lsqr_onepass(msp_ctx *ctx, const double *A, int64_t lda, int nc, int64_t n, const double *coef_dev,
                            const double *nal_dev, const double *U, const double *usc_dev, double *y,
                            double *partial, double *out_dev, const int *stop);
/* out_dev[j] = ||column j||^2 (DBR) */
int mspi_dense_colsumsq(msp_ctx *ctx, const double *A, int64_t lda, int nc, int64_t n, double *partial,
                        double *out_dev);

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
  double scale;        /* VecNormalize factor of the newest vector (also kept in sc[it]) */
  double bnorm;        /* ||b|| for the n == 0 test with a nonzero guess and no UIRNorm */
  double rtol, abstol, divtol, haptol, breakdowntol;
} mspi_gmres_state;

typedef struct {
  mspi_gmres_state *st; /* device */
  double *hh;           /* (m+2) x (m+1), HH(a,b) = hh[b*(m+2)+a] */
  double *cc, *ss, *grs; /* m+2 each */
  double *h;            /* m+2: MDot results h(0..it), then ||w||^2 at h(it+1) */
  double *sc;           /* m+2: deferred VecNormalize, VV(j) = stored VV(j) * sc[j] */
  double *hist;         /* hist_cap */
} mspi_gmres_dev;

/* one-lane kernels of the GMRES recurrence */
int mspi_gm_cycle_start(msp_ctx *ctx, mspi_gmres_dev g, const double *sumsq_dev);
int mspi_gm_iter_update(msp_ctx *ctx, mspi_gmres_dev g);
int mspi_gm_build(msp_ctx *ctx, mspi_gmres_dev g, int m); /* m: the restart H and GRS are sized for */
/* fold the ||w||^2 partials (stage-2 DBR) and run the Hessenberg update, one launch */
int mspi_gm_norm_update(msp_ctx *ctx, mspi_gmres_dev g, const double *partial, int64_t nchunks, int m);
/* CGS VecMAXPY + ||w||^2 partials, then mspi_gm_norm_update (h(it+1) = ||w||^2) */
int mspi_maxpy_norm_update(msp_ctx *ctx, const double *win, double *wout, int nv, const double *base, int64_t stride,
                           const double *scale, int64_t n, mspi_gmres_dev g, int it, int m, const int *stop);
/* data-path pieces with a stop flag; basis = VV(j) at base + j*stride, its value
   VV(j)[i] * scale[j] when scale (device) is not NULL */
int mspi_spmv_scaled(msp_mat *A, const double *x, const double *sdev, double *vout, double *y, const int *stop);
int mspi_spmv_mdot(msp_mat *A, const double *x, const double *sdev, double *y, int nv, const double *base,
                   int64_t stride, const double *scale, double *out_dev, const int *stop);
/* the W-free step for box stencils: mspi_spmv_mdot(.., y = NULL, ..) then mspi_maxpy_norm_update_march, which
   recomputes W = A (sdev[0] x) (x = VV(it), the basis' last vector) -- bitwise the stored-W step */
int mspi_gm_wfree(const msp_mat *A);
int mspi_maxpy_norm_update_march(msp_mat *A, const double *x, const double *sdev, double *wout, int nv,
                                 const double *base, int64_t stride, const double *scale, mspi_gmres_dev g, int m,
                                 const int *stop);
int mspi_mdot_basis(msp_ctx *ctx, const double *w, int nv, const double *base, int64_t stride, const double *scale,
                    int64_t n, double *out_dev, const int *stop);
int mspi_maxpy_norm_basis(msp_ctx *ctx, const double *win, double *wout, int nv, const double *base, int64_t stride,
                          const double *scale, int64_t n, const double *alpha_dev, double *sumsq_dev, const int *stop);
int mspi_maxpy_accum_basis(msp_ctx *ctx, double *x, const int *nvdev, const double *base, int64_t stride,
                           const double *scale, int64_t n, const double *coef_dev, int nv_expected);
int mspi_h2d_async(msp_ctx *ctx, void *dev, const void *host, size_t bytes);
/* ---- the GMRES step's MatMult inside the CGS kernels (A in DV storage, 8-code ELL layout) ---- */
int mspi_op_fusable(const msp_mat *A);
/* h(0..nv-1) = (A (sdev[0] x)) . scale_j VV(j): stage 1 computes each row of A(sc x) in registers */
int mspi_mdot_op(msp_mat *A, const double *x, const double *sdev, int nv, const double *base, int64_t stride,
                 const double *scale, double *out_dev, const int *stop);
/* VV(it+1) = A (sdev[0] x) - sum_j h_j scale_j VV(j), ||VV(it+1)||^2, then the Hessenberg update */
int mspi_maxpy_norm_update_op(msp_mat *A, const double *x, const double *sdev, double *wout, int nv,
                              const double *base, int64_t stride, const double *scale, mspi_gmres_dev g, int m,
                              const int *stop);
/* ---- HIP graphs of enqueued work (a GMRES restart cycle is replayed as one graph launch) ---- */
/* 1 unless MSPLIT_GRAPHS=0 or per-kernel timing is on (its events need eager launches) */
int mspi_graphs_enabled(msp_ctx *ctx);
/* the DBR partial buffer sized for n-element work, so nothing allocates during a capture */
int mspi_reserve_partial(msp_ctx *ctx, int64_t n);
int mspi_capture_begin(msp_ctx *ctx);
/* ok = 0: the enqueue failed, end and drop the capture; *exec receives the instantiated graph otherwise */
int mspi_capture_end(msp_ctx *ctx, int ok, void **exec);
int mspi_graph_launch(msp_ctx *ctx, void *exec);
void mspi_graph_destroy(void *exec);
/* changes whenever the kernels a product of A launches change (storage switch, CSR release) */
uint64_t mspi_mat_version(const msp_mat *A);
/* changes whenever a context buffer that enqueued work points at (the DBR partials) is reallocated */
uint64_t mspi_ctx_epoch(const msp_ctx *ctx);
int msk_get_tuning(void);
/* bumped by every launch-shape override (msk_set_march_z / _lines / msk_set_spmv_group) */
int msk_get_shape_epoch(void);
int msk_get_gm_wfree(void);
int mspi_h2d_sync(msp_ctx *ctx, void *dev, const void *host, size_t bytes);
/* free and total HBM of the context's device (hipMemGetInfo) */
int mspi_mem_info(msp_ctx *ctx, size_t *free_bytes, size_t *total_bytes);
/* ---- HBM mailboxes shared between processes (msplit_ipc.hip) ---- */
#define MSPI_IPC_HANDLE_BYTES 64
int mspi_dev_alloc(msp_ctx *ctx, size_t bytes, void **p); /* zeroed */
int mspi_dev_free(void *p);
int mspi_ipc_export(void *p, uint8_t *handle);
int mspi_ipc_open(msp_ctx *ctx, const uint8_t *handle, void **p);
int mspi_ipc_close(void *p);
/* height rows of width bytes, pitched, device to device; synchronises the context's stream */
int mspi_d2d_sync(msp_ctx *ctx, void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                  size_t height);
/* page-lock a host range (shared-memory mailboxes) for DMA */
/* the asynchronous device slots (amsg.c): a copy enqueued without waiting, and a word of a registered host region
 * stored by the stream once the work before it is done (system-scope release) */
int mspi_d2d_async(msp_ctx *ctx, void *dst, const void *src, size_t bytes);
int mspi_d2d_async2d(msp_ctx *ctx, void *dst, size_t dpitch, const void *src, size_t spitch, size_t width,
                     size_t height);
int mspi_host_device_ptr(void *host, void **dev);
uint64_t mspi_stream_key(const msp_ctx *ctx);
int mspi_stream_store_u64(msp_ctx *ctx, uint64_t *dev_word, uint64_t v);
int mspi_stream_store_u32(msp_ctx *ctx, uint32_t *dev_word, uint32_t v);
int mspi_host_register(void *p, size_t bytes);
int mspi_host_unregister(void *p);

/* ---- cross-process all-gather (msplit_comm.hip); comm may be NULL (1 rank) ---- */
int mspi_comm_allgather(msp_comm *comm, const double *send_dev, double *recv_dev, int64_t count);
int mspi_comm_size(const msp_comm *comm, int32_t *nranks, int32_t *rank);

/* ---- device-resident KSPLSQR state (msplit_lsqr.hip) ---- */
typedef struct {
  int32_t stop;        /* solve over: later kernels return at once */
  int32_t reason, its, nhist;
  int32_t i;           /* loop counter of KSPSolve_LSQR */
  int32_t max_it, conv_test, exact_norm, hist_cap;
  int32_t s;           /* columns of R */
  int32_t nblk;        /* row blocks over all ranks */
  int32_t pad;
  double rnorm, rnorm0, ttol, arnorm, anorm;
  double alpha, beta, phibar, rhobar;
  double uscale;       /* VecScale factor of the newest U (1/beta, or 1 when beta == 0) */
  double nalpha;       /* -alpha of VecAXPY(U1, -alpha, U) */
  double rtol, abstol, divtol;
} mspi_lsqr_state;

typedef struct {
  mspi_lsqr_state *st;  /* device */
  double *V, *V1, *W, *X; /* s entries each (X: the solution vector) */
  double *g;            /* all-gathered block partials, nblk * m */
  double *hist;         /* hist_cap */
} mspi_lsqr_dev;

/* ---- MSP_REDUCE_SEQ (msplit_seq.hip) ---- */
int mspi_reduce_seq(const msp_ctx *ctx);
#define MSPI_SEQ_MAXSEG 16
typedef struct {
  int32_t nseg;
  const double *x[MSPI_SEQ_MAXSEG]; /* segment k: column j at x[k] + j*ldx[k] */
  int64_t ldx[MSPI_SEQ_MAXSEG];
  const double *y[MSPI_SEQ_MAXSEG]; /* the vector each column is dotted with (unused by frob) */
  int64_t n[MSPI_SEQ_MAXSEG];
} mspi_seq_segs;
/* One sequential sum per column j < ncol of column_j . y chained over the segments in order
 * (frob != 0: one sum of the squares of every column, columns outer, segments inner).  out[k*m + j]
 * of the last segment k holds the sum (frob: the last segment's column ncol-1), every other slot
 * of the first ncol columns +0.0, so a block-order sum of the slots is the chained sum. */
int mspi_seq_chain(msp_ctx *ctx, const mspi_seq_segs *sg, int ncol, int frob, double *out, int m, const int *stop);

/* one-lane kernels of the LSQR recurrence (g holds nblk values / nblk*s values) */
int mspi_ls_start(msp_ctx *ctx, mspi_lsqr_dev d);
int mspi_ls_first(msp_ctx *ctx, mspi_lsqr_dev d, const double *gfrob);
int mspi_ls_beta(msp_ctx *ctx, mspi_lsqr_dev d);
int mspi_ls_step(msp_ctx *ctx, mspi_lsqr_dev d);
int mspi_ls_onepass_step(msp_ctx *ctx, mspi_lsqr_dev d);

#ifdef __cplusplus
}
#endif
#endif
