/*
 * msplit.h -- C ABI of the MI355X-native GMRES inner-solve path.
 *
 * The reference (craftman22/medane_tchakorom_ufc_thesis_repository) reaches
 * this path through PETSc 3.22.1's object API.  Every entry point below names
 * the reference call it replaces (file:line under the reference tree) and the
 * PETSc operation behind it.  Plain pointers and sizes only: no PETSc, HIP or
 * torch types cross this boundary.
 *
 * Conventions (mirroring PETSc's, src/utils/utils.c:12-17):
 *   - every function returns int: 0 (= PETSC_SUCCESS) or a PETSc error number
 *     (MSP_ERR_*); msp_get_last_error() gives the message of the calling
 *     thread's last failure;
 *   - objects are opaque handles; msp_xxx_destroy(&h) frees and NULLs h;
 *   - work is stream-ordered on the context's HIP stream; functions returning
 *     host scalars synchronise that stream;
 *   - not thread-safe per context; one host thread (or process) per GPU.
 *
 * Arithmetic (see DESIGN.md "Parity"): IEEE binary64 with no FMA contraction.
 * MatMult sums each row left to right over ascending columns (MatMult_SeqAIJ);
 * VecMAXPY uses PETSc's 4-vector grouping (VecMAXPY_Seq); VecDot/VecNorm/
 * VecMDot use the deterministic blocked reduction (DBR) order documented in
 * oracle/oracle.h, so results are bitwise reproducible run to run and equal
 * to the CPU oracle in its DBR mode.
 */
#ifndef MSPLIT_H
#define MSPLIT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error numbers: the PETSc values (petscerror.h) for the same conditions. */
#define MSP_SUCCESS 0
#define MSP_ERR_MEM 55          /* PETSC_ERR_MEM */
#define MSP_ERR_SUP 56          /* PETSC_ERR_SUP */
#define MSP_ERR_ARG_SIZ 60      /* PETSC_ERR_ARG_SIZ: incompatible sizes */
#define MSP_ERR_ARG_WRONG 62    /* PETSC_ERR_ARG_WRONG */
#define MSP_ERR_ARG_OUTOFRANGE 63
#define MSP_ERR_LIB 76          /* PETSC_ERR_LIB: HIP / RCCL runtime error */
#define MSP_ERR_ARG_NULL 85     /* PETSC_ERR_ARG_NULL */

/* KSPConvergedReason values (PETSc 3.22.1 include/petscksp.h). */
#define MSP_CONVERGED_ITERATING 0
#define MSP_CONVERGED_RTOL_NORMAL 1
#define MSP_CONVERGED_RTOL 2
#define MSP_CONVERGED_ATOL 3
#define MSP_CONVERGED_ITS 4
#define MSP_CONVERGED_ATOL_NORMAL 9
#define MSP_DIVERGED_NULL (-2)
#define MSP_DIVERGED_ITS (-3)
#define MSP_DIVERGED_DTOL (-4)
#define MSP_DIVERGED_BREAKDOWN (-5)
#define MSP_DIVERGED_NANORINF (-9)

/* Kernel classes for msp_ctx_get_kernel_stats(). */
#define MSP_KERNEL_SPMV 0       /* MatMult / MatResidual (CSR) */
#define MSP_KERNEL_MDOT 1       /* VecMDot (both DBR stages) */
#define MSP_KERNEL_MAXPY 2      /* VecMAXPY (CGS update and BuildSoln) */
#define MSP_KERNEL_NORM 3       /* VecNorm / VecDot (both DBR stages) */
#define MSP_KERNEL_SCALE 4      /* VecScale (VecNormalize) */
#define MSP_KERNEL_OTHER 5      /* copy/set/axpy/... */
#define MSP_KERNEL_SPMM 6       /* MatMatMult(AIJ, DENSE): R = A S */
#define MSP_KERNEL_DGEMV 7      /* dense MatMult (LSQR's R v - alpha u, and x = S alpha) */
#define MSP_KERNEL_DGEMVT 8     /* dense MatMultTranspose (LSQR's R^T u), both DBR stages */
#define MSP_KERNEL_SPMVDOT 9     /* GMRES MatMult fused with the VecMDot that follows (stage 1) */
#define MSP_KERNEL_NCLASSES 10

typedef struct msp_ctx msp_ctx;
typedef struct msp_mat msp_mat;
typedef struct msp_vec msp_vec;
typedef struct msp_ksp msp_ksp;
typedef struct msp_dense msp_dense;
typedef struct msp_lsqr msp_lsqr;
typedef struct msp_comm msp_comm;
typedef struct msp_amsg msp_amsg;
typedef struct msp_cvd msp_cvd;
typedef struct msp_abcast msp_abcast;

/* ---------------------------------------------------------------- context */
/* One context per GPU: device id + the HIP stream all work is ordered on.
 * stream == NULL creates a private non-blocking stream; otherwise the given
 * hipStream_t (passed as void*) is used and not destroyed.  Replaces the
 * per-rank PETSc/MPI setup: PetscInitialize + PetscSubcommCreate
 * (synchronous-multisplitting.c:40, :66-73) -- npb = 1, one block per GPU. */
int msp_ctx_create(int device, void *stream, msp_ctx **ctx);
/* msp_ctx_destroy drops the caller's reference: every object made on the context (Vec, Mat,
 * dense block, KSP, LSQR, comm, device slots) holds one of its own, so objects may be destroyed
 * before or after their context, in any order; the context is freed with the last of them. */
int msp_ctx_destroy(msp_ctx **ctx);
int msp_ctx_synchronize(msp_ctx *ctx);
int msp_get_device_count(int *count);
const char *msp_get_last_error(void);
/* SHA-256 (hex) of the library sources this build was compiled from (csrc/Makefile
 * DIGEST_SRCS): lets a host check that the loaded .so matches its source tree.
 * No reference counterpart (build identity only). */
const char *msp_build_source_digest(void);
/* Per-kernel-class HIP-event timing (used by bench.py; off by default).
 * enable = 0: off; 1: every logical kernel; N > 1: one in N of each class
 * (the event records between kernels cost ~2 % of a GMRES step when every
 * launch is bracketed; statistics then cover the sampled launches). */
int msp_ctx_set_timing(msp_ctx *ctx, int enable);
int msp_ctx_reset_kernel_stats(msp_ctx *ctx);
/* launches, summed kernel time (ms) and summed algorithmic bytes for one class;
 * synchronises the stream. */
int msp_ctx_get_kernel_stats(msp_ctx *ctx, int kernel_class, int64_t *launches, double *total_ms,
                             double *total_bytes);
/* Reduction order of every dot, norm, MDot and dense column sum on this context.
 * MSP_REDUCE_DBR (default): the deterministic blocked reduction (4096-element
 * chunks, wave butterflies; bitwise reproducible, full HBM bandwidth).
 * MSP_REDUCE_SEQ: PETSc's Seq order -- one running sum per result, elements in
 * index order (VecDot_Seq / VecNorm_Seq through f2cblaslapack ddot, VecMDot_Seq
 * per vector, MatMultTranspose_SeqDense's dgemv 'T' per column, MatNorm_SeqDense
 * NORM_FROBENIUS over the column-major array), and for an LSQR over several row
 * blocks of one process one running sum across the blocks in block order (the
 * reference's replicated R on one rank, SMSM-global.c:136).  A parity mode: one
 * lane per result, orders of magnitude slower; LSQR over more than one rank
 * returns MSP_ERR_SUP in it.  The environment variable MSPLIT_REDUCTION=seq
 * selects it at msp_ctx_create. */
#define MSP_REDUCE_DBR 0
#define MSP_REDUCE_SEQ 1
int msp_ctx_set_reduction(msp_ctx *ctx, int mode);
int msp_ctx_get_reduction(const msp_ctx *ctx, int *mode);

/* -------------------------------------------------------------------- Mat */
/* MATSEQAIJ from host CSR arrays (ascending columns per row), copied to HBM.
 * Replaces create_matrix_sparse + MatSetValue(s) + MatAssemblyBegin/End
 * (utils.c:139-155, :261-290) and MatCreateSubMatrix (utils.c:473). */
int msp_mat_create_csr(msp_ctx *ctx, int32_t nrows, int32_t ncols, const int32_t *rowptr,
                       const int32_t *col, const double *val, msp_mat **A);
/* Row-compressed AIJ: only the nlisted rows row_ids[] (ascending) hold entries;
 * every other row of the nrows x ncols matrix is empty.  This is how the
 * coupling block A_ij (utils.c:473; one boundary plane of nonzeros) is stored. */
int msp_mat_create_csr_rows(msp_ctx *ctx, int32_t nrows, int32_t ncols, int32_t nlisted,
                            const int32_t *row_ids, const int32_t *rowptr, const int32_t *col,
                            const double *val, msp_mat **A);
/* Device-side assembly of the dim-D box Laplacian with Dirichlet boundaries:
 * dim 3: nx*ny*nz 7-point (diag 6, off -1), row i + nx*j + nx*ny*k  (poisson3DMatrix,
 *        utils.c:30-121, restricted to one z-slab's own columns);
 * dim 2: nx = mesh columns (fastest), ny = mesh lines, 5-point (diag 4)
 *        (poisson2DMatrix, utils.c:247-293, restricted to whole-line row blocks).
 * Identical CSR to the host assembly, built in HBM (no host arrays). */
int msp_mat_create_box_stencil(msp_ctx *ctx, int dim, int32_t nx, int32_t ny, int32_t nz, msp_mat **A);
/* The same block rows with their coupling to the neighbour plane below (lo)
 * and/or above (hi) kept as extra columns: ncols = nrows + (lo+hi)*plane, the
 * column space being [plane below | own rows | plane above] (ascending global
 * order, so each row's sum order is MatMult_SeqAIJ's on the reference's
 * A_block_jacobi / A_block_jacobi_resdistributed rows, utils.c:30-121,
 * :247-293, :891-921).  plane = nx*ny (dim 3) or nx (dim 2).  This is the
 * operator of R = A S in the minimization variants (SMSM-global.c:326). */
/* The same operator applied without storage (MATSHELL-like): MatMult / MatResidual
 * and the GMRES SpMV compute exactly the assembled CSR's sums (ascending column
 * order, same coefficients) from the stencil, so results are bitwise those of
 * the assembled matrix while only the vectors cross HBM.  No MatMatMult /
 * get_csr (MSP_ERR_SUP).  peclet may be NULL (Poisson). */
int msp_mat_create_box_matfree(msp_ctx *ctx, int dim, int32_t nx, int32_t ny, int32_t nz, int32_t lo, int32_t hi,
                               const double *peclet, msp_mat **A);
int msp_mat_create_box_stencil_ext(msp_ctx *ctx, int dim, int32_t nx, int32_t ny, int32_t nz, int32_t lo,
                                   int32_t hi, msp_mat **A);
/* The convection-diffusion operator of BASELINE configs[4] (build-defined; the
 * reference has only Poisson): h^2 (-Lap u + beta . grad u), first-order upwind,
 * constant beta given as cell Peclet numbers peclet[d] = beta_d h / 2 (x fastest;
 * in 2D x and the line direction).  Lower neighbour in d: -1 - 2 max(P_d, 0);
 * upper: -1 + 2 min(P_d, 0); diagonal 2*dim + 2 sum |P_d| (summed x, y, z).
 * peclet = NULL or zeros gives the Poisson stencil bit for bit.  Same block /
 * column layout as msp_mat_create_box_stencil_ext. */
int msp_mat_create_box_convdiff(msp_ctx *ctx, int dim, int32_t nx, int32_t ny, int32_t nz, int32_t lo, int32_t hi,
                                const double *peclet, msp_mat **A);
int msp_mat_destroy(msp_mat **A);
int msp_mat_get_info(const msp_mat *A, int32_t *nrows, int32_t *ncols, int64_t *nnz);
/* Storage of an assembled matrix in HBM (the values and the order of every
 * product are the same in both; only the bytes a MatMult moves differ):
 *   MSP_STORAGE_CSR  rowptr int32, col int32, val f64 -- 12 bytes per entry;
 *   MSP_STORAGE_DV   one byte per entry naming a (col - row, value) pair of a
 *                    per-matrix dictionary (<= 256 pairs) and one byte per row
 *                    (its length, <= 255): ~1 byte per entry.  Every
 *                    constant-coefficient stencil fits (7 pairs in 3D).
 *   MSP_STORAGE_STENCIL  a 3D box stencil with per-row values (variable
 *                    coefficients: too many pairs for DV): one presence byte per
 *                    row and the row's seven values in per-neighbour arrays,
 *                    57 bytes per row against CSR's 88; taken when the columns of
 *                    every row are the box's neighbours {0, -+1, -+nx, -+nx*ny}
 *                    with no entry across a line or plane edge and the planes hold
 *                    whole 4096-row chunks (the z-march over chunk tiles).
 * A matrix that fits is given DV (else STENCIL) at assembly (MSPLIT_MAT_STORAGE=csr in the
 * environment keeps CSR); the CSR stays resident for the kernels that need it
 * (MatMatMult, get_csr).  This is MatSetType's choice of format inside one
 * type, like PETSc's AIJ variants, invisible to the caller.  Setting DV on a
 * matrix that does not fit: MSP_ERR_SUP.  get_storage reports
 * MSP_STORAGE_NONE for a matrix-free operator; ndict may be NULL. */
#define MSP_STORAGE_NONE (-1)
#define MSP_STORAGE_CSR 0
#define MSP_STORAGE_DV 1
#define MSP_STORAGE_STENCIL 2
int msp_mat_set_storage(msp_mat *A, int storage);
int msp_mat_get_storage(const msp_mat *A, int *storage, int *ndict);
/* The kernel family MatMult / MatResidual / the GMRES products launch for A under the current
 * storage and tuning (a static string; MatView-like information, no reference counterpart):
 * "k_spmv_lds8" / "k_spmv_csr" (CSR), "k_spmv_ell" / "k_spmv_dv" (DV storage), "k_spmv_box_march"
 * (the z-march family: k_spmv_box_march, k_spmv_box_lines, k_box_march_chunk, and in GMRES
 * k_box_spmv_mdot_march; DV storage of a box stencil -- generated, or assembled by the caller and recognised by
 * msp_mat_create_csr: a 7-point (5-point) dictionary with deltas {0, -+1, -+nx, -+nx*ny} and no
 * entry across a line or plane edge), "k_box_march_chunk_rv" (STENCIL storage; in GMRES fused with the VecMDot,
 * k_box_spmv_mdot_march with the rows' values), "k_stencil_spmv" (matrix-free), "k_spmv_rows" (row-compressed). */
int msp_mat_get_spmv_kernel(const msp_mat *A, const char **name);
/* Free the CSR arrays of a matrix in DV storage (col/val; rowptr too in the
 * ELL layout): 12 bytes per entry of HBM back, e.g. 11.7 GB per GPU for a
 * 1024^3 / 8 block.  MatMult, MatResidual, the GMRES products and, in the ELL
 * layout, MatMatMult keep working on the DV storage; msp_mat_get_csr and
 * msp_mat_set_storage(.., MSP_STORAGE_CSR) then return MSP_ERR_SUP.
 * MSP_ERR_SUP on a matrix not in DV storage. */
int msp_mat_release_csr(msp_mat *A);
/* Download the CSR (host buffers of nrows+1 / nnz entries); synchronising. */
int msp_mat_get_csr(const msp_mat *A, int32_t *rowptr, int32_t *col, double *val);
/* MatMult y = A x (utils.c:626; KSP_PCApplyBAorAB inside KSPGMRESCycle). */
int msp_mat_mult(msp_mat *A, const msp_vec *x, msp_vec *y);
/* MatResidual r = b - A x (utils.c:549, :565, :579, :946;
 * synchronous-multisplitting.c:187). */
int msp_mat_residual(msp_mat *A, const msp_vec *b, const msp_vec *x, msp_vec *r);
/* MatResidual on a row-compressed matrix (msp_mat_create_csr_rows) over the rows it lists only:
 * r_i = b_i - (A x)_i for those rows, every other row of r left as it is.  For updateLocalRHS
 * (utils.c:943-948) when r already holds b in the unlisted rows -- there b_i - 0 = b_i, so the
 * result is msp_mat_residual's bit for bit -- without copying b into r again (16 B per row). */
int msp_mat_residual_listed(msp_mat *A, const msp_vec *b, const msp_vec *x, msp_vec *r);

/* -------------------------------------------------------------------- Vec */
/* VecCreate/VecSetSizes/VecSetType (utils.c:157-168): zero-initialised, in HBM. */
int msp_vec_create(msp_ctx *ctx, int64_t n, msp_vec **v);
/* Wrap caller-owned device memory (VecCreateSeqWithArray analogue); not freed. */
int msp_vec_create_with_array(msp_ctx *ctx, int64_t n, double *device_ptr, msp_vec **v);
int msp_vec_destroy(msp_vec **v);
int msp_vec_get_size(const msp_vec *v, int64_t *n);
/* Device pointer of the storage (VecGetArray on the device). */
int msp_vec_get_array(msp_vec *v, double **device_ptr);
/* Host <-> device copies of [off, off+n) (VecSetValues / VecGetValues;
 * the reference's VecGetArray + MPI buffers, comm.c:132-138). get synchronises. */
int msp_vec_set_values(msp_vec *v, int64_t off, int64_t n, const double *host);
int msp_vec_get_values(const msp_vec *v, int64_t off, int64_t n, double *host);
/* dst[dst_off : dst_off+n] = src[src_off : src_off+n] on the device (halo packing). */
int msp_vec_copy_range(const msp_vec *src, int64_t src_off, msp_vec *dst, int64_t dst_off, int64_t n);
int msp_vec_set(msp_vec *v, double alpha);                                  /* VecSet */
int msp_vec_copy(const msp_vec *x, msp_vec *y);                             /* VecCopy */
int msp_vec_scale(msp_vec *x, double alpha);                                /* VecScale */
int msp_vec_axpy(msp_vec *y, double alpha, const msp_vec *x);               /* VecAXPY */
int msp_vec_aypx(msp_vec *y, double beta, const msp_vec *x);                /* VecAYPX */
int msp_vec_waxpy(msp_vec *w, double alpha, const msp_vec *x, const msp_vec *y); /* VecWAXPY, utils.c:1054 */
int msp_vec_dot(const msp_vec *x, const msp_vec *y, double *val);           /* VecDot */
int msp_vec_norm(const msp_vec *x, double *val);                            /* VecNorm NORM_2, utils.c:550-604 */
int msp_vec_normalize(msp_vec *x, double *val);                             /* VecNormalize */
/* VecMDot: val[j] = x . y[j], j < nv (KSPGMRESClassicalGramSchmidtOrthogonalization). */
int msp_vec_mdot(const msp_vec *x, int nv, const msp_vec *const *y, double *val);
/* VecMAXPY: y += sum_j alpha[j] x[j] (PETSc 4-grouping order). */
int msp_vec_maxpy(msp_vec *y, int nv, const double *alpha, const msp_vec *const *x);

/* -------------------------------------------------------------------- KSP */
/* KSPGMRES options -- the PETSc options database keys they stand for. */
typedef struct msp_ksp_opts {
  int32_t restart;       /* -ksp_gmres_restart           (30)    */
  int32_t max_it;        /* -ksp_max_it                  (10000) */
  double rtol;           /* -ksp_rtol                    (1e-5)  */
  double abstol;         /* -ksp_atol                    (1e-50) */
  double divtol;         /* -ksp_divtol                  (1e4)   */
  double haptol;         /* -ksp_gmres_haptol            (1e-30) */
  double breakdowntol;   /* -ksp_gmres_breakdown_tolerance (0.1) */
  int32_t uirnorm;       /* KSPConvergedDefaultSetUIRNorm / -ksp_converged_use_initial_residual_norm */
  int32_t guess_nonzero; /* KSPSetInitialGuessNonzero */
} msp_ksp_opts;

int msp_ksp_get_default_opts(msp_ksp_opts *o);
/* KSPCreate + KSPSetType(KSPGMRES) + PCNONE, CGS with REFINE_NEVER
 * (initializeKSP, utils.c:512-541; canonical options running_bulk_test_g5k:64-70). */
int msp_ksp_create(msp_ctx *ctx, msp_ksp **ksp);
int msp_ksp_destroy(msp_ksp **ksp);
int msp_ksp_set_operators(msp_ksp *ksp, msp_mat *A);                 /* KSPSetOperators, utils.c:518 */
int msp_ksp_set_opts(msp_ksp *ksp, const msp_ksp_opts *o);            /* KSPSetFromOptions, utils.c:530 */
int msp_ksp_get_opts(const msp_ksp *ksp, msp_ksp_opts *o);
int msp_ksp_set_up(msp_ksp *ksp);                                     /* KSPSetUp: Krylov basis in HBM */
/* KSPSolve (utils.c:958, gmres_solution.c:70): x is the initial guess when
 * guess_nonzero, and the solution on return. */
int msp_ksp_solve(msp_ksp *ksp, const msp_vec *b, msp_vec *x);
int msp_ksp_get_iteration_number(const msp_ksp *ksp, int32_t *its);  /* KSPGetIterationNumber, utils.c:960 */
int msp_ksp_get_residual_norm(const msp_ksp *ksp, double *rnorm);     /* KSPGetResidualNorm */
int msp_ksp_get_converged_reason(const msp_ksp *ksp, int32_t *reason);
/* Residual history of the last solve (KSPGetResidualHistory): its+1 entries. */
int msp_ksp_get_residual_history(const msp_ksp *ksp, const double **hist, int32_t *n);

/* ------------------------------------------------------------------ dense */
/* A block of rows of a MATDENSE / MATMPIDENSE matrix, column-major in HBM with
 * leading dimension lda >= nrows (create_matrix_dense, utils.c:123-137:
 * MatCreateDense + MatZeroEntries).  The minimization variants hold S (the s
 * most recent multisplitting iterates, one per column) and R = A S this way;
 * each GPU keeps only its own rows (plus, for S, the neighbour planes R needs). */
int msp_dense_create(msp_ctx *ctx, int64_t nrows, int32_t ncols, msp_dense **A);   /* zero entries */
int msp_dense_destroy(msp_dense **A);
int msp_dense_get_info(const msp_dense *A, int64_t *nrows, int32_t *ncols, int64_t *lda);
int msp_dense_get_array(msp_dense *A, double **device_ptr);                        /* MatDenseGetArray */
int msp_dense_zero_entries(msp_dense *A);                                          /* MatZeroEntries */
/* Host <-> device copies of the whole block (host column-major, leading dim ld). */
int msp_dense_set_values(msp_dense *A, const double *host, int64_t ld);
int msp_dense_get_values(const msp_dense *A, double *host, int64_t ld);
/* A[row0 : row0+n, j] = x[xoff : xoff+n] -- MatSetValuesLocal(S, n, rows, 1, &j, x)
 * (SMSM-global.c:314-316), device to device. */
int msp_dense_set_column(msp_dense *A, int32_t j, int64_t row0, const msp_vec *x, int64_t xoff, int64_t n);
/* y[yoff : yoff+n] = A[row0 : row0+n, :] alpha -- MatMult(S, alpha, x_minimized)
 * (outer_solver_norm_equation, utils.c:1076).  Per row, columns in order, from 0
 * (reference dgemv 'N').  alpha has ncols entries. */
int msp_dense_mult(msp_dense *A, const msp_vec *alpha, int64_t row0, int64_t n, msp_vec *y, int64_t yoff);
/* out[j] = column_j . u over this block's rows (DBR order) -- the local part of
 * MatMultTranspose (KSPSolve_LSQR); out has ncols entries. */
int msp_dense_mult_transpose(msp_dense *A, const msp_vec *u, msp_vec *out);
/* The normal-equations minimization of outer_solver (src/utils/utils.c:972-996: MatTransposeMatMult(R, R,
 * R_transpose_R), MatMultTranspose(R, b), then the outer KSP on R^T R; the step the reference's profiled
 * run took, tmp/function-calling-stack:32-41).  Gc = [R^T R | R^T b] over this block's rows, an
 * s x (s+1) dense block (column s = R^T b): one HBM pass over R and b.  Each entry is a sum over the
 * rows in the context's reduction order -- DBR: entry (i, j) = VecDot(R_i, R_j) bit for bit (the DBR
 * order of msp_vec_dot), G symmetric bit for bit; SEQ: the reference BLAS dgemm 'T','N' / dgemv 'T'
 * order, one running sum per entry (at most 31 columns).  A block publishes Gc (s(s+1) doubles)
 * instead of its rows of R. */
int msp_dense_gram(const msp_dense *R, const msp_vec *b, msp_dense *Gc);
/* out = ((0 + parts[0]) + parts[1]) + ... elementwise, parts in block order (all of out's shape):
 * the block-ordered sum of the Gram parts, bitwise the same on every rank that sums the same parts. */
int msp_dense_sum(int32_t nparts, const msp_dense *const *parts, msp_dense *out);
/* A dense block over columns [col0, col0+ncols) of A, sharing its storage (MatDenseGetSubMatrix,
 * as the reference's getHalfSubMatrixFromR, utils.c:926-931, takes column ranges); destroying the
 * view frees nothing of A.  The view must not outlive A's storage. */
int msp_dense_create_view(msp_dense *A, int32_t col0, int32_t ncols, msp_dense **view);
/* R = A S -- MatMatMult(A_block_jacobi_resdistributed, S, MAT_REUSE_MATRIX, R)
 * (SMSM-global.c:325-327): A is nrows(R) x nrows(S), R and S have the same
 * column count.  Per row of A and column of S: ascending columns, from 0. */
int msp_mat_matmult_dense(msp_mat *A, const msp_dense *S, msp_dense *R);

/* ------------------------------------------------------------------- comm */
/* Cross-process reductions of the distributed minimization (one rank per GPU).
 * The reference runs the whole least-squares solve redundantly on every block
 * after swapping halves of R (comm_sync_send_and_receive_minimization,
 * comm.c:252-286: (N/2)*s doubles per block per outer iteration); here R stays
 * row-distributed and only s+1 partial sums per block cross the link per LSQR
 * step, all-gathered so that every rank adds them in block order (bitwise
 * identical on every rank and independent of the collective's algorithm).
 *   rccl: an RCCL communicator over xGMI (ncclCommInitRank with an id from
 *         msp_comm_get_unique_id, distributed by the host, e.g. MPI_Bcast);
 *   host: a host callback all-gathers pinned host buffers (MPI_Allgather,
 *         gloo, ...); the device buffers are staged through it. */
#define MSP_COMM_ID_BYTES 128
typedef int (*msp_allgather_fn)(void *user, const double *send, double *recv, int64_t count);
int msp_comm_get_unique_id(uint8_t id[MSP_COMM_ID_BYTES]);
/* *ok = 1 when librccl.so.1 loads and exports what msp_comm needs: the readiness test of the ranks that do
 * not create the id (msp_comm_get_unique_id starts RCCL's bootstrap root -- a thread and a listening socket --
 * and belongs on rank 0 only). */
int msp_comm_rccl_available(int32_t *ok);
int msp_comm_create_rccl(msp_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t id[MSP_COMM_ID_BYTES],
                         msp_comm **comm);
int msp_comm_create_host(msp_ctx *ctx, int32_t nranks, int32_t rank, msp_allgather_fn fn, void *user,
                         msp_comm **comm);
int msp_comm_destroy(msp_comm **comm);
int msp_comm_get_size(const msp_comm *comm, int32_t *nranks, int32_t *rank);
/* recv[r*count + i] = rank r's send[i]; recv has nranks*count entries. */
int msp_comm_allgather(msp_comm *comm, const msp_vec *send, msp_vec *recv, int64_t count);
/* Boundary exchange between chain neighbours (comm_sync_send_and_receive,
 * comm.c:126-141; only the planes the neighbours' coupling rows read):
 * src[lo_src:+count] -> rank-1, src[hi_src:+count] -> rank+1; from rank-1 into
 * dst[lo_dst:+count], from rank+1 into dst[hi_dst:+count].  RCCL send/recv in
 * one group on the context's stream; host transport through the all-gather. */
int msp_comm_exchange_neighbors(msp_comm *comm, const msp_vec *src, int64_t lo_src, int64_t hi_src, msp_vec *dst,
                                int64_t lo_dst, int64_t hi_dst, int64_t count);
/* out[i] = sum over ranks of in[i] in rank order (host arrays): the outer residual
 * Allreduce of synchronous-multisplitting.c:192, bitwise the same on every rank. */
int msp_comm_sum_ordered(msp_comm *comm, const double *in, double *out, int32_t n);
/* The ranks' agreement on the outer loop's control state (no reference counterpart: the reference's drivers
 * assume it, synchronous-multisplitting.c:187-206, and a disagreement there is a deadlock in the next
 * collective).  Every rank passes a token (|token| <= 2^53, e.g. outer_its * 2 + stop); all tokens are
 * gathered; *all_equal = 1 when they match.  When they do not, every rank gets MSP_ERR_ARG_WRONG and an error
 * text naming the first differing rank, so a transport fault ends the run on every rank instead of hanging it. */
int msp_comm_agree(msp_comm *comm, int64_t token, int32_t *all_equal);

/* ------------------------------------------------------------------- LSQR */
/* KSPLSQR options (the outer solver of the minimization variants,
 * running_bulk_test_g5k:247-248). */
#define MSP_LSQR_CONV_DEFAULT 0 /* -ksp_convergence_test default: KSPConvergedDefault */
#define MSP_LSQR_CONV_LSQR 1    /* KSPLSQRConvergedDefault (KSPCreate_LSQR's choice)  */
#define MSP_LSQR_CONV_SKIP 2    /* -ksp_convergence_test skip                         */
typedef struct msp_lsqr_opts {
  int32_t max_it;       /* -ksp_max_it             (10000) */
  double rtol;          /* -ksp_rtol               (1e-5)  */
  double abstol;        /* -ksp_atol               (1e-50) */
  double divtol;        /* -ksp_divtol             (1e4)   */
  int32_t exact_norm;   /* -ksp_lsqr_exact_mat_norm         */
  int32_t conv_test;    /* MSP_LSQR_CONV_*                  */
} msp_lsqr_opts;

int msp_lsqr_get_default_opts(msp_lsqr_opts *o);
/* KSPCreate + KSPSetType(KSPLSQR) + PCNONE (initializeKSP(.., outer_ksp, NULL, ..),
 * SMSM-global.c:219). */
int msp_lsqr_create(msp_ctx *ctx, msp_lsqr **lsqr);
int msp_lsqr_destroy(msp_lsqr **lsqr);
int msp_lsqr_set_opts(msp_lsqr *lsqr, const msp_lsqr_opts *o);
int msp_lsqr_get_opts(const msp_lsqr *lsqr, msp_lsqr_opts *o);
/* KSPSetOperators(outer_ksp, R, R) (utils.c:1066): this process's row blocks of
 * R, in global block order; every rank passes the same count and column count.
 * The global operator is the blocks of rank 0, then rank 1, ... */
int msp_lsqr_set_operators(msp_lsqr *lsqr, int32_t nlocal, msp_dense *const *R);
/* Ranks that hold the other row blocks (NULL: all blocks are local). */
int msp_lsqr_set_comm(msp_lsqr *lsqr, msp_comm *comm);
/* KSPSolve(outer_ksp, b, alpha) with a zero initial guess (utils.c:1067-1068):
 * b[k] holds the rows of local block k; x (ncols entries) is replicated and
 * identical on every rank. */
int msp_lsqr_solve(msp_lsqr *lsqr, msp_vec *const *b, msp_vec *x);
int msp_lsqr_get_iteration_number(const msp_lsqr *lsqr, int32_t *its);
/* KSPGetResidualNorm(outer_ksp) (SMSM-global.c:341): LSQR's phibar. */
int msp_lsqr_get_residual_norm(const msp_lsqr *lsqr, double *rnorm);
int msp_lsqr_get_converged_reason(const msp_lsqr *lsqr, int32_t *reason);
/* KSPLSQRGetNorms: ||R^T r|| estimate and ||R||_F (exact or estimated). */
int msp_lsqr_get_norms(const msp_lsqr *lsqr, double *arnorm, double *anorm);
int msp_lsqr_get_residual_history(const msp_lsqr *lsqr, const double **hist, int32_t *n);

/* ------------------------------------------------------- async messages */
/* Newest-value message slots in POSIX shared memory between the blocks of an
 * asynchronous run on one node (one process or host thread per GPU).  They
 * replace the MPI layer of the asynchronous drivers: iterate exchange
 * (comm_async_test_and_send_prime / comm_async_probe_and_receive_prime,
 * comm.c:455-554) and the convergence-detection messages (TAG_SEND_RCV_*,
 * constants.h).  The reference drains every pending message of a kind and uses
 * the newest; a slot holds exactly that newest message (sequence-locked), so
 * a send never blocks and a receive never waits.  Iterate payloads (planes)
 * travel between chain neighbours only (|src - dst| = 1), up to data_cap
 * doubles.  Exactly one rank creates the region (owner = 1) before the others
 * open it; the owner unlinks it on destroy.  No GPU is needed except for the
 * *_vec variants. */
#define MSP_AMSG_DATA 0          /* TAG_MULTISPLITTING_DATA: (PhaseTag, iteration, plane) */
#define MSP_AMSG_PARTIAL_CV 1    /* TAG_SEND_RCV_PARTIAL_CV */
#define MSP_AMSG_VERIFICATION 2  /* TAG_SEND_RCV_VERIFICATION */
#define MSP_AMSG_RESPONSE 3      /* TAG_SEND_RCV_RESPONSE */
#define MSP_AMSG_VERDICT 4       /* TAG_SEND_RCV_VERDICT */
#define MSP_AMSG_NKINDS 5
int msp_amsg_create(const char *name, int32_t nranks, int32_t rank, int64_t data_cap, int32_t owner, msp_amsg **am);
int msp_amsg_destroy(msp_amsg **am);
/* number of ranks that have opened the region (for a start-up barrier) */
int msp_amsg_attached(const msp_amsg *am, int32_t *n);
/* up to 6 ints (tags) and, for MSP_AMSG_DATA, n doubles of payload */
int msp_amsg_send(msp_amsg *am, int32_t dst, int32_t kind, const int32_t *ints, int32_t nints, const double *data,
                  int64_t n);
/* got = 1 when a message newer than the last one taken from src arrived; it is copied out */
int msp_amsg_recv(msp_amsg *am, int32_t src, int32_t kind, int32_t *ints, int32_t nints, double *data, int64_t cap,
                  int64_t *n, int32_t *got);
/* the same for a plane v[off : off+n] in HBM (DMA to / from the registered region) */
int msp_amsg_send_vec(msp_amsg *am, int32_t dst, const int32_t *ints, int32_t nints, const msp_vec *v, int64_t off,
                      int64_t n);
int msp_amsg_recv_vec(msp_amsg *am, int32_t src, int32_t *ints, int32_t nints, msp_vec *v, int64_t off, int64_t cap,
                      int64_t *n, int32_t *got);
/* Device slots (the xGMI mailboxes of SURVEY.md section 8e): this rank's
 * outgoing planes live in its own HBM (two buffers per neighbour), exported by
 * HIP IPC; *_vec then move a plane HBM -> sender's slot and sender's slot ->
 * receiver's HBM (peer copy over xGMI), both enqueued on the context's stream
 * with no host wait: the stream itself publishes the plane (and releases the
 * buffer a receiver copied) once its copy is done.  A send whose previous copy
 * is not yet published, or whose free buffer the receiver still reads, is
 * skipped, as comm_async_test_and_send_prime posts a new MPI_Isend only when
 * MPI_Test reports the previous one done (comm.c:528-535).  Every rank enables
 * before the first send; close_peers (every rank; it drains the stream) must
 * precede destroy (which frees the slots).  get_stats: sends posted / skipped. */
int msp_amsg_enable_device(msp_amsg *am, msp_ctx *ctx);
int msp_amsg_close_peers(msp_amsg *am);
int msp_amsg_get_stats(const msp_amsg *am, int64_t *sent, int64_t *skipped);
/* End of run, after the detection finished and before close_peers (every rank):
 * comm_discard_pending_messages (comm.c:426-453) and the MPI_Cancel of the sends
 * still pending (asynchronous-multisplitting-asynchronous-minimization-global_prime.c:
 * 522-572).  Every message newer than the last one taken -- any source, any
 * kind -- is marked taken unread (discarded); this rank's device sends whose
 * copy is enqueued but not yet published (in_flight) cannot be withdrawn, a
 * DMA, so they are counted and completed by draining the stream. */
int msp_amsg_discard_pending(msp_amsg *am, int64_t *discarded, int64_t *in_flight);
/* diagnostics: the link src -> this rank as this rank sees it: data pub, data claim, data seen, partial-CV seq,
 * partial-CV seen, verdict seq, src's device slots opened, ranks attached (up to n of these 8) */
int msp_amsg_get_link_info(const msp_amsg *am, int32_t src, int64_t *info, int32_t n);

/* ------------------------------------------- async minimization broadcast */
/* Newest-value broadcast of each block's rows of R (AMAM-global), in POSIX
 * shared memory.  Replaces comm_async_test_and_send_min and
 * comm_async_probe_and_receive_min (comm.c:288-351; used at
 * asynchronous-multisplitting-asynchronous-minimization-global_prime.c:422-428):
 * publish sends this rank's nrows x ncols block unless the buffer it would fill
 * is still being read (the reference's "previous MPI_Isend not complete":
 * published = 0); fetch copies source src's newest block if it is newer than
 * the last one taken (got = 1), else leaves the destination as it was.  Two
 * buffers per source, a reader/writer word per buffer: no torn copies.
 * cap = the largest nrows x ncols any rank publishes.  One rank creates the
 * region (owner = 1) before the others open it. */
int msp_abcast_create(const char *name, int32_t nranks, int32_t rank, int64_t cap, int32_t owner, msp_abcast **bc);
int msp_abcast_destroy(msp_abcast **bc);
/* host payloads: column j at data + j*ld */
int msp_abcast_publish(msp_abcast *bc, const double *data, int64_t nrows, int32_t ncols, int64_t ld,
                       int32_t *published);
int msp_abcast_fetch(msp_abcast *bc, int32_t src, double *data, int64_t nrows, int32_t ncols, int64_t ld,
                     int32_t *got);
/* a dense block in HBM (DMA to / from the registered region) */
int msp_abcast_publish_dense(msp_abcast *bc, const msp_dense *D, int32_t *published);
int msp_abcast_fetch_dense(msp_abcast *bc, int32_t src, msp_dense *D, int32_t *got);
/* device buffers: the published blocks stay in the sender's HBM (HIP IPC), a fetch
 * is a peer copy over xGMI; enable on every rank before the first publish,
 * close_peers on every rank before destroy.  Neither end waits on the host: a
 * publish enqueues its copy and the stream publishes the block behind it; a
 * fetch enqueues the peer copy into D and the stream releases the source's
 * buffer behind it (D is ready in stream order).  A publish whose previous copy
 * is still unpublished, or whose buffer a reader still holds, is skipped
 * (published = 0).  nbuf = 2 (a publish fills the buffer readers are not using)
 * or 1 (half the HBM: readers skip a block being rewritten); 0 chooses: 2 while
 * a quarter of the GPU's HBM stays free after them, else 1.  At most 512 ranks.
 * msp_abcast_get_nbuf reports the count in use (0 before enable_device);
 * msp_abcast_get_stats the device publishes enqueued and skipped. */
int msp_abcast_enable_device(msp_abcast *bc, msp_ctx *ctx, int32_t nbuf);
int msp_abcast_get_nbuf(const msp_abcast *bc, int32_t *nbuf);
int msp_abcast_get_stats(const msp_abcast *bc, int64_t *sent, int64_t *skipped);
int msp_abcast_close_peers(msp_abcast *bc);
/* the same for the R rows (send_minimization_data_request, comm.c:288-351): every
 * source's block newer than the last one fetched is marked taken unread; this
 * rank's unpublished device publish is counted and completed */
int msp_abcast_discard_pending(msp_abcast *bc, int64_t *discarded, int64_t *in_flight);

/* ------------------------------------------------- convergence detection */
/* Algorithm 5.15 of Bahi/Contassot-Vivier/Couturier as the reference implements
 * it (src/utils/conv_detection_prime.c), one instance per block root, over the
 * amsg slots.  nb[]: spanning-tree neighbours (the reference's 2-block tree,
 * generalised to the chain of blocks); dep[]: the blocks whose iterates this
 * block reads.  strict = 0 reproduces the reference exactly (see conv_detect.c);
 * 1 also lets UnderThreshold veto during verification. */
#define MSP_CVD_NORMAL 0             /* State, constants.h */
#define MSP_CVD_WAIT4VERIFICATION 1
#define MSP_CVD_VERIFICATION 2
#define MSP_CVD_FINISHED 3
int msp_cvd_create(msp_amsg *am, int32_t rank, int32_t nnb, const int32_t *nb, int32_t ndep, const int32_t *dep,
                   int32_t strict, msp_cvd **cvd);
int msp_cvd_destroy(msp_cvd **cvd);
/* receive_data_dependency (conv_detection_prime.c:600-632): accept = 1 to take
 * an iterate of dependency index d stamped (src_tag, src_iter). */
int msp_cvd_data_received(msp_cvd *cvd, int32_t d, int32_t src_tag, int32_t src_iter, int32_t *accept);
/* one pass of comm_async_convDetection_prime + receive_partial_CV/verification/
 * response/verdict (asynchronous-multisplitting_prime.c:368-372) */
int msp_cvd_step(msp_cvd *cvd, int32_t under_threshold);
int msp_cvd_get_state(const msp_cvd *cvd, int32_t *state, int32_t *phase_tag);
/* state, phase_tag, elected, local_cv, pp_begin, pp_end, nb_not_recvd, partial_cv_sent */
int msp_cvd_get_info(const msp_cvd *cvd, int32_t *info, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
