/*
 * oracle.h -- CPU restatement of the reference's GMRES inner-solve path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library under
 * medane_tchakorom_ufc_thesis_repository_amd/) may link, load or call this
 * code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * use it, as the checker / the reported CPU baseline.
 *
 * What it restates (reference = /root/reference, PETSc 3.22.1 un-vendored):
 *   - stencil assembly    src/utils/utils.c:30-121   (poisson3DMatrix)
 *                         src/utils/utils.c:247-293  (poisson2DMatrix)
 *                         src/utils/utils.c:383-445  (poisson2DMatrix_complete)
 *   - block split         src/utils/utils.c:450-478  (divideSubDomainIntoBlockMatrices)
 *   - MatMult / MatResidual / VecNorm / VecMDot / VecMAXPY   [PETSc-ext, SeqAIJ/Seq kernels]
 *   - KSPSolve_GMRES / KSPGMRESCycle / CGS(REFINE_NEVER) / UpdateHessenberg /
 *     BuildSoln / KSPConvergedDefault                        [PETSc-ext]
 *   - inner_solver        src/utils/utils.c:950-970
 *   - updateLocalRHS      src/utils/utils.c:943-948
 *   - residual reduction  src/utils/utils.c:575-620
 *   - SM outer loop       src/synchronous-multisplitting/synchronous-multisplitting.c:155-206
 *   - KSPSolve_LSQR / KSPLSQRConvergedDefault (PCNONE)      [PETSc-ext]
 *   - MatMult / MatMultTranspose / MatNorm(FROBENIUS) of MATDENSE, MatMatMult(AIJ, DENSE) [PETSc-ext]
 *   - outer_solver_norm_equation src/utils/utils.c:1061-1078
 *   - SMSM-global loop    src/synchronous-multisplitting-synchronous-minimization-global/
 *                         synchronous-multisplitting-synchronous-minimization-global.c:288-363
 *
 * Parity status: the assembly and the residual-norm helper are pinned by the
 * reference's own known-answer tests (src/tests/utils_test.c:38-228).  The
 * GMRES/CGS/SpMV arithmetic lives in PETSc, which the reference does not
 * vendor and whose outputs no reference test pins: that part is
 * "parity unpinned" (restated from PETSc 3.22.1 semantics).
 *
 * Reductions come in two orders:
 *   ORC_REDUCE_SEQ  sequential left-to-right sums (PETSc Seq kernels / reference BLAS ddot,
 *                   no FMA contraction)
 *   ORC_REDUCE_DBR  the "deterministic blocked reduction" the HIP kernels use (chunked,
 *                   per-lane sequential, wave64 butterfly, fixed wave combine).  Used to
 *                   check the device bit for bit.
 */
#ifndef MSPLIT_ORACLE_H
#define MSPLIT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_REDUCE_SEQ = 0, ORC_REDUCE_DBR = 1, ORC_REDUCE_MT = 2 };
/* CPU-baseline threads (default 1): see oracle.c; ORC_REDUCE_MT = PETSc's MPI dot
 * order with one rank per thread. */
void orc_set_threads(int threads);

/* DBR geometry -- must match csrc/msplit_kernels.hip */
#define ORC_DBR_THREADS 256
#define ORC_DBR_VW 2
#define ORC_DBR_ITERS 8
#define ORC_DBR_CHUNK (ORC_DBR_THREADS * ORC_DBR_VW * ORC_DBR_ITERS)

/* KSPConvergedReason values (PETSc 3.22.1 include/petscksp.h) */
enum {
  ORC_CONVERGED_ITERATING = 0,
  ORC_CONVERGED_RTOL_NORMAL = 1,
  ORC_CONVERGED_ITS = 4,
  ORC_CONVERGED_ATOL_NORMAL = 9,
  ORC_CONVERGED_RTOL = 2,
  ORC_CONVERGED_ATOL = 3,
  ORC_CONVERGED_HAPPY_BREAKDOWN = 7,
  ORC_DIVERGED_NULL = -2,
  ORC_DIVERGED_ITS = -3,
  ORC_DIVERGED_DTOL = -4,
  ORC_DIVERGED_BREAKDOWN = -5,
  ORC_DIVERGED_NANORINF = -9
};

typedef struct {
  int32_t nrows, ncols;
  int64_t nnz;
  int32_t *rowptr; /* nrows+1 */
  int32_t *col;    /* nnz, ascending within a row (PETSc AIJ) */
  double *val;     /* nnz */
} orc_csr;

void orc_csr_free(orc_csr *A);

/* --- assembly ---------------------------------------------------------- */
/* Rows of planes [z0,z1) of the nx*ny*nz 7-point Laplacian (diag 6, off -1,
 * Dirichlet eliminated), GLOBAL column ids, local row = global row - z0*nx*ny. */
int orc_poisson3d_rows(int nx, int ny, int nz, int z0, int z1, orc_csr *A);
/* poisson2DMatrix: rows [row0,row1) of the m x n grid, i = Ii / n, diag 4. */
int orc_poisson2d_rows(int m, int n, int64_t row0, int64_t row1, orc_csr *A);
/* poisson2DMatrix_complete: full N = m*n square matrix, Ii = i*m + j. */
int orc_poisson2d_complete(int m, int n, orc_csr *A);
/* Convection-diffusion rows (BASELINE configs[4]; build-defined, the reference has only
 * Poisson): h^2(-Lap u + beta.grad u), first-order upwind, peclet[d] = beta_d h / 2, x fastest.
 * dim 3: rows of planes [z0,z1) of nx*ny*nz; dim 2: rows [row0,row1) of the m = ny... see oracle.c.
 * Lower neighbour in d: -1 - 2 max(P_d,0); upper: -1 + 2 min(P_d,0); diagonal
 * ((2 dim + 2|Px|) + 2|Py|) (+ 2|Pz|).  Global columns, ascending. */
int orc_convdiff_rows(int dim, int nx, int ny, int nz, int64_t row0, int64_t row1, const double *peclet, orc_csr *A);
/* Block split: A_ii = columns in [c0,c1) shifted by -c0; A_off = the other columns (kept global). */
int orc_split(const orc_csr *Ablock, int64_t c0, int64_t c1, orc_csr *Aii, orc_csr *Aoff);

/* --- Mat / Vec kernels --------------------------------------------------- */
void orc_spmv(const orc_csr *A, const double *x, double *y);                        /* MatMult */
void orc_residual(const orc_csr *A, const double *b, const double *x, double *r);  /* MatResidual */
double orc_dot(int mode, int64_t n, const double *x, const double *y);
double orc_norm2(int mode, int64_t n, const double *x);
void orc_mdot(int mode, int64_t n, int k, const double *w, const double *const *V, double *out);
void orc_maxpy(int64_t n, int k, const double *alpha, const double *const *V, double *w);

/* --- KSP GMRES ----------------------------------------------------------- */
typedef struct {
  int restart;        /* -ksp_gmres_restart (30) */
  int max_it;         /* -ksp_max_it (10000) */
  double rtol;        /* -ksp_rtol (1e-5) */
  double abstol;      /* -ksp_atol (1e-50) */
  double divtol;      /* -ksp_divtol (1e4) */
  double haptol;      /* -ksp_gmres_haptol (1e-30) */
  double breakdowntol;/* -ksp_gmres_breakdown_tolerance (0.1) */
  int uirnorm;        /* KSPConvergedDefaultSetUIRNorm */
  int guess_nonzero;  /* KSPSetInitialGuessNonzero */
  int reduce_mode;    /* ORC_REDUCE_* */
} orc_gmres_opts;

typedef struct {
  int its;
  int reason;
  double rnorm;
  int nhist;          /* entries written to hist (its+1 normally) */
} orc_gmres_result;

void orc_gmres_default_opts(orc_gmres_opts *o);
int orc_gmres_solve(const orc_csr *A, const double *b, double *x, const orc_gmres_opts *o,
                    orc_gmres_result *res, double *hist, int hist_cap);

/* --- reference glue ------------------------------------------------------ */
/* computeFinalResidualNorm_new (utils.c:597-620) for nb blocks held in one process:
 * sqrt( sum_b  ||b_b - A_b x||^2 ), each block's local norm squared after sqrt. */
double orc_final_residual_norm(int mode, int nb, const orc_csr *const *Ablocks, const double *x,
                               const double *const *bblocks);

/* Synchronous multisplitting (SM) generalised to nb contiguous-row blocks.
 * dim 3: (nx,ny,nz) z-slabs, nz % nb == 0.  dim 2: (m=nx, n=ny) rows, m*n % nb == 0.
 * Writes the outer residual-norm history (one per outer iteration) and the
 * per-outer, per-block inner iteration counts (outer_cap * nb ints, may be NULL). */
typedef struct {
  int dim, nx, ny, nz, nb;
  double rtol;        /* -rtol (outer) */
  double atol;        /* 1e-100 (synchronous-multisplitting.c:34) */
  int max_outer;      /* safety cap (the reference loops until convergence) */
  double peclet[3];   /* 0: the reference's Poisson operator; else orc_convdiff_rows */
} orc_sm_problem;

typedef struct {
  int outer_its;
  double norm0;       /* global_norm_0 */
  double final_norm;  /* last outer residual norm */
  double error;       /* ||x - u||_2, u = 1 */
  int64_t total_inner_its; /* sum over blocks and outer iterations */
} orc_sm_result;

int orc_sm_solve(const orc_sm_problem *p, const orc_gmres_opts *inner, orc_sm_result *res,
                 double *outer_hist, int outer_cap, int *inner_its, double *x_out);

/* --- KSP LSQR (outer least-squares solver of the minimization variants) --- */
/* The operator is a tall dense matrix R (N x s, column-major) held as nblk
 * row blocks: block b has nrows[b] rows, leading dimension lda[b] and data
 * R[b] (column j at R[b] + j*lda[b]).  The right-hand side is split the same
 * way (rhs[b]).  Reductions over the N rows:
 *   SEQ  one sequential sum over all N rows, block 0's rows first (the
 *        reference: every block holds the whole R and runs the same solve);
 *   DBR  DBR order inside each block, then the block sums added in block
 *        order from 0.0 (the device order: block-local reduction + all-gather). */
enum { ORC_LSQR_CONV_DEFAULT = 0, ORC_LSQR_CONV_LSQR = 1, ORC_LSQR_CONV_SKIP = 2 };

typedef struct {
  int max_it;         /* -ksp_max_it (10000) */
  double rtol;        /* -ksp_rtol (1e-5) */
  double abstol;      /* -ksp_atol (1e-50) */
  double divtol;      /* -ksp_divtol (1e4) */
  int exact_norm;     /* -ksp_lsqr_exact_mat_norm */
  int conv_test;      /* -ksp_convergence_test: default | lsqr (KSPCreate_LSQR's choice) | skip */
  int reduce_mode;    /* ORC_REDUCE_* */
  int onepass;        /* DBR only (default 1, the device's default): each step's R^T U1 is taken in the same pass
                       * over R as U1 = R V - alpha U, from the unscaled U1, and multiplied by 1/beta afterwards:
                       * V1_j = (sum_b dbr(R_j, U1)) * (1/beta) where PETSc's order scales U1 first,
                       * V1_j = sum_b dbr(R_j, U1 * (1/beta)).  0: PETSc's operation order (the device's
                       * MSPLIT_LSQR_ONEPASS=0).  SEQ always keeps PETSc's order. */
} orc_lsqr_opts;

typedef struct {
  int its;
  int reason;
  double rnorm;       /* ksp->rnorm = phibar (LSQR's estimate of ||b - R x||) */
  double arnorm;      /* estimate of ||R^T (b - R x)|| */
  double anorm;       /* Frobenius norm of R (exact or estimated) */
  int nhist;
} orc_lsqr_result;

void orc_lsqr_default_opts(orc_lsqr_opts *o);
/* KSPSolve(outer_ksp, b, x) with a zero initial guess; x has s entries. */
int orc_lsqr_solve(int nblk, const int64_t *nrows, int s, const double *const *R, const int64_t *lda,
                   const double *const *rhs, double *x, const orc_lsqr_opts *o, orc_lsqr_result *res,
                   double *hist, int hist_cap);
/* MatMult(S, alpha, y) of a column-major dense block: y[i] = sum_j S[i + j*lda] alpha[j]
 * (reference dgemv 'N': per row, columns in order, starting from 0). */
void orc_dense_mult(int64_t n, int s, const double *S, int64_t lda, const double *alpha, double *y);

/* outer_solver's normal equations (utils.c:972-996) over one block's rows: Gc = [R^T R | R^T b],
 * s x (s+1) column-major with leading dimension ldg.  SEQ: the SeqDense BLAS order (dgemm 'T','N',
 * dgemv 'T': one running sum per entry over the rows); DBR: each entry the device's dot order. */
void orc_dense_gram(int mode, int64_t n, int s, const double *R, int64_t lda, const double *b, double *Gc,
                    int64_t ldg);

/* --- SMSM, global minimization ------------------------------------------- */
typedef struct {
  int dim, nx, ny, nz, nb;
  int s;              /* -s: inner solves (basis vectors) per minimization */
  double rtol;        /* -rtol (outer) */
  double atol;        /* 1e-100 (SMSM-global.c:33) */
  int max_outer;      /* safety cap */
  double peclet[3];   /* as orc_sm_problem */
  int lean;           /* dim 3 only: the operators applied without storage and R = A S formed on the fly inside
                       * the LSQR (S is the only N x s array): bit for bit lean = 0, in a third of the memory --
                       * the records at 512^3 (tests/golden/make_configs2.py, make_smsm_block.py) */
} orc_smsm_problem;

typedef struct {
  int outer_its;
  double norm0;       /* global_norm_0 = ||b|| (x = 0) */
  double final_norm;  /* computeFinalResidualNorm of the last minimized iterate */
  double error;       /* ||x - u||_2 */
  int64_t total_inner_its;
} orc_smsm_result;

/* outer_hist[k]   : the outer LSQR residual norm of outer iteration k (the stop test's norm)
 * lsqr_its[k]     : its, lsqr_reason[k]: reason of that LSQR solve (may be NULL)
 * inner_its       : outer_cap * s * nb ints, [k][j][b] (may be NULL) */
int orc_smsm_solve(const orc_smsm_problem *p, const orc_gmres_opts *inner, const orc_lsqr_opts *outer,
                   orc_smsm_result *res, double *outer_hist, int outer_cap, int *lsqr_its,
                   int *lsqr_reason, int *inner_its, double *x_out);

#ifdef __cplusplus
}
#endif
#endif
