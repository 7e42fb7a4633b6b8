/*
 * oracle.c -- CPU restatement of the reference's GMRES inner-solve path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Compiled with -ffp-contract=off so
 * that every a*b+c is two roundings, as in PETSc's Seq kernels built without
 * FMA contraction.
 *
 * PETSc 3.22.1 is an external, un-vendored dependency of the reference
 * (README.md:31, makefile:36); its KSPGMRES behaviour is restated here from
 * that release's published semantics.  Functions carry the reference call site
 * they stand in for.
 */
#include "oracle.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define PMAX(a, b) ((a) < (b) ? (b) : (a)) /* PetscMax */
#define ORC_OK 0
#define ORC_ERR_MEM 55
#define ORC_ERR_ARG 62

/* Threads for the CPU-baseline timing (orc_set_threads): element-wise loops run
 * in parallel (each element's arithmetic is unchanged), and ORC_REDUCE_MT dots
 * sum per-thread contiguous pieces, then the pieces in thread order -- PETSc's
 * VecDot_MPI order (local ddot, then the Allreduce over ranks) with one rank per
 * thread.  The tests use 1 thread and the SEQ / DBR orders. */
static int orc_nthreads = 1;

void orc_set_threads(int t) { orc_nthreads = t > 0 ? t : 1; }

#define ORC_PAR _Pragma("omp parallel for schedule(static) num_threads(orc_nthreads) if (orc_nthreads > 1)")

void orc_csr_free(orc_csr *A) {
  if (!A) return;
  free(A->rowptr);
  free(A->col);
  free(A->val);
  memset(A, 0, sizeof(*A));
}

static int csr_alloc(orc_csr *A, int64_t nrows, int64_t ncols, int64_t nnz_cap) {
  memset(A, 0, sizeof(*A));
  if (nrows < 0 || nrows > INT32_MAX || ncols < 0 || ncols > INT32_MAX) return ORC_ERR_ARG;
  A->nrows = (int32_t)nrows;
  A->ncols = (int32_t)ncols;
  A->rowptr = (int32_t *)calloc((size_t)nrows + 1, sizeof(int32_t));
  A->col = (int32_t *)malloc((size_t)(nnz_cap > 0 ? nnz_cap : 1) * sizeof(int32_t));
  A->val = (double *)malloc((size_t)(nnz_cap > 0 ? nnz_cap : 1) * sizeof(double));
  if (!A->rowptr || !A->col || !A->val) {
    orc_csr_free(A);
    return ORC_ERR_MEM;
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* Assembly                                                                  */
/* ------------------------------------------------------------------------ */

/* poisson3DMatrix, src/utils/utils.c:30-121.  The reference inserts
 * (row, row-1, row+1, row-nx, row+nx, row-nxny, row+nxny) and PETSc AIJ keeps
 * each row's columns ascending, which is the order written here.  The
 * reference splits z at n_grid_columns/2 for its 2 blocks (utils.c:45,51);
 * this takes the plane range explicitly so nb blocks are z-slabs. */
int orc_poisson3d_rows(int nx, int ny, int nz, int z0, int z1, orc_csr *A) {
  if (nx <= 0 || ny <= 0 || nz <= 0 || z0 < 0 || z1 > nz || z0 > z1) return ORC_ERR_ARG;
  const int64_t nxny = (int64_t)nx * ny;
  const int64_t N = nxny * nz;
  if (N > INT32_MAX) return ORC_ERR_ARG;
  const int64_t nrows = nxny * (z1 - z0);
  int rc = csr_alloc(A, nrows, N, 7 * nrows);
  if (rc) return rc;
  int64_t p = 0, lr = 0;
  for (int k = z0; k < z1; ++k)
    for (int j = 0; j < ny; ++j)
      for (int i = 0; i < nx; ++i, ++lr) {
        const int64_t row = i + (int64_t)j * nx + (int64_t)k * nxny;
        A->rowptr[lr] = (int32_t)p;
        if (k > 0) { A->col[p] = (int32_t)(row - nxny); A->val[p++] = -1.0; }
        if (j > 0) { A->col[p] = (int32_t)(row - nx); A->val[p++] = -1.0; }
        if (i > 0) { A->col[p] = (int32_t)(row - 1); A->val[p++] = -1.0; }
        A->col[p] = (int32_t)row; A->val[p++] = 6.0;
        if (i < nx - 1) { A->col[p] = (int32_t)(row + 1); A->val[p++] = -1.0; }
        if (j < ny - 1) { A->col[p] = (int32_t)(row + nx); A->val[p++] = -1.0; }
        if (k < nz - 1) { A->col[p] = (int32_t)(row + nxny); A->val[p++] = -1.0; }
      }
  A->rowptr[nrows] = (int32_t)p;
  A->nnz = p;
  return ORC_OK;
}

/* poisson2DMatrix, src/utils/utils.c:247-293: global row Ii of an m x n grid,
 * i = Ii / n (n = n_grid_columns), j = Ii - i*n; neighbours Ii-+n (i), Ii-+1 (j);
 * diagonal 4.  Rows [row0,row1) of the block, local row = Ii - row0. */
int orc_poisson2d_rows(int m, int n, int64_t row0, int64_t row1, orc_csr *A) {
  if (m <= 0 || n <= 0) return ORC_ERR_ARG;
  const int64_t N = (int64_t)m * n;
  if (N > INT32_MAX || row0 < 0 || row1 > N || row0 > row1) return ORC_ERR_ARG;
  const int64_t nrows = row1 - row0;
  int rc = csr_alloc(A, nrows, N, 5 * nrows);
  if (rc) return rc;
  int64_t p = 0;
  for (int64_t Ii = row0; Ii < row1; ++Ii) {
    const int64_t i = Ii / n, j = Ii - i * n;
    A->rowptr[Ii - row0] = (int32_t)p;
    if (i > 0) { A->col[p] = (int32_t)(Ii - n); A->val[p++] = -1.0; }
    if (j > 0) { A->col[p] = (int32_t)(Ii - 1); A->val[p++] = -1.0; }
    A->col[p] = (int32_t)Ii; A->val[p++] = 4.0;
    if (j < n - 1) { A->col[p] = (int32_t)(Ii + 1); A->val[p++] = -1.0; }
    if (i < m - 1) { A->col[p] = (int32_t)(Ii + n); A->val[p++] = -1.0; }
  }
  A->rowptr[nrows] = (int32_t)p;
  A->nnz = p;
  return ORC_OK;
}

/* poisson2DMatrix_complete, src/utils/utils.c:383-445: Ii = i*N + j with
 * N = n_mesh_lines (the reference assumes a square mesh, utils.c:390). */
int orc_poisson2d_complete(int m, int n, orc_csr *A) {
  if (m <= 0 || n <= 0 || m != n) return ORC_ERR_ARG; /* square meshes only, as the reference */
  const int64_t Ntot = (int64_t)m * n, Nl = m;
  if (Ntot > INT32_MAX) return ORC_ERR_ARG;
  int rc = csr_alloc(A, Ntot, Ntot, 5 * Ntot);
  if (rc) return rc;
  /* rows are produced in Ii order only when n == m; build per-row lists */
  int64_t p = 0;
  for (int64_t Ii = 0; Ii < Ntot; ++Ii) {
    A->rowptr[Ii] = (int32_t)p;
    const int64_t i = Ii / Nl, j = Ii - i * Nl;
    if (i >= m || j >= n) continue; /* unreachable for square meshes */
    if (i > 0) { A->col[p] = (int32_t)(Ii - Nl); A->val[p++] = -1.0; }
    if (j > 0) { A->col[p] = (int32_t)(Ii - 1); A->val[p++] = -1.0; }
    A->col[p] = (int32_t)Ii; A->val[p++] = 4.0;
    if (j < Nl - 1) { A->col[p] = (int32_t)(Ii + 1); A->val[p++] = -1.0; }
    if (i < Nl - 1) { A->col[p] = (int32_t)(Ii + Nl); A->val[p++] = -1.0; }
  }
  A->rowptr[Ntot] = (int32_t)p;
  A->nnz = p;
  return ORC_OK;
}

/* divideSubDomainIntoBlockMatrices, src/utils/utils.c:450-478: A_sub[i] =
 * MatCreateSubMatrix(A_block, own rows, cols of block i).  Here the diagonal
 * block gets local columns and every off-block column goes to one coupling
 * matrix (global ids), which for 2 blocks is exactly the reference's A_ij. */
static double cd_lower(double p) { return -1.0 - 2.0 * (p > 0.0 ? p : 0.0); }
static double cd_upper(double p) { return -1.0 + 2.0 * (p < 0.0 ? p : 0.0); }

int orc_convdiff_rows(int dim, int nx, int ny, int nz, int64_t row0, int64_t row1, const double *P, orc_csr *A) {
  if (dim != 2 && dim != 3) return ORC_ERR_ARG;
  const int64_t n = row1 - row0;
  const int64_t N = (int64_t)nx * ny * (dim == 3 ? nz : 1);
  if (n < 0 || row0 < 0 || row1 > N) return ORC_ERR_ARG;
  int rc = csr_alloc(A, n, N, 7 * n);
  if (rc) return rc;
  const double px = P[0], py = P[1], pz = dim == 3 ? P[2] : 0.0;
  int64_t p = 0;
  A->rowptr[0] = 0;
  for (int64_t g = row0; g < row1; ++g) {
    const int64_t l = g - row0;
    if (dim == 3) {
      const int64_t i = g % nx, j = (g / nx) % ny, k = g / ((int64_t)nx * ny), pl = (int64_t)nx * ny;
      const double diag = ((6.0 + 2.0 * fabs(px)) + 2.0 * fabs(py)) + 2.0 * fabs(pz);
      if (k > 0) { A->col[p] = (int32_t)(g - pl); A->val[p++] = cd_lower(pz); }
      if (j > 0) { A->col[p] = (int32_t)(g - nx); A->val[p++] = cd_lower(py); }
      if (i > 0) { A->col[p] = (int32_t)(g - 1); A->val[p++] = cd_lower(px); }
      A->col[p] = (int32_t)g; A->val[p++] = diag;
      if (i < nx - 1) { A->col[p] = (int32_t)(g + 1); A->val[p++] = cd_upper(px); }
      if (j < ny - 1) { A->col[p] = (int32_t)(g + nx); A->val[p++] = cd_upper(py); }
      if (k < nz - 1) { A->col[p] = (int32_t)(g + pl); A->val[p++] = cd_upper(pz); }
    } else {
      /* nx = m mesh lines, ny = n mesh columns (poisson2DMatrix numbering): line = g / n */
      const int64_t m = nx, nn = ny, line = g / nn, c = g % nn;
      const double diag = (4.0 + 2.0 * fabs(px)) + 2.0 * fabs(py);
      if (line > 0) { A->col[p] = (int32_t)(g - nn); A->val[p++] = cd_lower(py); }
      if (c > 0) { A->col[p] = (int32_t)(g - 1); A->val[p++] = cd_lower(px); }
      A->col[p] = (int32_t)g; A->val[p++] = diag;
      if (c < nn - 1) { A->col[p] = (int32_t)(g + 1); A->val[p++] = cd_upper(px); }
      if (line < m - 1) { A->col[p] = (int32_t)(g + nn); A->val[p++] = cd_upper(py); }
    }
    A->rowptr[l + 1] = (int32_t)p;
  }
  A->nnz = p;
  return ORC_OK;
}

int orc_split(const orc_csr *Ab, int64_t c0, int64_t c1, orc_csr *Aii, orc_csr *Aoff) {
  int64_t nin = 0, nout = 0;
  for (int64_t k = 0; k < Ab->nnz; ++k) {
    if (Ab->col[k] >= c0 && Ab->col[k] < c1) ++nin; else ++nout;
  }
  int rc = csr_alloc(Aii, Ab->nrows, c1 - c0, nin);
  if (rc) return rc;
  rc = csr_alloc(Aoff, Ab->nrows, Ab->ncols, nout);
  if (rc) { orc_csr_free(Aii); return rc; }
  int64_t pi = 0, po = 0;
  for (int32_t r = 0; r < Ab->nrows; ++r) {
    Aii->rowptr[r] = (int32_t)pi;
    Aoff->rowptr[r] = (int32_t)po;
    for (int32_t k = Ab->rowptr[r]; k < Ab->rowptr[r + 1]; ++k) {
      const int32_t c = Ab->col[k];
      if (c >= c0 && c < c1) { Aii->col[pi] = (int32_t)(c - c0); Aii->val[pi++] = Ab->val[k]; }
      else { Aoff->col[po] = c; Aoff->val[po++] = Ab->val[k]; }
    }
  }
  Aii->rowptr[Ab->nrows] = (int32_t)pi;
  Aoff->rowptr[Ab->nrows] = (int32_t)po;
  Aii->nnz = pi;
  Aoff->nnz = po;
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* Mat / Vec kernels                                                         */
/* ------------------------------------------------------------------------ */

/* MatMult_SeqAIJ [PETSc-ext]: sum = 0; sum += aa[k]*x[aj[k]] left to right. */
void orc_spmv(const orc_csr *A, const double *x, double *y) {
  ORC_PAR
  for (int32_t r = 0; r < A->nrows; ++r) {
    double s = 0.0;
    for (int32_t k = A->rowptr[r]; k < A->rowptr[r + 1]; ++k) s += A->val[k] * x[A->col[k]];
    y[r] = s;
  }
}

/* MatResidual default [PETSc-ext]: MatMult(A,x,r); VecAYPX(r,-1,b) -> r = b - A x. */
void orc_residual(const orc_csr *A, const double *b, const double *x, double *r) {
  ORC_PAR
  for (int32_t row = 0; row < A->nrows; ++row) {
    double s = 0.0;
    for (int32_t k = A->rowptr[row]; k < A->rowptr[row + 1]; ++k) s += A->val[k] * x[A->col[k]];
    r[row] = b[row] - s;
  }
}

/* ---- Operators for the memory-lean records (orc_smsm_solve with lean = 1; test infrastructure) ----
 * An operator is either assembled rows (orc_csr) or the rows [r0, r1) of the dim-3 nx x ny x nz operator of
 * orc_convdiff_rows applied without storage (at P = 0 its values, -1 and 6, and its column order are exactly
 * orc_poisson3d_rows').  A stencil row sums the CSR row's terms in the CSR's column order from 0.0, so
 * op_spmv / op_residual are bit for bit orc_spmv / orc_residual of the assembled rows -- of the whole block rows
 * (OP_BLOCK, global columns), of orc_split's A_ii (OP_DIAG, columns in [r0, r1) shifted by -r0) or of its
 * coupling rows (OP_OFF, the other columns, global).  tests/test_oracle.py holds lean = 1 to lean = 0. */
enum { OP_BLOCK = 0, OP_DIAG = 1, OP_OFF = 2 };

typedef struct {
  const orc_csr *A; /* assembled, or NULL: the stencil */
  int part;
  int64_t nx, ny, nz, r0, r1;
  double lo[3], up[3], diag; /* lower / upper neighbour values in x, y, z; diagonal */
} orc_op;

static orc_op op_csr(const orc_csr *A) {
  orc_op o;
  memset(&o, 0, sizeof(o));
  o.A = A;
  return o;
}

static orc_op op_stencil(int nx, int ny, int nz, int64_t r0, int64_t r1, const double *P, int part) {
  orc_op o;
  memset(&o, 0, sizeof(o));
  o.part = part;
  o.nx = nx, o.ny = ny, o.nz = nz, o.r0 = r0, o.r1 = r1;
  for (int d = 0; d < 3; ++d) {
    o.lo[d] = cd_lower(P[d]);
    o.up[d] = cd_upper(P[d]);
  }
  o.diag = ((6.0 + 2.0 * fabs(P[0])) + 2.0 * fabs(P[1])) + 2.0 * fabs(P[2]);
  return o;
}

static int64_t op_rows(const orc_op *o) { return o->A ? o->A->nrows : o->r1 - o->r0; }

/* one term of a stencil row: column c (global) with value v, if this operator's part holds it */
#define OP_TERM(o, c, v, x, s)                                            \
  do {                                                                    \
    const int64_t c_ = (c);                                               \
    const int in_ = c_ >= (o)->r0 && c_ < (o)->r1;                        \
    if ((o)->part == OP_BLOCK) (s) += (v) * (x)[c_];                      \
    else if ((o)->part == OP_DIAG) { if (in_) (s) += (v) * (x)[c_ - (o)->r0]; } \
    else if (!in_) (s) += (v) * (x)[c_];                                  \
  } while (0)

/* row lr of the operator applied to x (x indexed as the part's columns) */
static inline double op_row(const orc_op *o, int64_t lr, const double *x) {
  double s = 0.0;
  if (o->A) {
    for (int32_t k = o->A->rowptr[lr]; k < o->A->rowptr[lr + 1]; ++k) s += o->A->val[k] * x[o->A->col[k]];
    return s;
  }
  const int64_t g = o->r0 + lr, nx = o->nx, pl = o->nx * o->ny;
  const int64_t i = g % nx, j = (g / nx) % o->ny, k = g / pl;
  if (k > 0) OP_TERM(o, g - pl, o->lo[2], x, s);
  if (j > 0) OP_TERM(o, g - nx, o->lo[1], x, s);
  if (i > 0) OP_TERM(o, g - 1, o->lo[0], x, s);
  OP_TERM(o, g, o->diag, x, s);
  if (i < nx - 1) OP_TERM(o, g + 1, o->up[0], x, s);
  if (j < o->ny - 1) OP_TERM(o, g + nx, o->up[1], x, s);
  if (k < o->nz - 1) OP_TERM(o, g + pl, o->up[2], x, s);
  return s;
}

static void op_spmv(const orc_op *o, const double *x, double *y) {
  if (o->A) {
    orc_spmv(o->A, x, y);
    return;
  }
  const int64_t n = op_rows(o);
  ORC_PAR
  for (int64_t r = 0; r < n; ++r) y[r] = op_row(o, r, x);
}

static void op_residual(const orc_op *o, const double *b, const double *x, double *r) {
  if (o->A) {
    orc_residual(o->A, b, x, r);
    return;
  }
  const int64_t n = op_rows(o);
  ORC_PAR
  for (int64_t row = 0; row < n; ++row) r[row] = b[row] - op_row(o, row, x);
}

/* Butterfly over one wave of 64 lane values: v[l] <- v[l] + v[l ^ off],
 * off = 32,16,...,1.  Lane 0 holds the result (all lanes agree). */
static double dbr_wave(const double *lanes) {
  double v[64], t[64];
  memcpy(v, lanes, sizeof(v));
  for (int off = 32; off >= 1; off >>= 1) {
    for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
    memcpy(v, t, sizeof(v));
  }
  return v[0];
}

/* One 256-thread workgroup: 4 wave butterflies, then (w0 + w1) + (w2 + w3). */
static double dbr_group(const double *lanes) {
  const double w0 = dbr_wave(lanes), w1 = dbr_wave(lanes + 64);
  const double w2 = dbr_wave(lanes + 128), w3 = dbr_wave(lanes + 192);
  return (w0 + w1) + (w2 + w3);
}

/* One DBR chunk of sum_i x[i]*y[i] over its len <= ORC_DBR_CHUNK elements (x, y at the chunk's first element):
 * lane t accumulates its elements j*(threads*vw) + vw*t + v in order, then the workgroup combine. */
static double dbr_chunk(int64_t len, const double *x, const double *y) {
  double lanes[ORC_DBR_THREADS];
  for (int t = 0; t < ORC_DBR_THREADS; ++t) {
    double acc = 0.0;
    for (int j = 0; j < ORC_DBR_ITERS; ++j) {
      const int64_t e = (int64_t)j * (ORC_DBR_THREADS * ORC_DBR_VW) + ORC_DBR_VW * t;
      for (int v = 0; v < ORC_DBR_VW; ++v)
        if (e + v < len) acc += x[e + v] * y[e + v];
    }
    lanes[t] = acc;
  }
  return dbr_group(lanes);
}

/* The second DBR stage: the chunk partials, lane t taking chunks t, t + threads, ... in order. */
static double dbr_finish(int64_t nchunks, const double *part) {
  double lanes[ORC_DBR_THREADS];
  for (int t = 0; t < ORC_DBR_THREADS; ++t) {
    double acc = 0.0;
    for (int64_t i = t; i < nchunks; i += ORC_DBR_THREADS) acc += part[i];
    lanes[t] = acc;
  }
  return dbr_group(lanes);
}

/* Deterministic blocked reduction of sum_i x[i]*y[i] (the device order). */
static double dbr_dot(int64_t n, const double *x, const double *y) {
  const int64_t nchunks = (n + ORC_DBR_CHUNK - 1) / ORC_DBR_CHUNK;
  double *part = (double *)malloc((size_t)(nchunks > 0 ? nchunks : 1) * sizeof(double));
  /* chunks are independent: threads split them, each chunk's arithmetic unchanged */
  ORC_PAR
  for (int64_t c = 0; c < nchunks; ++c) {
    const int64_t base = c * ORC_DBR_CHUNK;
    const int64_t len = n - base < ORC_DBR_CHUNK ? n - base : ORC_DBR_CHUNK;
    part[c] = dbr_chunk(len, x + base, y + base);
  }
  const double r = dbr_finish(nchunks, part);
  free(part);
  return r;
}

/* VecDot / BLAS ddot order: sequential (reference ddot's unroll-by-5 is
 * evaluated left to right, i.e. still sequential). */
static double seq_dot(int64_t n, const double *x, const double *y) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += x[i] * y[i];
  return s;
}

static double mt_dot(int64_t n, const double *x, const double *y) {
  double part[1024];
  int used = 1;
#pragma omp parallel num_threads(orc_nthreads > 1024 ? 1024 : orc_nthreads)
  {
#ifdef _OPENMP
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
#else
    const int t = 0, nt = 1;
#endif
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    double acc = 0.0;
    for (int64_t i = lo; i < hi; ++i) acc += x[i] * y[i];
    part[t] = acc;
    if (t == 0) used = nt;
  }
  double s = 0.0;
  for (int t = 0; t < used; ++t) s += part[t];
  return s;
}

double orc_dot(int mode, int64_t n, const double *x, const double *y) {
  if (mode == ORC_REDUCE_MT) return mt_dot(n, x, y);
  return mode == ORC_REDUCE_DBR ? dbr_dot(n, x, y) : seq_dot(n, x, y);
}

/* VecNorm(NORM_2) [PETSc-ext]: sqrt(ddot(x,x)). */
double orc_norm2(int mode, int64_t n, const double *x) { return sqrt(orc_dot(mode, n, x, x)); }

/* VecMDot_Seq [PETSc-ext]: out[j] = sum_i w[i]*V_j[i], sequential per vector. */
void orc_mdot(int mode, int64_t n, int k, const double *w, const double *const *V, double *out) {
  for (int j = 0; j < k; ++j) out[j] = orc_dot(mode, n, w, V[j]);
}

/* VecMAXPY_Seq [PETSc-ext]: the nv & 3 leading vectors first (PetscKernelAXPY3/2/1),
 * then groups of four (PetscKernelAXPY4): U += a0*p0 + a1*p1 + a2*p2 + a3*p3,
 * evaluated left to right and then added to U. */
void orc_maxpy(int64_t n, int k, const double *a, const double *const *V, double *w) {
  const int jrem = k & 3;
  ORC_PAR
  for (int64_t i = 0; i < n; ++i) {
    double u = w[i];
    if (jrem == 3) u = u + ((a[0] * V[0][i] + a[1] * V[1][i]) + a[2] * V[2][i]);
    else if (jrem == 2) u = u + (a[0] * V[0][i] + a[1] * V[1][i]);
    else if (jrem == 1) u = a[0] * V[0][i] + u;
    for (int j = jrem; j < k; j += 4)
      u = u + (((a[j] * V[j][i] + a[j + 1] * V[j + 1][i]) + a[j + 2] * V[j + 2][i]) + a[j + 3] * V[j + 3][i]);
    w[i] = u;
  }
}

/* ------------------------------------------------------------------------ */
/* KSPGMRES [PETSc-ext]                                                      */
/* ------------------------------------------------------------------------ */

void orc_gmres_default_opts(orc_gmres_opts *o) {
  o->restart = 30;
  o->max_it = 10000;
  o->rtol = 1e-5;
  o->abstol = 1e-50;
  o->divtol = 1e4;
  o->haptol = 1e-30;
  o->breakdowntol = 0.1;
  o->uirnorm = 0;
  o->guess_nonzero = 0;
  o->reduce_mode = ORC_REDUCE_SEQ;
}

typedef struct {
  const orc_op *A;
  const double *b;
  double *x;
  const orc_gmres_opts *o;
  int64_t n;
  int m;
  double **VV;     /* VEC_VV(0..m) */
  double *tmp;     /* VEC_TEMP */
  double *hh;      /* HH(a,b) = hh[b*(m+2)+a] */
  double *cc, *ss, *grs, *lhh;
  /* KSP state */
  int its, reason, guess_zero;
  double rnorm;    /* ksp->rnorm */
  double rnorm0;   /* ksp->rnorm0 (convergence test) */
  double ttol;
  double gm_rnorm0;/* gmres->rnorm0 */
  double *hist;
  int hist_cap, nhist;
} gm_t;

#define HH(g, a, b) ((g)->hh[(int64_t)(b) * ((g)->m + 2) + (a)])

static int is_bad(double v) { return isnan(v) || isinf(v); }

static void gm_log(gm_t *g, double r) {
  if (g->hist && g->nhist < g->hist_cap) g->hist[g->nhist] = r;
  g->nhist++;
}

/* KSPConvergedDefault [PETSc-ext] */
static void gm_converged(gm_t *g, int n, double rnorm) {
  g->reason = ORC_CONVERGED_ITERATING;
  if (n == 0) {
    if (!g->guess_zero && !g->o->uirnorm) {
      double snorm = orc_norm2(g->o->reduce_mode, g->n, g->b);
      if (snorm == 0.0) snorm = rnorm;
      g->rnorm0 = snorm;
    } else {
      g->rnorm0 = rnorm;
    }
    g->ttol = PMAX(g->o->rtol * g->rnorm0, g->o->abstol);
  }
  if (is_bad(rnorm)) {
    g->reason = ORC_DIVERGED_NANORINF;
  } else if (rnorm <= g->ttol) {
    g->reason = (rnorm < g->o->abstol) ? ORC_CONVERGED_ATOL : ORC_CONVERGED_RTOL;
  } else if (rnorm >= g->o->divtol * g->rnorm0) {
    g->reason = ORC_DIVERGED_DTOL;
  }
}

/* VecNormalize [PETSc-ext]: t = ||v||; v *= 1/t unless t is 0 or not finite. */
static double gm_normalize(gm_t *g, double *v) {
  const double t = orc_norm2(g->o->reduce_mode, g->n, v);
  if (t != 0.0 && !is_bad(t)) {
    const double s = 1.0 / t;
    ORC_PAR
    for (int64_t i = 0; i < g->n; ++i) v[i] = v[i] * s;
  }
  return t;
}

/* KSPGMRESUpdateHessenberg [PETSc-ext] */
static void gm_update_hessenberg(gm_t *g, int it, int hapend, double *res) {
  double *hh = &HH(g, 0, it);
  for (int j = 1; j <= it; ++j) {
    const double tt = hh[j - 1];
    hh[j - 1] = g->cc[j - 1] * tt + g->ss[j - 1] * hh[j];
    hh[j] = g->cc[j - 1] * hh[j] - (g->ss[j - 1] * tt);
  }
  if (!hapend) {
    const double tt = sqrt(hh[it] * hh[it] + hh[it + 1] * hh[it + 1]);
    if (tt == 0.0) {
      g->reason = ORC_DIVERGED_NULL;
      return;
    }
    g->cc[it] = hh[it] / tt;
    g->ss[it] = hh[it + 1] / tt;
    g->grs[it + 1] = -(g->ss[it] * g->grs[it]);
    g->grs[it] = g->cc[it] * g->grs[it];
    hh[it] = g->cc[it] * hh[it] + g->ss[it] * hh[it + 1];
    *res = fabs(g->grs[it + 1]);
  } else {
    *res = 0.0;
  }
}

/* KSPGMRESBuildSoln(GRS(0), x, x, ksp, it) [PETSc-ext]; nrs aliases GRS. */
static void gm_build_soln(gm_t *g, int it) {
  if (it < 0) return;
  double *nrs = g->grs;
  if (HH(g, it, it) != 0.0) {
    nrs[it] = g->grs[it] / HH(g, it, it);
  } else {
    g->reason = ORC_DIVERGED_BREAKDOWN;
    return;
  }
  for (int ii = 1; ii <= it; ++ii) {
    const int k = it - ii;
    double tt = g->grs[k];
    for (int j = k + 1; j <= it; ++j) tt = tt - HH(g, k, j) * nrs[j];
    if (HH(g, k, k) == 0.0) {
      g->reason = ORC_DIVERGED_BREAKDOWN;
      return;
    }
    nrs[k] = tt / HH(g, k, k);
  }
  /* VecSet(TEMP,0); VecMAXPY(TEMP,it+1,nrs,VV); KSPUnwindPreconditioner (PCNONE: identity);
   * VecAXPY(x, 1.0, TEMP) */
  ORC_PAR
  for (int64_t i = 0; i < g->n; ++i) g->tmp[i] = 0.0;
  orc_maxpy(g->n, it + 1, nrs, (const double *const *)g->VV, g->tmp);
  ORC_PAR
  for (int64_t i = 0; i < g->n; ++i) g->x[i] = g->x[i] + 1.0 * g->tmp[i];
}

/* KSPGMRESClassicalGramSchmidtOrthogonalization, REFINE_NEVER [PETSc-ext] */
static void gm_cgs(gm_t *g, int it) {
  double *hh = &HH(g, 0, it);
  for (int j = 0; j <= it; ++j) hh[j] = 0.0;
  orc_mdot(g->o->reduce_mode, g->n, it + 1, g->VV[it + 1], (const double *const *)g->VV, g->lhh);
  for (int j = 0; j <= it; ++j) {
    if (is_bad(g->lhh[j])) {
      g->reason = ORC_DIVERGED_NANORINF;
      return;
    }
    g->lhh[j] = -g->lhh[j];
  }
  orc_maxpy(g->n, it + 1, g->lhh, (const double *const *)g->VV, g->VV[it + 1]);
  for (int j = 0; j <= it; ++j) hh[j] -= g->lhh[j];
}

/* KSPGMRESCycle [PETSc-ext] */
static void gm_cycle(gm_t *g, int *itcount) {
  int it = 0, hapend = 0;
  double res;
  *itcount = 0;
  res = gm_normalize(g, g->VV[0]);
  if (is_bad(res)) { /* KSPCheckNorm */
    g->reason = ORC_DIVERGED_NANORINF;
    return;
  }
  if (g->rnorm > 0.0 && fabs(res - g->rnorm) > g->o->breakdowntol * g->gm_rnorm0) {
    g->reason = ORC_DIVERGED_BREAKDOWN;
    return;
  }
  g->grs[0] = g->gm_rnorm0 = res;
  g->rnorm = res;
  gm_log(g, res);
  if (res == 0.0) {
    g->reason = ORC_CONVERGED_ATOL;
    return;
  }
  gm_converged(g, g->its, res);
  while (!g->reason && it < g->m && g->its < g->o->max_it) {
    if (it) gm_log(g, res);
    /* KSP_PCApplyBAorAB, PCNONE: VV(it+1) = A * VV(it) */
    op_spmv(g->A, g->VV[it], g->VV[it + 1]);
    gm_cgs(g, it);
    if (g->reason) break;
    const double tt = gm_normalize(g, g->VV[it + 1]);
    if (is_bad(tt)) {
      g->reason = ORC_DIVERGED_NANORINF;
      return;
    }
    HH(g, it + 1, it) = tt;
    double hapbnd = fabs(tt / g->grs[it]);
    if (hapbnd > g->o->haptol) hapbnd = g->o->haptol;
    if (tt < hapbnd) hapend = 1;
    gm_update_hessenberg(g, it, hapend, &res);
    it++;
    g->its++;
    g->rnorm = res;
    if (g->reason) break;
    gm_converged(g, g->its, res);
    if (hapend) {
      if (!g->reason) {
        g->reason = ORC_DIVERGED_BREAKDOWN;
        break;
      }
    }
  }
  if (it && (g->reason || g->its >= g->o->max_it)) gm_log(g, res);
  *itcount = it;
  gm_build_soln(g, it - 1);
}

/* KSPSolve -> KSPSolve_GMRES [PETSc-ext] */
static int gmres_solve_op(const orc_op *A, const double *b, double *x, const orc_gmres_opts *o,
                          orc_gmres_result *res, double *hist, int hist_cap) {
  gm_t g;
  memset(&g, 0, sizeof(g));
  g.A = A;
  g.b = b;
  g.x = x;
  g.o = o;
  g.n = op_rows(A);
  g.m = o->restart;
  g.hist = hist;
  g.hist_cap = hist_cap;
  const int64_t n = g.n, m = g.m;
  g.VV = (double **)malloc((size_t)(m + 1) * sizeof(double *));
  double *vv = (double *)calloc((size_t)((m + 1) * n + n + 1), sizeof(double));
  g.hh = (double *)calloc((size_t)((m + 2) * (m + 1)), sizeof(double));
  g.cc = (double *)calloc((size_t)(m + 2), sizeof(double));
  g.ss = (double *)calloc((size_t)(m + 2), sizeof(double));
  g.grs = (double *)calloc((size_t)(m + 2), sizeof(double));
  g.lhh = (double *)calloc((size_t)(m + 2), sizeof(double));
  if (!g.VV || !vv || !g.hh || !g.cc || !g.ss || !g.grs || !g.lhh) {
    free(g.VV); free(vv); free(g.hh); free(g.cc); free(g.ss); free(g.grs); free(g.lhh);
    return ORC_ERR_MEM;
  }
  for (int64_t j = 0; j <= m; ++j) g.VV[j] = vv + j * n;
  g.tmp = vv + (m + 1) * n;

  g.guess_zero = !o->guess_nonzero;
  if (g.guess_zero)
    for (int64_t i = 0; i < n; ++i) x[i] = 0.0; /* KSPSolve zeroes x for a zero guess */
  g.its = 0;
  g.reason = 0;
  g.rnorm = -1.0; /* special marker for KSPGMRESCycle() */
  int itcount = 0;
  while (!g.reason) {
    /* KSPInitialResidual: r = b - A x (VecCopy + VecAXPY(-1)), or r = b for a zero guess */
    if (!g.guess_zero) {
      op_spmv(A, x, g.tmp);
      for (int64_t i = 0; i < n; ++i) g.VV[0][i] = b[i] + (-1.0) * g.tmp[i];
    } else {
      memcpy(g.VV[0], b, (size_t)n * sizeof(double));
    }
    int its = 0;
    gm_cycle(&g, &its);
    itcount += its;
    if (itcount >= o->max_it) {
      if (!g.reason) g.reason = ORC_DIVERGED_ITS;
      break;
    }
    g.guess_zero = 0;
  }
  if (res) {
    res->its = g.its;
    res->reason = g.reason;
    res->rnorm = g.rnorm;
    res->nhist = g.nhist;
  }
  free(g.VV); free(vv); free(g.hh); free(g.cc); free(g.ss); free(g.grs); free(g.lhh);
  return ORC_OK;
}

int orc_gmres_solve(const orc_csr *A, const double *b, double *x, const orc_gmres_opts *o,
                    orc_gmres_result *res, double *hist, int hist_cap) {
  if (!A || !o || o->restart < 1 || A->nrows != A->ncols) return ORC_ERR_ARG;
  const orc_op op = op_csr(A);
  return gmres_solve_op(&op, b, x, o, res, hist, hist_cap);
}

/* ------------------------------------------------------------------------ */
/* Reference glue                                                            */
/* ------------------------------------------------------------------------ */

/* computeFinalResidualNorm_new, src/utils/utils.c:597-620 (and the block-root
 * variant computeFinalResidualNorm, :575-595): VecNorm of each block's
 * residual, squared, summed over blocks (block order), square root. */
double orc_final_residual_norm(int mode, int nb, const orc_csr *const *Ab, const double *x,
                               const double *const *bb) {
  double total = 0.0;
  for (int b = 0; b < nb; ++b) {
    double *r = (double *)malloc((size_t)(Ab[b]->nrows > 0 ? Ab[b]->nrows : 1) * sizeof(double));
    orc_residual(Ab[b], bb[b], x, r);
    const double ln = orc_norm2(mode, Ab[b]->nrows, r);
    total += ln * ln;
    free(r);
  }
  return sqrt(total);
}

static double final_residual_norm_op(int mode, int nb, const orc_op *Ab, const double *x, const double *const *bb) {
  double total = 0.0;
  for (int b = 0; b < nb; ++b) {
    const int64_t n = op_rows(&Ab[b]);
    double *r = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    op_residual(&Ab[b], bb[b], x, r);
    const double ln = orc_norm2(mode, n, r);
    total += ln * ln;
    free(r);
  }
  return sqrt(total);
}

static int build_block(const orc_sm_problem *p, int b, orc_csr *Ablock, int64_t *r0, int64_t *r1) {
  const int cd = p->peclet[0] != 0.0 || p->peclet[1] != 0.0 || p->peclet[2] != 0.0;
  if (p->dim == 3) {
    const int ppb = p->nz / p->nb;
    const int64_t nxny = (int64_t)p->nx * p->ny;
    *r0 = (int64_t)b * ppb * nxny;
    *r1 = (int64_t)(b + 1) * ppb * nxny;
    if (cd) return orc_convdiff_rows(3, p->nx, p->ny, p->nz, *r0, *r1, p->peclet, Ablock);
    return orc_poisson3d_rows(p->nx, p->ny, p->nz, b * ppb, (b + 1) * ppb, Ablock);
  }
  const int64_t N = (int64_t)p->nx * p->ny, rbs = N / p->nb;
  *r0 = b * rbs;
  *r1 = (b + 1) * rbs;
  if (cd) return orc_convdiff_rows(2, p->nx, p->ny, 1, *r0, *r1, p->peclet, Ablock);
  return orc_poisson2d_rows(p->nx, p->ny, *r0, *r1, Ablock);
}

/* Synchronous multisplitting, src/synchronous-multisplitting/synchronous-multisplitting.c:
 * setup :101-164, loop :170-206; nb blocks simulated in block order.  For nb = 2
 * this is the reference loop; the block exchange (comm.c:126) is the copy of
 * every block's x_i into the global x before the RHS updates. */
int orc_sm_solve(const orc_sm_problem *p, const orc_gmres_opts *inner, orc_sm_result *res,
                 double *outer_hist, int outer_cap, int *inner_its, double *x_out) {
  const int nb = p->nb;
  if (nb < 1 || (p->dim != 2 && p->dim != 3)) return ORC_ERR_ARG;
  if (p->dim == 3 && p->nz % nb) return ORC_ERR_ARG;
  if (p->dim == 2 && ((int64_t)p->nx * p->ny) % nb) return ORC_ERR_ARG;
  const int64_t N = (int64_t)p->nx * p->ny * (p->dim == 3 ? p->nz : 1);
  const int mode = inner->reduce_mode;
  orc_csr *Ab = (orc_csr *)calloc((size_t)nb, sizeof(orc_csr));
  orc_csr *Aii = (orc_csr *)calloc((size_t)nb, sizeof(orc_csr));
  orc_csr *Aoff = (orc_csr *)calloc((size_t)nb, sizeof(orc_csr));
  int64_t *r0 = (int64_t *)calloc((size_t)nb, sizeof(int64_t));
  int64_t *r1 = (int64_t *)calloc((size_t)nb, sizeof(int64_t));
  double *x = (double *)calloc((size_t)N, sizeof(double));
  double *u = (double *)malloc((size_t)N * sizeof(double));
  double *bvec = (double *)calloc((size_t)N, sizeof(double));
  double *rhs = (double *)calloc((size_t)N, sizeof(double));
  double *r = (double *)calloc((size_t)N, sizeof(double));
  double *y = (double *)calloc((size_t)N, sizeof(double));
  const orc_csr **Abp = (const orc_csr **)calloc((size_t)nb, sizeof(orc_csr *));
  const double **bbp = (const double **)calloc((size_t)nb, sizeof(double *));
  int rc = ORC_OK;
  if (!Ab || !Aii || !Aoff || !r0 || !r1 || !x || !u || !bvec || !rhs || !r || !y || !Abp || !bbp) {
    rc = ORC_ERR_MEM;
    goto done;
  }
  for (int64_t i = 0; i < N; ++i) u[i] = 1.0;
  for (int b = 0; b < nb; ++b) {
    if ((rc = build_block(p, b, &Ab[b], &r0[b], &r1[b]))) goto done;
    if ((rc = orc_split(&Ab[b], r0[b], r1[b], &Aii[b], &Aoff[b]))) goto done;
    /* computeTheRightHandSideWithInitialGuess (utils.c:623-650): b_i = A_block u */
    orc_spmv(&Ab[b], u, bvec + r0[b]);
    Abp[b] = &Ab[b];
    bbp[b] = bvec + r0[b];
  }
  /* computeFinalResidualNorm at x = 0 (synchronous-multisplitting.c:162) */
  const double norm0 = orc_final_residual_norm(mode, nb, Abp, x, bbp);
  /* updateLocalRHS before the loop (:164) */
  for (int b = 0; b < nb; ++b) orc_residual(&Aoff[b], bvec + r0[b], x, rhs + r0[b]);

  orc_gmres_opts io = *inner;
  io.guess_nonzero = 1; /* inner_solver, utils.c:956-957 */
  io.uirnorm = 1;
  int outer = 0;
  double norm = 0.0;
  int64_t total_inner = 0;
  for (;;) {
    for (int b = 0; b < nb; ++b) {
      orc_gmres_result gr;
      if ((rc = orc_gmres_solve(&Aii[b], rhs + r0[b], x + r0[b], &io, &gr, NULL, 0))) goto done;
      if (inner_its && outer < outer_cap) inner_its[(int64_t)outer * nb + b] = gr.its;
      total_inner += gr.its;
    }
    /* comm_sync_send_and_receive: every block now sees every x_j (x is shared here) */
    double sum = 0.0;
    for (int b = 0; b < nb; ++b) {
      const int64_t nbk = r1[b] - r0[b];
      orc_residual(&Aoff[b], bvec + r0[b], x, rhs + r0[b]);     /* updateLocalRHS */
      orc_residual(&Aii[b], rhs + r0[b], x + r0[b], r + r0[b]);  /* MatResidual(A_ii,...) */
      const double ln = orc_norm2(mode, nbk, r + r0[b]);
      sum += ln * ln;                                            /* Allreduce(SUM) of squares */
    }
    norm = sqrt(sum);
    if (outer_hist && outer < outer_cap) outer_hist[outer] = norm;
    outer++;
    if (norm <= PMAX(p->atol, p->rtol * norm0)) break;
    if (p->max_outer > 0 && outer >= p->max_outer) break;
  }
  if (res) {
    res->outer_its = outer;
    res->norm0 = norm0;
    res->final_norm = orc_final_residual_norm(mode, nb, Abp, x, bbp);
    for (int64_t i = 0; i < N; ++i) y[i] = -1.0 * u[i] + x[i]; /* VecWAXPY(diff,-1,u,x) */
    res->error = orc_norm2(mode, N, y);
    res->total_inner_its = total_inner;
  }
  if (x_out) memcpy(x_out, x, (size_t)N * sizeof(double));
done:
  if (Ab)
    for (int b = 0; b < nb; ++b) { orc_csr_free(&Ab[b]); orc_csr_free(&Aii[b]); orc_csr_free(&Aoff[b]); }
  free(Ab); free(Aii); free(Aoff); free(r0); free(r1); free(x); free(u); free(bvec);
  free(rhs); free(r); free(y); free(Abp); free(bbp);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* KSPLSQR [PETSc-ext], PCNONE, over a row-distributed dense operator         */
/* ------------------------------------------------------------------------ */

void orc_lsqr_default_opts(orc_lsqr_opts *o) {
  o->max_it = 10000;
  o->rtol = 1e-5;
  o->abstol = 1e-50;
  o->divtol = 1e4;
  o->exact_norm = 0;
  o->conv_test = ORC_LSQR_CONV_LSQR; /* KSPCreate_LSQR installs KSPLSQRConvergedDefault */
  o->reduce_mode = ORC_REDUCE_SEQ;
  o->onepass = 1;
}

typedef struct {
  int nblk, s, mode;
  const int64_t *n;
} ls_layout;

/* sum over all rows of x[b][i]*y[b][i] (x[b], y[b] stride 1) */
static double ls_gdot(const ls_layout *L, const double *const *x, const double *const *y) {
  if (L->mode == ORC_REDUCE_SEQ) {
    double s = 0.0;
    for (int b = 0; b < L->nblk; ++b)
      for (int64_t i = 0; i < L->n[b]; ++i) s += x[b][i] * y[b][i];
    return s;
  }
  double t = 0.0;
  for (int b = 0; b < L->nblk; ++b) t += dbr_dot(L->n[b], x[b], y[b]);
  return t;
}

/* MatMultTranspose(R, u, out): out[j] = column_j . u (reference dgemv 'T' per column) */
static void ls_mult_transpose(const ls_layout *L, const double *const *R, const int64_t *lda,
                              const double *const *u, double *out) {
  const double **col = (const double **)malloc((size_t)L->nblk * sizeof(double *));
  for (int j = 0; j < L->s; ++j) {
    for (int b = 0; b < L->nblk; ++b) col[b] = R[b] + (int64_t)j * lda[b];
    out[j] = ls_gdot(L, col, u);
  }
  free(col);
}

/* MatNorm(R, NORM_FROBENIUS).  SEQ: one sum of squares over the columns in
 * order (each over all N rows), then sqrt -- PETSc 3.22.1's MatNorm_SeqDense in
 * a double build (R is MATMPIDENSE on a one-process block communicator,
 * SMSM-global.c:136): a plain running sum over the column-major array; BLASnrm2
 * only under PETSC_USE_REAL___FP16.  DBR: per block the column sums of squares
 * (DBR) added in column order, then blocks in order. */
static double ls_frobenius(const ls_layout *L, const double *const *R, const int64_t *lda) {
  double t = 0.0;
  if (L->mode == ORC_REDUCE_SEQ) {
    for (int j = 0; j < L->s; ++j)
      for (int b = 0; b < L->nblk; ++b) {
        const double *c = R[b] + (int64_t)j * lda[b];
        for (int64_t i = 0; i < L->n[b]; ++i) t += c[i] * c[i];
      }
    return sqrt(t);
  }
  for (int b = 0; b < L->nblk; ++b) {
    double tb = 0.0;
    for (int j = 0; j < L->s; ++j) {
      const double *c = R[b] + (int64_t)j * lda[b];
      tb += dbr_dot(L->n[b], c, c);
    }
    t += tb;
  }
  return sqrt(t);
}

void orc_dense_mult(int64_t n, int s, const double *S, int64_t lda, const double *alpha, double *y) {
  for (int64_t i = 0; i < n; ++i) {
    double acc = 0.0;
    for (int j = 0; j < s; ++j) acc = acc + alpha[j] * S[i + (int64_t)j * lda];
    y[i] = acc;
  }
}

/* outer_solver (src/utils/utils.c:972-996): MatTransposeMatMult(R, R, .., R_transpose_R) and
 * MatMultTranspose(R, b, vec_R_transpose_b) over one block's rows, as Gc = [R^T R | R^T b]
 * (s x (s+1), column-major, leading dimension ldg).  R is MATMPIDENSE on a one-rank block
 * communicator, so PETSc 3.22.1 runs the SeqDense kernels: BLASgemm_("T", "N") and dgemv 'T',
 * whose reference (f2cblaslapack) loops are, per entry, TEMP = TEMP + A(L,I)*B(L,J) over the
 * rows in order from zero and C(I,J) = ALPHA*TEMP with ALPHA = 1 (exact): ORC_REDUCE_SEQ.
 * ORC_REDUCE_DBR: each entry is the device order's dot (dbr_dot), so G(i,j) = G(j,i). */
void orc_dense_gram(int mode, int64_t n, int s, const double *R, int64_t lda, const double *b, double *Gc,
                    int64_t ldg) {
  for (int j = 0; j <= s; ++j) {
    const double *cj = j < s ? R + (int64_t)j * lda : b;
    for (int i = 0; i < s; ++i) {
      const double *ci = R + (int64_t)i * lda;
      double v;
      if (mode == ORC_REDUCE_DBR) {
        v = dbr_dot(n, ci, cj);
      } else {
        v = 0.0;
        for (int64_t l = 0; l < n; ++l) v = v + ci[l] * cj[l];
      }
      Gc[i + (int64_t)j * ldg] = v;
    }
  }
}

/* VecNorm of an s-vector (one rank holds it whole: sequential) */
static double ls_snorm(int s, const double *v) {
  double t = 0.0;
  for (int j = 0; j < s; ++j) t += v[j] * v[j];
  return sqrt(t);
}

/* VecScale(v, a): a == 0 sets, a == 1 leaves v alone */
static void ls_scale(int64_t n, double *v, double a) {
  if (a == 0.0) {
    for (int64_t i = 0; i < n; ++i) v[i] = 0.0;
  } else if (a != 1.0) {
    for (int64_t i = 0; i < n; ++i) v[i] = v[i] * a;
  }
}

/* VecAXPY(y, a, x): y = y + a*x, nothing when a == 0 */
static void ls_axpy(int64_t n, double *y, double a, const double *x) {
  if (a == 0.0) return;
  for (int64_t i = 0; i < n; ++i) y[i] = y[i] + a * x[i];
}

/* VecAYPX(y, a, x): y = x + a*y (a == 0: copy, a == 1: y + x) */
static void ls_aypx(int64_t n, double *y, double a, const double *x) {
  if (a == 0.0) {
    for (int64_t i = 0; i < n; ++i) y[i] = x[i];
  } else if (a == 1.0) {
    for (int64_t i = 0; i < n; ++i) y[i] = y[i] + x[i];
  } else {
    for (int64_t i = 0; i < n; ++i) y[i] = x[i] + a * y[i];
  }
}

/* The LSQR operator R as nblk row blocks: stored (R[b] + j*lda[b]), or -- the memory-lean records -- formed on
 * the fly as R_b = A_b S (A_b the block's rows over global columns, S column j at S + j*lds): every element is
 * the stored R's element (op_row is orc_spmv's row), so every sum below is bit for bit the stored one. */
#define ORC_RS_MAXS 256 /* columns of an on-the-fly R (s) */

typedef struct {
  const double *const *R;
  const int64_t *lda;
  const orc_op *A;
  const double *S;
  int64_t lds;
} ls_rsrc;

/* rows [i0, i1) of block b, columns [j0, j1), into buf (column-major, leading dimension i1 - i0).  A stencil row's
 * legs are found once per row (a presence mask) and then applied column by column, each column's rows in order:
 * every element still sums its row's terms in the row's order from 0.0. */
static void rs_fill(const ls_rsrc *src, int b, int64_t i0, int64_t i1, int j0, int j1, double *buf) {
  const int64_t m = i1 - i0;
  const orc_op *o = &src->A[b];
  if (o->A || o->part != OP_BLOCK) {
    for (int j = j0; j < j1; ++j) {
      const double *Sj = src->S + (int64_t)j * src->lds;
      double *d = buf + (int64_t)(j - j0) * m;
      for (int64_t i = i0; i < i1; ++i) d[i - i0] = op_row(o, i, Sj);
    }
    return;
  }
  const int64_t nx = o->nx, pl = o->nx * o->ny;
  const int64_t off[7] = {-pl, -nx, -1, 0, 1, nx, pl};
  const double val[7] = {o->lo[2], o->lo[1], o->lo[0], o->diag, o->up[0], o->up[1], o->up[2]};
  uint8_t *mask = (uint8_t *)malloc((size_t)(m > 0 ? m : 1));
  for (int64_t r = i0; r < i1; ++r) {
    const int64_t g = o->r0 + r, i = g % nx, jy = (g / nx) % o->ny, k = g / pl;
    mask[r - i0] = (uint8_t)((k > 0) | (jy > 0) << 1 | (i > 0) << 2 | 1 << 3 | (i < nx - 1) << 4 |
                             (jy < o->ny - 1) << 5 | (k < o->nz - 1) << 6);
  }
  for (int j = j0; j < j1; ++j) {
    const double *Sj = src->S + (int64_t)j * src->lds + o->r0;
    double *d = buf + (int64_t)(j - j0) * m;
    for (int64_t r = i0; r < i1; ++r) {
      const uint8_t mk = mask[r - i0];
      const double *c = Sj + r;
      double acc = 0.0;
      if (mk == 0x7f) {
        acc += val[0] * c[off[0]];
        acc += val[1] * c[off[1]];
        acc += val[2] * c[off[2]];
        acc += val[3] * c[0];
        acc += val[4] * c[off[4]];
        acc += val[5] * c[off[5]];
        acc += val[6] * c[off[6]];
      } else {
        for (int t = 0; t < 7; ++t)
          if (mk >> t & 1) acc += val[t] * c[off[t]];
      }
      d[r - i0] = acc;
    }
  }
  free(mask);
}

/* U1_b = R_b V (orc_dense_mult's row order) */
static void rs_mult(const ls_layout *L, const ls_rsrc *src, const double *V, double *const *U1) {
  for (int b = 0; b < L->nblk; ++b) {
    if (src->R) {
      orc_dense_mult(L->n[b], L->s, src->R[b], src->lda[b], V, U1[b]);
      continue;
    }
    const int64_t n = L->n[b], nt = (n + ORC_DBR_CHUNK - 1) / ORC_DBR_CHUNK;
    ORC_PAR
    for (int64_t t = 0; t < nt; ++t) {
      const int64_t i0 = t * ORC_DBR_CHUNK, i1 = i0 + ORC_DBR_CHUNK < n ? i0 + ORC_DBR_CHUNK : n, m = i1 - i0;
      double *tile = (double *)malloc((size_t)(m * L->s) * sizeof(double));
      rs_fill(src, b, i0, i1, 0, L->s, tile);
      orc_dense_mult(m, L->s, tile, m, V, U1[b] + i0);
      free(tile);
    }
  }
}

/* DBR dots of every column of R_b with y_b (y_b = NULL: with itself), out[j] */
static void rs_dbr_block_dots(const ls_layout *L, const ls_rsrc *src, int b, const double *y, double *out) {
  const int64_t n = L->n[b], nc = (n + ORC_DBR_CHUNK - 1) / ORC_DBR_CHUNK;
  const int s = L->s;
  double *part = (double *)malloc((size_t)((nc > 0 ? nc : 1) * s) * sizeof(double));
  ORC_PAR
  for (int64_t c = 0; c < nc; ++c) {
    const int64_t i0 = c * ORC_DBR_CHUNK, m = n - i0 < ORC_DBR_CHUNK ? n - i0 : ORC_DBR_CHUNK;
    double *tile = (double *)malloc((size_t)(m * s) * sizeof(double));
    rs_fill(src, b, i0, i0 + m, 0, s, tile);
    for (int j = 0; j < s; ++j) {
      const double *col = tile + (int64_t)j * m;
      part[(int64_t)j * nc + c] = dbr_chunk(m, col, y ? y + i0 : col);
    }
    free(tile);
  }
  for (int j = 0; j < s; ++j) out[j] = dbr_finish(nc, part + (int64_t)j * nc);
  free(part);
}

/* rows [i0, i0 + m) of block b, every column, filled by tiles in parallel (the sequential consumers stream them) */
static void rs_fill_rows(const ls_rsrc *src, int b, int s, int64_t i0, int64_t m, double *buf) {
  const int64_t nt = (m + ORC_DBR_CHUNK - 1) / ORC_DBR_CHUNK;
  ORC_PAR
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t a = t * ORC_DBR_CHUNK, e = a + ORC_DBR_CHUNK < m ? a + ORC_DBR_CHUNK : m;
    double *tile = (double *)malloc((size_t)((e - a) * s) * sizeof(double));
    rs_fill(src, b, i0 + a, i0 + e, 0, s, tile);
    for (int j = 0; j < s; ++j) memcpy(buf + (int64_t)j * m + a, tile + (int64_t)j * (e - a), (size_t)(e - a) * sizeof(double));
    free(tile);
  }
}

#define RS_BATCH ((int64_t)1 << 18) /* rows per batch of the sequential (SEQ-order) streams */

/* MatMultTranspose(R, u, out) */
static void rs_mult_transpose(const ls_layout *L, const ls_rsrc *src, const double *const *u, double *out) {
  if (src->R) {
    ls_mult_transpose(L, src->R, src->lda, u, out);
    return;
  }
  const int s = L->s;
  if (L->mode == ORC_REDUCE_SEQ) { /* one running sum per column over all rows, block 0's rows first */
    for (int j = 0; j < s; ++j) out[j] = 0.0;
    double *buf = (double *)malloc((size_t)(RS_BATCH * s) * sizeof(double));
    for (int b = 0; b < L->nblk; ++b)
      for (int64_t i0 = 0; i0 < L->n[b]; i0 += RS_BATCH) {
        const int64_t m = L->n[b] - i0 < RS_BATCH ? L->n[b] - i0 : RS_BATCH;
        rs_fill_rows(src, b, s, i0, m, buf);
        for (int j = 0; j < s; ++j) {
          double acc = out[j];
          const double *c = buf + (int64_t)j * m, *ub = u[b] + i0;
          for (int64_t i = 0; i < m; ++i) acc += c[i] * ub[i];
          out[j] = acc;
        }
      }
    free(buf);
    return;
  }
  double *d = (double *)malloc((size_t)s * sizeof(double));
  for (int j = 0; j < s; ++j) out[j] = 0.0;
  for (int b = 0; b < L->nblk; ++b) { /* ls_gdot: block sums added in block order from 0.0 */
    rs_dbr_block_dots(L, src, b, u[b], d);
    for (int j = 0; j < s; ++j) out[j] += d[j];
  }
  free(d);
}

/* The DBR one-pass step on an on-the-fly R (one formation of R per step instead of two): per DBR chunk of each
 * block, U1 = R V (orc_dense_mult's rows), U1 += -alpha U (ls_axpy), the chunk's U1.U1 partial and the chunk's
 * R_j.U1 partials; then per block the second stage of each, added over blocks in block order from 0.0 -- every
 * operation as rs_mult, ls_axpy, ls_gdot and rs_mult_transpose perform it, one chunk at a time. */
static void rs_onepass_step(const ls_layout *L, const ls_rsrc *src, const double *V, double alpha,
                            double *const *U, double *const *U1, double *beta_sq, double *RtU1) {
  const int s = L->s;
  double *d = (double *)malloc((size_t)(s + 1) * sizeof(double));
  double bsq = 0.0;
  for (int j = 0; j < s; ++j) RtU1[j] = 0.0;
  for (int b = 0; b < L->nblk; ++b) {
    const int64_t n = L->n[b], nc = (n + ORC_DBR_CHUNK - 1) / ORC_DBR_CHUNK;
    double *part = (double *)malloc((size_t)((nc > 0 ? nc : 1) * (s + 1)) * sizeof(double));
    ORC_PAR
    for (int64_t c = 0; c < nc; ++c) {
      const int64_t i0 = c * ORC_DBR_CHUNK, m = n - i0 < ORC_DBR_CHUNK ? n - i0 : ORC_DBR_CHUNK;
      double *tile = (double *)malloc((size_t)(m * s) * sizeof(double));
      rs_fill(src, b, i0, i0 + m, 0, s, tile);
      double *u1 = U1[b] + i0;
      orc_dense_mult(m, s, tile, m, V, u1);
      if (alpha != 0.0)
        for (int64_t i = 0; i < m; ++i) u1[i] = u1[i] + (-alpha) * U[b][i0 + i];
      part[(int64_t)s * nc + c] = dbr_chunk(m, u1, u1);
      for (int j = 0; j < s; ++j) part[(int64_t)j * nc + c] = dbr_chunk(m, tile + (int64_t)j * m, u1);
      free(tile);
    }
    for (int j = 0; j <= s; ++j) d[j] = dbr_finish(nc, part + (int64_t)j * nc);
    free(part);
    bsq += d[s];
    for (int j = 0; j < s; ++j) RtU1[j] += d[j];
  }
  *beta_sq = bsq;
  free(d);
}

/* MatNorm(R, NORM_FROBENIUS) in ls_frobenius' orders */
static double rs_frobenius(const ls_layout *L, const ls_rsrc *src) {
  if (src->R) return ls_frobenius(L, src->R, src->lda);
  const int s = L->s;
  double t = 0.0;
  if (L->mode == ORC_REDUCE_SEQ) { /* column-major: every row of column 0 (all blocks), then column 1, ... */
    double *buf = (double *)malloc((size_t)RS_BATCH * sizeof(double));
    for (int j = 0; j < s; ++j)
      for (int b = 0; b < L->nblk; ++b)
        for (int64_t i0 = 0; i0 < L->n[b]; i0 += RS_BATCH) {
          const int64_t m = L->n[b] - i0 < RS_BATCH ? L->n[b] - i0 : RS_BATCH;
          ls_rsrc one = *src;
          one.S = src->S + (int64_t)j * src->lds;
          rs_fill_rows(&one, b, 1, i0, m, buf);
          for (int64_t i = 0; i < m; ++i) t += buf[i] * buf[i];
        }
    free(buf);
    return sqrt(t);
  }
  double *d = (double *)malloc((size_t)s * sizeof(double));
  for (int b = 0; b < L->nblk; ++b) {
    rs_dbr_block_dots(L, src, b, NULL, d);
    double tb = 0.0;
    for (int j = 0; j < s; ++j) tb += d[j];
    t += tb;
  }
  free(d);
  return sqrt(t);
}

typedef struct {
  const orc_lsqr_opts *o;
  int reason, its, nhist, hist_cap;
  double rnorm0, ttol, arnorm, anorm;
  double *hist;
} ls_state;

/* KSPConvergedDefault (zero initial guess: rnorm0 = rnorm at n = 0), then for the
 * "lsqr" test KSPLSQRConvergedDefault's normal-equation checks. */
static void ls_converged(ls_state *k, int n, double rnorm) {
  k->reason = ORC_CONVERGED_ITERATING;
  if (k->o->conv_test == ORC_LSQR_CONV_SKIP) {
    if (n >= k->o->max_it) k->reason = ORC_CONVERGED_ITS;
    return;
  }
  if (n == 0) {
    k->rnorm0 = rnorm;
    k->ttol = PMAX(k->o->rtol * k->rnorm0, k->o->abstol);
  }
  if (is_bad(rnorm)) {
    k->reason = ORC_DIVERGED_NANORINF;
  } else if (rnorm <= k->ttol) {
    k->reason = (rnorm < k->o->abstol) ? ORC_CONVERGED_ATOL : ORC_CONVERGED_RTOL;
  } else if (rnorm >= k->o->divtol * k->rnorm0) {
    k->reason = ORC_DIVERGED_DTOL;
  }
  if (k->o->conv_test != ORC_LSQR_CONV_LSQR || n == 0 || k->reason) return;
  if (k->arnorm < k->o->abstol) k->reason = ORC_CONVERGED_ATOL_NORMAL;
  else if (k->arnorm < k->o->rtol * k->anorm * rnorm) k->reason = ORC_CONVERGED_RTOL_NORMAL;
}

static void ls_log(ls_state *k, double r) {
  if (k->hist && k->nhist < k->hist_cap) k->hist[k->nhist] = r;
  k->nhist++;
}

/* KSPSolve(outer_ksp, b, x) -> KSPSolve_LSQR [PETSc-ext] with PCNONE and a zero guess
 * (outer_solver_norm_equation, utils.c:1061-1078). */
static int lsqr_solve_src(int nblk, const int64_t *nrows, int s, const ls_rsrc *src, const double *const *rhs,
                          double *x, const orc_lsqr_opts *o, orc_lsqr_result *res, double *hist, int hist_cap) {
  if (nblk < 1 || s < 1 || !o) return ORC_ERR_ARG;
  ls_layout L = {nblk, s, o->reduce_mode, nrows};
  ls_state k;
  memset(&k, 0, sizeof(k));
  k.o = o;
  k.hist = hist;
  k.hist_cap = hist_cap;
  int64_t ntot = 0;
  for (int b = 0; b < nblk; ++b) ntot += nrows[b];
  double *ubuf = (double *)calloc((size_t)(2 * ntot + 2), sizeof(double));
  double *sbuf = (double *)calloc((size_t)(4 * s), sizeof(double));
  double **U = (double **)malloc((size_t)nblk * sizeof(double *));
  double **U1 = (double **)malloc((size_t)nblk * sizeof(double *));
  if (!ubuf || !sbuf || !U || !U1) {
    free(ubuf); free(sbuf); free(U); free(U1);
    return ORC_ERR_MEM;
  }
  int64_t off = 0;
  for (int b = 0; b < nblk; off += nrows[b], ++b) {
    U[b] = ubuf + off;
    U1[b] = ubuf + ntot + off;
  }
  double *V = sbuf, *V1 = sbuf + s, *W = sbuf + 2 * s;
  double rnorm = 0.0, beta, alpha;
  for (int j = 0; j < s; ++j) x[j] = 0.0; /* zero initial guess */

  /* u <- b (x is 0) */
  for (int b = 0; b < nblk; ++b) memcpy(U[b], rhs[b], (size_t)nrows[b] * sizeof(double));
  rnorm = sqrt(ls_gdot(&L, (const double *const *)U, (const double *const *)U));
  if (is_bad(rnorm)) { /* KSPCheckNorm */
    k.reason = ORC_DIVERGED_NANORINF;
    goto out;
  }
  k.its = 0;
  ls_log(&k, rnorm);
  ls_converged(&k, 0, rnorm);
  if (k.reason) goto out;

  beta = rnorm;
  for (int b = 0; b < nblk; ++b) ls_scale(nrows[b], U[b], 1.0 / beta);
  rs_mult_transpose(&L, src, (const double *const *)U, V);
  alpha = ls_snorm(s, V);
  ls_scale(s, V, 1.0 / alpha);
  memcpy(W, V, (size_t)s * sizeof(double));
  k.anorm = o->exact_norm ? rs_frobenius(&L, src) : 0.0;
  k.arnorm = alpha * beta;
  double phibar = beta, rhobar = alpha;
  int i = 0;
  do {
    /* DBR one-pass (the device's default): R^T U1 from the unscaled U1, in the pass that formed it */
    const int onepass = L.mode == ORC_REDUCE_DBR && o->onepass;
    if (onepass && !src->R) { /* an on-the-fly R: formed once for the whole step */
      double bsq;
      rs_onepass_step(&L, src, V, alpha, U, U1, &bsq, V1);
      beta = sqrt(bsq);
    } else {
      /* U1 = R V - alpha U */
      rs_mult(&L, src, V, U1);
      for (int b = 0; b < nblk; ++b) ls_axpy(nrows[b], U1[b], -alpha, U[b]);
      beta = sqrt(ls_gdot(&L, (const double *const *)U1, (const double *const *)U1));
      if (onepass) rs_mult_transpose(&L, src, (const double *const *)U1, V1);
    }
    if (is_bad(beta)) {
      k.reason = ORC_DIVERGED_NANORINF;
      break;
    }
    if (beta > 0.0) {
      for (int b = 0; b < nblk; ++b) ls_scale(nrows[b], U1[b], 1.0 / beta);
      if (!o->exact_norm) k.anorm = sqrt(k.anorm * k.anorm + alpha * alpha + beta * beta);
    }
    /* V1 = R^T U1 - beta V */
    if (onepass) {
      if (beta > 0.0) ls_scale(s, V1, 1.0 / beta); /* (R^T U1) * (1/beta) */
    } else {
      rs_mult_transpose(&L, src, (const double *const *)U1, V1);
    }
    ls_axpy(s, V1, -beta, V);
    alpha = ls_snorm(s, V1);
    if (is_bad(alpha)) {
      k.reason = ORC_DIVERGED_NANORINF;
      break;
    }
    ls_scale(s, V1, 1.0 / alpha);
    const double rho = sqrt(rhobar * rhobar + beta * beta);
    const double c = rhobar / rho;
    const double sn = beta / rho;
    const double theta = sn * alpha;
    rhobar = -c * alpha;
    const double phi = c * phibar;
    phibar = sn * phibar;
    const double tau = sn * phi;
    ls_axpy(s, x, phi / rho, W);        /* x <- x + (phi/rho) w */
    ls_aypx(s, W, -theta / rho, V1);    /* w <- v1 - (theta/rho) w */
    k.arnorm = alpha * fabs(tau);
    rnorm = phibar;
    k.its++;
    ls_log(&k, rnorm);
    ls_converged(&k, i + 1, rnorm);
    if (k.reason) break;
    double **t = U; U = U1; U1 = t;     /* SWAP(U1, U), SWAP(V1, V) */
    double *tv = V; V = V1; V1 = tv;
    i++;
  } while (i < o->max_it);
  if (i >= o->max_it && !k.reason) k.reason = ORC_DIVERGED_ITS;
out:
  if (res) {
    res->its = k.its;
    res->reason = k.reason;
    res->rnorm = rnorm;
    res->arnorm = k.arnorm;
    res->anorm = k.anorm;
    res->nhist = k.nhist;
  }
  free(ubuf); free(sbuf);
  free(U);
  free(U1);
  return ORC_OK;
}

int orc_lsqr_solve(int nblk, const int64_t *nrows, int s, const double *const *R, const int64_t *lda,
                   const double *const *rhs, double *x, const orc_lsqr_opts *o, orc_lsqr_result *res,
                   double *hist, int hist_cap) {
  const ls_rsrc src = {R, lda, NULL, NULL, 0};
  return lsqr_solve_src(nblk, nrows, s, &src, rhs, x, o, res, hist, hist_cap);
}

/* Synchronous multisplitting with synchronous global minimization (SMSM-global),
 * src/synchronous-multisplitting-synchronous-minimization-global/
 * synchronous-multisplitting-synchronous-minimization-global.c, setup :134-284,
 * loop :288-363, generalised to nb blocks:
 *   s times: rhs_i = b_i - A_ij x_j (updateLocalRHS, utils.c:943), inner GMRES
 *            (inner_solver, utils.c:950), exchange, S(:, k) = x           (:295-319)
 *   R = A S (MatMatMult of the block rows with S, PETSc AIJ x DENSE:
 *            per row, columns ascending, from 0)                           (:325-327)
 *   alpha = LSQR(R, b), x = S alpha (outer_solver_norm_equation)           (:331-333)
 *   stop when the LSQR residual norm <= max(atol, rtol * ||b||)            (:342-347)
 *   every block takes x = S alpha (scatter of x_minimized)                 (:349-352) */
int orc_smsm_solve(const orc_smsm_problem *p, const orc_gmres_opts *inner, const orc_lsqr_opts *outer,
                   orc_smsm_result *res, double *outer_hist, int outer_cap, int *lsqr_its,
                   int *lsqr_reason, int *inner_its, double *x_out) {
  const int nb = p->nb, s = p->s, lean = p->lean != 0;
  if (nb < 1 || s < 1 || (p->dim != 2 && p->dim != 3) || (lean && (p->dim != 3 || s > ORC_RS_MAXS))) return ORC_ERR_ARG;
  if (p->dim == 3 && p->nz % nb) return ORC_ERR_ARG;
  if (p->dim == 2 && ((int64_t)p->nx * p->ny) % nb) return ORC_ERR_ARG;
  orc_sm_problem sp = {p->dim, p->nx, p->ny, p->nz, nb, p->rtol, p->atol, p->max_outer,
                       {p->peclet[0], p->peclet[1], p->peclet[2]}};
  const int64_t N = (int64_t)p->nx * p->ny * (p->dim == 3 ? p->nz : 1);
  const int mode = inner->reduce_mode;
  const int progress = getenv("ORC_PROGRESS") != NULL; /* one stderr line per outer iteration (long records) */
  orc_csr *Ab = (orc_csr *)calloc((size_t)nb, sizeof(orc_csr));
  orc_csr *Aii = (orc_csr *)calloc((size_t)nb, sizeof(orc_csr));
  orc_csr *Aoff = (orc_csr *)calloc((size_t)nb, sizeof(orc_csr));
  orc_op *Abo = (orc_op *)calloc((size_t)nb, sizeof(orc_op));
  orc_op *Aiio = (orc_op *)calloc((size_t)nb, sizeof(orc_op));
  orc_op *Aoffo = (orc_op *)calloc((size_t)nb, sizeof(orc_op));
  int64_t *r0 = (int64_t *)calloc((size_t)nb, sizeof(int64_t));
  int64_t *r1 = (int64_t *)calloc((size_t)nb, sizeof(int64_t));
  int64_t *nrow = (int64_t *)calloc((size_t)nb, sizeof(int64_t));
  int64_t *ldab = (int64_t *)calloc((size_t)nb, sizeof(int64_t));
  double *x = (double *)calloc((size_t)N, sizeof(double));
  double *u = (double *)malloc((size_t)N * sizeof(double));
  double *bvec = (double *)calloc((size_t)N, sizeof(double));
  double *rhs = (double *)calloc((size_t)N, sizeof(double));
  double *y = (double *)calloc((size_t)N, sizeof(double));
  double *S = (double *)calloc((size_t)(N * s), sizeof(double));
  double *Rm = lean ? NULL : (double *)calloc((size_t)(N * s), sizeof(double));
  double *alpha = (double *)calloc((size_t)s, sizeof(double));
  const double **bbp = (const double **)calloc((size_t)nb, sizeof(double *));
  const double **Rp = (const double **)calloc((size_t)nb, sizeof(double *));
  int rc = ORC_OK;
  if (!Ab || !Aii || !Aoff || !Abo || !Aiio || !Aoffo || !r0 || !r1 || !nrow || !ldab || !x || !u || !bvec ||
      !rhs || !y || !S || (!lean && !Rm) || !alpha || !bbp || !Rp) {
    rc = ORC_ERR_MEM;
    goto done;
  }
  for (int64_t i = 0; i < N; ++i) u[i] = 1.0;
  for (int b = 0; b < nb; ++b) {
    if (lean) {
      const int64_t ppb = p->nz / nb, nxny = (int64_t)p->nx * p->ny;
      r0[b] = b * ppb * nxny;
      r1[b] = (b + 1) * ppb * nxny;
      Abo[b] = op_stencil(p->nx, p->ny, p->nz, r0[b], r1[b], p->peclet, OP_BLOCK);
      Aiio[b] = op_stencil(p->nx, p->ny, p->nz, r0[b], r1[b], p->peclet, OP_DIAG);
      Aoffo[b] = op_stencil(p->nx, p->ny, p->nz, r0[b], r1[b], p->peclet, OP_OFF);
    } else {
      if ((rc = build_block(&sp, b, &Ab[b], &r0[b], &r1[b]))) goto done;
      if ((rc = orc_split(&Ab[b], r0[b], r1[b], &Aii[b], &Aoff[b]))) goto done;
      Abo[b] = op_csr(&Ab[b]);
      Aiio[b] = op_csr(&Aii[b]);
      Aoffo[b] = op_csr(&Aoff[b]);
    }
    op_spmv(&Abo[b], u, bvec + r0[b]); /* computeTheRightHandSideWithInitialGuess */
    bbp[b] = bvec + r0[b];
    Rp[b] = lean ? NULL : Rm + r0[b];
    nrow[b] = r1[b] - r0[b];
    ldab[b] = N;
  }
  const double norm0 = final_residual_norm_op(mode, nb, Abo, x, bbp); /* :280 */
  orc_gmres_opts io = *inner;
  io.guess_nonzero = 1;
  io.uirnorm = 1;
  int outer_it = 0;
  int64_t total_inner = 0;
  const ls_rsrc src = {lean ? NULL : Rp, lean ? NULL : ldab, Abo, S, N};
  for (;;) {
    for (int k = 0; k < s; ++k) {
      for (int b = 0; b < nb; ++b) op_residual(&Aoffo[b], bvec + r0[b], x, rhs + r0[b]);
      for (int b = 0; b < nb; ++b) {
        orc_gmres_result gr;
        if ((rc = gmres_solve_op(&Aiio[b], rhs + r0[b], x + r0[b], &io, &gr, NULL, 0))) goto done;
        if (inner_its && outer_it < outer_cap) inner_its[((int64_t)outer_it * s + k) * nb + b] = gr.its;
        total_inner += gr.its;
      }
      memcpy(S + (int64_t)k * N, x, (size_t)N * sizeof(double)); /* MatSetValuesLocal(S, .., k, x) */
    }
    if (!lean)
      for (int b = 0; b < nb; ++b)
        for (int k = 0; k < s; ++k) orc_spmv(&Ab[b], S + (int64_t)k * N, Rm + (int64_t)k * N + r0[b]);
    orc_lsqr_result lr;
    if ((rc = lsqr_solve_src(nb, nrow, s, &src, bbp, alpha, outer, &lr, NULL, 0))) goto done;
    orc_dense_mult(N, s, S, N, alpha, x); /* x_minimized = S alpha */
    const double norm = lr.rnorm;         /* KSPGetResidualNorm(outer_ksp) */
    if (outer_it < outer_cap) {
      if (outer_hist) outer_hist[outer_it] = norm;
      if (lsqr_its) lsqr_its[outer_it] = lr.its;
      if (lsqr_reason) lsqr_reason[outer_it] = lr.reason;
    }
    if (progress) {
      fprintf(stderr, "orc_smsm_solve: outer %d lsqr_rnorm %a (%.17g) lsqr_its %d reason %d inner_total %lld\n",
              outer_it, norm, norm, lr.its, lr.reason, (long long)total_inner);
      fflush(stderr);
    }
    outer_it++;
    if (norm <= PMAX(p->atol, p->rtol * norm0)) break;
    if (p->max_outer > 0 && outer_it >= p->max_outer) break;
  }
  if (res) {
    res->outer_its = outer_it;
    res->norm0 = norm0;
    res->final_norm = final_residual_norm_op(mode, nb, Abo, x, bbp);
    for (int64_t i = 0; i < N; ++i) y[i] = -1.0 * u[i] + x[i];
    res->error = orc_norm2(mode, N, y);
    res->total_inner_its = total_inner;
  }
  if (x_out) memcpy(x_out, x, (size_t)N * sizeof(double));
done:
  if (Ab && !lean)
    for (int b = 0; b < nb; ++b) { orc_csr_free(&Ab[b]); orc_csr_free(&Aii[b]); orc_csr_free(&Aoff[b]); }
  free(Ab); free(Aii); free(Aoff); free(Abo); free(Aiio); free(Aoffo); free(r0); free(r1); free(nrow); free(ldab);
  free(x); free(u); free(bvec); free(rhs); free(y); free(S); free(Rm); free(alpha); free(bbp); free(Rp);
  return rc;
}
