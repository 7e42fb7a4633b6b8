// msplit_kernels.h -- launcher declarations shared by the .hip files (C++/HIP side only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#define MSK_MAX_GROUP 32
#define MSK_DBR_CHUNK 4096

enum { MSK_SET = 0, MSK_COPY, MSK_SCALE, MSK_AXPY, MSK_AYPX, MSK_WAXPY_P1, MSK_WAXPY_M1, MSK_WAXPY };

// A set of vectors: an explicit table (up to 32), or a strided basis
// V_j = base + j*stride (any count) when base != nullptr.  scale != nullptr:
// vector j is stored unnormalised and its value is V_j[i] * scale[j] (device
// array), the rounding VecScale would have stored -- a deferred VecNormalize.
struct Vecs {
  const double* p[MSK_MAX_GROUP];
  const double* base;
  int64_t stride;
  const double* scale;
};
struct Coefs {
  double a[MSK_MAX_GROUP];
};
// W = A (sc * x) computed where it is consumed (the GMRES step's MatMult fused
// into the CGS kernels): A in DV storage, ELL layout with 8 codes per row.
struct EllOp {
  const uint8_t* code8;   // nrows * 8 codes (+16 pad)
  const int32_t* ddelta;  // dictionary: col - row
  const double* dval;     //             value
  int ndict;              // <= 255
  const double* x;        // VV(it), stored unnormalised
  const double* sdev;     // its scale sc[it] (device)
};
// constant 7-point stencil values: slow-, y-, x-, diagonal, x+, y+, slow+
struct BoxCoef {
  double c[7];
};

// SpMV modes
enum { MSK_SPMV_MULT = 0, MSK_SPMV_RESID = 1, MSK_SPMV_SCALED = 2 };

// tuning flags
enum {
  MSK_TUNE_MDOT_REV = 1,
  MSK_TUNE_SPMV_TEMPORAL = 2,       // CSR SpMV: default-policy col/val loads and y stores (default: non-temporal)
  MSK_TUNE_SPMV_XCD = 4,
  MSK_TUNE_SPMV_STAGE1 = 8,         // CSR SpMV: register staging, one slice per lane at a time
  MSK_TUNE_VEC_TEMPORAL = 16,       // default-policy (not non-temporal) basis loads in MDot / MAXPY / dense
  MSK_TUNE_MAXPY_TEMPORAL_ST = 64,  // default-policy store of w in MAXPY
  MSK_TUNE_GM_UNFUSED = 128,        // separate ||w||^2 stage-2 and one-lane Hessenberg update launches
  MSK_TUNE_MAXPY_HALVES = 256,      // MAXPY: each chunk in two halves (fewer registers, more waves)
  MSK_TUNE_SPMV_ZCHUNK = 512,       // SpMV: XCD x takes the x-th eighth of the row blocks, in order
  MSK_TUNE_MDOT_SINGLE = 1024,      // MDot: one vector's loads at a time (before grouped loads)
  MSK_TUNE_GM_SPMV_MDOT = 2048,     // GMRES: MatMult fused with the VecMDot that follows (k_spmv_mdot)
  MSK_TUNE_SPMV_MDOT_G2 = 4096,     // k_spmv_mdot: two basis vectors per load group instead of four
  MSK_TUNE_DV_RPL1 = 8192,          // DV SpMV: one row per lane (256-row blocks)
  MSK_TUNE_DV_RPL2 = 16384,         // DV SpMV: two rows per lane (512-row blocks); default four
  MSK_TUNE_DV_NOELL = 32768,        // DV storage: CSR-order codes even where the ELL layout fits (at assembly)
  MSK_TUNE_GM_OPFUSE = 65536,       // GMRES: W = A (sc x) computed inside MDot and MAXPY instead of a MatMult kernel
  MSK_TUNE_MAXPY_UNROLL1 = 131072,  // MAXPY: one group of four per loop iteration (default: two, unrolled)
  MSK_TUNE_MDOT_UNROLL2 = 262144,   // MDot: two groups of four per loop iteration
  MSK_TUNE_ELL_TEMPORAL_Y = 1048576, // DV SpMV: default-policy y stores (default: non-temporal)
  MSK_TUNE_SPMV_NTY = 2097152,      // CSR SpMV: default-policy col/val loads, non-temporal y stores
  MSK_TUNE_SPMV_REG_STAGE = 4194304, // CSR SpMV: col/val staged through registers, 4 val + 2 col slices per lane
                                     // (round-1 form; default: LDS-DMA, global_load_lds_dwordx4)
  MSK_TUNE_DENSE_G1 = 8388608,      // LSQR dense kernels: one column per load group (round-1 kernels; default four)
  MSK_TUNE_DENSE_G2 = 16777216,     // LSQR dense kernels: two columns per load group
  MSK_TUNE_DENSE_TEMPORAL_ST = 33554432, // LSQR dense kernels: default-policy u / u/beta stores (default: non-temporal)
  MSK_TUNE_ELL_XCD_ON = 67108864,   // DV (ELL) SpMV: XCD-contiguous block order at any plane size
  MSK_TUNE_ELL_XCD_OFF = 134217728, // DV (ELL) SpMV: identity block order at any plane size (default: XCD order
                                    // from 2^18 rows per plane)
  MSK_TUNE_ELL_MARCH_OFF = 268435456, // box-stencil DV SpMV: the row-parallel ELL kernel (default: the z-march
                                      // kernel for every 3D box stencil with lo = hi = 0)
  MSK_TUNE_ELL_MARCH_NOXCD = 536870912, // z-march kernel: identity block order (default: XCD-contiguous runs)
  MSK_TUNE_GM_BOX_MDOT_OFF = 1073741824, // GMRES on a box stencil: separate MatMult and VecMDot kernels (default:
                                         // fused, k_box_spmv_mdot[_march]: W not re-read, +2.6-2.8 % per step)
  MSK_TUNE_BOX_MDOT_NOXCD = 524288, // k_box_spmv_mdot_march: tiles in plane order (default: XCD-contiguous eighths)
  MSK_TUNE_BOX_MDOT_FLAT = 32  // k_box_spmv_mdot: one plane per workgroup even where planes hold whole chunks (no z-march)
};

extern "C" {
void msk_set_tuning(int flags);
int msk_get_tuning(void);
void msk_set_spmv_group(int gb);
void msk_set_march_z(int z);  // z-march planes per workgroup (0: auto; A/B experiments)
void msk_set_march_lines(int l);  // z-march tile: 1 = 256 plane rows, 4 = four y lines, 16 = DBR chunk tiles (0: auto; A/B, tests)
// The CGS block with W = A (sc x) computed in the kernel (op) instead of read from w: stage 1 of
// W . V_v (v < nv <= 32), and the MAXPY wout = W - sum_j adev_j V_j with the ||wout||^2 partials.
int msk_dot_stage1_op(const EllOp* op, const Vecs* V, int nv, int64_t n, double* partial, int64_t nchunks,
                      const int* stop, hipStream_t s);
int msk_maxpy_op(const EllOp* op, double* wout, const Vecs* V, int nv, const double* adev, int64_t n,
                 double* partial, const int* stop, hipStream_t s);
// DBR stage 1 over nv <= 32 vectors (self: ||w||^2).  stop: device flag, skip when set (may be null).
int msk_dot_stage1(const double* w, const Vecs* V, int nv, int64_t n, double* partial, int64_t nchunks, int self,
                   const int* stop, hipStream_t s);
int msk_dot_stage2(const double* partial, int64_t nchunks, int nv, double* out, const int* stop, hipStream_t s);
// MSP_REDUCE_SEQ stage 1 (msplit_seq.hip): w . V_v (self: w . w) as one sequential sum per vector, written in
// the DBR partial layout (chunk 0 holds the sum, the others +0.0) so stage 2 folds it unchanged.
int msk_seq_stage1(const double* w, const Vecs* V, int nv, int64_t n, int self, double* partial, int64_t nchunks,
                   const int* stop, hipStream_t s);
// wout = win + sum_j a_j V_j (PETSc grouping), a_j = (negate ? -1 : 1) * (adev ? adev[j] : A->a[j]);
// nv = *nvdev when nvdev != null; accum: wout = win + (0 + sum); partial != null: DBR partial of ||wout||^2.
int msk_maxpy_chunk(const double* win, double* wout, const Vecs* V, int nv, const int* nvdev, const Coefs* A,
                    const double* adev, int negate, int64_t n, int accum, double* partial, const int* stop,
                    hipStream_t s);
// mode MULT: y = A x; RESID: y = b - A x; SCALED: sc = *sdev, y = A (sc*x) and, when vout != null, vout = sc*x.
// plane > 0: the operator is a stencil with this many rows per plane (XCD-aware schedule, MSK_TUNE_SPMV_XCD)
int msk_spmv(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* x,
             const double* b, double* y, int32_t lds_cap, int mode, const double* sdev, double* vout,
             const int* stop, int64_t plane, hipStream_t s);
// The same products over DV storage (len8: entries per row <= 255; code8: one byte per entry naming the
// (col - row, value) pair ddelta/dval[code]; rowptr read only at block starts); max_block: most entries in
// any 256-row block (sizes the LDS stage of the codes).  ell_w = 4, 8 or 16: ELL layout instead (row r's
// codes at code8 + r*ell_w, padded with code 255; rowptr, len8 and max_block unused; ndict <= 255).
int msk_spmv_dv(int32_t nrows, const int32_t* rowptr, const uint8_t* len8, const uint8_t* code8,
                const int32_t* ddelta, const double* dval, int ndict, int32_t max_block, int ell_w,
                const double* x, const double* b, double* y, int mode, const double* sdev, double* vout,
                const int* stop, int64_t plane, hipStream_t s);
// The same products for a 3D box stencil in the ELL layout with 8 codes per row whose dictionary is
// exactly the seven stencil pairs in column order (-nx*ny, -nx, -1, 0, +1, +nx, +nx*ny), lo = hi = 0:
// a z-marching kernel without gathers.  msk_box_march_pick: 1 when the tuning policy takes it for this
// box (default: always).
int msk_box_march_pick(int32_t nx, int32_t ny, int32_t nz);
// d2 = 1: a 2D box stencil (five pairs -nx, -1, 0, +1, +nx) passed as nx x 1 x ny.  mask: one presence
// byte per row (msk_march_mask: bit e = neighbour e of (-P, -nx, -1, 0, +1, +nx, +P)), read instead of the codes.
int msk_march_mask(int32_t nrows, int d2, const uint8_t* code8, uint8_t* mask, hipStream_t s);
// *fail (device) set when a row's presence byte names a neighbour across a line or plane edge of the
// nx x ny (x nz) box (the march kernels would read it as 0.0): such a matrix must keep the ELL kernel.
int msk_march_check(int32_t nrows, int32_t nx, int32_t ny, int d2, const uint8_t* mask, int* fail, hipStream_t s);
int msk_spmv_box_march(int32_t nx, int32_t ny, int32_t nz, int d2, const uint8_t* mask, const double* dval,
                       const double* x, const double* b, double* y, int mode, const double* sdev, double* vout,
                       const int* stop, hipStream_t s);
// The chunk-tile march (k_box_march_chunk): whether it takes a box of nx x ny planes; MatMult / MatResidual
// with the plane below (halo & 1) / above (halo & 2) in the column space (x = the column-space vector).
int msk_march_chunk_fits(int32_t nx, int32_t ny, int d2);
int msk_box_march_halo_fits(int32_t nx, int32_t ny, int32_t nz, int halo, const double *x, const double *b,
                            const double *y, int mode);
int msk_box_march_halo(int32_t nx, int32_t ny, int32_t nz, int halo, const uint8_t* mask, const double* dval,
                       const double* x, const double* b, double* y, int mode, hipStream_t s);
// GMRES: y = A (sc*x) for a box stencil with march presence bytes (nx <= 2048; P = the plane, or nx in 2D), fused
// with the DBR stage 1 of y . V_v (v < nv <= 32) into partial: W in the DBR lane layout, bitwise the march's.
// *self_out (may be NULL) = 1 when V's last vector is x and its dot came from the march's registers (not re-read).
// The stencil storage (a box stencil whose rows carry their own seven values, rv[e * rvs + row], e in column
// order): the chunk-tile march products, and the GMRES MatMult fused with VecMDot stage 1 (W stored).
int msk_box_march_chunk_rv(int32_t nx, int32_t ny, int32_t nz, const uint8_t* mask, const double* rv, int64_t rvs,
                           const double* x, const double* b, double* y, int mode, const double* sdev, double* vout,
                           const int* stop, hipStream_t s);
int msk_box_spmv_mdot_rv(int32_t nx, int64_t P, int64_t n, int d2, const uint8_t* mask, const double* dval,
                         const double* rv, int64_t rvs, const double* x, const double* sdev, double* y, const Vecs* V,
                         int nv, double* partial, int64_t nchunks, const int* stop, int* self_out, hipStream_t s);
int msk_box_spmv_mdot(int32_t nx, int64_t P, int64_t n, int d2, const uint8_t* mask, const double* dval,
                      const double* x, const double* sdev, double* y, const Vecs* V, int nv, double* partial,
                      int64_t nchunks, const int* stop, int* self_out, hipStream_t s);
// The W-free GMRES step: msk_box_spmv_mdot with y = null (W not stored), then msk_box_maxpy_march, which
// recomputes W for its rows on the same march tiles (bitwise) and runs the CGS VecMAXPY wout = W - sum_j adev_j
// VV(j) with the DBR partials of ||wout||^2 (k_maxpy_chunk's arithmetic; V's last vector must be x).
// msk_box_wfree_fits: 1 when msk_box_spmv_mdot takes the box and the W-free step is on (msk_set_gm_wfree); the
// MAXPY marches where the fused kernel does (planes of whole DBR chunks), else it takes one chunk per workgroup.
void msk_set_gm_wfree(int on);
int msk_get_gm_wfree(void);
int msk_box_wfree_fits(int32_t nx, int64_t P, int64_t n, int d2);
int msk_box_maxpy_march(int32_t nx, int64_t P, int64_t n, int d2, const uint8_t* mask, const double* dval, const double* x,
                        const double* sdev, double* wout, const Vecs* V, int nv, const double* adev, double* partial,
                        const int* stop, hipStream_t s);
// R[:, 0:nc] = A S[:, 0:nc] over DV storage in the ELL layout (W codes per row)
int msk_spmm_ell(int32_t nrows, int W, const uint8_t* code8, const int32_t* ddelta, const double* dval, int ndict,
                 const double* S, int64_t lds, int nc, double* R, int64_t ldr, hipStream_t s);
int msk_ell_encode(int32_t nrows, int W, const int32_t* rowptr, const int32_t* col, const double* val, int ndict,
                   const int32_t* ddelta, const double* dval, uint8_t* code8, int* fail, hipStream_t s);
// DV codes of an assembled CSR against a dictionary; *fail (device) set when it does not fit
int msk_dv_encode(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, int ndict,
                  const int32_t* ddelta, const double* dval, uint8_t* len8, uint8_t* code8, int* fail,
                  hipStream_t s);
// GMRES: y = A (sc*x), sc = *sdev, fused with the DBR stage 1 of y . V_v (v < nv <= 32) into partial;
// lds_cap: LDS entries for the col/val slice of any 512-row sub-block (> 0)
int msk_spmv_mdot(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* x,
                  const double* sdev, double* y, int32_t lds_cap, const Vecs* V, int nv, double* partial,
                  int64_t nchunks, const int* stop, hipStream_t s);
// R[:, 0:nc] = A S[:, 0:nc], column-major S (lds) and R (ldr); needs lds_cap > 0
int msk_spmm(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* S,
             int64_t lds, int nc, double* R, int64_t ldr, int32_t lds_cap, hipStream_t s);
int msk_spmv_rows(int32_t nlisted, const int32_t* row_ids, const int32_t* rowptr, const int32_t* col,
                  const double* val, const double* x, const double* b, double* y, int resid, hipStream_t s);
// lo/hi: extra coupling columns to the neighbour plane below/above (column space [lo | block | hi])
// matrix-free y = A x / b - A x / scaled form for the box stencil (bitwise the CSR SpMV of its assembly)
int msk_stencil_spmv(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows, int lo, int hi, const BoxCoef* cf,
                     const double* x, const double* b, double* y, int mode, const double* sdev, double* vout,
                     const int* stop, hipStream_t s);
int msk_box_stencil(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows, int lo, int hi, const BoxCoef* cf,
                    int32_t* rowptr, int32_t* col, double* val, hipStream_t s);
int msk_blas1(int op, double* y, const double* x, const double* z, double alpha, int64_t n, hipStream_t s);
}
