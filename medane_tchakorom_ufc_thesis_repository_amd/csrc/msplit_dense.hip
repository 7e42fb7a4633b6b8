// msplit_dense.hip -- dense row blocks (MATDENSE) and the tall-skinny kernels of
// the global-minimization step: R = A S (SpMM), the LSQR products R v and R^T u,
// and x = S alpha.
//
// All of it is HBM-bound f64 streaming: a dense block is column-major with
// lda a multiple of 512 doubles, so every column starts 4 KiB aligned and a
// DBR chunk (4096 rows) of a column is 32 KiB contiguous.  The kernels use the
// same chunk geometry as the GMRES path (lane t owns rows base + j*512 + 2t,
// +1), so their reductions are the DBR order of oracle/oracle.c (dbr_dot) and
// the per-row sums are the reference's dgemv/MatMatMult orders: per row,
// columns (or CSR entries) in order, starting from 0, no FMA contraction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "msplit_ctx.hpp"

namespace msd {

constexpr int kT = 256;
constexpr int kIters = 8;
constexpr int kChunk = kT * 2 * kIters;
constexpr int kMaxCols = 32;  // columns per dot launch (shared reduction slots)
static_assert(kChunk == MSK_DBR_CHUNK, "DBR chunk must match the oracle");

__device__ __forceinline__ bool stopped(const int* stop) { return stop && *stop; }

// Column loads: VEC 0 = scalar (unaligned / ragged), 1 = 16-byte default policy,
// 2 = 16-byte non-temporal (the default: the columns of S and R stream through
// once per launch and dwarf the MALL; msplit_kernels.hip, MSK_TUNE_VEC_TEMPORAL).
typedef double dx2 __attribute__((ext_vector_type(2)));
template <int VEC>
__device__ __forceinline__ double2 ld_col(const double* p) {
  if constexpr (VEC == 2) {
    const dx2 v = __builtin_nontemporal_load(reinterpret_cast<const dx2*>(p));
    return make_double2(v.x, v.y);
  } else {
    return *reinterpret_cast<const double2*>(p);
  }
}

// y/wout stores: NT (template, never a run-time bool: the optimizer merges the two
// stores of "if (nt) nontemporal_store else store" into one plain store) -- the
// vectors u and u/beta of an LSQR step stream through once per launch and exceed
// the MALL from ~32 M rows on (msplit_kernels.hip, st_pol).
template <bool NT>
__device__ __forceinline__ void st2(double* p, double a, double b) {
  if constexpr (NT) {
    dx2 o;
    o.x = a;
    o.y = b;
    __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(p));
  } else {
    *reinterpret_cast<double2*>(p) = make_double2(a, b);
  }
}

__device__ __forceinline__ double wave_butterfly(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
  return v;
}

// ------------------------------------------------------------------ gemv
// y = A[:, 0:nc] coef (+ nal * U, VecAXPY skipped when nal == 0), per row
// ((0 + c0 a0) + c1 a1) + ...; NORM: the DBR partial of ||y||^2 of this chunk.
// G columns per load group (FULL chunks): G x kIters 16-byte loads per lane issued
// together before their products are added; every u[j] still takes the columns in
// order q = 0, 1, ... (the dgemv order), so the result does not depend on G.
template <bool AXPY, bool NORM, bool FULL, int VEC, int G, bool NTS>
__device__ __forceinline__ void gemv_body(const double* __restrict__ A, int64_t lda, int nc,
                                          const double* __restrict__ coef, double nal, const double* __restrict__ U,
                                          double usc, double* __restrict__ y, int64_t base, int64_t n, double& sq) {
  double u[2 * kIters];
#pragma unroll
  for (int j = 0; j < 2 * kIters; ++j) u[j] = 0.0;
  int q0 = 0;
  if constexpr (FULL && G > 1) {
#pragma unroll 1
    for (; q0 + G <= nc; q0 += G) {
      double a[G];
      double2 p[G][kIters];
#pragma unroll
      for (int g = 0; g < G; ++g) a[g] = coef[q0 + g];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const double* __restrict__ col = A + (int64_t)(q0 + g) * lda;
#pragma unroll
        for (int j = 0; j < kIters; ++j) p[g][j] = ld_col<VEC>(col + base + j * (2 * kT));
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          u[2 * j] = u[2 * j] + a[g] * p[g][j].x;
          u[2 * j + 1] = u[2 * j + 1] + a[g] * p[g][j].y;
        }
      }
    }
  }
#pragma unroll 1
  for (int q = q0; q < nc; ++q) {
    const double a = coef[q];  // wave-uniform scalar load
    const double* __restrict__ col = A + (int64_t)q * lda;
    double p[2 * kIters];
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const int64_t e = base + j * (2 * kT);
      if (FULL) {
        const double2 v = ld_col<VEC>(col + e);
        p[2 * j] = v.x;
        p[2 * j + 1] = v.y;
      } else {
        p[2 * j] = e < n ? col[e] : 0.0;
        p[2 * j + 1] = e + 1 < n ? col[e + 1] : 0.0;
      }
    }
#pragma unroll
    for (int j = 0; j < 2 * kIters; ++j) u[j] = u[j] + a * p[j];
  }
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    const int64_t e = base + j * (2 * kT);
    double r0 = u[2 * j], r1 = u[2 * j + 1];
    if (FULL) {
      if (AXPY && nal != 0.0) {  // U stored unscaled: its value is U * usc, the rounding VecScale stored
        const double2 q = *reinterpret_cast<const double2*>(U + e);
        r0 = r0 + nal * (q.x * usc);
        r1 = r1 + nal * (q.y * usc);
      }
      st2<NTS>(y + e, r0, r1);
      if (NORM) {
        acc = acc + r0 * r0;
        acc = acc + r1 * r1;
      }
    } else {
      if (e < n) {
        if (AXPY && nal != 0.0) r0 = r0 + nal * (U[e] * usc);
        y[e] = r0;
        if (NORM) acc = acc + r0 * r0;
      }
      if (e + 1 < n) {
        if (AXPY && nal != 0.0) r1 = r1 + nal * (U[e + 1] * usc);
        y[e + 1] = r1;
        if (NORM) acc = acc + r1 * r1;
      }
    }
  }
  sq = acc;
}

template <bool AXPY, bool NORM, int VEC, int G, bool NTS>
__global__ __launch_bounds__(kT) void k_dense_gemv(const double* __restrict__ A, int64_t lda, int nc,
                                                   const double* __restrict__ coef, const double* __restrict__ naldev,
                                                   const double* __restrict__ U, const double* __restrict__ uscdev,
                                                   double* __restrict__ y, int64_t n,
                                                   double* __restrict__ partial, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  const double nal = AXPY ? *naldev : 0.0;
  const double usc = uscdev ? *uscdev : 1.0;  // x * 1.0 == x: no scale leaves U as stored
  double sq = 0.0;
  if (VEC && (c + 1) * kChunk <= n)
    gemv_body<AXPY, NORM, true, VEC, G, NTS>(A, lda, nc, coef, nal, U, usc, y, base, n, sq);
  else gemv_body<AXPY, NORM, false, VEC, 1, NTS>(A, lda, nc, coef, nal, U, usc, y, base, n, sq);
  if (NORM) {
    __shared__ double red[4];
    sq = wave_butterfly(sq);
    if ((t & 63) == 0) red[t >> 6] = sq;
    __syncthreads();
    if (t == 0) partial[c] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

// ------------------------------------------------------- scaled column dots
// w' = w * (*sc) (VecScale, written back to wout) when SCALE, then the DBR
// stage-1 partials of column_v . w' for v < nc: partial[v*nchunks + c].
template <bool SCALE, int VEC, int G, bool NTS>
__global__ __launch_bounds__(kT) void k_scaled_dot(const double* win, double* wout, const double* __restrict__ scdev,
                                                   const double* __restrict__ A, int64_t lda, int nc, int64_t n,
                                                   double* __restrict__ partial, int64_t nchunks,
                                                   const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double red[kMaxCols][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t c = blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  const bool full = VEC && (c + 1) * kChunk <= n;
  const double sc = SCALE ? *scdev : 1.0;
  double wr[2 * kIters];
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    const int64_t e = base + j * (2 * kT);
    if (full) {
      const double2 q = *reinterpret_cast<const double2*>(win + e);
      wr[2 * j] = q.x;
      wr[2 * j + 1] = q.y;
    } else {
      wr[2 * j] = e < n ? win[e] : 0.0;
      wr[2 * j + 1] = e + 1 < n ? win[e + 1] : 0.0;
    }
    if (SCALE) {
      wr[2 * j] = wr[2 * j] * sc;
      wr[2 * j + 1] = wr[2 * j + 1] * sc;
      if (!wout) {  // deferred VecScale: the scaled values are only dotted, the next reader rescales
      } else if (full) {
        st2<NTS>(wout + e, wr[2 * j], wr[2 * j + 1]);
      } else {
        if (e < n) wout[e] = wr[2 * j];
        if (e + 1 < n) wout[e + 1] = wr[2 * j + 1];
      }
    }
  }
  int v0 = 0;
  if constexpr (G > 1) {
    if (full) {  // G columns' loads together, then G independent sums and butterflies
#pragma unroll 1
      for (; v0 + G <= nc; v0 += G) {
        double2 q[G][kIters];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const double* __restrict__ col = A + (int64_t)(v0 + g) * lda;
#pragma unroll
          for (int j = 0; j < kIters; ++j) q[g][j] = ld_col<VEC>(col + base + j * (2 * kT));
        }
        double acc[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          acc[g] = 0.0;
#pragma unroll
          for (int j = 0; j < kIters; ++j) {
            acc[g] = acc[g] + wr[2 * j] * q[g][j].x;
            acc[g] = acc[g] + wr[2 * j + 1] * q[g][j].y;
          }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const double r = wave_butterfly(acc[g]);
          if (lane == 0) red[v0 + g][wv] = r;
        }
      }
    }
  }
#pragma unroll 1
  for (int v = v0; v < nc; ++v) {
    const double* __restrict__ col = A + (int64_t)v * lda;
    double acc = 0.0;
    if (full) {
      double2 q[kIters];
#pragma unroll
      for (int j = 0; j < kIters; ++j) q[j] = ld_col<VEC>(col + base + j * (2 * kT));
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        acc = acc + wr[2 * j] * q[j].x;
        acc = acc + wr[2 * j + 1] * q[j].y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        const int64_t e = base + j * (2 * kT);
        if (e < n) acc = acc + wr[2 * j] * col[e];
        if (e + 1 < n) acc = acc + wr[2 * j + 1] * col[e + 1];
      }
    }
    acc = wave_butterfly(acc);
    if (lane == 0) red[v][wv] = acc;
  }
  __syncthreads();
  if (t < nc) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
}

// ---------------------------------------------------- one-pass LSQR step (DBR)
// One LSQR step's two products over R in ONE pass (ksp_lsqr.c, the DBR default): y = U1 = A[:, 0:nc] coef
// + nal * (U * usc) per row in gemv_body's order (columns in order from 0, then the VecAXPY), stored
// unscaled, and in the same pass the DBR stage-1 partials of ||U1||^2 (m = 0: gemv's NORM partial) and of
// column_v . U1 (m = 1 + v: k_scaled_dot's partial of the unscaled U1).  The lane walks its 16 rows as the
// 8 row pairs j = 0..7 of the DBR element order, loading the pair's nc column values once for both: the
// row sums need every column of the pair, the dots every pair of the column.  Two pairs' loads are in
// flight (pa / pb).  NCT >= nc columns' accumulators in registers.  Ragged chunk: guarded scalar loads, and
// rows past n neither stored nor summed (as gemv_body / k_scaled_dot).
template <int NCT, bool NTS>
__device__ __forceinline__ void onepass_load(double2 (&p)[NCT], double2& up, const double* __restrict__ A,
                                             int64_t lda, int nc, const double* __restrict__ U, bool axpy,
                                             int64_t e, int64_t n, bool full) {
#pragma unroll
  for (int v = 0; v < NCT; ++v) {
    if (v < nc) {
      const double* __restrict__ col = A + (int64_t)v * lda + e;
      if (full) p[v] = ld_col<2>(col);
      else p[v] = make_double2(e < n ? col[0] : 0.0, e + 1 < n ? col[1] : 0.0);
    }
  }
  if (axpy) {
    if (full) up = *reinterpret_cast<const double2*>(U + e);
    else up = make_double2(e < n ? U[e] : 0.0, e + 1 < n ? U[e + 1] : 0.0);
  }
}

template <int NCT, bool NTS>
__device__ __forceinline__ void onepass_pair(const double2 (&p)[NCT], double2 up, const double (&a)[NCT], int nc,
                                             bool axpy, double nal, double usc, double* __restrict__ y, int64_t e,
                                             int64_t n, bool full, double& nacc, double (&acc)[NCT]) {
  double r0 = 0.0, r1 = 0.0;
#pragma unroll
  for (int v = 0; v < NCT; ++v) {
    if (v < nc) {
      r0 = r0 + a[v] * p[v].x;
      r1 = r1 + a[v] * p[v].y;
    }
  }
  if (axpy) {  // nal != 0 (uniform): U stored unscaled, its value is U * usc
    r0 = r0 + nal * (up.x * usc);
    r1 = r1 + nal * (up.y * usc);
  }
  const bool in0 = full || e < n, in1 = full || e + 1 < n;
  if (full) {
    st2<NTS>(y + e, r0, r1);
  } else {
    if (in0) y[e] = r0;
    if (in1) y[e + 1] = r1;
  }
  if (in0) nacc = nacc + r0 * r0;
  if (in1) nacc = nacc + r1 * r1;
#pragma unroll
  for (int v = 0; v < NCT; ++v) {
    if (v < nc) {
      if (in0) acc[v] = acc[v] + r0 * p[v].x;
      if (in1) acc[v] = acc[v] + r1 * p[v].y;
    }
  }
}

template <int NCT, bool NTS>
__global__ __launch_bounds__(kT) void k_lsqr_onepass(const double* __restrict__ A, int64_t lda, int nc,
                                                     const double* __restrict__ coef,
                                                     const double* __restrict__ naldev, const double* __restrict__ U,
                                                     const double* __restrict__ uscdev, double* __restrict__ y,
                                                     int64_t n, double* __restrict__ partial, int64_t nchunks,
                                                     const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double red[NCT + 1][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t c = blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  const double nal = *naldev;
  const bool axpy = U != nullptr && nal != 0.0;  // VecAXPY(y, 0, x) does nothing
  const double usc = uscdev ? *uscdev : 1.0;
  double a[NCT];
#pragma unroll
  for (int v = 0; v < NCT; ++v) a[v] = v < nc ? coef[v] : 0.0;
  double acc[NCT];
#pragma unroll
  for (int v = 0; v < NCT; ++v) acc[v] = 0.0;
  double nacc = 0.0;
  double2 pa[NCT], pb[NCT];
  double2 ua = make_double2(0.0, 0.0), ub = make_double2(0.0, 0.0);
  onepass_load<NCT, NTS>(pa, ua, A, lda, nc, U, axpy, base, n, full);
  onepass_load<NCT, NTS>(pb, ub, A, lda, nc, U, axpy, base + 2 * kT, n, full);
#pragma unroll 1
  for (int j = 0; j < kIters; j += 2) {
    const int64_t e = base + (int64_t)j * (2 * kT);
    onepass_pair<NCT, NTS>(pa, ua, a, nc, axpy, nal, usc, y, e, n, full, nacc, acc);
    if (j + 2 < kIters) onepass_load<NCT, NTS>(pa, ua, A, lda, nc, U, axpy, e + 2 * (2 * kT), n, full);
    onepass_pair<NCT, NTS>(pb, ub, a, nc, axpy, nal, usc, y, e + 2 * kT, n, full, nacc, acc);
    if (j + 3 < kIters) onepass_load<NCT, NTS>(pb, ub, A, lda, nc, U, axpy, e + 3 * (2 * kT), n, full);
  }
  nacc = wave_butterfly(nacc);
  if (lane == 0) red[0][wv] = nacc;
#pragma unroll
  for (int v = 0; v < NCT; ++v) {
    if (v < nc) {
      const double r = wave_butterfly(acc[v]);
      if (lane == 0) red[1 + v][wv] = r;
    }
  }
  __syncthreads();
  if (t <= nc) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
}

// ------------------------------------------------------------------ SpMM
// R[:, 0:nc] = A S[:, 0:nc]: one lane per row, the row's CSR entries read once
// for all nc columns; per column the MatMult_SeqAIJ order (ascending entries,
// from 0), as PETSc's MatMatMultNumericAdd_SeqAIJ_SeqDense accumulates.
template <int CG>
__global__ __launch_bounds__(kT) void k_spmm(int32_t nrows, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col, const double* __restrict__ val,
                                             const double* __restrict__ S, int64_t lds, int nc,
                                             double* __restrict__ R, int64_t ldr) {
  const int32_t r = blockIdx.x * kT + threadIdx.x;
  if (r >= nrows) return;
  double acc[CG];
#pragma unroll
  for (int q = 0; q < CG; ++q) acc[q] = 0.0;
  const int32_t k1 = rowptr[r + 1];
  for (int32_t k = rowptr[r]; k < k1; ++k) {
    const double a = val[k];
    const double* __restrict__ sp = S + col[k];
#pragma unroll
    for (int q = 0; q < CG; ++q)
      if (q < nc) acc[q] = acc[q] + a * sp[(int64_t)q * lds];
  }
#pragma unroll
  for (int q = 0; q < CG; ++q)
    if (q < nc) R[r + (int64_t)q * ldr] = acc[q];
}

// ------------------------------------------------------------------ Gram
// Gc = [R b]^T [R b] partials over one DBR chunk: the columns of R and b (column s) in tiles
// of kTB; workgroup (chunk c, tile pair p <= q) forms the kTB x kTB dots of tile p's columns with
// tile q's, each in the DBR lane order of k_scaled_dot (lane t: its 16 elements in order, then the
// wave butterfly and the fixed wave combine), so entry (i, j) is VecDot(col_i, col_j) bit for bit,
// and (i, j), (j, i) are the same sum (IEEE products commute).  Upper-triangle entries only:
// partial[tri(i, j) * nchunks + c].  Workgroups run XCD-major: XCD x takes the chunks c = x mod 8,
// each chunk's tile pairs back to back, so a chunk's columns (<= 8 x 32 KiB per workgroup) are
// read from HBM once and the other pairs find them in that XCD's L2.
constexpr int kTB = 4;
// packed upper triangle, column by column: entries (0..j, j) are contiguous
__device__ __forceinline__ int gram_tri(int i, int j) { return j * (j + 1) / 2 + i; }

__global__ __launch_bounds__(kT) void k_gram(const double* __restrict__ R, int64_t lda, int s,
                                             const double* __restrict__ b, int64_t n, int nbt, int npairs,
                                             int64_t nch, double* __restrict__ partial) {
  __shared__ double red[kTB * kTB][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t bid = blockIdx.x;
  const int64_t slot = bid / 8;
  const int64_t c = (slot / npairs) * 8 + (bid % 8);
  int pr = (int)(slot % npairs), p = 0;  // pair index -> (p, q), p <= q
  while (pr >= nbt - p) {
    pr -= nbt - p;
    ++p;
  }
  const int q = p + pr;
  if (c >= nch) return;  // uniform per workgroup
  const int m = s + 1;
  const int64_t base = c * kChunk + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  const double* colp[2 * kTB];
#pragma unroll
  for (int a = 0; a < 2 * kTB; ++a) {
    const int k = (a < kTB ? p : q) * kTB + (a % kTB);
    colp[a] = k < s ? R + (int64_t)k * lda : (k == s ? b : nullptr);
  }
  double acc[kTB][kTB];
#pragma unroll
  for (int a = 0; a < kTB; ++a)
#pragma unroll
    for (int e = 0; e < kTB; ++e) acc[a][e] = 0.0;
#pragma unroll 2
  for (int j = 0; j < kIters; ++j) {
    const int64_t e0 = base + j * (2 * kT);
    double2 v[2 * kTB];
#pragma unroll
    for (int a = 0; a < 2 * kTB; ++a) {
      if (!colp[a]) {
        v[a] = make_double2(0.0, 0.0);
      } else if (full) {
        v[a] = ld_col<2>(colp[a] + e0);
      } else {
        v[a].x = e0 < n ? colp[a][e0] : 0.0;
        v[a].y = e0 + 1 < n ? colp[a][e0 + 1] : 0.0;
      }
    }
#pragma unroll
    for (int a = 0; a < kTB; ++a)
#pragma unroll
      for (int e = 0; e < kTB; ++e) {
        acc[a][e] = acc[a][e] + v[a].x * v[kTB + e].x;
        acc[a][e] = acc[a][e] + v[a].y * v[kTB + e].y;
      }
  }
#pragma unroll
  for (int a = 0; a < kTB; ++a)
#pragma unroll
    for (int e = 0; e < kTB; ++e) {
      const double r = wave_butterfly(acc[a][e]);
      if (lane == 0) red[a * kTB + e][wv] = r;
    }
  __syncthreads();
  if (t < kTB * kTB) {
    const int i = p * kTB + t / kTB, jj = q * kTB + t % kTB;
    if (i < m && jj < m && i <= jj)
      partial[(int64_t)gram_tri(i, jj) * nch + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
  }
}

// Gc(i, j) = Gc(j, i) = out[tri(i, j)] for i, j < s, Gc(i, s) = out[tri(i, s)] (R^T b)
__global__ void k_gram_scatter(const double* __restrict__ out, int s, double* __restrict__ Gc, int64_t ldg) {
  for (int e = threadIdx.x; e < s * (s + 1); e += blockDim.x) {
    const int i = e % s, j = e / s;
    Gc[i + (int64_t)j * ldg] = out[i <= j ? gram_tri(i, j) : gram_tri(j, i)];
  }
}

// out = ((0 + parts[0]) + parts[1]) + ... elementwise (block order)
__global__ __launch_bounds__(kT) void k_dense_sum(const double* const* __restrict__ parts, const int64_t* __restrict__ ldp,
                                                  int np, int64_t nrows, int ncols, double* __restrict__ out,
                                                  int64_t ldo) {
  const int64_t total = nrows * ncols;
  for (int64_t e = (int64_t)blockIdx.x * kT + threadIdx.x; e < total; e += (int64_t)gridDim.x * kT) {
    const int64_t i = e % nrows, j = e / nrows;
    double acc = 0.0;
    for (int k = 0; k < np; ++k) acc = acc + parts[k][i + j * ldp[k]];
    out[i + j * ldo] = acc;
  }
}

}  // namespace msd

using namespace msd;

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// The dense kernels' tuning (msplit_kernels.h): columns per load group (4; DENSE_G1 / DENSE_G2) and the
// u, u/beta store policy (non-temporal; DENSE_TEMPORAL_ST).  false (error set) for a combination with no kernel.
static bool dense_tuning(int* grp, bool* nts) {
  const int tu = msk_get_tuning();
  if ((tu & MSK_TUNE_DENSE_G1) && (tu & MSK_TUNE_DENSE_G2)) {
    mspi_set_error(MSP_ERR_ARG_OUTOFRANGE, "tuning: DENSE_G1 and DENSE_G2 together select no kernel");
    return false;
  }
  *grp = (tu & MSK_TUNE_DENSE_G1) ? 1 : (tu & MSK_TUNE_DENSE_G2) ? 2 : 4;
  *nts = !(tu & MSK_TUNE_DENSE_TEMPORAL_ST);
  return true;
}

// ===================================================================== internal
extern "C" int mspi_dense_gemv(msp_ctx* c, const double* A, int64_t lda, int nc, int64_t n, const double* coef_dev,
                               const double* nal_dev, const double* U, const double* usc_dev, double* y,
                               double* partial, double* sumsq_dev, const int* stop) {
  if (n <= 0) {
    if (sumsq_dev) HIPCHK(hipMemsetAsync(sumsq_dev, 0, sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  const int64_t nch = nchunks_of(n);
  const int vec = !(aligned16(A) && (lda % 2 == 0) && aligned16(y) && (!U || aligned16(U))) ? 0
                  : (msk_get_tuning() & MSK_TUNE_VEC_TEMPORAL) ? 1 : 2;
  const bool axpy = U != nullptr, norm = sumsq_dev != nullptr;
  KTimer kt(c, MSP_KERNEL_DGEMV, 8.0 * (double)n * (nc + 1 + (axpy ? 1 : 0)));
  const dim3 g((unsigned)nch), b(kT);
  int grp = 4;
  bool nts = true;
  if (!dense_tuning(&grp, &nts)) return MSP_ERR_ARG_OUTOFRANGE;
#define GEMVK(AX, NO, VE, G_, NT_) \
  k_dense_gemv<AX, NO, VE, G_, NT_><<<g, b, 0, c->stream>>>(A, lda, nc, coef_dev, nal_dev, U, usc_dev, y, n, partial, \
                                                            stop)
#define GEMV(AX, NO, VE)                                         \
  do {                                                           \
    if (nts) {                                                   \
      if (grp == 4) GEMVK(AX, NO, VE, 4, true);                  \
      else if (grp == 2) GEMVK(AX, NO, VE, 2, true);             \
      else GEMVK(AX, NO, VE, 1, true);                           \
    } else {                                                     \
      if (grp == 4) GEMVK(AX, NO, VE, 4, false);                 \
      else if (grp == 2) GEMVK(AX, NO, VE, 2, false);            \
      else GEMVK(AX, NO, VE, 1, false);                          \
    }                                                            \
  } while (0)
#define GEMV3(AX, NO) \
  if (vec == 2) GEMV(AX, NO, 2); else if (vec == 1) GEMV(AX, NO, 1); else GEMV(AX, NO, 0);
  if (axpy && norm) { GEMV3(true, true) }
  else if (axpy) { GEMV3(true, false) }
  else if (norm) { GEMV3(false, true) }
  else { GEMV3(false, false) }
#undef GEMV3
#undef GEMV
#undef GEMVK
  KCHK((int)hipGetLastError());
  if (norm && mspi_reduce_seq(c)) {  // ||y||^2 in PETSc's order (msplit_seq.hip)
    Vecs v = {};
    KCHK(mspi_seq_stage1(c, y, &v, 1, n, 1, partial, nch, stop));
  }
  if (norm) KCHK(msk_dot_stage2(partial, nch, 1, sumsq_dev, stop, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_dense_scaled_dots(msp_ctx* c, const double* win, double* wout, const double* sc_dev,
                                      const double* A, int64_t lda, int nc, int64_t n, double* partial,
                                      double* out_dev, const int* stop) {
  if (nc <= 0) return MSP_SUCCESS;
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {
    HIPCHK(hipMemsetAsync(out_dev, 0, (size_t)nc * sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  KTimer kt(c, MSP_KERNEL_DGEMVT, 8.0 * (double)n * (nc + 1 + (sc_dev && wout ? 1 : 0)));
  int grp = 4;
  bool nts = true;
  if (!dense_tuning(&grp, &nts)) return MSP_ERR_ARG_OUTOFRANGE;
  const int vec = !(aligned16(A) && (lda % 2 == 0) && aligned16(win) && (!sc_dev || aligned16(wout))) ? 0
                  : (msk_get_tuning() & MSK_TUNE_VEC_TEMPORAL) ? 1 : 2;
  for (int g0 = 0; g0 < nc; g0 += kMaxCols) {
    const int g = std::min(kMaxCols, nc - g0);
    const double* Ag = A + (int64_t)g0 * lda;
    // scale once, later groups read the scaled vector; without wout (deferred scale) every group rescales win
    const bool scale = sc_dev && (g0 == 0 || !wout);
    const double* src = (sc_dev && g0 > 0 && wout) ? wout : win;
    const dim3 gr((unsigned)nch), b(kT);
#define SDOTK(SC, VE, WO, SD, G_, NT_) \
  k_scaled_dot<SC, VE, G_, NT_><<<gr, b, 0, c->stream>>>(src, WO, SD, Ag, lda, g, n, partial, nch, stop)
#define SDOT(SC, VE, WO, SD)                                        \
  do {                                                              \
    if (nts) {                                                      \
      if (grp == 4) SDOTK(SC, VE, WO, SD, 4, true);                 \
      else if (grp == 2) SDOTK(SC, VE, WO, SD, 2, true);            \
      else SDOTK(SC, VE, WO, SD, 1, true);                          \
    } else {                                                        \
      if (grp == 4) SDOTK(SC, VE, WO, SD, 4, false);                \
      else if (grp == 2) SDOTK(SC, VE, WO, SD, 2, false);           \
      else SDOTK(SC, VE, WO, SD, 1, false);                         \
    }                                                               \
  } while (0)
    if (scale) {
      if (vec == 2) SDOT(true, 2, wout, sc_dev);
      else if (vec == 1) SDOT(true, 1, wout, sc_dev);
      else SDOT(true, 0, wout, sc_dev);
    } else {
      if (vec == 2) SDOT(false, 2, nullptr, nullptr);
      else if (vec == 1) SDOT(false, 1, nullptr, nullptr);
      else SDOT(false, 0, nullptr, nullptr);
    }
#undef SDOT
#undef SDOTK
    KCHK((int)hipGetLastError());
    if (mspi_reduce_seq(c)) {  // dgemv 'T' order: each column . w in sequence (msplit_seq.hip)
      ARGCHK(!sc_dev || wout, MSP_ERR_SUP, "MSP_REDUCE_SEQ reads the scaled vector back: no deferred scale");
      Vecs v = {};
      v.base = Ag;
      v.stride = lda;
      KCHK(mspi_seq_stage1(c, sc_dev ? wout : win, &v, g, n, 0, partial, nch, stop));
    }
    KCHK(msk_dot_stage2(partial, nch, g, out_dev + g0, stop, c->stream));
  }
  return MSP_SUCCESS;
}

// One LSQR step's U1 = A coef + nal (U usc), stored unscaled, with out[0] = ||U1||^2 and out[1 + v] =
// column_v . U1 (DBR; k_lsqr_onepass), in one pass over A when it is 16-byte aligned and nc <= 32; otherwise
// (the same sums) through the gemv and an unscaled column-dot launch.  partial: nchunks * (nc + 1) doubles.
extern "C" int mspi_dense_lsqr_onepass(msp_ctx* c, const double* A, int64_t lda, int nc, int64_t n,
                                       const double* coef_dev, const double* nal_dev, const double* U,
                                       const double* usc_dev, double* y, double* partial, double* out_dev,
                                       const int* stop) {
  ARGCHK(!mspi_reduce_seq(c), MSP_ERR_SUP, "the one-pass LSQR step is the DBR order's");
  ARGCHK(nc >= 1, MSP_ERR_ARG_OUTOFRANGE, "%d columns", nc);
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {
    HIPCHK(hipMemsetAsync(out_dev, 0, (size_t)(nc + 1) * sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  const bool vec = aligned16(A) && (lda % 2 == 0) && aligned16(y) && (!U || aligned16(U)) &&
                   !(msk_get_tuning() & MSK_TUNE_VEC_TEMPORAL);
  int grp = 4;
  bool nts = true;
  if (!dense_tuning(&grp, &nts)) return MSP_ERR_ARG_OUTOFRANGE;
  if (!vec || nc > kMaxCols) {  // the same sums in two passes
    int rc = mspi_dense_gemv(c, A, lda, nc, n, coef_dev, nal_dev, U, usc_dev, y, partial, out_dev, stop);
    if (!rc) rc = mspi_dense_scaled_dots(c, y, nullptr, nullptr, A, lda, nc, n, partial, out_dev + 1, stop);
    return rc;
  }
  {
    KTimer kt(c, MSP_KERNEL_DGEMV, 8.0 * (double)n * (nc + 2 + (U ? 1 : 0)));
    const dim3 g((unsigned)nch), b(kT);
#define OPK(NCT_)                                                                                               \
  do {                                                                                                          \
    if (nts) k_lsqr_onepass<NCT_, true><<<g, b, 0, c->stream>>>(A, lda, nc, coef_dev, nal_dev, U, usc_dev, y, n,  \
                                                                 partial, nch, stop);                           \
    else k_lsqr_onepass<NCT_, false><<<g, b, 0, c->stream>>>(A, lda, nc, coef_dev, nal_dev, U, usc_dev, y, n,     \
                                                             partial, nch, stop);                               \
  } while (0)
    if (nc <= 4) OPK(4);
    else if (nc <= 8) OPK(8);
    else if (nc <= 12) OPK(12);
    else if (nc <= 16) OPK(16);
    else if (nc <= 20) OPK(20);
    else if (nc <= 24) OPK(24);
    else if (nc <= 28) OPK(28);
    else OPK(32);
#undef OPK
    KCHK((int)hipGetLastError());
  }
  KCHK(msk_dot_stage2(partial, nch, nc + 1, out_dev, stop, c->stream));
  return MSP_SUCCESS;
}

// out[j] = ||column j||^2 (DBR), j < nc
extern "C" int mspi_dense_colsumsq(msp_ctx* c, const double* A, int64_t lda, int nc, int64_t n, double* partial,
                                   double* out_dev) {
  if (nc <= 0) return MSP_SUCCESS;
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {
    HIPCHK(hipMemsetAsync(out_dev, 0, (size_t)nc * sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  KTimer kt(c, MSP_KERNEL_NORM, 8.0 * (double)n * nc);
  for (int j = 0; j < nc; ++j) {
    Vecs v = {};
    v.p[0] = A + (int64_t)j * lda;
    if (mspi_reduce_seq(c)) KCHK(mspi_seq_stage1(c, v.p[0], &v, 1, n, 1, partial, nch, nullptr));
    else KCHK(msk_dot_stage1(v.p[0], &v, 1, n, partial, nch, 1, nullptr, c->stream));
    KCHK(msk_dot_stage2(partial, nch, 1, out_dev + j, nullptr, c->stream));
  }
  return MSP_SUCCESS;
}

// ======================================================================= Gram
extern "C" int msp_dense_gram(const msp_dense* R, const msp_vec* b, msp_dense* Gc) {
  ARGCHK(R && b && Gc, MSP_ERR_ARG_NULL, "NULL argument");
  const int s = R->ncols;
  ARGCHK(b->n == R->nrows, MSP_ERR_ARG_SIZ, "b has %lld entries, R %lld rows", (long long)b->n, (long long)R->nrows);
  ARGCHK(Gc->nrows == s && Gc->ncols == s + 1, MSP_ERR_ARG_SIZ, "Gc must be %d x %d, got %lld x %d", s, s + 1,
         (long long)Gc->nrows, Gc->ncols);
  ARGCHK(R->ctx == Gc->ctx && b->ctx == R->ctx, MSP_ERR_ARG_WRONG, "R, b and Gc must share one context");
  msp_ctx* c = R->ctx;
  const int64_t n = R->nrows;
  const int m = s + 1, ntri = m * (m + 1) / 2;
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {  // no rows: every sum is the empty sum 0
    HIPCHK(hipMemsetAsync(Gc->d, 0, (size_t)Gc->lda * Gc->ncols * sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  const bool seq = mspi_reduce_seq(c);
  ARGCHK(!seq || m <= MSK_MAX_GROUP, MSP_ERR_SUP, "MSP_REDUCE_SEQ Gram of more than %d columns",
         MSK_MAX_GROUP - 1);
  ARGCHK(seq || (aligned16(R->d) && aligned16(b->d)), MSP_ERR_ARG_WRONG, "Gram operands must be 16-byte aligned");
  const int64_t pch = seq ? 1 : nch;  // SEQ: one running sum per entry (chunk 0)
  double* partial = nullptr;
  double* out = nullptr;
  int rc = mspi_malloc(c, (void**)&partial, (size_t)ntri * pch * sizeof(double));
  if (rc) return rc;
  if ((rc = mspi_malloc(c, (void**)&out, (size_t)ntri * sizeof(double)))) {
    mspi_free(c, partial);
    return rc;
  }
  {
    // each column of R and b read once (the tile pairs of a chunk meet in L2), Gc written
    KTimer kt(c, MSP_KERNEL_DGEMVT, 8.0 * (double)n * m + 8.0 * (double)s * m);
    if (seq) {  // reference dgemm 'T','N' / dgemv 'T': per entry one running sum over the rows in order
      // column j against columns 0..j (b = column s against R's columns, then b . b): entries (0..j, j),
      // contiguous in the packed triangle, each written as its own one-chunk sum (msk_seq_stage1)
      for (int j = 0; j < m && !rc; ++j) {
        Vecs v = {};
        v.base = R->d;
        v.stride = R->lda;
        const double* w = j < s ? R->d + (int64_t)j * R->lda : b->d;
        double* dst = out + j * (j + 1) / 2;
        rc = mspi_seq_stage1(c, w, &v, std::min(j + 1, s), n, 0, dst, 1, nullptr);
        if (!rc && j == s) {
          Vecs vb = {};
          rc = mspi_seq_stage1(c, b->d, &vb, 1, n, 1, dst + s, 1, nullptr);
        }
      }
    } else {
      const int nbt = (m + kTB - 1) / kTB, npairs = nbt * (nbt + 1) / 2;
      const int64_t grid = (nch + 7) / 8 * 8 * npairs;
      if (grid > INT32_MAX) rc = MSP_ERR_ARG_OUTOFRANGE;
      else {
        k_gram<<<dim3((unsigned)grid), dim3(kT), 0, c->stream>>>(R->d, R->lda, s, b->d, n, nbt, npairs, nch, partial);
        rc = (int)hipGetLastError();
        if (!rc) rc = msk_dot_stage2(partial, nch, ntri, out, nullptr, c->stream);
      }
    }
    if (!rc) {
      k_gram_scatter<<<1, 256, 0, c->stream>>>(out, s, Gc->d, Gc->lda);
      rc = (int)hipGetLastError();
    }
  }
  (void)hipStreamSynchronize(c->stream);
  mspi_free(c, partial);
  mspi_free(c, out);
  if (rc) {
    mspi_set_error(MSP_ERR_LIB, "Gram kernels failed: %s", hipGetErrorString((hipError_t)rc));
    return MSP_ERR_LIB;
  }
  return MSP_SUCCESS;
}

extern "C" int msp_dense_sum(int32_t nparts, const msp_dense* const* parts, msp_dense* out) {
  ARGCHK(parts && out && nparts >= 1, MSP_ERR_ARG_NULL, "NULL argument or no parts");
  ARGCHK(nparts <= 4096, MSP_ERR_ARG_OUTOFRANGE, "at most 4096 parts");
  msp_ctx* c = out->ctx;
  std::vector<const double*> hp((size_t)nparts);
  std::vector<int64_t> hl((size_t)nparts);
  for (int k = 0; k < nparts; ++k) {
    ARGCHK(parts[k], MSP_ERR_ARG_NULL, "part %d is NULL", k);
    ARGCHK(parts[k]->nrows == out->nrows && parts[k]->ncols == out->ncols, MSP_ERR_ARG_SIZ,
           "part %d is %lld x %d, out %lld x %d", k, (long long)parts[k]->nrows, parts[k]->ncols,
           (long long)out->nrows, out->ncols);
    ARGCHK(parts[k]->ctx == c, MSP_ERR_ARG_WRONG, "parts and out must share one context");
    hp[k] = parts[k]->d;
    hl[k] = parts[k]->lda;
  }
  if (out->nrows == 0) return MSP_SUCCESS;
  void* tab = nullptr;
  const size_t bytes = (size_t)nparts * (sizeof(double*) + sizeof(int64_t));
  int rc = mspi_malloc(c, &tab, bytes);
  if (rc) return rc;
  const double** dp = (const double**)tab;
  int64_t* dl = (int64_t*)((char*)tab + (size_t)nparts * sizeof(double*));
  rc = (int)hipMemcpyAsync(dp, hp.data(), (size_t)nparts * sizeof(double*), hipMemcpyHostToDevice, c->stream);
  if (!rc) rc = (int)hipMemcpyAsync(dl, hl.data(), (size_t)nparts * sizeof(int64_t), hipMemcpyHostToDevice, c->stream);
  if (!rc) {
    KTimer kt(c, MSP_KERNEL_OTHER, 8.0 * (double)out->nrows * out->ncols * (nparts + 1));
    const int64_t total = out->nrows * out->ncols;
    const unsigned g = (unsigned)std::min<int64_t>((total + kT - 1) / kT, 4096);
    k_dense_sum<<<g, kT, 0, c->stream>>>(dp, dl, nparts, out->nrows, out->ncols, out->d, out->lda);
    rc = (int)hipGetLastError();
  }
  (void)hipStreamSynchronize(c->stream);
  mspi_free(c, tab);
  if (rc) {
    mspi_set_error(MSP_ERR_LIB, "dense sum failed: %s", hipGetErrorString((hipError_t)rc));
    return MSP_ERR_LIB;
  }
  return MSP_SUCCESS;
}

extern "C" int msp_dense_create_view(msp_dense* A, int32_t col0, int32_t ncols, msp_dense** out) {
  ARGCHK(A && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(col0 >= 0 && ncols >= 1 && col0 + ncols <= A->ncols, MSP_ERR_ARG_OUTOFRANGE,
         "columns [%d, %d) outside the block's %d", col0, col0 + ncols, A->ncols);
  msp_dense* V = new msp_dense();
  V->ctx = A->ctx;
  mspi_ctx_retain(A->ctx);
  V->nrows = A->nrows;
  V->ncols = ncols;
  V->lda = A->lda;
  V->d = A->d + (int64_t)col0 * A->lda;
  V->view = 1;
  *out = V;
  return MSP_SUCCESS;
}

// ======================================================================= dense
// MSPLIT_DENSE_SKEW (doubles, rounded up to 512): extra leading-dimension padding for blocks of at least 2^20
// rows, so that the columns of a tall block are not an exact power-of-two apart (same-box A/B knob).
static int64_t lda_skew() {
  static const int64_t sk = [] {
    const char* e = getenv("MSPLIT_DENSE_SKEW");
    return e ? (atoll(e) + 511) / 512 * 512 : (int64_t)0;
  }();
  return sk;
}
static int64_t lda_for(int64_t nrows) {
  const int64_t l = std::max<int64_t>(512, (nrows + 511) / 512 * 512);
  return nrows >= (int64_t(1) << 20) ? l + lda_skew() : l;
}

extern "C" int msp_dense_create(msp_ctx* c, int64_t nrows, int32_t ncols, msp_dense** out) {
  ARGCHK(c && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(nrows >= 0 && ncols >= 1, MSP_ERR_ARG_SIZ, "dense block %lld x %d", (long long)nrows, ncols);
  msp_dense* A = new msp_dense();
  A->ctx = c;
  mspi_ctx_retain(c);
  A->nrows = nrows;
  A->ncols = ncols;
  A->lda = lda_for(nrows);
  const size_t bytes = (size_t)(A->lda * ncols + 512) * sizeof(double);
  if (mspi_big_alloc((void**)&A->d, bytes) != (int)hipSuccess) {
    delete A;
    mspi_ctx_release(c);
    mspi_set_error(MSP_ERR_MEM, "hipMalloc of a %lld x %d dense block failed", (long long)nrows, ncols);
    return MSP_ERR_MEM;
  }
  HIPCHK(hipMemsetAsync(A->d, 0, bytes, c->stream));
  *out = A;
  return MSP_SUCCESS;
}

extern "C" int msp_dense_destroy(msp_dense** pA) {
  if (!pA || !*pA) return MSP_SUCCESS;
  msp_dense* A = *pA;
  if (A->ctx && A->ctx->stream) (void)hipStreamSynchronize(A->ctx->stream);
  if (A->d && !A->view) (void)hipFree(A->d);
  msp_ctx* c = A->ctx;
  delete A;
  *pA = nullptr;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

extern "C" int msp_dense_get_info(const msp_dense* A, int64_t* nrows, int32_t* ncols, int64_t* lda) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "dense is NULL");
  if (nrows) *nrows = A->nrows;
  if (ncols) *ncols = A->ncols;
  if (lda) *lda = A->lda;
  return MSP_SUCCESS;
}

extern "C" int msp_dense_get_array(msp_dense* A, double** p) {
  ARGCHK(A && p, MSP_ERR_ARG_NULL, "NULL argument");
  *p = A->d;
  return MSP_SUCCESS;
}

extern "C" int msp_dense_zero_entries(msp_dense* A) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "dense is NULL");
  HIPCHK(hipMemsetAsync(A->d, 0, (size_t)A->lda * A->ncols * sizeof(double), A->ctx->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_dense_set_values(msp_dense* A, const double* host, int64_t ld) {
  ARGCHK(A && (host || A->nrows == 0), MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(ld >= A->nrows, MSP_ERR_ARG_SIZ, "ld %lld < nrows %lld", (long long)ld, (long long)A->nrows);
  if (A->nrows == 0) return MSP_SUCCESS;
  HIPCHK(hipMemcpy2DAsync(A->d, (size_t)A->lda * sizeof(double), host, (size_t)ld * sizeof(double),
                          (size_t)A->nrows * sizeof(double), (size_t)A->ncols, hipMemcpyHostToDevice,
                          A->ctx->stream));
  HIPCHK(hipStreamSynchronize(A->ctx->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_dense_get_values(const msp_dense* A, double* host, int64_t ld) {
  ARGCHK(A && (host || A->nrows == 0), MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(ld >= A->nrows, MSP_ERR_ARG_SIZ, "ld %lld < nrows %lld", (long long)ld, (long long)A->nrows);
  if (A->nrows == 0) return MSP_SUCCESS;
  HIPCHK(hipMemcpy2DAsync(host, (size_t)ld * sizeof(double), A->d, (size_t)A->lda * sizeof(double),
                          (size_t)A->nrows * sizeof(double), (size_t)A->ncols, hipMemcpyDeviceToHost,
                          A->ctx->stream));
  HIPCHK(hipStreamSynchronize(A->ctx->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_dense_set_column(msp_dense* A, int32_t j, int64_t row0, const msp_vec* x, int64_t xoff,
                                    int64_t n) {
  ARGCHK(A && x, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(j >= 0 && j < A->ncols, MSP_ERR_ARG_OUTOFRANGE, "column %d outside [0,%d)", j, A->ncols);
  ARGCHK(n >= 0 && row0 >= 0 && row0 + n <= A->nrows && xoff >= 0 && xoff + n <= x->n, MSP_ERR_ARG_OUTOFRANGE,
         "set_column range out of bounds");
  return mspi_copy(A->ctx, A->d + (int64_t)j * A->lda + row0, x->d + xoff, n);
}

extern "C" int msp_dense_mult(msp_dense* A, const msp_vec* alpha, int64_t row0, int64_t n, msp_vec* y, int64_t yoff) {
  ARGCHK(A && alpha && y, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(alpha->n == A->ncols, MSP_ERR_ARG_SIZ, "alpha has %lld entries, dense block %d columns",
         (long long)alpha->n, A->ncols);
  ARGCHK(n >= 0 && row0 >= 0 && row0 + n <= A->nrows && yoff >= 0 && yoff + n <= y->n, MSP_ERR_ARG_OUTOFRANGE,
         "dense mult range out of bounds");
  return mspi_dense_gemv(A->ctx, A->d + row0, A->lda, A->ncols, n, alpha->d, nullptr, nullptr, nullptr, y->d + yoff,
                         nullptr, nullptr, nullptr);
}

extern "C" int msp_dense_mult_transpose(msp_dense* A, const msp_vec* u, msp_vec* out) {
  ARGCHK(A && u && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(u->n == A->nrows && out->n == A->ncols, MSP_ERR_ARG_SIZ, "MatMultTranspose sizes");
  msp_ctx* c = A->ctx;
  double* partial = nullptr;
  const int64_t nch = std::max<int64_t>(1, nchunks_of(A->nrows));
  int rc = mspi_malloc(c, (void**)&partial, (size_t)nch * kMaxCols * sizeof(double));
  if (rc) return rc;
  rc = mspi_dense_scaled_dots(c, u->d, nullptr, nullptr, A->d, A->lda, A->ncols, A->nrows, partial, out->d, nullptr);
  (void)hipStreamSynchronize(c->stream);
  mspi_free(c, partial);
  return rc;
}

extern "C" int msp_mat_matmult_dense(msp_mat* A, const msp_dense* S, msp_dense* R) {
  ARGCHK(A && S && R, MSP_ERR_ARG_NULL, "NULL argument");
  int32_t nr, ncol;
  mspi_mat_dims(A, &nr, &ncol);
  ARGCHK(ncol == S->nrows && nr == R->nrows && S->ncols == R->ncols, MSP_ERR_ARG_SIZ,
         "MatMatMult sizes: A %d x %d, S %lld x %d, R %lld x %d", nr, ncol, (long long)S->nrows, S->ncols,
         (long long)R->nrows, R->ncols);
  const mspi_csr_view v = mspi_mat_csr(A);
  msp_ctx* c = mspi_mat_ctx(A);
  if (nr == 0) return MSP_SUCCESS;
  {  // DV storage (ELL): one byte per entry instead of 12
    int st = 0;
    msp_mat_get_storage(A, &st, nullptr);
    if (st == MSP_STORAGE_DV && mspi_mat_spmm_dv(A, S->d, S->lda, S->ncols, S->nrows, R->d, R->lda) == MSP_SUCCESS)
      return MSP_SUCCESS;
  }
  ARGCHK(v.rowptr && v.col, MSP_ERR_SUP, "MatMatMult needs a stored operator (not a matrix-free one, nor one whose "
         "CSR was released without an ELL-layout DV storage)");
  ARGCHK(!v.compressed, MSP_ERR_SUP, "MatMatMult with a row-compressed matrix");
  KTimer kt(c, MSP_KERNEL_SPMM,
            12.0 * (double)v.nnz + 4.0 * (nr + 1.0) + 8.0 * (double)S->ncols * ((double)S->nrows + (double)nr));
  if (v.lds_cap > 0) {  // CSR slice staged once per row block, columns streamed through it
    KCHK(msk_spmm(nr, v.rowptr, v.col, v.val, S->d, S->lda, S->ncols, R->d, R->lda, v.lds_cap, c->stream));
    return MSP_SUCCESS;
  }
  const dim3 g((unsigned)((nr + kT - 1) / kT)), b(kT);
  for (int j0 = 0; j0 < S->ncols; j0 += 32) {
    const int nc = std::min(32, S->ncols - j0);
    const double* Sg = S->d + (int64_t)j0 * S->lda;
    double* Rg = R->d + (int64_t)j0 * R->lda;
    if (nc <= 8) k_spmm<8><<<g, b, 0, c->stream>>>(nr, v.rowptr, v.col, v.val, Sg, S->lda, nc, Rg, R->lda);
    else if (nc <= 16) k_spmm<16><<<g, b, 0, c->stream>>>(nr, v.rowptr, v.col, v.val, Sg, S->lda, nc, Rg, R->lda);
    else k_spmm<32><<<g, b, 0, c->stream>>>(nr, v.rowptr, v.col, v.val, Sg, S->lda, nc, Rg, R->lda);
    KCHK((int)hipGetLastError());
  }
  return MSP_SUCCESS;
}
