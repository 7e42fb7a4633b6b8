// msplit_kernels.hip -- CDNA4 (gfx950) kernels of the GMRES inner-solve path.
//
// Everything here is HBM-bandwidth bound f64 work (no MFMA): CSR SpMV, the
// classical Gram-Schmidt VecMDot/VecMAXPY block and the BLAS-1 ops around it.
// Compiled with -ffp-contract=off: every a*b+c is a multiply and an add, as in
// PETSc's Seq kernels, so per-element results equal the CPU oracle's bit for
// bit.  Reductions use the deterministic blocked reduction (DBR) whose exact
// order is restated in oracle/oracle.c (dbr_dot): results never depend on the
// launch geometry, the XCD a workgroup lands on, or timing.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "msplit_kernels.h"

namespace msk {

constexpr int kT = 256;          // threads per workgroup (4 wave64)
constexpr int kIters = 8;        // double2 slices per thread per DBR chunk
constexpr int kChunk = kT * 2 * kIters;  // 4096 elements per DBR chunk

static_assert(kChunk == MSK_DBR_CHUNK, "DBR chunk must match the oracle");

__device__ __forceinline__ double wave_butterfly(double v) {
  // v[l] <- v[l] + v[l ^ off], off = 32..1: every lane ends with the same sum.
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------- DBR dots
// Stage 1: workgroup c reduces chunk c of every vector: lane t accumulates its
// elements base + j*512 + 2t, +1 (j = 0..7) in order, wave butterfly, then
// (w0 + w1) + (w2 + w3).  partial[v * nchunks + c].
template <int NV, bool SELF>
__global__ __launch_bounds__(kT) void k_dot_stage1(const double* __restrict__ w, VecGroup V, int64_t n,
                                                   double* __restrict__ partial, int64_t nchunks) {
  __shared__ double red[NV][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t c = blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  double wr[2 * kIters];
  if (full) {
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 q = *reinterpret_cast<const double2*>(w + base + j * (2 * kT));
      wr[2 * j] = q.x;
      wr[2 * j + 1] = q.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const int64_t e = base + j * (2 * kT);
      wr[2 * j] = e < n ? w[e] : 0.0;
      wr[2 * j + 1] = e + 1 < n ? w[e + 1] : 0.0;
    }
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double acc = 0.0;
    if (SELF) {
      if (full) {
#pragma unroll
        for (int j = 0; j < 2 * kIters; ++j) acc = acc + wr[j] * wr[j];
      } else {
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          const int64_t e = base + j * (2 * kT);
          if (e < n) acc = acc + wr[2 * j] * wr[2 * j];
          if (e + 1 < n) acc = acc + wr[2 * j + 1] * wr[2 * j + 1];
        }
      }
    } else {
      const double* __restrict__ y = V.p[v];
      if (full) {
        double2 q[kIters];
#pragma unroll
        for (int j = 0; j < kIters; ++j) q[j] = *reinterpret_cast<const double2*>(y + base + j * (2 * kT));
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          acc = acc + wr[2 * j] * q[j].x;
          acc = acc + wr[2 * j + 1] * q[j].y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          const int64_t e = base + j * (2 * kT);
          if (e < n) acc = acc + wr[2 * j] * y[e];
          if (e + 1 < n) acc = acc + wr[2 * j + 1] * y[e + 1];
        }
      }
    }
    acc = wave_butterfly(acc);
    if (lane == 0) red[v][wv] = acc;
  }
  __syncthreads();
  if (t < NV) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
}

// Stage 2: workgroup v folds the nchunks partials of vector v the same way.
__global__ __launch_bounds__(kT) void k_dot_stage2(const double* __restrict__ partial, int64_t nchunks,
                                                   double* __restrict__ out) {
  __shared__ double red[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* p = partial + blockIdx.x * nchunks;
  double acc = 0.0;
  for (int64_t i = t; i < nchunks; i += kT) acc = acc + p[i];
  acc = wave_butterfly(acc);
  if (lane == 0) red[wv] = acc;
  __syncthreads();
  if (t == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------ MAXPY
// u = w (or 0 when ACCUM); PETSc VecMAXPY_Seq grouping: the nv&3 leading
// vectors (AXPY3/AXPY2/AXPY), then groups of four; w = u (or x + u when ACCUM).
template <int NV>
__device__ __forceinline__ double maxpy_elem(double u, const double (&a)[NV], const double (&p)[NV]) {
  constexpr int jrem = NV & 3;
  if constexpr (jrem == 3) u = u + ((a[0] * p[0] + a[1] * p[1]) + a[2] * p[2]);
  else if constexpr (jrem == 2) u = u + (a[0] * p[0] + a[1] * p[1]);
  else if constexpr (jrem == 1) u = a[0] * p[0] + u;
#pragma unroll
  for (int j = jrem; j < NV; j += 4) u = u + (((a[j] * p[j] + a[j + 1] * p[j + 1]) + a[j + 2] * p[j + 2]) + a[j + 3] * p[j + 3]);
  return u;
}

template <int NV, bool ACCUM, int MINW>
__global__ __launch_bounds__(kT, MINW) void k_maxpy(double* __restrict__ w, VecGroup V, Coefs A, const double* __restrict__ adev,
                                              int negate, int64_t n) {
  double a[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const double aj = adev ? adev[j] : A.a[j];
    a[j] = negate ? -aj : aj;
  }
  const int64_t npair = n >> 1;
  const int64_t stride = (int64_t)gridDim.x * kT;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < npair; i += stride) {
    const double2 wv = *reinterpret_cast<const double2*>(w + 2 * i);
    double p0[NV], p1[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const double2 q = *reinterpret_cast<const double2*>(V.p[j] + 2 * i);
      p0[j] = q.x;
      p1[j] = q.y;
    }
    double u0 = maxpy_elem<NV>(ACCUM ? 0.0 : wv.x, a, p0);
    double u1 = maxpy_elem<NV>(ACCUM ? 0.0 : wv.y, a, p1);
    if (ACCUM) {
      u0 = wv.x + u0;
      u1 = wv.y + u1;
    }
    *reinterpret_cast<double2*>(w + 2 * i) = make_double2(u0, u1);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t e = n - 1;
    double p[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) p[j] = V.p[j][e];
    const double u = maxpy_elem<NV>(ACCUM ? 0.0 : w[e], a, p);
    w[e] = ACCUM ? w[e] + u : u;
  }
}

// Vector-major MAXPY in the DBR chunk layout: workgroup c owns elements
// [4096c, 4096c+4096); lane t owns base + j*512 + 2t, +1 (j = 0..7) and keeps
// their 16 running values in registers while the vectors stream past group by
// group (each group = up to 4 vectors x 32 KiB contiguous per workgroup).
// Per element the arithmetic is exactly PETSc's grouping (as maxpy_elem).
// NORM: also the DBR partial of ||w_new||^2 for this chunk (VecNorm fused).
template <int G>
__device__ __forceinline__ double group_sum(const double (&a)[G], const double (&p)[G]) {
  if constexpr (G == 1) {
    return a[0] * p[0];
  } else {
  double s = a[0] * p[0] + a[1] * p[1];
  if constexpr (G > 2) s = s + a[2] * p[2];
  if constexpr (G > 3) s = s + a[3] * p[3];
  return s;
  }
}

template <int G, bool FULL>
__device__ __forceinline__ void chunk_group(double (&u)[2 * kIters], const VecGroup& V, const Coefs& A,
                                            const double* __restrict__ adev, int negate, int g, int64_t base,
                                            int64_t n) {
  double a[G];
  const double* vp[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {  // wave-uniform: scalar loads from the kernel arguments / adev
    const double aq = adev ? adev[g + q] : A.a[g + q];
    a[q] = negate ? -aq : aq;
    vp[q] = V.p[g + q];
  }
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    const int64_t e = base + j * (2 * kT);
    double p0[G], p1[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (FULL) {
        const double2 v = *reinterpret_cast<const double2*>(vp[q] + e);
        p0[q] = v.x;
        p1[q] = v.y;
      } else {
        p0[q] = e < n ? vp[q][e] : 0.0;
        p1[q] = e + 1 < n ? vp[q][e + 1] : 0.0;
      }
    }
    const double s0 = group_sum<G>(a, p0), s1 = group_sum<G>(a, p1);
    if constexpr (G == 1) {  // PetscKernelAXPY: s = a*p; s += U
      u[2 * j] = s0 + u[2 * j];
      u[2 * j + 1] = s1 + u[2 * j + 1];
    } else {
      u[2 * j] = u[2 * j] + s0;
      u[2 * j + 1] = u[2 * j + 1] + s1;
    }
  }
}

template <bool ACCUM, bool NORM, bool FULL>
__device__ __forceinline__ void maxpy_chunk_body(double* __restrict__ w, const VecGroup& V, const Coefs& A,
                                                 const double* __restrict__ adev, int negate, int nv, int64_t base,
                                                 int64_t n, double& sq) {
  double u[2 * kIters];
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    const int64_t e = base + j * (2 * kT);
    if (ACCUM) {
      u[2 * j] = 0.0;
      u[2 * j + 1] = 0.0;
    } else if (FULL) {
      const double2 q = *reinterpret_cast<const double2*>(w + e);
      u[2 * j] = q.x;
      u[2 * j + 1] = q.y;
    } else {
      u[2 * j] = e < n ? w[e] : 0.0;
      u[2 * j + 1] = e + 1 < n ? w[e + 1] : 0.0;
    }
  }
  const int jrem = nv & 3;
  if (jrem == 3) chunk_group<3, FULL>(u, V, A, adev, negate, 0, base, n);
  else if (jrem == 2) chunk_group<2, FULL>(u, V, A, adev, negate, 0, base, n);
  else if (jrem == 1) chunk_group<1, FULL>(u, V, A, adev, negate, 0, base, n);
#pragma unroll 1
  for (int g = jrem; g < nv; g += 4) chunk_group<4, FULL>(u, V, A, adev, negate, g, base, n);
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    const int64_t e = base + j * (2 * kT);
    double r0 = u[2 * j], r1 = u[2 * j + 1];
    if (FULL) {
      if (ACCUM) {
        const double2 q = *reinterpret_cast<const double2*>(w + e);
        r0 = q.x + r0;
        r1 = q.y + r1;
      }
      *reinterpret_cast<double2*>(w + e) = make_double2(r0, r1);
      if (NORM) {
        acc = acc + r0 * r0;
        acc = acc + r1 * r1;
      }
    } else {
      if (e < n) {
        if (ACCUM) r0 = w[e] + r0;
        w[e] = r0;
        if (NORM) acc = acc + r0 * r0;
      }
      if (e + 1 < n) {
        if (ACCUM) r1 = w[e + 1] + r1;
        w[e + 1] = r1;
        if (NORM) acc = acc + r1 * r1;
      }
    }
  }
  sq = acc;
}

template <bool ACCUM, bool NORM>
__global__ __launch_bounds__(kT) void k_maxpy_chunk(double* __restrict__ w, VecGroup V, Coefs A,
                                                    const double* __restrict__ adev, int negate, int nv, int64_t n,
                                                    double* __restrict__ partial) {
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  double sq = 0.0;
  if ((c + 1) * kChunk <= n) maxpy_chunk_body<ACCUM, NORM, true>(w, V, A, adev, negate, nv, base, n, sq);
  else maxpy_chunk_body<ACCUM, NORM, false>(w, V, A, adev, negate, nv, base, n, sq);
  if (NORM) {
    __shared__ double red[4];
    sq = wave_butterfly(sq);
    if ((t & 63) == 0) red[t >> 6] = sq;
    __syncthreads();
    if (t == 0) partial[c] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

// ------------------------------------------------------------------- SpMV
// Row-blocked CSR: workgroup b owns rows [256b, 256b+256).  Its contiguous
// slice of col/val is staged into LDS with 16-byte coalesced loads, then lane
// t sums row 256b+t left to right over its columns (MatMult_SeqAIJ order),
// gathering x from L2/MALL.  RESID: r = b - sum.
template <bool RESID>
__global__ __launch_bounds__(kT) void k_spmv_lds(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ col, const double* __restrict__ val,
                                                 const double* __restrict__ x, const double* __restrict__ b,
                                                 double* __restrict__ y, int32_t lds_cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sval = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + (size_t)lds_cap * 8);
  const int t = threadIdx.x;
  const int32_t r0 = blockIdx.x * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  for (int32_t i = t; i < n2; i += kT) reinterpret_cast<double2*>(sval)[i] = v2[i];
  for (int32_t i = t; i < n4; i += kT) reinterpret_cast<int4*>(scol)[i] = c4[i];
  __syncthreads();
  const int32_t r = r0 + t;
  if (r < r1) {
    const int32_t k0 = rowptr[r], k1 = rowptr[r + 1];
    double s = 0.0;
    for (int32_t k = k0; k < k1; ++k) s = s + sval[k - s2] * x[scol[k - s4]];
    y[r] = RESID ? b[r] - s : s;
  }
}

// Same staging; the row is consumed in chunks of 8 entries whose 8 LDS reads
// and 8 x-gathers are all issued before the first product (indices clamped
// to the row, never branched around), so each lane keeps 8 gathers in flight.
// The sum is still left to right over the row.
template <bool RESID>
__global__ __launch_bounds__(kT) void k_spmv_lds8(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, const double* __restrict__ val,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  double* __restrict__ y, int32_t lds_cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sval = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + (size_t)lds_cap * 8);
  const int t = threadIdx.x;
  const int32_t r0 = blockIdx.x * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  const int32_t r = r0 + t;
  int32_t k0 = 0, k1 = 0;
  double bb = 0.0;
  if (r < r1) {
    k0 = rowptr[r];
    k1 = rowptr[r + 1];
    if (RESID) bb = b[r];
  }
  for (int32_t i = t; i < n2; i += kT) reinterpret_cast<double2*>(sval)[i] = v2[i];
  for (int32_t i = t; i < n4; i += kT) reinterpret_cast<int4*>(scol)[i] = c4[i];
  __syncthreads();
  if (r < r1) {
    double s = 0.0;
    for (int32_t kb = k0; kb < k1; kb += 8) {
      double av[8], xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int32_t k = min(kb + q, k1 - 1);
        av[q] = sval[k - s2];
        xv[q] = x[scol[k - s4]];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (kb + q < k1) s = s + av[q] * xv[q];
    }
    y[r] = RESID ? bb - s : s;
  }
}

// Rows too long for the LDS stage: one lane per row, direct loads (same order).
template <bool RESID>
__global__ __launch_bounds__(kT) void k_spmv_direct(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ col, const double* __restrict__ val,
                                                    const double* __restrict__ x, const double* __restrict__ b,
                                                    double* __restrict__ y) {
  const int32_t r = blockIdx.x * kT + threadIdx.x;
  if (r >= nrows) return;
  double s = 0.0;
  for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) s = s + val[k] * x[col[k]];
  y[r] = RESID ? b[r] - s : s;
}

// Row-compressed matrix: only rows row_ids[0..nlisted) hold entries.
// y[row] = sum (MatMult) or r[row] = b[row] - sum (MatResidual); the caller
// has already written 0 (MatMult) or b (MatResidual) into the other rows.
template <bool RESID>
__global__ __launch_bounds__(kT) void k_spmv_rows(int32_t nlisted, const int32_t* __restrict__ row_ids,
                                                  const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                  const double* __restrict__ val, const double* __restrict__ x,
                                                  const double* __restrict__ b, double* __restrict__ y) {
  const int32_t k = blockIdx.x * kT + threadIdx.x;
  if (k >= nlisted) return;
  double s = 0.0;
  for (int32_t q = rowptr[k]; q < rowptr[k + 1]; ++q) s = s + val[q] * x[col[q]];
  const int32_t r = row_ids[k];
  y[r] = RESID ? b[r] - s : s;
}

// -------------------------------------------------------------- assembly
// Box Laplacian with Dirichlet boundaries; rowptr in closed form (entries
// before row l = deg*l minus the missing neighbours of rows < l).
__device__ __forceinline__ int64_t box_rowptr(int dim, int64_t l, int64_t nx, int64_t ny, int64_t nz) {
  const int64_t cx0 = (l + nx - 1) / nx, cxN = l / nx;  // rows < l with i == 0 / i == nx-1
  const int64_t P = nx * ny;
  int64_t missing = cx0 + cxN;
  if (dim == 3) {
    const int64_t q = l / P, rem = l % P;
    const int64_t cy0 = q * nx + min(rem, nx);
    const int64_t cyN = q * nx + max((int64_t)0, rem - (ny - 1) * nx);
    const int64_t cz0 = min(l, P);
    const int64_t czN = max((int64_t)0, l - (nz - 1) * P);
    missing += cy0 + cyN + cz0 + czN;
    return 7 * l - missing;
  }
  const int64_t cy0 = min(l, nx);
  const int64_t cyN = max((int64_t)0, l - (ny - 1) * nx);
  missing += cy0 + cyN;
  return 5 * l - missing;
}

__global__ __launch_bounds__(kT) void k_box_stencil(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows,
                                                    int32_t* __restrict__ rowptr, int32_t* __restrict__ col,
                                                    double* __restrict__ val) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  for (int64_t l = (int64_t)blockIdx.x * kT + threadIdx.x; l <= nrows; l += stride) {
    const int64_t p0 = box_rowptr(dim, l, nx, ny, nz);
    rowptr[l] = (int32_t)p0;
    if (l == nrows) continue;
    const int64_t P = (int64_t)nx * ny;
    const int32_t i = (int32_t)(l % nx);
    const int32_t j = (int32_t)((l / nx) % ny);
    const int32_t k = dim == 3 ? (int32_t)(l / P) : 0;
    int64_t p = p0;
    const double diag = dim == 3 ? 6.0 : 4.0;
    if (dim == 3 && k > 0) { col[p] = (int32_t)(l - P); val[p++] = -1.0; }
    if (j > 0) { col[p] = (int32_t)(l - nx); val[p++] = -1.0; }
    if (i > 0) { col[p] = (int32_t)(l - 1); val[p++] = -1.0; }
    col[p] = (int32_t)l; val[p++] = diag;
    if (i < nx - 1) { col[p] = (int32_t)(l + 1); val[p++] = -1.0; }
    if (j < ny - 1) { col[p] = (int32_t)(l + nx); val[p++] = -1.0; }
    if (dim == 3 && k < nz - 1) { col[p] = (int32_t)(l + P); val[p++] = -1.0; }
  }
}

// --------------------------------------------------------------- BLAS-1
template <int OP>
__global__ __launch_bounds__(kT) void k_blas1(double* __restrict__ y, const double* __restrict__ x,
                                              const double* __restrict__ z, double alpha, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += stride) {
    double r;
    if (OP == MSK_SET) r = alpha;
    else if (OP == MSK_COPY) r = x[i];
    else if (OP == MSK_SCALE) r = y[i] * alpha;
    else if (OP == MSK_AXPY) r = y[i] + alpha * x[i];        // daxpy: dy = dy + da*dx
    else if (OP == MSK_AYPX) r = x[i] + alpha * y[i];        // VecAYPX: y = x + beta*y
    else if (OP == MSK_WAXPY_P1) r = z[i] + x[i];            // VecWAXPY alpha == 1
    else if (OP == MSK_WAXPY_M1) r = z[i] - x[i];            // VecWAXPY alpha == -1
    else r = z[i] + alpha * x[i];                            // VecWAXPY general
    y[i] = r;
  }
}

}  // namespace msk

// ===================================================================== launchers
using namespace msk;

// Kernel variants (A/B tuning; MSPLIT_VARIANT_<KERNEL>=<n> at context creation).
static int g_variant[MSK_NVAR] = {0};

extern "C" void msk_set_variant(int which, int v) {
  if (which >= 0 && which < MSK_NVAR) g_variant[which] = v;
}

static inline int grid_for(int64_t work, int cap) {
  int64_t g = (work + kT - 1) / kT;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <int NV>
static void launch_dot1(const double* w, const VecGroup& V, int64_t n, double* partial, int64_t nchunks, bool self,
                        hipStream_t s) {
  if (self) k_dot_stage1<1, true><<<dim3((unsigned)nchunks), dim3(kT), 0, s>>>(w, V, n, partial, nchunks);
  else k_dot_stage1<NV, false><<<dim3((unsigned)nchunks), dim3(kT), 0, s>>>(w, V, n, partial, nchunks);
}

template <int... Is>
struct Seq {};

template <int NV>
static void dot1_dispatch(int nv, const double* w, const VecGroup& V, int64_t n, double* partial, int64_t nchunks,
                          hipStream_t s) {
  if (nv == NV) launch_dot1<NV>(w, V, n, partial, nchunks, false, s);
  else if constexpr (NV < MSK_MAX_GROUP) dot1_dispatch<NV + 1>(nv, w, V, n, partial, nchunks, s);
}

extern "C" int msk_dot_stage1(const double* w, const VecGroup* V, int nv, int64_t n, double* partial,
                              int64_t nchunks, int self, hipStream_t s) {
  if (nchunks <= 0) return 0;
  if (self) launch_dot1<1>(w, *V, n, partial, nchunks, true, s);
  else dot1_dispatch<1>(nv, w, *V, n, partial, nchunks, s);
  return (int)hipGetLastError();
}

extern "C" int msk_dot_stage2(const double* partial, int64_t nchunks, int nv, double* out, hipStream_t s) {
  k_dot_stage2<<<dim3(nv), dim3(kT), 0, s>>>(partial, nchunks, out);
  return (int)hipGetLastError();
}

extern "C" int msk_maxpy_norm(double* w, const VecGroup* V, int nv, const Coefs* A, const double* adev, int negate,
                              int64_t n, int accum, double* partial, hipStream_t s) {
  if (n <= 0 || nv <= 0) return 0;
  const unsigned g = (unsigned)((n + kChunk - 1) / kChunk);
  if (partial) k_maxpy_chunk<false, true><<<dim3(g), dim3(kT), 0, s>>>(w, *V, *A, adev, negate, nv, n, partial);
  else if (accum) k_maxpy_chunk<true, false><<<dim3(g), dim3(kT), 0, s>>>(w, *V, *A, adev, negate, nv, n, partial);
  else k_maxpy_chunk<false, false><<<dim3(g), dim3(kT), 0, s>>>(w, *V, *A, adev, negate, nv, n, partial);
  return (int)hipGetLastError();
}

template <int NV>
static void maxpy_dispatch(int nv, double* w, const VecGroup& V, const Coefs& A, const double* adev, int negate,
                           int64_t n, int accum, hipStream_t s) {
  if (nv == NV) {
    const int g = grid_for((n + 1) / 2, 4096);
    if (g_variant[MSK_VAR_MAXPY] == 2) {
      if (accum) k_maxpy<NV, true, 4><<<dim3(g), dim3(kT), 0, s>>>(w, V, A, adev, negate, n);
      else k_maxpy<NV, false, 4><<<dim3(g), dim3(kT), 0, s>>>(w, V, A, adev, negate, n);
    } else {
      if (accum) k_maxpy<NV, true, 1><<<dim3(g), dim3(kT), 0, s>>>(w, V, A, adev, negate, n);
      else k_maxpy<NV, false, 1><<<dim3(g), dim3(kT), 0, s>>>(w, V, A, adev, negate, n);
    }
  } else if constexpr (NV < MSK_MAX_GROUP) {
    maxpy_dispatch<NV + 1>(nv, w, V, A, adev, negate, n, accum, s);
  }
}

extern "C" int msk_maxpy(double* w, const VecGroup* V, int nv, const Coefs* A, const double* adev, int negate,
                         int64_t n, int accum, hipStream_t s) {
  if (n <= 0 || nv <= 0) return 0;
  if (g_variant[MSK_VAR_MAXPY] == 0) return msk_maxpy_norm(w, V, nv, A, adev, negate, n, accum, nullptr, s);
  maxpy_dispatch<1>(nv, w, *V, *A, adev, negate, n, accum, s);
  return (int)hipGetLastError();
}

extern "C" int msk_spmv(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* x,
                        const double* b, double* y, int32_t lds_cap, int resid, hipStream_t s) {
  if (nrows <= 0) return 0;
  const unsigned g = (unsigned)((nrows + kT - 1) / kT);
  if (lds_cap > 0 && g_variant[MSK_VAR_SPMV] == 0) {
    const size_t lds = (size_t)lds_cap * 12;
    if (resid) k_spmv_lds8<true><<<dim3(g), dim3(kT), lds, s>>>(nrows, rowptr, col, val, x, b, y, lds_cap);
    else k_spmv_lds8<false><<<dim3(g), dim3(kT), lds, s>>>(nrows, rowptr, col, val, x, b, y, lds_cap);
  } else if (lds_cap > 0) {
    const size_t lds = (size_t)lds_cap * 12;
    if (resid) k_spmv_lds<true><<<dim3(g), dim3(kT), lds, s>>>(nrows, rowptr, col, val, x, b, y, lds_cap);
    else k_spmv_lds<false><<<dim3(g), dim3(kT), lds, s>>>(nrows, rowptr, col, val, x, b, y, lds_cap);
  } else {
    if (resid) k_spmv_direct<true><<<dim3(g), dim3(kT), 0, s>>>(nrows, rowptr, col, val, x, b, y);
    else k_spmv_direct<false><<<dim3(g), dim3(kT), 0, s>>>(nrows, rowptr, col, val, x, b, y);
  }
  return (int)hipGetLastError();
}

extern "C" int msk_spmv_rows(int32_t nlisted, const int32_t* row_ids, const int32_t* rowptr, const int32_t* col,
                             const double* val, const double* x, const double* b, double* y, int resid,
                             hipStream_t s) {
  if (nlisted <= 0) return 0;
  const unsigned g = (unsigned)((nlisted + kT - 1) / kT);
  if (resid) k_spmv_rows<true><<<dim3(g), dim3(kT), 0, s>>>(nlisted, row_ids, rowptr, col, val, x, b, y);
  else k_spmv_rows<false><<<dim3(g), dim3(kT), 0, s>>>(nlisted, row_ids, rowptr, col, val, x, b, y);
  return (int)hipGetLastError();
}

extern "C" int msk_box_stencil(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows, int32_t* rowptr,
                               int32_t* col, double* val, hipStream_t s) {
  const int g = grid_for(nrows + 1, 8192);
  k_box_stencil<<<dim3(g), dim3(kT), 0, s>>>(dim, nx, ny, nz, nrows, rowptr, col, val);
  return (int)hipGetLastError();
}

extern "C" int msk_blas1(int op, double* y, const double* x, const double* z, double alpha, int64_t n,
                         hipStream_t s) {
  if (n <= 0) return 0;
  const int g = grid_for(n, 4096);
  switch (op) {
    case MSK_SET: k_blas1<MSK_SET><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    case MSK_COPY: k_blas1<MSK_COPY><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    case MSK_SCALE: k_blas1<MSK_SCALE><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    case MSK_AXPY: k_blas1<MSK_AXPY><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    case MSK_AYPX: k_blas1<MSK_AYPX><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    case MSK_WAXPY_P1: k_blas1<MSK_WAXPY_P1><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    case MSK_WAXPY_M1: k_blas1<MSK_WAXPY_M1><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
    default: k_blas1<MSK_WAXPY><<<dim3(g), dim3(kT), 0, s>>>(y, x, z, alpha, n); break;
  }
  return (int)hipGetLastError();
}
