// msplit_kernels.hip -- CDNA4 (gfx950) kernels of the GMRES inner-solve path.
//
// Everything here is HBM-bandwidth bound f64 work (no MFMA): CSR SpMV, the
// classical Gram-Schmidt VecMDot/VecMAXPY block and the BLAS-1 ops around it.
// Compiled with -ffp-contract=off: every a*b+c is a multiply and an add, as in
// PETSc's Seq kernels, so per-element results equal the CPU oracle's bit for
// bit.  Reductions use the deterministic blocked reduction (DBR) whose exact
// order is restated in oracle/oracle.c (dbr_dot): results never depend on the
// launch geometry, the XCD a workgroup lands on, or timing.
//
// Kernels that run inside a GMRES cycle take a device `stop` flag: once the
// device-side convergence logic (msplit_gmres.hip) ends the cycle, the rest of
// the speculatively enqueued iterations return at once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "msplit_kernels.h"

// The launchers are split into parts that the Makefile compiles as separate objects (-DMSK_PART=1..6), so the
// large template sets (MDot and MAXPY over 1..32 vectors and their variants) build in parallel.  Without
// MSK_PART the file compiles every part into one object.
#ifndef MSK_PART
#define MSK_PART 0
#endif
#define MSK_IN(p) (MSK_PART == 0 || MSK_PART == (p))
#define MSK_PART_DOT 1
#define MSK_PART_MAXPY 2
#define MSK_PART_SPMV 3
#define MSK_PART_MISC 4
#define MSK_PART_DOT_A 5
#define MSK_PART_DOT_B 6

namespace msk {
namespace {  // internal linkage: this file is compiled once per part (see MSK_PART below)

constexpr int kT = 256;                  // threads per workgroup (4 wave64)
constexpr int kIters = 8;                // double2 slices per thread per DBR chunk
constexpr int kChunk = kT * 2 * kIters;  // 4096 elements per DBR chunk

static_assert(kChunk == MSK_DBR_CHUNK, "DBR chunk must match the oracle");

__device__ __forceinline__ bool stopped(const int* stop) { return stop && *stop; }

typedef double dx2 __attribute__((ext_vector_type(2)));
typedef int ix4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double2 ld_nt(const double2* p) {
  const dx2 v = __builtin_nontemporal_load(reinterpret_cast<const dx2*>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ int4 ld_nt(const int4* p) {
  const ix4 v = __builtin_nontemporal_load(reinterpret_cast<const ix4*>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ const double* vec_at(const Vecs& V, int j) {
  return V.base ? V.base + (int64_t)j * V.stride : V.p[j];
}
// deferred VecNormalize: element i of vector j is fl(V_j[i] * scale[j]); x * 1.0
// is exact for every double, so unscaled sets multiply by 1.0 (wave-uniform load)
__device__ __forceinline__ double vec_scale(const Vecs& V, int j) { return V.scale ? V.scale[j] : 1.0; }

// ---------------------------------------------- W = A (sc x) in the CGS kernels
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// Stage the DV dictionary in LDS (the caller synchronises before use).
__device__ __forceinline__ void ell_dict_stage(const EllOp& op, int32_t* sdel, double* sval) {
  const int t = threadIdx.x;
  if (t < op.ndict) {
    sdel[t] = op.ddelta[t];
    sval[t] = op.dval[t];
  } else {
    sdel[t] = 0;  // code 255 (no entry) and unused codes: delta 0, never added
    sval[t] = 0.0;
  }
}

// The lane's W values at its DBR positions base + j*512 + {0,1}, j in [J0, J0+JN):
// rows e, e+1 read their 2 x 8 codes with one 16-byte load, then every gather
// of the pair is issued before the first product (padding entries gather x[0]
// and are masked out).  Each row sums val * (x * sc) over its entries in CSR
// order from 0.0 -- k_spmv_ell's SCALED sum, term for term.  Rows >= n: 0.
template <int J0, int JN>
__device__ __forceinline__ void ell_rows(const EllOp& op, const int32_t* sdel, const double* sval, double sc,
                                         int64_t base, int64_t n, double (&wr)[2 * kIters]) {
#pragma unroll
  for (int j = J0; j < J0 + JN; ++j) {
    const int64_t e = base + j * (2 * kT);
    u32x4v cw = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (e + 1 < n) {
      cw = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(op.code8 + e * 8));
    } else if (e < n) {
      cw.x = reinterpret_cast<const uint32_t*>(op.code8 + e * 8)[0];
      cw.y = reinterpret_cast<const uint32_t*>(op.code8 + e * 8)[1];
    }
    int32_t ix[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t w4 = q < 4 ? cw.x : q < 8 ? cw.y : q < 12 ? cw.z : cw.w;
      const int c = (w4 >> (8 * (q & 3))) & 255;
      ix[q] = c != 255 ? (int32_t)(e + (q >> 3)) + sdel[c] : 0;
    }
    double xv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) xv[q] = op.x[ix[q]];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double acc = 0.0;
#pragma unroll
      for (int q = 8 * h; q < 8 * h + 8; ++q) {
        const uint32_t w4 = q < 4 ? cw.x : q < 8 ? cw.y : q < 12 ? cw.z : cw.w;
        const int c = (w4 >> (8 * (q & 3))) & 255;
        const double sn = acc + sval[c] * (xv[q] * sc);
        acc = c != 255 ? sn : acc;
      }
      wr[2 * j + h] = acc;
    }
  }
}

__device__ __forceinline__ double wave_butterfly(double v) {
  // v[l] <- v[l] + v[l ^ off], off = 32..1: every lane ends with the same sum.
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------- DBR dots
// Stage 1: workgroup c reduces chunk c of every vector: lane t accumulates its
// elements base + j*512 + 2t, +1 (j = 0..7) in order, wave butterfly, then
// (w0 + w1) + (w2 + w3).  partial[v * nchunks + c].  w stays in registers and
// each vector streams 32 KiB contiguous per workgroup.
// VAR: bit 0 = non-temporal loads of the basis vectors (the default: each
// vector streams through once per kernel and is far larger than the 256 MiB
// MALL, so caching it only evicts lines others still need; +8-16 % per kernel,
// +7.7 % per GMRES step on 256^3, same-box A/B); bit 2 = non-temporal store
// of w in MAXPY.  Results are identical.
// G vectors of a full chunk at once: all G*8 loads are issued before the first
// product (4 x 32 KiB in flight per workgroup instead of one vector's 32 KiB),
// then G independent accumulations and butterflies.  Per vector the sum is the
// same sequence as one at a time.
template <int G, int VAR>
__device__ __forceinline__ void dot_group_full(const double (&wr)[2 * kIters], const Vecs& V, int64_t base, int rev,
                                               int nv, int g, double (*red)[4], int lane, int wv) {
  double2 q[G][kIters];
  double sv[G];
  int vv[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    // load order only (each dot is independent): newest vector first when rev
    vv[u] = rev ? nv - 1 - (g + u) : g + u;
    const double* __restrict__ y = vec_at(V, vv[u]);
    sv[u] = vec_scale(V, vv[u]);
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2* pq = reinterpret_cast<const double2*>(y + base + j * (2 * kT));
      q[u][j] = (VAR & 1) ? ld_nt(pq) : *pq;
    }
  }
  double acc[G];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    acc[u] = 0.0;
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      acc[u] = acc[u] + wr[2 * j] * (q[u][j].x * sv[u]);
      acc[u] = acc[u] + wr[2 * j + 1] * (q[u][j].y * sv[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < G; ++u) {
    acc[u] = wave_butterfly(acc[u]);
    if (lane == 0) red[vv[u]][wv] = acc[u];
  }
}

// Stage 1: workgroup c reduces chunk c of every vector: lane t accumulates its
// elements base + j*512 + 2t, +1 (j = 0..7) in order, wave butterfly, then
// (w0 + w1) + (w2 + w3).  partial[v * nchunks + c].  w stays in registers and
// each vector streams 32 KiB contiguous per workgroup.
// VAR: bit 0 = non-temporal loads of the basis vectors (the default: each
// vector streams through once per kernel and is far larger than the 256 MiB
// MALL, so caching it only evicts lines others still need; +8-16 % per kernel,
// +7.7 % per GMRES step on 256^3, same-box A/B); bit 2 = non-temporal store
// of w in MAXPY; bit 4 = vectors one at a time in MDot (A/B of the grouped loads).
// Results are identical.
template <int NV, bool SELF, int VAR, bool OPW = false>
__device__ __forceinline__ void dot_chunk(const double* __restrict__ w, const Vecs& V, int64_t n,
                                          double* __restrict__ partial, int64_t nchunks, int rev, int64_t c,
                                          double (&red)[NV][4], const EllOp* op = nullptr,
                                          const int32_t* sdel = nullptr, const double* sval = nullptr) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t base = c * kChunk + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  double wr[2 * kIters];
  if constexpr (OPW) {
    ell_rows<0, kIters>(*op, sdel, sval, *op->sdev, base, n, wr);
  } else if (full) {
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
  if (!SELF && full && (VAR & 16) == 0) {
    constexpr int G = NV >= 4 ? 4 : NV;
    int g = 0;
    if constexpr ((VAR & 32) != 0) {  // two groups per iteration (MSK_TUNE_MDOT_UNROLL2)
#pragma unroll 2
      for (; g + G <= NV; g += G) dot_group_full<G, VAR>(wr, V, base, rev, NV, g, red, lane, wv);
    } else {
#pragma unroll 1
      for (; g + G <= NV; g += G) dot_group_full<G, VAR>(wr, V, base, rev, NV, g, red, lane, wv);
    }
    if constexpr (NV % G == 3) dot_group_full<3, VAR>(wr, V, base, rev, NV, g, red, lane, wv);
    if constexpr (NV % G == 2) dot_group_full<2, VAR>(wr, V, base, rev, NV, g, red, lane, wv);
    if constexpr (NV % G == 1) dot_group_full<1, VAR>(wr, V, base, rev, NV, g, red, lane, wv);
  } else {
#pragma unroll
  for (int vi = 0; vi < NV; ++vi) {
    // load order only (each dot is independent): newest vector first when rev,
    // so the CGS MAXPY that follows finds the oldest ones still in the MALL
    const int v = rev ? NV - 1 - vi : vi;
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
      const double* __restrict__ y = vec_at(V, v);
      const double sv = vec_scale(V, v);
      if (full) {
        double2 q[kIters];
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          const double2* pq = reinterpret_cast<const double2*>(y + base + j * (2 * kT));
          q[j] = (VAR & 1) ? ld_nt(pq) : *pq;
        }
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          acc = acc + wr[2 * j] * (q[j].x * sv);
          acc = acc + wr[2 * j + 1] * (q[j].y * sv);
        }
      } else {
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          const int64_t e = base + j * (2 * kT);
          if (e < n) acc = acc + wr[2 * j] * (y[e] * sv);
          if (e + 1 < n) acc = acc + wr[2 * j + 1] * (y[e + 1] * sv);
        }
      }
    }
    acc = wave_butterfly(acc);
    if (lane == 0) red[v][wv] = acc;
  }
  }
  __syncthreads();
  if (t < NV) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
}

template <int NV, bool SELF, int VAR>
__global__ __launch_bounds__(kT) void k_dot_stage1(const double* __restrict__ w, Vecs V, int64_t n,
                                                   double* __restrict__ partial, int64_t nchunks,
                                                   const int* __restrict__ stop, int rev) {
  if (stopped(stop)) return;
  __shared__ double red[NV][4];
  dot_chunk<NV, SELF, VAR>(w, V, n, partial, nchunks, rev, blockIdx.x, red);
}

// Stage 1 with W = A (sc x) computed in the kernel (no W vector in HBM).
template <int NV, int VAR>
__global__ __launch_bounds__(kT) void k_dot_stage1_op(EllOp op, Vecs V, int64_t n, double* __restrict__ partial,
                                                      int64_t nchunks, const int* __restrict__ stop) {
  __shared__ double red[NV][4];
  __shared__ int32_t sdel[kT];
  __shared__ double sval[kT];
  ell_dict_stage(op, sdel, sval);
  if (stopped(stop)) return;  // uniform: every lane reads the same flag
  __syncthreads();
  dot_chunk<NV, false, VAR, true>(nullptr, V, n, partial, nchunks, 0, blockIdx.x, red, &op, sdel, sval);
}

// Stage 2: workgroup v folds the nchunks partials of vector v the same way.
template <bool HS>
__global__ __launch_bounds__(kT) void k_dot_stage2(const double* __restrict__ partial, int64_t nchunks,
                                                   double* __restrict__ out, const int* __restrict__ stop) {
  // the stop flag (HS: stop is not null) is read together with the partials and tested after the
  // (convergent) butterfly, so a running cycle waits for one round of loads, not two
  bool skip = false;
  if constexpr (HS) skip = *stop != 0;
  __shared__ double red[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* p = partial + blockIdx.x * nchunks;
  double acc = 0.0;
  int64_t i = t;
  // 16, then 8 loads in flight per lane, added in the same order (lane t: p[t], p[t+256], ...)
  for (; i + 15 * kT < nchunks; i += 16 * kT) {
    double q[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) q[u] = p[i + u * kT];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = acc + q[u];
  }
  for (; i + 7 * kT < nchunks; i += 8 * kT) {
    double q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) q[u] = p[i + u * kT];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = acc + q[u];
  }
  for (; i < nchunks; i += kT) acc = acc + p[i];
  acc = wave_butterfly(acc);
  if (skip) return;  // uniform
  if (lane == 0) red[wv] = acc;
  __syncthreads();
  if (t == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------ MAXPY
// Vector-major MAXPY in the DBR chunk layout: workgroup c owns elements
// [4096c, 4096c+4096); lane t owns base + j*512 + 2t, +1 (j = 0..7) and keeps
// their 16 running values in registers while the vectors stream past group by
// group (each group = up to 4 vectors x 32 KiB contiguous per workgroup).
// Per element the arithmetic is PETSc VecMAXPY_Seq's: the nv&3 leading vectors
// (PetscKernelAXPY3/2/1), then groups of four (PetscKernelAXPY4),
// U += a0*p0 + a1*p1 + a2*p2 + a3*p3 evaluated left to right.
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

template <int G, bool FULL, int VAR, int J0, int JN>
__device__ __forceinline__ void chunk_group(double (&u)[2 * kIters], const Vecs& V, const Coefs& A,
                                            const double* __restrict__ adev, int negate, int g, int64_t base,
                                            int64_t n) {
  double a[G], sv[G];
  const double* vp[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {  // wave-uniform: scalar loads from the kernel arguments / adev
    const double aq = adev ? adev[g + q] : A.a[g + q];
    a[q] = negate ? -aq : aq;
    vp[q] = vec_at(V, g + q);
    sv[q] = vec_scale(V, g + q);
  }
#pragma unroll
  for (int j = J0; j < J0 + JN; ++j) {
    const int64_t e = base + j * (2 * kT);
    double p0[G], p1[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (FULL) {
        const double2* pv = reinterpret_cast<const double2*>(vp[q] + e);
        const double2 v = (VAR & 1) ? ld_nt(pv) : *pv;
        p0[q] = v.x * sv[q];
        p1[q] = v.y * sv[q];
      } else {
        p0[q] = e < n ? vp[q][e] * sv[q] : 0.0;
        p1[q] = e + 1 < n ? vp[q][e + 1] * sv[q] : 0.0;
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

// One slice [J0, J0+JN) of the lane's 8 double2 positions: load w, run every
// vector group over it, store and add its squares to acc in j order.  The
// chunk is one slice (VAR bit 3 clear) or two halves one after the other (set:
// half the registers, twice the waves per SIMD); per element nothing changes.
template <bool ACCUM, bool NORM, bool FULL, int VAR, int J0, int JN, bool OPW = false>
__device__ __forceinline__ void maxpy_slice(const double* __restrict__ win, double* __restrict__ wout,
                                            const Vecs& V, const Coefs& A, const double* __restrict__ adev,
                                            int negate, int nv, int64_t base, int64_t n, double& acc,
                                            const EllOp* op = nullptr, const int32_t* sdel = nullptr,
                                            const double* sval = nullptr) {
  double u[2 * kIters];
  if constexpr (OPW) {
    ell_rows<J0, JN>(*op, sdel, sval, *op->sdev, base, n, u);
  } else {
#pragma unroll
    for (int j = J0; j < J0 + JN; ++j) {
      const int64_t e = base + j * (2 * kT);
      if (ACCUM) {
        u[2 * j] = 0.0;
        u[2 * j + 1] = 0.0;
      } else if (FULL) {
        const double2 q = *reinterpret_cast<const double2*>(win + e);
        u[2 * j] = q.x;
        u[2 * j + 1] = q.y;
      } else {
        u[2 * j] = e < n ? win[e] : 0.0;
        u[2 * j + 1] = e + 1 < n ? win[e + 1] : 0.0;
      }
    }
  }
  const int jrem = nv & 3;
  if (jrem == 3) chunk_group<3, FULL, VAR, J0, JN>(u, V, A, adev, negate, 0, base, n);
  else if (jrem == 2) chunk_group<2, FULL, VAR, J0, JN>(u, V, A, adev, negate, 0, base, n);
  else if (jrem == 1) chunk_group<1, FULL, VAR, J0, JN>(u, V, A, adev, negate, 0, base, n);
  if constexpr ((VAR & 32) != 0) {  // two groups per iteration: the compiler issues 8 vectors' loads at once
#pragma unroll 2
    for (int g = jrem; g < nv; g += 4) chunk_group<4, FULL, VAR, J0, JN>(u, V, A, adev, negate, g, base, n);
  } else {
#pragma unroll 1
    for (int g = jrem; g < nv; g += 4) chunk_group<4, FULL, VAR, J0, JN>(u, V, A, adev, negate, g, base, n);
  }
#pragma unroll
  for (int j = J0; j < J0 + JN; ++j) {
    const int64_t e = base + j * (2 * kT);
    double r0 = u[2 * j], r1 = u[2 * j + 1];
    if (FULL) {
      if (ACCUM) {  // VecAXPY(x, 1.0, T): x + T
        const double2 q = *reinterpret_cast<const double2*>(win + e);
        r0 = q.x + r0;
        r1 = q.y + r1;
      }
      if constexpr ((VAR & 4) != 0) {
        dx2 o;
        o.x = r0;
        o.y = r1;
        __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(wout + e));
      } else {
        *reinterpret_cast<double2*>(wout + e) = make_double2(r0, r1);
      }
      if (NORM) {
        acc = acc + r0 * r0;
        acc = acc + r1 * r1;
      }
    } else {
      if (e < n) {
        if (ACCUM) r0 = win[e] + r0;
        wout[e] = r0;
        if (NORM) acc = acc + r0 * r0;
      }
      if (e + 1 < n) {
        if (ACCUM) r1 = win[e + 1] + r1;
        wout[e + 1] = r1;
        if (NORM) acc = acc + r1 * r1;
      }
    }
  }
}

template <bool ACCUM, bool NORM, bool FULL, int VAR, bool OPW = false>
__device__ __forceinline__ void maxpy_chunk_body(const double* __restrict__ win, double* __restrict__ wout,
                                                 const Vecs& V, const Coefs& A, const double* __restrict__ adev,
                                                 int negate, int nv, int64_t base, int64_t n, double& sq,
                                                 const EllOp* op = nullptr, const int32_t* sdel = nullptr,
                                                 const double* sval = nullptr) {
  double acc = 0.0;
  if constexpr ((VAR & 8) != 0) {
    maxpy_slice<ACCUM, NORM, FULL, VAR, 0, kIters / 2, OPW>(win, wout, V, A, adev, negate, nv, base, n, acc, op,
                                                            sdel, sval);
    maxpy_slice<ACCUM, NORM, FULL, VAR, kIters / 2, kIters / 2, OPW>(win, wout, V, A, adev, negate, nv, base, n,
                                                                     acc, op, sdel, sval);
  } else {
    maxpy_slice<ACCUM, NORM, FULL, VAR, 0, kIters, OPW>(win, wout, V, A, adev, negate, nv, base, n, acc, op, sdel,
                                                        sval);
  }
  sq = acc;
}

template <bool ACCUM, bool NORM, int VAR>
__global__ __launch_bounds__(kT) void k_maxpy_chunk(const double* win, double* wout, Vecs V, Coefs A,
                                                    const double* __restrict__ adev, int negate, int nv,
                                                    const int* __restrict__ nvdev, int64_t n,
                                                    double* __restrict__ partial, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  if (nvdev) nv = *nvdev;
  if (nv <= 0) return;
  const int t = threadIdx.x;
  const int64_t c = (VAR & 64) ? (int64_t)gridDim.x - 1 - blockIdx.x : blockIdx.x;  // 64: top chunks first
  const int64_t base = c * kChunk + 2 * t;
  double sq = 0.0;
  if ((c + 1) * kChunk <= n) maxpy_chunk_body<ACCUM, NORM, true, VAR>(win, wout, V, A, adev, negate, nv, base, n, sq);
  else maxpy_chunk_body<ACCUM, NORM, false, VAR>(win, wout, V, A, adev, negate, nv, base, n, sq);
  if (NORM) {
    __shared__ double red[4];
    sq = wave_butterfly(sq);
    if ((t & 63) == 0) red[t >> 6] = sq;
    __syncthreads();
    if (t == 0) partial[c] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

// CGS VecMAXPY with W = A (sc x) computed in the kernel, and the ||w||^2 partials.
template <int VAR>
__global__ __launch_bounds__(kT) void k_maxpy_op(EllOp op, double* wout, Vecs V, const double* __restrict__ adev,
                                                 int nv, int64_t n, double* __restrict__ partial,
                                                 const int* __restrict__ stop) {
  __shared__ int32_t sdel[kT];
  __shared__ double sval[kT];
  __shared__ double red[4];
  ell_dict_stage(op, sdel, sval);
  if (stopped(stop)) return;  // uniform
  __syncthreads();
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  const Coefs A = {};
  double sq = 0.0;
  if ((c + 1) * kChunk <= n)
    maxpy_chunk_body<false, true, true, VAR, true>(nullptr, wout, V, A, adev, 1, nv, base, n, sq, &op, sdel, sval);
  else
    maxpy_chunk_body<false, true, false, VAR, true>(nullptr, wout, V, A, adev, 1, nv, base, n, sq, &op, sdel, sval);
  sq = wave_butterfly(sq);
  if ((t & 63) == 0) red[t >> 6] = sq;
  __syncthreads();
  if (t == 0) partial[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ------------------------------------------------------------------- SpMV
// Row-blocked CSR: workgroup b owns rows [256b, 256b+256).  Its contiguous
// slice of col/val is staged into LDS with 16-byte coalesced loads; lane t then
// sums row 256b+t left to right over its columns (MatMult_SeqAIJ order), in
// chunks of 8 entries whose 8 LDS reads and 8 x-gathers are all issued before
// the first product (indices clamped to the row, never branched around), so
// each lane keeps 8 gathers in flight.
//   MULT: y = A x    RESID: y = b - A x
//   SCALED (VecNormalize fused into the next MatMult): sc = *sdev,
//     y = A (sc*x), each product val*(x*sc) rounded exactly as VecScale
//     followed by MatMult; vout[r] = x[r]*sc when vout != null (GMRES keeps
//     its basis unnormalised with the scales beside it and passes null).
// XCD-aware order (stencil operators whose plane is a multiple of 8 row
// blocks): workgroups are dealt round-robin over the 8 XCDs, so XCD x runs
// launches x, x+8, ...  Each plane's row blocks are cut into groups of gb
// blocks; XCD x sweeps its groups (x, x+8, ...) through all planes, plane by
// plane.  A row block's x-gathers at +-1 plane then hit lines its own XCD read
// gb blocks earlier (~gb*256 rows of traffic ago, inside the 4 MiB L2), and
// +-1 line stays inside the group.  Only the schedule changes: every row's sum
// is the same, so results are bitwise unchanged.
struct XcdMap {
  int32_t bp;  // row blocks per plane (0: identity order)
  int32_t gb;  // row blocks per group, (bp / gb) % 8 == 0
  int32_t np;  // planes
};

__device__ __forceinline__ int32_t row_block(XcdMap m) {
  const int32_t i = blockIdx.x;
  if (m.bp == 0) return i;
  if (m.bp < 0) return (i & 7) * m.np + (i >> 3);  // z-chunks: XCD x sweeps rows [x N/8, (x+1) N/8) in order
  const int32_t xcd = i & 7, j = i >> 3;
  const int32_t span = m.np * m.gb;  // blocks of one group over all planes
  const int32_t q = j / span, rem = j - q * span;
  const int32_t k = rem / m.gb, t = rem - k * m.gb;
  return k * m.bp + (xcd + 8 * q) * m.gb + t;
}

// Stage a row block's val/col slice (16-byte aligned-down views v2/c4 with n2/n4
// slices) into LDS.  SU > 1: issue SU val and SU/2 col loads per lane before the
// first LDS write, so staging costs one memory latency instead of one per slice.
// aux (cache policy) 2 = nt on gfx950 (global_load_lds_dwordx4 ... nt)
template <bool NT>
__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, NT ? 2 : 0);
}

// SU == 0: LDS-DMA staging.  Each wave-instruction writes 64 consecutive 16-byte
// slices (LDS destination wave-uniform, source per lane); the tail lanes of the
// last instruction re-read the last slice into slack LDS, so the LDS capacity is
// rounded up to 256 entries (msk_spmv).  The barrier after it waits for vmcnt(0).
template <bool NT, int SU>
__device__ __forceinline__ void stage_csr_block(int t, int32_t n2, int32_t n4, const double2* __restrict__ v2,
                                                const int4* __restrict__ c4, double* sval, int32_t* scol) {
  if constexpr (SU == 0) {
    const int lane = t & 63, w = t >> 6;
    for (int32_t ib = w * 64; ib < n2; ib += kT)
      glds16<NT>(v2 + min(ib + lane, n2 - 1), reinterpret_cast<char*>(sval) + (size_t)ib * 16);
    for (int32_t ib = w * 64; ib < n4; ib += kT)
      glds16<NT>(c4 + min(ib + lane, n4 - 1), reinterpret_cast<char*>(scol) + (size_t)ib * 16);
  } else if constexpr (SU == 1) {
    for (int32_t i = t; i < n2; i += kT) reinterpret_cast<double2*>(sval)[i] = NT ? ld_nt(v2 + i) : v2[i];
    for (int32_t i = t; i < n4; i += kT) reinterpret_cast<int4*>(scol)[i] = NT ? ld_nt(c4 + i) : c4[i];
  } else {
    for (int32_t i0 = t; i0 < n2 || i0 < n4; i0 += SU * kT) {
      double2 vt[SU];
      int4 ct[SU / 2 > 0 ? SU / 2 : 1];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n2) vt[u] = NT ? ld_nt(v2 + i) : v2[i];
      }
#pragma unroll
      for (int u = 0; u < SU / 2; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n4) ct[u] = NT ? ld_nt(c4 + i) : c4[i];
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n2) reinterpret_cast<double2*>(sval)[i] = vt[u];
      }
#pragma unroll
      for (int u = 0; u < SU / 2; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n4) reinterpret_cast<int4*>(scol)[i] = ct[u];
      }
      if (i0 + (SU / 2) * kT < n4) {  // col slices beyond SU/2 (rows longer than ~8 entries)
        for (int32_t i = i0 + (SU / 2) * kT; i < n4 && i < i0 + SU * kT; i += kT)
          reinterpret_cast<int4*>(scol)[i] = NT ? ld_nt(c4 + i) : c4[i];
      }
    }
  }
}

// POL bit 0: non-temporal col/val loads; bit 1: non-temporal y (and vout)
// stores.  Default POL 3 in every mode: col/val stream through once and y is
// not re-read by this kernel, so neither should displace x (re-read across the
// +-plane gathers) from L2/MALL.  Same box, same allocation, interleaved
// (tools/spmv_policy_ab.py, profiles/r02/nt_ab/): 512^3 MatMult 0.689 (POL 0)
// -> 0.711 (POL 2) -> 0.723 (POL 3) of 8 TB/s; 256^3 0.696 -> 0.771.
// MSK_TUNE_SPMV_TEMPORAL selects POL 0, MSK_TUNE_SPMV_NTY POL 2.
// A template, not a run-time bool: with "if (nt) nontemporal_store(p) else
// store(p)" the optimizer merges the two stores to the same address into one
// plain store (the non-temporal hint is dropped), which it did here until
// round 2 -- the disassembly of every policy now shows the intended store.
template <bool NT>
__device__ __forceinline__ void st_pol(double* p, double v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int MODE, int POL, int SU>
__global__ __launch_bounds__(kT) void k_spmv_lds8(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, const double* __restrict__ val,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  double* __restrict__ y, int32_t lds_cap,
                                                  const double* __restrict__ sdev, double* __restrict__ vout,
                                                  const int* __restrict__ stop, XcdMap xm) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sval = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + (size_t)lds_cap * 8);
  const int t = threadIdx.x;
  const int32_t r0 = row_block(xm) * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  const int32_t r = r0 + t;
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  int32_t k0 = 0, k1 = 0;
  double bb = 0.0;
  if (r < r1) {
    k0 = rowptr[r];
    k1 = rowptr[r + 1];
    if (MODE == MSK_SPMV_RESID) bb = b[r];
    if (MODE == MSK_SPMV_SCALED && vout) st_pol<(POL & 2) != 0>(vout + r, x[r] * sc);
  }
  stage_csr_block<(POL & 1) != 0, SU>(t, n2, n4, v2, c4, sval, scol);
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
      for (int q = 0; q < 8; ++q) {
        if (MODE == MSK_SPMV_SCALED) xv[q] = xv[q] * sc;
        if (kb + q < k1) s = s + av[q] * xv[q];
      }
    }
    st_pol<(POL & 2) != 0>(y + r, MODE == MSK_SPMV_RESID ? bb - s : s);
  }
}

// GMRES step, MatMult fused with the VecMDot that follows it:
//   W = A (sc*X)  and  partial[v][c] = DBR chunk c of W . (scale_v V_v), v < nv.
// Workgroup c owns DBR chunk c (rows [4096c, 4096c+4096)) and runs it as 8
// sub-blocks of 512 rows; in sub-block j lane t computes rows j*512 + 2t and
// 2t+1 -- exactly the elements the DBR order gives lane t -- so W never leaves
// the registers between the two phases: MDot reads neither W nor (from HBM)
// V(it) = X, which this workgroup has just gathered.  Each row is summed as in
// k_spmv_lds8 (MatMult_SeqAIJ order, val*(x*sc)); each dot as in dot_chunk.
// Needs every 512-row sub-block's col/val slice to fit lds_cap entries.
template <int VAR>
__device__ __forceinline__ void row_pair_sums(int32_t kA0, int32_t kA1, int32_t kB1, const double* sval,
                                              const int32_t* scol, int32_t s2, int32_t s4,
                                              const double* __restrict__ x, double sc, double& wa, double& wb) {
  double sa = 0.0, sb = 0.0;
  const int32_t la = kA1 - kA0, lb = kB1 - kA1;
  const int32_t lmax = la > lb ? la : lb;
  for (int32_t q0 = 0; q0 < lmax; q0 += 8) {
    double av[8], xa[8], bv[8], xb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {  // 16 gathers in flight, indices clamped to the row
      // an empty row reads nothing (its slot of the slice may hold another block's indices)
      const int32_t ka = kA0 + min(q0 + q, la - 1);
      const int32_t kb = kA1 + min(q0 + q, lb - 1);
      av[q] = la > 0 ? sval[ka - s2] : 0.0;
      xa[q] = la > 0 ? x[scol[ka - s4]] : 0.0;
      bv[q] = lb > 0 ? sval[kb - s2] : 0.0;
      xb[q] = lb > 0 ? x[scol[kb - s4]] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (q0 + q < la) sa = sa + av[q] * (xa[q] * sc);
      if (q0 + q < lb) sb = sb + bv[q] * (xb[q] * sc);
    }
  }
  wa = sa;
  wb = sb;
}

template <int VAR, int GF>
__global__ __launch_bounds__(kT) void k_spmv_mdot(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, const double* __restrict__ val,
                                                  const double* __restrict__ x, const double* __restrict__ sdev,
                                                  double* __restrict__ y, int32_t lds_cap, Vecs V, int nv,
                                                  double* __restrict__ partial, int64_t nchunks,
                                                  const int* __restrict__ stop) {
  if (stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sval = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + (size_t)lds_cap * 8);
  __shared__ double red[MSK_MAX_GROUP][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t c = blockIdx.x;
  const int64_t n = nrows;
  const int64_t base = c * kChunk + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  const double sc = *sdev;
  double wr[2 * kIters];
#pragma unroll 1
  for (int j = 0; j < kIters; ++j) {
    const int32_t r0 = (int32_t)(c * kChunk + j * (2 * kT));
    if (r0 >= nrows) {  // uniform: the chunk's tail past the last row
      for (int jj = j; jj < kIters; ++jj) wr[2 * jj] = wr[2 * jj + 1] = 0.0;
      break;
    }
    const int32_t r1 = min(r0 + 2 * kT, nrows);
    const int32_t start = rowptr[r0], end = rowptr[r1];
    const int32_t s2 = start & ~1, s4 = start & ~3;
    const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
    const int32_t ra = r0 + 2 * t;
    int32_t kA0 = 0, kA1 = 0, kB1 = 0;
    if (ra < r1) {
      kA0 = rowptr[ra];
      kA1 = rowptr[ra + 1];
      kB1 = ra + 1 < r1 ? rowptr[ra + 2] : kA1;
    }
    if (j) __syncthreads();  // the previous sub-block's slice is no longer read
    stage_csr_block<false, 8>(t, n2, n4, reinterpret_cast<const double2*>(val + s2),
                              reinterpret_cast<const int4*>(col + s4), sval, scol);
    __syncthreads();
    double wa = 0.0, wb = 0.0;
    if (ra < r1) {
      row_pair_sums<VAR>(kA0, kA1, kB1, sval, scol, s2, s4, x, sc, wa, wb);
      if (ra + 1 < r1) *reinterpret_cast<double2*>(y + ra) = make_double2(wa, wb);
      else y[ra] = wa;
    }
    wr[2 * j] = wa;
    wr[2 * j + 1] = wb;
  }
  // VecMDot of W against the nv basis vectors, this chunk (dot_chunk's order)
  if (full) {
    int g = 0;
#pragma unroll 1
    for (; g + GF <= nv; g += GF) dot_group_full<GF, VAR>(wr, V, base, 0, nv, g, red, lane, wv);
    switch (nv - g) {
      case 3: dot_group_full<3, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      case 2: dot_group_full<2, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      case 1: dot_group_full<1, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      default: break;
    }
  } else {
#pragma unroll 1
    for (int v = 0; v < nv; ++v) {
      const double* __restrict__ yv = vec_at(V, v);
      const double sv = vec_scale(V, v);
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        const int64_t e = base + j * (2 * kT);
        if (e < n) acc = acc + wr[2 * j] * (yv[e] * sv);
        if (e + 1 < n) acc = acc + wr[2 * j + 1] * (yv[e + 1] * sv);
      }
      acc = wave_butterfly(acc);
      if (lane == 0) red[v][wv] = acc;
    }
  }
  __syncthreads();
  if (t < nv) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
}

// R[:, 0:nc] = A S[:, 0:nc] (MatMatMult(AIJ, DENSE)): the row block's CSR slice
// is staged once, then each column streams through it like one SpMV (per row:
// entries in order, from 0), so A is read once for all nc columns.
__global__ __launch_bounds__(kT) void k_spmm_lds8(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, const double* __restrict__ val,
                                                  const double* __restrict__ S, int64_t lds, int nc,
                                                  double* __restrict__ R, int64_t ldr, int32_t lds_cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sval = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + (size_t)lds_cap * 8);
  const int t = threadIdx.x;
  const int32_t r0 = blockIdx.x * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const int32_t r = r0 + t;
  int32_t k0 = 0, k1 = 0;
  if (r < r1) {
    k0 = rowptr[r];
    k1 = rowptr[r + 1];
  }
  stage_csr_block<false, 4>(t, n2, n4, reinterpret_cast<const double2*>(val + s2),
                            reinterpret_cast<const int4*>(col + s4), sval, scol);
  __syncthreads();
  if (r >= r1) return;
#pragma unroll 1
  for (int q = 0; q < nc; ++q) {
    const double* __restrict__ x = S + (int64_t)q * lds;
    double s = 0.0;
    for (int32_t kb = k0; kb < k1; kb += 8) {
      double av[8], xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int32_t k = min(kb + u, k1 - 1);
        av[u] = sval[k - s2];
        xv[u] = x[scol[k - s4]];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (kb + u < k1) s = s + av[u] * xv[u];
    }
    R[r + (int64_t)q * ldr] = s;
  }
}

// Rows too long for the LDS stage: one lane per row, direct loads (same order).
template <int MODE>
__global__ __launch_bounds__(kT) void k_spmv_direct(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ col, const double* __restrict__ val,
                                                    const double* __restrict__ x, const double* __restrict__ b,
                                                    double* __restrict__ y, const double* __restrict__ sdev,
                                                    double* __restrict__ vout, const int* __restrict__ stop) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  const int32_t r = blockIdx.x * kT + threadIdx.x;
  if (r >= nrows) return;
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  double s = 0.0;
  for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
    double xv = x[col[k]];
    if (MODE == MSK_SPMV_SCALED) xv = xv * sc;
    s = s + val[k] * xv;
  }
  if (MODE == MSK_SPMV_SCALED && vout) vout[r] = x[r] * sc;
  y[r] = MODE == MSK_SPMV_RESID ? b[r] - s : s;
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

// lo / hi: the block also couples to the neighbour plane below / above (one
// plane of the slowest direction: z in 3D, mesh lines in 2D), stored as extra
// columns before / after the block's own: column space [plane_lo | block |
// plane_hi], still ascending in global order (the rows of the reference's
// A_block_jacobi, utils.c:30-121 / :247-293, with their column ids shifted).
// coef: the 7 constant stencil values (slow-, y-, x-, diagonal, x+, y+, slow+);
// the Poisson operator is {-1,-1,-1,6,-1,-1,-1} (3D) / {-1,0,-1,4,-1,0,-1} (2D).
__global__ __launch_bounds__(kT) void k_box_stencil(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows,
                                                    int lo, int hi, BoxCoef cf, int32_t* __restrict__ rowptr,
                                                    int32_t* __restrict__ col, double* __restrict__ val) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  const int64_t P = dim == 3 ? (int64_t)nx * ny : (int64_t)nx;  // slab plane
  const int64_t ns = dim == 3 ? nz : ny;                           // planes in the block
  const int64_t off = lo ? P : 0;
  for (int64_t l = (int64_t)blockIdx.x * kT + threadIdx.x; l <= nrows; l += stride) {
    int64_t p0 = box_rowptr(dim, l, nx, ny, nz);
    if (lo) p0 += min(l, P);
    if (hi) p0 += max((int64_t)0, l - (ns - 1) * P);
    rowptr[l] = (int32_t)p0;
    if (l == nrows) continue;
    const int32_t i = (int32_t)(l % nx);
    const int32_t j = (int32_t)((l / nx) % ny);
    const int64_t sl = l / P;  // slab-plane index (k in 3D, j in 2D)
    const int64_t e = l + off;
    int64_t p = p0;
    if (sl > 0 || lo) { col[p] = (int32_t)(e - P); val[p++] = cf.c[0]; }
    if (dim == 3 && j > 0) { col[p] = (int32_t)(e - nx); val[p++] = cf.c[1]; }
    if (i > 0) { col[p] = (int32_t)(e - 1); val[p++] = cf.c[2]; }
    col[p] = (int32_t)e; val[p++] = cf.c[3];
    if (i < nx - 1) { col[p] = (int32_t)(e + 1); val[p++] = cf.c[4]; }
    if (dim == 3 && j < ny - 1) { col[p] = (int32_t)(e + nx); val[p++] = cf.c[5]; }
    if (sl < ns - 1 || hi) { col[p] = (int32_t)(e + P); val[p++] = cf.c[6]; }
  }
}

// ------------------------------------------------ matrix-free box stencil
// y = A x for the operator k_box_stencil assembles, without storing it: row l
// sums the same terms in the same (ascending column) order from 0.0, with the
// same coefficients, so every result equals the CSR SpMV's bit for bit; only
// x (its neighbours through L2/MALL) and y cross HBM.  MODE as k_spmv_lds8.
// One workgroup per (x-segment, y, z) of the box: i, j and the slab plane come
// from the grid, so no integer division per row.  V2 (nx even): each lane
// takes two neighbouring rows, so x, y and the neighbour planes move as 16-byte
// pairs; each row's sum is the same sequence either way.
template <int MODE, bool V2>
__global__ __launch_bounds__(kT) void k_stencil_spmv(int dim, int32_t nx, int32_t ny, int32_t nz, int lo, int hi,
                                                     BoxCoef cf, const double* __restrict__ x,
                                                     const double* __restrict__ b, double* __restrict__ y,
                                                     const double* __restrict__ sdev, double* __restrict__ vout,
                                                     const int* __restrict__ stop) {
  if (stopped(stop)) return;
  constexpr int R = V2 ? 2 : 1;
  const int32_t i0 = ((int32_t)blockIdx.x * kT + (int32_t)threadIdx.x) * R;
  if (i0 >= nx) return;
  const int32_t j = (int32_t)blockIdx.y;       // y in 3D, the mesh line in 2D
  const int32_t k = (int32_t)blockIdx.z;       // z in 3D (0 in 2D)
  const int64_t P = dim == 3 ? (int64_t)nx * ny : (int64_t)nx;
  const int64_t ns = dim == 3 ? nz : ny;
  const int64_t sl = dim == 3 ? k : j;         // slab-plane index
  const int64_t l0 = (dim == 3 ? (int64_t)k * P + (int64_t)j * nx : (int64_t)j * nx) + i0;
  const int64_t e0 = l0 + (lo ? P : 0);
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  const bool has_lo = sl > 0 || lo, has_hi = sl < ns - 1 || hi;
  const bool has_ym = dim == 3 && j > 0, has_yp = dim == 3 && j < ny - 1;
  // the values each row reads: own pair, its x neighbours, the y and slab neighbours
  double xc[R], xlo[R], xhi[R], xym[R], xyp[R];
  double xm1, xpR;
  if constexpr (V2) {
    const double2 c = *reinterpret_cast<const double2*>(x + e0);
    xc[0] = c.x;
    xc[1] = c.y;
    xm1 = i0 > 0 ? x[e0 - 1] : 0.0;
    xpR = i0 + 2 < nx ? x[e0 + 2] : 0.0;
    if (has_lo) { const double2 v = *reinterpret_cast<const double2*>(x + e0 - P); xlo[0] = v.x; xlo[1] = v.y; }
    if (has_hi) { const double2 v = *reinterpret_cast<const double2*>(x + e0 + P); xhi[0] = v.x; xhi[1] = v.y; }
    if (has_ym) { const double2 v = *reinterpret_cast<const double2*>(x + e0 - nx); xym[0] = v.x; xym[1] = v.y; }
    if (has_yp) { const double2 v = *reinterpret_cast<const double2*>(x + e0 + nx); xyp[0] = v.x; xyp[1] = v.y; }
  } else {
    xc[0] = x[e0];
    xm1 = i0 > 0 ? x[e0 - 1] : 0.0;
    xpR = i0 + 1 < nx ? x[e0 + 1] : 0.0;
    if (has_lo) xlo[0] = x[e0 - P];
    if (has_hi) xhi[0] = x[e0 + P];
    if (has_ym) xym[0] = x[e0 - nx];
    if (has_yp) xyp[0] = x[e0 + nx];
  }
  auto S = [&](double v) { return MODE == MSK_SPMV_SCALED ? v * sc : v; };
  double out[R], vo[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int32_t i = i0 + r;
    const double left = r == 0 ? xm1 : xc[r - 1];
    const double right = r == R - 1 ? xpR : xc[r + 1];
    double s = 0.0;
    if (has_lo) s = s + cf.c[0] * S(xlo[r]);
    if (has_ym) s = s + cf.c[1] * S(xym[r]);
    if (i > 0) s = s + cf.c[2] * S(left);
    const double xd = S(xc[r]);
    s = s + cf.c[3] * xd;
    if (i < nx - 1) s = s + cf.c[4] * S(right);
    if (has_yp) s = s + cf.c[5] * S(xyp[r]);
    if (has_hi) s = s + cf.c[6] * S(xhi[r]);
    out[r] = s;
    vo[r] = xd;
  }
  if constexpr (V2) {
    if (MODE == MSK_SPMV_RESID) {
      const double2 bb = *reinterpret_cast<const double2*>(b + l0);
      out[0] = bb.x - out[0];
      out[1] = bb.y - out[1];
    }
    *reinterpret_cast<double2*>(y + l0) = make_double2(out[0], out[1]);
    if (MODE == MSK_SPMV_SCALED && vout) *reinterpret_cast<double2*>(vout + l0) = make_double2(vo[0], vo[1]);
  } else {
    y[l0] = MODE == MSK_SPMV_RESID ? b[l0] - out[0] : out[0];
    if (MODE == MSK_SPMV_SCALED && vout) vout[l0] = vo[0];
  }
}

// ------------------------------------------ DV storage (delta/value dictionary)
// The same assembled matrix, its entries stored as one byte each: entry k of
// row r is code[k], naming the pair (col - r, value) in a per-matrix
// dictionary of at most 256 pairs, and row r holds len[r] <= 255 entries.  Row
// starts come from the scan of len inside the workgroup, block starts from the
// CSR rowptr at multiples of 256.  A 7-point operator needs 7 pairs, so an
// entry moves 1 byte instead of 12 (col + val) and a row ~8 instead of ~88.
// The entries keep the CSR order, so each row's sum is MatMult_SeqAIJ's
// sequence term for term and results equal k_spmv_lds8's bit for bit.
template <int MODE>
__global__ __launch_bounds__(kT) void k_spmv_dv(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                const uint8_t* __restrict__ len8, const uint8_t* __restrict__ code8,
                                                const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                                int ndict, const double* __restrict__ x, const double* __restrict__ b,
                                                double* __restrict__ y, const double* __restrict__ sdev,
                                                double* __restrict__ vout, const int* __restrict__ stop, XcdMap xm) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // the block's codes
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  __shared__ int32_t wtot[kT / 64];
  const uint8_t* scode = reinterpret_cast<const uint8_t*>(smem);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int32_t r0 = row_block(xm) * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s16 = start & ~15;
  const int32_t n16 = (end - s16 + 15) >> 4;
  const int32_t r = r0 + t;
  int32_t len = 0;
  double bb = 0.0;
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  if (r < r1) {
    len = len8[r];
    if (MODE == MSK_SPMV_RESID) bb = b[r];
    if (MODE == MSK_SPMV_SCALED && vout) vout[r] = x[r] * sc;
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  const uint4* c16 = reinterpret_cast<const uint4*>(code8 + s16);
  for (int32_t i = t; i < n16; i += kT) reinterpret_cast<uint4*>(smem)[i] = c16[i];
  // exclusive scan of the row lengths: wave inclusive scan, then the waves before
  int32_t inc = len;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t u = __shfl_up(inc, off, 64);
    if (lane >= off) inc += u;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int32_t k0 = (start - s16) + inc - len;
#pragma unroll
  for (int u = 0; u < kT / 64 - 1; ++u)
    if (u < w) k0 += wtot[u];
  if (r < r1) {
    double s = 0.0;
    for (int32_t q0 = 0; q0 < len; q0 += 8) {
      double av[8], xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // 8 gathers in flight, entries clamped to the row
        const int c = scode[k0 + min(q0 + q, len - 1)];
        av[q] = sval[c];
        xv[q] = x[r + sdel[c]];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (MODE == MSK_SPMV_SCALED) xv[q] = xv[q] * sc;
        if (q0 + q < len) s = s + av[q] * xv[q];
      }
    }
    y[r] = MODE == MSK_SPMV_RESID ? bb - s : s;
  }
}

// The same over blocks of RPL*256 rows: lane t takes rows t, t+256, ..
// (each sub-block of 256 rows coalesced), all RPL rows' gathers issued before
// the first product, so one block's chain of dependent loads (rowptr -> codes
// -> x) covers RPL times the rows.  Row lengths arrive as RPL consecutive
// bytes per lane; the scan runs over those and hands each row its code offset
// through LDS.
template <int MODE, int RPL>
__global__ __launch_bounds__(kT) void k_spmv_dvb(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                 const uint8_t* __restrict__ len8, const uint8_t* __restrict__ code8,
                                                 const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                                 int ndict, const double* __restrict__ x,
                                                 const double* __restrict__ b, double* __restrict__ y,
                                                 const double* __restrict__ sdev, double* __restrict__ vout,
                                                 const int* __restrict__ stop) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  constexpr int RB = kT * RPL;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // the block's codes
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  __shared__ int32_t soff[RB];
  __shared__ int32_t wtot[kT / 64];
  const uint8_t* scode = reinterpret_cast<const uint8_t*>(smem);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int32_t r0 = (int32_t)blockIdx.x * RB;
  const int32_t r1 = min(r0 + RB, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s16 = start & ~15;
  const int32_t n16 = (end - s16 + 15) >> 4;
  // lengths of rows r0 + RPL*t + j
  int32_t l[RPL];
  const int32_t rl = r0 + RPL * t;
  if (rl + RPL <= r1) {
    if constexpr (RPL == 4) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(len8 + rl);
#pragma unroll
      for (int j = 0; j < 4; ++j) l[j] = (v >> (8 * j)) & 255;
    } else if constexpr (RPL == 2) {
      const uint16_t v = *reinterpret_cast<const uint16_t*>(len8 + rl);
      l[0] = v & 255;
      l[1] = v >> 8;
    } else {
      l[0] = len8[rl];
    }
  } else {
#pragma unroll
    for (int j = 0; j < RPL; ++j) l[j] = rl + j < r1 ? len8[rl + j] : 0;
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  const uint4* c16 = reinterpret_cast<const uint4*>(code8 + s16);
  for (int32_t i = t; i < n16; i += kT) reinterpret_cast<uint4*>(smem)[i] = c16[i];
  int32_t tot = 0;
#pragma unroll
  for (int j = 0; j < RPL; ++j) tot += l[j];
  int32_t inc = tot;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t u = __shfl_up(inc, off, 64);
    if (lane >= off) inc += u;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int32_t k = (start - s16) + inc - tot;
#pragma unroll
  for (int u = 0; u < kT / 64 - 1; ++u)
    if (u < w) k += wtot[u];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    soff[RPL * t + j] = (k << 8) | l[j];  // offset (< 2^23) and length packed
    k += l[j];
  }
  __syncthreads();
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  int32_t k0[RPL], ln[RPL];
  int32_t lmax = 0;
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    const int32_t pk = r < r1 ? soff[t + kT * j] : 0;
    k0[j] = pk >> 8;
    ln[j] = pk & 255;
    lmax = max(lmax, ln[j]);
  }
  double s[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) s[j] = 0.0;
  for (int32_t q0 = 0; q0 < lmax; q0 += 8) {
    double av[RPL][8], xv[RPL][8];
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const int32_t r = r0 + t + kT * j;
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // every row's gathers in flight together, entries clamped to the row
        if (ln[j] > 0) {
          const int c = scode[k0[j] + min(q0 + q, ln[j] - 1)];
          av[j][q] = sval[c];
          xv[j][q] = x[r + sdel[c]];
        } else {
          av[j][q] = 0.0;
          xv[j][q] = 0.0;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (MODE == MSK_SPMV_SCALED) xv[j][q] = xv[j][q] * sc;
        if (q0 + q < ln[j]) s[j] = s[j] + av[j][q] * xv[j][q];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    if (r < r1) {
      if (MODE == MSK_SPMV_SCALED && vout) vout[r] = x[r] * sc;
      y[r] = MODE == MSK_SPMV_RESID ? b[r] - s[j] : s[j];
    }
  }
}

// DV storage in ELL layout, for matrices whose rows hold at most 16 entries:
// row r's codes are the W bytes at r*W (W = 4, 8 or 16), its entries in CSR
// order followed by code 255 (no entry).  A lane reads its row's codes with
// one 4/8/16-byte load -- no row pointers, no scan, no LDS stage -- so the
// chain of dependent loads per row is codes -> x -> y.  RPL rows per lane
// (t, t+256, ..) keep RPL*W gathers in flight.  Each row's sum is the CSR
// sequence term for term (code 255 entries are skipped, not added as zeros).
template <int W>
struct EllWord;
template <>
struct EllWord<4> {
  typedef uint32_t T;
  static __device__ __forceinline__ int byte(const T& v, int q) { return (v >> (8 * q)) & 255; }
  static __device__ __forceinline__ T empty() { return 0xFFFFFFFFu; }
};
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <>
struct EllWord<8> {
  typedef u32x2 T;
  static __device__ __forceinline__ int byte(const T& v, int q) {
    return ((q < 4 ? v.x : v.y) >> (8 * (q & 3))) & 255;
  }
  static __device__ __forceinline__ T empty() { return T{0xFFFFFFFFu, 0xFFFFFFFFu}; }
};
template <>
struct EllWord<16> {
  typedef u32x4 T;
  static __device__ __forceinline__ int byte(const T& v, int q) {
    const uint32_t w = q < 4 ? v.x : q < 8 ? v.y : q < 12 ? v.z : v.w;
    return (w >> (8 * (q & 3))) & 255;
  }
  static __device__ __forceinline__ T empty() { return T{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}; }
};

// Block order of the ELL SpMV.  xwin > 0: in each window of 8*xwin blocks, XCD x
// (blockIdx % 8) takes the x-th contiguous run of xwin blocks, so neighbouring row
// blocks -- which share the +-1 / +-line x gathers across their edges -- run on one
// XCD and meet in its L2.  Pays for long lines (512^3: 833 -> 772 us, 1024-wide:
// see DESIGN), costs 2-4 % at 256^3 (tools/ell_lab.hip, profiles/r02/ell_lab/), so
// msk_spmv_dv turns it on from 2^18 rows per plane.  Tail blocks keep their order.
__device__ __forceinline__ int32_t ell_block(int32_t xwin) {
  const int32_t i = (int32_t)blockIdx.x;
  if (xwin <= 0) return i;
  const int32_t span = 8 * xwin;
  const int32_t full = (int32_t)(gridDim.x / (unsigned)span) * span;
  if (i >= full) return i;
  const int32_t w = i / span, rem = i - w * span;
  return w * span + (rem & 7) * xwin + (rem >> 3);
}

template <int MODE, int W, int RPL, bool NTY>
__global__ __launch_bounds__(kT) void k_spmv_ell(int32_t nrows, const uint8_t* __restrict__ code8,
                                                 const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                                 int ndict, const double* __restrict__ x,
                                                 const double* __restrict__ b, double* __restrict__ y,
                                                 const double* __restrict__ sdev, double* __restrict__ vout,
                                                 const int* __restrict__ stop, int32_t xwin) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  typedef EllWord<W> EW;
  typedef typename EW::T CT;
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r0 = ell_block(xwin) * (kT * RPL);
  CT cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const CT*>(code8) + r) : EW::empty();
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  __syncthreads();
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  double xv[RPL][W];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const int c = EW::byte(cw[j], q);
      xv[j][q] = c != 255 ? x[r + sdel[c]] : 0.0;
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const int c = EW::byte(cw[j], q);
      if (c != 255) {
        const double xx = MODE == MSK_SPMV_SCALED ? xv[j][q] * sc : xv[j][q];
        s = s + sval[c] * xx;
      }
    }
    if (r < nrows) {
      if (MODE == MSK_SPMV_SCALED && vout) st_pol<NTY>(vout + r, x[r] * sc);
      st_pol<NTY>(y + r, MODE == MSK_SPMV_RESID ? b[r] - s : s);
    }
  }
}

// The march kernels name neighbours e = 0..6 as (-P, -nx, -1, 0, +1, +nx, +P).  A 2D box
// stencil (d2 = 1) is marched as a 3D box of nx x 1 x ny: its five codes (-nx, -1, 0, +1,
// +nx) are neighbours 0, 2, 3, 4, 6 with P = nx.
template <bool D2>
__device__ __forceinline__ int march_code(int c) { return D2 ? c + (c >= 1) + (c >= 4) : c; }
template <bool D2>
__device__ __forceinline__ void march_values(const double* __restrict__ dval, double* v) {
  if constexpr (D2) {
    v[0] = dval[0];
    v[1] = 0.0;
    v[2] = dval[1];
    v[3] = dval[2];
    v[4] = dval[3];
    v[5] = 0.0;
    v[6] = dval[4];
  } else {
#pragma unroll
    for (int e = 0; e < 7; ++e) v[e] = dval[e];
  }
}

// The ELL SpMV of a 3D box stencil, marching in z.  The dictionary is the stencil's
// seven pairs in column order (-P, -nx, -1, 0, +1, +nx, +P) -- the host guarantees it
// (msp_mat_create_box_convdiff, lo = hi = 0) -- so code e always names neighbour e
// and a row's codes only say which neighbours exist: the kernels read them as one
// presence byte per row (bit e: neighbour e; k_march_mask builds it from the ELL codes
// at assembly), 1 B/row instead of the 8 code bytes.  A workgroup owns 256
// consecutive rows of a plane (a 256-wide x segment of one y line when nx % 256 == 0;
// parts of several lines otherwise, the plane's last segment ragged) and marches
// zt planes: x(z-1), x(z), x(z+1) stay in registers, x(y-+1) = x[r -+ nx] are
// coalesced loads, x(i-+1) come from the segment's row in LDS.  No gathers.  A
// neighbour is read only where it lies inside the plane, and added only where the
// row's codes name it.  xwin > 0: XCD x takes runs of xwin consecutive workgroups
// (ell_block), i.e. neighbouring segments of one z tile, so the x(y-+1) loads of one
// workgroup are the x(z) rows of its neighbours and meet in that XCD's L2.  With
// xwin = 32 (tools/ell_lab.hip, back to back): 256^3 92 -> 74 us, 512^3 821 -> 628 us; in identity
// order 99 / 697 us (profiles/r02/ell_lab/).  Inside the GMRES step: 103 -> 82 us (rocprof).  The products are added in CSR order
// from 0.0, the same terms as k_spmv_ell, so the result is bitwise identical.
template <int MODE, bool NTY, bool D2>
__global__ __launch_bounds__(kT) void k_spmv_box_march(int32_t nx, int32_t ny, int32_t nz,
                                                       const uint8_t* __restrict__ mask,
                                                       const double* __restrict__ dval, const double* __restrict__ x,
                                                       const double* __restrict__ b, double* __restrict__ y,
                                                       const double* __restrict__ sdev, double* __restrict__ vout,
                                                       const int* __restrict__ stop, int32_t zt, int32_t xwin) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  __shared__ double sx[kT + 2];
  const int t = threadIdx.x;
  const int32_t P = nx * ny;  // nx * ny * nz <= INT32_MAX (checked by the launcher)
  const int32_t nps = (P + kT - 1) / kT;
  const int32_t bid = ell_block(xwin);
  const int32_t z0 = (bid / nps) * zt, z1 = min(z0 + zt, nz);
  const int32_t rl = (bid % nps) * kT + t;  // the row's offset within its plane
  const bool in = rl < P;
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  double v[7];
  march_values<D2>(dval, v);
  const bool hs = in && rl >= nx, hn = in && rl + nx < P, hl = t == 0 && rl > 0, hr = t == kT - 1 && rl + 1 < P;
  double xm = in && z0 > 0 ? x[rl + (int64_t)(z0 - 1) * P] : 0.0;
  double xc = in ? x[rl + (int64_t)z0 * P] : 0.0;
  for (int32_t z = z0; z < z1; ++z) {
    const int64_t r = rl + (int64_t)z * P;
    const uint32_t m = in ? __builtin_nontemporal_load(mask + r) : 0u;
    const double xp = in && z + 1 < nz ? x[r + P] : 0.0;
    const double xs = hs ? x[r - nx] : 0.0;
    const double xn = hn ? x[r + nx] : 0.0;
    const double el = hl ? x[r - 1] : 0.0;
    const double er = hr ? x[r + 1] : 0.0;
    __syncthreads();  // the previous plane's reads of sx are done
    sx[t + 1] = xc;
    if (t == 0) sx[0] = el;
    if (t == kT - 1) sx[kT + 1] = er;
    __syncthreads();
    const double xl = sx[t], xr = sx[t + 2];
    const double xq[7] = {xm, xs, xl, xc, xr, xn, xp};
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < 7; ++e)
      if (m & (1u << e)) s = s + v[e] * (MODE == MSK_SPMV_SCALED ? xq[e] * sc : xq[e]);
    if (in) {
      if (MODE == MSK_SPMV_SCALED && vout) st_pol<NTY>(vout + r, xc * sc);
      st_pol<NTY>(y + r, MODE == MSK_SPMV_RESID ? b[r] - s : s);
    }
    xm = xc;
    xc = xp;
  }
}

// The same march over tiles of L whole y lines (nx % 256 == 0): a workgroup owns a
// 256-wide x segment of L consecutive lines; the tile's x(z) rows and the two halo line
// segments (y0 - 1 and y0 + L) go to LDS each plane, so x(y-+1) of interior lines is
// read from LDS and only 2 / L halo loads per row remain (against 2 for one line).
// Lines past ny are idle (a ragged last tile).  Back to back: 256^3 74 us against 82 for one
// line, 512^3 590 against 679 (profiles/r02/march/sizes4/); inside the GMRES step 82 against 85 us,
// SMSM block 283 against 301 (march/lines_ab/).
// Bitwise k_spmv_box_march (same terms, same order).
template <int MODE, bool NTY, int L, bool D2 = false>
__global__ __launch_bounds__(kT) void k_spmv_box_lines(int32_t nx, int32_t ny, int32_t nz,
                                                       const uint8_t* __restrict__ mask,
                                                       const double* __restrict__ dval, const double* __restrict__ x,
                                                       const double* __restrict__ b, double* __restrict__ y,
                                                       const double* __restrict__ sdev, double* __restrict__ vout,
                                                       const int* __restrict__ stop, int32_t zt, int32_t xwin) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  __shared__ double sx[L + 2][kT + 2];
  const int t = threadIdx.x;
  const int32_t nseg = nx / kT, nyt = (ny + L - 1) / L;
  const int32_t bid = ell_block(xwin);
  const int32_t seg = bid % nseg, yt = (bid / nseg) % nyt, z0 = (bid / (nseg * nyt)) * zt;
  const int32_t z1 = min(z0 + zt, nz), y0 = yt * L;
  const int32_t i = seg * kT + t;
  const int32_t P = nx * ny;  // nx * ny * nz <= INT32_MAX (checked by the launcher)
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  double v[7];
  march_values<D2>(dval, v);
  double xm[L], xc[L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const bool ok = y0 + l < ny;
    const int32_t rl = i + (y0 + l) * nx;
    xm[l] = ok && z0 > 0 ? x[rl + (int64_t)(z0 - 1) * P] : 0.0;
    xc[l] = ok ? x[rl + (int64_t)z0 * P] : 0.0;
  }
  const bool hs = y0 > 0, hn = y0 + L < ny, hl = t == 0 && i > 0, hr = t == kT - 1 && i + 1 < nx;
  for (int32_t z = z0; z < z1; ++z) {
    const int64_t zP = (int64_t)z * P;
    uint32_t mk[L];
    double xp[L], el[L], er[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const bool ok = y0 + l < ny;
      const int64_t r = i + (int64_t)(y0 + l) * nx + zP;
      mk[l] = ok ? __builtin_nontemporal_load(mask + r) : 0u;
      xp[l] = ok && z + 1 < nz ? x[r + P] : 0.0;
      el[l] = ok && hl ? x[r - 1] : 0.0;
      er[l] = ok && hr ? x[r + 1] : 0.0;
    }
    const int64_t rb = i + (int64_t)y0 * nx + zP;
    const double hsv = hs ? x[rb - nx] : 0.0;
    const double hnv = hn ? x[rb + (int64_t)L * nx] : 0.0;
    __syncthreads();  // the previous plane's reads of sx are done
    sx[0][t + 1] = hsv;
    sx[L + 1][t + 1] = hnv;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      sx[l + 1][t + 1] = xc[l];
      if (t == 0) sx[l + 1][0] = el[l];
      if (t == kT - 1) sx[l + 1][kT + 1] = er[l];
    }
    __syncthreads();
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const uint32_t m = mk[l];
      const double xq[7] = {xm[l], sx[l][t + 1], sx[l + 1][t], xc[l], sx[l + 1][t + 2], sx[l + 2][t + 1], xp[l]};
      double s = 0.0;
#pragma unroll
      for (int e = 0; e < 7; ++e)
        if (m & (1u << e)) s = s + v[e] * (MODE == MSK_SPMV_SCALED ? xq[e] * sc : xq[e]);
      if (y0 + l < ny) {
        const int64_t r = i + (int64_t)(y0 + l) * nx + zP;
        if (MODE == MSK_SPMV_SCALED && vout) st_pol<NTY>(vout + r, xc[l] * sc);
        st_pol<NTY>(y + r, MODE == MSK_SPMV_RESID ? b[r] - s : s);
      }
      xm[l] = xc[l];
      xc[l] = xp[l];
    }
  }
}

// The stencil storage's value of leg k for the lane's row pair j of the chunk at c0 (rows c0 + j*512 + 2t, +1).
// rvs > 0: structure of arrays, rv[k * rvs + row]; rvs == 0: chunk-blocked, the 7 legs of each 512-row slice
// of a chunk next to each other (rv[7 * c0 + j * 3584 + k * 512 + (row % 512)]), so a chunk tile's 229 KB of
// values are one contiguous region instead of seven regions 8n bytes apart.
__device__ __forceinline__ const double2* rv_pair(const double* __restrict__ rv, int64_t rvs, int64_t c0, int k,
                                                  int j, int t) {
  return reinterpret_cast<const double2*>(rvs ? rv + k * rvs + c0 + j * (2 * kT) + 2 * t
                                              : rv + 7 * c0 + j * (7 * 2 * kT) + k * (2 * kT) + 2 * t);
}

// The symmetric stencil storage (rvs < 0; rv_attach checks A[r, r + d] == A[r + d, r] bit for bit): per row only
// the diagonal and the three upper legs, k = 0 d, 1 x+1, 2 y+1, 3 z+1, chunk-blocked (rv[4 * c0 + j * 2048 +
// k * 512 + row % 512]); a row's lower legs are its lower neighbours' upper ones: A[r, r-1] = ux[r-1],
// A[r, r-nx] = uy[r-nx], A[r, r-P] = uz[r-P] -- 32 value bytes per row instead of 56.
__device__ __forceinline__ const double* rvs_at(const double* __restrict__ rv, int64_t row, int k) {
  const int64_t o = row % kChunk;
  return rv + 4 * (row - o) + (o / (2 * kT)) * (4 * 2 * kT) + k * (2 * kT) + o % (2 * kT);
}
__device__ __forceinline__ const double2* rvs_pair(const double* __restrict__ rv, int64_t c0, int k, int j, int t) {
  return reinterpret_cast<const double2*>(rv + 4 * c0 + j * (4 * 2 * kT) + k * (2 * kT) + 2 * t);
}

// Symmetric storage, one plane of a chunk tile: the lane's own four legs (prefetched with x(z+1)), then the x+1 /
// y+1 legs of the window [c0 - nx, c0 + 4096) to LDS (sux, suy; the window's first nx rows are the line below the
// tile), so that a row's x-1 / y-1 values are read where its neighbour's upper legs lie.
struct SymTile {
  double2 own[kIters][4];
  double2 hx, hy;  // lane t < nx/2: the halo line's x+1 / y+1 legs at c0 - nx + 2t
};

__device__ __forceinline__ void sym_load(SymTile& st, const double* __restrict__ rv, int64_t c0, int nx, int t) {
#pragma unroll
  for (int j = 0; j < kIters; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) st.own[j][k] = ld_nt(rvs_pair(rv, c0, k, j, t));
  st.hx = st.hy = make_double2(0.0, 0.0);
  if (t < nx / 2 && c0 - nx >= 0) {
    st.hx = *reinterpret_cast<const double2*>(rvs_at(rv, c0 - nx + 2 * t, 1));
    st.hy = *reinterpret_cast<const double2*>(rvs_at(rv, c0 - nx + 2 * t, 2));
  }
}

// after the barrier that ends the previous plane's LDS reads
__device__ __forceinline__ void sym_store(const SymTile& st, double* sux, double* suy, const double* __restrict__ rv,
                                          int64_t c0, int nx, int t) {
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    *reinterpret_cast<double2*>(sux + nx + j * (2 * kT) + 2 * t) = st.own[j][1];
    *reinterpret_cast<double2*>(suy + nx + j * (2 * kT) + 2 * t) = st.own[j][2];
  }
  if (t < nx / 2) {
    *reinterpret_cast<double2*>(sux + 2 * t) = st.hx;
    *reinterpret_cast<double2*>(suy + 2 * t) = st.hy;
  }
  for (int i = t + kT; i < nx / 2; i += kT) {  // nx > 512: the rest of the halo line
    const bool in = c0 - nx >= 0;
    *reinterpret_cast<double2*>(sux + 2 * i) =
        in ? *reinterpret_cast<const double2*>(rvs_at(rv, c0 - nx + 2 * i, 1)) : make_double2(0.0, 0.0);
    *reinterpret_cast<double2*>(suy + 2 * i) =
        in ? *reinterpret_cast<const double2*>(rvs_at(rv, c0 - nx + 2 * i, 2)) : make_double2(0.0, 0.0);
  }
}

// the seven values of row (j, q) in column order: z-1 (carried uz of the plane below), y-1, x-1 (LDS), d, x+1,
// y+1, z+1 (own); e = the row's window index (nx + j * 512 + 2t + q)
__device__ __forceinline__ void sym_values(const SymTile& st, const double* sux, const double* suy, double uzm, int j,
                                           int q, int e, int nx, double (&vv)[7]) {
  vv[0] = uzm;
  vv[1] = suy[e - nx];
  vv[2] = sux[e - 1];
  vv[3] = q ? st.own[j][0].y : st.own[j][0].x;
  vv[4] = q ? st.own[j][1].y : st.own[j][1].x;
  vv[5] = q ? st.own[j][2].y : st.own[j][2].x;
  vv[6] = q ? st.own[j][3].y : st.own[j][3].x;
}

// The box march over DBR chunk tiles (planes of whole chunks: P % 4096 == 0), for MatMult, MatResidual
// and the scaled MatMult on their own: the tiling of k_box_spmv_mdot_march without the dots.  A lane owns
// 16 rows of the tile (rows 2t, 2t+1 + 512j) and loads x, x(z+1), b and the presence bytes as 16- and
// 2-byte vectors, so each lane keeps 8 x(z+1) loads and 8 b loads in flight where the line kernels keep
// one; the tile's window [-nx, 4096+nx) of plane z is in LDS.  Same terms in the same order as
// k_spmv_box_march: bitwise its products.
// RV (the stencil storage, MSP_STORAGE_STENCIL): each row's seven values from the per-leg arrays
// rv[e * rvs + row] (0 where the row has no such neighbour, never added) instead of the dictionary: a box
// stencil with variable coefficients, 56 value bytes per row read as 16-byte non-temporal vectors, against
// 88 bytes of CSR (col + val + rowptr).  Same terms, same order: bitwise the CSR kernels' sums.
// RV: 0 dictionary, 1 the seven per-row legs, 2 the symmetric storage (SymTile; lanes carry uz of the plane below).
template <int MODE, bool NTY, int RV>
__global__ __launch_bounds__(kT) void k_box_march_chunk(int32_t nx, int64_t P, int32_t nz, int32_t zt, int xcd,
                                                        int halo, const uint8_t* __restrict__ mask,
                                                        const double* __restrict__ dval,
                                                        const double* __restrict__ rv, int64_t rvs,
                                                        const double* __restrict__ x,
                                                        const double* __restrict__ b, double* __restrict__ y,
                                                        const double* __restrict__ sdev, double* __restrict__ vout,
                                                        const int* __restrict__ stop) {
  if (MODE == MSK_SPMV_SCALED && stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sx = reinterpret_cast<double*>(smem);  // window of plane z: kChunk + 2 nx doubles
  const int t = threadIdx.x;
  const int64_t cpp = P / kChunk;
  int64_t tile, zg;
  if (xcd) {  // XCD-contiguous eighths of the plane's tiles (as k_box_spmv_mdot_march)
    const int64_t per = cpp / 8, slot = blockIdx.x / 8;
    tile = (blockIdx.x % 8) * per + slot % per;
    zg = slot / per;
  } else {
    tile = blockIdx.x % cpp;
    zg = blockIdx.x / cpp;
  }
  const int32_t z0 = (int32_t)zg * zt, z1 = min(z0 + zt, nz);
  const double sc = MODE == MSK_SPMV_SCALED ? *sdev : 1.0;
  double v[7];
  if constexpr (!RV) march_values<false>(dval, v);
  const int nh = nx / 2;  // double2 per halo line
  double xm[2 * kIters], xc[2 * kIters], xp[2 * kIters];
  double* sux = sx + kChunk + 2 * nx;  // RV == 2: x+1 / y+1 legs of the window [c0 - nx, c0 + 4096)
  double* suy = sux + kChunk + nx;
  double uzm[RV == 2 ? 2 * kIters : 1];  // RV == 2: uz of the lane's rows one plane below
  if constexpr (RV == 2) {
    const int64_t cb = ((int64_t)z0 - 1) * P + tile * kChunk;
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 u = z0 > 0 ? ld_nt(rvs_pair(rv, cb, 3, j, t)) : make_double2(0.0, 0.0);
      uzm[2 * j] = u.x;
      uzm[2 * j + 1] = u.y;
    }
  }
  {
    const int64_t b0 = (int64_t)z0 * P + tile * kChunk + 2 * t;
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 a = *reinterpret_cast<const double2*>(x + b0 + j * (2 * kT));
      xc[2 * j] = a.x;
      xc[2 * j + 1] = a.y;
      if (z0 > 0 || (halo & 1)) {  // halo & 1: the plane below the box is the column space's lo plane
        const double2 m2 = *reinterpret_cast<const double2*>(x + b0 - P + j * (2 * kT));
        xm[2 * j] = m2.x;
        xm[2 * j + 1] = m2.y;
      } else {
        xm[2 * j] = xm[2 * j + 1] = 0.0;
      }
    }
  }
  for (int32_t z = z0; z < z1; ++z) {
    const int64_t c0 = ((int64_t)z * cpp + tile) * kChunk, base = c0 + 2 * t;
    uint32_t m[kIters];
    double2 bb[kIters];
#pragma unroll
    for (int j = 0; j < kIters; ++j) {  // plane z+1, b, the presence bytes: issued before the LDS turn-around
      if (z + 1 < nz || (halo & 2)) {  // halo & 2: the plane above the box is the hi plane
        const double2 p2 = *reinterpret_cast<const double2*>(x + base + P + j * (2 * kT));
        xp[2 * j] = p2.x;
        xp[2 * j + 1] = p2.y;
      } else {
        xp[2 * j] = xp[2 * j + 1] = 0.0;
      }
      m[j] = *reinterpret_cast<const uint16_t*>(mask + base + j * (2 * kT));
      if constexpr (MODE == MSK_SPMV_RESID) bb[j] = ld_nt(reinterpret_cast<const double2*>(b + base + j * (2 * kT)));
    }
    SymTile st;
    if constexpr (RV == 2) sym_load(st, rv, c0, nx, t);
    double2 hl = make_double2(0.0, 0.0), hh = make_double2(0.0, 0.0);
    const bool hasl = t < nh && c0 - nx >= 0, hash = t < nh && c0 + kChunk + nx <= (int64_t)nz * P;
    if (hasl) hl = *reinterpret_cast<const double2*>(x + c0 - nx + 2 * t);
    if (hash) hh = *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * t);
    __syncthreads();  // the previous plane's window reads are done
#pragma unroll
    for (int j = 0; j < kIters; ++j)
      *reinterpret_cast<double2*>(sx + nx + j * (2 * kT) + 2 * t) = make_double2(xc[2 * j], xc[2 * j + 1]);
    if (t < nh) {
      *reinterpret_cast<double2*>(sx + 2 * t) = hl;
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * t) = hh;
    }
    for (int i = t + kT; i < nh; i += kT) {  // nx > 512: the rest of the halo lines
      *reinterpret_cast<double2*>(sx + 2 * i) =
          c0 - nx >= 0 ? *reinterpret_cast<const double2*>(x + c0 - nx + 2 * i) : make_double2(0.0, 0.0);
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * i) =
          c0 + kChunk + nx <= (int64_t)nz * P ? *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * i)
                                              : make_double2(0.0, 0.0);
    }
    if constexpr (RV == 2) sym_store(st, sux, suy, rv, c0, nx, t);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      double2 rq[7];
      if constexpr (RV == 1) {
#pragma unroll
        for (int k = 0; k < 7; ++k) rq[k] = ld_nt(rv_pair(rv, rvs, c0, k, j, t));
      }
      double o[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = j * (2 * kT) + 2 * t + q + nx;
        const uint32_t mr = (m[j] >> (8 * q)) & 255u;
        const double xq[7] = {xm[2 * j + q], sx[e - nx], sx[e - 1], xc[2 * j + q], sx[e + 1], sx[e + nx],
                              xp[2 * j + q]};
        double vv[7];
        if constexpr (RV == 2) sym_values(st, sux, suy, uzm[2 * j + q], j, q, e, nx, vv);
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const double vk = RV == 2 ? vv[k] : RV ? (q ? rq[k].y : rq[k].x) : v[k];
          if (mr & (1u << k)) s = s + vk * (MODE == MSK_SPMV_SCALED ? xq[k] * sc : xq[k]);
        }
        if constexpr (MODE == MSK_SPMV_RESID) s = (q ? bb[j].y : bb[j].x) - s;
        o[q] = s;
      }
      const int64_t r = base + j * (2 * kT);
      if constexpr (NTY) {
        dx2 w2;
        w2.x = o[0];
        w2.y = o[1];
        __builtin_nontemporal_store(w2, reinterpret_cast<dx2*>(y + r));
      } else {
        *reinterpret_cast<double2*>(y + r) = make_double2(o[0], o[1]);
      }
      if (MODE == MSK_SPMV_SCALED && vout) {
        if constexpr (NTY) {
          dx2 w2;
          w2.x = xc[2 * j] * sc;
          w2.y = xc[2 * j + 1] * sc;
          __builtin_nontemporal_store(w2, reinterpret_cast<dx2*>(vout + r));
        } else {
          *reinterpret_cast<double2*>(vout + r) = make_double2(xc[2 * j] * sc, xc[2 * j + 1] * sc);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2 * kIters; ++i) {
      xm[i] = xc[i];
      xc[i] = xp[i];
    }
    if constexpr (RV == 2) {
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        uzm[2 * j] = st.own[j][3].x;
        uzm[2 * j + 1] = st.own[j][3].y;
      }
    }
  }
}

// The GMRES step's MatMult of a box stencil fused with the VecMDot after it.  Workgroup c owns
// DBR chunk c and computes W = A (sc x) for its rows in the DBR lane layout (lane t: rows
// c*4096 + j*512 + 2t, +1), so W never leaves the registers before the dots: the MDot
// reads the nv basis vectors but not W (8 bytes per row less).  The chunk's x window
// [c*4096 - nx, c*4096 + 4096 + nx) -- every x-+1 and y-+1 neighbour of its rows -- is staged
// in LDS; x(z-+1) are coalesced loads.  A row adds v[e] * (x[r + delta_e] * sc) for the
// neighbours its presence byte names, e = 0..6 in column order from 0.0: the march kernels'
// terms in their order, so W is bitwise k_spmv_box_march's, and each dot is dot_chunk's.
// Neighbours are read at their global index, so unlike the march this needs no edge check.
template <bool D2, int VAR, bool NTY>
__global__ __launch_bounds__(kT) void k_box_spmv_mdot(int32_t nx, int64_t P, int64_t n, const uint8_t* __restrict__ mask,
                                                      const double* __restrict__ dval, const double* __restrict__ x,
                                                      const double* __restrict__ sdev, double* __restrict__ y, Vecs V,
                                                      int nv, double* __restrict__ partial, int64_t nchunks,
                                                      const int* __restrict__ stop) {
  if (stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sx = reinterpret_cast<double*>(smem);  // window of kChunk + 2 nx doubles
  __shared__ double red[MSK_MAX_GROUP][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t c = blockIdx.x, c0 = c * kChunk, lo = c0 - nx;
  const int64_t base = c0 + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  const int wlen = kChunk + 2 * nx;
  if ((nx & 1) == 0 && lo >= 0 && lo + wlen <= n) {  // 16-byte aligned interior window
    const double2* x2 = reinterpret_cast<const double2*>(x + lo);
    for (int i = t; i < wlen / 2; i += kT) reinterpret_cast<double2*>(sx)[i] = x2[i];
  } else {
    for (int i = t; i < wlen; i += kT) {
      const int64_t r = lo + i;
      sx[i] = r >= 0 && r < n ? x[r] : 0.0;
    }
  }
  const double sc = *sdev;
  double v[7];
  march_values<D2>(dval, v);
  uint32_t m[2 * kIters];
  double xm[2 * kIters], xp[2 * kIters];
#pragma unroll
  for (int j = 0; j < kIters; ++j) {  // presence bytes and the -+plane neighbours, issued before the LDS wait
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t r = base + j * (2 * kT) + q;
      const uint32_t mr = r < n ? (uint32_t)mask[r] : 0u;
      m[2 * j + q] = mr;
      xm[2 * j + q] = (mr & 1u) ? x[r - P] : 0.0;
      xp[2 * j + q] = (mr & 64u) ? x[r + P] : 0.0;
    }
  }
  __syncthreads();
  double wr[2 * kIters];
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = j * (2 * kT) + 2 * t + q + nx;  // the row's place in the window
      const uint32_t mr = m[2 * j + q];
      const double xq[7] = {xm[2 * j + q], sx[e - nx], sx[e - 1], sx[e], sx[e + 1], sx[e + nx], xp[2 * j + q]};
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 7; ++k)
        if (mr & (1u << k)) s = s + v[k] * (xq[k] * sc);
      wr[2 * j + q] = s;
    }
    const int64_t r = base + j * (2 * kT);
    if (!y) continue;  // uniform: the W-free step (k_box_maxpy recomputes W)
    if (full) {
      if constexpr (NTY) {
        dx2 o;
        o.x = wr[2 * j];
        o.y = wr[2 * j + 1];
        __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(y + r));
      } else {
        *reinterpret_cast<double2*>(y + r) = make_double2(wr[2 * j], wr[2 * j + 1]);
      }
    } else {
      if (r < n) y[r] = wr[2 * j];
      if (r + 1 < n) y[r + 1] = wr[2 * j + 1];
    }
  }
  // VecMDot of W against the nv basis vectors, this chunk (dot_chunk's order)
  if (full) {
    int g = 0;
#pragma unroll 1
    for (; g + 4 <= nv; g += 4) dot_group_full<4, VAR>(wr, V, base, 0, nv, g, red, lane, wv);
    switch (nv - g) {
      case 3: dot_group_full<3, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      case 2: dot_group_full<2, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      case 1: dot_group_full<1, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      default: break;
    }
  } else {
#pragma unroll 1
    for (int vi = 0; vi < nv; ++vi) {
      const double* __restrict__ yv = vec_at(V, vi);
      const double sv = vec_scale(V, vi);
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        const int64_t e = base + j * (2 * kT);
        if (e < n) acc = acc + wr[2 * j] * (yv[e] * sv);
        if (e + 1 < n) acc = acc + wr[2 * j + 1] * (yv[e + 1] * sv);
      }
      acc = wave_butterfly(acc);
      if (lane == 0) red[vi][wv] = acc;
    }
  }
  __syncthreads();
  if (t < nv) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
}

// The same fused step marching in z: when a plane holds a whole number of DBR chunks (P % 4096 == 0),
// chunk c + P/4096 is chunk c's tile one plane up, so workgroup w takes tile w % cpp through zt
// planes.  The lane's own x rows of planes z-1, z, z+1 stay in registers (xm, xc, xp); per plane
// only x(z+1), the two halo lines of the window and the presence bytes are loaded, the window's
// own rows are written to LDS from xc.  W and every dot are the unmarched kernel's, bit for bit.
// RV: the stencil storage's per-row values (as k_box_march_chunk<.., RV>); W is then stored (y != null):
// recomputing it in the MAXPY would re-read the 56 value bytes per row to save W's 16.
// RVP (RV only): the row pairs j < RVP have their values issued with x(z+1), before the LDS turn-around; the
// others right before their W rows (fewer registers held across the barriers; MSPLIT_RV_PREFETCH, the A/B).
template <int VAR, bool NTY, int RV, int RVP = kIters>
__global__ __launch_bounds__(kT) void k_box_spmv_mdot_march(int32_t nx, int64_t P, int32_t nz, int32_t zt, int xcd,
                                                            const uint8_t* __restrict__ mask,
                                                            const double* __restrict__ dval,
                                                            const double* __restrict__ rv, int64_t rvs,
                                                            const double* __restrict__ x,
                                                            const double* __restrict__ sdev, double* __restrict__ y,
                                                            Vecs V, int nv, int self, double* __restrict__ partial,
                                                            int64_t nchunks, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sx = reinterpret_cast<double*>(smem);  // window of plane z: kChunk + 2 nx doubles
  __shared__ double red[MSK_MAX_GROUP][4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t cpp = P / kChunk;
  int64_t tile, zg;
  if (xcd & 1) {  // XCD x (workgroups x, x+8, ...) takes a contiguous eighth of the plane's tiles: neighbouring
                  // tiles share their halo lines through that XCD's L2
    const int64_t per = cpp / 8, slot = blockIdx.x / 8;
    tile = (blockIdx.x % 8) * per + slot % per;
    zg = slot / per;
  } else {
    tile = blockIdx.x % cpp;
    zg = blockIdx.x / cpp;
  }
  if (xcd & 2) zg = (nz + zt - 1) / zt - 1 - zg;  // top plane groups first
  const int32_t z0 = (int32_t)zg * zt, z1 = min(z0 + zt, nz);
  // xcd & 4: odd plane groups march down (round 6).  A group reads one plane of x beyond each end of its range (and,
  // RV == 2, the z+1 leg of the plane below): marching up, the plane below at its start and the plane above at its
  // end, which its neighbour groups read at their opposite ends, a whole group's time apart -- from HBM twice.
  // Groups marching toward each other in pairs meet their neighbours at the shared boundary at the same moment
  // (both start there, or both end there; same tile, same XCD), so the second read finds the first in the L2.
  // The march order changes nothing else: every chunk's terms, sums and stores are the same (bitwise).
  const bool down = RV != 2 && (xcd & 4) && (zg & 1);
  const double sc = *sdev;
  double v[7];
  if constexpr (!RV) march_values<false>(dval, v);
  const int nh = nx / 2;  // double2 per halo line
  double xm[2 * kIters], xc[2 * kIters], xp[2 * kIters];
  double* sux = sx + kChunk + 2 * nx;  // RV == 2 (symmetric storage): x+1 / y+1 legs of the window
  double* suy = sux + kChunk + nx;
  double uzm[RV == 2 ? 2 * kIters : 1];  // RV == 2: uz of the lane's rows one plane below
  if constexpr (RV == 2) {
    const int64_t cb = ((int64_t)z0 - 1) * P + tile * kChunk;
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 u = z0 > 0 ? ld_nt(rvs_pair(rv, cb, 3, j, t)) : make_double2(0.0, 0.0);
      uzm[2 * j] = u.x;
      uzm[2 * j + 1] = u.y;
    }
  }
  {  // xc: the first plane; xm: the plane marched from (z-1 going up, z+1 going down), 0 beyond the box
    const int32_t zf = down ? z1 - 1 : z0;
    const bool hasm = down ? z1 < nz : z0 > 0;
    const int64_t b0 = (int64_t)zf * P + tile * kChunk + 2 * t, bm = b0 + (down ? P : -P);
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 a = *reinterpret_cast<const double2*>(x + b0 + j * (2 * kT));
      xc[2 * j] = a.x;
      xc[2 * j + 1] = a.y;
      if (hasm) {
        const double2 m2 = *reinterpret_cast<const double2*>(x + bm + j * (2 * kT));
        xm[2 * j] = m2.x;
        xm[2 * j + 1] = m2.y;
      } else {
        xm[2 * j] = xm[2 * j + 1] = 0.0;
      }
    }
  }
  for (int32_t zi = 0; zi < z1 - z0; ++zi) {
    const int32_t z = down ? z1 - 1 - zi : z0 + zi;
    const int64_t c = (int64_t)z * cpp + tile, c0 = c * kChunk, base = c0 + 2 * t;
    const bool hasp = down ? z > 0 : z + 1 < nz;  // xp: the plane marched to (z+1 going up, z-1 going down)
    const int64_t dp = down ? -P : P;
    uint32_t m[kIters];
#pragma unroll
    for (int j = 0; j < kIters; ++j) {  // the next plane, the presence bytes: issued before the LDS turn-around
      if (hasp) {
        const double2 p2 = *reinterpret_cast<const double2*>(x + base + dp + j * (2 * kT));
        xp[2 * j] = p2.x;
        xp[2 * j + 1] = p2.y;
      } else {
        xp[2 * j] = xp[2 * j + 1] = 0.0;
      }
      m[j] = *reinterpret_cast<const uint16_t*>(mask + base + j * (2 * kT));
    }
    // RV: the plane's seven value legs for all the lane's rows, issued with x(z+1) before the LDS turn-around (the
    // kernel runs one workgroup per CU, so the unified register file holds them; loaded after the barrier they
    // were a second, exposed round trip per plane)
    double2 rqa[RV == 1 ? kIters : 1][7];
    SymTile st;
    if constexpr (RV == 2) sym_load(st, rv, c0, nx, t);
    if constexpr (RV == 1) {
#pragma unroll
      for (int j = 0; j < RVP; ++j)
#pragma unroll
        for (int k = 0; k < 7; ++k) rqa[j][k] = ld_nt(rv_pair(rv, rvs, c0, k, j, t));
    }
    double2 hl = make_double2(0.0, 0.0), hh = make_double2(0.0, 0.0);
    const bool hasl = t < nh && c0 - nx >= 0, hash = t < nh && c0 + kChunk + nx <= (int64_t)nz * P;
    if (hasl) hl = *reinterpret_cast<const double2*>(x + c0 - nx + 2 * t);
    if (hash) hh = *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * t);
    __syncthreads();  // the previous plane's window reads (and its partial writes) are done
#pragma unroll
    for (int j = 0; j < kIters; ++j)
      *reinterpret_cast<double2*>(sx + nx + j * (2 * kT) + 2 * t) = make_double2(xc[2 * j], xc[2 * j + 1]);
    if (t < nh) {
      *reinterpret_cast<double2*>(sx + 2 * t) = hl;
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * t) = hh;
    }
    for (int i = t + kT; i < nh; i += kT) {  // nx > 512: the rest of the halo lines
      *reinterpret_cast<double2*>(sx + 2 * i) =
          c0 - nx >= 0 ? *reinterpret_cast<const double2*>(x + c0 - nx + 2 * i) : make_double2(0.0, 0.0);
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * i) =
          c0 + kChunk + nx <= (int64_t)nz * P ? *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * i)
                                              : make_double2(0.0, 0.0);
    }
    if constexpr (RV == 2) sym_store(st, sux, suy, rv, c0, nx, t);
    __syncthreads();
    double wr[2 * kIters];
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      if constexpr (RV == 1) {
        if (j >= RVP) {
#pragma unroll
          for (int k = 0; k < 7; ++k) rqa[j][k] = ld_nt(rv_pair(rv, rvs, c0, k, j, t));
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = j * (2 * kT) + 2 * t + q + nx;
        const uint32_t mr = (m[j] >> (8 * q)) & 255u;
        const double xq[7] = {down ? xp[2 * j + q] : xm[2 * j + q], sx[e - nx], sx[e - 1], xc[2 * j + q],
                              sx[e + 1], sx[e + nx], down ? xm[2 * j + q] : xp[2 * j + q]};
        double vv[7];
        if constexpr (RV == 2) sym_values(st, sux, suy, uzm[2 * j + q], j, q, e, nx, vv);
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const double vk = RV == 2 ? vv[k] : RV ? (q ? rqa[RV == 1 ? j : 0][k].y : rqa[RV == 1 ? j : 0][k].x) : v[k];
          if (mr & (1u << k)) s = s + vk * (xq[k] * sc);
        }
        wr[2 * j + q] = s;
      }
      if (!y) continue;  // uniform: W is recomputed by the MAXPY after (k_box_maxpy_march), not stored
      if constexpr (NTY) {
        dx2 o;
        o.x = wr[2 * j];
        o.y = wr[2 * j + 1];
        __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(y + base + j * (2 * kT)));
      } else {
        *reinterpret_cast<double2*>(y + base + j * (2 * kT)) = make_double2(wr[2 * j], wr[2 * j + 1]);
      }
    }
    // self: the last basis vector is x itself, whose rows of this plane the lane holds in xc at exactly
    // its DBR positions: that dot is taken from the registers (8n bytes fewer), the same sum term for term
    const int nvm = nv - self;
    int g = 0;
#pragma unroll 1
    for (; g + 4 <= nvm; g += 4) dot_group_full<4, VAR>(wr, V, base, 0, nv, g, red, lane, wv);
    switch (nvm - g) {
      case 3: dot_group_full<3, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      case 2: dot_group_full<2, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      case 1: dot_group_full<1, VAR>(wr, V, base, 0, nv, g, red, lane, wv); break;
      default: break;
    }
    if (self) {
      const double sv = vec_scale(V, nv - 1);
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        acc = acc + wr[2 * j] * (xc[2 * j] * sv);
        acc = acc + wr[2 * j + 1] * (xc[2 * j + 1] * sv);
      }
      acc = wave_butterfly(acc);
      if (lane == 0) red[nv - 1][wv] = acc;
    }
    __syncthreads();
    if (t < nv) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
#pragma unroll
    for (int i = 0; i < 2 * kIters; ++i) {
      xm[i] = xc[i];
      xc[i] = xp[i];
    }
    if constexpr (RV == 2) {
#pragma unroll
      for (int j = 0; j < kIters; ++j) {
        uzm[2 * j] = st.own[j][3].x;
        uzm[2 * j + 1] = st.own[j][3].y;
      }
    }
  }
}

// The symmetric STENCIL fused step with two threads per DBR lane (round 5): 512 threads a tile, thread t < 256 takes
// the lane's row pairs j = 0..3, thread t + 256 its pairs j = 4..7 -- half the registers of the one-thread form
// (legs, x(z-1..z+1), uz), so a CU holds eight waves of it where it held four.  The rows' W values are exchanged
// through LDS (the x+1 leg window's space, free once the rows are done), then each half takes every other pair of
// basis vectors over all 16 rows of its lane: lane t's sum, the butterflies and the (w0 + w1) + (w2 + w3) of
// every vector are k_box_spmv_mdot_march<.., 2>'s, term for term, and so are W and the values (bitwise).  The
// x(z) dot comes from the LDS window.  nx <= 512 (LDS: the windows of x and of the x+1 / y+1 legs).
template <int VAR, bool NTY>
__global__ __launch_bounds__(2 * kT) void k_box_spmv_mdot_march_sym2(int32_t nx, int64_t P, int32_t nz, int32_t zt,
                                                                    int xcd, const uint8_t* __restrict__ mask,
                                                                    const double* __restrict__ rv,
                                                                    const double* __restrict__ x,
                                                                    const double* __restrict__ sdev,
                                                                    double* __restrict__ y, Vecs V, int nv, int self,
                                                                    double* __restrict__ partial, int64_t nchunks,
                                                                    const int* __restrict__ stop) {
  constexpr int H = kIters / 2;  // row pairs per thread
  if (stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sx = reinterpret_cast<double*>(smem);  // window of plane z: kChunk + 2 nx doubles
  double* sux = sx + kChunk + 2 * nx;           // x+1 / y+1 legs of the window [c0 - nx, c0 + 4096)
  double* suy = sux + kChunk + nx;
  __shared__ double red[MSK_MAX_GROUP][4];
  const int t = threadIdx.x, h = t >> 8, tl = t & (kT - 1), lane = t & 63, wv = (t >> 6) & 3;
  const int j0 = h * H;  // this thread's first row pair
  const int64_t cpp = P / kChunk;
  int64_t tile, zg;
  if (xcd & 1) {
    const int64_t per = cpp / 8, slot = blockIdx.x / 8;
    tile = (blockIdx.x % 8) * per + slot % per;
    zg = slot / per;
  } else {
    tile = blockIdx.x % cpp;
    zg = blockIdx.x / cpp;
  }
  if (xcd & 2) zg = (nz + zt - 1) / zt - 1 - zg;
  const int32_t z0 = (int32_t)zg * zt, z1 = min(z0 + zt, nz);
  // xcd & 4: odd plane groups march down (as k_box_spmv_mdot_march).  Going down, plane z's z-1 values are the z+1
  // legs of the plane below, the plane marched to: they are loaded with its x (own[.][3] holds them), and its z+1
  // values are its own z+1 legs, loaded one plane earlier (uzm).  Going up it is the other way round.
  const bool down = (xcd & 4) && (zg & 1);
  const double sc = *sdev;
  const int nh = nx / 2;
  double xm[2 * H], xc[2 * H], xp[2 * H], uzm[2 * H];
  {  // xc: the first plane; xm: the plane marched from; uzm: the z+1 legs of the plane below the first (up) or of
     // the first plane itself (down)
    const int32_t zf = down ? z1 - 1 : z0;
    const bool hasm = down ? z1 < nz : z0 > 0;
    const int64_t cb = ((int64_t)(down ? zf : z0 - 1)) * P + tile * kChunk;
    const int64_t b0 = (int64_t)zf * P + tile * kChunk + 2 * tl, bm = b0 + (down ? P : -P);
#pragma unroll
    for (int jj = 0; jj < H; ++jj) {
      const int j = j0 + jj;
      const double2 u = down || z0 > 0 ? ld_nt(rvs_pair(rv, cb, 3, j, tl)) : make_double2(0.0, 0.0);
      uzm[2 * jj] = u.x;
      uzm[2 * jj + 1] = u.y;
      const double2 a = *reinterpret_cast<const double2*>(x + b0 + j * (2 * kT));
      xc[2 * jj] = a.x;
      xc[2 * jj + 1] = a.y;
      const double2 m2 = hasm ? *reinterpret_cast<const double2*>(x + bm + j * (2 * kT)) : make_double2(0.0, 0.0);
      xm[2 * jj] = m2.x;
      xm[2 * jj + 1] = m2.y;
    }
  }
  for (int32_t zi = 0; zi < z1 - z0; ++zi) {
    const int32_t z = down ? z1 - 1 - zi : z0 + zi;
    const int64_t c = (int64_t)z * cpp + tile, c0 = c * kChunk, base = c0 + 2 * tl;
    const bool hasp = down ? z > 0 : z + 1 < nz;  // xp: the plane marched to
    const int64_t dp = down ? -P : P;
    uint32_t m[H];
    double2 own[H][4];  // own[.][3]: the z+1 legs of plane z (up) or of the plane below (down)
#pragma unroll
    for (int jj = 0; jj < H; ++jj) {
      const int j = j0 + jj;
      if (hasp) {
        const double2 p2 = *reinterpret_cast<const double2*>(x + base + dp + j * (2 * kT));
        xp[2 * jj] = p2.x;
        xp[2 * jj + 1] = p2.y;
      } else {
        xp[2 * jj] = xp[2 * jj + 1] = 0.0;
      }
      m[jj] = *reinterpret_cast<const uint16_t*>(mask + base + j * (2 * kT));
#pragma unroll
      for (int k = 0; k < 3; ++k) own[jj][k] = ld_nt(rvs_pair(rv, c0, k, j, tl));
      own[jj][3] = !down ? ld_nt(rvs_pair(rv, c0, 3, j, tl))
                         : hasp ? ld_nt(rvs_pair(rv, c0 - P, 3, j, tl)) : make_double2(0.0, 0.0);
    }
    double2 hl = make_double2(0.0, 0.0), hh = make_double2(0.0, 0.0), hx = hl, hy = hl;
    const bool hal = h == 0 && tl < nh;
    if (hal && c0 - nx >= 0) {
      hl = *reinterpret_cast<const double2*>(x + c0 - nx + 2 * tl);
      hx = *reinterpret_cast<const double2*>(rvs_at(rv, c0 - nx + 2 * tl, 1));
      hy = *reinterpret_cast<const double2*>(rvs_at(rv, c0 - nx + 2 * tl, 2));
    }
    if (hal && c0 + kChunk + nx <= (int64_t)nz * P) hh = *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * tl);
    __syncthreads();  // the previous plane's window and exchange reads (and its partial writes) are done
#pragma unroll
    for (int jj = 0; jj < H; ++jj) {
      const int o = nx + (j0 + jj) * (2 * kT) + 2 * tl;
      *reinterpret_cast<double2*>(sx + o) = make_double2(xc[2 * jj], xc[2 * jj + 1]);
      *reinterpret_cast<double2*>(sux + o) = own[jj][1];
      *reinterpret_cast<double2*>(suy + o) = own[jj][2];
    }
    if (hal) {
      *reinterpret_cast<double2*>(sx + 2 * tl) = hl;
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * tl) = hh;
      *reinterpret_cast<double2*>(sux + 2 * tl) = hx;
      *reinterpret_cast<double2*>(suy + 2 * tl) = hy;
    }
    __syncthreads();
    double wr[2 * H];
#pragma unroll
    for (int jj = 0; jj < H; ++jj) {
      const int j = j0 + jj;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = j * (2 * kT) + 2 * tl + q + nx;
        const uint32_t mr = (m[jj] >> (8 * q)) & 255u;
        const double xq[7] = {down ? xp[2 * jj + q] : xm[2 * jj + q], sx[e - nx], sx[e - 1], xc[2 * jj + q],
                              sx[e + 1], sx[e + nx], down ? xm[2 * jj + q] : xp[2 * jj + q]};
        const double uf = q ? own[jj][3].y : own[jj][3].x;
        const double vv[7] = {down ? uf : uzm[2 * jj + q], suy[e - nx], sux[e - 1], q ? own[jj][0].y : own[jj][0].x,
                              q ? own[jj][1].y : own[jj][1].x, q ? own[jj][2].y : own[jj][2].x,
                              down ? uzm[2 * jj + q] : uf};
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k)
          if (mr & (1u << k)) s = s + vv[k] * (xq[k] * sc);
        wr[2 * jj + q] = s;
      }
      if constexpr (NTY) {
        dx2 o;
        o.x = wr[2 * jj];
        o.y = wr[2 * jj + 1];
        __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(y + base + j * (2 * kT)));
      } else {
        *reinterpret_cast<double2*>(y + base + j * (2 * kT)) = make_double2(wr[2 * jj], wr[2 * jj + 1]);
      }
      uzm[2 * jj] = own[jj][3].x;  // the next plane's z-1 values (up) or its z+1 values (down)
      uzm[2 * jj + 1] = own[jj][3].y;
    }
    __syncthreads();  // every row is done with the leg windows: the x+1 window's space takes the W exchange
    double* wx = sux;
#pragma unroll
    for (int jj = 0; jj < H; ++jj)
      *reinterpret_cast<double2*>(wx + (j0 + jj) * (2 * kT) + 2 * tl) = make_double2(wr[2 * jj], wr[2 * jj + 1]);
    __syncthreads();
    double wf[2 * kIters];  // all 16 W values of lane tl, in its DBR order
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 a = *reinterpret_cast<const double2*>(wx + j * (2 * kT) + 2 * tl);
      wf[2 * j] = a.x;
      wf[2 * j + 1] = a.y;
    }
    // pairs of vectors alternate between the halves (two vectors' 16 rows in flight per thread: the registers of the
    // one-thread form's groups of four, spread over twice the threads); the odd vector and x(z)'s dot go to the
    // half with fewer pairs
    const int nvm = nv - self, ng = nvm / 2;
#pragma unroll 1
    for (int gi = h; gi < ng; gi += 2) dot_group_full<2, VAR>(wf, V, base, 0, nv, 2 * gi, red, lane, wv);
    const int hr = ng & 1;  // the half that took one pair fewer (or as many)
    if (h == hr) {
      if (nvm & 1) dot_group_full<1, VAR>(wf, V, base, 0, nv, 2 * ng, red, lane, wv);
      if (self) {
        const double sv = vec_scale(V, nv - 1);
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < kIters; ++j) {
          const double2 xr = *reinterpret_cast<const double2*>(sx + nx + j * (2 * kT) + 2 * tl);
          acc = acc + wf[2 * j] * (xr.x * sv);
          acc = acc + wf[2 * j + 1] * (xr.y * sv);
        }
        acc = wave_butterfly(acc);
        if (lane == 0) red[nv - 1][wv] = acc;
      }
    }
    __syncthreads();
    if (t < nv) partial[t * nchunks + c] = (red[t][0] + red[t][1]) + (red[t][2] + red[t][3]);
#pragma unroll
    for (int i = 0; i < 2 * H; ++i) {
      xm[i] = xc[i];
      xc[i] = xp[i];
    }
  }
}

// One vector group of the CGS MAXPY over a full chunk, u += sum_q a_q (V_{g+q} * s_q) in chunk_group's
// arithmetic (group_sum left to right; G == 1: s + u), a_q = -adev[g + q].  SELF: the group's last vector is
// x itself, whose 16 values of this chunk the caller holds in xs (the march registers): not read again.
template <int G, int VAR, bool SELF>
__device__ __forceinline__ void march_maxpy_group(double (&u)[2 * kIters], const Vecs& V,
                                                  const double* __restrict__ adev, int g, int64_t base,
                                                  const double (&xs)[2 * kIters]) {
  double a[G], sv[G];
  const double* vp[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    a[q] = -adev[g + q];
    vp[q] = vec_at(V, g + q);
    sv[q] = vec_scale(V, g + q);
  }
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    double p0[G], p1[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (SELF && q == G - 1) {
        p0[q] = xs[2 * j] * sv[q];
        p1[q] = xs[2 * j + 1] * sv[q];
      } else {
        const double2* pv = reinterpret_cast<const double2*>(vp[q] + base + j * (2 * kT));
        const double2 v = (VAR & 1) ? ld_nt(pv) : *pv;
        p0[q] = v.x * sv[q];
        p1[q] = v.y * sv[q];
      }
    }
    const double s0 = group_sum<G>(a, p0), s1 = group_sum<G>(a, p1);
    if constexpr (G == 1) {
      u[2 * j] = s0 + u[2 * j];
      u[2 * j + 1] = s1 + u[2 * j + 1];
    } else {
      u[2 * j] = u[2 * j] + s0;
      u[2 * j + 1] = u[2 * j + 1] + s1;
    }
  }
}

// The GMRES step's CGS VecMAXPY for a box stencil whose fused MatMult+MDot (k_box_spmv_mdot_march, y = null)
// did not store W: this kernel recomputes W = A (sc x) for its rows on the same chunk tiles, with the same
// terms in the same order (bitwise that kernel's W), then wout = W - sum_j h_j VV(j) in k_maxpy_chunk's
// grouping (the nv & 3 leading vectors, then groups of four), the last basis vector being x itself, taken
// from the march registers.  It stores wout and the DBR partial of ||wout||^2 per chunk exactly as
// k_maxpy_chunk<false, true, .> does.  Bytes per row: the presence byte, x once (+ the tile's halo lines),
// nv - 1 basis vectors and wout, against 8 (nv + 2) for k_maxpy_chunk plus the 8 the MatMult spent storing W.
// xcd & 1: XCD-contiguous eighths of each plane's tiles; xcd & 2: top plane groups first.
template <int VAR, bool NTY>
__global__ __launch_bounds__(kT) void k_box_maxpy_march(int32_t nx, int64_t P, int32_t nz, int32_t zt, int xcd,
                                                        const uint8_t* __restrict__ mask,
                                                        const double* __restrict__ dval,
                                                        const double* __restrict__ x,
                                                        const double* __restrict__ sdev, double* __restrict__ wout,
                                                        Vecs V, int nv, const double* __restrict__ adev,
                                                        double* __restrict__ partial, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sx = reinterpret_cast<double*>(smem);  // window of plane z: kChunk + 2 nx doubles
  __shared__ double red[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t cpp = P / kChunk;
  int64_t tile, zg;
  if (xcd & 1) {
    const int64_t per = cpp / 8, slot = blockIdx.x / 8;
    tile = (blockIdx.x % 8) * per + slot % per;
    zg = slot / per;
  } else {
    tile = blockIdx.x % cpp;
    zg = blockIdx.x / cpp;
  }
  if (xcd & 2) zg = (nz + zt - 1) / zt - 1 - zg;
  const int32_t z0 = (int32_t)zg * zt, z1 = min(z0 + zt, nz);
  const double sc = *sdev;
  double v[7];
  march_values<false>(dval, v);
  const int nh = nx / 2;
  double xm[2 * kIters], xc[2 * kIters], xp[2 * kIters];
  {
    const int64_t b0 = (int64_t)z0 * P + tile * kChunk + 2 * t;
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double2 a = *reinterpret_cast<const double2*>(x + b0 + j * (2 * kT));
      xc[2 * j] = a.x;
      xc[2 * j + 1] = a.y;
      if (z0 > 0) {
        const double2 m2 = *reinterpret_cast<const double2*>(x + b0 - P + j * (2 * kT));
        xm[2 * j] = m2.x;
        xm[2 * j + 1] = m2.y;
      } else {
        xm[2 * j] = xm[2 * j + 1] = 0.0;
      }
    }
  }
  const int jrem = nv & 3;
  for (int32_t z = z0; z < z1; ++z) {
    const int64_t c = (int64_t)z * cpp + tile, c0 = c * kChunk, base = c0 + 2 * t;
    uint32_t m[kIters];
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      if (z + 1 < nz) {
        const double2 p2 = *reinterpret_cast<const double2*>(x + base + P + j * (2 * kT));
        xp[2 * j] = p2.x;
        xp[2 * j + 1] = p2.y;
      } else {
        xp[2 * j] = xp[2 * j + 1] = 0.0;
      }
      m[j] = *reinterpret_cast<const uint16_t*>(mask + base + j * (2 * kT));
    }
    double2 hl = make_double2(0.0, 0.0), hh = make_double2(0.0, 0.0);
    const bool hasl = t < nh && c0 - nx >= 0, hash = t < nh && c0 + kChunk + nx <= (int64_t)nz * P;
    if (hasl) hl = *reinterpret_cast<const double2*>(x + c0 - nx + 2 * t);
    if (hash) hh = *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * t);
    __syncthreads();  // the previous plane's window reads (and its red reads) are done
#pragma unroll
    for (int j = 0; j < kIters; ++j)
      *reinterpret_cast<double2*>(sx + nx + j * (2 * kT) + 2 * t) = make_double2(xc[2 * j], xc[2 * j + 1]);
    if (t < nh) {
      *reinterpret_cast<double2*>(sx + 2 * t) = hl;
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * t) = hh;
    }
    for (int i = t + kT; i < nh; i += kT) {
      *reinterpret_cast<double2*>(sx + 2 * i) =
          c0 - nx >= 0 ? *reinterpret_cast<const double2*>(x + c0 - nx + 2 * i) : make_double2(0.0, 0.0);
      *reinterpret_cast<double2*>(sx + nx + kChunk + 2 * i) =
          c0 + kChunk + nx <= (int64_t)nz * P ? *reinterpret_cast<const double2*>(x + c0 + kChunk + 2 * i)
                                              : make_double2(0.0, 0.0);
    }
    __syncthreads();
    double u[2 * kIters];
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = j * (2 * kT) + 2 * t + q + nx;
        const uint32_t mr = (m[j] >> (8 * q)) & 255u;
        const double xq[7] = {xm[2 * j + q], sx[e - nx], sx[e - 1], xc[2 * j + q], sx[e + 1], sx[e + nx],
                              xp[2 * j + q]};
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k)
          if (mr & (1u << k)) s = s + v[k] * (xq[k] * sc);
        u[2 * j + q] = s;
      }
    }
    // u -= sum_j h_j VV(j): leading nv & 3 vectors, then groups of four; VV(nv - 1) = x from xc
    if (nv <= 3) {
      if (jrem == 3) march_maxpy_group<3, VAR, true>(u, V, adev, 0, base, xc);
      else if (jrem == 2) march_maxpy_group<2, VAR, true>(u, V, adev, 0, base, xc);
      else march_maxpy_group<1, VAR, true>(u, V, adev, 0, base, xc);
    } else {
      if (jrem == 3) march_maxpy_group<3, VAR, false>(u, V, adev, 0, base, xc);
      else if (jrem == 2) march_maxpy_group<2, VAR, false>(u, V, adev, 0, base, xc);
      else if (jrem == 1) march_maxpy_group<1, VAR, false>(u, V, adev, 0, base, xc);
      if constexpr ((VAR & 32) != 0) {  // two groups per iteration: 8 vectors' loads in one burst
#pragma unroll 2
        for (int g = jrem; g + 4 < nv; g += 4) march_maxpy_group<4, VAR, false>(u, V, adev, g, base, xc);
      } else {
#pragma unroll 1
        for (int g = jrem; g + 4 < nv; g += 4) march_maxpy_group<4, VAR, false>(u, V, adev, g, base, xc);
      }
      march_maxpy_group<4, VAR, true>(u, V, adev, nv - 4, base, xc);
    }
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double r0 = u[2 * j], r1 = u[2 * j + 1];
      if constexpr (NTY) {
        dx2 o;
        o.x = r0;
        o.y = r1;
        __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(wout + base + j * (2 * kT)));
      } else {
        *reinterpret_cast<double2*>(wout + base + j * (2 * kT)) = make_double2(r0, r1);
      }
      acc = acc + r0 * r0;
      acc = acc + r1 * r1;
    }
    acc = wave_butterfly(acc);
    if (lane == 0) red[wv] = acc;
    __syncthreads();
    if (t == 0) partial[c] = (red[0] + red[1]) + (red[2] + red[3]);
#pragma unroll
    for (int i = 0; i < 2 * kIters; ++i) {
      xm[i] = xc[i];
      xc[i] = xp[i];
    }
  }
}

// march_maxpy_group for a ragged last chunk: chunk_group<G, FULL = false>'s guarded loads (rows >= n add 0.0).
template <int G, bool SELF>
__device__ __forceinline__ void ragged_maxpy_group(double (&u)[2 * kIters], const Vecs& V,
                                                   const double* __restrict__ adev, int g, int64_t base, int64_t n,
                                                   const double (&xs)[2 * kIters]) {
  double a[G], sv[G];
  const double* vp[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    a[q] = -adev[g + q];
    vp[q] = vec_at(V, g + q);
    sv[q] = vec_scale(V, g + q);
  }
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
    const int64_t e = base + j * (2 * kT);
    double p0[G], p1[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      if (SELF && q == G - 1) {
        p0[q] = e < n ? xs[2 * j] * sv[q] : 0.0;
        p1[q] = e + 1 < n ? xs[2 * j + 1] * sv[q] : 0.0;
      } else {
        p0[q] = e < n ? vp[q][e] * sv[q] : 0.0;
        p1[q] = e + 1 < n ? vp[q][e + 1] * sv[q] : 0.0;
      }
    }
    const double s0 = group_sum<G>(a, p0), s1 = group_sum<G>(a, p1);
    if constexpr (G == 1) {
      u[2 * j] = s0 + u[2 * j];
      u[2 * j + 1] = s1 + u[2 * j + 1];
    } else {
      u[2 * j] = u[2 * j] + s0;
      u[2 * j + 1] = u[2 * j + 1] + s1;
    }
  }
}

// The W-free MAXPY where the fused kernel does not march (k_box_spmv_mdot: one DBR chunk per workgroup, 2D boxes,
// planes that do not hold whole chunks, a ragged last chunk): W for the chunk's rows exactly as k_box_spmv_mdot
// computes it (the same window, the same terms in the same order), then k_box_maxpy_march's MAXPY, x's values from
// the window's own rows; a ragged chunk follows k_maxpy_chunk's guarded path (stores and squares for rows < n).
template <bool D2, int VAR, bool NTY>
__global__ __launch_bounds__(kT) void k_box_maxpy(int32_t nx, int64_t P, int64_t n, const uint8_t* __restrict__ mask,
                                                  const double* __restrict__ dval, const double* __restrict__ x,
                                                  const double* __restrict__ sdev, double* __restrict__ wout, Vecs V,
                                                  int nv, const double* __restrict__ adev,
                                                  double* __restrict__ partial, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sx = reinterpret_cast<double*>(smem);  // window of kChunk + 2 nx doubles
  __shared__ double red[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t c = blockIdx.x, c0 = c * kChunk, lo = c0 - nx;
  const int64_t base = c0 + 2 * t;
  const bool full = (c + 1) * kChunk <= n;
  const int wlen = kChunk + 2 * nx;
  if ((nx & 1) == 0 && lo >= 0 && lo + wlen <= n) {
    const double2* x2 = reinterpret_cast<const double2*>(x + lo);
    for (int i = t; i < wlen / 2; i += kT) reinterpret_cast<double2*>(sx)[i] = x2[i];
  } else {
    for (int i = t; i < wlen; i += kT) {
      const int64_t r = lo + i;
      sx[i] = r >= 0 && r < n ? x[r] : 0.0;
    }
  }
  const double sc = *sdev;
  double v[7];
  march_values<D2>(dval, v);
  uint32_t m[2 * kIters];
  double xm[2 * kIters], xp[2 * kIters];
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t r = base + j * (2 * kT) + q;
      const uint32_t mr = r < n ? (uint32_t)mask[r] : 0u;
      m[2 * j + q] = mr;
      xm[2 * j + q] = (mr & 1u) ? x[r - P] : 0.0;
      xp[2 * j + q] = (mr & 64u) ? x[r + P] : 0.0;
    }
  }
  __syncthreads();
  double u[2 * kIters], xs[2 * kIters];
#pragma unroll
  for (int j = 0; j < kIters; ++j) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = j * (2 * kT) + 2 * t + q + nx;
      const uint32_t mr = m[2 * j + q];
      const double xq[7] = {xm[2 * j + q], sx[e - nx], sx[e - 1], sx[e], sx[e + 1], sx[e + nx], xp[2 * j + q]};
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 7; ++k)
        if (mr & (1u << k)) s = s + v[k] * (xq[k] * sc);
      u[2 * j + q] = s;
      xs[2 * j + q] = sx[e];
    }
  }
  const int jrem = nv & 3;
  double acc = 0.0;
  if (full) {
    if (nv <= 3) {
      if (jrem == 3) march_maxpy_group<3, VAR, true>(u, V, adev, 0, base, xs);
      else if (jrem == 2) march_maxpy_group<2, VAR, true>(u, V, adev, 0, base, xs);
      else march_maxpy_group<1, VAR, true>(u, V, adev, 0, base, xs);
    } else {
      if (jrem == 3) march_maxpy_group<3, VAR, false>(u, V, adev, 0, base, xs);
      else if (jrem == 2) march_maxpy_group<2, VAR, false>(u, V, adev, 0, base, xs);
      else if (jrem == 1) march_maxpy_group<1, VAR, false>(u, V, adev, 0, base, xs);
#pragma unroll 1
      for (int g = jrem; g + 4 < nv; g += 4) march_maxpy_group<4, VAR, false>(u, V, adev, g, base, xs);
      march_maxpy_group<4, VAR, true>(u, V, adev, nv - 4, base, xs);
    }
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const double r0 = u[2 * j], r1 = u[2 * j + 1];
      if constexpr (NTY) {
        dx2 o;
        o.x = r0;
        o.y = r1;
        __builtin_nontemporal_store(o, reinterpret_cast<dx2*>(wout + base + j * (2 * kT)));
      } else {
        *reinterpret_cast<double2*>(wout + base + j * (2 * kT)) = make_double2(r0, r1);
      }
      acc = acc + r0 * r0;
      acc = acc + r1 * r1;
    }
  } else {
    if (nv <= 3) {
      if (jrem == 3) ragged_maxpy_group<3, true>(u, V, adev, 0, base, n, xs);
      else if (jrem == 2) ragged_maxpy_group<2, true>(u, V, adev, 0, base, n, xs);
      else ragged_maxpy_group<1, true>(u, V, adev, 0, base, n, xs);
    } else {
      if (jrem == 3) ragged_maxpy_group<3, false>(u, V, adev, 0, base, n, xs);
      else if (jrem == 2) ragged_maxpy_group<2, false>(u, V, adev, 0, base, n, xs);
      else if (jrem == 1) ragged_maxpy_group<1, false>(u, V, adev, 0, base, n, xs);
#pragma unroll 1
      for (int g = jrem; g + 4 < nv; g += 4) ragged_maxpy_group<4, false>(u, V, adev, g, base, n, xs);
      ragged_maxpy_group<4, true>(u, V, adev, nv - 4, base, n, xs);
    }
#pragma unroll
    for (int j = 0; j < kIters; ++j) {
      const int64_t e = base + j * (2 * kT);
      if (e < n) {
        wout[e] = u[2 * j];
        acc = acc + u[2 * j] * u[2 * j];
      }
      if (e + 1 < n) {
        wout[e + 1] = u[2 * j + 1];
        acc = acc + u[2 * j + 1] * u[2 * j + 1];
      }
    }
  }
  acc = wave_butterfly(acc);
  if (lane == 0) red[wv] = acc;
  __syncthreads();
  if (t == 0) partial[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

// The presence byte of each row of a box stencil in the ELL layout (8 codes per row):
// bit e set when the row holds neighbour e (march_code).  Built once at assembly.
template <bool D2>
__global__ __launch_bounds__(kT) void k_march_mask(int32_t nrows, const uint8_t* __restrict__ code8,
                                                   uint8_t* __restrict__ mask) {
  const int32_t r = (int32_t)blockIdx.x * kT + (int32_t)threadIdx.x;
  if (r >= nrows) return;
  const u32x2 cw = reinterpret_cast<const u32x2*>(code8)[r];
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = EllWord<8>::byte(cw, q);
    if (c != 255) m |= 1u << march_code<D2>(c);
  }
  mask[r] = (uint8_t)m;
}

// Whether the march kernels compute every row of an assembled matrix exactly: they read
// neighbour e at its place in the box, and x(i-+1) / x(y-+1) as 0.0 across a line / plane
// edge, so a row whose entry wraps across one (a -1 entry at i = 0, +1 at i = nx - 1, -nx at
// y = 0, +nx at y = ny - 1; in 3D) would be summed wrong.  *fail is set for any such row
// (msp_mat_create_csr's box detection; a generated box stencil never has one).
__global__ __launch_bounds__(kT) void k_march_check(int32_t nrows, int32_t nx, int32_t ny, int d2,
                                                    const uint8_t* __restrict__ mask, int* __restrict__ fail) {
  const int32_t r = (int32_t)blockIdx.x * kT + (int32_t)threadIdx.x;
  if (r >= nrows) return;
  const uint32_t m = mask[r];
  const int32_t i = r % nx;
  bool bad = ((m & 4u) && i == 0) || ((m & 16u) && i == nx - 1);
  if (!d2) {
    const int32_t yy = (r / nx) % ny;
    bad = bad || ((m & 2u) && yy == 0) || ((m & 32u) && yy == ny - 1);
  }
  if (bad) atomicOr(fail, 1);
}

// MatMatMult R = A S over DV storage (ELL layout): lane per row, its codes
// decoded once into (delta, value) registers, then every column of S streamed
// past them; each R(r, q) is the CSR row sum of k_spmm_lds8 term for term.
template <int W>
__global__ __launch_bounds__(kT) void k_spmm_ell(int32_t nrows, const uint8_t* __restrict__ code8,
                                                 const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                                 int ndict, const double* __restrict__ S, int64_t lds, int nc,
                                                 double* __restrict__ R, int64_t ldr) {
  typedef EllWord<W> EW;
  typedef typename EW::T CT;
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r = (int32_t)blockIdx.x * kT + t;
  const CT cw = r < nrows ? reinterpret_cast<const CT*>(code8)[r] : EW::empty();
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  __syncthreads();
  if (r >= nrows) return;
  int32_t dl[W];
  double av[W];
  bool ok[W];
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const int c = EW::byte(cw, q);
    ok[q] = c != 255;
    dl[q] = ok[q] ? sdel[c] : 0;
    av[q] = ok[q] ? sval[c] : 0.0;
  }
#pragma unroll 1
  for (int j = 0; j < nc; ++j) {
    const double* __restrict__ x = S + (int64_t)j * lds;
    double xv[W];
#pragma unroll
    for (int q = 0; q < W; ++q) xv[q] = ok[q] ? x[r + dl[q]] : 0.0;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < W; ++q)
      if (ok[q]) s = s + av[q] * xv[q];
    R[r + (int64_t)j * ldr] = s;
  }
}

// ELL-layout encode: row r's W codes, then 255 padding; *fail when a row is
// longer than W or an entry is not in the dictionary (ndict <= 255).
__global__ __launch_bounds__(kT) void k_ell_encode(int32_t nrows, int W, const int32_t* __restrict__ rowptr,
                                                   const int32_t* __restrict__ col, const double* __restrict__ val,
                                                   int ndict, const int32_t* __restrict__ ddelta,
                                                   const double* __restrict__ dval, uint8_t* __restrict__ code8,
                                                   int* __restrict__ fail) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  for (int64_t r = (int64_t)blockIdx.x * kT + threadIdx.x; r < nrows; r += stride) {
    const int32_t k0 = rowptr[r], k1 = rowptr[r + 1];
    if (k1 - k0 > W) {
      atomicOr(fail, 1);
      continue;
    }
    for (int q = 0; q < W; ++q) {
      int j = 255;
      if (k0 + q < k1) {
        const int32_t k = k0 + q;
        const int32_t d = col[k] - (int32_t)r;
        const long long bits = __double_as_longlong(val[k]);
        j = 0;
        while (j < ndict && !(ddelta[j] == d && __double_as_longlong(dval[j]) == bits)) ++j;
        if (j == ndict || j == 255) {
          atomicOr(fail, 1);
          j = 255;
        }
      }
      code8[r * W + q] = (uint8_t)j;
    }
  }
}

// Encode an assembled CSR into DV storage against a given dictionary (one lane
// per row); *fail is set when a row is longer than 255 or an entry's
// (col - row, value bits) is not in the dictionary.
__global__ __launch_bounds__(kT) void k_dv_encode(int32_t nrows, const int32_t* __restrict__ rowptr,
                                                  const int32_t* __restrict__ col, const double* __restrict__ val,
                                                  int ndict, const int32_t* __restrict__ ddelta,
                                                  const double* __restrict__ dval, uint8_t* __restrict__ len8,
                                                  uint8_t* __restrict__ code8, int* __restrict__ fail) {
  const int64_t stride = (int64_t)gridDim.x * kT;
  for (int64_t r = (int64_t)blockIdx.x * kT + threadIdx.x; r < nrows; r += stride) {
    const int32_t k0 = rowptr[r], k1 = rowptr[r + 1];
    if (k1 - k0 > 255) {
      atomicOr(fail, 1);
      continue;
    }
    len8[r] = (uint8_t)(k1 - k0);
    for (int32_t k = k0; k < k1; ++k) {
      const int32_t d = col[k] - (int32_t)r;
      const long long bits = __double_as_longlong(val[k]);
      int j = 0;
      while (j < ndict && !(ddelta[j] == d && __double_as_longlong(dval[j]) == bits)) ++j;
      if (j == ndict) {
        atomicOr(fail, 1);
        break;
      }
      code8[k] = (uint8_t)j;
    }
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

}  // namespace
}  // namespace msk

// ===================================================================== launchers
using namespace msk;

// Tuning flags (A/B experiments; MSPLIT_TUNING at context creation), defined once (the MISC part).
#if MSK_IN(MSK_PART_MISC)
__attribute__((visibility("hidden"))) int msk_tuning_flags = 0;
__attribute__((visibility("hidden"))) int msk_spmv_gb_override = 0;  // XCD group size override (0: auto)
__attribute__((visibility("hidden"))) int msk_march_z_override = 0;  // z-march planes per workgroup (0: auto)
__attribute__((visibility("hidden"))) int msk_march_lines_override = 0;  // z-march tile: 1 row block, 4 lines (0: auto)
extern "C" void msk_set_tuning(int flags) { msk_tuning_flags = flags; }
extern "C" int msk_get_tuning(void) { return msk_tuning_flags; }
// Launch-shape overrides change what a captured GMRES cycle (ksp_gmres.c run_cycle) would replay:
// every change bumps msk_shape_epoch, which is part of the graph key.
__attribute__((visibility("hidden"))) int msk_shape_epoch = 0;
extern "C" void msk_set_spmv_group(int gb) {
  msk_spmv_gb_override = gb;
  ++msk_shape_epoch;
}
extern "C" void msk_set_march_z(int z) {
  msk_march_z_override = z;
  ++msk_shape_epoch;
}
extern "C" void msk_set_march_lines(int l) {
  msk_march_lines_override = l;
  ++msk_shape_epoch;
}
extern "C" int msk_get_shape_epoch(void) { return msk_shape_epoch; }
// The W-free GMRES step for box stencils (k_box_maxpy_march recomputes W; the fused MatMult+MDot does not store
// it): on unless MSPLIT_GM_WFREE=0; msk_set_gm_wfree switches it (A/B, tests) and re-keys captured cycles.
__attribute__((visibility("hidden"))) int msk_gm_wfree = [] {
  const char* e = getenv("MSPLIT_GM_WFREE");
  return e ? (atoi(e) ? 1 : 0) : 1;
}();
extern "C" void msk_set_gm_wfree(int on) {
  msk_gm_wfree = on ? 1 : 0;
  ++msk_shape_epoch;
}
extern "C" int msk_get_gm_wfree(void) { return msk_gm_wfree; }
#else
extern __attribute__((visibility("hidden"))) int msk_tuning_flags;
extern __attribute__((visibility("hidden"))) int msk_spmv_gb_override;
extern __attribute__((visibility("hidden"))) int msk_march_z_override;
extern __attribute__((visibility("hidden"))) int msk_march_lines_override;
extern __attribute__((visibility("hidden"))) int msk_gm_wfree;
#endif

[[maybe_unused]] static inline XcdMap xcd_map(int32_t nrows, int64_t plane) {
  XcdMap m = {0, 0, 0};
  if (msk_tuning_flags & MSK_TUNE_SPMV_ZCHUNK) {  // A/B: each XCD a contiguous eighth of the rows
    const int32_t nblk = (nrows + kT - 1) / kT;
    if (nblk % 8 == 0) {
      m.bp = -1;
      m.np = nblk / 8;
    }
    return m;
  }
  if (!(msk_tuning_flags & MSK_TUNE_SPMV_XCD) || plane <= 0 || plane % kT || nrows % plane) return m;
  const int32_t bp = (int32_t)(plane / kT);
  int32_t gb = msk_spmv_gb_override > 0 ? msk_spmv_gb_override : std::min(bp / 8, 64);
  if (gb <= 0 || bp % gb || (bp / gb) % 8) return m;
  m.bp = bp;
  m.gb = gb;
  m.np = (int32_t)(nrows / plane);
  return m;
}

[[maybe_unused]] static inline int grid_for(int64_t work, int cap) {
  int64_t g = (work + kT - 1) / kT;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// basis-vector load policy: non-temporal unless MSK_TUNE_VEC_TEMPORAL (A/B)
[[maybe_unused]] static inline int vec_var() { return (msk_tuning_flags & MSK_TUNE_VEC_TEMPORAL) ? 0 : 1; }

__attribute__((visibility("hidden"))) int msk_dot1_variants_a(int var, int nv, const double* w, const Vecs& V,
                                                               int64_t n, double* partial, int64_t nchunks,
                                                               const int* stop, hipStream_t s);
__attribute__((visibility("hidden"))) int msk_dot1_variants_b(int var, int nv, const double* w, const Vecs& V,
                                                               int64_t n, double* partial, int64_t nchunks,
                                                               const int* stop, hipStream_t s);

template <int NV, int VAR>
static void dot1_dispatch(int nv, const double* w, const Vecs& V, int64_t n, double* partial, int64_t nchunks,
                          const int* stop, hipStream_t s) {
  if (nv == NV) {
    k_dot_stage1<NV, false, VAR><<<dim3((unsigned)nchunks), dim3(kT), 0, s>>>(
        w, V, n, partial, nchunks, stop, (msk_tuning_flags & MSK_TUNE_MDOT_REV) ? 1 : 0);
  } else if constexpr (NV < MSK_MAX_GROUP) {
    dot1_dispatch<NV + 1, VAR>(nv, w, V, n, partial, nchunks, stop, s);
  }
}

#if MSK_IN(MSK_PART_DOT)
extern "C" int msk_dot_stage1(const double* w, const Vecs* V, int nv, int64_t n, double* partial, int64_t nchunks,
                              int self, const int* stop, hipStream_t s) {
  if (nchunks <= 0) return 0;
  if (!self && (nv < 1 || nv > MSK_MAX_GROUP)) return (int)hipErrorInvalidValue;
  const int var = vec_var() | ((msk_tuning_flags & MSK_TUNE_MDOT_SINGLE) ? 16 : 0) |
                  ((msk_tuning_flags & MSK_TUNE_MDOT_UNROLL2) ? 32 : 0);
  if (self)
    k_dot_stage1<1, true, 0><<<dim3((unsigned)nchunks), dim3(kT), 0, s>>>(w, *V, n, partial, nchunks, stop, 0);
  else if (var == 1) dot1_dispatch<1, 1>(nv, w, *V, n, partial, nchunks, stop, s);
  else if (msk_dot1_variants_a(var, nv, w, *V, n, partial, nchunks, stop, s) &&
           msk_dot1_variants_b(var, nv, w, *V, n, partial, nchunks, stop, s))
    return (int)hipErrorInvalidValue;  // a tuning combination with no kernel: fail, never run another one
  return (int)hipGetLastError();
}
#endif  // part

// The A/B variants of the MDot kernel, in parts of their own (each variant is 32 instantiations).
// Return 0 when they launched the variant, 1 when it is not theirs.
#if MSK_IN(MSK_PART_DOT_A)
int msk_dot1_variants_a(int var, int nv, const double* w, const Vecs& V, int64_t n, double* partial,
                        int64_t nchunks, const int* stop, hipStream_t s) {
  if (var == 0) dot1_dispatch<1, 0>(nv, w, V, n, partial, nchunks, stop, s);
  else if (var == 16) dot1_dispatch<1, 16>(nv, w, V, n, partial, nchunks, stop, s);
  else return 1;
  return 0;
}
#endif  // part
#if MSK_IN(MSK_PART_DOT_B)
int msk_dot1_variants_b(int var, int nv, const double* w, const Vecs& V, int64_t n, double* partial,
                        int64_t nchunks, const int* stop, hipStream_t s) {
  if (var == 17) dot1_dispatch<1, 17>(nv, w, V, n, partial, nchunks, stop, s);
  else if (var == 32) dot1_dispatch<1, 32>(nv, w, V, n, partial, nchunks, stop, s);
  else if (var == 33) dot1_dispatch<1, 33>(nv, w, V, n, partial, nchunks, stop, s);
  else return 1;
  return 0;
}
#endif  // part
#if MSK_IN(MSK_PART_DOT)

template <int NV, int VAR>
static void dot1_op_dispatch(int nv, const EllOp& op, const Vecs& V, int64_t n, double* partial, int64_t nchunks,
                             const int* stop, hipStream_t s) {
  if (nv == NV) {
    k_dot_stage1_op<NV, VAR><<<dim3((unsigned)nchunks), dim3(kT), 0, s>>>(op, V, n, partial, nchunks, stop);
  } else if constexpr (NV < MSK_MAX_GROUP) {
    dot1_op_dispatch<NV + 1, VAR>(nv, op, V, n, partial, nchunks, stop, s);
  }
}

extern "C" int msk_dot_stage1_op(const EllOp* op, const Vecs* V, int nv, int64_t n, double* partial,
                                 int64_t nchunks, const int* stop, hipStream_t s) {
  if (nchunks <= 0) return 0;
  if (nv < 1 || nv > MSK_MAX_GROUP || op->ndict > 255) return (int)hipErrorInvalidValue;
  if (vec_var()) dot1_op_dispatch<1, 1>(nv, *op, *V, n, partial, nchunks, stop, s);
  else dot1_op_dispatch<1, 0>(nv, *op, *V, n, partial, nchunks, stop, s);
  return (int)hipGetLastError();
}
#endif  // part

#if MSK_IN(MSK_PART_MAXPY)
extern "C" int msk_maxpy_op(const EllOp* op, double* wout, const Vecs* V, int nv, const double* adev, int64_t n,
                            double* partial, const int* stop, hipStream_t s) {
  if (n <= 0 || nv <= 0) return 0;
  if (op->ndict > 255) return (int)hipErrorInvalidValue;
  const unsigned g = (unsigned)((n + kChunk - 1) / kChunk);
  const int var = vec_var() | ((msk_tuning_flags & MSK_TUNE_MAXPY_TEMPORAL_ST) ? 0 : 4);
  if (var == 5) k_maxpy_op<5><<<g, kT, 0, s>>>(*op, wout, *V, adev, nv, n, partial, stop);
  else if (var == 4) k_maxpy_op<4><<<g, kT, 0, s>>>(*op, wout, *V, adev, nv, n, partial, stop);
  else if (var == 1) k_maxpy_op<1><<<g, kT, 0, s>>>(*op, wout, *V, adev, nv, n, partial, stop);
  else k_maxpy_op<0><<<g, kT, 0, s>>>(*op, wout, *V, adev, nv, n, partial, stop);
  return (int)hipGetLastError();
}
#endif  // part

#if MSK_IN(MSK_PART_DOT)
extern "C" int msk_dot_stage2(const double* partial, int64_t nchunks, int nv, double* out, const int* stop,
                              hipStream_t s) {
  if (stop) k_dot_stage2<true><<<dim3(nv), dim3(kT), 0, s>>>(partial, nchunks, out, stop);
  else k_dot_stage2<false><<<dim3(nv), dim3(kT), 0, s>>>(partial, nchunks, out, nullptr);
  return (int)hipGetLastError();
}
#endif  // part

#if MSK_IN(MSK_PART_MAXPY)
extern "C" int msk_maxpy_chunk(const double* win, double* wout, const Vecs* V, int nv, const int* nvdev,
                               const Coefs* A, const double* adev, int negate, int64_t n, int accum, double* partial,
                               const int* stop, hipStream_t s) {
  if (n <= 0 || (nv <= 0 && !nvdev)) return 0;
  // non-temporal store of w too unless MSK_TUNE_MAXPY_TEMPORAL_ST (+0.4 % per step); the group loop
  // unrolled by two unless MSK_TUNE_MAXPY_UNROLL1 (+1.7 % per step: 64-load bursts at one wave per SIMD)
  const int var = vec_var() | ((msk_tuning_flags & MSK_TUNE_MAXPY_TEMPORAL_ST) ? 0 : 4) |
                  ((msk_tuning_flags & MSK_TUNE_MAXPY_HALVES) ? 8 : 0) | ((msk_tuning_flags & MSK_TUNE_MAXPY_UNROLL1) ? 0 : 32);
  // Top chunk first where a vector outgrows the 256 MiB MALL (n > 2^25): MAXPY then starts on the rows the
  // fused MatMult+MDot (or the MDot) left in the MALL and ends on those the next one starts with (SMSM's
  // 512x512x256 block +1.0 %, MAXPY 5.68 -> 5.86 TB/s; at 256^3, where whole vectors fit, -0.7 %; same box,
  // profiles/r03/rev_ab/).  MSPLIT_MAXPY_REV=0/1 forces either order.
  static const int rev_env = [] {
    const char* e = getenv("MSPLIT_MAXPY_REV");
    return e ? (atoi(e) ? 1 : 0) : -1;
  }();
  const int rev = (rev_env < 0 ? n > ((int64_t)1 << 25) : rev_env) ? 64 : 0;
  const unsigned g = (unsigned)((n + kChunk - 1) / kChunk);
#define MSK_MAXPY_LAUNCH(V_)                                                                                     \
  if (partial)                                                                                                  \
    k_maxpy_chunk<false, true, V_><<<dim3(g), dim3(kT), 0, s>>>(win, wout, *V, *A, adev, negate, nv, nvdev, n,   \
                                                                partial, stop);                                \
  else if (accum)                                                                                               \
    k_maxpy_chunk<true, false, V_><<<dim3(g), dim3(kT), 0, s>>>(win, wout, *V, *A, adev, negate, nv, nvdev, n,   \
                                                                partial, stop);                                \
  else                                                                                                          \
    k_maxpy_chunk<false, false, V_><<<dim3(g), dim3(kT), 0, s>>>(win, wout, *V, *A, adev, negate, nv, nvdev, n,  \
                                                                 partial, stop);
  switch (var) {
    case 0: MSK_MAXPY_LAUNCH(0) break;
    case 1: MSK_MAXPY_LAUNCH(1) break;
    case 4: MSK_MAXPY_LAUNCH(4) break;
    case 5: MSK_MAXPY_LAUNCH(5) break;
    case 13: MSK_MAXPY_LAUNCH(13) break;
    case 32: MSK_MAXPY_LAUNCH(32) break;
    case 33: if (rev) { MSK_MAXPY_LAUNCH(97) } else { MSK_MAXPY_LAUNCH(33) } break;
    case 36: MSK_MAXPY_LAUNCH(36) break;
    case 37: if (rev) { MSK_MAXPY_LAUNCH(101) } else { MSK_MAXPY_LAUNCH(37) } break;
    case 45: MSK_MAXPY_LAUNCH(45) break;
    default: return (int)hipErrorInvalidValue;  // a tuning combination with no kernel: fail, never run another one
  }
#undef MSK_MAXPY_LAUNCH
  return (int)hipGetLastError();
}
#endif  // part

#if MSK_IN(MSK_PART_SPMV)
extern "C" int msk_spmv(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* x,
                        const double* b, double* y, int32_t lds_cap, int mode, const double* sdev, double* vout,
                        const int* stop, int64_t plane, hipStream_t s) {
  if (nrows <= 0) return 0;
  const unsigned g = (unsigned)((nrows + kT - 1) / kT);
  const XcdMap xm = xcd_map(nrows, plane);
  if (lds_cap > 0) {
    const bool tmp = (msk_tuning_flags & MSK_TUNE_SPMV_TEMPORAL) != 0, nty = (msk_tuning_flags & MSK_TUNE_SPMV_NTY) != 0;
    // staging: LDS-DMA by default (512^3 MatMult +1.4 %, CSR GMRES step +0.3 % same box, profiles/r02/glds/);
    // MSK_TUNE_SPMV_REG_STAGE / _STAGE1: through registers (round-1 forms)
    const bool reg = (msk_tuning_flags & MSK_TUNE_SPMV_REG_STAGE) != 0, stage1 = (msk_tuning_flags & MSK_TUNE_SPMV_STAGE1) != 0;
    const bool glds = !reg && !stage1;
    // a combination with no kernel fails instead of running another variant
    if ((tmp && nty) || (reg && stage1)) return (int)hipErrorInvalidValue;
    const bool nt = !tmp && !nty;
    const bool ntst = !tmp;
    const int32_t cap = glds ? ((lds_cap + 255) & ~255) : lds_cap;
    const size_t ldsb = (size_t)cap * 12;  // LDS-DMA: slack for the last instruction's tail lanes
#define LAUNCH_LDS8(M, POL_)                                                                                  \
  do {                                                                                                         \
    if (glds)                                                                                                  \
      k_spmv_lds8<M, POL_, 0><<<dim3(g), dim3(kT), ldsb, s>>>(nrows, rowptr, col, val, x, b, y, cap, sdev,     \
                                                               vout, stop, xm);                                \
    else if (stage1)                                                                                           \
      k_spmv_lds8<M, POL_, 1><<<dim3(g), dim3(kT), ldsb, s>>>(nrows, rowptr, col, val, x, b, y, cap, sdev,     \
                                                               vout, stop, xm);                                \
    else                                                                                                       \
      k_spmv_lds8<M, POL_, 4><<<dim3(g), dim3(kT), ldsb, s>>>(nrows, rowptr, col, val, x, b, y, cap, sdev,     \
                                                               vout, stop, xm);                                \
  } while (0)
#define LAUNCH_POL(M)                            \
  do {                                           \
    if (nt) LAUNCH_LDS8(M, 3);                   \
    else if (ntst) LAUNCH_LDS8(M, 2);            \
    else LAUNCH_LDS8(M, 0);                      \
  } while (0)
    if (mode == MSK_SPMV_RESID) LAUNCH_POL(MSK_SPMV_RESID);
    else if (mode == MSK_SPMV_SCALED) LAUNCH_POL(MSK_SPMV_SCALED);
    else LAUNCH_POL(MSK_SPMV_MULT);
#undef LAUNCH_POL
#undef LAUNCH_LDS8
  } else {
    if (mode == MSK_SPMV_RESID)
      k_spmv_direct<MSK_SPMV_RESID><<<dim3(g), dim3(kT), 0, s>>>(nrows, rowptr, col, val, x, b, y, sdev, vout, stop);
    else if (mode == MSK_SPMV_SCALED)
      k_spmv_direct<MSK_SPMV_SCALED><<<dim3(g), dim3(kT), 0, s>>>(nrows, rowptr, col, val, x, b, y, sdev, vout, stop);
    else
      k_spmv_direct<MSK_SPMV_MULT><<<dim3(g), dim3(kT), 0, s>>>(nrows, rowptr, col, val, x, b, y, sdev, vout, stop);
  }
  return (int)hipGetLastError();
}

template <int W, int RPL, bool NTY>
static void launch_ell_pol(int mode, unsigned g, int32_t nrows, const uint8_t* code8, const int32_t* ddelta,
                           const double* dval, int ndict, const double* x, const double* b, double* y,
                           const double* sdev, double* vout, const int* stop, int32_t xwin, hipStream_t s) {
  if (mode == MSK_SPMV_RESID)
    k_spmv_ell<MSK_SPMV_RESID, W, RPL, NTY><<<g, kT, 0, s>>>(nrows, code8, ddelta, dval, ndict, x, b, y, sdev, vout,
                                                             stop, xwin);
  else if (mode == MSK_SPMV_SCALED)
    k_spmv_ell<MSK_SPMV_SCALED, W, RPL, NTY><<<g, kT, 0, s>>>(nrows, code8, ddelta, dval, ndict, x, b, y, sdev, vout,
                                                              stop, xwin);
  else
    k_spmv_ell<MSK_SPMV_MULT, W, RPL, NTY><<<g, kT, 0, s>>>(nrows, code8, ddelta, dval, ndict, x, b, y, sdev, vout,
                                                            stop, xwin);
}

template <int W, int RPL>
static void launch_ell(int mode, int32_t nrows, const uint8_t* code8, const int32_t* ddelta, const double* dval,
                       int ndict, const double* x, const double* b, double* y, const double* sdev, double* vout,
                       const int* stop, int64_t plane, hipStream_t s) {
  const unsigned g = (unsigned)((nrows + kT * RPL - 1) / (kT * RPL));
  const bool xon = (msk_tuning_flags & MSK_TUNE_ELL_XCD_ON) || (plane >= (1 << 18) && !(msk_tuning_flags & MSK_TUNE_ELL_XCD_OFF));
  const int32_t xwin = xon ? 8 : 0;
  if (!(msk_tuning_flags & MSK_TUNE_ELL_TEMPORAL_Y))  // default: non-temporal y (GMRES step +1.1 %, profiles/r02/nt_ab/)
    launch_ell_pol<W, RPL, true>(mode, g, nrows, code8, ddelta, dval, ndict, x, b, y, sdev, vout, stop, xwin, s);
  else
    launch_ell_pol<W, RPL, false>(mode, g, nrows, code8, ddelta, dval, ndict, x, b, y, sdev, vout, stop, xwin, s);
}

// DV SpMV flag pairs that name no kernel: an error on every DV path, whichever kernel the operator takes
static bool dv_flags_bad() {
  const int f = msk_tuning_flags;
  return ((f & MSK_TUNE_ELL_XCD_ON) && (f & MSK_TUNE_ELL_XCD_OFF)) ||
         ((f & MSK_TUNE_ELL_MARCH_NOXCD) && (f & MSK_TUNE_ELL_MARCH_OFF));
}

// L = 0: k_spmv_box_march (256 plane rows per workgroup); L = 4: k_spmv_box_lines (3D only)
template <bool NTY, int L, bool D2>
static void launch_box_march(int mode, unsigned g, int32_t nx, int32_t ny, int32_t nz, const uint8_t* mask,
                             const double* dval, const double* x, const double* b, double* y, const double* sdev,
                             double* vout, const int* stop, int32_t zt, int32_t xwin, hipStream_t s) {
#define MSK_BM(M)                                                                                                 \
  do {                                                                                                            \
    if constexpr (L == 0)                                                                                         \
      k_spmv_box_march<M, NTY, D2><<<g, kT, 0, s>>>(nx, ny, nz, mask, dval, x, b, y, sdev, vout, stop, zt, xwin);    \
    else                                                                                                          \
      k_spmv_box_lines<M, NTY, L><<<g, kT, 0, s>>>(nx, ny, nz, mask, dval, x, b, y, sdev, vout, stop, zt, xwin); \
  } while (0)
  if (mode == MSK_SPMV_RESID) MSK_BM(MSK_SPMV_RESID);
  else if (mode == MSK_SPMV_SCALED) MSK_BM(MSK_SPMV_SCALED);
  else MSK_BM(MSK_SPMV_MULT);
#undef MSK_BM
}

// Kernel and shape: nx % 256 == 0 takes tiles of 4 lines (k_spmv_box_lines) when 16 planes per workgroup,
// halved down to 1, give at least 1024 workgroups; otherwise k_spmv_box_march with 16 planes per workgroup,
// halved while the grid would hold fewer than 2048.  msk_set_march_lines (1: the 256-row kernel; 4: lines)
// and msk_set_march_z override the choice (A/B experiments, tests).
static void march_shape(int32_t nx, int32_t ny, int32_t nz, int32_t* lines, int32_t* zt, int64_t* grid) {
  const int32_t Lq = 4;
  int32_t L = 1, z = 16;
  if (nx % kT == 0 && ny >= Lq && msk_march_lines_override != 1) {
    const int64_t tiles = (int64_t)(nx / kT) * ((ny + Lq - 1) / Lq);
    while (z > 1 && tiles * ((nz + z - 1) / z) < 1024) z /= 2;
    if (tiles * ((nz + z - 1) / z) >= 1024 || msk_march_lines_override == Lq) L = Lq;
    else z = 16;
  }
  const int64_t tiles = L > 1 ? (int64_t)(nx / kT) * ((ny + L - 1) / L) : ((int64_t)nx * ny + kT - 1) / kT;
  if (L == 1)
    while (z > 1 && tiles * ((nz + z - 1) / z) < 2048) z /= 2;
  if (msk_march_z_override > 0) z = msk_march_z_override;
  *lines = L;
  *zt = z;
  *grid = tiles * ((nz + z - 1) / z);
}

extern "C" int msk_box_march_pick(int32_t nx, int32_t ny, int32_t nz) {
  const int f = msk_tuning_flags;
  if (nx <= 0 || ny <= 0 || nz <= 0) return 0;
  return !(f & MSK_TUNE_ELL_MARCH_OFF);
}

// Whether the chunk-tile march (k_box_march_chunk) takes this box: 3D, planes of whole DBR chunks, nx even
// and at most 2048 (the LDS window); by default (march lines override 0) unless MSPLIT_MARCH_CHUNK=0, or
// forced by the override 16.
static bool march_chunk_ok(int32_t nx, int32_t ny, int d2) {
  const int64_t P = (int64_t)nx * ny;
  return !d2 && P % kChunk == 0 && (nx & 1) == 0 && nx >= 2 && nx <= 2048;
}

// The chunk-tile march launch (k_box_march_chunk) for a box whose planes hold whole DBR chunks; halo bit 0/1:
// the column space has the plane below / above the box (x points at the box's first row).
static int launch_march_chunk(int32_t nx, int32_t ny, int32_t nz, int halo, const uint8_t* mask, const double* dval,
                              const double* x, const double* b, double* y, int mode, const double* sdev, double* vout,
                              const int* stop, hipStream_t s, const double* rv = nullptr, int64_t rvs = 0) {
  // depth: the tile-planes dealt to 512 workgroups (two per CU, one wave of the grid; back to back
  // 256^3 56.6 us at 8 planes against 61-64 at 4, 6, 12, 16; 512x512x256 219.6 us at 32 against 228-234 at
  // 8-16; profiles/r03/chunk/), or the msk_set_march_z override
  const int64_t P = (int64_t)nx * ny, cpp = P / kChunk;
  const int32_t zt = msk_march_z_override > 0
                         ? msk_march_z_override
                         : (int32_t)std::max<int64_t>(1, std::min<int64_t>(nz, (cpp * nz + 511) / 512));
  const int64_t grid = cpp * ((nz + zt - 1) / zt);
  if (grid > INT32_MAX || (int64_t)nx * ny * nz > INT32_MAX) return (int)hipErrorInvalidValue;
  const int xcd = cpp % 8 == 0 && cpp >= 32 && !(msk_tuning_flags & MSK_TUNE_ELL_MARCH_NOXCD);
  const bool nty = !(msk_tuning_flags & MSK_TUNE_ELL_TEMPORAL_Y);
  const size_t lds = (size_t)(kChunk + 2 * nx + (rv && rvs < 0 ? 2 * (kChunk + nx) : 0)) * sizeof(double);
#define MSK_BMC(M, NT_, RV_)                                                                                    \
  k_box_march_chunk<M, NT_, RV_><<<dim3((unsigned)grid), dim3(kT), lds, s>>>(nx, P, nz, zt, xcd, halo, mask, dval, rv, \
                                                                             rvs, x, b, y, sdev, vout, stop)
#define MSK_BMC2(M)                                                           \
  do {                                                                        \
    if (rv && rvs < 0) { if (nty) MSK_BMC(M, true, 2); else MSK_BMC(M, false, 2); } \
    else if (rv) { if (nty) MSK_BMC(M, true, 1); else MSK_BMC(M, false, 1); }          \
    else { if (nty) MSK_BMC(M, true, 0); else MSK_BMC(M, false, 0); }                  \
  } while (0)
  if (mode == MSK_SPMV_RESID) MSK_BMC2(MSK_SPMV_RESID);
  else if (mode == MSK_SPMV_SCALED) MSK_BMC2(MSK_SPMV_SCALED);
  else MSK_BMC2(MSK_SPMV_MULT);
#undef MSK_BMC2
#undef MSK_BMC
  return (int)hipGetLastError();
}

extern "C" int msk_spmv_box_march(int32_t nx, int32_t ny, int32_t nz, int d2, const uint8_t* mask,
                                  const double* dval, const double* x, const double* b, double* y, int mode,
                                  const double* sdev, double* vout, const int* stop, hipStream_t s) {
  if (nx <= 0 || ny <= 0 || nz <= 0 || dv_flags_bad()) return (int)hipErrorInvalidValue;
  if (msk_march_lines_override != 0 && msk_march_lines_override != 1 && msk_march_lines_override != 4 &&
      msk_march_lines_override != 16)
    return (int)hipErrorInvalidValue;
  if (msk_march_lines_override == 4 && nx % kT) return (int)hipErrorInvalidValue;
  if (d2 && msk_march_lines_override == 4) return (int)hipErrorInvalidValue;
  static const int chunk_env = [] {
    const char* e = getenv("MSPLIT_MARCH_CHUNK");
    return e ? atoi(e) : 1;
  }();
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const bool chunk_ok = march_chunk_ok(nx, ny, d2) && a16(x) && a16(y) &&
                        (mode != MSK_SPMV_RESID || a16(b)) && (mode != MSK_SPMV_SCALED || !vout || a16(vout));
  if (msk_march_lines_override == 16 && !chunk_ok) return (int)hipErrorInvalidValue;
  if (chunk_ok && (msk_march_lines_override == 16 || (msk_march_lines_override == 0 && chunk_env != 0)))
    return launch_march_chunk(nx, ny, nz, 0, mask, dval, x, b, y, mode, sdev, vout, stop, s);
  int32_t L, zt;
  int64_t g;
  march_shape(nx, ny, nz, &L, &zt, &g);
  if (g > INT32_MAX || (int64_t)nx * ny * nz > INT32_MAX) return (int)hipErrorInvalidValue;
  const int32_t xwin = (msk_tuning_flags & MSK_TUNE_ELL_MARCH_NOXCD) ? 0 : 32;
  const bool nty = !(msk_tuning_flags & MSK_TUNE_ELL_TEMPORAL_Y);
#define MSK_BML(NT, LL, D) \
  launch_box_march<NT, LL, D>(mode, (unsigned)g, nx, ny, nz, mask, dval, x, b, y, sdev, vout, stop, zt, xwin, s)
  if (d2) {
    if (nty) MSK_BML(true, 0, true);
    else MSK_BML(false, 0, true);
  } else if (L == 4) {
    if (nty) MSK_BML(true, 4, false);
    else MSK_BML(false, 4, false);
  } else {
    if (nty) MSK_BML(true, 0, false);
    else MSK_BML(false, 0, false);
  }
#undef MSK_BML
  return (int)hipGetLastError();
}

// Whether the chunk-tile march takes a box of nx x ny planes (and MSPLIT_MARCH_CHUNK does not turn it off).
extern "C" int msk_march_chunk_fits(int32_t nx, int32_t ny, int d2) {
  static const int chunk_env = [] {
    const char* e = getenv("MSPLIT_MARCH_CHUNK");
    return e ? atoi(e) : 1;
  }();
  return chunk_env != 0 && march_chunk_ok(nx, ny, d2);
}

// MatMult / MatResidual of a box stencil whose column space adds the plane below (halo & 1) and / or above
// (halo & 2) the box -- a block's rows of the block-Jacobi operator with its coupling columns -- over chunk
// tiles; x is the column-space vector (the lo plane first).  Only boxes k_box_march_chunk takes.
// Whether msk_box_march_halo takes these operands (the caller's choice of kernel, made before the launch so that a
// launch error is never mistaken for "does not fit"): chunk tiles that fit the plane, 16-byte aligned x (past the
// lower coupling plane), y and, for MatResidual, b.
extern "C" int msk_box_march_halo_fits(int32_t nx, int32_t ny, int32_t nz, int halo, const double* x,
                                       const double* b, const double* y, int mode) {
  if (nx <= 0 || ny <= 0 || nz <= 0 || dv_flags_bad() || mode == MSK_SPMV_SCALED) return 0;
  const double* xo = x + ((halo & 1) ? (int64_t)nx * ny : 0);
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return march_chunk_ok(nx, ny, 0) && a16(xo) && a16(y) && (mode != MSK_SPMV_RESID || a16(b));
}

extern "C" int msk_box_march_halo(int32_t nx, int32_t ny, int32_t nz, int halo, const uint8_t* mask,
                                  const double* dval, const double* x, const double* b, double* y, int mode,
                                  hipStream_t s) {
  if (!msk_box_march_halo_fits(nx, ny, nz, halo, x, b, y, mode)) return (int)hipErrorInvalidValue;
  const double* xo = x + ((halo & 1) ? (int64_t)nx * ny : 0);
  return launch_march_chunk(nx, ny, nz, halo, mask, dval, xo, b, y, mode, nullptr, nullptr, nullptr, s);
}

// The stencil storage's products (k_box_march_chunk<.., RV>): MatMult, MatResidual or the scaled MatMult of a 3D box
// (no coupling planes) whose rows carry their own seven values, rv[e * rvs + row].  Only boxes the chunk-tile march
// takes; every operand 16-byte aligned.
extern "C" int msk_box_march_chunk_rv(int32_t nx, int32_t ny, int32_t nz, const uint8_t* mask, const double* rv,
                                      int64_t rvs, const double* x, const double* b, double* y, int mode,
                                      const double* sdev, double* vout, const int* stop, hipStream_t s) {
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (nx <= 0 || ny <= 0 || nz <= 0 || dv_flags_bad() || !march_chunk_ok(nx, ny, 0) || !rv || (rvs > 0 && (rvs & 1)) ||
      (rvs > 0 && rvs < (int64_t)nx * ny * nz) || (rvs < 0 && nx > 1024) || !a16(rv) || !a16(x) || !a16(y) ||
      (mode == MSK_SPMV_RESID && !a16(b)) ||
      (mode == MSK_SPMV_SCALED && vout && !a16(vout)))
    return (int)hipErrorInvalidValue;
  return launch_march_chunk(nx, ny, nz, 0, mask, nullptr, x, b, y, mode, sdev, vout, stop, s, rv, rvs);
}

extern "C" int msk_march_mask(int32_t nrows, int d2, const uint8_t* code8, uint8_t* mask, hipStream_t s) {
  if (nrows <= 0) return 0;
  const unsigned g = (unsigned)((nrows + kT - 1) / kT);
  if (d2) k_march_mask<true><<<g, kT, 0, s>>>(nrows, code8, mask);
  else k_march_mask<false><<<g, kT, 0, s>>>(nrows, code8, mask);
  return (int)hipGetLastError();
}

extern "C" int msk_march_check(int32_t nrows, int32_t nx, int32_t ny, int d2, const uint8_t* mask, int* fail,
                               hipStream_t s) {
  if (nrows <= 0) return 0;
  if (nx <= 0 || ny <= 0) return (int)hipErrorInvalidValue;
  k_march_check<<<(unsigned)((nrows + kT - 1) / kT), kT, 0, s>>>(nrows, nx, ny, d2, mask, fail);
  return (int)hipGetLastError();
}

extern "C" int msk_spmv_dv(int32_t nrows, const int32_t* rowptr, const uint8_t* len8, const uint8_t* code8,
                           const int32_t* ddelta, const double* dval, int ndict, int32_t max_block, int ell_w,
                           const double* x, const double* b, double* y, int mode, const double* sdev, double* vout,
                           const int* stop, int64_t plane, hipStream_t s) {
  if (nrows <= 0) return 0;
  if (max_block < 0 || ndict < 0 || ndict > 256) return (int)hipErrorInvalidValue;
  if (dv_flags_bad()) return (int)hipErrorInvalidValue;
  if (ell_w) {
    if (ndict > 255) return (int)hipErrorInvalidValue;
    const int rpl = (msk_tuning_flags & MSK_TUNE_DV_RPL1) ? 1 : (msk_tuning_flags & MSK_TUNE_DV_RPL2) ? 2 : (ell_w == 16 ? 2 : 4);
#define MSK_ELL(W_, R_) launch_ell<W_, R_>(mode, nrows, code8, ddelta, dval, ndict, x, b, y, sdev, vout, stop, plane, s)
    if (ell_w == 4) { if (rpl == 1) MSK_ELL(4, 1); else if (rpl == 2) MSK_ELL(4, 2); else MSK_ELL(4, 4); }
    else if (ell_w == 8) { if (rpl == 1) MSK_ELL(8, 1); else if (rpl == 2) MSK_ELL(8, 2); else MSK_ELL(8, 4); }
    else if (ell_w == 16) { if (rpl == 1) MSK_ELL(16, 1); else MSK_ELL(16, 2); }
    else return (int)hipErrorInvalidValue;
#undef MSK_ELL
    return (int)hipGetLastError();
  }
  const int rpl = (msk_tuning_flags & MSK_TUNE_DV_RPL1) ? 1 : (msk_tuning_flags & MSK_TUNE_DV_RPL2) ? 2 : 4;
  // LDS for the codes of one block: its entries plus both 16-byte roundings
  const size_t cap = ((size_t)rpl * max_block + 30 + 15) & ~(size_t)15;
  if (rpl == 1) {
    const unsigned g = (unsigned)((nrows + kT - 1) / kT);
    const XcdMap xm = xcd_map(nrows, plane);
#define MSK_DV(M) \
  k_spmv_dv<M><<<dim3(g), dim3(kT), cap, s>>>(nrows, rowptr, len8, code8, ddelta, dval, ndict, x, b, y, sdev, vout, \
                                              stop, xm)
    if (mode == MSK_SPMV_RESID) MSK_DV(MSK_SPMV_RESID);
    else if (mode == MSK_SPMV_SCALED) MSK_DV(MSK_SPMV_SCALED);
    else MSK_DV(MSK_SPMV_MULT);
#undef MSK_DV
    return (int)hipGetLastError();
  }
  const unsigned g = (unsigned)((nrows + kT * rpl - 1) / (kT * rpl));
#define MSK_DVB(M, R) \
  k_spmv_dvb<M, R><<<dim3(g), dim3(kT), cap, s>>>(nrows, rowptr, len8, code8, ddelta, dval, ndict, x, b, y, sdev, \
                                                  vout, stop)
  if (rpl == 2) {
    if (mode == MSK_SPMV_RESID) MSK_DVB(MSK_SPMV_RESID, 2);
    else if (mode == MSK_SPMV_SCALED) MSK_DVB(MSK_SPMV_SCALED, 2);
    else MSK_DVB(MSK_SPMV_MULT, 2);
  } else {
    if (mode == MSK_SPMV_RESID) MSK_DVB(MSK_SPMV_RESID, 4);
    else if (mode == MSK_SPMV_SCALED) MSK_DVB(MSK_SPMV_SCALED, 4);
    else MSK_DVB(MSK_SPMV_MULT, 4);
  }
#undef MSK_DVB
  return (int)hipGetLastError();
}

extern "C" int msk_spmm_ell(int32_t nrows, int W, const uint8_t* code8, const int32_t* ddelta, const double* dval,
                            int ndict, const double* S, int64_t lds, int nc, double* R, int64_t ldr, hipStream_t s) {
  if (nrows <= 0 || nc <= 0) return 0;
  const unsigned g = (unsigned)((nrows + kT - 1) / kT);
  if (W == 4) k_spmm_ell<4><<<g, kT, 0, s>>>(nrows, code8, ddelta, dval, ndict, S, lds, nc, R, ldr);
  else if (W == 8) k_spmm_ell<8><<<g, kT, 0, s>>>(nrows, code8, ddelta, dval, ndict, S, lds, nc, R, ldr);
  else if (W == 16) k_spmm_ell<16><<<g, kT, 0, s>>>(nrows, code8, ddelta, dval, ndict, S, lds, nc, R, ldr);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

extern "C" int msk_ell_encode(int32_t nrows, int W, const int32_t* rowptr, const int32_t* col, const double* val,
                              int ndict, const int32_t* ddelta, const double* dval, uint8_t* code8, int* fail,
                              hipStream_t s) {
  if (nrows <= 0) return 0;
  k_ell_encode<<<dim3(grid_for(nrows, 4096)), dim3(kT), 0, s>>>(nrows, W, rowptr, col, val, ndict, ddelta, dval,
                                                                code8, fail);
  return (int)hipGetLastError();
}

extern "C" int msk_dv_encode(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, int ndict,
                             const int32_t* ddelta, const double* dval, uint8_t* len8, uint8_t* code8, int* fail,
                             hipStream_t s) {
  if (nrows <= 0) return 0;
  k_dv_encode<<<dim3(grid_for(nrows, 4096)), dim3(kT), 0, s>>>(nrows, rowptr, col, val, ndict, ddelta, dval, len8,
                                                               code8, fail);
  return (int)hipGetLastError();
}

extern "C" int msk_spmv_mdot(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val,
                             const double* x, const double* sdev, double* y, int32_t lds_cap, const Vecs* V, int nv,
                             double* partial, int64_t nchunks, const int* stop, hipStream_t s) {
  if (nrows <= 0 || nchunks <= 0) return 0;
  if (lds_cap <= 0 || nv < 1 || nv > MSK_MAX_GROUP) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)lds_cap * 12;
  const dim3 g((unsigned)nchunks), b(kT);
#define MSK_SMD(VAR_, GF_) \
  k_spmv_mdot<VAR_, GF_><<<g, b, lds, s>>>(nrows, rowptr, col, val, x, sdev, y, lds_cap, *V, nv, partial, nchunks, stop)
  const bool g2 = (msk_tuning_flags & MSK_TUNE_SPMV_MDOT_G2) != 0;
  if (vec_var()) { if (g2) MSK_SMD(1, 2); else MSK_SMD(1, 4); }
  else { if (g2) MSK_SMD(0, 2); else MSK_SMD(0, 4); }
#undef MSK_SMD
  return (int)hipGetLastError();
}

extern "C" int msk_box_spmv_mdot(int32_t nx, int64_t P, int64_t n, int d2, const uint8_t* mask, const double* dval,
                                 const double* x, const double* sdev, double* y, const Vecs* V, int nv, double* partial,
                                 int64_t nchunks, const int* stop, int* self_out, hipStream_t s) {
  return msk_box_spmv_mdot_rv(nx, P, n, d2, mask, dval, nullptr, 0, x, sdev, y, V, nv, partial, nchunks, stop,
                              self_out, s);
}

// rv != null: the stencil storage's per-row values (marched form only, W stored)
extern "C" int msk_box_spmv_mdot_rv(int32_t nx, int64_t P, int64_t n, int d2, const uint8_t* mask, const double* dval,
                                    const double* rv, int64_t rvs, const double* x, const double* sdev, double* y,
                                    const Vecs* V, int nv, double* partial, int64_t nchunks, const int* stop,
                                    int* self_out, hipStream_t s) {
  if (self_out) *self_out = 0;
  if (n <= 0 || nchunks <= 0) return 0;
  if (nx < 2 || nx > 2048 || P < nx || nv < 1 || nv > MSK_MAX_GROUP || dv_flags_bad()) return (int)hipErrorInvalidValue;
  if (rv && (!y || d2 || P % kChunk || n % P || (nx & 1) || (rvs < 0 && nx > 1024))) return (int)hipErrorInvalidValue;
  // the symmetric storage adds the x+1 / y+1 legs' windows (2 x (4096 + nx) doubles; nx <= 1024: <= 128 KiB in all)
  const size_t lds = (size_t)(kChunk + 2 * nx + (rv && rvs < 0 ? 2 * (kChunk + nx) : 0)) * sizeof(double);
  const dim3 g((unsigned)nchunks), b(kT);
  const bool nty = !(msk_tuning_flags & MSK_TUNE_ELL_TEMPORAL_Y);
  if (!d2 && P % kChunk == 0 && n % P == 0 && (nx & 1) == 0 && (rv || !(msk_tuning_flags & MSK_TUNE_BOX_MDOT_FLAT))) {
    // whole chunks per plane: march zt planes per workgroup (MSPLIT_BOXMDOT_ZT overrides the depth, A/B)
    static const int zenv = [] {
      const char* e = getenv("MSPLIT_BOXMDOT_ZT");
      return e ? atoi(e) : 0;
    }();
    const int32_t nz = (int32_t)(n / P);
    // four planes per workgroup: half the workgroup prologues (the dependent loads of the plane below the first: x,
    // and for the STENCIL storage its z+1 leg) -- STENCIL step +1.9 %, SMSM block +0.3 %, 256^3 GMRES +0.1 % against
    // two (profiles/r05/stencil_sym2/zt/, profiles/r05/zt_dv/); one plane was -1.0 % (profiles/r03/wfree/fused_depth/)
    const int32_t zt = zenv > 0 ? zenv : 4;
    const int64_t grid = (P / kChunk) * ((nz + zt - 1) / zt);
    if (grid > INT32_MAX) return (int)hipErrorInvalidValue;
    // XCD-contiguous eighths from 32 tiles per plane (SMSM's 512^2 planes: +1.9 % over plane order, same box);
    // smaller planes in plane order (256^2: +1.4 % over the eighths; profiles/r03/boxmdot/xcd/)
    static const int rev = [] {
      const char* e = getenv("MSPLIT_BOXMDOT_REV");
      return e && atoi(e) ? 2 : 0;
    }();
    // MSPLIT_BOXMDOT_ALT=1: odd plane groups march down (k_box_spmv_mdot_march, xcd & 4), so the boundary planes
    // two groups both read are read at the same moment, the second time from the L2.  Measured (round 6,
    // profiles/r06/march_alt/): PMC 1.048 -> 1.019 of the algorithmic bytes for the symmetric STENCIL step and
    // 1.035 -> 1.011 for the DV step, but no faster (STENCIL -2.9 %, DV -0.1 %): those re-reads were MALL hits, the
    // kernels are bound by their streaming rate.  Off by default; read per call (the tests hold both orders to each
    // other and to the oracle).
    const char* alte = getenv("MSPLIT_BOXMDOT_ALT");
    const int alt = alte && alte[0] == '1' ? 4 : 0;
    const int xcd =
        ((P / kChunk) % 8 == 0 && P / kChunk >= 32 && !(msk_tuning_flags & MSK_TUNE_BOX_MDOT_NOXCD)) | rev | alt;
    // GMRES's basis ends with x (VV(it)): its dot from the march registers (MSPLIT_BOXMDOT_SELF=0: streamed, A/B)
    static const int self_env = [] {
      const char* e = getenv("MSPLIT_BOXMDOT_SELF");
      return e ? atoi(e) : 1;
    }();
    const double* last = V->base ? V->base + (int64_t)(nv - 1) * V->stride : V->p[nv - 1];
    const int self = self_env != 0 && last == x;
    if (self_out) *self_out = self;
    static const int rvp = [] {  // MSPLIT_RV_PREFETCH: row pairs whose values go before the barriers (8, 4 or 2)
      const char* e = getenv("MSPLIT_RV_PREFETCH");
      const int v = e ? atoi(e) : kIters;
      return v == 4 || v == 2 ? v : kIters;
    }();
#define MSK_BSMM_P(VAR_, NT_, RV_, P_)                                                                          \
  k_box_spmv_mdot_march<VAR_, NT_, RV_, P_><<<dim3((unsigned)grid), b, lds, s>>>(nx, P, nz, zt, xcd, mask, dval, rv, \
                                                                                 rvs, x, sdev, y, *V, nv, self,     \
                                                                                 partial, nchunks, stop)
#define MSK_BSMM(VAR_, NT_, RV_)                                                                              \
  do {                                                                                                        \
    if (RV_ == 1 && rvp == 4) MSK_BSMM_P(VAR_, NT_, RV_, 4);                                                  \
    else if (RV_ == 1 && rvp == 2) MSK_BSMM_P(VAR_, NT_, RV_, 2);                                             \
    else MSK_BSMM_P(VAR_, NT_, RV_, kIters);                                                                  \
  } while (0)
    // the symmetric storage: two threads per DBR lane where the windows fit (nx <= 512; MSPLIT_RV_SYM2=0: one, A/B)
    const char* s2e = getenv("MSPLIT_RV_SYM2");  // read per call: the tests hold the two forms to each other
    const bool sym2 = !(s2e && s2e[0] == '0') && nx <= 512;
#define MSK_SYM2(VAR_, NT_)                                                                               \
  k_box_spmv_mdot_march_sym2<VAR_, NT_><<<dim3((unsigned)grid), dim3(2 * kT), lds, s>>>(                   \
      nx, P, nz, zt, xcd, mask, rv, x, sdev, y, *V, nv, self, partial, nchunks, stop)
    if (rv && rvs < 0 && sym2) {
      if (vec_var()) { if (nty) MSK_SYM2(1, true); else MSK_SYM2(1, false); }
      else { if (nty) MSK_SYM2(0, true); else MSK_SYM2(0, false); }
    } else if (rv && rvs < 0) {  // the symmetric storage
      if (vec_var()) { if (nty) MSK_BSMM(1, true, 2); else MSK_BSMM(1, false, 2); }
      else { if (nty) MSK_BSMM(0, true, 2); else MSK_BSMM(0, false, 2); }
    } else if (rv) {
      if (vec_var()) { if (nty) MSK_BSMM(1, true, 1); else MSK_BSMM(1, false, 1); }
      else { if (nty) MSK_BSMM(0, true, 1); else MSK_BSMM(0, false, 1); }
    } else {
      if (vec_var()) { if (nty) MSK_BSMM(1, true, 0); else MSK_BSMM(1, false, 0); }
      else { if (nty) MSK_BSMM(0, true, 0); else MSK_BSMM(0, false, 0); }
    }
#undef MSK_SYM2
#undef MSK_BSMM
#undef MSK_BSMM_P
    return (int)hipGetLastError();
  }
#define MSK_BSM(D, VAR_, NT_) \
  k_box_spmv_mdot<D, VAR_, NT_><<<g, b, lds, s>>>(nx, P, n, mask, dval, x, sdev, y, *V, nv, partial, nchunks, stop)
#define MSK_BSM2(D)                                              \
  do {                                                           \
    if (vec_var()) { if (nty) MSK_BSM(D, 1, true); else MSK_BSM(D, 1, false); } \
    else { if (nty) MSK_BSM(D, 0, true); else MSK_BSM(D, 0, false); }           \
  } while (0)
  if (d2) MSK_BSM2(true);
  else MSK_BSM2(false);
#undef MSK_BSM2
#undef MSK_BSM
  return (int)hipGetLastError();
}

// whether msk_box_spmv_mdot takes its z-march form for this box (the condition above)
static bool box_mdot_marches(int32_t nx, int64_t P, int64_t n, int d2) {
  return !d2 && nx >= 2 && nx <= 2048 && P >= nx && P % kChunk == 0 && n > 0 && n % P == 0 && (nx & 1) == 0 &&
         !(msk_tuning_flags & MSK_TUNE_BOX_MDOT_FLAT) && !dv_flags_bad() && (n / P) <= INT32_MAX;
}

// the boxes msk_box_spmv_mdot takes (marched or not)
static bool box_mdot_fits(int32_t nx, int64_t P) { return nx >= 2 && nx <= 2048 && P >= nx && !dv_flags_bad(); }

extern "C" int msk_box_wfree_fits(int32_t nx, int64_t P, int64_t n, int d2) {
  return msk_gm_wfree && n > 0 && box_mdot_fits(nx, P) ? 1 : 0;
}

extern "C" int msk_box_maxpy_march(int32_t nx, int64_t P, int64_t n, int d2, const uint8_t* mask, const double* dval,
                                   const double* x, const double* sdev, double* wout, const Vecs* V, int nv,
                                   const double* adev, double* partial, const int* stop, hipStream_t s) {
  if (n <= 0) return 0;
  if (!box_mdot_fits(nx, P) || nv < 1) return (int)hipErrorInvalidValue;
  const double* last = V->base ? V->base + (int64_t)(nv - 1) * V->stride : (nv <= MSK_MAX_GROUP ? V->p[nv - 1] : nullptr);
  if (last != x) return (int)hipErrorInvalidValue;  // the basis must end with x (GMRES: VV(it))
  const bool nt = !(msk_tuning_flags & MSK_TUNE_MAXPY_TEMPORAL_ST);
  if (!box_mdot_marches(nx, P, n, d2)) {  // the unmarched form, one chunk per workgroup (as k_box_spmv_mdot)
    const int64_t nch = (n + kChunk - 1) / kChunk;
    if (nch > INT32_MAX) return (int)hipErrorInvalidValue;
    const size_t ldsu = (size_t)(kChunk + 2 * nx) * sizeof(double);
#define MSK_BMU(D_, VAR_, NT_)                                                                                      \
  k_box_maxpy<D_, VAR_, NT_><<<dim3((unsigned)nch), dim3(kT), ldsu, s>>>(nx, P, n, mask, dval, x, sdev, wout, *V, nv, \
                                                                        adev, partial, stop)
#define MSK_BMU2(D_)                                                                          \
  do {                                                                                        \
    if (vec_var()) { if (nt) MSK_BMU(D_, 1, true); else MSK_BMU(D_, 1, false); }              \
    else { if (nt) MSK_BMU(D_, 0, true); else MSK_BMU(D_, 0, false); }                        \
  } while (0)
    if (d2) MSK_BMU2(true);
    else MSK_BMU2(false);
#undef MSK_BMU2
#undef MSK_BMU
    return (int)hipGetLastError();
  }
  static const int zenv = [] {
    const char* e = getenv("MSPLIT_MAXPY_ZT");
    return e ? atoi(e) : 0;
  }();
  static const int rev_env = [] {
    const char* e = getenv("MSPLIT_MAXPY_REV");
    return e ? (atoi(e) ? 1 : 0) : -1;
  }();
  const int32_t nz = (int32_t)(n / P);
  // one plane per workgroup (x(z-+1) loaded per plane, twice the workgroups of the fused kernel's 2-plane march):
  // 256^3 GMRES step 2.261 -> 2.336e10 over 2 planes, MAXPY 392 -> 368 us (profiles/r03/wfree/ab/)
  const int32_t zt = zenv > 0 ? zenv : 1;
  const int64_t grid = (P / kChunk) * ((nz + zt - 1) / zt);
  if (grid > INT32_MAX) return (int)hipErrorInvalidValue;
  const int rev = (rev_env < 0 ? n > ((int64_t)1 << 25) : rev_env) ? 2 : 0;
  const int xcd = ((P / kChunk) % 8 == 0 && P / kChunk >= 32 && !(msk_tuning_flags & MSK_TUNE_BOX_MDOT_NOXCD)) | rev;
  const size_t lds = (size_t)(kChunk + 2 * nx) * sizeof(double);
  const bool nty = nt;
  // MSPLIT_MAXPY_MARCH_U2=1: the group loop unrolled by two (A/B)
  static const int u2 = [] {
    const char* e = getenv("MSPLIT_MAXPY_MARCH_U2");
    return e ? atoi(e) : 0;
  }();
#define MSK_BMM(VAR_, NT_)                                                                                      \
  k_box_maxpy_march<VAR_, NT_><<<dim3((unsigned)grid), dim3(kT), lds, s>>>(nx, P, nz, zt, xcd, mask, dval, x,  \
                                                                           sdev, wout, *V, nv, adev, partial, stop)
  if (u2 && vec_var() && nty) MSK_BMM(33, true);
  else if (vec_var()) { if (nty) MSK_BMM(1, true); else MSK_BMM(1, false); }
  else { if (nty) MSK_BMM(0, true); else MSK_BMM(0, false); }
#undef MSK_BMM
  return (int)hipGetLastError();
}

extern "C" int msk_spmm(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* S,
                        int64_t lds, int nc, double* R, int64_t ldr, int32_t lds_cap, hipStream_t s) {
  if (nrows <= 0 || nc <= 0) return 0;
  if (lds_cap <= 0) return (int)hipErrorInvalidValue;  // rows too long for the LDS stage
  const unsigned g = (unsigned)((nrows + kT - 1) / kT);
  k_spmm_lds8<<<dim3(g), dim3(kT), (size_t)lds_cap * 12, s>>>(nrows, rowptr, col, val, S, lds, nc, R, ldr, lds_cap);
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
#endif  // part

#if MSK_IN(MSK_PART_MISC)
extern "C" int msk_box_stencil(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows, int lo, int hi,
                               const BoxCoef* cf, int32_t* rowptr, int32_t* col, double* val, hipStream_t s) {
  const int g = grid_for(nrows + 1, 8192);
  k_box_stencil<<<dim3(g), dim3(kT), 0, s>>>(dim, nx, ny, nz, nrows, lo, hi, *cf, rowptr, col, val);
  return (int)hipGetLastError();
}

extern "C" int msk_stencil_spmv(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows, int lo, int hi,
                                const BoxCoef* cf, const double* x, const double* b, double* y, int mode,
                                const double* sdev, double* vout, const int* stop, hipStream_t s) {
  if (nrows <= 0) return 0;
  // pairs need an even line length and 16-byte aligned vectors (x offset by a whole plane when lo)
  const int64_t P = dim == 3 ? (int64_t)nx * ny : (int64_t)nx;
  const bool v2 = nx % 2 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                  (!b || ((uintptr_t)b & 15) == 0) && (!vout || ((uintptr_t)vout & 15) == 0) && (!lo || P % 2 == 0);
  const int per = v2 ? 2 * kT : kT;
  const dim3 g((unsigned)((nx + per - 1) / per), (unsigned)ny, (unsigned)(dim == 3 ? nz : 1));
#define MSK_ST(M, V) k_stencil_spmv<M, V><<<g, dim3(kT), 0, s>>>(dim, nx, ny, nz, lo, hi, *cf, x, b, y, sdev, vout, stop)
  if (mode == MSK_SPMV_RESID) { if (v2) MSK_ST(MSK_SPMV_RESID, true); else MSK_ST(MSK_SPMV_RESID, false); }
  else if (mode == MSK_SPMV_SCALED) { if (v2) MSK_ST(MSK_SPMV_SCALED, true); else MSK_ST(MSK_SPMV_SCALED, false); }
  else { if (v2) MSK_ST(MSK_SPMV_MULT, true); else MSK_ST(MSK_SPMV_MULT, false); }
#undef MSK_ST
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
#endif  // part
