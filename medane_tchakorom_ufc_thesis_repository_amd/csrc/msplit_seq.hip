// msplit_seq.hip -- the parity reduction order, MSP_REDUCE_SEQ (include/msplit.h).
//
// PETSc's Seq kernels form every reduction as one running sum with the
// elements in index order:
//   VecDot_Seq / VecNorm_Seq (NORM_2)  BLASdot = f2cblaslapack ddot (the
//                                      reference's --download-f2cblaslapack,
//                                      config/petsc/arch-linux-mpich-g5k-opt.py);
//                                      its unroll-by-5 body is evaluated left to
//                                      right, i.e. still sequential
//   VecMDot_Seq                        per vector, sequential
//   MatMultTranspose_SeqDense          dgemv 'T': per column, sequential
//   MatNorm_SeqDense NORM_FROBENIUS    a plain sum of squares over the
//                                      column-major array (BLASnrm2 only under
//                                      PETSC_USE_REAL___FP16), then sqrt
// and the reference's outer LSQR runs on one rank over the whole of R
// (SMSM-global.c:136, comm_jacobi_block with one process per block), so its
// sums run across the row blocks in block order.  oracle/oracle.c's
// ORC_REDUCE_SEQ restates exactly this.
//
// A sequential sum cannot be parallelised without changing its roundings, so
// this is a parity mode, not a fast path: the products are formed by the
// whole workgroup into LDS (the loads stay coalesced, and each product is the
// same IEEE multiplication the DBR kernels do), and one lane adds them in
// order while the other waves form the next tile.  Results go out in the DBR
// partial layout -- partial[v*nchunks + 0] = the sum, the other chunks +0.0 --
// so the unchanged stage 2 (or the fused GMRES norm/Hessenberg update) folds
// them to exactly the sequential sum: x + (+0.0) == x for every x a sum of
// products starting at +0.0 can produce.
#include <hip/hip_runtime.h>

#include "msplit_ctx.hpp"

namespace {

constexpr int kT = 256;      // threads per workgroup
constexpr int kTile = 2048;  // products per LDS tile

__device__ __forceinline__ bool stopped(const int* stop) { return stop && *stop; }

// One segment: x[i] * (y[i] * sy) (y == nullptr: x[i] * x[i]), added to acc in
// index order.  Wave 0 lane 0 sums; waves 1..3 form the next tile meanwhile.
__device__ double seq_segment(const double* __restrict__ x, const double* __restrict__ y, double sy, int64_t n,
                              double acc, double (*buf)[kTile]) {
  const int t = threadIdx.x;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  auto fill = [&](int64_t tile, double* dst, int t0, int nt) {
    const int64_t base = tile * kTile;
    const int cnt = (int)((n - base) < kTile ? (n - base) : kTile);
    for (int i = t0; i < cnt; i += nt) {
      const double xi = x[base + i];
      dst[i] = y ? xi * (y[base + i] * sy) : xi * xi;
    }
  };
  if (ntiles > 0) fill(0, buf[0], t, kT);
  __syncthreads();
  for (int64_t tile = 0; tile < ntiles; ++tile) {
    if (t >= 64) {
      if (tile + 1 < ntiles) fill(tile + 1, buf[(tile + 1) & 1], t - 64, kT - 64);
    } else if (t == 0) {
      const double* p = buf[tile & 1];
      const int64_t base = tile * kTile;
      const int cnt = (int)((n - base) < kTile ? (n - base) : kTile);
      int i = 0;
      for (; i + 32 <= cnt; i += 32) {
        double q[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) q[u] = p[i + u];
#pragma unroll
        for (int u = 0; u < 32; ++u) acc = acc + q[u];
      }
      for (; i < cnt; ++i) acc = acc + p[i];
    }
    __syncthreads();
  }
  return acc;
}

// Workgroup v: w . V_v (self: w . w) in sequential order, written in the DBR
// partial layout of row v.
__global__ __launch_bounds__(kT) void k_seq_stage1(const double* __restrict__ w, Vecs V, int64_t n, int self,
                                                   double* __restrict__ partial, int64_t nchunks,
                                                   const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double buf[2][kTile];
  const int v = blockIdx.x;
  const double* y = self ? nullptr : (V.base ? V.base + (int64_t)v * V.stride : V.p[v]);
  const double sy = (!self && V.scale) ? V.scale[v] : 1.0;
  const double acc = seq_segment(w, y, sy, n, 0.0, buf);
  double* row = partial + (int64_t)v * nchunks;
  for (int64_t c = threadIdx.x; c < nchunks; c += kT) row[c] = c == 0 ? acc : 0.0;
}

// Chained sums over the row blocks of one process (LSQR): workgroup j sums
// column_j . y over segment 0, then segment 1, ... (frob: one workgroup, the
// squares of column 0 over all segments, then column 1, ...).
__global__ __launch_bounds__(kT) void k_seq_chain(mspi_seq_segs sg, int ncol, int frob, double* __restrict__ out,
                                                  int m, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double buf[2][kTile];
  const int j = blockIdx.x;
  double acc = 0.0;
  const int j0 = frob ? 0 : j, j1 = frob ? ncol : j + 1;
  for (int jj = j0; jj < j1; ++jj)
    for (int k = 0; k < sg.nseg; ++k) {
      const double* x = sg.x[k] + (int64_t)jj * sg.ldx[k];
      acc = seq_segment(x, frob ? nullptr : sg.y[k], 1.0, sg.n[k], acc, buf);
    }
  if (threadIdx.x != 0) return;
  // only the last block's slot carries the sum: a block-order sum of the slots is the chain
  if (frob) {
    for (int k = 0; k < sg.nseg; ++k)
      for (int jj = 0; jj < ncol; ++jj) out[k * m + jj] = (k == sg.nseg - 1 && jj == ncol - 1) ? acc : 0.0;
  } else {
    for (int k = 0; k < sg.nseg; ++k) out[k * m + j] = k == sg.nseg - 1 ? acc : 0.0;
  }
}

}  // namespace

extern "C" int msk_seq_stage1(const double* w, const Vecs* V, int nv, int64_t n, int self, double* partial,
                              int64_t nchunks, const int* stop, hipStream_t s) {
  if (nv < 1 || nv > MSK_MAX_GROUP || (self && nv != 1) || nchunks < 1) return (int)hipErrorInvalidValue;
  k_seq_stage1<<<dim3(nv), dim3(kT), 0, s>>>(w, *V, n, self, partial, nchunks, stop);
  return (int)hipGetLastError();
}

extern "C" int mspi_reduce_seq(const msp_ctx* c) { return c->reduce == MSP_REDUCE_SEQ; }

extern "C" int mspi_seq_chain(msp_ctx* c, const mspi_seq_segs* sg, int ncol, int frob, double* out, int m,
                              const int* stop) {
  ARGCHK(sg && out && sg->nseg >= 1 && sg->nseg <= MSPI_SEQ_MAXSEG && ncol >= 1 && ncol <= m, MSP_ERR_ARG_OUTOFRANGE,
         "sequential chain over %d segments, %d columns", sg ? sg->nseg : -1, ncol);
  k_seq_chain<<<dim3(frob ? 1 : ncol), dim3(kT), 0, c->stream>>>(*sg, ncol, frob, out, m, stop);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}
