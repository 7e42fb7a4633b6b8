// msplit_gmres.hip -- the scalar recurrence of KSPGMRES on the device.
//
// PETSc's KSPGMRESCycle alternates vector work with a few scalar steps (the
// Givens update of one Hessenberg column, the happy-breakdown and convergence
// tests, the residual history).  Doing those on the host costs a device->host
// round trip per Arnoldi step.  Here they run in one-lane kernels reading and
// writing a device-resident state (mspi_gmres_state), so the host enqueues a
// whole restart cycle and synchronises once per cycle.  Each one-lane kernel is
// a literal restatement of the corresponding PETSc 3.22.1 code (the same
// statements as oracle/oracle.c); with IEEE division and square root correctly
// rounded on gfx950 and no FMA contraction, the recurrence is bitwise the
// host's.
#include <hip/hip_runtime.h>

#include <cmath>

#include "msplit.h"
#include "msplit_internal.h"

namespace {

#define HHD(a, b) (g.hh[(int64_t)(b) * (st->m + 2) + (a)])

__device__ inline bool bad(double v) { return isnan(v) || isinf(v); }

__device__ inline void log_res(const mspi_gmres_dev& g, double r) {
  mspi_gmres_state* st = g.st;
  if (st->nhist < st->hist_cap) g.hist[st->nhist] = r;
  st->nhist++;
}

// KSPConvergedDefault
__device__ inline void converged(const mspi_gmres_dev& g, int n, double rnorm) {
  mspi_gmres_state* st = g.st;
  st->reason = MSP_CONVERGED_ITERATING;
  if (n == 0) {
    if (!st->guess_zero && !st->uirnorm) {
      double snorm = st->bnorm;
      if (snorm == 0.0) snorm = rnorm;
      st->rnorm0 = snorm;
    } else {
      st->rnorm0 = rnorm;
    }
    const double t = st->rtol * st->rnorm0;
    st->ttol = t < st->abstol ? st->abstol : t;  // PetscMax
  }
  if (bad(rnorm)) st->reason = MSP_DIVERGED_NANORINF;
  else if (rnorm <= st->ttol) st->reason = (rnorm < st->abstol) ? MSP_CONVERGED_ATOL : MSP_CONVERGED_RTOL;
  else if (rnorm >= st->divtol * st->rnorm0) st->reason = MSP_DIVERGED_DTOL;
}

// Start of KSPGMRESCycle, after VecNorm(VV(0)).  VecNormalize is deferred: VV(0)
// stays as stored and sc[0] = 1/||VV(0)|| multiplies every read of it.
__global__ void k_cycle_start(mspi_gmres_dev g, const double* __restrict__ sumsq) {
  mspi_gmres_state* st = g.st;
  st->it = 0;
  st->stop = 0;
  st->skip_build = 0;
  const double res = sqrt(*sumsq);
  st->scale = (res != 0.0 && !bad(res)) ? 1.0 / res : 1.0;
  g.sc[0] = st->scale;
  if (bad(res)) {  // KSPCheckNorm: return
    st->reason = MSP_DIVERGED_NANORINF;
    st->stop = st->skip_build = 1;
    return;
  }
  if (st->rnorm > 0.0 && fabs(res - st->rnorm) > st->breakdowntol * st->gm_rnorm0) {
    st->reason = MSP_DIVERGED_BREAKDOWN;
    st->stop = st->skip_build = 1;
    return;
  }
  g.grs[0] = st->gm_rnorm0 = res;
  st->rnorm = res;
  st->res = res;
  log_res(g, res);
  if (res == 0.0) {
    st->reason = MSP_CONVERGED_ATOL;
    st->stop = st->skip_build = 1;
    return;
  }
  converged(g, st->its, res);
  if (st->reason || !(st->its < st->max_it) || st->m < 1) st->stop = 1;  // the while loop does not run
}

// KSPGMRESUpdateHessenberg
__device__ inline void update_hessenberg(const mspi_gmres_dev& g, int it, int hapend, double* res) {
  mspi_gmres_state* st = g.st;
  double* hh = &HHD(0, it);
  for (int j = 1; j <= it; ++j) {
    const double tt = hh[j - 1];
    hh[j - 1] = g.cc[j - 1] * tt + g.ss[j - 1] * hh[j];
    hh[j] = g.cc[j - 1] * hh[j] - (g.ss[j - 1] * tt);
  }
  if (!hapend) {
    const double tt = sqrt(hh[it] * hh[it] + hh[it + 1] * hh[it + 1]);
    if (tt == 0.0) {
      st->reason = MSP_DIVERGED_NULL;
      return;
    }
    g.cc[it] = hh[it] / tt;
    g.ss[it] = hh[it + 1] / tt;
    g.grs[it + 1] = -(g.ss[it] * g.grs[it]);
    g.grs[it] = g.cc[it] * g.grs[it];
    hh[it] = g.cc[it] * hh[it] + g.ss[it] * hh[it + 1];
    *res = fabs(g.grs[it + 1]);
  } else {
    *res = 0.0;
  }
}

// The rest of one KSPGMRESCycle iteration once h(0..it) = VecMDot and
// h(it+1) = ||w||^2 (after the CGS VecMAXPY) are in HBM.
__global__ void k_iter_update(mspi_gmres_dev g) {
  mspi_gmres_state* st = g.st;
  if (st->stop) return;
  const int it = st->it;
  double* hh = &HHD(0, it);
  bool nan_dot = false;
  for (int j = 0; j <= it; ++j) {
    hh[j] = 0.0;
    if (bad(g.h[j])) nan_dot = true;
  }
  double res = st->res;
  int hapend = 0;
  if (nan_dot) {  // KSPCheckDot in the orthogonalisation -> break
    st->reason = MSP_DIVERGED_NANORINF;
  } else {
    for (int j = 0; j <= it; ++j) hh[j] -= -g.h[j];  // lhh = -lhh; hh -= lhh
    const double tt = sqrt(g.h[it + 1]);
    if (bad(tt)) {  // KSPCheckNorm: return without BuildSoln
      st->reason = MSP_DIVERGED_NANORINF;
      st->stop = st->skip_build = 1;
      return;
    }
    st->scale = (tt != 0.0) ? 1.0 / tt : 1.0;  // VecNormalize of VV(it+1), deferred to its readers
    g.sc[it + 1] = st->scale;
    HHD(it + 1, it) = tt;
    double hapbnd = fabs(tt / g.grs[it]);
    if (hapbnd > st->haptol) hapbnd = st->haptol;
    if (tt < hapbnd) hapend = 1;
    update_hessenberg(g, it, hapend, &res);
    st->it = it + 1;
    st->its++;
    st->rnorm = res;
    st->res = res;
    if (!st->reason) {
      converged(g, st->its, res);
      if (hapend && !st->reason) st->reason = MSP_DIVERGED_BREAKDOWN;
    }
  }
  const int itn = st->it;
  if (!st->reason && itn < st->m && st->its < st->max_it) {
    log_res(g, res);  // "if (it) log" at the top of the next iteration
    return;
  }
  st->stop = 1;  // loop exit
  if (itn && (st->reason || st->its >= st->max_it)) log_res(g, res);
}

// The same step fused with the stage-2 DBR reduction of ||w||^2 (the partials the
// norm-fused CGS VecMAXPY left): one launch instead of two, and the serial
// recurrence reads the column, cc and ss from LDS (staged by all lanes) instead of
// one dependent global load after another.  The sum is k_dot_stage2's, the
// recurrence k_iter_update's statement for statement: results are identical.
constexpr int kUT = 256;

__device__ inline double fold_partials(const double* __restrict__ p, int64_t nchunks, double* red) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double acc = 0.0;
  int64_t i = t;
  // k_dot_stage2's order: lane t adds p[t], p[t+256], ... (16 loads in flight, then 8, then one at a time)
  for (; i + 15 * kUT < nchunks; i += 16 * kUT) {
    double q[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) q[u] = p[i + u * kUT];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = acc + q[u];
  }
  for (; i + 7 * kUT < nchunks; i += 8 * kUT) {
    double q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) q[u] = p[i + u * kUT];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = acc + q[u];
  }
  for (; i < nchunks; i += kUT) acc = acc + p[i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
  if (lane == 0) red[wv] = acc;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// The state, the column h(0..m+1), cc, ss and grs are loaded into LDS by all lanes together with the
// partials, so the serial recurrence of lane 0 waits for one round of loads, not one per field; the
// state is stored back at the end.  m = the restart length the arrays are sized for (st->m).
constexpr int kStW = (int)(sizeof(mspi_gmres_state) / sizeof(int32_t));
static_assert(sizeof(mspi_gmres_state) % sizeof(int32_t) == 0, "state copied as 32-bit words");
static_assert(kStW <= kUT, "one word per lane");

__global__ __launch_bounds__(kUT) void k_norm_update(mspi_gmres_dev g, const double* __restrict__ partial,
                                                     int64_t nchunks, int m) {
  __shared__ double red[4];
  __shared__ mspi_gmres_state lst;
  extern __shared__ double lds[];  // hh column, cc, ss, grs: m+2 each
  const int t = threadIdx.x, m2 = m + 2;
  double* lh = lds;
  double* lc = lds + m2;
  double* ls = lds + 2 * m2;
  double* lg = lds + 3 * m2;
  if (t < kStW) reinterpret_cast<int32_t*>(&lst)[t] = reinterpret_cast<const int32_t*>(g.st)[t];
  for (int j = t; j < m2; j += kUT) {
    lh[j] = g.h[j];
    lc[j] = g.cc[j];
    ls[j] = g.ss[j];
    lg[j] = g.grs[j];
  }
  const double sumsq = fold_partials(partial, nchunks, red);  // its barrier publishes the LDS copies too
  if (lst.stop) return;                                       // uniform
  mspi_gmres_dev gl = g;
  gl.st = &lst;  // converged() and log_res() on the LDS state
  mspi_gmres_state* st = &lst;
  const int it = st->it;
  __shared__ int ncol;
  if (t == 0) {
    g.h[it + 1] = sumsq;
    ncol = 0;
    bool nan_dot = false;
    for (int j = 0; j <= it; ++j)
      if (bad(lh[j])) nan_dot = true;
    double* hh = lh;  // the column, built in LDS: hh[j] = 0 - (-h[j])
    double res = st->res;
    int hapend = 0;
    bool done = false;
    if (nan_dot) {
      st->reason = MSP_DIVERGED_NANORINF;
      for (int j = 0; j <= it; ++j) hh[j] = 0.0;
      ncol = it + 1;
    } else {
      for (int j = 0; j <= it; ++j) {
        double v = 0.0;
        v -= -hh[j];
        hh[j] = v;
      }
      const double tt = sqrt(sumsq);
      if (bad(tt)) {
        st->reason = MSP_DIVERGED_NANORINF;
        st->stop = st->skip_build = 1;
        ncol = it + 1;
        done = true;
      } else {
        st->scale = (tt != 0.0) ? 1.0 / tt : 1.0;  // VecNormalize of VV(it+1), deferred to its readers
        g.sc[it + 1] = st->scale;
        hh[it + 1] = tt;
        double hapbnd = fabs(tt / lg[it]);
        if (hapbnd > st->haptol) hapbnd = st->haptol;
        if (tt < hapbnd) hapend = 1;
        // KSPGMRESUpdateHessenberg on the LDS column
        for (int j = 1; j <= it; ++j) {
          const double a = hh[j - 1];
          hh[j - 1] = lc[j - 1] * a + ls[j - 1] * hh[j];
          hh[j] = lc[j - 1] * hh[j] - (ls[j - 1] * a);
        }
        if (!hapend) {
          const double r = sqrt(hh[it] * hh[it] + hh[it + 1] * hh[it + 1]);
          if (r == 0.0) {
            st->reason = MSP_DIVERGED_NULL;
          } else {
            const double c = hh[it] / r, sn = hh[it + 1] / r;
            g.cc[it] = c;
            g.ss[it] = sn;
            const double grs = lg[it];
            g.grs[it + 1] = -(sn * grs);
            g.grs[it] = c * grs;
            hh[it] = c * hh[it] + sn * hh[it + 1];
            res = fabs(-(sn * grs));
          }
        } else {
          res = 0.0;
        }
        ncol = it + 2;
        st->it = it + 1;
        st->its++;
        st->rnorm = res;
        st->res = res;
        if (!st->reason) {
          converged(gl, st->its, res);
          if (hapend && !st->reason) st->reason = MSP_DIVERGED_BREAKDOWN;
        }
      }
    }
    if (!done) {
      const int itn = st->it;
      if (!st->reason && itn < st->m && st->its < st->max_it) {
        log_res(gl, res);
      } else {
        st->stop = 1;
        if (itn && (st->reason || st->its >= st->max_it)) log_res(gl, res);
      }
    }
  }
  __syncthreads();
  double* col = &HHD(0, it);
  for (int j = t; j < ncol; j += kUT) col[j] = lh[j];
  if (t < kStW) const_cast<int32_t*>(reinterpret_cast<const int32_t*>(g.st))[t] = reinterpret_cast<int32_t*>(&lst)[t];
}

// KSPGMRESBuildSoln(GRS(0), x, x, ksp, it - 1): back-solve in place (nrs
// aliases GRS); the x update is the accumulate-MAXPY that follows.
__global__ void k_build(mspi_gmres_dev g) {
  mspi_gmres_state* st = g.st;
  st->nbuild = 0;
  if (st->skip_build) return;
  const int it = st->it - 1;
  if (it < 0) return;
  double* nrs = g.grs;
  if (HHD(it, it) != 0.0) {
    nrs[it] = g.grs[it] / HHD(it, it);
  } else {
    st->reason = MSP_DIVERGED_BREAKDOWN;
    return;
  }
  for (int ii = 1; ii <= it; ++ii) {
    const int k = it - ii;
    double tt = g.grs[k];
    for (int j = k + 1; j <= it; ++j) tt = tt - HHD(k, j) * nrs[j];
    if (HHD(k, k) == 0.0) {
      st->reason = MSP_DIVERGED_BREAKDOWN;
      return;
    }
    nrs[k] = tt / HHD(k, k);
  }
  st->nbuild = it + 1;
}

// The same back-solve with H(0..it, 0..it) and GRS staged in LDS by all lanes first, so lane 0's serial loop
// reads LDS instead of one dependent HBM/L2 load per term; the same statements in the same order (bitwise
// k_build).  m: the restart the arrays are sized for (H has m+1 columns of m+2 entries).
__global__ __launch_bounds__(kUT) void k_build_lds(mspi_gmres_dev g, int m) {
  __shared__ mspi_gmres_state lst;
  extern __shared__ double lds[];  // H: (m+1) x (m+2), then GRS: m+2
  const int t = threadIdx.x, m2 = m + 2;
  double* lh = lds;
  double* lg = lds + (size_t)(m + 1) * m2;
  if (t < kStW) reinterpret_cast<int32_t*>(&lst)[t] = reinterpret_cast<const int32_t*>(g.st)[t];
  for (int i = t; i < (m + 1) * m2; i += kUT) lh[i] = g.hh[i];
  for (int i = t; i < m2; i += kUT) lg[i] = g.grs[i];
  __syncthreads();
  mspi_gmres_state* st = &lst;
  __shared__ int nw;  // GRS entries to write back
  if (t == 0) {
    nw = 0;
    st->nbuild = 0;
    const int it = st->it - 1;
    if (!st->skip_build && it >= 0) {
#define LHH(a, b) lh[(b) * m2 + (a)]
      double* nrs = lg;
      bool ok = true;
      if (LHH(it, it) != 0.0) {
        nrs[it] = lg[it] / LHH(it, it);
      } else {
        st->reason = MSP_DIVERGED_BREAKDOWN;
        ok = false;
      }
      for (int ii = 1; ok && ii <= it; ++ii) {
        const int k = it - ii;
        double tt = lg[k];
#pragma unroll 8
        for (int j = k + 1; j <= it; ++j) tt = tt - LHH(k, j) * nrs[j];  // the LDS reads of 8 terms issued together
        if (LHH(k, k) == 0.0) {
          st->reason = MSP_DIVERGED_BREAKDOWN;
          ok = false;
          nw = it + 1;
          break;
        }
        nrs[k] = tt / LHH(k, k);
      }
#undef LHH
      nw = it + 1;
      if (ok) st->nbuild = it + 1;
    }
  }
  __syncthreads();
  for (int i = t; i < nw; i += kUT) g.grs[i] = lg[i];
  if (t < kStW) const_cast<int32_t*>(reinterpret_cast<const int32_t*>(g.st))[t] = reinterpret_cast<int32_t*>(&lst)[t];
}

}  // namespace

// ctx stream accessor lives in msplit_runtime.hip
extern "C" hipStream_t mspi_stream(msp_ctx* ctx);

extern "C" int mspi_gm_cycle_start(msp_ctx* ctx, mspi_gmres_dev g, const double* sumsq_dev) {
  k_cycle_start<<<1, 1, 0, mspi_stream(ctx)>>>(g, sumsq_dev);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    mspi_set_error(MSP_ERR_LIB, "k_cycle_start: %s", hipGetErrorString(e));
    return MSP_ERR_LIB;
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_gm_iter_update(msp_ctx* ctx, mspi_gmres_dev g) {
  k_iter_update<<<1, 1, 0, mspi_stream(ctx)>>>(g);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    mspi_set_error(MSP_ERR_LIB, "k_iter_update: %s", hipGetErrorString(e));
    return MSP_ERR_LIB;
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_gm_norm_update(msp_ctx* ctx, mspi_gmres_dev g, const double* partial, int64_t nchunks, int m) {
  const size_t lds = (size_t)4 * (m + 2) * sizeof(double);
  k_norm_update<<<1, kUT, lds, mspi_stream(ctx)>>>(g, partial, nchunks, m);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    mspi_set_error(MSP_ERR_LIB, "k_norm_update: %s", hipGetErrorString(e));
    return MSP_ERR_LIB;
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_gm_build(msp_ctx* ctx, mspi_gmres_dev g, int m) {
  const size_t lds = ((size_t)(m + 1) * (m + 2) + (m + 2)) * sizeof(double);
  if (lds <= 48 * 1024) k_build_lds<<<1, kUT, lds, mspi_stream(ctx)>>>(g, m);  // restart <= 75
  else k_build<<<1, 1, 0, mspi_stream(ctx)>>>(g);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    mspi_set_error(MSP_ERR_LIB, "k_build: %s", hipGetErrorString(e));
    return MSP_ERR_LIB;
  }
  return MSP_SUCCESS;
}
