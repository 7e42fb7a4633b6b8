// msplit_lsqr.hip -- the scalar recurrence of KSPSolve_LSQR [PETSc-ext] on the
// device (one lane), so an LSQR solve is enqueued without a host round trip
// per step (ksp_lsqr.c syncs once per chunk of steps).  The s-vectors
// (V, V1, W, x: s <= a few tens) live here too; they are replicated on every
// rank and computed identically from the all-gathered block partials.
//
// The operation sequence and every rounding are the oracle's
// (oracle/oracle.c, orc_lsqr_solve): block partials added in block order from
// 0.0, s-vector norms as sequential sums, VecScale/VecAXPY/VecAYPX with their
// PETSc special cases (alpha == 0 / 1), no FMA contraction.
#include <hip/hip_runtime.h>

#include <cmath>

#include "msplit_ctx.hpp"

namespace {

__device__ __forceinline__ bool bad(double v) { return isnan(v) || isinf(v); }

__device__ void ls_log(mspi_lsqr_dev d, double r) {
  mspi_lsqr_state* st = d.st;
  if (st->nhist < st->hist_cap) d.hist[st->nhist] = r;
  st->nhist++;
}

// KSPConvergedDefault (zero guess) + KSPLSQRConvergedDefault / KSPConvergedSkip
__device__ void ls_converged(mspi_lsqr_state* st, int n, double rnorm) {
  st->reason = MSP_CONVERGED_ITERATING;
  if (st->conv_test == MSP_LSQR_CONV_SKIP) {
    if (n >= st->max_it) st->reason = MSP_CONVERGED_ITS;
    return;
  }
  if (n == 0) {
    st->rnorm0 = rnorm;
    const double t = st->rtol * st->rnorm0;
    st->ttol = t < st->abstol ? st->abstol : t;  // PetscMax
  }
  if (bad(rnorm)) {
    st->reason = MSP_DIVERGED_NANORINF;
  } else if (rnorm <= st->ttol) {
    st->reason = rnorm < st->abstol ? MSP_CONVERGED_ATOL : MSP_CONVERGED_RTOL;
  } else if (rnorm >= st->divtol * st->rnorm0) {
    st->reason = MSP_DIVERGED_DTOL;
  }
  if (st->conv_test != MSP_LSQR_CONV_LSQR || n == 0 || st->reason) return;
  if (st->arnorm < st->abstol) st->reason = MSP_CONVERGED_ATOL_NORMAL;
  else if (st->arnorm < st->rtol * st->anorm * rnorm) st->reason = MSP_CONVERGED_RTOL_NORMAL;
}

__device__ double block_sum(const double* g, int nblk, int m, int j) {
  double t = 0.0;
  for (int b = 0; b < nblk; ++b) t += g[b * m + j];
  return t;
}

__device__ double snorm(const double* v, int s) {
  double t = 0.0;
  for (int j = 0; j < s; ++j) t += v[j] * v[j];
  return sqrt(t);
}

__device__ void vscale(double* v, int s, double a) {  // VecScale
  if (a == 0.0) {
    for (int j = 0; j < s; ++j) v[j] = 0.0;
  } else if (a != 1.0) {
    for (int j = 0; j < s; ++j) v[j] = v[j] * a;
  }
}

__device__ void vaxpy(double* y, int s, double a, const double* x) {  // VecAXPY
  if (a == 0.0) return;
  for (int j = 0; j < s; ++j) y[j] = y[j] + a * x[j];
}

__device__ void vaypx(double* y, int s, double a, const double* x) {  // VecAYPX
  if (a == 0.0) {
    for (int j = 0; j < s; ++j) y[j] = x[j];
  } else if (a == 1.0) {
    for (int j = 0; j < s; ++j) y[j] = y[j] + x[j];
  } else {
    for (int j = 0; j < s; ++j) y[j] = x[j] + a * y[j];
  }
}

// rnorm = ||b|| from the block partials; n = 0 test; U scale 1/beta
__global__ void k_ls_start(mspi_lsqr_dev d) {
  mspi_lsqr_state* st = d.st;
  if (st->stop) return;
  for (int j = 0; j < st->s; ++j) d.X[j] = 0.0;  // zero initial guess
  const double rnorm = sqrt(block_sum(d.g, st->nblk, 1, 0));
  st->rnorm = rnorm;
  if (bad(rnorm)) {  // KSPCheckNorm
    st->reason = MSP_DIVERGED_NANORINF;
    st->stop = 1;
    return;
  }
  st->its = 0;
  ls_log(d, rnorm);
  ls_converged(st, 0, rnorm);
  if (st->reason) {
    st->stop = 1;
    return;
  }
  st->beta = rnorm;
  st->uscale = 1.0 / rnorm;
}

// V = R^T U (gathered), alpha = ||V||, V /= alpha, W = V, the LSQR scalars
__global__ void k_ls_first(mspi_lsqr_dev d, const double* gfrob) {
  mspi_lsqr_state* st = d.st;
  if (st->stop) return;
  const int s = st->s, nb = st->nblk;
  for (int j = 0; j < s; ++j) d.V[j] = block_sum(d.g, nb, s, j);
  const double alpha = snorm(d.V, s);
  vscale(d.V, s, 1.0 / alpha);
  for (int j = 0; j < s; ++j) d.W[j] = d.V[j];
  if (st->exact_norm && gfrob) {  // MatNorm(FROBENIUS): per block, columns in order, then blocks in order
    double t = 0.0;
    for (int b = 0; b < nb; ++b) {
      double tb = 0.0;
      for (int j = 0; j < s; ++j) tb += gfrob[b * s + j];
      t += tb;
    }
    st->anorm = sqrt(t);
  } else {
    st->anorm = 0.0;
  }
  st->arnorm = alpha * st->beta;
  st->phibar = st->beta;
  st->rhobar = alpha;
  st->alpha = alpha;
  st->nalpha = -alpha;
  st->i = 0;
}

// beta = ||R V - alpha U||; U1 scale; anorm estimate
__global__ void k_ls_beta(mspi_lsqr_dev d) {
  mspi_lsqr_state* st = d.st;
  if (st->stop) return;
  const double beta = sqrt(block_sum(d.g, st->nblk, 1, 0));
  if (bad(beta)) {
    st->reason = MSP_DIVERGED_NANORINF;
    st->stop = 1;
    return;
  }
  st->beta = beta;
  if (beta > 0.0) {
    st->uscale = 1.0 / beta;
    if (!st->exact_norm)
      st->anorm = sqrt(st->anorm * st->anorm + st->alpha * st->alpha + beta * beta);
  } else {
    st->uscale = 1.0;
  }
}

// V1 = R^T U1 - beta V, alpha, the plane rotation, x and w updates, the test
__global__ void k_ls_step(mspi_lsqr_dev d) {
  mspi_lsqr_state* st = d.st;
  if (st->stop) return;
  const int s = st->s, nb = st->nblk;
  const double beta = st->beta;
  for (int j = 0; j < s; ++j) d.V1[j] = block_sum(d.g, nb, s, j);
  vaxpy(d.V1, s, -beta, d.V);
  const double alpha = snorm(d.V1, s);
  if (bad(alpha)) {
    st->reason = MSP_DIVERGED_NANORINF;
    st->stop = 1;
    return;
  }
  vscale(d.V1, s, 1.0 / alpha);
  const double rhobar0 = st->rhobar;
  const double rho = sqrt(rhobar0 * rhobar0 + beta * beta);
  const double c = rhobar0 / rho;
  const double sn = beta / rho;
  const double theta = sn * alpha;
  st->rhobar = -c * alpha;
  const double phi = c * st->phibar;
  st->phibar = sn * st->phibar;
  const double tau = sn * phi;
  vaxpy(d.X, s, phi / rho, d.W);
  vaypx(d.W, s, -theta / rho, d.V1);
  st->arnorm = alpha * fabs(tau);
  const double rnorm = st->phibar;
  st->rnorm = rnorm;
  st->its++;
  ls_log(d, rnorm);
  ls_converged(st, st->i + 1, rnorm);
  st->alpha = alpha;
  if (st->reason) {
    st->stop = 1;
    return;
  }
  for (int j = 0; j < s; ++j) d.V[j] = d.V1[j];  // SWAP(V1, V)
  st->i++;
  st->nalpha = -alpha;
  if (st->i >= st->max_it) {
    st->reason = MSP_DIVERGED_ITS;
    st->stop = 1;
  }
}

// The one-pass DBR step (ksp_lsqr.c): the gathered block partials are [||U1||^2 | R^T U1] per block (stride
// s + 1); beta as k_ls_beta, then V1 = (R^T U1) * (1/beta) (unscaled U1's products, scaled after the block sum;
// beta = 0 leaves them, as VecScale was skipped) and k_ls_step's recurrence.
__global__ void k_ls_onepass_step(mspi_lsqr_dev d) {
  mspi_lsqr_state* st = d.st;
  if (st->stop) return;
  const int s = st->s, nb = st->nblk;
  const double beta = sqrt(block_sum(d.g, nb, s + 1, 0));
  if (bad(beta)) {
    st->reason = MSP_DIVERGED_NANORINF;
    st->stop = 1;
    return;
  }
  st->beta = beta;
  if (beta > 0.0) {
    st->uscale = 1.0 / beta;
    if (!st->exact_norm) st->anorm = sqrt(st->anorm * st->anorm + st->alpha * st->alpha + beta * beta);
  } else {
    st->uscale = 1.0;
  }
  for (int j = 0; j < s; ++j) d.V1[j] = block_sum(d.g, nb, s + 1, 1 + j);
  if (beta > 0.0) vscale(d.V1, s, st->uscale);
  vaxpy(d.V1, s, -beta, d.V);
  const double alpha = snorm(d.V1, s);
  if (bad(alpha)) {
    st->reason = MSP_DIVERGED_NANORINF;
    st->stop = 1;
    return;
  }
  vscale(d.V1, s, 1.0 / alpha);
  const double rhobar0 = st->rhobar;
  const double rho = sqrt(rhobar0 * rhobar0 + beta * beta);
  const double c = rhobar0 / rho;
  const double sn = beta / rho;
  const double theta = sn * alpha;
  st->rhobar = -c * alpha;
  const double phi = c * st->phibar;
  st->phibar = sn * st->phibar;
  const double tau = sn * phi;
  vaxpy(d.X, s, phi / rho, d.W);
  vaypx(d.W, s, -theta / rho, d.V1);
  st->arnorm = alpha * fabs(tau);
  const double rnorm = st->phibar;
  st->rnorm = rnorm;
  st->its++;
  ls_log(d, rnorm);
  ls_converged(st, st->i + 1, rnorm);
  st->alpha = alpha;
  if (st->reason) {
    st->stop = 1;
    return;
  }
  for (int j = 0; j < s; ++j) d.V[j] = d.V1[j];  // SWAP(V1, V)
  st->i++;
  st->nalpha = -alpha;
  if (st->i >= st->max_it) {
    st->reason = MSP_DIVERGED_ITS;
    st->stop = 1;
  }
}

}  // namespace

extern "C" int mspi_ls_onepass_step(msp_ctx* c, mspi_lsqr_dev d) {
  k_ls_onepass_step<<<1, 1, 0, c->stream>>>(d);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}

extern "C" int mspi_ls_start(msp_ctx* c, mspi_lsqr_dev d) {
  k_ls_start<<<1, 1, 0, c->stream>>>(d);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}
extern "C" int mspi_ls_first(msp_ctx* c, mspi_lsqr_dev d, const double* gfrob) {
  k_ls_first<<<1, 1, 0, c->stream>>>(d, gfrob);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}
extern "C" int mspi_ls_beta(msp_ctx* c, mspi_lsqr_dev d) {
  k_ls_beta<<<1, 1, 0, c->stream>>>(d);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}
extern "C" int mspi_ls_step(msp_ctx* c, mspi_lsqr_dev d) {
  k_ls_step<<<1, 1, 0, c->stream>>>(d);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}
