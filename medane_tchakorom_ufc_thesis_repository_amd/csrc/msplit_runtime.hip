// msplit_runtime.hip -- context, Mat and Vec objects of the C ABI (include/msplit.h).
//
// One context per GPU owns one HIP stream; every Mat/Vec op is enqueued on it.
// Host scalars (norms, dots) come back through a pinned staging buffer.
// The KSP (GMRES) host logic lives in ksp_gmres.c and calls the mspi_* entry
// points defined here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "msplit.h"
#include "msplit_internal.h"
#include "msplit_kernels.h"
#include "msplit_ctx.hpp"

// ----------------------------------------------------------------- errors
static thread_local char g_err[512] = "no error";

extern "C" void mspi_set_error(int code, const char* fmt, ...) {
  char buf[448];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  snprintf(g_err, sizeof(g_err), "[msplit error %d] %s", code, buf);
}

extern "C" const char* msp_get_last_error(void) { return g_err; }

extern "C" int msp_get_device_count(int* count) {
  ARGCHK(count, MSP_ERR_ARG_NULL, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_create(int device, void* stream, msp_ctx** out) {
  ARGCHK(out, MSP_ERR_ARG_NULL, "ctx out-pointer is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    mspi_set_error(MSP_ERR_LIB, "no HIP device visible (the MI355X path needs a GPU; there is no CPU fallback)");
    return MSP_ERR_LIB;
  }
  ARGCHK(device >= 0 && device < ndev, MSP_ERR_ARG_OUTOFRANGE, "device %d out of range [0,%d)", device, ndev);
  HIPCHK(hipSetDevice(device));
  if (const char* e = getenv("MSPLIT_TUNING")) msk_set_tuning(atoi(e));
  if (const char* e = getenv("MSPLIT_MARCH_LINES")) msk_set_march_lines(atoi(e));  // A/B: 1 or 4 (0: auto)
  msp_ctx* c = new msp_ctx();
  c->device = device;
  if (const char* e = getenv("MSPLIT_REDUCTION")) c->reduce = (e[0] == 's' || e[0] == 'S') ? MSP_REDUCE_SEQ : MSP_REDUCE_DBR;
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      mspi_set_error(MSP_ERR_LIB, "hipStreamCreate failed");
      return MSP_ERR_LIB;
    }
    c->own_stream = true;
  }
  if (hipMalloc((void**)&c->dscratch, kScratch * sizeof(double)) != hipSuccess ||
      hipHostMalloc((void**)&c->hscratch, kScratch * sizeof(double), hipHostMallocDefault) != hipSuccess) {
    mspi_set_error(MSP_ERR_MEM, "scratch allocation failed");
    msp_ctx_destroy(&c);
    return MSP_ERR_MEM;
  }
  *out = c;
  return MSP_SUCCESS;
}

static void ctx_free(msp_ctx* c) {
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto e : c->pool) (void)hipEventDestroy(e);
  if (c->partial) (void)hipFree(c->partial);
  if (c->seqbuf) (void)hipFree(c->seqbuf);
  if (c->seqready) (void)hipFree(c->seqready);
  if (c->seq_aux) (void)hipStreamSynchronize(c->seq_aux), (void)hipStreamDestroy(c->seq_aux);
  if (c->seq_walk) (void)hipStreamSynchronize(c->seq_walk), (void)hipStreamDestroy(c->seq_walk);
  for (auto e : c->seq_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->seqacc) (void)hipFree(c->seqacc);
  if (c->dscratch) (void)hipFree(c->dscratch);
  if (c->hscratch) (void)hipHostFree(c->hscratch);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" void mspi_ctx_retain(msp_ctx* c) {
  if (c) c->refs.fetch_add(1);
}
extern "C" void mspi_ctx_release(msp_ctx* c) {
  if (c && c->refs.fetch_sub(1) == 1) ctx_free(c);
}

// The context is freed when the caller's reference and those of every object made on it are gone.
extern "C" int msp_ctx_destroy(msp_ctx** pc) {
  if (!pc || !*pc) return MSP_SUCCESS;
  msp_ctx* c = *pc;
  *pc = nullptr;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_synchronize(msp_ctx* c) {
  ARGCHK(c, MSP_ERR_ARG_NULL, "ctx is NULL");
  HIPCHK(hipStreamSynchronize(c->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_set_timing(msp_ctx* c, int enable) {
  ARGCHK(c, MSP_ERR_ARG_NULL, "ctx is NULL");
  ARGCHK(enable >= 0, MSP_ERR_ARG_OUTOFRANGE, "timing %d", enable);
  static_assert(MSP_KERNEL_NCLASSES <= 16, "per-class counters");
  c->timing = enable != 0;
  c->timing_every = enable > 1 ? enable : 1;
  for (auto& v : c->timing_seen) v = 0;
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_set_reduction(msp_ctx* c, int mode) {
  ARGCHK(c, MSP_ERR_ARG_NULL, "ctx is NULL");
  ARGCHK(mode == MSP_REDUCE_DBR || mode == MSP_REDUCE_SEQ, MSP_ERR_ARG_OUTOFRANGE, "reduction mode %d", mode);
  c->reduce = mode;
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_get_reduction(const msp_ctx* c, int* mode) {
  ARGCHK(c && mode, MSP_ERR_ARG_NULL, "NULL argument");
  *mode = c->reduce;
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_reset_kernel_stats(msp_ctx* c) {
  ARGCHK(c, MSP_ERR_ARG_NULL, "ctx is NULL");
  HIPCHK(hipStreamSynchronize(c->stream));
  c->recs.clear();
  c->pool_used = 0;
  return MSP_SUCCESS;
}

extern "C" int msp_ctx_get_kernel_stats(msp_ctx* c, int cls, int64_t* launches, double* total_ms, double* total_bytes) {
  ARGCHK(c, MSP_ERR_ARG_NULL, "ctx is NULL");
  ARGCHK(cls >= 0 && cls < MSP_KERNEL_NCLASSES, MSP_ERR_ARG_OUTOFRANGE, "kernel class %d", cls);
  HIPCHK(hipStreamSynchronize(c->stream));
  int64_t n = 0;
  double ms = 0.0, by = 0.0;
  for (const auto& r : c->recs) {
    if (r.cls != cls) continue;
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, c->pool[r.ev], c->pool[r.ev + 1]));
    ++n;
    ms += t;
    by += r.bytes;
  }
  if (launches) *launches = n;
  if (total_ms) *total_ms = ms;
  if (total_bytes) *total_bytes = by;
  return MSP_SUCCESS;
}

extern "C" double* mspi_dev_scratch(msp_ctx* c) { return c->dscratch; }
extern "C" double* mspi_host_scratch(msp_ctx* c) { return c->hscratch; }

// Device allocation of the large buffers (vectors, the Krylov basis, dense blocks): from 64 MiB up they are
// requested physically contiguous (hipDeviceMallocContiguous), falling back to hipMalloc when the driver cannot.
// Same box, three interleaved pairs (profiles/r03/contig/): MAXPY at the SMSM block 0.915 -> 0.895 ms, the 256^3
// GMRES step +0.6 %, the SMSM block +0.2 %: fewer address-translation misses for streams of 134-537 MB vectors.
// MSPLIT_ALLOC_CONTIGUOUS=0 keeps plain hipMalloc.
extern "C" int mspi_big_alloc(void** p, size_t bytes) {
  static const int contig = [] {
    const char* e = getenv("MSPLIT_ALLOC_CONTIGUOUS");
    return e ? atoi(e) : 1;
  }();
  if (contig && bytes >= ((size_t)64 << 20)) {
    if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) return (int)hipSuccess;
    (void)hipGetLastError();
  }
  return (int)hipMalloc(p, bytes);
}

extern "C" int mspi_malloc(msp_ctx* c, void** p, size_t bytes) {
  (void)c;
  if (mspi_big_alloc(p, bytes ? bytes : 16) != (int)hipSuccess) {
    *p = nullptr;
    mspi_set_error(MSP_ERR_MEM, "hipMalloc(%zu bytes) failed", bytes);
    return MSP_ERR_MEM;
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_free(msp_ctx* c, void* p) {
  (void)c;
  if (p) HIPCHK(hipFree(p));
  return MSP_SUCCESS;
}

extern "C" int mspi_host_malloc(void** p, size_t bytes) {
  if (hipHostMalloc(p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) {
    *p = nullptr;
    mspi_set_error(MSP_ERR_MEM, "hipHostMalloc(%zu bytes) failed", bytes);
    return MSP_ERR_MEM;
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_host_free(void* p) {
  if (p) HIPCHK(hipHostFree(p));
  return MSP_SUCCESS;
}

extern "C" int mspi_set_device(msp_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return MSP_SUCCESS;
}

extern "C" int mspi_d2h_sync(msp_ctx* c, void* host, const void* dev, size_t bytes) {
  HIPCHK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MSP_SUCCESS;
}

// --------------------------------------------------------------- internal ops
// Stage 1 of a reduction in the context's order (DBR, or MSP_REDUCE_SEQ's sequential sums
// written in the DBR partial layout).
static int stage1(msp_ctx* c, const double* w, const Vecs* V, int nv, int64_t n, int self, int64_t nch,
                  const int* stop) {
  if (c->reduce == MSP_REDUCE_SEQ) return mspi_seq_stage1(c, w, V, nv, n, self, c->partial, nch, stop);
  return msk_dot_stage1(w, V, nv, n, c->partial, nch, self, stop, c->stream);
}

extern "C" int mspi_mdot(msp_ctx* c, const double* w, int nv, const double* const* V, int64_t n, double* out_dev) {
  if (nv <= 0) return MSP_SUCCESS;
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {  // empty vectors: every dot is +0
    HIPCHK(hipMemsetAsync(out_dev, 0, (size_t)nv * sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  int rc = ensure_partial(c, nch * MSPI_MAX_GROUP);
  if (rc) return rc;
  KTimer kt(c, MSP_KERNEL_MDOT, 8.0 * (double)n * (nv + 1));
  for (int g0 = 0; g0 < nv; g0 += MSPI_MAX_GROUP) {
    const int g = std::min(MSPI_MAX_GROUP, nv - g0);
    Vecs vg = {};
    for (int j = 0; j < g; ++j) vg.p[j] = V[g0 + j];
    KCHK(stage1(c, w, &vg, g, n, 0, nch, nullptr));
    KCHK(msk_dot_stage2(c->partial, nch, g, out_dev + g0, nullptr, c->stream));
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_norm2sq(msp_ctx* c, const double* x, int64_t n, double* out_dev) {
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {
    HIPCHK(hipMemsetAsync(out_dev, 0, sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  int rc = ensure_partial(c, nch * MSPI_MAX_GROUP);
  if (rc) return rc;
  KTimer kt(c, MSP_KERNEL_NORM, 8.0 * (double)n);
  Vecs vg = {};
  vg.p[0] = x;
  KCHK(stage1(c, x, &vg, 1, n, 1, nch, nullptr));
  KCHK(msk_dot_stage2(c->partial, nch, 1, out_dev, nullptr, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_maxpy(msp_ctx* c, double* w, int nv, const double* const* V, int64_t n, const double* alpha_host,
                          const double* alpha_dev, int negate, int accumulate) {
  if (nv <= 0 || n <= 0) return MSP_SUCCESS;
  if (accumulate && nv > MSPI_MAX_GROUP) {
    mspi_set_error(MSP_ERR_SUP, "accumulating MAXPY over more than %d vectors", MSPI_MAX_GROUP);
    return MSP_ERR_SUP;
  }
  KTimer kt(c, MSP_KERNEL_MAXPY, 8.0 * (double)n * (nv + 2));
  // Launches of up to 32 vectors compose exactly into PETSc's order (the
  // nv & 3 leading vectors, then groups of four) when the FIRST launch takes
  // nv mod 32 vectors: its own leading group is then nv & 3 and every later
  // launch is a whole number of 4-groups.
  int g = nv % MSPI_MAX_GROUP ? nv % MSPI_MAX_GROUP : MSPI_MAX_GROUP;
  for (int g0 = 0; g0 < nv; g0 += g, g = MSPI_MAX_GROUP) {
    Vecs vg = {};
    Coefs cf;
    for (int j = 0; j < g; ++j) {
      vg.p[j] = V[g0 + j];
      cf.a[j] = alpha_host ? alpha_host[g0 + j] : 0.0;
    }
    KCHK(msk_maxpy_chunk(w, w, &vg, g, nullptr, &cf, alpha_dev ? alpha_dev + g0 : nullptr, negate, n, accumulate,
                         nullptr, nullptr, c->stream));
  }
  return MSP_SUCCESS;
}

extern "C" hipStream_t mspi_stream(msp_ctx* c) { return c->stream; }

extern "C" int mspi_h2d_async(msp_ctx* c, void* dev, const void* host, size_t bytes) {
  HIPCHK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_h2d_sync(msp_ctx* c, void* dev, const void* host, size_t bytes) {
  HIPCHK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_mem_info(msp_ctx* c, size_t* free_bytes, size_t* total_bytes) {
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemGetInfo(free_bytes, total_bytes));
  return MSP_SUCCESS;
}

extern "C" int mspi_host_register(void* p, size_t bytes) {
  HIPCHK(hipHostRegister(p, bytes, hipHostRegisterMapped));  // mapped: the GPU also stores into it (amsg.c)
  return MSP_SUCCESS;
}

extern "C" int mspi_host_unregister(void* p) {
  HIPCHK(hipHostUnregister(p));
  return MSP_SUCCESS;
}

extern "C" int mspi_mdot_basis(msp_ctx* c, const double* w, int nv, const double* base, int64_t stride,
                               const double* scale, int64_t n, double* out_dev, const int* stop) {
  if (nv <= 0) return MSP_SUCCESS;
  const int64_t nch = nchunks_of(n);
  if (nch == 0) {
    HIPCHK(hipMemsetAsync(out_dev, 0, (size_t)nv * sizeof(double), c->stream));
    return MSP_SUCCESS;
  }
  KTimer kt(c, MSP_KERNEL_MDOT, 8.0 * (double)n * (nv + 1));
  for (int g0 = 0; g0 < nv; g0 += MSPI_MAX_GROUP) {
    const int g = std::min(MSPI_MAX_GROUP, nv - g0);
    Vecs vg = {};
    vg.base = base + (int64_t)g0 * stride;
    vg.stride = stride;
    vg.scale = scale ? scale + g0 : nullptr;
    KCHK(stage1(c, w, &vg, g, n, 0, nch, stop));
    KCHK(msk_dot_stage2(c->partial, nch, g, out_dev + g0, stop, c->stream));
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_maxpy_norm_basis(msp_ctx* c, const double* win, double* wout, int nv, const double* base,
                                     int64_t stride, const double* scale, int64_t n, const double* alpha_dev,
                                     double* sumsq_dev, const int* stop) {
  const int64_t nch = nchunks_of(n);
  if (nch == 0 || nv <= 0) {
    mspi_set_error(MSP_ERR_ARG_SIZ, "maxpy_norm on an empty basis");
    return MSP_ERR_ARG_SIZ;
  }
  KTimer kt(c, MSP_KERNEL_MAXPY, 8.0 * (double)n * (nv + 2));
  Vecs vg = {};
  vg.base = base;
  vg.stride = stride;
  vg.scale = scale;
  Coefs cf = {};
  KCHK(msk_maxpy_chunk(win, wout, &vg, nv, nullptr, &cf, alpha_dev, 1, n, 0, c->partial, stop, c->stream));
  if (c->reduce == MSP_REDUCE_SEQ) KCHK(stage1(c, wout, &vg, 1, n, 1, nch, stop));  // ||wout||^2 in order
  KCHK(msk_dot_stage2(c->partial, nch, 1, sumsq_dev, stop, c->stream));
  return MSP_SUCCESS;
}

// CGS VecMAXPY with the fused ||w||^2 partials, then one launch that folds them and
// runs the Hessenberg update (k_norm_update).  MSK_TUNE_GM_UNFUSED: the separate
// stage-2 and one-lane update launches (A/B).
extern "C" int mspi_maxpy_norm_update(msp_ctx* c, const double* win, double* wout, int nv, const double* base,
                                      int64_t stride, const double* scale, int64_t n, mspi_gmres_dev g, int it, int m,
                                      const int* stop) {
  if (msk_get_tuning() & MSK_TUNE_GM_UNFUSED) {
    int rc = mspi_maxpy_norm_basis(c, win, wout, nv, base, stride, scale, n, g.h, g.h + it + 1, stop);
    return rc ? rc : mspi_gm_iter_update(c, g);
  }
  const int64_t nch = nchunks_of(n);
  if (nch == 0 || nv <= 0) {
    mspi_set_error(MSP_ERR_ARG_SIZ, "maxpy_norm on an empty basis");
    return MSP_ERR_ARG_SIZ;
  }
  {
    KTimer kt(c, MSP_KERNEL_MAXPY, 8.0 * (double)n * (nv + 2));
    Vecs vg = {};
    vg.base = base;
    vg.stride = stride;
    vg.scale = scale;
    Coefs cf = {};
    KCHK(msk_maxpy_chunk(win, wout, &vg, nv, nullptr, &cf, g.h, 1, n, 0, c->partial, stop, c->stream));
    if (c->reduce == MSP_REDUCE_SEQ) KCHK(stage1(c, wout, &vg, 1, n, 1, nch, stop));  // ||wout||^2 in order
  }
  return mspi_gm_norm_update(c, g, c->partial, nch, m);
}

extern "C" int mspi_maxpy_accum_basis(msp_ctx* c, double* x, const int* nvdev, const double* base, int64_t stride,
                                      const double* scale, int64_t n, const double* coef_dev, int nv_expected) {
  if (n <= 0) return MSP_SUCCESS;
  // BuildSoln: the vector count lives on the device; bytes use the host's expectation
  KTimer kt(c, MSP_KERNEL_MAXPY, 8.0 * (double)n * (nv_expected + 2));
  Vecs vg = {};
  vg.base = base;
  vg.stride = stride;
  vg.scale = scale;
  Coefs cf = {};
  KCHK(msk_maxpy_chunk(x, x, &vg, 0, nvdev, &cf, coef_dev, 0, n, 1, nullptr, nullptr, c->stream));
  return MSP_SUCCESS;
}


extern "C" int mspi_scale(msp_ctx* c, double* x, int64_t n, double alpha) {
  KTimer kt(c, MSP_KERNEL_SCALE, 16.0 * (double)n);
  KCHK(msk_blas1(MSK_SCALE, x, nullptr, nullptr, alpha, n, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_copy(msp_ctx* c, double* dst, const double* src, int64_t n) {
  if (n <= 0 || dst == src) return MSP_SUCCESS;
  KTimer kt(c, MSP_KERNEL_OTHER, 16.0 * (double)n);
  HIPCHK(hipMemcpyAsync(dst, src, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_set(msp_ctx* c, double* x, int64_t n, double alpha) {
  if (n <= 0) return MSP_SUCCESS;
  KTimer kt(c, MSP_KERNEL_OTHER, 8.0 * (double)n);
  KCHK(msk_blas1(MSK_SET, x, nullptr, nullptr, alpha, n, c->stream));
  return MSP_SUCCESS;
}

// -------------------------------------------------------------------- Mat
static uint64_t next_version() {
  static std::atomic<uint64_t> v{1};
  return v.fetch_add(1 << 20);  // objects 2^20 apart: a million storage switches before two could meet
}

struct msp_mat {
  msp_ctx* ctx = nullptr;
  int32_t nrows = 0, ncols = 0;
  int64_t nnz = 0;
  int32_t* rowptr = nullptr;  // nrows+1 (or nlisted+1 when compressed)
  int32_t* col = nullptr;     // nnz (+4 pad)
  double* val = nullptr;      // nnz (+2 pad)
  int32_t lds_cap = 0;        // LDS entries per 256-row block (0: direct kernel)
  int32_t lds_cap512 = 0;     // LDS entries per 512-row block (0: no fused SpMV + MDot)
  bool compressed = false;
  int64_t plane = 0;          // rows per stencil plane (box-stencil operators), 0 otherwise
  int32_t nlisted = 0;
  int32_t* row_ids = nullptr;
  bool matfree = false;       // box stencil applied without storage (msp_mat_create_box_matfree)
  int dim = 0, lo = 0, hi = 0;
  int32_t bx = 0, by = 0, bz = 0;
  BoxCoef cf = {};
  // DV storage (k_spmv_dv): one byte per entry naming a (col - row, value) pair
  uint8_t* dv_len = nullptr;   // nrows (+16 pad)
  uint8_t* dv_code = nullptr;  // nnz (+16 pad)
  int32_t* dv_delta = nullptr; // ndict
  double* dv_val = nullptr;    // ndict
  int32_t ndict = 0;
  int32_t dv_mb = 0;           // most entries in one 256-row block (sizes the LDS stage)
  int32_t dv_w = 0;            // ELL layout: codes per row (4, 8, 16); 0: CSR-order codes + row lengths
  bool dv_on = false;          // products read the DV storage
  // box stencil (lo = hi = 0) whose ELL dictionary is the seven (3D) or five (2D) stencil pairs in column order:
  // its extents, for the z-march SpMV (msk_spmv_box_march); 0 otherwise
  int32_t march_nx = 0, march_ny = 0, march_nz = 0;
  int32_t march_d2 = 0;        // 2D box stencil (five pairs), marched as nx x 1 x ny
  int32_t march_halo = 0;      // bit 0 / 1: the column space adds the plane below / above the box (chunk march only)
  uint8_t* march_mask = nullptr;  // nrows (+16 pad): the rows' presence bytes (msk_march_mask)
  // STENCIL storage (rv_attach): a 3D box stencil whose rows carry their own values; rv_stride == -1: symmetric,
  // the diagonal and upper legs only (rvs_pair), 0: chunk-blocked seven legs (rv_pair), else rv_val[e * rv_stride + r] is
  // row r's entry at neighbour e (column order; 0.0 where the row has none), march_* and march_mask as above
  double* rv_val = nullptr;
  int64_t rv_stride = 0;
  bool rv_on = false;
  bool csr_released = false;   // msp_mat_release_csr: col/val freed (and rowptr in the ELL layout)
  uint64_t version = next_version();  // unique per object and bumped when its products' kernels change
};

extern "C" int mspi_mat_dims(const msp_mat* A, int32_t* nr, int32_t* nc) {
  *nr = A->nrows;
  *nc = A->ncols;
  return MSP_SUCCESS;
}
extern "C" msp_ctx* mspi_mat_ctx(const msp_mat* A) { return A->ctx; }
extern "C" mspi_csr_view mspi_mat_csr(const msp_mat* A) {
  mspi_csr_view v = {A->rowptr, A->col, A->val, A->nnz, A->compressed ? 1 : 0, A->lds_cap};
  return v;
}

static const int32_t kMaxLdsCap = 4096;  // 48 KiB of col+val per 256-row block
static const int64_t kMaxDvBlock = 12288;  // DV codes per 256-row block (CSR-order layout)

static int32_t lds_cap_for(int64_t max_block_nnz) {
  if (max_block_nnz + 8 > kMaxLdsCap) return 0;
  return (int32_t)((max_block_nnz + 8 + 3) & ~(int64_t)3);
}

// Storage chosen at assembly: DV whenever the matrix fits it, unless
// MSPLIT_MAT_STORAGE=csr (then msp_mat_set_storage can still switch).
static bool dv_default() {
  const char* e = getenv("MSPLIT_MAT_STORAGE");
  return !(e && strcmp(e, "csr") == 0);
}

static void rv_free(msp_mat* A) {
  if (A->rv_val) (void)hipFree(A->rv_val);
  A->rv_val = nullptr;
  A->rv_stride = 0;
  A->rv_on = false;
}

static void dv_free(msp_mat* A) {
  if (A->dv_len) (void)hipFree(A->dv_len);
  if (A->dv_code) (void)hipFree(A->dv_code);
  if (A->dv_delta) (void)hipFree(A->dv_delta);
  if (A->dv_val) (void)hipFree(A->dv_val);
  A->dv_len = A->dv_code = nullptr;
  A->dv_delta = nullptr;
  A->dv_val = nullptr;
  A->ndict = 0;
  A->dv_mb = 0;
  A->dv_w = 0;
  A->dv_on = false;
  if (A->march_mask) (void)hipFree(A->march_mask);
  A->march_mask = nullptr;
  A->march_nx = A->march_ny = A->march_nz = 0;
  A->march_d2 = 0;
  A->march_halo = 0;
}

// Encode the device CSR of A against the dictionary (host arrays, nd <= 256).
// Rows of at most 16 entries take the ELL layout (W codes per row, padded)
// unless padding would add more than half the entries; other matrices take
// CSR-order codes with a length byte per row.  A matrix the dictionary does
// not cover keeps CSR storage only (returns 0).
static int dv_build(msp_mat* A, int nd, const int32_t* delta, const double* val, int64_t max_block,
                    int32_t max_len) {
  msp_ctx* c = A->ctx;
  if (A->compressed || A->matfree || A->nrows == 0 || nd < 1 || nd > 256) return MSP_SUCCESS;
  const int W = max_len <= 4 ? 4 : max_len <= 8 ? 8 : max_len <= 16 ? 16 : 0;
  const bool ell = W && nd <= 255 && !(msk_get_tuning() & MSK_TUNE_DV_NOELL) &&
                   (double)W * A->nrows <= 1.5 * (double)A->nnz + 2.0 * A->nrows;
  // CSR-order codes: one block's codes (up to 4 x 256 rows) are staged in LDS, at most 48 KiB
  if (!ell && max_block > kMaxDvBlock) return MSP_SUCCESS;
  A->dv_mb = (int32_t)max_block;
  A->dv_w = ell ? W : 0;
  if (!ell) HIPCHK((hipError_t)mspi_big_alloc((void**)&A->dv_len, (size_t)A->nrows + 16));
  const size_t ncode = ell ? (size_t)W * A->nrows : (size_t)A->nnz;
  HIPCHK((hipError_t)mspi_big_alloc((void**)&A->dv_code, ncode + 16));
  HIPCHK(hipMalloc((void**)&A->dv_delta, 256 * sizeof(int32_t)));
  HIPCHK(hipMalloc((void**)&A->dv_val, 256 * sizeof(double)));
  HIPCHK(hipMemsetAsync(A->dv_code + ncode, 0, 16, c->stream));
  HIPCHK(hipMemcpyAsync(A->dv_delta, delta, (size_t)nd * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(A->dv_val, val, (size_t)nd * sizeof(double), hipMemcpyHostToDevice, c->stream));
  int* fail = reinterpret_cast<int*>(mspi_dev_scratch(c));
  HIPCHK(hipMemsetAsync(fail, 0, sizeof(int), c->stream));
  if (ell)
    KCHK(msk_ell_encode(A->nrows, W, A->rowptr, A->col, A->val, nd, A->dv_delta, A->dv_val, A->dv_code, fail,
                        c->stream));
  else
    KCHK(msk_dv_encode(A->nrows, A->rowptr, A->col, A->val, nd, A->dv_delta, A->dv_val, A->dv_len, A->dv_code, fail,
                       c->stream));
  int hfail = 0;
  HIPCHK(hipMemcpyAsync(&hfail, fail, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (hfail) {
    dv_free(A);
    return MSP_SUCCESS;
  }
  A->ndict = nd;
  A->dv_on = dv_default();
  return MSP_SUCCESS;
}

struct DvKey {
  int32_t d;
  uint64_t bits;
  bool operator==(const DvKey& o) const { return d == o.d && bits == o.bits; }
};
struct DvKeyHash {
  size_t operator()(const DvKey& k) const { return (size_t)(k.bits * 0x9E3779B97F4A7C15ull ^ (uint32_t)k.d); }
};

// The dictionary of a host CSR: its distinct (col - row, value bits) pairs in
// order of first appearance; none (0) when there are more than 256 or a row
// holds more than 255 entries.
static int dv_dictionary(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val,
                         std::vector<int32_t>& delta, std::vector<double>& dval) {
  // a stencil has a handful of pairs: a linear scan of the dictionary beats hashing until it grows
  std::vector<DvKey> keys;
  std::unordered_map<DvKey, int, DvKeyHash> seen;
  for (int32_t r = 0; r < nrows; ++r) {
    if (rowptr[r + 1] - rowptr[r] > 255) return 0;
    for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      DvKey key;
      key.d = col[k] - r;
      memcpy(&key.bits, &val[k], 8);
      bool found = false;
      if (keys.size() <= 16) {
        for (const DvKey& e : keys)
          if (e == key) {
            found = true;
            break;
          }
      } else {
        found = seen.count(key) != 0;
      }
      if (found) continue;
      if (keys.size() == 256) return 0;
      keys.push_back(key);
      seen.emplace(key, (int)delta.size());
      delta.push_back(key.d);
      dval.push_back(val[k]);
    }
  }
  return (int)delta.size();
}

// Attach the z-march SpMV (msk_spmv_box_march) to a matrix in DV storage whose ELL dictionary
// (8 codes per row) is the box stencil's pairs in column order: (-P, -nx, -1, 0, +1, +nx, +P) in 3D
// (nx x ny x nz, P = nx ny), or (-nx, -1, 0, +1, +nx) for a 2D box marched as nx x 1 x nz.  The
// deltas must be distinct (nx > 1, and ny > 1 in 3D): with ny == 1, +nx and +P are one column
// offset, the encoder names the +P coupling +nx and the march would drop it.  check: verify on the
// device that no row holds a neighbour across a line or plane edge (k_march_check), for matrices
// the caller assembled; a failed check leaves the matrix on the row-parallel ELL kernel.
static int march_attach(msp_mat* A, int32_t nx, int32_t ny, int32_t nz, int d2, bool check, int halo = 0) {
  msp_ctx* c = A->ctx;
  const int nd = d2 ? 5 : 7;
  const int64_t P = (int64_t)nx * ny;
  const int64_t ext = P * (((halo & 1) ? 1 : 0) + ((halo & 2) ? 1 : 0));
  if (A->ndict != nd || A->dv_w != 8 || nx <= 1 || (!d2 && ny <= 1) || nz < 1 ||
      (int64_t)nx * ny * nz != (int64_t)A->nrows || (int64_t)A->ncols != (int64_t)A->nrows + ext)
    return MSP_SUCCESS;
  // with coupling planes in the column space only the chunk-tile march reads them (3D, whole-chunk planes)
  if (halo && (d2 || !msk_march_chunk_fits(nx, ny, d2))) return MSP_SUCCESS;
  if (mspi_big_alloc((void**)&A->march_mask, (size_t)A->nrows + 16) != (int)hipSuccess) {
    A->march_mask = nullptr;
    mspi_set_error(MSP_ERR_MEM, "hipMalloc of the march presence bytes failed");
    return MSP_ERR_MEM;
  }
  HIPCHK(hipMemsetAsync(A->march_mask + A->nrows, 0, 16, c->stream));
  KCHK(msk_march_mask(A->nrows, d2, A->dv_code, A->march_mask, c->stream));
  if (check) {
    int* fail = reinterpret_cast<int*>(mspi_dev_scratch(c));
    HIPCHK(hipMemsetAsync(fail, 0, sizeof(int), c->stream));
    KCHK(msk_march_check(A->nrows, nx, d2 ? 1 : ny, d2, A->march_mask, fail, c->stream));
    int hfail = 0;
    HIPCHK(hipMemcpyAsync(&hfail, fail, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (hfail) {
      (void)hipFree(A->march_mask);
      A->march_mask = nullptr;
      return MSP_SUCCESS;
    }
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  A->march_nx = nx;
  A->march_ny = d2 ? 1 : ny;
  A->march_nz = nz;
  A->march_d2 = d2;
  A->march_halo = halo;
  return MSP_SUCCESS;
}

// A host dictionary that is a box stencil's, up to order: 7 pairs with distinct deltas
// {-a b, -a, -1, 0, 1, a, a b} (a > 1, b > 1, nrows % (a b) == 0) or 5 with {-a, -1, 0, 1, a}
// (a > 1, nrows % a == 0).  On success the pairs are sorted into column order and the box
// extents returned (2D: nx = a, nz = nrows / a, d2 = 1).
static bool box_dictionary(int32_t nrows, std::vector<int32_t>& dd, std::vector<double>& dv, int32_t* nx,
                           int32_t* ny, int32_t* nz, int* d2) {
  const size_t nd = dd.size();
  if (nd != 5 && nd != 7) return false;
  std::vector<size_t> ord(nd);
  for (size_t q = 0; q < nd; ++q) ord[q] = q;
  std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return dd[a] < dd[b]; });
  std::vector<int32_t> sd(nd);
  std::vector<double> sv(nd);
  for (size_t q = 0; q < nd; ++q) {
    sd[q] = dd[ord[q]];
    sv[q] = dv[ord[q]];
    if (q && sd[q] == sd[q - 1]) return false;  // two values on one diagonal: not a constant stencil
  }
  const size_t m = nd / 2;  // the diagonal
  if (sd[m] != 0 || sd[m - 1] != -1 || sd[m + 1] != 1 || sd[m - 2] != -sd[m + 2]) return false;
  const int32_t a = sd[m + 2];
  if (a <= 1 || nrows % a) return false;
  if (nd == 7) {
    const int32_t P = sd[6];
    if (sd[0] != -P || P <= a || P % a || nrows % P) return false;
    *nx = a;
    *ny = P / a;
    *nz = nrows / P;
    *d2 = 0;
  } else {
    *nx = a;
    *ny = 1;
    *nz = nrows / a;
    *d2 = 1;
  }
  dd = sd;
  dv = sv;
  return true;
}

// The STENCIL storage of an assembled square CSR that no dictionary covers (variable coefficients): when the
// distinct column offsets of its rows are a 3D box stencil's seven {-P, -nx, -1, 0, 1, nx, P} (box_dictionary on
// the offsets) and the chunk-tile march takes the box, every row's entries go to per-neighbour value arrays
// (rv_val[e * stride + r], 0.0 where absent) with one presence byte per row, and the device checks that no row
// holds a neighbour across a line or plane edge (k_march_check); a failed check keeps CSR.  The products add
// the present entries in column order from 0.0, as the CSR kernels: bitwise the same.
// The storage is optional: under MSPLIT_MAT_STORAGE=csr it is not built, and when HBM cannot hold its 57 B/row
// next to the resident CSR (which stays: release_csr needs DV storage) the matrix simply stays in CSR.
static int rv_attach(msp_mat* A, const int32_t* rowptr, const int32_t* col, const double* val) {
  msp_ctx* c = A->ctx;
  const int32_t n = A->nrows;
  // built whatever MSPLIT_MAT_STORAGE says (as the DV storage is): under "csr" the products stay in CSR until
  // msp_mat_set_storage(MSP_STORAGE_STENCIL) switches
  if (A->compressed || A->matfree || n == 0 || A->ncols != n || A->dv_on) return MSP_SUCCESS;
  std::vector<int32_t> dd;
  for (int32_t r = 0; r < n; ++r)
    for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      const int32_t d = col[k] - r;
      if (std::find(dd.begin(), dd.end(), d) == dd.end()) {
        if (dd.size() == 7) return MSP_SUCCESS;  // more than a 7-point stencil's offsets
        dd.push_back(d);
      }
    }
  std::vector<double> dummy(dd.size(), 0.0);
  int32_t nx = 0, ny = 0, nz = 0;
  int d2 = 0;
  if (!box_dictionary(n, dd, dummy, &nx, &ny, &nz, &d2) || d2 || !msk_march_chunk_fits(nx, ny, 0)) return MSP_SUCCESS;
  const int64_t stride = ((int64_t)n + 511) / 512 * 512;
  // the value layout: chunk-blocked (every plane is whole DBR chunks here, so n % 4096 == 0) unless
  // MSPLIT_RV_LAYOUT=soa (per-leg arrays; the A/B)
  const char* lay = getenv("MSPLIT_RV_LAYOUT");
  const bool blocked = !(lay && strcmp(lay, "soa") == 0) && n % MSK_DBR_CHUNK == 0;
  std::vector<uint8_t> mask((size_t)n + 16, 0);
  std::vector<double> rv((size_t)7 * stride, 0.0);  // per-leg arrays first
  for (int32_t r = 0; r < n; ++r)
    for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      const int e = (int)(std::find(dd.begin(), dd.end(), col[k] - r) - dd.begin());  // dd is in column order now
      mask[r] |= (uint8_t)(1u << e);
      rv[(size_t)e * stride + r] = val[k];
    }
  // The symmetric storage (like PETSc's SBAIJ, which keeps one triangle): when every upper entry A[r, r + d] has
  // its mirror A[r + d, r] with the same bits (and every lower entry its upper one), only the diagonal and the
  // three upper legs are kept (32 B/row instead of 56) and a row's lower values are read at its lower neighbours.
  // Chunk-blocked only, planes up to 1024 wide (the kernels' LDS windows); MSPLIT_RV_SYM=0 keeps the seven legs.
  const char* syme = getenv("MSPLIT_RV_SYM");
  bool sym = blocked && nx <= 1024 && !(syme && syme[0] == '0');
  {
    const int64_t P = (int64_t)nx * ny;
    const int64_t dlt[3] = {1, nx, P};  // upper leg 4 + i mirrors lower leg 2 - i
    for (int32_t r = 0; r < n && sym; ++r)
      for (int i = 0; i < 3 && sym; ++i) {
        const int up = 4 + i, lo = 2 - i;
        if (mask[r] & (1u << up)) {
          const int64_t c = r + dlt[i];
          uint64_t a, b;
          std::memcpy(&a, &rv[(size_t)up * stride + r], 8);
          if (c >= n || !(mask[c] & (1u << lo))) { sym = false; break; }
          std::memcpy(&b, &rv[(size_t)lo * stride + c], 8);
          sym = a == b;
        }
        if (sym && (mask[r] & (1u << lo)) && (r - dlt[i] < 0 || !(mask[r - dlt[i]] & (1u << up)))) sym = false;
      }
  }
  const int nleg = sym ? 4 : 7;
  // the HBM it takes, sized once the leg count is known (the symmetric storage needs four legs, not seven)
  const size_t need = (size_t)n + 16 + (size_t)nleg * stride * sizeof(double);
  size_t fr = 0, tot = 0;
  if (mspi_mem_info(c, &fr, &tot) || fr < need + (tot >> 5)) {  // keep 1/32 of HBM free after it
    (void)hipGetLastError();
    return MSP_SUCCESS;
  }
  if (blocked) {  // chunk-blocked: the legs of each 512-row slice of a DBR chunk next to each other
    std::vector<double> bl((size_t)nleg * stride, 0.0);
    const int legs[7] = {0, 1, 2, 3, 4, 5, 6}, sym_legs[4] = {3, 4, 5, 6};  // d, x+1, y+1, z+1
    for (int32_t r = 0; r < n; ++r) {
      const int64_t o = r % MSK_DBR_CHUNK;
      for (int k = 0; k < nleg; ++k)
        bl[(size_t)(nleg * (r - o) + (o / 512) * (nleg * 512) + k * 512 + o % 512)] =
            rv[(size_t)(sym ? sym_legs[k] : legs[k]) * stride + r];
    }
    rv.swap(bl);
  }
  if (mspi_big_alloc((void**)&A->march_mask, (size_t)n + 16) != (int)hipSuccess ||
      mspi_big_alloc((void**)&A->rv_val, (size_t)nleg * stride * sizeof(double)) != (int)hipSuccess) {
    (void)hipGetLastError();  // the allocation failure is not the caller's error: the matrix stays in CSR
    rv_free(A);
    if (A->march_mask) (void)hipFree(A->march_mask);
    A->march_mask = nullptr;
    return MSP_SUCCESS;
  }
  HIPCHK(hipMemcpyAsync(A->march_mask, mask.data(), (size_t)n + 16, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(A->rv_val, rv.data(), (size_t)nleg * stride * sizeof(double), hipMemcpyHostToDevice,
                        c->stream));
  int* fail = reinterpret_cast<int*>(mspi_dev_scratch(c));
  HIPCHK(hipMemsetAsync(fail, 0, sizeof(int), c->stream));
  KCHK(msk_march_check(n, nx, ny, 0, A->march_mask, fail, c->stream));
  int hfail = 0;
  HIPCHK(hipMemcpyAsync(&hfail, fail, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));  // also: the host arrays above are read before they go
  if (hfail) {
    rv_free(A);
    (void)hipFree(A->march_mask);
    A->march_mask = nullptr;
    return MSP_SUCCESS;
  }
  A->rv_stride = sym ? -1 : blocked ? 0 : stride;  // -1: the symmetric storage (msplit_kernels.hip rvs_pair)
  A->march_nx = nx;
  A->march_ny = ny;
  A->march_nz = nz;
  A->march_d2 = 0;
  A->march_halo = 0;
  A->rv_on = dv_default();
  return MSP_SUCCESS;
}

static int mat_alloc(msp_ctx* c, msp_mat* A, int64_t nptr, int64_t nnz) {
  HIPCHK((hipError_t)mspi_big_alloc((void**)&A->rowptr, (size_t)nptr * sizeof(int32_t)));
  HIPCHK((hipError_t)mspi_big_alloc((void**)&A->col, (size_t)(nnz + 4) * sizeof(int32_t)));
  HIPCHK((hipError_t)mspi_big_alloc((void**)&A->val, (size_t)(nnz + 2) * sizeof(double)));
  HIPCHK(hipMemsetAsync(A->col + nnz, 0, 4 * sizeof(int32_t), c->stream));
  HIPCHK(hipMemsetAsync(A->val + nnz, 0, 2 * sizeof(double), c->stream));
  return MSP_SUCCESS;
}

static int check_csr(int32_t nrows, int32_t ncols, const int32_t* rowptr, const int32_t* col, int64_t* nnz_out,
                     int64_t* max_block, int64_t* max_block512) {
  ARGCHK(rowptr[0] == 0, MSP_ERR_ARG_WRONG, "rowptr[0] = %d, expected 0", rowptr[0]);
  int64_t mb = 0, mb2 = 0;
  for (int32_t r = 0; r < nrows; ++r) {
    ARGCHK(rowptr[r + 1] >= rowptr[r], MSP_ERR_ARG_WRONG, "rowptr not monotone at row %d", r);
    for (int32_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      ARGCHK(col[k] >= 0 && col[k] < ncols, MSP_ERR_ARG_OUTOFRANGE, "column %d out of range [0,%d) in row %d",
             col[k], ncols, r);
      ARGCHK(k == rowptr[r] || col[k] > col[k - 1], MSP_ERR_ARG_WRONG,
             "columns of row %d not strictly ascending (PETSc AIJ order)", r);
    }
    if ((r & 255) == 0) {
      const int32_t r1 = std::min(r + 256, nrows);
      mb = std::max<int64_t>(mb, (int64_t)rowptr[r1] - rowptr[r]);
    }
    if ((r & 511) == 0) {
      const int32_t r1 = std::min(r + 512, nrows);
      mb2 = std::max<int64_t>(mb2, (int64_t)rowptr[r1] - rowptr[r]);
    }
  }
  *nnz_out = rowptr[nrows];
  *max_block = mb;
  *max_block512 = mb2;
  return MSP_SUCCESS;
}

extern "C" int msp_mat_create_csr(msp_ctx* c, int32_t nrows, int32_t ncols, const int32_t* rowptr, const int32_t* col,
                                  const double* val, msp_mat** out) {
  ARGCHK(c && out && rowptr, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(nrows >= 0 && ncols >= 0, MSP_ERR_ARG_SIZ, "negative size %d x %d", nrows, ncols);
  int64_t nnz = 0, mb = 0, mb2 = 0;
  int rc = check_csr(nrows, ncols, rowptr, col, &nnz, &mb, &mb2);
  if (rc) return rc;
  ARGCHK(nnz == 0 || (col && val), MSP_ERR_ARG_NULL, "col/val NULL with nnz=%lld", (long long)nnz);
  msp_mat* A = new msp_mat();
  A->ctx = c;
  mspi_ctx_retain(c);
  A->nrows = nrows;
  A->ncols = ncols;
  A->nnz = nnz;
  A->lds_cap = lds_cap_for(mb);
  A->lds_cap512 = lds_cap_for(mb2);
  if ((rc = mat_alloc(c, A, (int64_t)nrows + 1, nnz))) {
    msp_mat_destroy(&A);
    return rc;
  }
  HIPCHK(hipMemcpyAsync(A->rowptr, rowptr, ((size_t)nrows + 1) * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  if (nnz) {
    HIPCHK(hipMemcpyAsync(A->col, col, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(A->val, val, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));  // host arrays stay the caller's
  if (nnz) {
    std::vector<int32_t> dd;
    std::vector<double> dvv;
    const int nd = dv_dictionary(nrows, rowptr, col, val, dd, dvv);
    int32_t ml = 0;
    for (int32_t r = 0; r < nrows; ++r) ml = std::max(ml, rowptr[r + 1] - rowptr[r]);
    // an assembled box stencil (the reference's poisson3DMatrix / poisson2DMatrix rows cut to a
    // block, utils.c:30-121, :247-293, :450-478): its dictionary in column order, so the z-march
    // SpMV can take it once the device has checked that no entry wraps across an edge
    int32_t bx = 0, by = 0, bz = 0;
    int d2 = 0;
    const bool box = nd && ncols == nrows && box_dictionary(nrows, dd, dvv, &bx, &by, &bz, &d2);
    if (nd && (rc = dv_build(A, nd, dd.data(), dvv.data(), mb, ml))) {
      msp_mat_destroy(&A);
      return rc;
    }
    if (box && (rc = march_attach(A, bx, by, bz, d2, true))) {
      msp_mat_destroy(&A);
      return rc;
    }
    // no dictionary covers it (variable coefficients): the stencil storage, if it is a box stencil's shape
    if (!A->dv_on && A->ndict == 0 && (rc = rv_attach(A, rowptr, col, val))) {
      msp_mat_destroy(&A);
      return rc;
    }
  }
  *out = A;
  return MSP_SUCCESS;
}

extern "C" int msp_mat_create_csr_rows(msp_ctx* c, int32_t nrows, int32_t ncols, int32_t nlisted,
                                       const int32_t* row_ids, const int32_t* rowptr, const int32_t* col,
                                       const double* val, msp_mat** out) {
  ARGCHK(c && out && (nlisted == 0 || (row_ids && rowptr)), MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(nrows >= 0 && ncols >= 0 && nlisted >= 0 && nlisted <= nrows, MSP_ERR_ARG_SIZ, "bad sizes");
  for (int32_t k = 0; k < nlisted; ++k) {
    ARGCHK(row_ids[k] >= 0 && row_ids[k] < nrows, MSP_ERR_ARG_OUTOFRANGE, "row id %d out of range", row_ids[k]);
    ARGCHK(k == 0 || row_ids[k] > row_ids[k - 1], MSP_ERR_ARG_WRONG, "row ids not strictly ascending");
  }
  int64_t nnz = 0, mb = 0;
  int32_t zero = 0;
  int64_t mb2 = 0;
  int rc = check_csr(nlisted, ncols, nlisted ? rowptr : &zero, col, &nnz, &mb, &mb2);
  if (rc) return rc;
  msp_mat* A = new msp_mat();
  A->ctx = c;
  mspi_ctx_retain(c);
  A->nrows = nrows;
  A->ncols = ncols;
  A->nnz = nnz;
  A->compressed = true;
  A->nlisted = nlisted;
  if ((rc = mat_alloc(c, A, (int64_t)nlisted + 1, nnz))) {
    msp_mat_destroy(&A);
    return rc;
  }
  HIPCHK(hipMalloc((void**)&A->row_ids, (size_t)(nlisted + 1) * sizeof(int32_t)));
  if (nlisted) {
    HIPCHK(hipMemcpyAsync(A->row_ids, row_ids, (size_t)nlisted * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(A->rowptr, rowptr, ((size_t)nlisted + 1) * sizeof(int32_t), hipMemcpyHostToDevice,
                          c->stream));
  } else {
    HIPCHK(hipMemsetAsync(A->rowptr, 0, sizeof(int32_t), c->stream));
  }
  if (nnz) {
    HIPCHK(hipMemcpyAsync(A->col, col, (size_t)nnz * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(A->val, val, (size_t)nnz * sizeof(double), hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  *out = A;
  return MSP_SUCCESS;
}

// The 7 stencil values of the upwind convection-diffusion operator h^2 (-Lap u + beta . grad u)
// in cell Peclet numbers P_d = beta_d h / 2 (x fastest; 2D: x and the line direction y):
//   lower neighbour in d: -1 - 2 max(P_d, 0), upper: -1 + 2 min(P_d, 0),
//   diagonal ((2*dim + 2|Px|) + 2|Py|) (+ 2|Pz| in 3D); P = 0 is the Poisson operator, exactly.
static BoxCoef box_coefs(int dim, const double* P) {
  const double px = P ? P[0] : 0.0, py = P ? P[1] : 0.0, pz = (P && dim == 3) ? P[2] : 0.0;
  auto cm = [](double p) { return -1.0 - 2.0 * (p > 0.0 ? p : 0.0); };
  auto cp = [](double p) { return -1.0 + 2.0 * (p < 0.0 ? p : 0.0); };
  BoxCoef c;
  if (dim == 3) {
    c.c[0] = cm(pz); c.c[1] = cm(py); c.c[2] = cm(px);
    c.c[3] = ((6.0 + 2.0 * fabs(px)) + 2.0 * fabs(py)) + 2.0 * fabs(pz);
    c.c[4] = cp(px); c.c[5] = cp(py); c.c[6] = cp(pz);
  } else {
    c.c[0] = cm(py); c.c[1] = 0.0; c.c[2] = cm(px);
    c.c[3] = (4.0 + 2.0 * fabs(px)) + 2.0 * fabs(py);
    c.c[4] = cp(px); c.c[5] = 0.0; c.c[6] = cp(py);
  }
  return c;
}

extern "C" int msp_mat_create_box_convdiff(msp_ctx* c, int dim, int32_t nx, int32_t ny, int32_t nz, int32_t lo,
                                           int32_t hi, const double* peclet, msp_mat** out) {
  ARGCHK(c && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(dim == 2 || dim == 3, MSP_ERR_ARG_WRONG, "dim must be 2 or 3, got %d", dim);
  if (dim == 2) nz = 1;
  ARGCHK(nx > 0 && ny > 0 && nz > 0, MSP_ERR_ARG_SIZ, "box %d x %d x %d", nx, ny, nz);
  lo = lo ? 1 : 0;
  hi = hi ? 1 : 0;
  const int64_t nrows = (int64_t)nx * ny * nz;
  const int64_t plane = dim == 3 ? (int64_t)nx * ny : (int64_t)nx;
  const int64_t ncols = nrows + (lo + hi) * plane;
  const int64_t deg = dim == 3 ? 7 : 5;
  ARGCHK(ncols <= INT32_MAX && deg * nrows <= INT32_MAX, MSP_ERR_ARG_OUTOFRANGE,
         "box of %lld rows exceeds 32-bit PetscInt indexing", (long long)nrows);
  ARGCHK(!peclet || (std::isfinite(peclet[0]) && std::isfinite(peclet[1]) && std::isfinite(peclet[2])),
         MSP_ERR_ARG_WRONG, "Peclet numbers must be finite");
  msp_mat* A = new msp_mat();
  A->ctx = c;
  mspi_ctx_retain(c);
  A->nrows = (int32_t)nrows;
  A->ncols = (int32_t)ncols;
  // exact nnz: deg*N minus missing neighbours on each face, plus the halo couplings
  int64_t nnz = deg * nrows - 2 * (nrows / nx) - 2 * (nrows / ny);
  if (dim == 3) nnz -= 2 * (nrows / nz);
  nnz += (lo + hi) * plane;
  A->nnz = nnz;
  A->lds_cap = lds_cap_for(deg * 256);
  A->lds_cap512 = lds_cap_for(deg * 512);
  A->plane = dim == 3 ? plane : 0;
  int rc = mat_alloc(c, A, nrows + 1, nnz);
  if (rc) {
    msp_mat_destroy(&A);
    return rc;
  }
  const BoxCoef cf = box_coefs(dim, peclet);
  {  // on a HIP failure A is destroyed, which also drops its reference on the context
    const int e1 = msk_box_stencil(dim, nx, ny, nz, nrows, lo, hi, &cf, A->rowptr, A->col, A->val, c->stream);
    const int e2 = e1 ? 0 : (int)hipStreamSynchronize(c->stream);
    if (e1 || e2) {
      msp_mat_destroy(&A);
      mspi_set_error(MSP_ERR_LIB, "box stencil assembly failed: %s", hipGetErrorString((hipError_t)(e1 ? e1 : e2)));
      return MSP_ERR_LIB;
    }
  }
  {  // the stencil's pairs: (slow-, y-, x-, diagonal, x+, y+, slow+) with the column shift of a lo plane
    const int32_t off = lo ? (int32_t)plane : 0, P = (int32_t)plane;
    std::vector<int32_t> dd;
    std::vector<double> dvv;
    const int32_t d3[7] = {off - P, off - nx, off - 1, off, off + 1, off + nx, off + P};
    for (int q = 0; q < 7; ++q) {
      if (dim == 2 && (q == 1 || q == 5)) continue;
      dd.push_back(d3[q]);
      dvv.push_back(cf.c[q]);
    }
    if ((rc = dv_build(A, (int)dd.size(), dd.data(), dvv.data(), deg * 256, (int32_t)deg))) {
      msp_mat_destroy(&A);
      return rc;
    }
    // the presence bytes the march kernels read instead of the codes (2D: marched as nx x 1 x ny)
    if ((rc = march_attach(A, nx, dim == 3 ? ny : 1, dim == 3 ? nz : ny, dim == 2, false,
                           (lo ? 1 : 0) | (hi ? 2 : 0)))) {
      msp_mat_destroy(&A);
      return rc;
    }
  }
  *out = A;
  return MSP_SUCCESS;
}

// The box operator applied without storage: same rows, same arithmetic as the
// assembled CSR (k_stencil_spmv), none of its 12 bytes per entry in HBM.
extern "C" int msp_mat_create_box_matfree(msp_ctx* c, int dim, int32_t nx, int32_t ny, int32_t nz, int32_t lo,
                                          int32_t hi, const double* peclet, msp_mat** out) {
  ARGCHK(c && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(dim == 2 || dim == 3, MSP_ERR_ARG_WRONG, "dim must be 2 or 3, got %d", dim);
  if (dim == 2) nz = 1;
  ARGCHK(nx > 0 && ny > 0 && nz > 0, MSP_ERR_ARG_SIZ, "box %d x %d x %d", nx, ny, nz);
  const int64_t P = dim == 3 ? (int64_t)nx * ny : (int64_t)nx;
  const int64_t nrows = P * (dim == 3 ? nz : ny);
  ARGCHK(nrows + (lo ? P : 0) + (hi ? P : 0) < INT32_MAX, MSP_ERR_ARG_SIZ, "box too large for int32 rows");
  ARGCHK(ny <= 65535 && nz <= 65535, MSP_ERR_ARG_SIZ, "matrix-free box: at most 65535 lines / planes (grid y, z)");
  msp_mat* A = new msp_mat();
  A->ctx = c;
  mspi_ctx_retain(c);
  A->matfree = true;
  A->dim = dim;
  A->bx = nx;
  A->by = ny;
  A->bz = nz;
  A->lo = lo ? 1 : 0;
  A->hi = hi ? 1 : 0;
  A->nrows = (int32_t)nrows;
  A->ncols = (int32_t)(nrows + (lo ? P : 0) + (hi ? P : 0));
  A->plane = P;
  A->cf = box_coefs(dim, peclet);
  // entries the assembled operator would hold: 7 (5) per row less the missing neighbours on the faces
  int64_t nnz = nrows * (dim == 3 ? 7 : 5);
  nnz -= 2 * (dim == 3 ? (int64_t)ny * nz + (int64_t)nx * nz : (int64_t)ny);  // x and (3D) y faces
  nnz -= (lo ? 0 : P) + (hi ? 0 : P);                                          // slow-direction faces
  A->nnz = nnz;
  *out = A;
  return MSP_SUCCESS;
}

extern "C" int msp_mat_create_box_stencil_ext(msp_ctx* c, int dim, int32_t nx, int32_t ny, int32_t nz, int32_t lo,
                                              int32_t hi, msp_mat** out) {
  return msp_mat_create_box_convdiff(c, dim, nx, ny, nz, lo, hi, nullptr, out);
}

extern "C" int msp_mat_create_box_stencil(msp_ctx* c, int dim, int32_t nx, int32_t ny, int32_t nz, msp_mat** out) {
  return msp_mat_create_box_stencil_ext(c, dim, nx, ny, nz, 0, 0, out);
}

extern "C" int msp_mat_destroy(msp_mat** pA) {
  if (!pA || !*pA) return MSP_SUCCESS;
  msp_mat* A = *pA;
  if (A->ctx && A->ctx->stream) (void)hipStreamSynchronize(A->ctx->stream);
  if (A->rowptr) (void)hipFree(A->rowptr);
  if (A->col) (void)hipFree(A->col);
  if (A->val) (void)hipFree(A->val);
  if (A->row_ids) (void)hipFree(A->row_ids);
  rv_free(A);
  dv_free(A);
  msp_ctx* c = A->ctx;
  delete A;
  *pA = nullptr;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

extern "C" int msp_mat_get_info(const msp_mat* A, int32_t* nrows, int32_t* ncols, int64_t* nnz) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "mat is NULL");
  if (nrows) *nrows = A->nrows;
  if (ncols) *ncols = A->ncols;
  if (nnz) *nnz = A->nnz;
  return MSP_SUCCESS;
}

extern "C" int msp_mat_get_csr(const msp_mat* A, int32_t* rowptr, int32_t* col, double* val) {
  ARGCHK(A && !A->matfree, A ? MSP_ERR_SUP : MSP_ERR_ARG_NULL, "no stored CSR (matrix-free operator)");
  ARGCHK(A && rowptr, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(!A->compressed, MSP_ERR_SUP, "msp_mat_get_csr on a row-compressed matrix");
  ARGCHK(!A->csr_released, MSP_ERR_SUP, "CSR storage released (msp_mat_release_csr)");
  hipStream_t s = A->ctx->stream;
  HIPCHK(hipMemcpyAsync(rowptr, A->rowptr, ((size_t)A->nrows + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (A->nnz) {
    ARGCHK(col && val, MSP_ERR_ARG_NULL, "col/val NULL");
    HIPCHK(hipMemcpyAsync(col, A->col, (size_t)A->nnz * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(val, A->val, (size_t)A->nnz * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  return MSP_SUCCESS;
}

static double spmv_bytes(const msp_mat* A, bool resid) {
  const double rows = A->compressed ? (double)A->nlisted : (double)A->nrows;
  const double xs = A->compressed ? (double)A->nnz : (double)A->ncols;
  return 12.0 * (double)A->nnz + 4.0 * (rows + 1) + 8.0 * xs + 8.0 * rows + (resid ? 8.0 * rows : 0.0);
}

// DV storage: 1 byte per entry and per row, the block starts, x read once, y written (b read, vout written)
static double dv_bytes(const msp_mat* A, bool resid, bool vout) {
  const double rows = (double)A->nrows;
  const double codes = A->dv_w ? (double)A->dv_w * rows : (double)A->nnz + rows + 4.0 * (rows / 256.0 + 1.0);
  return codes + 8.0 * (double)A->ncols + 8.0 * rows +
         (resid ? 8.0 * rows : 0.0) + (vout ? 8.0 * rows : 0.0);
}

// DV products of a box stencil take the z-march kernel when the tuning policy picks it
static bool box_march(const msp_mat* A) {
  return A->march_nx > 0 && A->march_halo == 0 && msk_box_march_pick(A->march_nx, A->march_ny, A->march_nz);
}

// a box with coupling planes in its column space: MatMult / MatResidual / MatMatMult by the chunk-tile march
static bool box_march_halo(const msp_mat* A) {
  return A->march_nx > 0 && A->march_halo != 0 && msk_box_march_pick(A->march_nx, A->march_ny, A->march_nz);
}

// the march reads one presence byte per row instead of the codes
static double march_bytes(const msp_mat* A, bool resid, bool vout) {
  const double rows = (double)A->nrows;
  return rows + 8.0 * (double)A->ncols + 8.0 * rows + (resid ? 8.0 * rows : 0.0) + (vout ? 8.0 * rows : 0.0);
}

// STENCIL storage: the presence byte and the seven values of every row, x once, y written (b read, vout written)
static double rv_bytes(const msp_mat* A, bool resid, bool vout) {  // 7 legs, or the symmetric storage's 4
  return (A->rv_stride < 0 ? 32.0 : 56.0) * (double)A->nrows + march_bytes(A, resid, vout);
}

extern "C" int msp_mat_set_storage(msp_mat* A, int storage) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "mat is NULL");
  ARGCHK(storage == MSP_STORAGE_CSR || storage == MSP_STORAGE_DV || storage == MSP_STORAGE_STENCIL,
         MSP_ERR_ARG_OUTOFRANGE, "unknown storage %d", storage);
  ARGCHK(!(A->csr_released && storage == MSP_STORAGE_CSR), MSP_ERR_SUP, "CSR storage released (msp_mat_release_csr)");
  if (storage == MSP_STORAGE_DV)
    ARGCHK(A->ndict > 0, MSP_ERR_SUP, "matrix has no DV storage (more than 256 (col - row, value) pairs, a row "
           "longer than 255, or not an assembled square-block CSR)");
  if (storage == MSP_STORAGE_STENCIL)
    ARGCHK(A->rv_val, MSP_ERR_SUP, "matrix has no stencil storage (not a 3D box stencil the chunk march takes, or "
           "a dictionary covers it)");
  A->dv_on = storage == MSP_STORAGE_DV;
  A->rv_on = storage == MSP_STORAGE_STENCIL;
  A->version++;
  return MSP_SUCCESS;
}

extern "C" int msp_mat_release_csr(msp_mat* A) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "mat is NULL");
  if (A->csr_released) return MSP_SUCCESS;
  ARGCHK(A->ndict > 0 && A->dv_on, MSP_ERR_SUP, "release_csr needs the matrix in DV storage");
  HIPCHK(hipStreamSynchronize(A->ctx->stream));
  if (A->col) HIPCHK(hipFree(A->col));
  if (A->val) HIPCHK(hipFree(A->val));
  A->col = nullptr;
  A->val = nullptr;
  if (A->dv_w) {  // the ELL layout reads no row pointers
    if (A->rowptr) HIPCHK(hipFree(A->rowptr));
    A->rowptr = nullptr;
  }
  A->lds_cap = A->lds_cap512 = 0;
  A->csr_released = true;
  A->version++;
  return MSP_SUCCESS;
}

extern "C" uint64_t mspi_mat_version(const msp_mat* A) { return A->version; }
extern "C" uint64_t mspi_ctx_epoch(const msp_ctx* c) { return c->epoch; }

// The GMRES step's MatMult folded into the CGS kernels (MSK_TUNE_GM_OPFUSE): A
// square, in DV storage with the 8-code ELL layout.  Bitwise the separate
// MatMult, and it saves W's 24 bytes per row, but measured 26 % slower per
// GMRES step (MDot 6.7 -> 4.3 TB/s): at the 2-3 waves per SIMD the CGS kernels
// run at, the far (+-plane) gathers of each row pair are 8 exposed round trips
// per workgroup, which the standalone SpMV hides with 6-8 waves.
extern "C" int mspi_op_fusable(const msp_mat* A) {
  return A && A->ctx->reduce == MSP_REDUCE_DBR && A->dv_on && A->dv_w == 8 && A->ndict <= 255 &&
         A->nrows == A->ncols && A->nrows > 0 &&
         (msk_get_tuning() & MSK_TUNE_GM_OPFUSE);
}

static EllOp ell_op(const msp_mat* A, const double* x, const double* sdev) {
  EllOp op;
  op.code8 = A->dv_code;
  op.ddelta = A->dv_delta;
  op.dval = A->dv_val;
  op.ndict = A->ndict;
  op.x = x;
  op.sdev = sdev;
  return op;
}

extern "C" int mspi_mdot_op(msp_mat* A, const double* x, const double* sdev, int nv, const double* base,
                            int64_t stride, const double* scale, double* out_dev, const int* stop) {
  if (!mspi_op_fusable(A) || nv < 1 || nv > MSPI_MAX_GROUP) return MSP_ERR_SUP;
  msp_ctx* c = A->ctx;
  const int64_t n = A->nrows, nch = nchunks_of(n);
  int rc = ensure_partial(c, nch * MSPI_MAX_GROUP);
  if (rc) return rc;
  {
    // codes once, the nv basis vectors (VV(it), the operator's x, among them)
    KTimer kt(c, MSP_KERNEL_MDOT, 8.0 * (double)n + 8.0 * (double)n * nv);
    const EllOp op = ell_op(A, x, sdev);
    Vecs vg = {};
    vg.base = base;
    vg.stride = stride;
    vg.scale = scale;
    KCHK(msk_dot_stage1_op(&op, &vg, nv, n, c->partial, nch, stop, c->stream));
  }
  KCHK(msk_dot_stage2(c->partial, nch, nv, out_dev, stop, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_maxpy_norm_update_op(msp_mat* A, const double* x, const double* sdev, double* wout, int nv,
                                         const double* base, int64_t stride, const double* scale, mspi_gmres_dev g,
                                         int m, const int* stop) {
  if (!mspi_op_fusable(A) || nv < 1) return MSP_ERR_SUP;
  msp_ctx* c = A->ctx;
  const int64_t n = A->nrows, nch = nchunks_of(n);
  int rc = ensure_partial(c, nch);
  if (rc) return rc;
  {
    // codes, the nv basis vectors read, VV(it+1) written
    KTimer kt(c, MSP_KERNEL_MAXPY, 8.0 * (double)n + 8.0 * (double)n * (nv + 1));
    const EllOp op = ell_op(A, x, sdev);
    Vecs vg = {};
    vg.base = base;
    vg.stride = stride;
    vg.scale = scale;
    KCHK(msk_maxpy_op(&op, wout, &vg, nv, g.h, n, c->partial, stop, c->stream));
  }
  return mspi_gm_norm_update(c, g, c->partial, nch, m);
}

extern "C" int mspi_graphs_enabled(msp_ctx* c) {
  if (c->timing || c->reduce == MSP_REDUCE_SEQ) return 0;
  const char* e = getenv("MSPLIT_GRAPHS");
  return !(e && e[0] == '0');
}

extern "C" int mspi_reserve_partial(msp_ctx* c, int64_t n) {
  return ensure_partial(c, std::max<int64_t>(nchunks_of(n), 1) * MSPI_MAX_GROUP);
}

extern "C" int mspi_capture_begin(msp_ctx* c) {
  if (!c->stream) return MSP_ERR_SUP;  // the legacy null stream cannot be captured
  if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed) != hipSuccess) {
    (void)hipGetLastError();  // the caller falls back to eager launches: leave no sticky error behind
    return MSP_ERR_SUP;
  }
  return MSP_SUCCESS;
}

extern "C" int mspi_capture_end(msp_ctx* c, int ok, void** exec) {
  hipGraph_t g = nullptr;
  *exec = nullptr;
  const hipError_t e = hipStreamEndCapture(c->stream, &g);
  if (!ok || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
    return ok ? MSP_ERR_SUP : MSP_SUCCESS;
  }
  hipGraphExec_t x = nullptr;
  const hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (ei != hipSuccess) {
    (void)hipGetLastError();
    return MSP_ERR_SUP;
  }
  *exec = (void*)x;
  return MSP_SUCCESS;
}

extern "C" int mspi_graph_launch(msp_ctx* c, void* exec) {
  HIPCHK(hipGraphLaunch((hipGraphExec_t)exec, c->stream));
  return MSP_SUCCESS;
}

extern "C" void mspi_graph_destroy(void* exec) {
  if (exec) (void)hipGraphExecDestroy((hipGraphExec_t)exec);
}

extern "C" int mspi_mat_spmm_dv(msp_mat* A, const double* S, int64_t lds, int nc, int64_t srows, double* R,
                                int64_t ldr) {
  if (!A->dv_on || !A->dv_w) return MSP_ERR_SUP;
  const bool bm = box_march(A), bh = !bm && box_march_halo(A);
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if ((bm || bh) && msk_march_chunk_fits(A->march_nx, A->march_ny, A->march_d2) && a16(S) && a16(R) &&
      lds % 2 == 0 && ldr % 2 == 0) {
    // a box stencil: column by column through the chunk-tile march (each R(r, q) the same CSR-order row sum as
    // the ELL SpMM's), presence bytes and S's columns read once per column, R written
    KTimer kt(A->ctx, MSP_KERNEL_SPMM, (double)nc * (march_bytes(A, false, false)));
    for (int q = 0; q < nc; ++q) {
      const double* sq = S + (int64_t)q * lds;
      double* rq = R + (int64_t)q * ldr;
      if (bm)
        KCHK(msk_spmv_box_march(A->march_nx, A->march_ny, A->march_nz, A->march_d2, A->march_mask, A->dv_val, sq,
                                nullptr, rq, MSK_SPMV_MULT, nullptr, nullptr, nullptr, A->ctx->stream));
      else
        KCHK(msk_box_march_halo(A->march_nx, A->march_ny, A->march_nz, A->march_halo, A->march_mask, A->dv_val, sq,
                                nullptr, rq, MSK_SPMV_MULT, A->ctx->stream));
    }
    return MSP_SUCCESS;
  }
  // codes once, S's columns read once, R written
  KTimer kt(A->ctx, MSP_KERNEL_SPMM, (double)A->dv_w * A->nrows + 8.0 * nc * ((double)srows + A->nrows));
  KCHK(msk_spmm_ell(A->nrows, A->dv_w, A->dv_code, A->dv_delta, A->dv_val, A->ndict, S, lds, nc, R, ldr,
                    A->ctx->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_mat_get_storage(const msp_mat* A, int* storage, int* ndict) {
  ARGCHK(A && storage, MSP_ERR_ARG_NULL, "NULL argument");
  *storage = A->matfree ? MSP_STORAGE_NONE
             : A->dv_on  ? MSP_STORAGE_DV
             : A->rv_on  ? MSP_STORAGE_STENCIL
                         : MSP_STORAGE_CSR;
  if (ndict) *ndict = A->ndict;
  return MSP_SUCCESS;
}

extern "C" int msp_mat_get_spmv_kernel(const msp_mat* A, const char** name) {
  ARGCHK(A && name, MSP_ERR_ARG_NULL, "NULL argument");
  if (A->matfree) *name = "k_stencil_spmv";
  else if (A->compressed) *name = "k_spmv_rows";
  else if (A->rv_on) *name = A->rv_stride < 0 ? "k_box_march_chunk_rv_sym" : "k_box_march_chunk_rv";
  else if (A->dv_on && (box_march(A) || box_march_halo(A))) *name = "k_spmv_box_march";
  else if (A->dv_on) *name = A->dv_w ? "k_spmv_ell" : "k_spmv_dv";
  else *name = A->lds_cap > 0 ? "k_spmv_lds8" : "k_spmv_csr";
  return MSP_SUCCESS;
}

static int spmv_impl(msp_mat* A, const double* b, const double* x, double* y, bool resid) {
  msp_ctx* c = A->ctx;
  if (A->matfree) {  // x and y (and b) only
    KTimer kt(c, MSP_KERNEL_SPMV, 8.0 * (double)A->ncols + 8.0 * A->nrows * (resid ? 2.0 : 1.0));
    KCHK(msk_stencil_spmv(A->dim, A->bx, A->by, A->bz, A->nrows, A->lo, A->hi, &A->cf, x, b, y,
                          resid ? MSK_SPMV_RESID : MSK_SPMV_MULT, nullptr, nullptr, nullptr, c->stream));
    return MSP_SUCCESS;
  }
  if (A->compressed) {
    KTimer kt(c, MSP_KERNEL_SPMV, spmv_bytes(A, resid));
    // rows that hold no entries: y = 0 (MatMult) or r = b - 0 = b (MatResidual)
    if (resid) {
      if (y != b) HIPCHK(hipMemcpyAsync(y, b, (size_t)A->nrows * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    } else {
      KCHK(msk_blas1(MSK_SET, y, nullptr, nullptr, 0.0, A->nrows, c->stream));
    }
    KCHK(msk_spmv_rows(A->nlisted, A->row_ids, A->rowptr, A->col, A->val, x, b, y, resid ? 1 : 0, c->stream));
    return MSP_SUCCESS;
  }
  if (A->rv_on) {
    KTimer kt(c, MSP_KERNEL_SPMV, rv_bytes(A, resid, false));
    KCHK(msk_box_march_chunk_rv(A->march_nx, A->march_ny, A->march_nz, A->march_mask, A->rv_val, A->rv_stride, x, b, y,
                                resid ? MSK_SPMV_RESID : MSK_SPMV_MULT, nullptr, nullptr, nullptr, c->stream));
    return MSP_SUCCESS;
  }
  if (A->dv_on) {
    const int mode = resid ? MSK_SPMV_RESID : MSK_SPMV_MULT;
    const bool bm = box_march(A);
    // a block's A_ext with coupling planes: the chunk march when its operands fit (a vector not 16-byte aligned
    // takes the row-parallel kernel below), decided before the launch so a launch error is reported, not hidden
    const bool bh = !bm && box_march_halo(A) &&
                    msk_box_march_halo_fits(A->march_nx, A->march_ny, A->march_nz, A->march_halo, x, b, y, mode);
    KTimer kt(c, MSP_KERNEL_SPMV, bm || bh ? march_bytes(A, resid, false) : dv_bytes(A, resid, false));
    if (bm) {
      KCHK(msk_spmv_box_march(A->march_nx, A->march_ny, A->march_nz, A->march_d2, A->march_mask, A->dv_val, x, b, y,
                              mode, nullptr, nullptr, nullptr, c->stream));
      return MSP_SUCCESS;
    }
    if (bh) {
      KCHK(msk_box_march_halo(A->march_nx, A->march_ny, A->march_nz, A->march_halo, A->march_mask, A->dv_val, x, b, y,
                              mode, c->stream));
      return MSP_SUCCESS;
    }
    KCHK(msk_spmv_dv(A->nrows, A->rowptr, A->dv_len, A->dv_code, A->dv_delta, A->dv_val, A->ndict, A->dv_mb, A->dv_w, x, b,
                     y, resid ? MSK_SPMV_RESID : MSK_SPMV_MULT, nullptr, nullptr, nullptr, A->plane, c->stream));
    return MSP_SUCCESS;
  }
  KTimer kt(c, MSP_KERNEL_SPMV, spmv_bytes(A, resid));
  KCHK(msk_spmv(A->nrows, A->rowptr, A->col, A->val, x, b, y, A->lds_cap, resid ? MSK_SPMV_RESID : MSK_SPMV_MULT,
                nullptr, nullptr, nullptr, A->plane, c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_spmv(msp_mat* A, const double* x, double* y) { return spmv_impl(A, nullptr, x, y, false); }
extern "C" int mspi_residual(msp_mat* A, const double* b, const double* x, double* r) {
  return spmv_impl(A, b, x, r, true);
}

extern "C" int mspi_spmv_scaled(msp_mat* A, const double* x, const double* sdev, double* vout, double* y,
                                const int* stop) {
  msp_ctx* c = A->ctx;
  if (A->compressed || A->nrows != A->ncols) {
    mspi_set_error(MSP_ERR_SUP, "scaled MatMult needs a square, uncompressed operator");
    return MSP_ERR_SUP;
  }
  if (A->matfree) {
    KTimer kt(c, MSP_KERNEL_SPMV, 8.0 * (double)A->ncols + (vout ? 16.0 : 8.0) * (double)A->nrows);
    KCHK(msk_stencil_spmv(A->dim, A->bx, A->by, A->bz, A->nrows, A->lo, A->hi, &A->cf, x, nullptr, y,
                          MSK_SPMV_SCALED, sdev, vout, stop, c->stream));
    return MSP_SUCCESS;
  }
  if (A->rv_on) {
    KTimer kt(c, MSP_KERNEL_SPMV, rv_bytes(A, false, vout != nullptr));
    KCHK(msk_box_march_chunk_rv(A->march_nx, A->march_ny, A->march_nz, A->march_mask, A->rv_val, A->rv_stride, x,
                                nullptr, y, MSK_SPMV_SCALED, sdev, vout, stop, c->stream));
    return MSP_SUCCESS;
  }
  if (A->dv_on) {
    const bool bm = box_march(A);
    KTimer kt(c, MSP_KERNEL_SPMV, bm ? march_bytes(A, false, vout != nullptr) : dv_bytes(A, false, vout != nullptr));
    if (bm) {
      KCHK(msk_spmv_box_march(A->march_nx, A->march_ny, A->march_nz, A->march_d2, A->march_mask, A->dv_val, x, nullptr, y,
                              MSK_SPMV_SCALED, sdev, vout, stop, c->stream));
      return MSP_SUCCESS;
    }
    KCHK(msk_spmv_dv(A->nrows, A->rowptr, A->dv_len, A->dv_code, A->dv_delta, A->dv_val, A->ndict, A->dv_mb, A->dv_w, x,
                     nullptr, y, MSK_SPMV_SCALED, sdev, vout, stop, A->plane, c->stream));
    return MSP_SUCCESS;
  }
  KTimer kt(c, MSP_KERNEL_SPMV, spmv_bytes(A, false) + (vout ? 8.0 * (double)A->nrows : 0.0));
  KCHK(msk_spmv(A->nrows, A->rowptr, A->col, A->val, x, nullptr, y, A->lds_cap, MSK_SPMV_SCALED, sdev, vout, stop,
                A->plane, c->stream));
  return MSP_SUCCESS;
}

// GMRES: y = A (sc*x) fused with VecMDot(y, basis 0..nv-1) into out_dev (both DBR
// stages); returns MSP_ERR_SUP when the operator cannot take the fused kernel (the
// caller then runs mspi_spmv_scaled + mspi_mdot_basis, with identical results).
extern "C" int mspi_spmv_mdot(msp_mat* A, const double* x, const double* sdev, double* y, int nv, const double* base,
                              int64_t stride, const double* scale, double* out_dev, const int* stop) {
  msp_ctx* c = A->ctx;
  const int64_t n = A->nrows;
  const int64_t nch = nchunks_of(n);
  if (c->reduce == MSP_REDUCE_DBR && A->rv_on && y && nv >= 1 && nv <= MSPI_MAX_GROUP && nch > 0 &&
      !(msk_get_tuning() & MSK_TUNE_GM_BOX_MDOT_OFF)) {
    // the stencil storage: the chunk-tile march with the rows' values, W stored (the MAXPY reads it), the dots
    // from the registers; bytes as the march's plus the 56 value bytes per row
    int rc = ensure_partial(c, nch * MSPI_MAX_GROUP);
    if (rc) return rc;
    {
      KTimer kt(c, MSP_KERNEL_SPMVDOT, rv_bytes(A, false, false) + 8.0 * (double)n * nv);
      Vecs vg = {};
      vg.base = base;
      vg.stride = stride;
      vg.scale = scale;
      const int64_t P = (int64_t)A->march_nx * A->march_ny;
      int self = 0;
      KCHK(msk_box_spmv_mdot_rv(A->march_nx, P, n, 0, A->march_mask, nullptr, A->rv_val, A->rv_stride, x, sdev, y,
                                &vg, nv, c->partial, nch, stop, &self, c->stream));
      if (self) kt.set_bytes(rv_bytes(A, false, false) + 8.0 * (double)n * (nv - 1));
    }
    KCHK(msk_dot_stage2(c->partial, nch, nv, out_dev, stop, c->stream));
    return MSP_SUCCESS;
  }
  if (c->reduce == MSP_REDUCE_DBR && A->dv_on && box_march(A) && A->march_nx <= 2048 && nv >= 1 &&
      nv <= MSPI_MAX_GROUP && nch > 0 && !(msk_get_tuning() & MSK_TUNE_GM_BOX_MDOT_OFF)) {
    int rc = ensure_partial(c, nch * MSPI_MAX_GROUP);
    if (rc) return rc;
    {
      // the march's bytes (presence byte, x, W written) and MDot's nv basis vectors; W is not re-read, and
      // neither is x when it is the basis' last vector (its dot comes from the march's registers)
      // (y = NULL: the W-free step, W not written; mspi_maxpy_norm_update_march recomputes it)
      const double wb = y ? 0.0 : 8.0 * (double)n;
      KTimer kt(c, MSP_KERNEL_SPMVDOT, march_bytes(A, false, false) - wb + 8.0 * (double)n * nv);
      Vecs vg = {};
      vg.base = base;
      vg.stride = stride;
      vg.scale = scale;
      const int64_t P = (int64_t)A->march_nx * A->march_ny;
      int self = 0;
      KCHK(msk_box_spmv_mdot(A->march_nx, P, n, A->march_d2, A->march_mask, A->dv_val, x, sdev, y, &vg, nv,
                             c->partial, nch, stop, &self, c->stream));
      if (self) kt.set_bytes(march_bytes(A, false, false) - wb + 8.0 * (double)n * (nv - 1));
    }
    KCHK(msk_dot_stage2(c->partial, nch, nv, out_dev, stop, c->stream));
    return MSP_SUCCESS;
  }
  if (c->reduce == MSP_REDUCE_SEQ || A->matfree || A->compressed || A->csr_released || A->nrows != A->ncols ||
      A->lds_cap512 <= 0 || nv < 1 ||
      nv > MSPI_MAX_GROUP ||
      nch == 0 || !(msk_get_tuning() & MSK_TUNE_GM_SPMV_MDOT))
    return MSP_ERR_SUP;
  int rc = ensure_partial(c, nch * MSPI_MAX_GROUP);
  if (rc) return rc;
  {
    // bytes: the SpMV's (x read, y written) plus MDot's nv basis vectors; W is not re-read
    KTimer kt(c, MSP_KERNEL_SPMVDOT, spmv_bytes(A, false) + 8.0 * (double)n * nv);
    Vecs vg = {};
    vg.base = base;
    vg.stride = stride;
    vg.scale = scale;
    KCHK(msk_spmv_mdot(A->nrows, A->rowptr, A->col, A->val, x, sdev, y, A->lds_cap512, &vg, nv, c->partial, nch,
                       stop, c->stream));
  }
  KCHK(msk_dot_stage2(c->partial, nch, nv, out_dev, stop, c->stream));  // ~4 us, not in the class stats
  return MSP_SUCCESS;
}

// The W-free GMRES step (DBR order, box stencil taking the fused march): mspi_spmv_mdot is called with
// y = NULL and mspi_maxpy_norm_update_march recomputes W.  1 when A takes it.
extern "C" int mspi_gm_wfree(const msp_mat* A) {
  const msp_ctx* c = A->ctx;
  if (c->reduce != MSP_REDUCE_DBR || !A->dv_on || !box_march(A) || (msk_get_tuning() & MSK_TUNE_GM_BOX_MDOT_OFF))
    return 0;
  return msk_box_wfree_fits(A->march_nx, (int64_t)A->march_nx * A->march_ny, A->nrows, A->march_d2);
}

// VV(it+1) = A (sc x) - sum_j h_j VV(j), x = VV(it) the basis' last vector, with the ||VV(it+1)||^2 partials
// (k_box_maxpy_march), then the fold + Hessenberg update (k_norm_update) as mspi_maxpy_norm_update.
extern "C" int mspi_maxpy_norm_update_march(msp_mat* A, const double* x, const double* sdev, double* wout, int nv,
                                            const double* base, int64_t stride, const double* scale,
                                            mspi_gmres_dev g, int m, const int* stop) {
  msp_ctx* c = A->ctx;
  const int64_t n = A->nrows, nch = nchunks_of(n);
  if (nch == 0 || nv <= 0 || !mspi_gm_wfree(A)) {
    mspi_set_error(MSP_ERR_SUP, "W-free MAXPY on an operator that does not take it");
    return MSP_ERR_SUP;
  }
  {
    // the march's presence byte and x (VV(it), read once: also the basis' last vector), nv - 1 basis vectors, wout
    KTimer kt(c, MSP_KERNEL_MAXPY, (double)n + 8.0 * (double)A->ncols + 8.0 * (double)n * nv);
    Vecs vg = {};
    vg.base = base;
    vg.stride = stride;
    vg.scale = scale;
    KCHK(msk_box_maxpy_march(A->march_nx, (int64_t)A->march_nx * A->march_ny, n, A->march_d2, A->march_mask, A->dv_val, x, sdev,
                             wout, &vg, nv, g.h, c->partial, stop, c->stream));
  }
  return mspi_gm_norm_update(c, g, c->partial, nch, m);
}

static int vec_ok(const msp_vec* v, const char* name) {
  if (!v) {
    mspi_set_error(MSP_ERR_ARG_NULL, "%s is NULL", name);
    return MSP_ERR_ARG_NULL;
  }
  return MSP_SUCCESS;
}

extern "C" int msp_mat_mult(msp_mat* A, const msp_vec* x, msp_vec* y) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "mat is NULL");
  int rc;
  if ((rc = vec_ok(x, "x")) || (rc = vec_ok(y, "y"))) return rc;
  ARGCHK(x->n == A->ncols && y->n == A->nrows, MSP_ERR_ARG_SIZ,
         "MatMult sizes: A %d x %d, x %lld, y %lld", A->nrows, A->ncols, (long long)x->n, (long long)y->n);
  ARGCHK(x->d != y->d, MSP_ERR_ARG_WRONG, "x and y must be different vectors");
  return mspi_spmv(A, x->d, y->d);
}

extern "C" int msp_mat_residual(msp_mat* A, const msp_vec* b, const msp_vec* x, msp_vec* r) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "mat is NULL");
  int rc;
  if ((rc = vec_ok(b, "b")) || (rc = vec_ok(x, "x")) || (rc = vec_ok(r, "r"))) return rc;
  ARGCHK(x->n == A->ncols && b->n == A->nrows && r->n == A->nrows, MSP_ERR_ARG_SIZ,
         "MatResidual sizes: A %d x %d, b %lld, x %lld, r %lld", A->nrows, A->ncols, (long long)b->n,
         (long long)x->n, (long long)r->n);
  ARGCHK(x->d != r->d, MSP_ERR_ARG_WRONG, "x and r must be different vectors");
  return mspi_residual(A, b->d, x->d, r->d);
}

extern "C" int msp_mat_residual_listed(msp_mat* A, const msp_vec* b, const msp_vec* x, msp_vec* r) {
  ARGCHK(A, MSP_ERR_ARG_NULL, "mat is NULL");
  int rc;
  if ((rc = vec_ok(b, "b")) || (rc = vec_ok(x, "x")) || (rc = vec_ok(r, "r"))) return rc;
  ARGCHK(A->compressed, MSP_ERR_SUP, "msp_mat_residual_listed needs a row-compressed matrix");
  ARGCHK(x->n == A->ncols && b->n == A->nrows && r->n == A->nrows, MSP_ERR_ARG_SIZ,
         "MatResidual sizes: A %d x %d, b %lld, x %lld, r %lld", A->nrows, A->ncols, (long long)b->n,
         (long long)x->n, (long long)r->n);
  ARGCHK(x->d != r->d, MSP_ERR_ARG_WRONG, "x and r must be different vectors");
  msp_ctx* c = A->ctx;
  // the listed rows' entries and b, their x reads, r written
  KTimer kt(c, MSP_KERNEL_SPMV,
            12.0 * (double)A->nnz + 8.0 * (double)A->nlisted * 3.0 + 4.0 * (double)A->nlisted + 8.0 * (double)A->nnz);
  KCHK(msk_spmv_rows(A->nlisted, A->row_ids, A->rowptr, A->col, A->val, x->d, b->d, r->d, 1, c->stream));
  return MSP_SUCCESS;
}

// -------------------------------------------------------------------- Vec
extern "C" int msp_vec_create(msp_ctx* c, int64_t n, msp_vec** out) {
  ARGCHK(c && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(n >= 0, MSP_ERR_ARG_SIZ, "negative vector size %lld", (long long)n);
  msp_vec* v = new msp_vec();
  v->ctx = c;
  mspi_ctx_retain(c);
  v->n = n;
  v->owned = 1;
  // pad to 512 doubles so every vector is 4 KiB aligned and double2 loads stay in bounds
  const size_t bytes = (size_t)((n + 511) / 512 * 512 + 512) * sizeof(double);
  if (mspi_big_alloc((void**)&v->d, bytes) != (int)hipSuccess) {
    delete v;
    mspi_ctx_release(c);
    mspi_set_error(MSP_ERR_MEM, "hipMalloc of a %lld-entry vector failed", (long long)n);
    return MSP_ERR_MEM;
  }
  HIPCHK(hipMemsetAsync(v->d, 0, bytes, c->stream));
  *out = v;
  return MSP_SUCCESS;
}

extern "C" int msp_vec_create_with_array(msp_ctx* c, int64_t n, double* dptr, msp_vec** out) {
  ARGCHK(c && out && (dptr || n == 0), MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(n >= 0, MSP_ERR_ARG_SIZ, "negative vector size");
  ARGCHK(((uintptr_t)dptr & 15) == 0, MSP_ERR_ARG_WRONG, "device array must be 16-byte aligned");
  msp_vec* v = new msp_vec();
  v->ctx = c;
  mspi_ctx_retain(c);
  v->n = n;
  v->d = dptr;
  v->owned = 0;
  *out = v;
  return MSP_SUCCESS;
}

extern "C" int msp_vec_destroy(msp_vec** pv) {
  if (!pv || !*pv) return MSP_SUCCESS;
  msp_vec* v = *pv;
  if (v->owned && v->d) {
    (void)hipStreamSynchronize(v->ctx->stream);
    (void)hipFree(v->d);
  }
  msp_ctx* c = v->ctx;
  delete v;
  *pv = nullptr;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

extern "C" int msp_vec_get_size(const msp_vec* v, int64_t* n) {
  ARGCHK(v && n, MSP_ERR_ARG_NULL, "NULL argument");
  *n = v->n;
  return MSP_SUCCESS;
}

extern "C" int msp_vec_get_array(msp_vec* v, double** p) {
  ARGCHK(v && p, MSP_ERR_ARG_NULL, "NULL argument");
  *p = v->d;
  return MSP_SUCCESS;
}

extern "C" int msp_vec_set_values(msp_vec* v, int64_t off, int64_t n, const double* host) {
  ARGCHK(v && (host || n == 0), MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(off >= 0 && n >= 0 && off + n <= v->n, MSP_ERR_ARG_OUTOFRANGE, "range [%lld,%lld) outside [0,%lld)",
         (long long)off, (long long)(off + n), (long long)v->n);
  if (n == 0) return MSP_SUCCESS;
  HIPCHK(hipMemcpyAsync(v->d + off, host, (size_t)n * sizeof(double), hipMemcpyHostToDevice, v->ctx->stream));
  HIPCHK(hipStreamSynchronize(v->ctx->stream));  // the host buffer stays the caller's
  return MSP_SUCCESS;
}

extern "C" int msp_vec_get_values(const msp_vec* v, int64_t off, int64_t n, double* host) {
  ARGCHK(v && (host || n == 0), MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(off >= 0 && n >= 0 && off + n <= v->n, MSP_ERR_ARG_OUTOFRANGE, "range [%lld,%lld) outside [0,%lld)",
         (long long)off, (long long)(off + n), (long long)v->n);
  if (n == 0) return MSP_SUCCESS;
  HIPCHK(hipMemcpyAsync(host, v->d + off, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, v->ctx->stream));
  HIPCHK(hipStreamSynchronize(v->ctx->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_vec_copy_range(const msp_vec* src, int64_t so, msp_vec* dst, int64_t dof, int64_t n) {
  ARGCHK(src && dst, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(n >= 0 && so >= 0 && dof >= 0 && so + n <= src->n && dof + n <= dst->n, MSP_ERR_ARG_OUTOFRANGE,
         "copy_range out of bounds");
  if (n == 0) return MSP_SUCCESS;
  return mspi_copy(dst->ctx, dst->d + dof, src->d + so, n);
}

extern "C" int msp_vec_set(msp_vec* v, double a) {
  int rc = vec_ok(v, "v");
  if (rc) return rc;
  return mspi_set(v->ctx, v->d, v->n, a);
}

extern "C" int msp_vec_copy(const msp_vec* x, msp_vec* y) {
  int rc;
  if ((rc = vec_ok(x, "x")) || (rc = vec_ok(y, "y"))) return rc;
  ARGCHK(x->n == y->n, MSP_ERR_ARG_SIZ, "VecCopy sizes %lld vs %lld", (long long)x->n, (long long)y->n);
  return mspi_copy(y->ctx, y->d, x->d, x->n);
}

extern "C" int msp_vec_scale(msp_vec* x, double a) {
  int rc = vec_ok(x, "x");
  if (rc) return rc;
  if (a == 1.0) return MSP_SUCCESS;  // VecScale returns early for alpha == 1
  return mspi_scale(x->ctx, x->d, x->n, a);
}

static int blas1(msp_ctx* c, int op, double* y, const double* x, const double* z, double a, int64_t n, double bytes) {
  KTimer kt(c, MSP_KERNEL_OTHER, bytes);
  KCHK(msk_blas1(op, y, x, z, a, n, c->stream));
  return MSP_SUCCESS;
}

extern "C" int msp_vec_axpy(msp_vec* y, double a, const msp_vec* x) {
  int rc;
  if ((rc = vec_ok(x, "x")) || (rc = vec_ok(y, "y"))) return rc;
  ARGCHK(x->n == y->n, MSP_ERR_ARG_SIZ, "VecAXPY sizes");
  if (a == 0.0) return MSP_SUCCESS;  // daxpy returns for da == 0
  return blas1(y->ctx, MSK_AXPY, y->d, x->d, nullptr, a, y->n, 24.0 * y->n);
}

extern "C" int msp_vec_aypx(msp_vec* y, double b, const msp_vec* x) {
  int rc;
  if ((rc = vec_ok(x, "x")) || (rc = vec_ok(y, "y"))) return rc;
  ARGCHK(x->n == y->n, MSP_ERR_ARG_SIZ, "VecAYPX sizes");
  return blas1(y->ctx, MSK_AYPX, y->d, x->d, nullptr, b, y->n, 24.0 * y->n);
}

extern "C" int msp_vec_waxpy(msp_vec* w, double a, const msp_vec* x, const msp_vec* y) {
  int rc;
  if ((rc = vec_ok(w, "w")) || (rc = vec_ok(x, "x")) || (rc = vec_ok(y, "y"))) return rc;
  ARGCHK(x->n == y->n && w->n == x->n, MSP_ERR_ARG_SIZ, "VecWAXPY sizes");
  int op = a == 1.0 ? MSK_WAXPY_P1 : (a == -1.0 ? MSK_WAXPY_M1 : MSK_WAXPY);
  if (a == 0.0) return mspi_copy(w->ctx, w->d, y->d, w->n);
  return blas1(w->ctx, op, w->d, x->d, y->d, a, w->n, 24.0 * w->n);
}

extern "C" int msp_vec_dot(const msp_vec* x, const msp_vec* y, double* val) {
  int rc;
  if ((rc = vec_ok(x, "x")) || (rc = vec_ok(y, "y"))) return rc;
  ARGCHK(val, MSP_ERR_ARG_NULL, "val is NULL");
  ARGCHK(x->n == y->n, MSP_ERR_ARG_SIZ, "VecDot sizes");
  msp_ctx* c = x->ctx;
  const double* V[1] = {y->d};
  if ((rc = mspi_mdot(c, x->d, 1, V, x->n, c->dscratch))) return rc;
  if ((rc = mspi_d2h_sync(c, c->hscratch, c->dscratch, sizeof(double)))) return rc;
  *val = c->hscratch[0];
  return MSP_SUCCESS;
}

extern "C" int msp_vec_norm(const msp_vec* x, double* val) {
  int rc = vec_ok(x, "x");
  if (rc) return rc;
  ARGCHK(val, MSP_ERR_ARG_NULL, "val is NULL");
  msp_ctx* c = x->ctx;
  if ((rc = mspi_norm2sq(c, x->d, x->n, c->dscratch))) return rc;
  if ((rc = mspi_d2h_sync(c, c->hscratch, c->dscratch, sizeof(double)))) return rc;
  *val = sqrt(c->hscratch[0]);
  return MSP_SUCCESS;
}

extern "C" int msp_vec_normalize(msp_vec* x, double* val) {
  double t = 0.0;
  int rc = msp_vec_norm(x, &t);
  if (rc) return rc;
  if (t != 0.0 && !std::isnan(t) && !std::isinf(t)) {
    const double s = 1.0 / t;
    if ((rc = mspi_scale(x->ctx, x->d, x->n, s))) return rc;
  }
  if (val) *val = t;
  return MSP_SUCCESS;
}

extern "C" int msp_vec_mdot(const msp_vec* x, int nv, const msp_vec* const* y, double* val) {
  int rc = vec_ok(x, "x");
  if (rc) return rc;
  ARGCHK(nv >= 0 && (nv == 0 || (y && val)), MSP_ERR_ARG_NULL, "NULL argument");
  std::vector<const double*> V(nv);
  for (int j = 0; j < nv; ++j) {
    if ((rc = vec_ok(y[j], "y[j]"))) return rc;
    ARGCHK(y[j]->n == x->n, MSP_ERR_ARG_SIZ, "VecMDot sizes");
    V[j] = y[j]->d;
  }
  msp_ctx* c = x->ctx;
  const int step = kScratch - 8;
  for (int g0 = 0; g0 < nv; g0 += step) {
    const int g = std::min(step, nv - g0);
    if ((rc = mspi_mdot(c, x->d, g, V.data() + g0, x->n, c->dscratch))) return rc;
    if ((rc = mspi_d2h_sync(c, c->hscratch, c->dscratch, (size_t)g * sizeof(double)))) return rc;
    memcpy(val + g0, c->hscratch, (size_t)g * sizeof(double));
  }
  return MSP_SUCCESS;
}

extern "C" int msp_vec_maxpy(msp_vec* y, int nv, const double* alpha, const msp_vec* const* x) {
  int rc = vec_ok(y, "y");
  if (rc) return rc;
  ARGCHK(nv >= 0 && (nv == 0 || (x && alpha)), MSP_ERR_ARG_NULL, "NULL argument");
  std::vector<const double*> V(nv);
  for (int j = 0; j < nv; ++j) {
    if ((rc = vec_ok(x[j], "x[j]"))) return rc;
    ARGCHK(x[j]->n == y->n, MSP_ERR_ARG_SIZ, "VecMAXPY sizes");
    ARGCHK(((uintptr_t)x[j]->d & 15) == 0, MSP_ERR_ARG_WRONG, "unaligned vector");
    V[j] = x[j]->d;
  }
  return mspi_maxpy(y->ctx, y->d, nv, V.data(), y->n, alpha, nullptr, 0, 0);
}
