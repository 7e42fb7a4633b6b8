// msplit_comm.hip -- cross-process all-gather for the distributed minimization.
//
// The reference reduces nothing here: it ships half of R (N/2 x s doubles) to
// the other block every outer iteration and both blocks run the same LSQR
// (comm.c:252-286, SMSM-global.c:329).  With R row-distributed over the GPUs,
// one LSQR step needs two reductions of at most s+1 doubles per block; they
// are all-gathered and added in block order on every rank, so the result is
// bitwise the same on every rank and for any collective algorithm.
//
// RCCL is opened lazily with dlopen("librccl.so.1"): in a process that already
// loaded it (PyTorch's ProcessGroupNCCL) the same copy is reused, and code that
// never builds a communicator never loads it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "msplit_ctx.hpp"

namespace {

struct RcclApi {
  bool ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*get_error_string)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
  static RcclApi api;
  static bool tried = false;
  if (tried) return api;
  tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return api;
  api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
  api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
  api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
  api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
  api.get_error_string = (decltype(api.get_error_string))dlsym(h, "ncclGetErrorString");
  api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_gather && api.get_error_string;
  return api;
}

}  // namespace

enum { COMM_RCCL = 0, COMM_HOST = 1 };

struct msp_comm {
  msp_ctx* ctx = nullptr;
  int kind = COMM_RCCL;
  int32_t nranks = 1, rank = 0;
  ncclComm_t nccl = nullptr;
  msp_allgather_fn fn = nullptr;
  void* user = nullptr;
  double* hsend = nullptr;  // pinned staging (host transport)
  double* hrecv = nullptr;
  int64_t hcap = 0;         // doubles per rank
};

#define NCCLCHK(call)                                                                            \
  do {                                                                                           \
    ncclResult_t r_ = (call);                                                                    \
    if (r_ != ncclSuccess) {                                                                     \
      mspi_set_error(MSP_ERR_LIB, "%s failed: %s", #call, rccl().get_error_string(r_));           \
      return MSP_ERR_LIB;                                                                        \
    }                                                                                            \
  } while (0)

extern "C" int msp_comm_get_unique_id(uint8_t id[MSP_COMM_ID_BYTES]) {
  ARGCHK(id, MSP_ERR_ARG_NULL, "id is NULL");
  ARGCHK(rccl().ok, MSP_ERR_LIB, "librccl.so.1 could not be loaded");
  static_assert(sizeof(ncclUniqueId) == MSP_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  NCCLCHK(rccl().get_unique_id(&u));
  memcpy(id, &u, sizeof(u));
  return MSP_SUCCESS;
}

extern "C" int msp_comm_create_rccl(msp_ctx* c, int32_t nranks, int32_t rank, const uint8_t id[MSP_COMM_ID_BYTES],
                                    msp_comm** out) {
  ARGCHK(c && id && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(nranks >= 1 && rank >= 0 && rank < nranks, MSP_ERR_ARG_OUTOFRANGE, "rank %d of %d", rank, nranks);
  ARGCHK(rccl().ok, MSP_ERR_LIB, "librccl.so.1 could not be loaded");
  HIPCHK(hipSetDevice(c->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t nc = nullptr;
  NCCLCHK(rccl().comm_init_rank(&nc, nranks, u, rank));
  msp_comm* m = new msp_comm();
  m->ctx = c;
  m->kind = COMM_RCCL;
  m->nranks = nranks;
  m->rank = rank;
  m->nccl = nc;
  *out = m;
  return MSP_SUCCESS;
}

extern "C" int msp_comm_create_host(msp_ctx* c, int32_t nranks, int32_t rank, msp_allgather_fn fn, void* user,
                                    msp_comm** out) {
  ARGCHK(c && fn && out, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(nranks >= 1 && rank >= 0 && rank < nranks, MSP_ERR_ARG_OUTOFRANGE, "rank %d of %d", rank, nranks);
  msp_comm* m = new msp_comm();
  m->ctx = c;
  m->kind = COMM_HOST;
  m->nranks = nranks;
  m->rank = rank;
  m->fn = fn;
  m->user = user;
  *out = m;
  return MSP_SUCCESS;
}

extern "C" int msp_comm_destroy(msp_comm** pm) {
  if (!pm || !*pm) return MSP_SUCCESS;
  msp_comm* m = *pm;
  if (m->ctx && m->ctx->stream) (void)hipStreamSynchronize(m->ctx->stream);
  if (m->nccl) (void)rccl().comm_destroy(m->nccl);
  if (m->hsend) (void)hipHostFree(m->hsend);
  if (m->hrecv) (void)hipHostFree(m->hrecv);
  delete m;
  *pm = nullptr;
  return MSP_SUCCESS;
}

extern "C" int msp_comm_get_size(const msp_comm* m, int32_t* nranks, int32_t* rank) {
  ARGCHK(m, MSP_ERR_ARG_NULL, "comm is NULL");
  if (nranks) *nranks = m->nranks;
  if (rank) *rank = m->rank;
  return MSP_SUCCESS;
}

extern "C" int mspi_comm_allgather(msp_comm* m, const double* send, double* recv, int64_t count) {
  msp_ctx* c = m->ctx;
  if (count <= 0) return MSP_SUCCESS;
  if (m->kind == COMM_RCCL) {
    NCCLCHK(rccl().all_gather(send, recv, (size_t)count, ncclDouble, m->nccl, c->stream));
    return MSP_SUCCESS;
  }
  if (count > m->hcap) {
    HIPCHK(hipStreamSynchronize(c->stream));
    if (m->hsend) HIPCHK(hipHostFree(m->hsend));
    if (m->hrecv) HIPCHK(hipHostFree(m->hrecv));
    m->hsend = m->hrecv = nullptr;
    m->hcap = 0;
    HIPCHK(hipHostMalloc((void**)&m->hsend, (size_t)count * sizeof(double), hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&m->hrecv, (size_t)count * m->nranks * sizeof(double), hipHostMallocDefault));
    m->hcap = count;
  }
  HIPCHK(hipMemcpyAsync(m->hsend, send, (size_t)count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int rc = m->fn(m->user, m->hsend, m->hrecv, count);
  if (rc) {
    mspi_set_error(MSP_ERR_LIB, "host all-gather callback failed with %d", rc);
    return MSP_ERR_LIB;
  }
  HIPCHK(hipMemcpyAsync(recv, m->hrecv, (size_t)count * m->nranks * sizeof(double), hipMemcpyHostToDevice,
                        c->stream));
  return MSP_SUCCESS;
}

extern "C" int mspi_comm_size(const msp_comm* m, int32_t* nranks, int32_t* rank) {
  *nranks = m ? m->nranks : 1;
  *rank = m ? m->rank : 0;
  return MSP_SUCCESS;
}

extern "C" int msp_comm_allgather(msp_comm* m, const msp_vec* send, msp_vec* recv, int64_t count) {
  ARGCHK(m && send && recv, MSP_ERR_ARG_NULL, "NULL argument");
  ARGCHK(count >= 0 && count <= send->n && count * m->nranks <= recv->n, MSP_ERR_ARG_SIZ,
         "allgather of %lld per rank: send %lld, recv %lld", (long long)count, (long long)send->n,
         (long long)recv->n);
  return mspi_comm_allgather(m, send->d, recv->d, count);
}
