// msplit_ctx.hpp -- the context object and the error/timing helpers shared by
// the C++/HIP translation units (runtime, dense/LSQR, comm).  Internal only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <atomic>
#include <vector>

#include "msplit.h"
#include "msplit_internal.h"
#include "msplit_kernels.h"

#define HIPCHK(call)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess) {                                                                       \
      mspi_set_error(MSP_ERR_LIB, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                     __LINE__);                                                                   \
      return MSP_ERR_LIB;                                                                         \
    }                                                                                             \
  } while (0)

#define KCHK(call)                                                                                  \
  do {                                                                                              \
    int e_ = (call);                                                                                \
    if (e_) {                                                                                       \
      mspi_set_error(MSP_ERR_LIB, "kernel launch %s failed: %s", #call,                             \
                     hipGetErrorString((hipError_t)e_));                                            \
      return MSP_ERR_LIB;                                                                           \
    }                                                                                               \
  } while (0)

#define ARGCHK(cond, code, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      mspi_set_error(code, __VA_ARGS__); \
      return code;                     \
    }                                  \
  } while (0)

// ---------------------------------------------------------------- context
struct TimedRec {
  int cls;
  int ev;  // index of the start event in the pool; stop = ev + 1
  double bytes;
};

struct msp_ctx {
  // msp_ctx_destroy drops the caller's reference; every object made on the context holds one more
  // (mspi_ctx_retain / mspi_ctx_release), so objects may be destroyed after their context in any order
  std::atomic<int> refs{1};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  double* dscratch = nullptr;  // device scalars
  double* hscratch = nullptr;  // pinned host scalars
  double* partial = nullptr;   // DBR stage-1 partials
  int64_t partial_cap = 0;     // doubles
  void* seqbuf = nullptr;      // MSP_REDUCE_SEQ's transducers and guesses (msplit_seq.hip)
  int64_t seqbuf_cap = 0;      // bytes
  uint32_t seq_epoch = 0;      // the overlapped transducer builds' flag value (msplit_seq.hip seqx_core)
  int64_t seq_spin = 400000000; // the device's g_seq_spin_ticks as this context last set it (msplit_seq.hip)
  hipStream_t seq_aux = nullptr;   // their stream (CU-masked), the walks' stream (the other CUs), and the events
  hipStream_t seq_walk = nullptr;  // that order them with the context's
  hipEvent_t seq_ev[3] = {nullptr, nullptr, nullptr};
  uint32_t* seqready = nullptr;  // the builds' per-segment ready words (zeroed when allocated; never hold anything else)
  int64_t seqready_cap = 0;      // words
  double* seqacc = nullptr;    // MSP_REDUCE_SEQ chains: two rows of MSK_MAX_GROUP running sums
  uint64_t epoch = 0;          // bumped when a buffer captured graphs point at is reallocated
  int reduce = MSP_REDUCE_DBR;  // MSP_REDUCE_SEQ: PETSc's sequential order (msplit_seq.hip)
  bool timing = false;
  int timing_every = 1;         // time one logical kernel in timing_every per class
  int64_t timing_seen[16] = {};  // per-class launch counters (MSP_KERNEL_NCLASSES <= 16)
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  std::vector<TimedRec> recs;
};

static const int kScratch = 4 * MSPI_MAX_GROUP + 64;

// Brackets one logical kernel (possibly two launches) with a pair of events.
struct KTimer {
  msp_ctx* c;
  int ev = -1;
  KTimer(msp_ctx* ctx, int cls, double bytes) : c(ctx) {
    if (!c->timing) return;
    if (c->timing_every > 1 && (c->timing_seen[cls & 15]++ % c->timing_every) != 0) return;
    if (c->pool_used + 2 > c->pool.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->pool.push_back(e);
      }
    }
    ev = (int)c->pool_used;
    c->pool_used += 2;
    (void)hipEventRecord(c->pool[ev], c->stream);
    c->recs.push_back({cls, ev, bytes});
  }
  void set_bytes(double b) {  // the launch turned out to move b algorithmic bytes (this timer's record is the last)
    if (ev >= 0) c->recs.back().bytes = b;
  }
  ~KTimer() {
    if (ev >= 0) (void)hipEventRecord(c->pool[ev + 1], c->stream);
  }
};


static inline int ensure_partial(msp_ctx* c, int64_t need) {
  if (need <= c->partial_cap) return MSP_SUCCESS;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->partial) HIPCHK(hipFree(c->partial));
  c->partial = nullptr;
  c->partial_cap = 0;
  HIPCHK(hipMalloc((void**)&c->partial, (size_t)need * sizeof(double)));
  c->partial_cap = need;
  c->epoch++;
  return MSP_SUCCESS;
}

// MSP_REDUCE_SEQ's stage 1 (msplit_seq.hip): the sequential sums in the DBR partial layout
int mspi_seq_stage1(msp_ctx* c, const double* w, const Vecs* V, int nv, int64_t n, int self, double* partial,
                    int64_t nchunks, const int* stop);

static inline int64_t nchunks_of(int64_t n) { return (n + MSK_DBR_CHUNK - 1) / MSK_DBR_CHUNK; }

