/*
 * amsg.c -- newest-value message slots between the blocks of an asynchronous
 * multisplitting run, in POSIX shared memory (one node, one process -- or one
 * host thread -- per GPU).
 *
 * Replaces the MPI point-to-point layer of the asynchronous drivers:
 *   - iterate exchange: comm_async_test_and_send_prime / _probe_and_receive_prime
 *     (src/utils/comm.c:455-554): MPI_Isend of (PhaseTag, iteration, x_i), the
 *     receiver draining every pending message with MPI_Iprobe/MPI_Recv and keeping
 *     the newest;
 *   - convergence-detection control (src/utils/conv_detection_prime.c): partial-CV,
 *     verification, response and verdict messages, each received by the same
 *     drain-to-newest loop.
 * A receiver only ever uses the newest message of a (source, kind) pair, so
 * each pair is one slot holding the newest message, written under a sequence
 * lock: seq odd while the writer fills it, even when complete; a reader takes
 * the slot when seq is even, newer than the last one it took, and unchanged
 * across its copy.  No queue, no allocation, no message can block a sender.
 *
 * Iterate payloads are boundary planes: only chain neighbours (|src - dst| = 1,
 * the z-slab blocks) get a data slot of data_cap doubles.  *_vec variants move
 * the plane between HBM and the slot (the region is registered with the HIP
 * runtime, so the copies are DMA transfers).
 *
 * Device slots (msp_amsg_enable_device): the payload lives in the sender's HBM,
 * two buffers per neighbour, exported by HIP IPC, and neither end waits for a
 * copy on the host.  A send claims the buffer that is not the newest, enqueues
 * the plane's copy into it and, behind the copy on the sender's stream, a
 * one-lane kernel that publishes (count, buffer) into the shared word `pub`
 * (a system-scope store into this registered region).  A receive that sees a
 * newer `pub` marks that buffer as being read, enqueues the copy out of it
 * (over xGMI) and, behind it, a kernel that clears the mark.  A send whose
 * previous copy is still unpublished, or whose buffer the receiver still
 * holds, is skipped -- the reference's comm_async_test_and_send_prime, which
 * posts a new MPI_Isend only when MPI_Test says the previous one completed
 * (comm.c:528-535).  The claim / mark handshake is Dekker's (each side stores
 * its word, then loads the other's, sequentially consistent), so a buffer is
 * never written while it is read.  When sender and receiver share one stream
 * (the blocks of a process, run round-robin), stream order already serialises
 * every copy, so publication and release are immediate host stores: the
 * schedule, and every result, is that of synchronous copies.
 *
 * Host code only: no GPU is needed for the control messages (the CPU tests use
 * them across processes).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "msplit.h"
#include "msplit_internal.h"

#define AMSG_MAGIC 0x4d53504c414d5347ULL /* "MSPLAMSG" */
#define AMSG_INTS 6

typedef struct {
  _Atomic uint64_t seq;
  int32_t ints[AMSG_INTS];
  int64_t n;
  uint8_t pad[64 - 8 - 4 * AMSG_INTS - 8];
} ctrl_slot; /* one cache line */

typedef struct {
  uint64_t magic;
  int32_t nranks;
  int32_t pad0;
  int64_t data_cap;
  _Atomic int32_t attached;
  uint8_t pad[64 - 28];
} region_header;

/* one per rank, after the data slots: the rank's exported device slots */
typedef struct {
  _Atomic int32_t ready;
  int32_t pid;
  uint64_t rawptr; /* valid in the exporting process only */
  uint64_t stream; /* the exporting context's stream (same process: same stream => stream-ordered copies) */
  uint8_t handle[MSPI_IPC_HANDLE_BYTES];
  uint8_t pad[128 - 24 - MSPI_IPC_HANDLE_BYTES];
} ipc_entry;

/* device-slot state of one (src, direction) link, in the shared region */
typedef struct {
  _Atomic uint64_t pub;         /* (count << 1) | buffer of the newest complete message; 0: none yet (GPU-written) */
  _Atomic uint64_t claim;       /* (count << 1) | buffer of the sender's latest send; == pub: nothing in flight */
  _Atomic uint32_t reading[2];  /* the receiver's copy out of buffer b is pending (cleared by its stream) */
  int32_t ints[2][AMSG_INTS];   /* the tags of the message in buffer b */
  int64_t n[2];
  uint8_t pad[128 - 24 - 8 * AMSG_INTS - 16];
} dslot_state;

struct msp_amsg {
  char name[128];
  int32_t nranks, rank, owner;
  int64_t data_cap;
  size_t bytes;
  uint8_t *base;
  region_header *hdr;
  ctrl_slot *ctrl;   /* [src][dst][kind] */
  uint8_t *data;     /* [src][dir] slots of data_bytes */
  size_t data_bytes; /* header line + data_cap doubles, rounded to 4 KiB */
  uint64_t *seen;    /* [src][kind] last sequence number taken by this rank */
  int registered;
  ipc_entry *ipc;    /* [rank] */
  dslot_state *dst_; /* [src][dir] device-slot states */
  dslot_state *dst_dev; /* the same words as the GPU addresses them (registered region) */
  msp_ctx *dctx;     /* device slots enabled: the context their copies run on */
  uint64_t skey;     /* its stream */
  double *dslots;    /* this rank's 2 directions x 2 buffers x data_cap device slots (dir 0: to rank-1) */
  double **peer;     /* [src] resolved device slots of src (NULL: not yet) */
  uint8_t *opened;   /* [src] peer[src] came from hipIpcOpenMemHandle */
  int64_t sent, skipped; /* device-slot sends posted / skipped (previous one in flight, or buffer still read) */
};

static int aerr(int code, const char *msg) {
  mspi_set_error(code, "%s", msg);
  return code;
}

static size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static ctrl_slot *ctrl_at(msp_amsg *m, int src, int dst, int kind) {
  return m->ctrl + ((size_t)src * m->nranks + dst) * MSP_AMSG_NKINDS + kind;
}

/* data slot of the (src -> dst) chain link, or NULL */
static ctrl_slot *data_at(msp_amsg *m, int src, int dst) {
  int dir;
  if (dst == src - 1) dir = 0;
  else if (dst == src + 1) dir = 1;
  else return NULL;
  return (ctrl_slot *)(m->data + ((size_t)src * 2 + dir) * m->data_bytes);
}

static ctrl_slot *slot_for(msp_amsg *m, int src, int dst, int kind) {
  if (kind == MSP_AMSG_DATA) return data_at(m, src, dst);
  return ctrl_at(m, src, dst, kind);
}

int msp_amsg_create(const char *name, int32_t nranks, int32_t rank, int64_t data_cap, int32_t owner,
                    msp_amsg **out) {
  if (!name || !out) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  if (nranks < 1 || nranks > 4096 || rank < 0 || rank >= nranks || data_cap < 0)
    return aerr(MSP_ERR_ARG_OUTOFRANGE, "bad amsg sizes");
  if (strlen(name) >= sizeof(((msp_amsg *)0)->name) || name[0] != '/')
    return aerr(MSP_ERR_ARG_WRONG, "shared-memory name must start with '/' and be < 128 chars");
  msp_amsg *m = (msp_amsg *)calloc(1, sizeof(msp_amsg));
  if (!m) return aerr(MSP_ERR_MEM, "allocation failed");
  strcpy(m->name, name);
  m->nranks = nranks;
  m->rank = rank;
  m->owner = owner ? 1 : 0;
  m->data_cap = data_cap;
  m->data_bytes = round_up(sizeof(ctrl_slot) + (size_t)data_cap * sizeof(double), 4096);
  const size_t ctrl_bytes = round_up((size_t)nranks * nranks * MSP_AMSG_NKINDS * sizeof(ctrl_slot), 4096);
  const size_t ipc_bytes = round_up((size_t)nranks * sizeof(ipc_entry), 4096);
  const size_t dstate_bytes = round_up((size_t)nranks * 2 * sizeof(dslot_state), 4096);
  m->bytes = 4096 + ctrl_bytes + (size_t)nranks * 2 * m->data_bytes + ipc_bytes + dstate_bytes;
  int fd;
  if (m->owner) {
    shm_unlink(name); /* a stale region of an earlier run */
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)m->bytes) != 0) {
      close(fd);
      fd = -1;
    }
  } else {
    fd = shm_open(name, O_RDWR, 0600);
  }
  if (fd < 0) {
    free(m);
    mspi_set_error(MSP_ERR_LIB, "shm_open(%s) failed: %s", name, strerror(errno));
    return MSP_ERR_LIB;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < m->bytes) {
    close(fd);
    free(m);
    return aerr(MSP_ERR_ARG_SIZ, "shared-memory region smaller than the layout (sizes differ between ranks?)");
  }
  m->base = (uint8_t *)mmap(NULL, m->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m->base == MAP_FAILED) {
    free(m);
    return aerr(MSP_ERR_MEM, "mmap of the shared-memory region failed");
  }
  m->hdr = (region_header *)m->base;
  m->ctrl = (ctrl_slot *)(m->base + 4096);
  m->data = m->base + 4096 + ctrl_bytes;
  m->ipc = (ipc_entry *)(m->data + (size_t)nranks * 2 * m->data_bytes);
  m->dst_ = (dslot_state *)((uint8_t *)m->ipc + ipc_bytes);
  if (m->owner) {
    m->hdr->nranks = nranks;
    m->hdr->data_cap = data_cap;
    atomic_store_explicit(&m->hdr->attached, 0, memory_order_relaxed);
    atomic_thread_fence(memory_order_release);
    m->hdr->magic = AMSG_MAGIC; /* ftruncate zeroed every slot: seq = 0, nothing sent */
  } else if (m->hdr->magic != AMSG_MAGIC || m->hdr->nranks != nranks || m->hdr->data_cap != data_cap) {
    munmap(m->base, m->bytes);
    free(m);
    return aerr(MSP_ERR_ARG_WRONG, "shared-memory region not initialised by the owner, or different sizes");
  }
  m->seen = (uint64_t *)calloc((size_t)nranks * (MSP_AMSG_NKINDS), sizeof(uint64_t));
  if (!m->seen) {
    munmap(m->base, m->bytes);
    free(m);
    return aerr(MSP_ERR_MEM, "allocation failed");
  }
  atomic_fetch_add_explicit(&m->hdr->attached, 1, memory_order_acq_rel);
  *out = m;
  return MSP_SUCCESS;
}

int msp_amsg_attached(const msp_amsg *m, int32_t *n) {
  if (!m || !n) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  *n = atomic_load_explicit(&m->hdr->attached, memory_order_acquire);
  return MSP_SUCCESS;
}

static int ensure_registered(msp_amsg *m);

int msp_amsg_enable_device(msp_amsg *m, msp_ctx *ctx) {
  if (!m || !ctx) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  if (m->dctx) return MSP_SUCCESS;
  m->peer = (double **)calloc((size_t)m->nranks, sizeof(double *));
  m->opened = (uint8_t *)calloc((size_t)m->nranks, 1);
  if (!m->peer || !m->opened) return aerr(MSP_ERR_MEM, "allocation failed");
  /* the GPU publishes and releases through the state words: the region must be mapped for it */
  int rc = ensure_registered(m);
  if (rc) return rc;
  void *dp = NULL;
  if ((rc = mspi_host_device_ptr(m->dst_, &dp))) return rc;
  m->dst_dev = (dslot_state *)dp;
  void *p = NULL;
  rc = mspi_dev_alloc(ctx, (size_t)4 * (size_t)(m->data_cap > 0 ? m->data_cap : 1) * sizeof(double), &p);
  if (rc) return rc;
  ipc_entry *e = &m->ipc[m->rank];
  if ((rc = mspi_ipc_export(p, e->handle))) {
    mspi_dev_free(p);
    return rc;
  }
  m->dslots = (double *)p;
  m->dctx = ctx;
  m->skey = mspi_stream_key(ctx);
  mspi_ctx_retain(ctx);
  e->pid = (int32_t)getpid();
  e->rawptr = (uint64_t)(uintptr_t)p;
  e->stream = m->skey;
  atomic_store_explicit(&e->ready, 1, memory_order_release);
  return MSP_SUCCESS;
}

int msp_amsg_get_stats(const msp_amsg *m, int64_t *sent, int64_t *skipped) {
  if (!m) return aerr(MSP_ERR_ARG_NULL, "amsg is NULL");
  if (sent) *sent = m->sent;
  if (skipped) *skipped = m->skipped;
  return MSP_SUCCESS;
}

int msp_amsg_close_peers(msp_amsg *m) {
  if (!m) return aerr(MSP_ERR_ARG_NULL, "amsg is NULL");
  if (!m->peer) return MSP_SUCCESS;
  /* this rank's copies out of the peers' slots (and its publish / release stores) are stream-ordered: let them
   * finish before the mappings go (the drivers call close_peers on every rank, barrier, then destroy) */
  if (m->dctx) {
    int rc = msp_ctx_synchronize(m->dctx);
    if (rc) return rc;
  }
  for (int r = 0; r < m->nranks; ++r) {
    if (m->opened[r]) mspi_ipc_close(m->peer[r]);
    m->peer[r] = NULL;
    m->opened[r] = 0;
  }
  return MSP_SUCCESS;
}

static dslot_state *dstate(msp_amsg *m, int src, int dir);

/* comm_discard_pending_messages (comm.c:426-453) and the MPI_Cancel of the sends still pending at the end of a run
 * (AMAM-global_prime.c:522-572).  Every message newer than the last one this rank took -- any source, any kind --
 * is marked taken without being read; this rank's device sends whose copy is enqueued but not yet published cannot
 * be withdrawn (a DMA), so they are counted and completed by draining the stream. */
int msp_amsg_discard_pending(msp_amsg *m, int64_t *discarded, int64_t *in_flight) {
  if (!m) return aerr(MSP_ERR_ARG_NULL, "amsg is NULL");
  int64_t nd = 0, nf = 0;
  for (int src = 0; src < m->nranks; ++src) {
    if (src == m->rank) continue;
    for (int kind = 0; kind < MSP_AMSG_NKINDS; ++kind) {
      uint64_t *seen = m->seen + (size_t)src * MSP_AMSG_NKINDS + kind;
      if (kind == MSP_AMSG_DATA && !data_at(m, src, m->rank)) continue;
      if (kind == MSP_AMSG_DATA && m->dctx) {
        dslot_state *d = dstate(m, src, m->rank == src - 1 ? 0 : 1);
        const uint64_t P = atomic_load_explicit(&d->pub, memory_order_seq_cst);
        if (P && P != *seen) {
          *seen = P;
          ++nd;
        }
        continue;
      }
      ctrl_slot *s = slot_for(m, src, m->rank, kind);
      const uint64_t q = atomic_load_explicit(&s->seq, memory_order_acquire);
      if (!(q & 1) && q != *seen) {
        *seen = q;
        ++nd;
      }
    }
  }
  if (m->dctx) {
    for (int dir = 0; dir < 2; ++dir) {
      dslot_state *d = dstate(m, m->rank, dir);
      if (atomic_load_explicit(&d->claim, memory_order_seq_cst) != atomic_load_explicit(&d->pub, memory_order_seq_cst))
        ++nf;
    }
    int rc = msp_ctx_synchronize(m->dctx);
    if (rc) return rc;
  }
  if (discarded) *discarded = nd;
  if (in_flight) *in_flight = nf;
  return MSP_SUCCESS;
}

/* diagnostics (tools, tests): the state of the link src -> this rank as this rank sees it */
int msp_amsg_get_link_info(const msp_amsg *m, int32_t src, int64_t *info, int32_t n) {
  if (!m || !info) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  if (src < 0 || src >= m->nranks || src == m->rank) return aerr(MSP_ERR_ARG_OUTOFRANGE, "peer rank out of range");
  int64_t v[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  msp_amsg *mm = (msp_amsg *)m;
  if (data_at(mm, src, m->rank) && m->dst_) {
    dslot_state *d = mm->dst_ + (size_t)src * 2 + (m->rank == src - 1 ? 0 : 1);
    v[0] = (int64_t)atomic_load_explicit(&d->pub, memory_order_seq_cst);
    v[1] = (int64_t)atomic_load_explicit(&d->claim, memory_order_seq_cst);
  }
  v[2] = (int64_t)m->seen[(size_t)src * MSP_AMSG_NKINDS + MSP_AMSG_DATA];
  v[3] = (int64_t)atomic_load_explicit(&ctrl_at(mm, src, m->rank, MSP_AMSG_PARTIAL_CV)->seq, memory_order_acquire);
  v[4] = (int64_t)m->seen[(size_t)src * MSP_AMSG_NKINDS + MSP_AMSG_PARTIAL_CV];
  v[5] = (int64_t)atomic_load_explicit(&ctrl_at(mm, src, m->rank, MSP_AMSG_VERDICT)->seq, memory_order_acquire);
  v[6] = m->peer ? (int64_t)(m->peer[src] != NULL) : -1;
  v[7] = (int64_t)atomic_load_explicit(&m->hdr->attached, memory_order_acquire);
  for (int i = 0; i < n && i < 8; ++i) info[i] = v[i];
  return MSP_SUCCESS;
}

/* the device slots of src, opened on first use; NULL while src has not enabled them */
static int peer_slots(msp_amsg *m, int src, double **out) {
  *out = m->peer[src];
  if (*out) return MSP_SUCCESS;
  ipc_entry *e = &m->ipc[src];
  if (!atomic_load_explicit(&e->ready, memory_order_acquire)) return MSP_SUCCESS;
  if (e->pid == (int32_t)getpid()) {
    m->peer[src] = (double *)(uintptr_t)e->rawptr; /* same process: the allocation itself */
  } else {
    void *p = NULL;
    int rc = mspi_ipc_open(m->dctx, e->handle, &p);
    if (rc) return rc;
    m->peer[src] = (double *)p;
    m->opened[src] = 1;
  }
  *out = m->peer[src];
  return MSP_SUCCESS;
}

int msp_amsg_destroy(msp_amsg **pm) {
  if (!pm || !*pm) return MSP_SUCCESS;
  msp_amsg *m = *pm;
  msp_amsg_close_peers(m); /* also drains this rank's stream: no GPU store into the region is left pending */
  if (m->dslots) {
    atomic_store_explicit(&m->ipc[m->rank].ready, 0, memory_order_release);
    mspi_dev_free(m->dslots);
  }
  free(m->peer);
  free(m->opened);
  if (m->registered) mspi_host_unregister(m->base);
  munmap(m->base, m->bytes);
  if (m->owner) shm_unlink(m->name);
  free(m->seen);
  msp_ctx *c = m->dctx;
  free(m);
  *pm = NULL;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

/* the slot direction of this rank's messages to dst (0: dst = rank - 1, 1: dst = rank + 1) */
static int dst_rank_dir(const msp_amsg *m, int dst) { return dst == m->rank - 1 ? 0 : 1; }

/* seqlock writer: seq odd, payload, seq even */
static void write_begin(ctrl_slot *s) {
  const uint64_t q = atomic_load_explicit(&s->seq, memory_order_relaxed);
  atomic_store_explicit(&s->seq, q + 1, memory_order_relaxed);
  atomic_thread_fence(memory_order_release);
}

static void write_end(ctrl_slot *s) {
  const uint64_t q = atomic_load_explicit(&s->seq, memory_order_relaxed);
  atomic_store_explicit(&s->seq, q + 1, memory_order_release);
}

static int check_pair(msp_amsg *m, int peer, int kind) {
  if (peer < 0 || peer >= m->nranks || peer == m->rank) return aerr(MSP_ERR_ARG_OUTOFRANGE, "peer rank out of range");
  if (kind < 0 || kind >= MSP_AMSG_NKINDS) return aerr(MSP_ERR_ARG_OUTOFRANGE, "unknown message kind");
  return MSP_SUCCESS;
}

int msp_amsg_send(msp_amsg *m, int32_t dst, int32_t kind, const int32_t *ints, int32_t nints, const double *data,
                  int64_t n) {
  if (!m) return aerr(MSP_ERR_ARG_NULL, "amsg is NULL");
  int rc = check_pair(m, dst, kind);
  if (rc) return rc;
  if (nints < 0 || nints > AMSG_INTS || (nints && !ints)) return aerr(MSP_ERR_ARG_SIZ, "at most 6 ints per message");
  ctrl_slot *s = slot_for(m, m->rank, dst, kind);
  if (!s) return aerr(MSP_ERR_ARG_WRONG, "iterate data only travels between chain neighbours");
  if (kind == MSP_AMSG_DATA && m->dctx) return aerr(MSP_ERR_ARG_WRONG, "device slots enabled: send planes with *_vec");
  if (kind == MSP_AMSG_DATA ? (n < 0 || n > m->data_cap || (n && !data)) : n != 0)
    return aerr(MSP_ERR_ARG_SIZ, "payload larger than the data slot");
  write_begin(s);
  memset(s->ints, 0, sizeof(s->ints));
  if (nints) memcpy(s->ints, ints, (size_t)nints * sizeof(int32_t));
  s->n = n;
  if (n) memcpy((double *)(s + 1), data, (size_t)n * sizeof(double));
  write_end(s);
  return MSP_SUCCESS;
}

/* seqlock reader; got = 1 when a newer complete message was copied out */
static int read_slot(msp_amsg *m, int src, int kind, int32_t *ints, int32_t nints, double *data, int64_t cap,
                     int64_t *n, int32_t *got, msp_vec *v, int64_t voff) {
  ctrl_slot *s = slot_for(m, src, m->rank, kind);
  if (!s) return aerr(MSP_ERR_ARG_WRONG, "iterate data only travels between chain neighbours");
  uint64_t *seen = m->seen + (size_t)src * MSP_AMSG_NKINDS + kind;
  *got = 0;
  for (int attempt = 0; attempt < 8; ++attempt) {
    const uint64_t s1 = atomic_load_explicit(&s->seq, memory_order_acquire);
    if ((s1 & 1) || s1 == *seen) return MSP_SUCCESS; /* being written, or nothing new: try next round */
    int32_t tmp[AMSG_INTS];
    memcpy(tmp, s->ints, sizeof(tmp));
    const int64_t len = s->n;
    if (len < 0 || len > m->data_cap) continue;
    if (len) {
      if (len > cap) return aerr(MSP_ERR_ARG_SIZ, "receive buffer smaller than the message");
      if (v) {
        int rc = mspi_h2d_sync(v->ctx, v->d + voff, (const double *)(s + 1), (size_t)len * sizeof(double));
        if (rc) return rc;
      } else {
        memcpy(data, (const double *)(s + 1), (size_t)len * sizeof(double));
      }
    }
    atomic_thread_fence(memory_order_acquire);
    const uint64_t s2 = atomic_load_explicit(&s->seq, memory_order_relaxed);
    if (s1 != s2) continue; /* overwritten while copying: take the newer one */
    if (nints) memcpy(ints, tmp, (size_t)nints * sizeof(int32_t));
    if (n) *n = len;
    *seen = s1;
    *got = 1;
    return MSP_SUCCESS;
  }
  return MSP_SUCCESS;
}

int msp_amsg_recv(msp_amsg *m, int32_t src, int32_t kind, int32_t *ints, int32_t nints, double *data, int64_t cap,
                  int64_t *n, int32_t *got) {
  if (!m || !got) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  int rc = check_pair(m, src, kind);
  if (rc) return rc;
  if (nints < 0 || nints > AMSG_INTS || (nints && !ints)) return aerr(MSP_ERR_ARG_SIZ, "at most 6 ints per message");
  if (kind == MSP_AMSG_DATA && m->dctx) return aerr(MSP_ERR_ARG_WRONG, "device slots enabled: receive planes with *_vec");
  return read_slot(m, src, kind, ints, nints, data, cap, n, got, NULL, 0);
}

static int ensure_registered(msp_amsg *m) {
  if (m->registered) return MSP_SUCCESS;
  int rc = mspi_host_register(m->base, m->bytes);
  if (rc) return rc;
  m->registered = 1;
  return MSP_SUCCESS;
}

/* ------------------------------------------------------------ device slots */
static dslot_state *dstate(msp_amsg *m, int src, int dir) { return m->dst_ + (size_t)src * 2 + dir; }
static dslot_state *dstate_dev(msp_amsg *m, int src, int dir) { return m->dst_dev + (size_t)src * 2 + dir; }

/* peer's slots driven by this very stream (the blocks of one process): stream order serialises every copy */
static int same_stream(msp_amsg *m, int peer) {
  ipc_entry *e = &m->ipc[peer];
  return atomic_load_explicit(&e->ready, memory_order_acquire) && e->pid == (int32_t)getpid() && e->stream == m->skey;
}

static double *slot_buf(double *base, const msp_amsg *m, int dir, int b) {
  return base + ((size_t)dir * 2 + (size_t)b) * (size_t)m->data_cap;
}

static int send_vec_device(msp_amsg *m, int dst, const int32_t *ints, int32_t nints, const msp_vec *v, int64_t off,
                           int64_t n) {
  const int dir = dst_rank_dir(m, dst);
  dslot_state *d = dstate(m, m->rank, dir);
  const uint64_t P = atomic_load_explicit(&d->pub, memory_order_seq_cst);
  if (atomic_load_explicit(&d->claim, memory_order_relaxed) != P) { /* the previous copy is not published yet */
    m->skipped++;
    return MSP_SUCCESS;
  }
  const int b = P ? 1 - (int)(P & 1) : 0; /* the buffer that is not the newest */
  const uint64_t W = ((P >> 1) + 1) << 1 | (uint64_t)b;
  atomic_store_explicit(&d->claim, W, memory_order_seq_cst);
  if (atomic_load_explicit(&d->reading[b], memory_order_seq_cst)) { /* the receiver still copies out of b */
    atomic_store_explicit(&d->claim, P, memory_order_seq_cst);
    m->skipped++;
    return MSP_SUCCESS;
  }
  memset(d->ints[b], 0, sizeof(d->ints[b]));
  if (nints) memcpy(d->ints[b], ints, (size_t)nints * sizeof(int32_t));
  d->n[b] = n;
  atomic_thread_fence(memory_order_release);
  int rc;
  if (n && (rc = mspi_d2d_async(m->dctx, slot_buf(m->dslots, m, dir, b), v->d + off, (size_t)n * sizeof(double)))) {
    atomic_store_explicit(&d->claim, P, memory_order_seq_cst);
    return rc;
  }
  if (same_stream(m, dst)) atomic_store_explicit(&d->pub, W, memory_order_seq_cst);
  else if ((rc = mspi_stream_store_u64(m->dctx, (uint64_t *)&dstate_dev(m, m->rank, dir)->pub, W))) return rc;
  m->sent++;
  return MSP_SUCCESS;
}

static int recv_vec_device(msp_amsg *m, int src, int32_t *ints, int32_t nints, msp_vec *v, int64_t voff, int64_t cap,
                           int64_t *n, int32_t *got) {
  *got = 0;
  double *ps = NULL;
  int rc = peer_slots(m, src, &ps);
  if (rc) return rc;
  if (!ps) return MSP_SUCCESS; /* src has not enabled its slots: nothing sent yet */
  const int dir = m->rank == src - 1 ? 0 : 1; /* src's direction towards this rank */
  dslot_state *d = dstate(m, src, dir);
  uint64_t *seen = m->seen + (size_t)src * MSP_AMSG_NKINDS + MSP_AMSG_DATA;
  const uint64_t P = atomic_load_explicit(&d->pub, memory_order_seq_cst);
  if (!P || P == *seen) return MSP_SUCCESS; /* nothing newer than the last plane taken */
  const int b = (int)(P & 1);
  atomic_store_explicit(&d->reading[b], 1, memory_order_seq_cst);
  if (atomic_load_explicit(&d->pub, memory_order_seq_cst) != P) { /* a newer one landed: take it next time */
    atomic_store_explicit(&d->reading[b], 0, memory_order_seq_cst);
    return MSP_SUCCESS;
  }
  int32_t tmp[AMSG_INTS];
  memcpy(tmp, d->ints[b], sizeof(tmp));
  const int64_t len = d->n[b];
  if (len < 0 || len > m->data_cap || len > cap) {
    atomic_store_explicit(&d->reading[b], 0, memory_order_seq_cst);
    return aerr(MSP_ERR_ARG_SIZ, "receive buffer smaller than the message");
  }
  if (len && (rc = mspi_d2d_async(m->dctx, v->d + voff, slot_buf(ps, m, dir, b), (size_t)len * sizeof(double)))) {
    atomic_store_explicit(&d->reading[b], 0, memory_order_seq_cst);
    return rc;
  }
  if (same_stream(m, src)) atomic_store_explicit(&d->reading[b], 0, memory_order_seq_cst);
  else if ((rc = mspi_stream_store_u32(m->dctx, (uint32_t *)&dstate_dev(m, src, dir)->reading[b], 0))) return rc;
  if (nints) memcpy(ints, tmp, (size_t)nints * sizeof(int32_t));
  if (n) *n = len;
  *seen = P;
  *got = 1;
  return MSP_SUCCESS;
}

int msp_amsg_send_vec(msp_amsg *m, int32_t dst, const int32_t *ints, int32_t nints, const msp_vec *v, int64_t off,
                      int64_t n) {
  if (!m || !v) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  int rc = check_pair(m, dst, MSP_AMSG_DATA);
  if (rc) return rc;
  if (nints < 0 || nints > AMSG_INTS || (nints && !ints)) return aerr(MSP_ERR_ARG_SIZ, "at most 6 ints per message");
  if (off < 0 || n < 0 || off + n > v->n || n > m->data_cap) return aerr(MSP_ERR_ARG_OUTOFRANGE, "range");
  ctrl_slot *s = data_at(m, m->rank, dst);
  if (!s) return aerr(MSP_ERR_ARG_WRONG, "iterate data only travels between chain neighbours");
  if (m->dctx) { /* a plane of another context: its producer done before the copy, the copy before its next use */
    if (v->ctx != m->dctx && (rc = msp_ctx_synchronize(v->ctx))) return rc;
    rc = send_vec_device(m, dst, ints, nints, v, off, n);
    return !rc && v->ctx != m->dctx ? msp_ctx_synchronize(m->dctx) : rc;
  }
  if ((rc = ensure_registered(m))) return rc;
  write_begin(s);
  memset(s->ints, 0, sizeof(s->ints));
  if (nints) memcpy(s->ints, ints, (size_t)nints * sizeof(int32_t));
  s->n = n;
  if (n && (rc = mspi_d2h_sync(v->ctx, (double *)(s + 1), v->d + off, (size_t)n * sizeof(double)))) {
    s->n = 0; /* publish an empty message rather than a partial plane */
    write_end(s);
    return rc;
  }
  write_end(s);
  return MSP_SUCCESS;
}

int msp_amsg_recv_vec(msp_amsg *m, int32_t src, int32_t *ints, int32_t nints, msp_vec *v, int64_t off, int64_t cap,
                      int64_t *n, int32_t *got) {
  if (!m || !v || !got) return aerr(MSP_ERR_ARG_NULL, "NULL argument");
  int rc = check_pair(m, src, MSP_AMSG_DATA);
  if (rc) return rc;
  if (nints < 0 || nints > AMSG_INTS || (nints && !ints)) return aerr(MSP_ERR_ARG_SIZ, "at most 6 ints per message");
  if (off < 0 || cap < 0 || off + cap > v->n) return aerr(MSP_ERR_ARG_OUTOFRANGE, "range");
  if (!data_at(m, src, m->rank)) return aerr(MSP_ERR_ARG_WRONG, "iterate data only travels between chain neighbours");
  if (m->dctx) {
    if (v->ctx != m->dctx && (rc = msp_ctx_synchronize(v->ctx))) return rc;
    rc = recv_vec_device(m, src, ints, nints, v, off, cap, n, got);
    return !rc && v->ctx != m->dctx ? msp_ctx_synchronize(m->dctx) : rc;
  }
  if ((rc = ensure_registered(m))) return rc;
  return read_slot(m, src, MSP_AMSG_DATA, ints, nints, NULL, cap, n, got, v, off);
}
