/*
 * abcast.c -- newest-value broadcast of each block's rows of R between the
 * blocks of an asynchronous run with global minimization, in POSIX shared
 * memory (one node, one process -- or one host thread -- per GPU).
 *
 * Replaces comm_async_test_and_send_min / comm_async_probe_and_receive_min
 * (src/utils/comm.c:288-351) as AMAM-global uses them
 * (asynchronous-multisplitting-asynchronous-minimization-global_prime.c:422-428):
 *   - the sender MPI_Isends its rows of R, unless its previous send has not
 *     completed (MPI_Test), in which case this round sends nothing;
 *   - the receiver drains every pending message and copies the newest into
 *     its replicated R, or keeps what it had (zeros before the first one).
 * Each source has two buffers.  A publish fills the one that is not the
 * newest and then makes it the newest; a fetch copies the newest one out.
 * Per buffer, a reader-count / writer-bit word admits either readers or the
 * writer, never both, so a fetch never sees a half-written R and a publish
 * that would overwrite a buffer still being read is skipped -- the reference's
 * "previous send not complete".  Payloads move HBM <-> the registered region
 * by DMA, or, with device buffers enabled (msp_abcast_enable_device), stay in
 * the sender's HBM (HIP IPC): a publish is one HBM -> HBM copy, a fetch one
 * peer copy over xGMI.
 *
 * Device buffers never wait on the host (the R rows of configs[3] are 21.5 GB
 * per block).  A publish claims the buffer that is not the newest (the only
 * one with a single buffer), enqueues the copy into it and, behind the copy on
 * the sender's stream, a one-lane kernel that publishes (count, buffer) into
 * the source's shared word `pub`.  A fetch marks the newest buffer as being
 * read by this rank, enqueues the peer copy out of it, and its stream clears
 * the mark behind the copy.  Claim and mark are Dekker's handshake (each side
 * stores its word, then loads the other's), so a buffer is never written while
 * a reader's pending copy reads it: a publish whose previous copy is still
 * unpublished, or whose buffer a reader still holds, is skipped -- the
 * reference's MPI_Test of the previous Isend (comm.c:288-351).  Ranks of one
 * process on one stream (round-robin) publish and release at once: stream
 * order already serialises their copies (as amsg.c's planes).
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

#define ABC_MAGIC 0x4d53504142434153ULL /* "MSPABCAS" */
#define ABC_WRITER 0x80000000u

typedef struct {
  _Atomic int32_t newest;   /* buffer index of the newest complete payload, -1 before the first */
  int32_t pad0;
  _Atomic uint32_t lock[2]; /* ABC_WRITER | reader count */
  uint64_t version[2];      /* publish number of the payload each buffer holds */
  int64_t nrows[2], ncols[2];
  uint64_t published;       /* publishes so far (written by the source only) */
  uint8_t pad[128 - 8 - 8 - 16 - 32 - 8];
} src_line;

typedef struct {
  uint64_t magic;
  int32_t nranks;
  int32_t pad0;
  int64_t cap;
  uint8_t pad[64 - 24];
} abc_header;

typedef struct {
  _Atomic int32_t ready;
  int32_t pid;
  uint64_t rawptr; /* valid in the exporting process only */
  uint64_t stream; /* the exporting context's stream (same process and stream: copies ordered by the stream) */
  uint8_t handle[MSPI_IPC_HANDLE_BYTES];
  uint8_t pad[128 - 24 - MSPI_IPC_HANDLE_BYTES];
} abc_ipc;

/* device-buffer state of one source, in the shared region (GPU-written words: pub, reading) */
typedef struct {
  _Atomic uint64_t pub;   /* (count << 1) | buffer of the newest complete payload; 0: none yet */
  _Atomic uint64_t claim; /* (count << 1) | buffer of the source's latest publish; == pub: nothing in flight */
  int64_t nrows[2], ncols[2];
  int32_t nbuf;           /* the source's device buffers (1 or 2) */
  uint8_t pad[128 - 16 - 32 - 4];
} abc_dline;

#define ABC_MAX_DEVICE_RANKS 512 /* the reading words are nranks x 2 x nranks */

struct msp_abcast {
  char name[128];
  int32_t nranks, rank, owner;
  int64_t cap;
  size_t bytes, buf_bytes;
  uint8_t *base;
  src_line *lines;
  uint8_t *bufs;   /* [src][2] buffers of cap doubles */
  uint64_t *seen;  /* [src] version last fetched */
  int registered;
  abc_ipc *ipc;    /* [rank] exported device buffers */
  abc_dline *dl;   /* [src] device-buffer state */
  _Atomic uint32_t *reading;  /* [src][buffer][reader]: reader's copy out of src's buffer pending */
  uint8_t *dstate_dev;        /* the same region as the GPU addresses it (dl first) */
  size_t dstate_off;          /* offset of dl in the region */
  uint64_t skey;              /* this rank's stream */
  int dregistered;            /* the device-state part (dl, reading) is registered */
  uint64_t *dseen; /* [src] the pub word of the last payload fetched (device buffers) */
  int64_t sent, skipped;      /* device publishes enqueued / skipped */
  msp_ctx *dctx;   /* device buffers enabled */
  double *dbufs;   /* this rank's nbuf_dev x cap device buffers */
  int nbuf_dev;    /* 2, or 1 where HBM is short: a publish then waits out the readers of the newest block */
  double **peer;   /* [src] resolved device buffers */
  uint8_t *opened; /* [src] came from hipIpcOpenMemHandle */
};

static int berr(int code, const char *msg) {
  mspi_set_error(code, "%s", msg);
  return code;
}

static size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static int ensure_registered(msp_abcast *b);

static double *buf_at(msp_abcast *b, int src, int k) {
  return (double *)(b->bufs + ((size_t)src * 2 + (size_t)k) * b->buf_bytes);
}

int msp_abcast_create(const char *name, int32_t nranks, int32_t rank, int64_t cap, int32_t owner, msp_abcast **out) {
  if (!name || !out) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  if (nranks < 1 || nranks > 4096 || rank < 0 || rank >= nranks || cap < 0)
    return berr(MSP_ERR_ARG_OUTOFRANGE, "bad abcast sizes");
  if (strlen(name) >= sizeof(((msp_abcast *)0)->name) || name[0] != '/')
    return berr(MSP_ERR_ARG_WRONG, "shared-memory name must start with '/' and be < 128 chars");
  msp_abcast *b = (msp_abcast *)calloc(1, sizeof(msp_abcast));
  if (!b) return berr(MSP_ERR_MEM, "allocation failed");
  strcpy(b->name, name);
  b->nranks = nranks;
  b->rank = rank;
  b->owner = owner ? 1 : 0;
  b->cap = cap;
  b->buf_bytes = round_up((size_t)(cap > 0 ? cap : 1) * sizeof(double), 4096);
  const size_t lines_bytes = round_up((size_t)nranks * sizeof(src_line), 4096);
  const size_t ipc_bytes = round_up((size_t)nranks * sizeof(abc_ipc), 4096);
  const size_t dl_bytes = round_up((size_t)nranks * sizeof(abc_dline), 4096);
  const size_t rd_bytes =
      nranks <= ABC_MAX_DEVICE_RANKS ? round_up((size_t)nranks * 2 * (size_t)nranks * sizeof(uint32_t), 4096) : 0;
  b->dstate_off = 4096 + lines_bytes + (size_t)nranks * 2 * b->buf_bytes + ipc_bytes;
  b->bytes = b->dstate_off + dl_bytes + rd_bytes;
  int fd;
  if (b->owner) {
    shm_unlink(name);
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0 && ftruncate(fd, (off_t)b->bytes) != 0) {
      close(fd);
      fd = -1;
    }
  } else {
    fd = shm_open(name, O_RDWR, 0600);
  }
  if (fd < 0) {
    free(b);
    mspi_set_error(MSP_ERR_LIB, "shm_open(%s) failed: %s", name, strerror(errno));
    return MSP_ERR_LIB;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < b->bytes) {
    close(fd);
    free(b);
    return berr(MSP_ERR_ARG_SIZ, "shared-memory region smaller than the layout (sizes differ between ranks?)");
  }
  b->base = (uint8_t *)mmap(NULL, b->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (b->base == MAP_FAILED) {
    free(b);
    return berr(MSP_ERR_MEM, "mmap of the shared-memory region failed");
  }
  abc_header *h = (abc_header *)b->base;
  b->lines = (src_line *)(b->base + 4096);
  b->bufs = b->base + 4096 + lines_bytes;
  b->ipc = (abc_ipc *)(b->bufs + (size_t)nranks * 2 * b->buf_bytes);
  b->dl = (abc_dline *)(b->base + b->dstate_off);
  b->reading = rd_bytes ? (_Atomic uint32_t *)((uint8_t *)b->dl + dl_bytes) : NULL;
  if (b->owner) {
    h->nranks = nranks;
    h->cap = cap;
    for (int r = 0; r < nranks; ++r) atomic_store_explicit(&b->lines[r].newest, -1, memory_order_relaxed);
    atomic_thread_fence(memory_order_release);
    h->magic = ABC_MAGIC;
  } else if (h->magic != ABC_MAGIC || h->nranks != nranks || h->cap != cap) {
    munmap(b->base, b->bytes);
    free(b);
    return berr(MSP_ERR_ARG_WRONG, "shared-memory region not initialised by the owner, or different sizes");
  }
  b->seen = (uint64_t *)calloc((size_t)nranks, sizeof(uint64_t));
  b->dseen = (uint64_t *)calloc((size_t)nranks, sizeof(uint64_t));
  if (!b->seen || !b->dseen) {
    free(b->seen);
    free(b->dseen);
    munmap(b->base, b->bytes);
    free(b);
    return berr(MSP_ERR_MEM, "allocation failed");
  }
  *out = b;
  return MSP_SUCCESS;
}

int msp_abcast_enable_device(msp_abcast *b, msp_ctx *ctx, int32_t nbuf) {
  if (!b || !ctx) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  if (nbuf < 0 || nbuf > 2) return berr(MSP_ERR_ARG_OUTOFRANGE, "nbuf must be 0 (auto), 1 or 2");
  if (b->dctx) return MSP_SUCCESS;
  if (!b->reading) return berr(MSP_ERR_SUP, "device buffers take at most 512 ranks");
  const size_t buf_bytes = (size_t)(b->cap > 0 ? b->cap : 1) * sizeof(double);
  if (nbuf == 0) {
    /* auto: two buffers only while a quarter of the GPU's HBM stays free after them -- the run allocates more
     * afterwards (configs[3]'s replicated-R rank: 100 GB free here, 24 GB of peer blocks and the LSQR's work
     * still to come; one 21.5 GB buffer instead of two: DESIGN.md section 6.5) */
    size_t fr = 0, tot = 0;
    int rc = mspi_mem_info(ctx, &fr, &tot);
    if (rc) return rc;
    nbuf = fr >= 2 * buf_bytes && fr - 2 * buf_bytes >= tot / 4 ? 2 : 1;
  }
  b->peer = (double **)calloc((size_t)b->nranks, sizeof(double *));
  b->opened = (uint8_t *)calloc((size_t)b->nranks, 1);
  if (!b->peer || !b->opened) return berr(MSP_ERR_MEM, "allocation failed");
  /* the streams publish and release through the state words: that part of the region (page aligned, a few KiB)
   * is mapped for the GPU -- never the host-staged payload buffers before it, which are nranks x 2 x cap doubles
   * of untouched sparse memory (a configs[3] rank: 344 GB) that registering would pin */
  const size_t dbytes = b->bytes - b->dstate_off;
  int rc = mspi_host_register(b->dl, dbytes);
  if (rc) return rc;
  b->dregistered = 1;
  void *dp = NULL;
  if ((rc = mspi_host_device_ptr(b->dl, &dp))) return rc;
  b->dstate_dev = (uint8_t *)dp;
  void *p = NULL;
  rc = mspi_dev_alloc(ctx, (size_t)nbuf * buf_bytes, &p);
  if (rc) return rc;
  b->nbuf_dev = nbuf;
  abc_ipc *e = &b->ipc[b->rank];
  if ((rc = mspi_ipc_export(p, e->handle))) {
    mspi_dev_free(p);
    return rc;
  }
  b->dbufs = (double *)p;
  b->dctx = ctx;
  b->skey = mspi_stream_key(ctx);
  mspi_ctx_retain(ctx);
  b->dl[b->rank].nbuf = nbuf;
  e->pid = (int32_t)getpid();
  e->rawptr = (uint64_t)(uintptr_t)p;
  e->stream = b->skey;
  atomic_store_explicit(&e->ready, 1, memory_order_release);
  return MSP_SUCCESS;
}

int msp_abcast_get_stats(const msp_abcast *b, int64_t *sent, int64_t *skipped) {
  if (!b) return berr(MSP_ERR_ARG_NULL, "abcast is NULL");
  if (sent) *sent = b->sent;
  if (skipped) *skipped = b->skipped;
  return MSP_SUCCESS;
}

int msp_abcast_get_nbuf(const msp_abcast *b, int32_t *nbuf) {
  if (!b || !nbuf) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  *nbuf = b->dctx ? b->nbuf_dev : 0;
  return MSP_SUCCESS;
}

int msp_abcast_close_peers(msp_abcast *b) {
  if (!b) return berr(MSP_ERR_ARG_NULL, "abcast is NULL");
  if (!b->peer) return MSP_SUCCESS;
  /* this rank's copies out of the peers' buffers, and its publish / release stores, are stream-ordered: let them
   * finish before the mappings go */
  if (b->dctx) {
    int rc = msp_ctx_synchronize(b->dctx);
    if (rc) return rc;
  }
  for (int r = 0; r < b->nranks; ++r) {
    if (b->opened[r]) mspi_ipc_close(b->peer[r]);
    b->peer[r] = NULL;
    b->opened[r] = 0;
  }
  return MSP_SUCCESS;
}

/* comm_discard_pending_messages (comm.c:426-453) for the R rows and the MPI_Cancel of
 * send_minimization_data_request (AMAM-global_prime.c:522-572): every source's block newer than the last one taken
 * is marked taken without being copied; this rank's own publish whose copy is enqueued but not yet published is
 * counted and completed by draining the stream (a DMA cannot be withdrawn). */
int msp_abcast_discard_pending(msp_abcast *b, int64_t *discarded, int64_t *in_flight) {
  if (!b) return berr(MSP_ERR_ARG_NULL, "abcast is NULL");
  int64_t nd = 0, nf = 0;
  for (int src = 0; src < b->nranks; ++src) {
    if (src == b->rank) continue;
    if (b->dctx) {
      const uint64_t P = atomic_load_explicit(&b->dl[src].pub, memory_order_seq_cst);
      if (P && P != b->dseen[src]) {
        b->dseen[src] = P;
        ++nd;
      }
      continue;
    }
    src_line *L = &b->lines[src];
    const int32_t k = atomic_load_explicit(&L->newest, memory_order_acquire);
    if (k >= 0 && L->version[k] != b->seen[src]) {
      b->seen[src] = L->version[k];
      ++nd;
    }
  }
  if (b->dctx) {
    abc_dline *d = &b->dl[b->rank];
    if (atomic_load_explicit(&d->claim, memory_order_seq_cst) != atomic_load_explicit(&d->pub, memory_order_seq_cst))
      ++nf;
    int rc = msp_ctx_synchronize(b->dctx);
    if (rc) return rc;
  }
  if (discarded) *discarded = nd;
  if (in_flight) *in_flight = nf;
  return MSP_SUCCESS;
}

static int peer_bufs(msp_abcast *b, int src, double **out) {
  *out = b->peer[src];
  if (*out) return MSP_SUCCESS;
  abc_ipc *e = &b->ipc[src];
  if (!atomic_load_explicit(&e->ready, memory_order_acquire)) return MSP_SUCCESS;
  if (e->pid == (int32_t)getpid()) {
    b->peer[src] = (double *)(uintptr_t)e->rawptr;
  } else {
    void *p = NULL;
    int rc = mspi_ipc_open(b->dctx, e->handle, &p);
    if (rc) return rc;
    b->peer[src] = (double *)p;
    b->opened[src] = 1;
  }
  *out = b->peer[src];
  return MSP_SUCCESS;
}

int msp_abcast_destroy(msp_abcast **pb) {
  if (!pb || !*pb) return MSP_SUCCESS;
  msp_abcast *b = *pb;
  msp_abcast_close_peers(b);
  if (b->dbufs) {
    atomic_store_explicit(&b->ipc[b->rank].ready, 0, memory_order_release);
    mspi_dev_free(b->dbufs);
  }
  free(b->peer);
  free(b->opened);
  if (b->registered) mspi_host_unregister(b->base);
  if (b->dregistered) mspi_host_unregister(b->dl);
  munmap(b->base, b->bytes);
  if (b->owner) shm_unlink(b->name);
  free(b->seen);
  free(b->dseen);
  msp_ctx *c = b->dctx;
  free(b);
  *pb = NULL;
  mspi_ctx_release(c);
  return MSP_SUCCESS;
}

static int ensure_registered(msp_abcast *b) {
  if (b->registered) return MSP_SUCCESS;
  int rc = mspi_host_register(b->base, b->bytes);
  if (rc) return rc;
  b->registered = 1;
  return MSP_SUCCESS;
}

/* one payload of nrows x ncols, column j at src + j*ld, either in HBM (ctx != NULL) or host memory */
typedef struct {
  msp_ctx *ctx;
  double *p;
  int64_t nrows, ld;
  int32_t ncols;
} abc_view;

static int copy_out(const abc_view *v, double *dst) {
  int rc = MSP_SUCCESS;
  for (int32_t j = 0; j < v->ncols && !rc; ++j) {
    const double *col = v->p + (size_t)j * v->ld;
    double *d = dst + (size_t)j * v->nrows;
    if (v->ctx) rc = mspi_d2h_sync(v->ctx, d, col, (size_t)v->nrows * sizeof(double));
    else memcpy(d, col, (size_t)v->nrows * sizeof(double));
  }
  return rc;
}

static int copy_in(const abc_view *v, const double *srcp) {
  int rc = MSP_SUCCESS;
  for (int32_t j = 0; j < v->ncols && !rc; ++j) {
    double *col = v->p + (size_t)j * v->ld;
    const double *s = srcp + (size_t)j * v->nrows;
    if (v->ctx) rc = mspi_h2d_sync(v->ctx, col, s, (size_t)v->nrows * sizeof(double));
    else memcpy(col, s, (size_t)v->nrows * sizeof(double));
  }
  return rc;
}

/* ------------------------------------------------------------ device buffers */
static _Atomic uint32_t *reading_at(msp_abcast *b, int src, int k, int reader) {
  return b->reading + ((size_t)src * 2 + (size_t)k) * (size_t)b->nranks + (size_t)reader;
}

static uint8_t *dev_addr(msp_abcast *b, const void *host_word) {
  return b->dstate_dev + ((const uint8_t *)host_word - (const uint8_t *)b->dl);
}

/* peer's buffers driven by this very stream (the blocks of one process): stream order serialises every copy */
static int same_stream(msp_abcast *b, int peer) {
  abc_ipc *e = &b->ipc[peer];
  return atomic_load_explicit(&e->ready, memory_order_acquire) && e->pid == (int32_t)getpid() && e->stream == b->skey;
}

static int all_same_stream(msp_abcast *b) {
  for (int r = 0; r < b->nranks; ++r)
    if (r != b->rank && !same_stream(b, r)) return 0;
  return 1;
}

static int publish_device(msp_abcast *b, const abc_view *v, int32_t *published) {
  abc_dline *d = &b->dl[b->rank];
  const uint64_t P = atomic_load_explicit(&d->pub, memory_order_seq_cst);
  if (atomic_load_explicit(&d->claim, memory_order_relaxed) != P) { /* the previous copy is not published yet */
    b->skipped++;
    return MSP_SUCCESS;
  }
  const int k = b->nbuf_dev == 1 ? 0 : (P ? 1 - (int)(P & 1) : 0); /* the buffer that is not the newest */
  const uint64_t W = (((P >> 1) + 1) << 1) | (uint64_t)k;
  atomic_store_explicit(&d->claim, W, memory_order_seq_cst);
  for (int r = 0; r < b->nranks; ++r)
    if (r != b->rank && atomic_load_explicit(reading_at(b, b->rank, k, r), memory_order_seq_cst)) {
      atomic_store_explicit(&d->claim, P, memory_order_seq_cst); /* a reader still copies out of it */
      b->skipped++;
      return MSP_SUCCESS;
    }
  d->nrows[k] = v->nrows;
  d->ncols[k] = v->ncols;
  atomic_thread_fence(memory_order_release);
  const size_t rowb = (size_t)v->nrows * sizeof(double);
  int rc = mspi_d2d_async2d(b->dctx, b->dbufs + (size_t)k * (size_t)b->cap, rowb, v->p, (size_t)v->ld * sizeof(double),
                            rowb, (size_t)v->ncols);
  if (rc) {
    atomic_store_explicit(&d->claim, P, memory_order_seq_cst);
    return rc;
  }
  if (all_same_stream(b)) atomic_store_explicit(&d->pub, W, memory_order_seq_cst);
  else if ((rc = mspi_stream_store_u64(b->dctx, (uint64_t *)dev_addr(b, &d->pub), W))) return rc;
  b->sent++;
  *published = 1;
  return MSP_SUCCESS;
}

static int fetch_device(msp_abcast *b, int32_t src, const abc_view *v, int32_t *got) {
  double *pbuf = NULL;
  int rc = peer_bufs(b, src, &pbuf);
  if (rc) return rc;
  if (!pbuf) return MSP_SUCCESS; /* src has not enabled its buffers: nothing sent yet */
  abc_dline *d = &b->dl[src];
  const int one = d->nbuf == 1; /* one buffer: the source rewrites the newest itself */
  const uint64_t P = atomic_load_explicit(&d->pub, memory_order_seq_cst);
  if (!P || P == b->dseen[src]) return MSP_SUCCESS; /* nothing newer than the last block taken */
  if (one && atomic_load_explicit(&d->claim, memory_order_seq_cst) != P) return MSP_SUCCESS; /* being rewritten */
  const int k = (int)(P & 1);
  _Atomic uint32_t *mark = reading_at(b, src, k, b->rank);
  atomic_store_explicit(mark, 1u, memory_order_seq_cst);
  if (atomic_load_explicit(&d->pub, memory_order_seq_cst) != P ||
      (one && atomic_load_explicit(&d->claim, memory_order_seq_cst) != P)) { /* moved on: take it next time */
    atomic_store_explicit(mark, 0u, memory_order_seq_cst);
    return MSP_SUCCESS;
  }
  if (d->nrows[k] != v->nrows || d->ncols[k] != v->ncols) {
    atomic_store_explicit(mark, 0u, memory_order_seq_cst);
    return berr(MSP_ERR_ARG_SIZ, "received block has a different shape");
  }
  const size_t rowb = (size_t)v->nrows * sizeof(double);
  if ((rc = mspi_d2d_async2d(b->dctx, v->p, (size_t)v->ld * sizeof(double), pbuf + (size_t)k * (size_t)b->cap, rowb,
                             rowb, (size_t)v->ncols))) {
    atomic_store_explicit(mark, 0u, memory_order_seq_cst);
    return rc;
  }
  if (same_stream(b, src)) atomic_store_explicit(mark, 0u, memory_order_seq_cst);
  else if ((rc = mspi_stream_store_u32(b->dctx, (uint32_t *)dev_addr(b, (const void *)mark), 0u))) return rc;
  b->dseen[src] = P;
  *got = 1;
  return MSP_SUCCESS;
}

/* ------------------------------------------------------------ publish / fetch */
/* A dense block of another context (another stream) than the one the device buffers' copies run on: its producer's
 * work is finished before the copy is enqueued, and the copy before the caller's stream can touch the block again
 * (same context: stream order does both). */
static int fence_in(const msp_abcast *b, const abc_view *v) {
  return v->ctx != b->dctx ? msp_ctx_synchronize(v->ctx) : MSP_SUCCESS;
}

static int fence_out(const msp_abcast *b, const abc_view *v, int rc) {
  return !rc && v->ctx != b->dctx ? msp_ctx_synchronize(b->dctx) : rc;
}

static int publish(msp_abcast *b, const abc_view *v, int32_t *published) {
  *published = 0;
  if (b->dctx && !v->ctx) return berr(MSP_ERR_ARG_WRONG, "device buffers enabled: publish a dense block in HBM");
  if (v->nrows < 0 || v->ncols < 0 || v->ld < v->nrows || (v->nrows > 0 && v->ncols > 0 && !v->p))
    return berr(MSP_ERR_ARG_WRONG, "bad payload shape");
  if (v->nrows * (int64_t)v->ncols > b->cap) return berr(MSP_ERR_ARG_SIZ, "payload larger than the broadcast slot");
  int rc;
  if (b->dctx) {
    rc = fence_in(b, v);
    return rc ? rc : fence_out(b, v, publish_device(b, v, published));
  }
  rc = v->ctx ? ensure_registered(b) : MSP_SUCCESS;
  if (rc) return rc;
  src_line *L = &b->lines[b->rank];
  const int32_t newest = atomic_load_explicit(&L->newest, memory_order_acquire);
  const int w = newest == 0 ? 1 : 0; /* the buffer that is not the newest */
  uint32_t expect = 0;
  if (!atomic_compare_exchange_strong_explicit(&L->lock[w], &expect, ABC_WRITER, memory_order_acq_rel,
                                               memory_order_relaxed))
    return MSP_SUCCESS; /* a reader still holds it: the previous send has not completed */
  rc = copy_out(v, buf_at(b, b->rank, w));
  if (rc) {
    atomic_store_explicit(&L->lock[w], 0u, memory_order_release);
    return rc;
  }
  L->nrows[w] = v->nrows;
  L->ncols[w] = v->ncols;
  L->version[w] = ++L->published;
  atomic_store_explicit(&L->lock[w], 0u, memory_order_release);
  atomic_store_explicit(&L->newest, w, memory_order_release);
  *published = 1;
  return MSP_SUCCESS;
}

static int fetch(msp_abcast *b, int32_t src, const abc_view *v, int32_t *got) {
  *got = 0;
  if (b->dctx && !v->ctx) return berr(MSP_ERR_ARG_WRONG, "device buffers enabled: fetch into a dense block in HBM");
  if (src < 0 || src >= b->nranks || src == b->rank) return berr(MSP_ERR_ARG_OUTOFRANGE, "source rank out of range");
  if (v->nrows < 0 || v->ncols < 0 || v->ld < v->nrows || (v->nrows > 0 && v->ncols > 0 && !v->p))
    return berr(MSP_ERR_ARG_WRONG, "bad payload shape");
  int rc;
  if (b->dctx) {
    rc = fence_in(b, v);
    return rc ? rc : fence_out(b, v, fetch_device(b, src, v, got));
  }
  rc = v->ctx ? ensure_registered(b) : MSP_SUCCESS;
  if (rc) return rc;
  src_line *L = &b->lines[src];
  for (int attempt = 0; attempt < 64; ++attempt) {
    const int32_t k = atomic_load_explicit(&L->newest, memory_order_acquire);
    if (k < 0) return MSP_SUCCESS; /* nothing sent yet */
    uint32_t cur = atomic_load_explicit(&L->lock[k], memory_order_relaxed);
    if (cur & ABC_WRITER) continue; /* the source moved on and is refilling it: look again */
    if (!atomic_compare_exchange_weak_explicit(&L->lock[k], &cur, cur + 1, memory_order_acq_rel, memory_order_relaxed))
      continue;
    const uint64_t ver = L->version[k];
    if (ver == b->seen[src]) {
      atomic_fetch_sub_explicit(&L->lock[k], 1u, memory_order_release);
      return MSP_SUCCESS; /* nothing newer */
    }
    if (L->nrows[k] != v->nrows || L->ncols[k] != v->ncols) {
      atomic_fetch_sub_explicit(&L->lock[k], 1u, memory_order_release);
      return berr(MSP_ERR_ARG_SIZ, "received block has a different shape");
    }
    rc = copy_in(v, buf_at(b, src, k));
    atomic_fetch_sub_explicit(&L->lock[k], 1u, memory_order_release);
    if (rc) return rc;
    b->seen[src] = ver;
    *got = 1;
    return MSP_SUCCESS;
  }
  return MSP_SUCCESS; /* the source kept refilling: try next round */
}

int msp_abcast_publish(msp_abcast *b, const double *data, int64_t nrows, int32_t ncols, int64_t ld,
                       int32_t *published) {
  if (!b || !published) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  const abc_view v = {NULL, (double *)data, nrows, ld, ncols};
  return publish(b, &v, published);
}

int msp_abcast_fetch(msp_abcast *b, int32_t src, double *data, int64_t nrows, int32_t ncols, int64_t ld,
                     int32_t *got) {
  if (!b || !got) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  const abc_view v = {NULL, data, nrows, ld, ncols};
  return fetch(b, src, &v, got);
}

int msp_abcast_publish_dense(msp_abcast *b, const msp_dense *D, int32_t *published) {
  if (!b || !D || !published) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  const abc_view v = {D->ctx, D->d, D->nrows, D->lda, D->ncols};
  return publish(b, &v, published);
}

int msp_abcast_fetch_dense(msp_abcast *b, int32_t src, msp_dense *D, int32_t *got) {
  if (!b || !D || !got) return berr(MSP_ERR_ARG_NULL, "NULL argument");
  const abc_view v = {D->ctx, D->d, D->nrows, D->lda, D->ncols};
  return fetch(b, src, &v, got);
}
