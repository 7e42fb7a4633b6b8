/*
 * msplit_drivers.h -- the reference's multisplitting drivers as a C host over
 * the C ABI (include/msplit.h): the host side in the reference's own language.
 *
 *   synchronous-multisplitting                       (synchronous-multisplitting.c:155-206)
 *   synchronous-multisplitting-synchronous-minimization-global   (SMSM-global.c:288-363)
 *   asynchronous-multisplitting                      (asynchronous-multisplitting_prime.c:333-427)
 *   asynchronous-multisplitting-asynchronous-minimization-global  (AMAM-global_prime.c:238-481;
 *                                                     configs[3] / configs[4]'s algorithm)
 *
 * One block per MPI rank (one GPU each; RCCL or MPI all-gathers through
 * msp_comm), or every block in one process (nb blocks, round-robin on one GPU).
 * Each block's arithmetic goes through the same library calls, in the same
 * order, as the Python host (medane_tchakorom_ufc_thesis_repository_amd/
 * multisplitting.py, asynchronous.py), so the two hosts agree bit for bit.
 */
#ifndef MSPLIT_DRIVERS_H
#define MSPLIT_DRIVERS_H

#include <stdint.h>

#include "msplit.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- options database (PetscOptionsGet* over argv) ---- */
typedef struct msd_options msd_options;
msd_options *msd_options_parse(int argc, char **argv); /* argv[0] is skipped */
void msd_options_free(msd_options *o);
int msd_opt_has(const msd_options *o, const char *prefix, const char *key);
const char *msd_opt_str(const msd_options *o, const char *prefix, const char *key, const char *dflt);
int64_t msd_opt_int(const msd_options *o, const char *prefix, const char *key, int64_t dflt);
double msd_opt_real(const msd_options *o, const char *prefix, const char *key, double dflt);

/* ---- the block partition (utils.py block_layout) ---- */
typedef struct {
  int dim, nb, b;
  int32_t nx, ny, nz;  /* 3D: nx x ny x nz; 2D: nx = mesh lines, ny = mesh columns */
  int64_t r0, r1, plane;
  int has_lo, has_hi;  /* neighbour below (b-1) / above (b+1) */
  int64_t halo_size;   /* [plane of b-1 | plane of b+1] */
  int32_t box[4];      /* dim, fast, middle, slow extents of A_ii's box stencil */
  double peclet[3];
} msd_layout;

int msd_layout_make(int dim, int32_t nx, int32_t ny, int32_t nz, int nb, int b, const double *peclet,
                    msd_layout *L);

/* ---- transport: all blocks local (world == 1) or one block per rank ---- */
typedef struct {
  int world, rank;
  msp_comm *comm;               /* world > 1: neighbour exchange, ordered sums, LSQR partials */
  void (*barrier)(void *user);  /* world > 1 */
  void (*bcast)(void *user, void *buf, int bytes, int root);
  void *user;
} msd_transport;

/* ---- results ---- */
#define MSD_HIST_CAP 4096
typedef struct {
  int outer_its;           /* SM / SMSM */
  double hist[MSD_HIST_CAP]; /* SM / SMSM: the stop test's norm of each outer iteration (first MSD_HIST_CAP) */
  int lsqr_its[MSD_HIST_CAP]; /* SMSM: the outer LSQR's iteration count of each outer iteration */
  int iterations[64];      /* AM: per local block */
  int states[64], tags[64]; /* AM: the detection's state and phase tag of each local block at the end */
  int64_t discarded[64];   /* AM: messages / R blocks discarded unread at shutdown (comm_discard_pending_messages) */
  int64_t in_flight[64];   /* AM: own sends still in flight at shutdown (the reference's MPI_Cancel), completed */
  int nlocal;
  double norm0, final_norm, error, elapsed;
  double last_norm;        /* the stop test's last value */
} msd_result;

typedef struct {
  int dim, nb;
  int32_t nx, ny, nz;
  int s;
  double rtol, atol, peclet[3];
  int max_outer;
  int matfree;             /* -msplit_operator matfree: A_ii without storage */
  int async_host;          /* -msplit_async_transport host: shared-memory staging instead of HBM slots */
  int rtr;                 /* -msplit_minimization rtr: AMAM-global through outer_solver's normal equations */
} msd_problem;

int msd_sm_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t, msd_result *r);
int msd_smsm_global_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t,
                          msd_result *r);
int msd_am_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t, msd_result *r);
int msd_amam_global_solve(msp_ctx *ctx, const msd_problem *p, const msd_options *o, const msd_transport *t,
                          msd_result *r);

#ifdef __cplusplus
}
#endif
#endif
