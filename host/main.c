/*
 * main.c -- the reference's multisplitting executables as a C host:
 *
 *   msplit_driver <program> -m M -n N [-s S] [-rtol R] [-atol A] [-dim 3 -p P]
 *                 [-peclet px,py,pz] [-nb B] [-json] [-inner{b}_ksp_* ...] [-outer{b}_ksp_* ...]
 *
 * <program>: synchronous-multisplitting,
 *            synchronous-multisplitting-synchronous-minimization-global,
 *            asynchronous-multisplitting,
 *            asynchronous-multisplitting-asynchronous-minimization-global.
 * Built with MPI (msplit_driver_mpi, MPICH): one block per rank, each rank on
 * GPU (rank mod devices); the neighbour exchange, ordered sums and LSQR
 * partials go through msp_comm -- RCCL (-msplit_transport rccl, the default)
 * or MPI_Allgather (-msplit_transport host).  Without MPI: -nb blocks in one
 * process, round-robin on GPU 0.  Output lines follow the reference
 * (printElapsedTime, printFinalResidualNorm, computeError; utils.c:665-730).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "msplit_drivers.h"

#ifdef MSD_MPI
#include <mpi.h>

static void mpi_barrier(void *u) {
  (void)u;
  MPI_Barrier(MPI_COMM_WORLD);
}

static void mpi_bcast(void *u, void *buf, int bytes, int root) {
  (void)u;
  MPI_Bcast(buf, bytes, MPI_BYTE, root, MPI_COMM_WORLD);
}

static int mpi_allgather(void *u, const double *send, double *recv, int64_t count) {
  (void)u;
  return MPI_Allgather(send, (int)count, MPI_DOUBLE, recv, (int)count, MPI_DOUBLE, MPI_COMM_WORLD) != MPI_SUCCESS;
}
#endif

static int usage(void) {
  fprintf(stderr, "usage: msplit_driver <synchronous-multisplitting | "
                  "synchronous-multisplitting-synchronous-minimization-global | asynchronous-multisplitting | "
                  "asynchronous-multisplitting-asynchronous-minimization-global> "
                  "-m M -n N [-s S] [-rtol R] [-dim 3 -p P] [-peclet px,py,pz] [-nb B] [-msplit_reduction dbr|seq] [-msplit_minimization lsqr|rtr] [-json] ...\n");
  return 2;
}

int main(int argc, char **argv) {
  int world = 1, rank = 0;
#ifdef MSD_MPI
  MPI_Init(&argc, &argv);
  MPI_Comm_size(MPI_COMM_WORLD, &world);
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
#endif
  if (argc < 2) return usage();
  const char *prog = argv[1];
  int kind;
  if (!strcmp(prog, "synchronous-multisplitting")) kind = 0;
  else if (!strcmp(prog, "synchronous-multisplitting-synchronous-minimization-global")) kind = 1;
  else if (!strcmp(prog, "asynchronous-multisplitting")) kind = 2;
  else if (!strcmp(prog, "asynchronous-multisplitting-asynchronous-minimization-global")) kind = 3;
  else return usage();
  msd_options *o = msd_options_parse(argc - 1, argv + 1);
  msd_problem p;
  memset(&p, 0, sizeof(p));
  p.dim = (int)msd_opt_int(o, NULL, "dim", 2);
  p.nx = (int32_t)msd_opt_int(o, NULL, "m", 256);
  p.ny = (int32_t)msd_opt_int(o, NULL, "n", 256);
  p.nz = p.dim == 3 ? (int32_t)msd_opt_int(o, NULL, "p", p.ny) : 1;
  p.s = (int)msd_opt_int(o, NULL, "s", 4);
  p.rtol = msd_opt_real(o, NULL, "rtol", 1e-6);
  p.atol = msd_opt_real(o, NULL, "atol", 1e-100);
  p.max_outer = (int)msd_opt_int(o, NULL, "max_outer", 100000);
  p.nb = world > 1 ? world : (int)msd_opt_int(o, NULL, "nb", 2);
  p.matfree = !strcmp(msd_opt_str(o, NULL, "msplit_operator", "csr"), "matfree");
  p.async_host = !strcmp(msd_opt_str(o, NULL, "msplit_async_transport", "device"), "host");
  const char *mini = msd_opt_str(o, NULL, "msplit_minimization", "lsqr");
  if (strcmp(mini, "lsqr") && strcmp(mini, "rtr")) return usage();
  p.rtr = !strcmp(mini, "rtr");
  const char *pe = msd_opt_str(o, NULL, "peclet", NULL);
  if (pe && sscanf(pe, "%lf,%lf,%lf", &p.peclet[0], &p.peclet[1], &p.peclet[2]) != 3) return usage();
  if (msd_opt_int(o, NULL, "npb", 1) != 1) {
    fprintf(stderr, "-npb must be 1: one GPU (one process) per block\n");
    return 2;
  }
  int ndev = 1;
  msp_get_device_count(&ndev);
  msp_ctx *ctx;
  if (msp_ctx_create(ndev > 0 ? rank % ndev : 0, NULL, &ctx)) {
    fprintf(stderr, "msp_ctx_create: %s\n", msp_get_last_error());
    return 1;
  }
  /* -msplit_reduction seq: every dot, norm and MDot in PETSc's Seq order (the parity mode,
   * msp_ctx_set_reduction): iteration counts and histories are the reference's bit for bit */
  const char *red = msd_opt_str(o, NULL, "msplit_reduction", "dbr");
  if (strcmp(red, "dbr") && strcmp(red, "seq")) return usage();
  if (!strcmp(red, "seq") && msp_ctx_set_reduction(ctx, MSP_REDUCE_SEQ)) {
    fprintf(stderr, "msp_ctx_set_reduction: %s\n", msp_get_last_error());
    return 1;
  }
  msd_transport t;
  memset(&t, 0, sizeof(t));
  t.world = world;
  t.rank = rank;
  const char *tname = "none"; /* the transport that actually carries the exchange and the sums */
#ifdef MSD_MPI
  t.barrier = mpi_barrier;
  t.bcast = mpi_bcast;
  if (world > 1) {
    int ok = 0;
    if (!strcmp(msd_opt_str(o, NULL, "msplit_transport", "rccl"), "rccl")) {
      uint8_t id[MSP_COMM_ID_BYTES];
      memset(id, 0, sizeof(id));
      int have = rank == 0 ? msp_comm_get_unique_id(id) == 0 : 0;
      MPI_Bcast(&have, 1, MPI_INT, 0, MPI_COMM_WORLD);
      MPI_Bcast(id, MSP_COMM_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
      ok = have && msp_comm_create_rccl(ctx, world, rank, id, &t.comm) == 0;
      int all = 0;
      MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
      if (!all) { /* every rank takes the MPI path (e.g. two ranks sharing one GPU) */
        if (t.comm) msp_comm_destroy(&t.comm);
        if (rank == 0) fprintf(stderr, "msplit: RCCL communicator unavailable, using MPI_Allgather\n");
        ok = 0;
      }
    }
    /* -msplit_require_rccl: a run that would fall back to the host transport stops before any solve, so an
     * N-GPU measurement can never silently take the MPI path (bench.py --require-rccl) */
    if (!ok && msd_opt_has(o, NULL, "msplit_require_rccl")) {
      if (rank == 0) fprintf(stderr, "msplit: -msplit_require_rccl but the RCCL communicator is unavailable\n");
      MPI_Finalize();
      return 3;
    }
    if (!ok && msp_comm_create_host(ctx, world, rank, mpi_allgather, NULL, &t.comm)) {
      fprintf(stderr, "msp_comm_create_host: %s\n", msp_get_last_error());
      return 1;
    }
    tname = ok ? "rccl" : "host";
  }
#endif
  msd_result r;
  int rc = kind == 0   ? msd_sm_solve(ctx, &p, o, &t, &r)
           : kind == 1 ? msd_smsm_global_solve(ctx, &p, o, &t, &r)
           : kind == 2 ? msd_am_solve(ctx, &p, o, &t, &r)
                       : msd_amam_global_solve(ctx, &p, o, &t, &r);
  const int async = kind >= 2;
  if (rc == MSP_ERR_ARG_OUTOFRANGE && async) rc = 0; /* stopped at -max_outer: still report */
  /* asynchronous runs: every block's own end state -- detection state, phase tag, iterations, messages discarded
   * and sends still in flight at shutdown, and the final residual as that block's rank computed it -- gathered on
   * rank 0 (one block per rank under MPI, every block locally otherwise) */
  enum { REP = 8 };
  double rep[64 * REP];
  int nrep = 0;
  if (async && !rc) {
    double mine[64 * REP];
    for (int i = 0; i < r.nlocal; ++i) {
      double *q = mine + i * REP;
      q[0] = world > 1 ? rank : i;
      q[1] = r.iterations[i];
      q[2] = r.states[i];
      q[3] = r.tags[i];
      q[4] = (double)r.discarded[i];
      q[5] = (double)r.in_flight[i];
      q[6] = r.final_norm;
      q[7] = r.error;
    }
#ifdef MSD_MPI
    if (world > 1) {
      MPI_Gather(mine, REP, MPI_DOUBLE, rep, REP, MPI_DOUBLE, 0, MPI_COMM_WORLD);
      nrep = world;
    } else
#endif
    {
      memcpy(rep, mine, sizeof(double) * REP * (size_t)r.nlocal);
      nrep = r.nlocal;
    }
  }
  if (!rc && rank == 0) {
    if (msd_opt_has(o, NULL, "json")) {
      printf("{\"program\": \"%s\", \"host\": \"c\", \"ranks\": %d, \"blocks\": %d, \"transport\": \"%s\", ", prog,
             world, p.nb, tname);
      if (async) {
        printf("\"iterations\": [");
        for (int i = 0; i < r.nlocal; ++i) printf("%s%d", i ? ", " : "", r.iterations[i]);
        printf("], \"blocks_report\": [");
        for (int i = 0; i < nrep; ++i) {
          const double *q = rep + i * REP;
          printf("%s{\"block\": %d, \"iterations\": %d, \"state\": %d, \"tag\": %d, \"discarded\": %lld, "
                 "\"in_flight\": %lld, \"final_norm\": %.17g, \"error\": %.17g}",
                 i ? ", " : "", (int)q[0], (int)q[1], (int)q[2], (int)q[3], (long long)q[4], (long long)q[5], q[6], q[7]);
        }
        printf("], ");
      } else {
        printf("\"outer_its\": %d, \"hist_hex\": [", r.outer_its);
        const int nh = r.outer_its < MSD_HIST_CAP ? r.outer_its : MSD_HIST_CAP;
        for (int i = 0; i < nh; ++i) printf("%s\"%a\"", i ? ", " : "", r.hist[i]);
        printf("], ");
        if (kind == 1) {
          printf("\"lsqr_its\": [");
          for (int i = 0; i < nh; ++i) printf("%s%d", i ? ", " : "", r.lsqr_its[i]);
          printf("], ");
        }
      }
      printf("\"norm0\": %.17g, \"final_norm\": %.17g, \"error\": %.17g, \"elapsed\": %.6f}\n", r.norm0, r.final_norm,
             r.error, r.elapsed);
    } else {
      printf("Elapsed time (iterations):   %f  seconds \n", r.elapsed);
      if (async)
        for (int i = 0; i < r.nlocal; ++i)
          printf("[ Block rank %d ] Total number of iterations (outer_iterations) = %d \n", i, r.iterations[i]);
      else
        printf("Total number of iterations (outer_iterations) = %d \n", r.outer_its);
      printf("Final residual norm 2 = %e \n", r.final_norm);
      printf("Erreur  : %e  \n", r.error);
    }
  }
  if (t.comm) msp_comm_destroy(&t.comm);
  msp_ctx_destroy(&ctx);
  msd_options_free(o);
#ifdef MSD_MPI
  MPI_Finalize();
#endif
  return rc ? 1 : 0;
}
