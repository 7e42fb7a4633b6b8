/*
 * gmres_solution.c -- a C host on the drop-in boundary alone (include/msplit.h):
 * the reference's gmres_solution driver (src/gmres_solution/gmres_solution.c:
 * assemble the operator, b = A u with u = 1, x0 = 0, KSPSolve with
 * GMRES(restart) and PCNONE, report iterations, residual and error), on the
 * MI355X with the operator assembled in HBM.  No Python, no PETSc.
 *
 *   ./gmres_solution [-n 64] [-restart 30] [-max_it 300] [-rtol 1e-4] [-dim 3] [-peclet px py pz]
 *
 * Prints one line of %.17g values so callers can compare bit for bit.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "msplit.h"

#define CHK(call)                                                                  \
  do {                                                                             \
    int rc_ = (call);                                                              \
    if (rc_) {                                                                     \
      fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, msp_get_last_error()); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

int main(int argc, char **argv) {
  int n = 64, restart = 30, max_it = 300, dim = 3;
  double rtol = 1e-4, pe[3] = {0.0, 0.0, 0.0};
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "-n") && i + 1 < argc) n = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-restart") && i + 1 < argc) restart = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-max_it") && i + 1 < argc) max_it = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-rtol") && i + 1 < argc) rtol = atof(argv[++i]);
    else if (!strcmp(argv[i], "-dim") && i + 1 < argc) dim = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-peclet") && i + 3 < argc) {
      for (int d = 0; d < 3; ++d) pe[d] = atof(argv[++i]);
    } else {
      fprintf(stderr, "unknown option %s\n", argv[i]);
      return 2;
    }
  }
  msp_ctx *ctx;
  CHK(msp_ctx_create(0, NULL, &ctx));
  msp_mat *A;
  CHK(msp_mat_create_box_convdiff(ctx, dim, n, n, dim == 3 ? n : 1, 0, 0, pe, &A));
  int32_t nrows, ncols;
  int64_t nnz;
  CHK(msp_mat_get_info(A, &nrows, &ncols, &nnz));
  msp_vec *u, *b, *x, *e;
  CHK(msp_vec_create(ctx, nrows, &u));
  CHK(msp_vec_create(ctx, nrows, &b));
  CHK(msp_vec_create(ctx, nrows, &x));
  CHK(msp_vec_create(ctx, nrows, &e));
  CHK(msp_vec_set(u, 1.0));
  CHK(msp_mat_mult(A, u, b)); /* computeTheRightHandSideWithInitialGuess: b = A u */
  msp_ksp *ksp;
  msp_ksp_opts o;
  CHK(msp_ksp_create(ctx, &ksp));
  CHK(msp_ksp_get_default_opts(&o));
  o.restart = restart;
  o.max_it = max_it;
  o.rtol = rtol;
  CHK(msp_ksp_set_opts(ksp, &o));
  CHK(msp_ksp_set_operators(ksp, A));
  CHK(msp_ksp_solve(ksp, b, x));
  int32_t its, reason;
  double rnorm, err;
  CHK(msp_ksp_get_iteration_number(ksp, &its));
  CHK(msp_ksp_get_converged_reason(ksp, &reason));
  CHK(msp_ksp_get_residual_norm(ksp, &rnorm));
  CHK(msp_vec_waxpy(e, -1.0, u, x)); /* computeError: ||x - u|| */
  CHK(msp_vec_norm(e, &err));
  printf("rows %d nnz %lld its %d reason %d rnorm %.17g error %.17g\n", nrows, (long long)nnz, its, reason, rnorm,
         err);
  msp_ksp_destroy(&ksp);
  msp_vec_destroy(&u);
  msp_vec_destroy(&b);
  msp_vec_destroy(&x);
  msp_vec_destroy(&e);
  msp_mat_destroy(&A);
  msp_ctx_destroy(&ctx);
  return 0;
}
