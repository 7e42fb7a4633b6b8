/* petsc_msplit_ksp.c -- KSPType "msplitgmres": KSPGMRES(restart) with PCNONE on the MI355X. */
#include <stdlib.h>

#include <petsc/private/kspimpl.h>
#include "msplit.h"

typedef struct {
  msp_ctx *ctx;        /* the process's shared context (MSplitContext): not owned */
  msp_mat *A;
  PetscBool A_borrowed; /* A is an aijmsplit matrix's own HBM mirror: not destroyed here */
  msp_ksp *ksp;
  msp_vec *b, *x;
  PetscInt restart;
  PetscReal haptol, breakdowntol;
  PetscInt reduction; /* -msplit_reduction dbr|seq on this KSP's prefix; -1: the shared context's order */
} KSP_MSplit;

/* -msplit_reduction: the device reduction order (include/msplit.h msp_ctx_set_reduction).  "seq" is
 * the parity mode -- every dot, norm and MDot summed in PETSc's Seq order, so iteration counts and
 * residual histories are the reference's bit for bit -- at a fraction of the speed (bench.py seq_mode). */
static const char *const MSplitReductions[] = {"dbr", "seq", "MSplitReduction", "MSPLIT_REDUCTION_", NULL};

#define MSPCall(e) do { int _rc = (e); PetscCheck(!_rc, PETSC_COMM_SELF, _rc, "%s", msp_get_last_error()); } while (0)

/* -msplit_reduction under a KSP's prefix: that order for this KSP's solves only.  The process's one context also
 * serves every VECMSPLIT / aijmsplit operation (the drivers' outer VecNorm / VecDot / MatResidual), whose order is
 * the global -msplit_reduction: a solve sets its KSP's order and restores the context's on every exit, so one KSP's
 * choice never leaks into the outer residual norms or into another KSP. */
static PetscErrorCode MSplitSetFromOptionsReduction(PetscOptionItems *PetscOptionsObject, PetscInt *reduction)
{
  PetscEnum red = (PetscEnum)(*reduction >= 0 ? *reduction : 0);
  PetscBool set = PETSC_FALSE;
  PetscFunctionBegin;
  PetscCall(PetscOptionsEnum("-msplit_reduction", "device reduction order (seq: PETSc's, bitwise)", NULL,
                             MSplitReductions, red, &red, &set));
  if (set) *reduction = (PetscInt)red;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode MSplitSolveInOrder(KSP ksp, msp_ctx *ctx, PetscInt reduction, PetscErrorCode (*body)(KSP))
{
  int saved = 0;
  PetscFunctionBegin;
  if (reduction < 0) {
    PetscCall(body(ksp));
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  MSPCall(msp_ctx_get_reduction(ctx, &saved));
  MSPCall(msp_ctx_set_reduction(ctx, (int)reduction));
  PetscErrorCode ierr = body(ksp);
  MSPCall(msp_ctx_set_reduction(ctx, saved));
  PetscCall(ierr);
  PetscFunctionReturn(PETSC_SUCCESS);
}

#if defined(PETSC_USE_64BIT_INDICES)
#error "the MI355X path takes PetscInt = int32 (msp_mat_create_csr); configure PETSc without --with-64-bit-indices"
#endif

/* The process's node-local rank, found once where every rank calls collectively (PetscDLLibraryRegister_petsc_msplit
 * or MSplitRegisterAll, both inside or right after PetscInitialize): the per-object paths below (KSPSetUp of each
 * block's KSP, the first VECMSPLIT) run at different times on different ranks in the asynchronous drivers, so they
 * must not call a collective.  -1 until cached; then the launcher's local-rank variable is the fallback. */
static int g_local_rank = -1;

static PetscErrorCode MSplitCacheLocalRank(void)
{
  MPI_Comm    node;
  PetscMPIInt local = 0;

  PetscFunctionBegin;
  if (g_local_rank >= 0) PetscFunctionReturn(PETSC_SUCCESS);
  PetscCallMPI(MPI_Comm_split_type(PETSC_COMM_WORLD, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node));
  PetscCallMPI(MPI_Comm_rank(node, &local));
  PetscCallMPI(MPI_Comm_free(&node));
  g_local_rank = (int)local;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static int MSplitLocalRankFromEnv(void)
{
  const char *vars[] = {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "MV2_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID",
                        "LOCAL_RANK"};
  for (size_t i = 0; i < sizeof(vars) / sizeof(vars[0]); ++i) {
    const char *v = getenv(vars[i]);
    if (v && *v) return atoi(v);
  }
  return 0;
}

/* The block's GPU: -msplit_device when given, else the rank's index on its node modulo the devices it sees (one
 * block per rank, one rank per GPU, as petscmpiexec -n 8 places them on an 8-GPU node).  Not collective.  Shared
 * with petsc_msplit_vecmat.c. */
PetscErrorCode MSplitDefaultDevice(int *dev)
{
  PetscInt  d    = -1;
  PetscBool set  = PETSC_FALSE;
  int       ndev = 0;

  PetscFunctionBegin;
  PetscCall(PetscOptionsGetInt(NULL, NULL, "-msplit_device", &d, &set));
  if (set) {
    *dev = (int)d;
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  const int local = g_local_rank >= 0 ? g_local_rank : MSplitLocalRankFromEnv();
  MSPCall(msp_get_device_count(&ndev));
  *dev = ndev > 0 ? local % ndev : 0;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* petsc_msplit_vecmat.c: the process's one context (its GPU and stream, shared by every Vec, Mat and KSP of the
 * plugin, so their work is ordered on one stream), and the HBM mirror of an aijmsplit matrix (NULL otherwise) */
PetscErrorCode MSplitContext(msp_ctx **ctx);
PetscErrorCode MSplitMatGetDevice(Mat A, msp_mat **d);

/* The inner operator as a sequential CSR (npb = 1: one rank per block, utils.c:473's MatCreateSubMatrix on the
 * block's communicator).  MATSEQAIJ and aijmsplit are the CSR itself; MATMPIAIJ on one rank is its diagonal
 * block, whose off-diagonal block must be empty.  Anything else is refused. */
static PetscErrorCode MSplitSeqOperator(Mat A, Mat *Ad)
{
  PetscBool   seq, mpi, ams;
  PetscMPIInt size;

  PetscFunctionBegin;
  PetscCall(PetscObjectTypeCompare((PetscObject)A, MATSEQAIJ, &seq));
  PetscCall(PetscObjectTypeCompare((PetscObject)A, "aijmsplit", &ams));
  PetscCall(PetscObjectTypeCompare((PetscObject)A, MATMPIAIJ, &mpi));
  if (seq || ams) {
    *Ad = A;
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  PetscCheck(mpi, PetscObjectComm((PetscObject)A), PETSC_ERR_SUP,
             "msplitgmres: the operator must be MATSEQAIJ, aijmsplit or MATMPIAIJ (got %s)", ((PetscObject)A)->type_name);
  PetscCallMPI(MPI_Comm_size(PetscObjectComm((PetscObject)A), &size));
  PetscCheck(size == 1, PetscObjectComm((PetscObject)A), PETSC_ERR_SUP,
             "msplitgmres: one rank per block (-npb 1); the operator's communicator has %d", (int)size);
  Mat     Ao;
  MatInfo info;
  PetscCall(MatMPIAIJGetSeqAIJ(A, Ad, &Ao, NULL));
  PetscCall(MatGetInfo(Ao, MAT_LOCAL, &info));
  PetscCheck(info.nz_used == 0, PETSC_COMM_SELF, PETSC_ERR_SUP,
             "msplitgmres: the MATMPIAIJ operator couples outside its rank (%g off-diagonal entries)", info.nz_used);
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSetUp_MSplitGMRES(KSP ksp)
{
  KSP_MSplit        *ms = (KSP_MSplit *)ksp->data;
  Mat                A, Ad;
  msp_mat           *mirror = NULL;
  PetscInt           n, nr;
  const PetscInt    *ia, *ja;
  const PetscScalar *aa;
  PetscBool          done;

  PetscFunctionBegin;
  PetscCall(KSPGetOperators(ksp, &A, NULL));
  PetscCall(MSplitSeqOperator(A, &Ad));
  if (!ms->ctx) PetscCall(MSplitContext(&ms->ctx));
  if (!ms->A_borrowed) MSPCall(msp_mat_destroy(&ms->A));
  ms->A = NULL;
  PetscCall(MSplitMatGetDevice(Ad, &mirror));
  if (mirror) { /* aijmsplit: its MatAssemblyEnd already put the CSR in HBM -- no second upload */
    ms->A          = mirror;
    ms->A_borrowed = PETSC_TRUE;
    PetscCall(MatGetLocalSize(Ad, &nr, NULL));
  } else {
    PetscCall(MatGetRowIJ(Ad, 0, PETSC_FALSE, PETSC_FALSE, &nr, &ia, &ja, &done));
    PetscCheck(done, PETSC_COMM_SELF, PETSC_ERR_SUP, "msplitgmres: MatGetRowIJ could not give the CSR");
    PetscCall(MatSeqAIJGetArrayRead(Ad, &aa));
    MSPCall(msp_mat_create_csr(ms->ctx, (int32_t)nr, (int32_t)nr, ia, ja, aa, &ms->A));
    ms->A_borrowed = PETSC_FALSE;
    PetscCall(MatSeqAIJRestoreArrayRead(Ad, &aa));
    PetscCall(MatRestoreRowIJ(Ad, 0, PETSC_FALSE, PETSC_FALSE, &n, &ia, &ja, &done));
  }
  if (!ms->ksp) MSPCall(msp_ksp_create(ms->ctx, &ms->ksp));
  MSPCall(msp_ksp_set_operators(ms->ksp, ms->A));
  if (ms->b) {
    int64_t have = 0;
    MSPCall(msp_vec_get_size(ms->b, &have));
    if (have != (int64_t)nr) { /* KSPSetOperators with an operator of another size */
      MSPCall(msp_vec_destroy(&ms->b));
      MSPCall(msp_vec_destroy(&ms->x));
    }
  }
  if (!ms->b) {
    MSPCall(msp_vec_create(ms->ctx, nr, &ms->b));
    MSPCall(msp_vec_create(ms->ctx, nr, &ms->x));
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSolve_MSplitGMRES_Body(KSP ksp)
{
  KSP_MSplit        *ms = (KSP_MSplit *)ksp->data;
  msp_ksp_opts       o;
  const PetscScalar *b;
  PetscScalar       *x;
  PetscInt           n;
  int32_t            its, reason;
  double             rnorm;
  KSPConvergedDefaultCtx *cctx = (KSPConvergedDefaultCtx *)ksp->cnvP;

  PetscFunctionBegin;
  if (ms->A_borrowed) { /* an aijmsplit operator re-assembled since KSPSetUp has a new HBM mirror: follow it */
    Mat      A, Ad;
    msp_mat *mirror = NULL;
    PetscCall(KSPGetOperators(ksp, &A, NULL));
    PetscCall(MSplitSeqOperator(A, &Ad));
    PetscCall(MSplitMatGetDevice(Ad, &mirror));
    PetscCheck(mirror, PETSC_COMM_SELF, PETSC_ERR_ARG_WRONGSTATE, "msplitgmres: the aijmsplit operator lost its mirror");
    if (mirror != ms->A) {
      ms->A = mirror;
      MSPCall(msp_ksp_set_operators(ms->ksp, ms->A));
    }
  }
  MSPCall(msp_ksp_get_default_opts(&o));
  o.restart       = (int32_t)ms->restart;
  o.max_it        = (int32_t)ksp->max_it;
  o.rtol          = ksp->rtol;
  o.abstol        = ksp->abstol;
  o.divtol        = ksp->divtol;
  o.haptol        = ms->haptol;
  o.breakdowntol  = ms->breakdowntol;
  o.uirnorm       = cctx ? (int32_t)cctx->initialrtol : 0;   /* KSPConvergedDefaultSetUIRNorm */
  o.guess_nonzero = ksp->guess_zero ? 0 : 1;
  MSPCall(msp_ksp_set_opts(ms->ksp, &o));
  PetscCall(VecGetLocalSize(ksp->vec_rhs, &n));
  PetscCall(VecGetArrayRead(ksp->vec_rhs, &b));
  MSPCall(msp_vec_set_values(ms->b, 0, n, b));
  PetscCall(VecRestoreArrayRead(ksp->vec_rhs, &b));
  PetscCall(VecGetArray(ksp->vec_sol, &x));
  if (!ksp->guess_zero) MSPCall(msp_vec_set_values(ms->x, 0, n, x));
  MSPCall(msp_ksp_solve(ms->ksp, ms->b, ms->x));
  MSPCall(msp_vec_get_values(ms->x, 0, n, x));
  PetscCall(VecRestoreArray(ksp->vec_sol, &x));
  MSPCall(msp_ksp_get_iteration_number(ms->ksp, &its));
  MSPCall(msp_ksp_get_residual_norm(ms->ksp, &rnorm));
  MSPCall(msp_ksp_get_converged_reason(ms->ksp, &reason));
  ksp->its    = its;
  ksp->rnorm  = rnorm;
  ksp->reason = (KSPConvergedReason)reason;                  /* same numbering as petscksp.h */
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSolve_MSplitGMRES(KSP ksp)
{
  KSP_MSplit *ms = (KSP_MSplit *)ksp->data;
  PetscFunctionBegin;
  PetscCall(MSplitSolveInOrder(ksp, ms->ctx, ms->reduction, KSPSolve_MSplitGMRES_Body));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSetFromOptions_MSplitGMRES(KSP ksp, PetscOptionItems *PetscOptionsObject)
{
  KSP_MSplit *ms = (KSP_MSplit *)ksp->data;
  PetscFunctionBegin;
  PetscOptionsHeadBegin(PetscOptionsObject, "KSP MSplit GMRES Options");
  PetscCall(PetscOptionsInt("-ksp_gmres_restart", "Krylov directions", NULL, ms->restart, &ms->restart, NULL));
  PetscCall(PetscOptionsReal("-ksp_gmres_haptol", "happy breakdown tolerance", NULL, ms->haptol, &ms->haptol, NULL));
  PetscCall(MSplitSetFromOptionsReduction(PetscOptionsObject, &ms->reduction));
  PetscCall(PetscOptionsReal("-ksp_gmres_breakdown_tolerance", "restart breakdown tolerance", NULL, ms->breakdowntol,
                             &ms->breakdowntol, NULL));
  PetscOptionsHeadEnd();
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPDestroy_MSplitGMRES(KSP ksp)
{
  KSP_MSplit *ms = (KSP_MSplit *)ksp->data;
  PetscFunctionBegin;
  msp_vec_destroy(&ms->b);
  msp_vec_destroy(&ms->x);
  msp_ksp_destroy(&ms->ksp);
  if (!ms->A_borrowed) msp_mat_destroy(&ms->A);
  ms->ctx = NULL; /* shared, not owned */
  PetscCall(PetscFree(ksp->data));
  PetscFunctionReturn(PETSC_SUCCESS);
}

PetscErrorCode KSPCreate_MSplitGMRES(KSP ksp)
{
  KSP_MSplit *ms;
  PetscFunctionBegin;
  PetscCall(PetscNew(&ms));
  ms->restart = 30; ms->haptol = 1.0e-30; ms->breakdowntol = 0.1; ms->reduction = -1;
  ksp->data = (void *)ms;
  PetscCall(KSPSetSupportedNorm(ksp, KSP_NORM_PRECONDITIONED, PC_LEFT, 3));
  PetscCall(KSPSetSupportedNorm(ksp, KSP_NORM_UNPRECONDITIONED, PC_RIGHT, 2));
  ksp->ops->setup          = KSPSetUp_MSplitGMRES;
  ksp->ops->solve          = KSPSolve_MSplitGMRES;
  ksp->ops->setfromoptions = KSPSetFromOptions_MSplitGMRES;
  ksp->ops->destroy        = KSPDestroy_MSplitGMRES;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* ------------------------------------------------------------------------ */
/* KSPType "msplitlsqr": KSPLSQR with PCNONE and a zero guess on the MI355X, the
 * outer solver of the minimization variants (outer_solver_norm_equation,
 * utils.c:1061-1078).  The operator is the block's MATDENSE/MATMPIDENSE R (one
 * rank per block, as the reference runs it); it is copied to HBM at KSPSetUp
 * (the drivers call KSPSetOperators every outer iteration, SMSM-global.c:331). */
typedef struct {
  msp_ctx *ctx; /* the process's shared context: not owned */
  msp_dense *R;
  msp_lsqr *lsqr;
  msp_vec *b, *x;
  PetscBool exact_norm;
  PetscInt reduction; /* -msplit_reduction, as for msplitgmres (-1: the shared context's order) */
} KSP_MSplitLSQR;

static PetscErrorCode KSPSetUp_MSplitLSQR(KSP ksp)
{
  KSP_MSplitLSQR    *ms = (KSP_MSplitLSQR *)ksp->data;
  Mat                A, Al;
  PetscInt           m, n, lda;
  const PetscScalar *a;
  PetscBool          isdense;

  PetscFunctionBegin;
  PetscCall(KSPGetOperators(ksp, &A, NULL));
  PetscCall(PetscObjectTypeCompare((PetscObject)A, MATMPIDENSE, &isdense));
  if (isdense) PetscCall(MatDenseGetLocalMatrix(A, &Al));
  else Al = A;
  PetscCall(MatGetSize(Al, &m, &n));
  PetscCall(MatDenseGetLDA(Al, &lda));
  if (!ms->ctx) PetscCall(MSplitContext(&ms->ctx));
  MSPCall(msp_dense_destroy(&ms->R));
  MSPCall(msp_dense_create(ms->ctx, m, (int32_t)n, &ms->R));
  PetscCall(MatDenseGetArrayRead(Al, &a));
  MSPCall(msp_dense_set_values(ms->R, a, lda));
  PetscCall(MatDenseRestoreArrayRead(Al, &a));
  if (!ms->lsqr) MSPCall(msp_lsqr_create(ms->ctx, &ms->lsqr));
  MSPCall(msp_lsqr_set_operators(ms->lsqr, 1, &ms->R));
  MSPCall(msp_vec_destroy(&ms->b));
  MSPCall(msp_vec_destroy(&ms->x));
  MSPCall(msp_vec_create(ms->ctx, m, &ms->b));
  MSPCall(msp_vec_create(ms->ctx, n, &ms->x));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSolve_MSplitLSQR_Body(KSP ksp)
{
  KSP_MSplitLSQR    *ms = (KSP_MSplitLSQR *)ksp->data;
  msp_lsqr_opts      o;
  const PetscScalar *b;
  PetscScalar       *x;
  PetscInt           m, n;
  int32_t            its, reason;
  double             rnorm;

  PetscFunctionBegin;
  MSPCall(msp_lsqr_get_default_opts(&o));
  o.max_it     = (int32_t)ksp->max_it;
  o.rtol       = ksp->rtol;
  o.abstol     = ksp->abstol;
  o.divtol     = ksp->divtol;
  o.exact_norm = ms->exact_norm ? 1 : 0;
  if (ksp->converged == KSPConvergedDefault) o.conv_test = MSP_LSQR_CONV_DEFAULT;   /* -ksp_convergence_test default */
  else if (ksp->converged == KSPConvergedSkip) o.conv_test = MSP_LSQR_CONV_SKIP;
  else o.conv_test = MSP_LSQR_CONV_LSQR;                                          /* KSPLSQRConvergedDefault */
  MSPCall(msp_lsqr_set_opts(ms->lsqr, &o));
  PetscCall(VecGetLocalSize(ksp->vec_rhs, &m));
  PetscCall(VecGetArrayRead(ksp->vec_rhs, &b));
  MSPCall(msp_vec_set_values(ms->b, 0, m, b));
  PetscCall(VecRestoreArrayRead(ksp->vec_rhs, &b));
  MSPCall(msp_lsqr_solve(ms->lsqr, &ms->b, ms->x));               /* zero initial guess */
  PetscCall(VecGetLocalSize(ksp->vec_sol, &n));
  PetscCall(VecGetArray(ksp->vec_sol, &x));
  MSPCall(msp_vec_get_values(ms->x, 0, n, x));
  PetscCall(VecRestoreArray(ksp->vec_sol, &x));
  MSPCall(msp_lsqr_get_iteration_number(ms->lsqr, &its));
  MSPCall(msp_lsqr_get_residual_norm(ms->lsqr, &rnorm));
  MSPCall(msp_lsqr_get_converged_reason(ms->lsqr, &reason));
  ksp->its    = its;
  ksp->rnorm  = rnorm;                                             /* KSPGetResidualNorm, SMSM-global.c:341 */
  ksp->reason = (KSPConvergedReason)reason;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSolve_MSplitLSQR(KSP ksp)
{
  KSP_MSplitLSQR *ms = (KSP_MSplitLSQR *)ksp->data;
  PetscFunctionBegin;
  PetscCall(MSplitSolveInOrder(ksp, ms->ctx, ms->reduction, KSPSolve_MSplitLSQR_Body));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPSetFromOptions_MSplitLSQR(KSP ksp, PetscOptionItems *PetscOptionsObject)
{
  KSP_MSplitLSQR *ms = (KSP_MSplitLSQR *)ksp->data;
  PetscFunctionBegin;
  PetscOptionsHeadBegin(PetscOptionsObject, "KSP MSplit LSQR Options");
  PetscCall(MSplitSetFromOptionsReduction(PetscOptionsObject, &ms->reduction));
  PetscCall(PetscOptionsBool("-ksp_lsqr_exact_mat_norm", "exact Frobenius norm of the operator", NULL,
                             ms->exact_norm, &ms->exact_norm, NULL));
  PetscOptionsHeadEnd();
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode KSPDestroy_MSplitLSQR(KSP ksp)
{
  KSP_MSplitLSQR *ms = (KSP_MSplitLSQR *)ksp->data;
  PetscFunctionBegin;
  msp_vec_destroy(&ms->b);
  msp_vec_destroy(&ms->x);
  msp_lsqr_destroy(&ms->lsqr);
  msp_dense_destroy(&ms->R);
  ms->ctx = NULL; /* shared, not owned */
  PetscCall(PetscFree(ksp->data));
  PetscFunctionReturn(PETSC_SUCCESS);
}

PetscErrorCode KSPCreate_MSplitLSQR(KSP ksp)
{
  KSP_MSplitLSQR *ms;
  PetscFunctionBegin;
  PetscCall(PetscNew(&ms));
  ms->reduction = -1;
  ksp->data = (void *)ms;
  PetscCall(KSPSetSupportedNorm(ksp, KSP_NORM_UNPRECONDITIONED, PC_LEFT, 3));
  PetscCall(KSPSetSupportedNorm(ksp, KSP_NORM_NONE, PC_LEFT, 1));
  PetscCall(KSPSetConvergenceTest(ksp, KSPLSQRConvergedDefault, NULL, NULL)); /* as KSPCreate_LSQR */
  ksp->ops->setup          = KSPSetUp_MSplitLSQR;
  ksp->ops->solve          = KSPSolve_MSplitLSQR;
  ksp->ops->setfromoptions = KSPSetFromOptions_MSplitLSQR;
  ksp->ops->destroy        = KSPDestroy_MSplitLSQR;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* Call once after PetscInitialize (or load as a PETSc dynamic library):
 *   -inner1_ksp_type msplitgmres ... -outer1_ksp_type msplitlsqr ... */
PetscErrorCode MSplitRegisterAll(void)
{
  PetscFunctionBegin;
  PetscCall(MSplitCacheLocalRank()); /* collective on PETSC_COMM_WORLD: every rank is here */
  PetscCall(KSPRegister("msplitgmres", KSPCreate_MSplitGMRES));
  PetscCall(KSPRegister("msplitlsqr", KSPCreate_MSplitLSQR));
  PetscFunctionReturn(PETSC_SUCCESS);
}

PetscErrorCode MSplitRegisterVecMat(void); /* petsc_msplit_vecmat.c */

/* The entry point PETSc's dynamic-library loader calls: `-dll_append /path/libpetsc_msplit.so` (or
 * -dll_prepend) makes PetscInitialize open the library and call PetscDLLibraryRegister_<name>, the name being
 * the file's basename without "lib" and the suffix.  It registers the two KSP types, the VecType and the MatType,
 * so the reference's executables pick them up through their existing KSPSetFromOptions / MatSetFromOptions /
 * VecSetFromOptions calls (utils.c:130, :146, :164, :530) with no source change and no relink:
 *   petscmpiexec -n 2 ./bin/synchronous-multisplitting ... -dll_append libpetsc_msplit.so \
 *       -inner1_ksp_type msplitgmres -inner2_ksp_type msplitgmres */
PETSC_EXTERN PetscErrorCode PetscDLLibraryRegister_petsc_msplit(void)
{
  PetscFunctionBegin;
  PetscCall(MSplitRegisterAll());
  PetscCall(MSplitRegisterVecMat());
  PetscFunctionReturn(PETSC_SUCCESS);
}
