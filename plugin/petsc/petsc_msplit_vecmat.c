/*
 * petsc_msplit_vecmat.c -- VecType "msplit" and MatType "aijmsplit": the
 * north star's MatType/VecType registration of the C ABI (include/msplit.h),
 * for PETSc 3.22.1.  Not compiled in this repository (the image has no PETSc);
 * plugin/petsc/Makefile builds it with the KSP types next to it.
 *
 * VECMSPLIT is VECSEQ with a device mirror (v->spptr, PETSc's offload mask, as
 * PETSc's own device vectors do): the KSPGMRES vector ops (VecMDot, VecMAXPY,
 * VecNorm, VecDot, VecScale, VecAXPY, VecAYPX, VecWAXPY, VecCopy, VecSet) run
 * in HBM through msp_vec_*; any other op, and every VecGetArray*, first brings
 * the host array up to date and leaves the host copy authoritative after a
 * write.  One rank per block (-npb 1): the vector's communicator has one rank.
 *
 * MATAIJMSPLIT is MATSEQAIJ whose assembled CSR is mirrored in HBM at
 * MatAssemblyEnd; MatMult with VECMSPLIT vectors is msp_mat_mult.  Its
 * MatCreateVecs default is VECMSPLIT.  MatCreateSubMatrix is SeqAIJ's (see
 * the reference's inner operator comes from it, which is why
 * the KSP types in petsc_msplit_ksp.c are the primary drop-in).
 *
 *   -vec_type msplit -mat_type aijmsplit      (create_vector / create_matrix_sparse,
 *                                               utils.c:139-168, call *SetFromOptions)
 */
#include <petsc/private/matimpl.h>
#include <petsc/private/vecimpl.h>
#include <../src/mat/impls/aij/seq/aij.h>
#include <../src/vec/vec/impls/dvecimpl.h>
#include "msplit.h"

#define VECMSPLIT "msplit"
#define MATAIJMSPLIT "aijmsplit"

#define MSPCall(e) do { int _rc = (e); PetscCheck(!_rc, PETSC_COMM_SELF, PETSC_ERR_LIB, "%s", msp_get_last_error()); } while (0)

static msp_ctx *g_ctx; /* one context (GPU) per process: the block's GPU */

PetscErrorCode MSplitDefaultDevice(int *dev); /* petsc_msplit_ksp.c: -msplit_device, else node-local rank % ndev */

/* The process's one context, shared by every Vec, Mat and KSP of the plugin (petsc_msplit_ksp.c): one stream
 * orders all of their work.  It lives until the process ends. */
PetscErrorCode MSplitContext(msp_ctx **ctx)
{
  PetscFunctionBegin;
  if (!g_ctx) {
    int dev = 0;
    PetscCall(MSplitDefaultDevice(&dev));
    MSPCall(msp_ctx_create(dev, NULL, &g_ctx));
    /* -msplit_reduction seq: VecDot/VecNorm/VecMDot of the drivers' outer tests in PETSc's order too */
    const char *const red[] = {"dbr", "seq"};
    PetscInt  r   = 0;
    PetscBool set = PETSC_FALSE;
    PetscCall(PetscOptionsGetEList(NULL, NULL, "-msplit_reduction", red, 2, &r, &set));
    if (set) MSPCall(msp_ctx_set_reduction(g_ctx, (int)r));
  }
  *ctx = g_ctx;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* ------------------------------------------------------------------ Vec */
typedef struct {
  msp_vec *d;
  struct _VecOps seq; /* VECSEQ's ops, for everything not overridden */
} Vec_MSplit;

#define VMS(v) ((Vec_MSplit *)(v)->spptr)

static PetscErrorCode MSplitVecToDevice(Vec v)
{
  PetscFunctionBegin;
  if (v->offloadmask == PETSC_OFFLOAD_CPU) {
    MSPCall(msp_vec_set_values(VMS(v)->d, 0, v->map->n, ((Vec_Seq *)v->data)->array));
    v->offloadmask = PETSC_OFFLOAD_BOTH;
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode MSplitVecToHost(Vec v)
{
  PetscFunctionBegin;
  if (v->offloadmask == PETSC_OFFLOAD_GPU) {
    MSPCall(msp_vec_get_values(VMS(v)->d, 0, v->map->n, ((Vec_Seq *)v->data)->array));
    v->offloadmask = PETSC_OFFLOAD_BOTH;
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode MSplitVecIs(Vec v, PetscBool *is)
{
  PetscFunctionBegin;
  PetscCall(PetscObjectTypeCompare((PetscObject)v, VECMSPLIT, is));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecGetArray_MSplit(Vec v, PetscScalar **a)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToHost(v));
  *a = ((Vec_Seq *)v->data)->array;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecRestoreArray_MSplit(Vec v, PetscScalar **a)
{
  PetscFunctionBegin;
  v->offloadmask = PETSC_OFFLOAD_CPU; /* the host copy may have been written */
  if (a) *a = NULL;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecGetArrayRead_MSplit(Vec v, const PetscScalar **a)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToHost(v));
  *a = ((Vec_Seq *)v->data)->array;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecRestoreArrayRead_MSplit(Vec v, const PetscScalar **a)
{
  PetscFunctionBegin;
  if (a) *a = NULL;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecGetArrayWrite_MSplit(Vec v, PetscScalar **a)
{
  PetscFunctionBegin;
  *a = ((Vec_Seq *)v->data)->array; /* overwritten whole: no download */
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* Device ops.  Each brings its operands to HBM, runs msp_*, and leaves the
 * device copy authoritative for what it wrote. */
static PetscErrorCode VecDot_MSplit(Vec x, Vec y, PetscScalar *z)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  PetscCall(MSplitVecToDevice(y));
  MSPCall(msp_vec_dot(VMS(x)->d, VMS(y)->d, z));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecMDot_MSplit(Vec x, PetscInt nv, const Vec y[], PetscScalar *z)
{
  const msp_vec *dy[64];
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  for (PetscInt i0 = 0; i0 < nv; i0 += 64) {
    const PetscInt g = PetscMin(64, nv - i0);
    for (PetscInt j = 0; j < g; ++j) {
      PetscCall(MSplitVecToDevice(y[i0 + j]));
      dy[j] = VMS(y[i0 + j])->d;
    }
    MSPCall(msp_vec_mdot(VMS(x)->d, (int)g, dy, z + i0));
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecMAXPY_MSplit(Vec y, PetscInt nv, const PetscScalar *alpha, Vec *x)
{
  const msp_vec **dx;
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(y));
  PetscCall(PetscMalloc1(nv, &dx));
  for (PetscInt j = 0; j < nv; ++j) { /* all at once: the library applies VecMAXPY_Seq's grouping of 4 */
    PetscCall(MSplitVecToDevice(x[j]));
    dx[j] = VMS(x[j])->d;
  }
  MSPCall(msp_vec_maxpy(VMS(y)->d, (int)nv, alpha, dx));
  PetscCall(PetscFree(dx));
  y->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecNorm_MSplit(Vec x, NormType type, PetscReal *z)
{
  PetscFunctionBegin;
  if (type != NORM_2) { /* other norms on the host */
    PetscCall(MSplitVecToHost(x));
    PetscCall(VMS(x)->seq.norm(x, type, z));
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  PetscCall(MSplitVecToDevice(x));
  MSPCall(msp_vec_norm(VMS(x)->d, z));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecScale_MSplit(Vec x, PetscScalar a)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  MSPCall(msp_vec_scale(VMS(x)->d, a));
  x->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecSet_MSplit(Vec x, PetscScalar a)
{
  PetscFunctionBegin;
  MSPCall(msp_vec_set(VMS(x)->d, a));
  x->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecCopy_MSplit(Vec x, Vec y)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  MSPCall(msp_vec_copy(VMS(x)->d, VMS(y)->d));
  y->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecAXPY_MSplit(Vec y, PetscScalar a, Vec x)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  PetscCall(MSplitVecToDevice(y));
  MSPCall(msp_vec_axpy(VMS(y)->d, a, VMS(x)->d));
  y->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecAYPX_MSplit(Vec y, PetscScalar b, Vec x)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  PetscCall(MSplitVecToDevice(y));
  MSPCall(msp_vec_aypx(VMS(y)->d, b, VMS(x)->d));
  y->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecWAXPY_MSplit(Vec w, PetscScalar a, Vec x, Vec y)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToDevice(x));
  PetscCall(MSplitVecToDevice(y));
  MSPCall(msp_vec_waxpy(VMS(w)->d, a, VMS(x)->d, VMS(y)->d));
  w->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* Host-side ops that write the array directly: make the host current first,
 * then the host copy is the authoritative one. */
static PetscErrorCode VecSetValues_MSplit(Vec x, PetscInt ni, const PetscInt ix[], const PetscScalar y[],
                                          InsertMode mode)
{
  PetscFunctionBegin;
  PetscCall(MSplitVecToHost(x));
  PetscCall(VMS(x)->seq.setvalues(x, ni, ix, y, mode));
  x->offloadmask = PETSC_OFFLOAD_CPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecCreate_MSplit(Vec);

static PetscErrorCode VecDuplicate_MSplit(Vec x, Vec *y)
{
  PetscFunctionBegin;
  PetscCall(VecCreate(PetscObjectComm((PetscObject)x), y));
  PetscCall(PetscLayoutReference(x->map, &(*y)->map));
  PetscCall(VecSetType(*y, VECMSPLIT));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecDestroy_MSplit(Vec v)
{
  Vec_MSplit *d = VMS(v);
  PetscFunctionBegin;
  if (d) {
    msp_vec_destroy(&d->d);
    PetscCall(VMS(v)->seq.destroy(v));
    PetscCall(PetscFree(d));
    v->spptr = NULL;
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode VecCreate_MSplit(Vec v)
{
  Vec_MSplit *d;
  msp_ctx *ctx;
  PetscMPIInt size;
  PetscFunctionBegin;
  PetscCallMPI(MPI_Comm_size(PetscObjectComm((PetscObject)v), &size));
  PetscCheck(size == 1, PETSC_COMM_SELF, PETSC_ERR_SUP, "VECMSPLIT: one rank per block (-npb 1)");
  PetscCall(VecCreate_Seq(v));
  PetscCall(PetscObjectChangeTypeName((PetscObject)v, VECMSPLIT));
  PetscCall(PetscNew(&d));
  d->seq = *v->ops;
  v->spptr = d;
  PetscCall(MSplitContext(&ctx));
  MSPCall(msp_vec_create(ctx, v->map->n, &d->d));
  v->offloadmask = PETSC_OFFLOAD_CPU; /* VecCreate_Seq zeroed the host array */
  v->ops->dot               = VecDot_MSplit;
  v->ops->mdot              = VecMDot_MSplit;
  v->ops->maxpy             = VecMAXPY_MSplit;
  v->ops->norm              = VecNorm_MSplit;
  v->ops->scale             = VecScale_MSplit;
  v->ops->set               = VecSet_MSplit;
  v->ops->copy              = VecCopy_MSplit;
  v->ops->axpy              = VecAXPY_MSplit;
  v->ops->aypx              = VecAYPX_MSplit;
  v->ops->waxpy             = VecWAXPY_MSplit;
  v->ops->setvalues         = VecSetValues_MSplit;
  v->ops->duplicate         = VecDuplicate_MSplit;
  v->ops->destroy           = VecDestroy_MSplit;
  v->ops->getarray          = VecGetArray_MSplit;
  v->ops->restorearray      = VecRestoreArray_MSplit;
  v->ops->getarrayread      = VecGetArrayRead_MSplit;
  v->ops->restorearrayread  = VecRestoreArrayRead_MSplit;
  v->ops->getarraywrite     = VecGetArrayWrite_MSplit;
  v->ops->restorearraywrite = VecRestoreArray_MSplit;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* ------------------------------------------------------------------ Mat */
typedef struct {
  msp_mat *d;
  PetscErrorCode (*seq_assemblyend)(Mat, MatAssemblyType);
  PetscErrorCode (*seq_mult)(Mat, Vec, Vec);
  PetscErrorCode (*seq_destroy)(Mat);
} Mat_MSplit;

#define MMS(A) ((Mat_MSplit *)(A)->spptr)

static PetscErrorCode MatAssemblyEnd_AIJMSplit(Mat A, MatAssemblyType t)
{
  Mat_SeqAIJ *a = (Mat_SeqAIJ *)A->data;
  msp_ctx    *ctx;
  PetscFunctionBegin;
  PetscCall(MMS(A)->seq_assemblyend(A, t));
  if (t == MAT_FLUSH_ASSEMBLY) PetscFunctionReturn(PETSC_SUCCESS);
  PetscCall(MSplitContext(&ctx));
  MSPCall(msp_mat_destroy(&MMS(A)->d)); /* CSR in HBM (PetscInt = int32, sorted columns as in AIJ) */
  MSPCall(msp_mat_create_csr(ctx, (int32_t)A->rmap->n, (int32_t)A->cmap->n, a->i, a->j, a->a, &MMS(A)->d));
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode MatMult_AIJMSplit(Mat A, Vec x, Vec y)
{
  PetscBool dx, dy;
  PetscFunctionBegin;
  PetscCall(MSplitVecIs(x, &dx));
  PetscCall(MSplitVecIs(y, &dy));
  if (!dx || !dy || !MMS(A)->d) { /* host vectors: SeqAIJ's own MatMult */
    PetscCall(MMS(A)->seq_mult(A, x, y));
    PetscFunctionReturn(PETSC_SUCCESS);
  }
  PetscCall(MSplitVecToDevice(x));
  MSPCall(msp_mat_mult(MMS(A)->d, VMS(x)->d, VMS(y)->d));
  y->offloadmask = PETSC_OFFLOAD_GPU;
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode MatDestroy_AIJMSplit(Mat A)
{
  Mat_MSplit *m = MMS(A);
  PetscFunctionBegin;
  if (m) {
    msp_mat_destroy(&m->d);
    A->spptr = NULL;
    PetscCall(m->seq_destroy(A));
    PetscCall(PetscFree(m));
  }
  PetscFunctionReturn(PETSC_SUCCESS);
}

static PetscErrorCode MatCreate_AIJMSplit(Mat A)
{
  Mat_MSplit *m;
  PetscMPIInt size;
  PetscFunctionBegin;
  PetscCallMPI(MPI_Comm_size(PetscObjectComm((PetscObject)A), &size));
  PetscCheck(size == 1, PETSC_COMM_SELF, PETSC_ERR_SUP, "MATAIJMSPLIT: one rank per block (-npb 1)");
  PetscCall(MatSetType(A, MATSEQAIJ));
  PetscCall(PetscObjectChangeTypeName((PetscObject)A, MATAIJMSPLIT));
  PetscCall(PetscNew(&m));
  m->seq_assemblyend = A->ops->assemblyend;
  m->seq_mult        = A->ops->mult;
  m->seq_destroy     = A->ops->destroy;
  A->spptr           = m;
  A->ops->assemblyend = MatAssemblyEnd_AIJMSplit;
  A->ops->mult        = MatMult_AIJMSplit;
  A->ops->destroy     = MatDestroy_AIJMSplit;
  PetscCall(PetscFree(A->defaultvectype));
  PetscCall(PetscStrallocpy(VECMSPLIT, &A->defaultvectype)); /* MatCreateVecs -> VECMSPLIT */
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* The HBM mirror of an aijmsplit matrix (made at its MatAssemblyEnd), or NULL for any other Mat: msplitgmres
 * runs on it instead of uploading the CSR again (petsc_msplit_ksp.c KSPSetUp_MSplitGMRES). */
PetscErrorCode MSplitMatGetDevice(Mat A, msp_mat **d)
{
  PetscBool is;
  PetscFunctionBegin;
  *d = NULL;
  PetscCall(PetscObjectTypeCompare((PetscObject)A, MATAIJMSPLIT, &is));
  if (is && A->spptr) *d = MMS(A)->d;
  PetscFunctionReturn(PETSC_SUCCESS);
}

/* Call once after PetscInitialize, with MSplitRegisterAll (petsc_msplit_ksp.c) -- or let -dll_append load the
 * library, whose PetscDLLibraryRegister_petsc_msplit calls both. */
PetscErrorCode MSplitRegisterVecMat(void)
{
  PetscFunctionBegin;
  PetscCall(VecRegister(VECMSPLIT, VecCreate_MSplit));
  PetscCall(MatRegister(MATAIJMSPLIT, MatCreate_AIJMSplit));
  PetscFunctionReturn(PETSC_SUCCESS);
}
