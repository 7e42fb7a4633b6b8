// msplit_kernels.h -- launcher declarations shared by msplit_kernels.hip and
// msplit_runtime.hip (C++/HIP side only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#define MSK_MAX_GROUP 32
#define MSK_DBR_CHUNK 4096

enum { MSK_SET = 0, MSK_COPY, MSK_SCALE, MSK_AXPY, MSK_AYPX, MSK_WAXPY_P1, MSK_WAXPY_M1, MSK_WAXPY };

struct VecGroup {
  const double* p[MSK_MAX_GROUP];
};
struct Coefs {
  double a[MSK_MAX_GROUP];
};

enum { MSK_VAR_SPMV = 0, MSK_VAR_MDOT, MSK_VAR_MAXPY, MSK_NVAR };

extern "C" {
void msk_set_variant(int which, int v);
int msk_dot_stage1(const double* w, const VecGroup* V, int nv, int64_t n, double* partial, int64_t nchunks, int self,
                   hipStream_t s);
int msk_dot_stage2(const double* partial, int64_t nchunks, int nv, double* out, hipStream_t s);
int msk_maxpy(double* w, const VecGroup* V, int nv, const Coefs* A, const double* adev, int negate, int64_t n, int accum,
              hipStream_t s);
int msk_maxpy_norm(double* w, const VecGroup* V, int nv, const Coefs* A, const double* adev, int negate, int64_t n,
                   int accum, double* partial, hipStream_t s);
int msk_spmv(int32_t nrows, const int32_t* rowptr, const int32_t* col, const double* val, const double* x,
             const double* b, double* y, int32_t lds_cap, int resid, hipStream_t s);
int msk_spmv_rows(int32_t nlisted, const int32_t* row_ids, const int32_t* rowptr, const int32_t* col,
                  const double* val, const double* x, const double* b, double* y, int resid, hipStream_t s);
int msk_box_stencil(int dim, int32_t nx, int32_t ny, int32_t nz, int64_t nrows, int32_t* rowptr, int32_t* col,
                    double* val, hipStream_t s);
int msk_blas1(int op, double* y, const double* x, const double* z, double alpha, int64_t n, hipStream_t s);
}
