// spmv_lab.hip -- standalone A/B bench for CSR SpMV variants on the n^3 7-point
// operator (diagnostics for the library's k_spmv_lds8; not linked into it).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/spmv_lab tools/spmv_lab.hip
//   tools/spmv_lab [n] [reps]
//
// Every variant that computes y = A x is checked bitwise against variant 0.
// Algorithmic bytes per launch: 12 nnz + 4 (N + 1) + 8 N (x) + 8 N (y).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

constexpr int kT = 256;

// --- assembly: row r of the n^3 7-point Laplacian, columns ascending
__global__ void k_rowlen(int n, int32_t* len) {
  const int64_t N = (int64_t)n * n * n;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const int i = r % n, j = (r / n) % n, k = r / ((int64_t)n * n);
  len[r] = 1 + (i > 0) + (i < n - 1) + (j > 0) + (j < n - 1) + (k > 0) + (k < n - 1);
}
__global__ void k_fill(int n, const int32_t* rowptr, int32_t* col, double* val) {
  const int64_t N = (int64_t)n * n * n;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const int i = r % n, j = (r / n) % n, k = r / ((int64_t)n * n);
  const int64_t P = (int64_t)n * n;
  int32_t p = rowptr[r];
  if (k > 0) { col[p] = (int32_t)(r - P); val[p++] = -1.0; }
  if (j > 0) { col[p] = (int32_t)(r - n); val[p++] = -1.0; }
  if (i > 0) { col[p] = (int32_t)(r - 1); val[p++] = -1.0; }
  col[p] = (int32_t)r; val[p++] = 6.0;
  if (i < n - 1) { col[p] = (int32_t)(r + 1); val[p++] = -1.0; }
  if (j < n - 1) { col[p] = (int32_t)(r + n); val[p++] = -1.0; }
  if (k < n - 1) { col[p] = (int32_t)(r + P); val[p++] = -1.0; }
}
__global__ void k_randx(int64_t N, double* x) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  uint64_t z = (uint64_t)r * 0x9E3779B97F4A7C15ull + 20251121ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  x[r] = (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

__device__ __forceinline__ void st_nt(double* p, double v) { __builtin_nontemporal_store(v, p); }
typedef double dx2 __attribute__((ext_vector_type(2)));
typedef int ix4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int4 ld_nt(const int4* p) {
  const ix4 v = __builtin_nontemporal_load(reinterpret_cast<const ix4*>(p));
  return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ double2 ld_nt(const double2* p) {
  const dx2 v = __builtin_nontemporal_load(reinterpret_cast<const dx2*>(p));
  return make_double2(v.x, v.y);
}

// --- variant 0: the library's k_spmv_lds8 (MULT, SU = 4), restated
// VAR bit 0: non-temporal y store; bit 1: skip the x gathers (diagnostic: x[r] only)
template <int VAR, int RPL>
__global__ __launch_bounds__(kT) void k_lds8(int32_t nrows, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col, const double* __restrict__ val,
                                             const double* __restrict__ x, double* __restrict__ y, int32_t lds_cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sval = reinterpret_cast<double*>(smem);
  int32_t* scol = reinterpret_cast<int32_t*>(smem + (size_t)lds_cap * 8);
  const int t = threadIdx.x;
  const int32_t r0 = blockIdx.x * kT * RPL;
  const int32_t r1 = min(r0 + kT * RPL, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  int32_t k0[RPL], k1[RPL];
#pragma unroll
  for (int h = 0; h < RPL; ++h) {
    const int32_t r = r0 + t + h * kT;
    k0[h] = k1[h] = 0;
    if (r < r1) {
      k0[h] = rowptr[r];
      k1[h] = rowptr[r + 1];
    }
  }
  if constexpr ((VAR & 16) != 0) {  // the library's stage_csr_block<NT, 4>: conditional loads
    for (int32_t i0 = t; i0 < n2 || i0 < n4; i0 += 4 * kT) {
      double2 vt[4];
      int4 ct[2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n2) vt[u] = (VAR & 4) ? ld_nt(v2 + i) : v2[i];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n4) ct[u] = (VAR & 8) ? ld_nt(c4 + i) : c4[i];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n2) reinterpret_cast<double2*>(sval)[i] = vt[u];
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int32_t i = i0 + u * kT;
        if (i < n4) reinterpret_cast<int4*>(scol)[i] = ct[u];
      }
      if (i0 + 2 * kT < n4) {
        for (int32_t i = i0 + 2 * kT; i < n4 && i < i0 + 4 * kT; i += kT)
          reinterpret_cast<int4*>(scol)[i] = (VAR & 8) ? ld_nt(c4 + i) : c4[i];
      }
    }
  } else   {
  constexpr int SU = 4 * RPL;  // slices per lane: 7-point rows need <= 3.5 RPL double2 / 1.75 RPL int4
  {
    double2 vt[SU];
    int4 ct[SU / 2];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int32_t i = min(t + u * kT, max(n2 - 1, 0));
      vt[u] = (VAR & 4) ? ld_nt(v2 + i) : v2[i];
    }
#pragma unroll
    for (int u = 0; u < SU / 2; ++u) {
      const int32_t i = min(t + u * kT, max(n4 - 1, 0));
      ct[u] = (VAR & 8) ? ld_nt(c4 + i) : c4[i];
    }
#pragma unroll
    for (int u = 0; u < SU; ++u)
      if (t + u * kT < n2) reinterpret_cast<double2*>(sval)[t + u * kT] = vt[u];
#pragma unroll
    for (int u = 0; u < SU / 2; ++u)
      if (t + u * kT < n4) reinterpret_cast<int4*>(scol)[t + u * kT] = ct[u];
  }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < RPL; ++h) {
    const int32_t r = r0 + t + h * kT;
    if (r < r1) {
      double s = 0.0;
      for (int32_t kb = k0[h]; kb < k1[h]; kb += 8) {
        double av[8], xv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int32_t k = min(kb + q, k1[h] - 1);
          av[q] = sval[k - s2];
          xv[q] = (VAR & 2) ? x[r] + (double)scol[k - s4] : x[scol[k - s4]];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (kb + q < k1[h]) s = s + av[q] * xv[q];
      }
      if (VAR & 1) st_nt(y + r, s); else y[r] = s;
    }
  }
}

// --- variant: direct CSR without LDS, one lane per row (each lane reads its own
// row's col/val: uncoalesced within an instruction, all bytes used via L1)
__global__ __launch_bounds__(kT) void k_direct(int32_t nrows, const int32_t* __restrict__ rowptr,
                                               const int32_t* __restrict__ col, const double* __restrict__ val,
                                               const double* __restrict__ x, double* __restrict__ y) {
  const int32_t r = blockIdx.x * kT + threadIdx.x;
  if (r >= nrows) return;
  const int32_t k0 = rowptr[r], k1 = rowptr[r + 1];
  double s = 0.0;
  for (int32_t kb = k0; kb < k1; kb += 8) {
    double av[8], xv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int32_t k = min(kb + q, k1 - 1);
      av[q] = val[k];
      xv[q] = x[col[k]];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (kb + q < k1) s = s + av[q] * xv[q];
  }
  y[r] = s;
}

// --- ceiling: stream val, col, rowptr and x once, write y (no dependent loads);
// RPL row blocks of 256 per workgroup
template <int RPL>
__global__ __launch_bounds__(kT) void k_stream(int32_t nrows, int64_t nnz, const int32_t* __restrict__ rowptr,
                                               const int32_t* __restrict__ col, const double* __restrict__ val,
                                               const double* __restrict__ x, double* __restrict__ y) {
  const int t = threadIdx.x;
  const int32_t r0 = blockIdx.x * kT * RPL, r1 = min(r0 + kT * RPL, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  double2 vt[4 * RPL];
  int4 ct[2 * RPL];
  double xr[RPL];
  int32_t rp[RPL];
#pragma unroll
  for (int u = 0; u < 4 * RPL; ++u) vt[u] = v2[min(t + u * kT, max(n2 - 1, 0))];
#pragma unroll
  for (int u = 0; u < 2 * RPL; ++u) ct[u] = c4[min(t + u * kT, max(n4 - 1, 0))];
#pragma unroll
  for (int h = 0; h < RPL; ++h) {
    const int32_t r = min(r0 + t + h * kT, nrows - 1);
    xr[h] = x[r];
    rp[h] = rowptr[r];
  }
  double acc = 0.0;
#pragma unroll
  for (int u = 0; u < 4 * RPL; ++u) acc += vt[u].x + vt[u].y;
#pragma unroll
  for (int u = 0; u < 2 * RPL; ++u) acc += (double)(ct[u].x + ct[u].y + ct[u].z + ct[u].w);
#pragma unroll
  for (int h = 0; h < RPL; ++h) {
    const int32_t r = r0 + t + h * kT;
    if (r < r1) y[r] = acc + xr[h] + (double)rp[h];
  }
}


// --- variant: wave-granular staging.  Each wave owns 64 consecutive rows and
// stages their col/val slice into its own LDS region; no workgroup barrier
// (LDS ops of one wave complete in order), so waves never wait on each other.
// VAR bit 0: non-temporal y store.
template <int VAR>
__global__ __launch_bounds__(kT) void k_wave(int32_t nrows, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col, const double* __restrict__ val,
                                             const double* __restrict__ x, double* __restrict__ y, int32_t wcap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* base = smem + (size_t)w * wcap * 12;
  double* sval = reinterpret_cast<double*>(base);
  int32_t* scol = reinterpret_cast<int32_t*>(base + (size_t)wcap * 8);
  const int32_t r0 = ((int32_t)blockIdx.x * 4 + w) * 64;
  if (r0 >= nrows) return;
  const int32_t r1 = min(r0 + 64, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  const int32_t r = r0 + lane;
  int32_t k0 = 0, k1 = 0;
  if (r < r1) {
    k0 = rowptr[r];
    k1 = rowptr[r + 1];
  }
  for (int32_t i0 = lane; i0 < n2 || i0 < n4; i0 += 4 * 64) {
    double2 vt[4];
    int4 ct[2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int32_t i = i0 + u * 64;
      if (i < n2) vt[u] = v2[i];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int32_t i = i0 + u * 64;
      if (i < n4) ct[u] = c4[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int32_t i = i0 + u * 64;
      if (i < n2) reinterpret_cast<double2*>(sval)[i] = vt[u];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int32_t i = i0 + u * 64;
      if (i < n4) reinterpret_cast<int4*>(scol)[i] = ct[u];
    }
    for (int32_t i = i0 + 2 * 64; i < n4 && i < i0 + 4 * 64; i += 64) reinterpret_cast<int4*>(scol)[i] = c4[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (r < r1) {
    double s = 0.0;
    for (int32_t kb = k0; kb < k1; kb += 8) {
      double av[8], xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int32_t k = min(kb + q, k1 - 1);
        av[q] = sval[k - s2];
        xv[q] = x[scol[k - s4]];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (kb + q < k1) s = s + av[q] * xv[q];
    }
    if (VAR & 1) st_nt(y + r, s); else y[r] = s;
  }
}

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// --- variant: workgroup staging with LDS-DMA (global_load_lds_dwordx4): the
// col/val slice goes to LDS with no VGPR round trip.  Each wave-instruction
// writes 64 consecutive 16-byte slices; tail lanes re-read the last slice into
// slack LDS (cap rounded up to 256 entries).  VAR bit 0: non-temporal y store.
template <int VAR>
__global__ __launch_bounds__(kT) void k_glds(int32_t nrows, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col, const double* __restrict__ val,
                                             const double* __restrict__ x, double* __restrict__ y, int32_t cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sv = smem;
  char* sc = smem + (size_t)cap * 8;
  const double* sval = reinterpret_cast<const double*>(sv);
  const int32_t* scol = reinterpret_cast<const int32_t*>(sc);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int32_t r0 = (int32_t)blockIdx.x * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1, s4 = start & ~3;
  const int32_t n2 = (end - s2 + 1) >> 1, n4 = (end - s4 + 3) >> 2;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int4* c4 = reinterpret_cast<const int4*>(col + s4);
  for (int32_t ib = w * 64; ib < n2; ib += kT) glds16(v2 + min(ib + lane, n2 - 1), sv + (size_t)ib * 16);
  for (int32_t ib = w * 64; ib < n4; ib += kT) glds16(c4 + min(ib + lane, n4 - 1), sc + (size_t)ib * 16);
  const int32_t r = r0 + t;
  int32_t k0 = 0, k1 = 0;
  if (r < r1) {
    k0 = rowptr[r];
    k1 = rowptr[r + 1];
  }
  __syncthreads();
  if (r < r1) {
    double s = 0.0;
    for (int32_t kb = k0; kb < k1; kb += 8) {
      double av[8], xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int32_t k = min(kb + q, k1 - 1);
        av[q] = sval[k - s2];
        xv[q] = x[scol[k - s4]];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (kb + q < k1) s = s + av[q] * xv[q];
    }
    if (VAR & 1) st_nt(y + r, s); else y[r] = s;
  }
}

// --- variant: product staging.  Entry-major (coalesced) pass: lane i loads
// val pair i and col pair i, gathers the two x values and writes the two
// products val*x to LDS (8 B per entry instead of 12); then lane r adds its
// row's products left to right.  Same products, same order: bitwise.
template <int VAR>
__global__ __launch_bounds__(kT) void k_prod(int32_t nrows, const int32_t* __restrict__ rowptr,
                                             const int32_t* __restrict__ col, const double* __restrict__ val,
                                             const double* __restrict__ x, double* __restrict__ y, int32_t cap) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sp = reinterpret_cast<double*>(smem);
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * kT;
  const int32_t r1 = min(r0 + kT, nrows);
  const int32_t start = rowptr[r0], end = rowptr[r1];
  const int32_t s2 = start & ~1;
  const int32_t n2 = (end - s2 + 1) >> 1;
  const double2* v2 = reinterpret_cast<const double2*>(val + s2);
  const int2* c2 = reinterpret_cast<const int2*>(col + s2);
  for (int32_t i0 = t; i0 < n2; i0 += 4 * kT) {
    double2 vt[4];
    int2 ct[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int32_t i = min(i0 + u * kT, n2 - 1);
      vt[u] = v2[i];
      ct[u] = c2[i];
    }
    double xa[4], xb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int32_t e = s2 + 2 * (i0 + u * kT);
      xa[u] = (e >= start && e < end) ? x[ct[u].x] : 0.0;
      xb[u] = (e + 1 >= start && e + 1 < end) ? x[ct[u].y] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int32_t i = i0 + u * kT;
      if (i < n2) reinterpret_cast<double2*>(sp)[i] = make_double2(vt[u].x * xa[u], vt[u].y * xb[u]);
    }
  }
  const int32_t r = r0 + t;
  int32_t k0 = 0, k1 = 0;
  if (r < r1) {
    k0 = rowptr[r];
    k1 = rowptr[r + 1];
  }
  __syncthreads();
  if (r < r1) {
    double s = 0.0;
    for (int32_t k = k0; k < k1; ++k) s = s + sp[k - s2];
    if (VAR & 1) st_nt(y + r, s); else y[r] = s;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const bool per_launch_events = argc > 3 && atoi(argv[3]) != 0;
  const int group = argc > 4 ? atoi(argv[4]) : 0;  // 0: the original set; 1: staging variants
  const int64_t N = (int64_t)n * n * n;
  const int nblk = (int)((N + kT - 1) / kT);
  int32_t *rowptr, *col;
  double *val, *x, *y, *y0;
  CK(hipMalloc(&rowptr, (N + 1) * 4));
  CK(hipMemset(rowptr, 0, 4));
  int32_t* len;
  CK(hipMalloc(&len, N * 4));
  k_rowlen<<<(unsigned)((N + 255) / 256), 256>>>(n, len);
  // exclusive scan on the host (simple, one-time)
  std::vector<int32_t> h(N), hp(N + 1);
  CK(hipMemcpy(h.data(), len, N * 4, hipMemcpyDeviceToHost));
  hp[0] = 0;
  for (int64_t i = 0; i < N; ++i) hp[i + 1] = hp[i] + h[i];
  const int64_t nnz = hp[N];
  int64_t maxblk = 0;
  for (int64_t b = 0; b < nblk; ++b) {
    const int64_t e = std::min<int64_t>((b + 1) * kT, N);
    maxblk = std::max<int64_t>(maxblk, hp[e] - hp[b * kT]);
  }
  int64_t maxblk2 = 0;
  for (int64_t b = 0; b < (N + 511) / 512; ++b) {
    const int64_t e = std::min<int64_t>((b + 1) * 512, N);
    maxblk2 = std::max<int64_t>(maxblk2, hp[e] - hp[b * 512]);
  }
  CK(hipMemcpy(rowptr, hp.data(), (N + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&col, (nnz + 4) * 4));
  CK(hipMalloc(&val, (nnz + 2) * 8));
  CK(hipMalloc(&x, N * 8));
  CK(hipMalloc(&y, N * 8));
  CK(hipMalloc(&y0, N * 8));
  k_fill<<<(unsigned)((N + 255) / 256), 256>>>(n, rowptr, col, val);
  k_randx<<<(unsigned)((N + 255) / 256), 256>>>(N, x);
  CK(hipDeviceSynchronize());
  const int32_t cap = (int32_t)((maxblk + 8 + 3) & ~3LL);
  const int32_t cap2 = (int32_t)((maxblk2 + 8 + 3) & ~3LL);
  int64_t maxw = 0;
  for (int64_t b = 0; b < (N + 63) / 64; ++b) {
    const int64_t e = std::min<int64_t>((b + 1) * 64, N);
    maxw = std::max<int64_t>(maxw, hp[e] - hp[b * 64]);
  }
  const int32_t wcap = (int32_t)((maxw + 8 + 3) & ~3LL);
  const int32_t gcap = (int32_t)((maxblk + 8 + 255) & ~255LL);
  const int nblk_w = (int)((N + 255) / 256);
  const double bytes = 12.0 * nnz + 4.0 * (N + 1) + 16.0 * N;
  printf("{\"n\": %d, \"nnz\": %lld, \"alg_bytes\": %.0f, \"lds_cap\": %d, \"results\": {", n, (long long)nnz, bytes, cap);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> hy(N), hy0(N);
  bool first = true;
  int round_ = 0;
  double* ycheck = nullptr;
  auto run = [&](const char* name, auto launch, bool check) {
    launch();
    CK(hipDeviceSynchronize());
    float ms = 0;
    if (per_launch_events) {  // every launch between its own pair of events (the library's kernel timing)
      std::vector<hipEvent_t> ev(2 * reps);
      for (auto& e : ev) CK(hipEventCreate(&e));
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(ev[2 * i]));
        launch();
        CK(hipEventRecord(ev[2 * i + 1]));
      }
      CK(hipDeviceSynchronize());
      for (int i = 0; i < reps; ++i) {
        float m = 0;
        CK(hipEventElapsedTime(&m, ev[2 * i], ev[2 * i + 1]));
        ms += m;
      }
      for (auto& e : ev) CK(hipEventDestroy(e));
    } else {
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double us = ms * 1e3 / reps;
    const double gbs = bytes / (us * 1e-6) / 1e9;
    const char* eq = "null";
    if (check) {
      CK(hipMemcpy(hy.data(), ycheck ? ycheck : y, N * 8, hipMemcpyDeviceToHost));
      eq = memcmp(hy.data(), hy0.data(), N * 8) == 0 ? "true" : "false";
    }
    printf("%s\"%s/%d\": {\"us\": %.1f, \"GBps\": %.1f, \"frac\": %.4f, \"bitwise\": %s}", first ? "" : ", ", name, round_, us, gbs,
           gbs / 8000.0, eq);
    first = false;
    fflush(stdout);
  };
  // reference result
  k_lds8<0, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y0, cap);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hy0.data(), y0, N * 8, hipMemcpyDeviceToHost));
  if (group == 2) {  // the same arrays allocated physically contiguous (hipDeviceMallocContiguous)
    int32_t *colC, *rpC;
    double *valC, *xC, *yC;
    CK(hipExtMallocWithFlags((void**)&rpC, (N + 1) * 4, hipDeviceMallocContiguous));
    CK(hipExtMallocWithFlags((void**)&colC, (nnz + 4) * 4, hipDeviceMallocContiguous));
    CK(hipExtMallocWithFlags((void**)&valC, (nnz + 2) * 8, hipDeviceMallocContiguous));
    CK(hipExtMallocWithFlags((void**)&xC, N * 8, hipDeviceMallocContiguous));
    CK(hipExtMallocWithFlags((void**)&yC, N * 8, hipDeviceMallocContiguous));
    CK(hipMemcpy(rpC, rowptr, (N + 1) * 4, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(colC, col, (nnz + 4) * 4, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(valC, val, (nnz + 2) * 8, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(xC, x, N * 8, hipMemcpyDeviceToDevice));
    CK(hipDeviceSynchronize());
    for (round_ = 0; round_ < 3; ++round_) {
      ycheck = nullptr;
      run("lib_t", [&] { k_lds8<16, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
      run("glds_nty", [&] { k_glds<1><<<nblk, kT, gcap * 12>>>((int32_t)N, rowptr, col, val, x, y, gcap); }, true);
      run("lib_ntvcy", [&] { k_lds8<29, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
      ycheck = yC;
      run("lib_t_contig", [&] { k_lds8<16, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rpC, colC, valC, xC, yC, cap); }, true);
      run("glds_nty_contig", [&] { k_glds<1><<<nblk, kT, gcap * 12>>>((int32_t)N, rpC, colC, valC, xC, yC, gcap); }, true);
      run("lib_ntvcy_contig", [&] { k_lds8<29, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rpC, colC, valC, xC, yC, cap); }, true);
    }
    ycheck = nullptr;
  }
  for (round_ = 0; round_ < 3 && group == 1; ++round_) {
    run("lib_t", [&] { k_lds8<16, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lib_nty", [&] { k_lds8<17, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lib_ntvcy", [&] { k_lds8<29, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("wave", [&] { k_wave<0><<<nblk_w, kT, wcap * 12 * 4>>>((int32_t)N, rowptr, col, val, x, y, wcap); }, true);
    run("wave_nty", [&] { k_wave<1><<<nblk_w, kT, wcap * 12 * 4>>>((int32_t)N, rowptr, col, val, x, y, wcap); }, true);
    run("glds", [&] { k_glds<0><<<nblk, kT, gcap * 12>>>((int32_t)N, rowptr, col, val, x, y, gcap); }, true);
    run("glds_nty", [&] { k_glds<1><<<nblk, kT, gcap * 12>>>((int32_t)N, rowptr, col, val, x, y, gcap); }, true);
    run("prod", [&] { k_prod<0><<<nblk, kT, cap * 8>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("prod_nty", [&] { k_prod<1><<<nblk, kT, cap * 8>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("stream", [&] { k_stream<1><<<nblk, kT>>>((int32_t)N, nnz, rowptr, col, val, x, y); }, false);
  }
  for (round_ = 0; round_ < 3 && group == 0; ++round_) {
    run("lds8", [&] { k_lds8<0, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lds8_nty", [&] { k_lds8<1, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lds8_rpl2", [&] { k_lds8<0, 2><<<(nblk + 1) / 2, kT, cap2 * 12>>>((int32_t)N, rowptr, col, val, x, y, cap2); }, true);
    run("lds8_nogather", [&] { k_lds8<2, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, false);
    run("direct", [&] { k_direct<<<nblk, kT>>>((int32_t)N, rowptr, col, val, x, y); }, true);
    run("lds8_ntv", [&] { k_lds8<4, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lds8_ntvy", [&] { k_lds8<5, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lds8_ntcy", [&] { k_lds8<9, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lds8_ntvcy", [&] { k_lds8<13, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lib_t", [&] { k_lds8<16, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lib_ntvcy", [&] { k_lds8<29, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("lib_nty", [&] { k_lds8<17, 1><<<nblk, kT, cap * 12>>>((int32_t)N, rowptr, col, val, x, y, cap); }, true);
    run("stream", [&] { k_stream<1><<<nblk, kT>>>((int32_t)N, nnz, rowptr, col, val, x, y); }, false);
    run("stream_rpl2", [&] { k_stream<2><<<(nblk + 1) / 2, kT>>>((int32_t)N, nnz, rowptr, col, val, x, y); }, false);
    run("stream_rpl4", [&] { k_stream<4><<<(nblk + 3) / 4, kT>>>((int32_t)N, nnz, rowptr, col, val, x, y); }, false);
  }
  printf("}}\n");
  return 0;
}
