// stream_ceiling: what HBM rate can a kernel with the GMRES step's access mix reach on this MI355X?
// Four plain streaming kernels over vectors of n doubles, 16-byte non-temporal accesses, one 4096-element
// chunk per 256-lane workgroup (the DBR layout the product kernels use), no reductions, no ordering
// constraints:
//   read K   : s += V_j[i] for j < K (a store of one double per lane so nothing is dead code)
//   copy     : y = x
//   mix K    : y = x + sum_{j<K} V_j (K + 1 reads : 1 write, the CGS VecMAXPY's mix)
//   fill     : y = c
// Prints one JSON object: TB/s per kernel (bytes the kernel requests / time per launch, HIP events).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/stream_ceiling.hip -o tools/stream_ceiling
//   tools/stream_ceiling <n> <reps> [contig]   (contig: buffers physically contiguous, as the library allocates them)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kT = 256, kIt = 8, kChunk = kT * 2 * kIt;
typedef double dx2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ dx2 ld(const double* p) { return __builtin_nontemporal_load(reinterpret_cast<const dx2*>(p)); }
__device__ __forceinline__ void st(double* p, dx2 v) { __builtin_nontemporal_store(v, reinterpret_cast<dx2*>(p)); }

template <int U>
__global__ __launch_bounds__(kT) void k_read(const double* __restrict__ V, int64_t stride, int K,
                                             double* __restrict__ out) {
  const int64_t base = (int64_t)blockIdx.x * kChunk + 2 * threadIdx.x;
  dx2 acc[kIt];
#pragma unroll
  for (int j = 0; j < kIt; ++j) acc[j] = dx2{0.0, 0.0};
#pragma unroll U
  for (int v = 0; v < K; ++v) {
    const double* p = V + (int64_t)v * stride + base;
#pragma unroll
    for (int j = 0; j < kIt; ++j) acc[j] += ld(p + j * 2 * kT);
  }
  dx2 s = acc[0];
#pragma unroll
  for (int j = 1; j < kIt; ++j) s += acc[j];
  out[(int64_t)blockIdx.x * kT + threadIdx.x] = s.x + s.y;
}

template <int U>
__global__ __launch_bounds__(kT) void k_mix(const double* __restrict__ x, const double* __restrict__ V, int64_t stride,
                                            int K, double* __restrict__ y) {
  const int64_t base = (int64_t)blockIdx.x * kChunk + 2 * threadIdx.x;
  dx2 u[kIt];
#pragma unroll
  for (int j = 0; j < kIt; ++j) u[j] = ld(x + base + j * 2 * kT);
#pragma unroll U
  for (int v = 0; v < K; ++v) {
    const double* p = V + (int64_t)v * stride + base;
#pragma unroll
    for (int j = 0; j < kIt; ++j) u[j] += ld(p + j * 2 * kT);
  }
#pragma unroll
  for (int j = 0; j < kIt; ++j) st(y + base + j * 2 * kT, u[j]);
}

__global__ __launch_bounds__(kT) void k_copy(const double* __restrict__ x, double* __restrict__ y) {
  const int64_t base = (int64_t)blockIdx.x * kChunk + 2 * threadIdx.x;
  dx2 u[kIt];
#pragma unroll
  for (int j = 0; j < kIt; ++j) u[j] = ld(x + base + j * 2 * kT);
#pragma unroll
  for (int j = 0; j < kIt; ++j) st(y + base + j * 2 * kT, u[j]);
}

__global__ __launch_bounds__(kT) void k_fill(double* __restrict__ y, double c) {
  const int64_t base = (int64_t)blockIdx.x * kChunk + 2 * threadIdx.x;
#pragma unroll
  for (int j = 0; j < kIt; ++j) st(y + base + j * 2 * kT, dx2{c, c});
}

template <typename F>
static double time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (int64_t)1 << 24;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  if (n <= 0 || n % kChunk != 0) {
    fprintf(stderr, "n must be a positive multiple of %d\n", kChunk);
    return 2;
  }
  const bool contig = argc > 3 && std::string(argv[3]) == "contig";
  auto alloc = [&](double** p, size_t bytes) {
    if (contig && hipExtMallocWithFlags((void**)p, bytes, hipDeviceMallocContiguous) == hipSuccess) return;
    (void)hipGetLastError();
    CK(hipMalloc(p, bytes));
  };
  const int KMAX = 16;
  const int64_t stride = n;
  double *V, *x, *y, *out;
  alloc(&V, sizeof(double) * stride * KMAX);
  alloc(&x, sizeof(double) * n);
  alloc(&y, sizeof(double) * n);
  const unsigned g = (unsigned)(n / kChunk);
  CK(hipMalloc(&out, sizeof(double) * (size_t)g * kT));
  CK(hipMemset(V, 0, sizeof(double) * stride * KMAX));
  CK(hipMemset(x, 0, sizeof(double) * n));
  const double B = 8.0 * (double)n;
  printf("{\"n\": %lld, \"reps\": %d, \"contiguous\": %s", (long long)n, reps, contig ? "true" : "false");
  for (int K : {4, 8, 16}) {
    double ms = time_ms([&] { k_read<4><<<g, kT>>>(V, stride, K, out); }, reps);
    printf(", \"read%d_TBps\": %.3f", K, B * K / (ms * 1e-3) / 1e12);
    ms = time_ms([&] { k_read<8><<<g, kT>>>(V, stride, K, out); }, reps);
    printf(", \"read%d_u8_TBps\": %.3f", K, B * K / (ms * 1e-3) / 1e12);
  }
  for (int K : {4, 8, 15}) {
    double ms = time_ms([&] { k_mix<4><<<g, kT>>>(x, V, stride, K, y); }, reps);
    printf(", \"mix%d_TBps\": %.3f", K, B * (K + 2) / (ms * 1e-3) / 1e12);
    ms = time_ms([&] { k_mix<8><<<g, kT>>>(x, V, stride, K, y); }, reps);
    printf(", \"mix%d_u8_TBps\": %.3f", K, B * (K + 2) / (ms * 1e-3) / 1e12);
  }
  double ms = time_ms([&] { k_copy<<<g, kT>>>(x, y); }, reps);
  printf(", \"copy_TBps\": %.3f", 2 * B / (ms * 1e-3) / 1e12);
  ms = time_ms([&] { k_fill<<<g, kT>>>(y, 1.0); }, reps);
  printf(", \"fill_TBps\": %.3f}\n", B / (ms * 1e-3) / 1e12);
  CK(hipGetLastError());
  CK(hipFree(V));
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(out));
  return 0;
}
