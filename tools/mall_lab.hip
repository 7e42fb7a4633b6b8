// mall_lab: can the CGS block's VecMAXPY reuse what the VecMDot before it left in the
// Infinity Cache (MALL, 256 MiB)?  MDot-like pass (w . V_j over DBR chunks, forward
// order) followed by a MAXPY-like pass (w -= sum a_j V_j), with the basis loads
// non-temporal or default-policy in each pass and the MAXPY's chunks forward or reversed
// (reversed starts on the chunks the MDot read last).  Prints one JSON object.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/mall_lab.hip -o tools/mall_lab
//   tools/mall_lab <n> <reps>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

template <bool NT>
__device__ __forceinline__ dx2 ld(const double* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const dx2*>(p));
  else return *reinterpret_cast<const dx2*>(p);
}

// partial[c*K + j] = sum over the chunk of w . V_j (lane-local sums, then a plain LDS tree)
template <bool NT>
__global__ __launch_bounds__(kT) void k_rd(const double* __restrict__ w, const double* __restrict__ V, int K,
                                           int64_t n, double* __restrict__ partial) {
  __shared__ double red[kT];
  const int t = threadIdx.x;
  const int64_t c = blockIdx.x, base = c * kChunk + 2 * t;
  dx2 wv[kIt];
#pragma unroll
  for (int i = 0; i < kIt; ++i) wv[i] = *reinterpret_cast<const dx2*>(w + base + i * 2 * kT);
  for (int j = 0; j < K; j += 4) {
    double s[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double* v = V + (int64_t)(j + q) * n;
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        const dx2 x = ld<NT>(v + base + i * 2 * kT);
        s[q] = s[q] + wv[i].x * x.x;
        s[q] = s[q] + wv[i].y * x.y;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      red[t] = s[q];
      __syncthreads();
      for (int o = kT / 2; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
      }
      if (t == 0) partial[c * K + j + q] = red[0];
      __syncthreads();
    }
  }
}

template <bool NT, bool REV>
__global__ __launch_bounds__(kT) void k_mx(double* __restrict__ w, const double* __restrict__ V, int K, int64_t n,
                                           double a) {
  const int t = threadIdx.x;
  const int64_t c = REV ? (int64_t)(gridDim.x - 1 - blockIdx.x) : (int64_t)blockIdx.x;
  const int64_t base = c * kChunk + 2 * t;
  dx2 u[kIt];
#pragma unroll
  for (int i = 0; i < kIt; ++i) u[i] = *reinterpret_cast<const dx2*>(w + base + i * 2 * kT);
#pragma unroll 2
  for (int j = 0; j < K; j += 4) {
    dx2 x[4][kIt];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kIt; ++i) x[q][i] = ld<NT>(V + (int64_t)(j + q) * n + base + i * 2 * kT);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kIt; ++i) {
        u[i].x = u[i].x - a * x[q][i].x;
        u[i].y = u[i].y - a * x[q][i].y;
      }
  }
#pragma unroll
  for (int i = 0; i < kIt; ++i) __builtin_nontemporal_store(u[i], reinterpret_cast<dx2*>(w + base + i * 2 * kT));
}

__global__ void k_fill(double* p, int64_t n, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + 1e-9 * (double)(i & 1023);
}

int main(int argc, char** argv) {
  const int n3 = argc > 1 ? atoi(argv[1]) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t n = (int64_t)n3 * n3 * n3;
  if (n % kChunk) return 2;
  const int Kmax = 32;
  double *w, *V, *partial;
  CK(hipMalloc(&w, n * 8));
  CK(hipMalloc(&V, n * 8 * Kmax));
  const int64_t G = n / kChunk;
  CK(hipMalloc(&partial, G * Kmax * 8));
  k_fill<<<(unsigned)((n + 255) / 256), 256>>>(w, n, 1.0);
  k_fill<<<(unsigned)((n * Kmax + 255) / 256), 256>>>(V, n * Kmax, 0.5);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  printf("{\"n\": %lld, \"results\": {", (long long)n);
  bool first = true;
  for (int K : {8, 16, 28}) {
    for (int rnt = 0; rnt < 2; ++rnt)
      for (int mnt = 0; mnt < 2; ++mnt)
        for (int rev = 0; rev < 2; ++rev) {
          auto rd = [&] {
            if (rnt) k_rd<true><<<(unsigned)G, kT>>>(w, V, K, n, partial);
            else k_rd<false><<<(unsigned)G, kT>>>(w, V, K, n, partial);
          };
          auto mx = [&] {
            if (mnt && rev) k_mx<true, true><<<(unsigned)G, kT>>>(w, V, K, n, 1e-300);
            else if (mnt) k_mx<true, false><<<(unsigned)G, kT>>>(w, V, K, n, 1e-300);
            else if (rev) k_mx<false, true><<<(unsigned)G, kT>>>(w, V, K, n, 1e-300);
            else k_mx<false, false><<<(unsigned)G, kT>>>(w, V, K, n, 1e-300);
          };
          double trd = 0, tmx = 0;
          for (int r = 0; r < reps + 1; ++r) {
            float a = 0, b = 0;
            CK(hipEventRecord(e0));
            rd();
            CK(hipEventRecord(e1));
            mx();
            CK(hipEventRecord(e2));
            CK(hipEventSynchronize(e2));
            CK(hipEventElapsedTime(&a, e0, e1));
            CK(hipEventElapsedTime(&b, e1, e2));
            if (r) {
              trd += a;
              tmx += b;
            }
          }
          trd /= reps;
          tmx /= reps;
          const double brd = 8.0 * n * (K + 1), bmx = 8.0 * n * (K + 2);
          printf("%s\"K%d/rd_%s/mx_%s/%s\": {\"rd_us\": %.1f, \"rd_GBps\": %.0f, \"mx_us\": %.1f, \"mx_GBps\": %.0f, "
                 "\"pair_GBps\": %.0f}",
                 first ? "" : ", ", K, rnt ? "nt" : "tmp", mnt ? "nt" : "tmp", rev ? "rev" : "fwd", trd * 1e3,
                 brd / (trd * 1e-3) / 1e9, tmx * 1e3, bmx / (tmx * 1e-3) / 1e9, (brd + bmx) / ((trd + tmx) * 1e-3) / 1e9);
          first = false;
          fflush(stdout);
        }
  }
  printf("}}\n");
  return 0;
}
