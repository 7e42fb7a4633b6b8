// ell_lab.hip -- standalone A/B bench for the DV (delta/value dictionary) SpMV in
// its ELL layout on the n^3 7-point operator (diagnostics for the library's
// k_spmv_ell; not linked into it).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ell_lab tools/ell_lab.hip
//   tools/ell_lab [n] [reps]
//
// Storage: row r's 8 one-byte codes at code8 + 8r, in CSR (ascending column)
// order, padded with 255; code c names the pair (ddelta[c], dval[c]).  Every
// variant that computes y = A x is checked bitwise against variant "base".
// Algorithmic bytes per launch: 8 N (codes) + 8 N (x) + 8 N (y).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kT = 256;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef double dx2 __attribute__((ext_vector_type(2)));

// codes of row r: the 7-point stencil's present entries (dictionary order = ascending delta)
__global__ void k_codes(int n, uint8_t* code8) {
  const int64_t N = (int64_t)n * n * n;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const int i = r % n, j = (r / n) % n, k = r / ((int64_t)n * n);
  uint8_t c[8];
  int p = 0;
  if (k > 0) c[p++] = 0;
  if (j > 0) c[p++] = 1;
  if (i > 0) c[p++] = 2;
  c[p++] = 3;
  if (i < n - 1) c[p++] = 4;
  if (j < n - 1) c[p++] = 5;
  if (k < n - 1) c[p++] = 6;
  while (p < 8) c[p++] = 255;
  for (int q = 0; q < 8; ++q) code8[r * 8 + q] = c[q];
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

__device__ __forceinline__ int cbyte(const u32x2& v, int q) { return ((q < 4 ? v.x : v.y) >> (8 * (q & 3))) & 255; }
__device__ __forceinline__ void st_nt(double* p, double v) { __builtin_nontemporal_store(v, p); }

// --- base: the library's k_spmv_ell<MULT, 8, RPL, NTY = true>, restated
template <int RPL>
__global__ __launch_bounds__(kT) void k_base(int32_t nrows, const uint8_t* __restrict__ code8,
                                             const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                             int ndict, const double* __restrict__ x, double* __restrict__ y) {
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  u32x2 cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  __syncthreads();
  double xv[RPL][8];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      xv[j][q] = c != 255 ? x[r + sdel[c]] : 0.0;
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) s = s + sval[c] * xv[j][q];
    }
    if (r < nrows) st_nt(y + r, s);
  }
}

// --- uni: when a row slot's 8 codes are the same in every lane of the wave (interior
// rows; rows on the same x-line boundary), the codes, deltas and values are
// wave-uniform: scalar loads from the dictionary, and the gathers x[r + delta] issue
// with no LDS round trip.  Other waves take the base path.
template <int RPL>
__global__ __launch_bounds__(kT) void k_uni(int32_t nrows, const uint8_t* __restrict__ code8,
                                            const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                            int ndict, const double* __restrict__ x, double* __restrict__ y) {
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  u32x2 cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    const uint32_t ulo = __builtin_amdgcn_readfirstlane(cw[j].x), uhi = __builtin_amdgcn_readfirstlane(cw[j].y);
    const bool same = cw[j].x == ulo && cw[j].y == uhi;
    double s = 0.0;
    if (__all(same)) {
      double xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = ((q < 4 ? ulo : uhi) >> (8 * (q & 3))) & 255;
        xv[q] = c != 255 ? x[r + ddelta[c]] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = ((q < 4 ? ulo : uhi) >> (8 * (q & 3))) & 255;
        if (c != 255) s = s + dval[c] * xv[q];
      }
    } else {
      double xv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = cbyte(cw[j], q);
        xv[q] = c != 255 ? x[r + sdel[c]] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = cbyte(cw[j], q);
        if (c != 255) s = s + sval[c] * xv[q];
      }
    }
    if (r < nrows) st_nt(y + r, s);
  }
}

// --- noxg (diagnostic): the same code/y streams, but every entry multiplies x[r]
// (one coalesced load per row): what the kernel costs without the neighbour gathers.
template <int RPL>
__global__ __launch_bounds__(kT) void k_noxg(int32_t nrows, const uint8_t* __restrict__ code8,
                                             const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                             int ndict, const double* __restrict__ x, double* __restrict__ y) {
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  u32x2 cw[RPL];
  double xr[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
    xr[j] = r < nrows ? x[r] : 0.0;
  }
  if (t < ndict) sval[t] = dval[t];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) s = s + sval[c] * xr[j];
    }
    if (r < nrows) st_nt(y + r, s);
  }
}

// --- sel: deltas and values from registers (a select chain over the <= 8 dictionary
// entries, loaded once as scalars), no LDS in the gather address path.
template <int RPL>
__global__ __launch_bounds__(kT) void k_sel(int32_t nrows, const uint8_t* __restrict__ code8,
                                            const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                            int ndict, const double* __restrict__ x, double* __restrict__ y) {
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  int32_t dd[8];
  double dv[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    dd[c] = c < ndict ? ddelta[c] : 0;
    dv[c] = c < ndict ? dval[c] : 0.0;
  }
  u32x2 cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
  }
  double xv[RPL][8];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      int32_t d = dd[0];
#pragma unroll
      for (int e = 1; e < 8; ++e) d = c == e ? dd[e] : d;
      xv[j][q] = c != 255 ? x[r + d] : 0.0;
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      double a = dv[0];
#pragma unroll
      for (int e = 1; e < 8; ++e) a = c == e ? dv[e] : a;
      if (c != 255) s = s + a * xv[j][q];
    }
    if (r < nrows) st_nt(y + r, s);
  }
}


// --- diagnostics: only some of the neighbour gathers are real; the others read x[r]
// (MASK bit c set: code c gathers x[r + delta]).  near = codes 1,2,4,5 (+-1, +-n);
// far = codes 0,6 (+-plane).
template <int RPL, int MASK>
__global__ __launch_bounds__(kT) void k_part(int32_t nrows, const uint8_t* __restrict__ code8,
                                             const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                             int ndict, const double* __restrict__ x, double* __restrict__ y) {
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  u32x2 cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
  }
  if (t < ndict) {
    sdel[t] = ((MASK >> t) & 1) ? ddelta[t] : 0;
    sval[t] = dval[t];
  }
  __syncthreads();
  double xv[RPL][8];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      xv[j][q] = c != 255 ? x[r + sdel[c]] : 0.0;
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) s = s + sval[c] * xv[j][q];
    }
    if (r < nrows) st_nt(y + r, s);
  }
}

// --- win: x[r0 + lo .. r0 + RPL*256 + hi) staged in LDS (coalesced, default policy);
// entries whose delta lies in [lo, hi] read LDS, the others gather from x.  lo/hi
// come from the host: the dictionary's deltas that fit the LDS window.
template <int RPL>
__global__ __launch_bounds__(kT) void k_win(int32_t nrows, const uint8_t* __restrict__ code8,
                                            const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                            int ndict, const double* __restrict__ x, double* __restrict__ y,
                                            int32_t lo, int32_t hi) {
  extern __shared__ __attribute__((aligned(16))) double sx[];
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  u32x2 cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
  }
  const int32_t wn = RPL * kT + hi - lo;  // window entries: x[r0 + lo + i]
  for (int32_t i = t; i < wn; i += kT) {
    const int32_t g = r0 + lo + i;
    sx[i] = (g >= 0 && g < nrows) ? x[g] : 0.0;
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  __syncthreads();
  double xv[RPL][8];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) {
        const int32_t d = sdel[c];
        xv[j][q] = (d >= lo && d <= hi) ? sx[t + kT * j + d - lo] : x[r + d];
      } else {
        xv[j][q] = 0.0;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) s = s + sval[c] * xv[j][q];
    }
    if (r < nrows) st_nt(y + r, s);
  }
}


// --- pair: lane t holds CONSECUTIVE rows r = r0 + 2t (+512 k) and r + 1.  Where the
// two rows carry the same code at position q (interior rows), one 16-byte load at
// r + d (d even: aligned) serves both rows' gathers; SHFL: d = 0 is that load, and
// d = -1 / +1 come from the neighbouring lanes' loads (x[r-1] = lane t-1's x[r+1];
// x[r+2] = lane t+1's x[r]), the wave's edge lanes loading their own.  Rows whose
// codes differ take one scalar gather per entry.  Same products, same order.
template <int P, bool SHFL>
__global__ __launch_bounds__(kT) void k_pair(int32_t nrows, const uint8_t* __restrict__ code8,
                                             const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                             int ndict, const double* __restrict__ x, double* __restrict__ y) {
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x, lane = t & 63;
  const int32_t r0 = (int32_t)blockIdx.x * (2 * kT * P);
  u32x2 ca[P], cb[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int32_t r = r0 + 2 * t + 2 * kT * k;
    const u32x2 e = {0xFFFFFFFFu, 0xFFFFFFFFu};
    ca[k] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r) : e;
    cb[k] = r + 1 < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r + 1) : e;
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  double2 ctr[P];
  double lft[P], rgt[P];
  if (SHFL) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int32_t r = r0 + 2 * t + 2 * kT * k;
      ctr[k] = r + 1 < nrows ? *reinterpret_cast<const double2*>(x + r) : make_double2(r < nrows ? x[r] : 0.0, 0.0);
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int32_t r = r0 + 2 * t + 2 * kT * k;
      lft[k] = __shfl_up(ctr[k].y, 1, 64);
      rgt[k] = __shfl_down(ctr[k].x, 1, 64);
      if (lane == 0) lft[k] = r >= 1 && r - 1 < nrows ? x[r - 1] : 0.0;
      if (lane == 63) rgt[k] = r + 2 < nrows ? x[r + 2] : 0.0;
    }
  }
  __syncthreads();
  double xa[P][8], xb[P][8];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int32_t r = r0 + 2 * t + 2 * kT * k;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(ca[k], q), c2 = cbyte(cb[k], q);
      xa[k][q] = 0.0;
      xb[k][q] = 0.0;
      if (c == c2) {
        if (c != 255) {
          const int32_t d = sdel[c];
          if (SHFL && d == 0) {
            xa[k][q] = ctr[k].x;
            xb[k][q] = ctr[k].y;
          } else if (SHFL && d == -1) {
            xa[k][q] = lft[k];
            xb[k][q] = ctr[k].x;
          } else if (SHFL && d == 1) {
            xa[k][q] = ctr[k].y;
            xb[k][q] = rgt[k];
          } else if ((d & 1) == 0) {
            const double2 v = *reinterpret_cast<const double2*>(x + r + d);
            xa[k][q] = v.x;
            xb[k][q] = v.y;
          } else {
            xa[k][q] = x[r + d];
            xb[k][q] = x[r + 1 + d];
          }
        }
      } else {
        if (c != 255) xa[k][q] = x[r + sdel[c]];
        if (c2 != 255) xb[k][q] = x[r + 1 + sdel[c2]];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int32_t r = r0 + 2 * t + 2 * kT * k;
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(ca[k], q), c2 = cbyte(cb[k], q);
      if (c != 255) sa = sa + sval[c] * xa[k][q];
      if (c2 != 255) sb = sb + sval[c2] * xb[k][q];
    }
    if (r + 1 < nrows) {
      __builtin_nontemporal_store(dx2{sa, sb}, reinterpret_cast<dx2*>(y + r));
    } else if (r < nrows) {
      st_nt(y + r, sa);
    }
  }
}


// --- dord: loop over the DICTIONARY (sorted by delta, then value) instead of over a
// row's code positions.  A row holds at most one entry per column, so visiting the
// dictionary in ascending delta visits each row's entries in CSR order: the same
// sum.  The delta of entry e is wave-uniform (scalar load), so x[r] serves d = 0, its
// lane neighbours (shuffles) d = -1 / +1, and only the other deltas gather; a row
// without entry e masks its lane off (presence bitmask from its 8 codes).
// ND: dictionary size bound (<= 32), all entries' loads in flight together.
template <int RPL, int ND>
__global__ __launch_bounds__(kT) void k_dord(int32_t nrows, const uint8_t* __restrict__ code8,
                                             const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                             int ndict, const double* __restrict__ x, double* __restrict__ y) {
  const int t = threadIdx.x, lane = t & 63;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  uint32_t pm[RPL];
  double xr[RPL], xm[RPL], xp[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    const u32x2 cw = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                               : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw, q);
      if (c != 255) m |= 1u << c;
    }
    pm[j] = m;
    xr[j] = r < nrows ? x[r] : 0.0;
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    xm[j] = __shfl_up(xr[j], 1, 64);
    xp[j] = __shfl_down(xr[j], 1, 64);
    if (lane == 0) xm[j] = (r >= 1 && r - 1 < nrows) ? x[r - 1] : 0.0;
    if (lane == 63) xp[j] = (r + 1 < nrows) ? x[r + 1] : 0.0;
  }
  int32_t dd[ND];
  double dv[ND];
#pragma unroll
  for (int e = 0; e < ND; ++e) {
    dd[e] = e < ndict ? ddelta[e] : 0x40000000;   // beyond ndict: no row is marked present
    dv[e] = e < ndict ? dval[e] : 0.0;
  }
  double xv[RPL][ND];
#pragma unroll
  for (int e = 0; e < ND; ++e) {
    const int32_t d = dd[e];  // wave-uniform: these are scalar branches
    if (d == 0) {
#pragma unroll
      for (int j = 0; j < RPL; ++j) xv[j][e] = xr[j];
    } else if (d == -1) {
#pragma unroll
      for (int j = 0; j < RPL; ++j) xv[j][e] = xm[j];
    } else if (d == 1) {
#pragma unroll
      for (int j = 0; j < RPL; ++j) xv[j][e] = xp[j];
    } else {
#pragma unroll
      for (int j = 0; j < RPL; ++j) {
        const int32_t r = r0 + t + kT * j;
        xv[j][e] = ((pm[j] >> e) & 1) ? x[r + d] : 0.0;
      }
    }
  }
  double s[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    s[j] = 0.0;
#pragma unroll
    for (int e = 0; e < ND; ++e)
      if ((pm[j] >> e) & 1) s[j] = s[j] + dv[e] * xv[j][e];
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    if (r < nrows) st_nt(y + r, s[j]);
  }
}


// --- dspec: dord with the gathers issued for every lane, independent of the codes
// (addresses clamped into [0, nrows)); presence only gates the sum.  All loads of a
// row (codes, x[r], the far deltas) leave together; d = -1/+1 from lane shuffles.
template <int RPL, int ND>
__global__ __launch_bounds__(kT) void k_dspec(int32_t nrows, const uint8_t* __restrict__ code8,
                                              const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                              int ndict, const double* __restrict__ x, double* __restrict__ y) {
  const int t = threadIdx.x, lane = t & 63;
  const int32_t r0 = (int32_t)blockIdx.x * (kT * RPL);
  int32_t dd[ND];
  double dv[ND];
#pragma unroll
  for (int e = 0; e < ND; ++e) {
    dd[e] = e < ndict ? ddelta[e] : 0;
    dv[e] = e < ndict ? dval[e] : 0.0;
  }
  u32x2 cw[RPL];
  double xr[RPL];
  double xv[RPL][ND];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    const int32_t rc = min(r, nrows - 1);
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
    xr[j] = x[rc];
#pragma unroll
    for (int e = 0; e < ND; ++e) {
      const int32_t d = dd[e];
      if (d != 0 && d != -1 && d != 1) xv[j][e] = x[min(max(rc + d, 0), nrows - 1)];
    }
  }
  double s[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double xm = __shfl_up(xr[j], 1, 64), xp = __shfl_down(xr[j], 1, 64);
    if (lane == 0) xm = (r >= 1 && r - 1 < nrows) ? x[r - 1] : 0.0;
    if (lane == 63) xp = (r + 1 < nrows) ? x[r + 1] : 0.0;
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) m |= 1u << c;
    }
    s[j] = 0.0;
#pragma unroll
    for (int e = 0; e < ND; ++e) {
      const int32_t d = dd[e];
      double v;
      if (d == 0) v = xr[j];
      else if (d == -1) v = xm;
      else if (d == 1) v = xp;
      else v = xv[j][e];
      if ((m >> e) & 1) s[j] = s[j] + dv[e] * v;
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    if (r < nrows) st_nt(y + r, s[j]);
  }
}


// --- dpair: dictionary-ordered (deltas wave-uniform, ascending = CSR order) over
// PAIRS of consecutive rows per lane: one 16-byte load at x + r + d (8-byte aligned;
// clamped into [0, nrows-2], the element picked by select) serves both rows' entry d,
// and one 16-byte code load both rows' codes.  VMEM per row pair: 1 + ndict (base: 2 + 2W).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int P, int ND>
__global__ __launch_bounds__(kT) void k_dpair(int32_t nrows, const uint8_t* __restrict__ code8,
                                              const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                              int ndict, const double* __restrict__ x, double* __restrict__ y) {
  const int t = threadIdx.x;
  const int32_t r0 = (int32_t)blockIdx.x * (2 * kT * P);
  int32_t dd[ND];
  double dv[ND];
#pragma unroll
  for (int e = 0; e < ND; ++e) {
    dd[e] = e < ndict ? ddelta[e] : 0;
    dv[e] = e < ndict ? dval[e] : 0.0;
  }
  uint32_t ma[P], mb[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int32_t r = r0 + 2 * (t + kT * k);
    u32x4 cw = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    if (r < nrows) cw = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(code8 + (size_t)r * 8));
    if (r + 1 >= nrows) cw.z = cw.w = 0xFFFFFFFFu;
    uint32_t a = 0, b = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int ca = ((q < 4 ? cw.x : cw.y) >> (8 * (q & 3))) & 255;
      const int cb = ((q < 4 ? cw.z : cw.w) >> (8 * (q & 3))) & 255;
      if (ca != 255) a |= 1u << ca;
      if (cb != 255) b |= 1u << cb;
    }
    ma[k] = a;
    mb[k] = b;
  }
  double xa[P][ND], xb[P][ND];
#pragma unroll
  for (int e = 0; e < ND; ++e) {
    if (e < ndict) {
      const int32_t d = dd[e];
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int32_t r = r0 + 2 * (t + kT * k);
        const int32_t a = r + d, ac = min(max(a, 0), nrows - 2);
        double2 q = make_double2(0.0, 0.0);
        if (((ma[k] | mb[k]) >> e) & 1) q = *reinterpret_cast<const double2*>(x + ac);
        xa[k][e] = ac == a ? q.x : q.y;
        xb[k][e] = ac == a ? q.y : q.x;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int32_t r = r0 + 2 * (t + kT * k);
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int e = 0; e < ND; ++e) {
      if ((ma[k] >> e) & 1) sa = sa + dv[e] * xa[k][e];
      if ((mb[k] >> e) & 1) sb = sb + dv[e] * xb[k][e];
    }
    if (r + 1 < nrows) __builtin_nontemporal_store(dx2{sa, sb}, reinterpret_cast<dx2*>(y + r));
    else if (r < nrows) st_nt(y + r, sa);
  }
}


// --- zm: stencil-aware marching.  The dictionary is the box stencil's seven pairs in the
// order (-P, -n, -1, 0, +1, +n, +P) (the host checks it), so each code names a fixed neighbour.
// A workgroup owns a 256-wide x segment of one y line and marches Z planes in z: x(z-1), x(z)
// and x(z+1) stay in registers, x(y+-1) are two coalesced loads, x(i+-1) come from the
// segment's values in LDS (edges loaded by the end lanes).  No gathers; per row: codes,
// 3 coalesced x loads, 1 store.  Same products in CSR order: bitwise.
template <int Z>
__global__ __launch_bounds__(kT) void k_zm(int nx, int ny, int nz, const uint8_t* __restrict__ code8,
                                           const double* __restrict__ dval, const double* __restrict__ x,
                                           double* __restrict__ y, int xwin = 0) {
  __shared__ double sx[kT + 2];
  const int t = threadIdx.x;
  const int nseg = nx / kT;
  int bid = (int)blockIdx.x;
  if (xwin > 0) {  // XCD x (blockIdx % 8) takes a contiguous run of xwin blocks in each window of 8*xwin
    const int span = 8 * xwin, full = (int)(gridDim.x / (unsigned)span) * span;
    if (bid < full) {
      const int w = bid / span, rem = bid - w * span;
      bid = w * span + (rem & 7) * xwin + (rem >> 3);
    }
  }
  const int seg = bid % nseg, yl = (bid / nseg) % ny, zt = bid / (nseg * ny);
  const int z0 = zt * Z, z1 = min(z0 + Z, nz);
  const int i = seg * kT + t;
  const int64_t P = (int64_t)nx * ny;
  double v[7];
#pragma unroll
  for (int e = 0; e < 7; ++e) v[e] = dval[e];
  const int64_t rl = i + (int64_t)yl * nx;   // row offset within a plane
  double xm = z0 > 0 ? x[rl + (z0 - 1) * P] : 0.0;
  double xc = x[rl + z0 * P];
  for (int z = z0; z < z1; ++z) {
    const int64_t r = rl + z * P;
    const u32x2 cw = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r);
    const double xp = z + 1 < nz ? x[r + P] : 0.0;
    const double xs = yl > 0 ? x[r - nx] : 0.0;
    const double xn = yl < ny - 1 ? x[r + nx] : 0.0;
    double el = 0.0, er = 0.0;
    if (t == 0 && i > 0) el = x[r - 1];
    if (t == kT - 1 && i + 1 < nx) er = x[r + 1];
    __syncthreads();               // the previous step's reads of sx are done
    sx[t + 1] = xc;
    if (t == 0) sx[0] = el;
    if (t == kT - 1) sx[kT + 1] = er;
    __syncthreads();
    const double xl = sx[t], xr = sx[t + 2];
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw, q);
      if (c != 255) m |= 1u << c;
    }
    double s = 0.0;
    if (m & 1) s = s + v[0] * xm;
    if (m & 2) s = s + v[1] * xs;
    if (m & 4) s = s + v[2] * xl;
    if (m & 8) s = s + v[3] * xc;
    if (m & 16) s = s + v[4] * xr;
    if (m & 32) s = s + v[5] * xn;
    if (m & 64) s = s + v[6] * xp;
    st_nt(y + r, s);
    xm = xc;
    xc = xp;
  }
}


// --- zmp: k_zm with the next plane's loads (codes, the y+-1 lines, x(z+2), the segment
// edges) issued before the current plane is summed, and the LDS row in two buffers (one
// barrier per plane): the march keeps one plane of loads in flight.
template <int Z>
__global__ __launch_bounds__(kT) void k_zmp(int nx, int ny, int nz, const uint8_t* __restrict__ code8,
                                            const double* __restrict__ dval, const double* __restrict__ x,
                                            double* __restrict__ y, int xwin = 0) {
  __shared__ double sx[2][kT + 2];
  const int t = threadIdx.x;
  const int nseg = nx / kT;
  int bid = (int)blockIdx.x;
  if (xwin > 0) {
    const int span = 8 * xwin, full = (int)(gridDim.x / (unsigned)span) * span;
    if (bid < full) {
      const int w = bid / span, rem = bid - w * span;
      bid = w * span + (rem & 7) * xwin + (rem >> 3);
    }
  }
  const int seg = bid % nseg, yl = (bid / nseg) % ny, zt = bid / (nseg * ny);
  const int z0 = zt * Z, z1 = min(z0 + Z, nz);
  const int i = seg * kT + t;
  const int64_t P = (int64_t)nx * ny;
  double v[7];
#pragma unroll
  for (int e = 0; e < 7; ++e) v[e] = dval[e];
  const int64_t rl = i + (int64_t)yl * nx;
  const bool hs = yl > 0, hn = yl < ny - 1, hl = t == 0 && i > 0, hr = t == kT - 1 && i + 1 < nx;
  auto load = [&](int z, u32x2& cw, double& xs, double& xn, double& xp, double& el, double& er) {
    const int64_t r = rl + z * P;
    cw = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r);
    xs = hs ? x[r - nx] : 0.0;
    xn = hn ? x[r + nx] : 0.0;
    xp = z + 1 < nz ? x[r + P] : 0.0;
    el = hl ? x[r - 1] : 0.0;
    er = hr ? x[r + 1] : 0.0;
  };
  double xm = z0 > 0 ? x[rl + (z0 - 1) * P] : 0.0;
  double xc = x[rl + z0 * P];
  u32x2 cw;
  double xs, xn, xp, el, er;
  load(z0, cw, xs, xn, xp, el, er);
  for (int z = z0; z < z1; ++z) {
    u32x2 cwN = cw;
    double xsN = 0.0, xnN = 0.0, xpN = 0.0, elN = 0.0, erN = 0.0;
    if (z + 1 < z1) load(z + 1, cwN, xsN, xnN, xpN, elN, erN);
    const int b = z & 1;
    sx[b][t + 1] = xc;
    if (t == 0) sx[b][0] = el;
    if (t == kT - 1) sx[b][kT + 1] = er;
    __syncthreads();
    const double xl = sx[b][t], xr = sx[b][t + 2];
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw, q);
      if (c != 255) m |= 1u << c;
    }
    double s = 0.0;
    if (m & 1) s = s + v[0] * xm;
    if (m & 2) s = s + v[1] * xs;
    if (m & 4) s = s + v[2] * xl;
    if (m & 8) s = s + v[3] * xc;
    if (m & 16) s = s + v[4] * xr;
    if (m & 32) s = s + v[5] * xn;
    if (m & 64) s = s + v[6] * xp;
    st_nt(y + rl + z * P, s);
    xm = xc;
    xc = xp;
    cw = cwN;
    xs = xsN;
    xn = xnN;
    xp = xpN;
    el = elN;
    er = erN;
  }
}

// --- zt: z-march over a tile of L y lines (256-wide x segment): the tile's lines in LDS,
// so x(y-+1) of interior lines come from LDS and only the two halo lines are loaded.
template <int L, int Z>
__global__ __launch_bounds__(kT) void k_zt(int nx, int ny, int nz, const uint8_t* __restrict__ code8,
                                           const double* __restrict__ dval, const double* __restrict__ x,
                                           double* __restrict__ y, int xwin) {
  __shared__ double sx[L + 2][kT + 2];
  const int t = threadIdx.x;
  const int nseg = nx / kT, nyt = (ny + L - 1) / L;
  int bid = (int)blockIdx.x;
  if (xwin > 0) {
    const int span = 8 * xwin, full = (int)(gridDim.x / (unsigned)span) * span;
    if (bid < full) {
      const int w = bid / span, rem = bid - w * span;
      bid = w * span + (rem & 7) * xwin + (rem >> 3);
    }
  }
  const int seg = bid % nseg, yt = (bid / nseg) % nyt, zt = bid / (nseg * nyt);
  const int y0 = yt * L, z0 = zt * Z, z1 = min(z0 + Z, nz);
  const int i = seg * kT + t;
  const int64_t P = (int64_t)nx * ny;
  double v[7];
#pragma unroll
  for (int e = 0; e < 7; ++e) v[e] = dval[e];
  double xm[L], xc[L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const bool ok = y0 + l < ny;
    const int64_t rl = i + (int64_t)(y0 + l) * nx;
    xm[l] = ok && z0 > 0 ? x[rl + (z0 - 1) * P] : 0.0;
    xc[l] = ok ? x[rl + z0 * P] : 0.0;
  }
  const bool hs = y0 > 0, hn = y0 + L < ny;
  for (int z = z0; z < z1; ++z) {
    u32x2 cw[L];
    double xp[L], el[L], er[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      const bool ok = y0 + l < ny;
      const int64_t r = i + (int64_t)(y0 + l) * nx + z * P;
      cw[l] = ok ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r) : u32x2{~0u, ~0u};
      xp[l] = ok && z + 1 < nz ? x[r + P] : 0.0;
      el[l] = ok && t == 0 && i > 0 ? x[r - 1] : 0.0;
      er[l] = ok && t == kT - 1 && i + 1 < nx ? x[r + 1] : 0.0;
    }
    const int64_t rb = i + (int64_t)y0 * nx + z * P;
    const double hsv = hs ? x[rb - nx] : 0.0;
    const double hnv = hn ? x[rb + (int64_t)L * nx] : 0.0;
    __syncthreads();
    sx[0][t + 1] = hsv;
    sx[L + 1][t + 1] = hnv;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      sx[l + 1][t + 1] = xc[l];
      if (t == 0) sx[l + 1][0] = el[l];
      if (t == kT - 1) sx[l + 1][kT + 1] = er[l];
    }
    __syncthreads();
#pragma unroll
    for (int l = 0; l < L; ++l) {
      if (y0 + l >= ny) continue;
      uint32_t m = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = cbyte(cw[l], q);
        if (c != 255) m |= 1u << c;
      }
      const double xq[7] = {xm[l], sx[l][t + 1], sx[l + 1][t], xc[l], sx[l + 1][t + 2], sx[l + 2][t + 1], xp[l]};
      double s = 0.0;
#pragma unroll
      for (int e = 0; e < 7; ++e)
        if (m & (1u << e)) s = s + v[e] * xq[e];
      st_nt(y + i + (int64_t)(y0 + l) * nx + z * P, s);
    }
#pragma unroll
    for (int l = 0; l < L; ++l) {
      xm[l] = xc[l];
      xc[l] = xp[l];
    }
  }
}

// block order remap: XCD x (blockIdx % 8) takes the blocks of its eighth of a z-window
template <int RPL>
__global__ __launch_bounds__(kT) void k_basex(int32_t nrows, const uint8_t* __restrict__ code8,
                                              const int32_t* __restrict__ ddelta, const double* __restrict__ dval,
                                              int ndict, const double* __restrict__ x, double* __restrict__ y,
                                              int32_t win) {
  __shared__ int32_t sdel[256];
  __shared__ double sval[256];
  const int t = threadIdx.x;
  // blocks in windows of 8*win: XCD x gets the x-th contiguous run of win blocks of each window
  const int32_t i = blockIdx.x, wdw = i / (8 * win), rem = i - wdw * 8 * win;
  const int32_t blk = wdw * 8 * win + (rem & 7) * win + (rem >> 3);
  const int32_t r0 = blk * (kT * RPL);
  u32x2 cw[RPL];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    cw[j] = r < nrows ? __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(code8) + r)
                      : u32x2{0xFFFFFFFFu, 0xFFFFFFFFu};
  }
  if (t < ndict) {
    sdel[t] = ddelta[t];
    sval[t] = dval[t];
  }
  __syncthreads();
  double xv[RPL][8];
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      xv[j][q] = c != 255 ? x[r + sdel[c]] : 0.0;
    }
  }
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    const int32_t r = r0 + t + kT * j;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = cbyte(cw[j], q);
      if (c != 255) s = s + sval[c] * xv[j][q];
    }
    if (r < nrows) st_nt(y + r, s);
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int64_t N = (int64_t)n * n * n;
  uint8_t* code8;
  int32_t* ddelta;
  double *dval, *x, *y;
  CK(hipMalloc(&code8, N * 8 + 16));
  CK(hipMalloc(&ddelta, 256 * 4));
  CK(hipMalloc(&dval, 256 * 8));
  CK(hipMalloc(&x, N * 8 + 4096));
  CK(hipMalloc(&y, N * 8 + 4096));
  const int32_t P = n * n;
  const int32_t hd[7] = {-P, -n, -1, 0, 1, n, P};
  const double hv[7] = {-1.0, -1.0, -1.0, 6.0, -1.0, -1.0, -1.0};
  CK(hipMemcpy(ddelta, hd, sizeof(hd), hipMemcpyHostToDevice));
  CK(hipMemcpy(dval, hv, sizeof(hv), hipMemcpyHostToDevice));
  k_codes<<<(unsigned)((N + 255) / 256), 256>>>(n, code8);
  k_randx<<<(unsigned)((N + 255) / 256), 256>>>(N, x);
  CK(hipDeviceSynchronize());
  const double bytes = 24.0 * N;
  std::vector<double> hy(N), hy0(N);
  const unsigned g4 = (unsigned)((N + 1023) / 1024), g2 = (unsigned)((N + 511) / 512), g1 = (unsigned)((N + 255) / 256);
  k_base<4><<<g4, kT>>>((int32_t)N, code8, ddelta, dval, 7, x, y);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hy0.data(), y, N * 8, hipMemcpyDeviceToHost));
  printf("{\"n\": %d, \"alg_bytes\": %.0f, \"results\": {", n, bytes);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  bool first = true;
  int round_ = 0;
  auto run = [&](const char* name, auto launch, bool check) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipMemset(y, 0, N * 8));
    float ms = 0;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const char* eq = "null";
    if (check) {
      CK(hipMemcpy(hy.data(), y, N * 8, hipMemcpyDeviceToHost));
      eq = memcmp(hy.data(), hy0.data(), N * 8) == 0 ? "true" : "false";
    }
    printf("%s\"%s/%d\": {\"us\": %.1f, \"GBps\": %.1f, \"bitwise\": %s}", first ? "" : ", ", name, round_, us,
           bytes / (us * 1e-6) / 1e9, eq);
    first = false;
    fflush(stdout);
  };
  for (round_ = 0; round_ < 3; ++round_) {
    run("base4", [&] { k_base<4><<<g4, kT>>>((int32_t)N, code8, ddelta, dval, 7, x, y); }, true);
    run("base2", [&] { k_base<2><<<g2, kT>>>((int32_t)N, code8, ddelta, dval, 7, x, y); }, true);

    {
      const int nseg = n / kT;
      for (int Z : {16}) {
        const unsigned gz = (unsigned)(nseg * n * ((n + Z - 1) / Z));
        for (int xw : {32}) {
          char nm[32];
          snprintf(nm, sizeof(nm), "zm%d_x%d", Z, xw);
          if (Z == 8) run(nm, [&] { k_zm<8><<<gz, kT>>>(n, n, n, code8, dval, x, y, xw); }, true);
          if (Z == 16) run(nm, [&] { k_zm<16><<<gz, kT>>>(n, n, n, code8, dval, x, y, xw); }, true);
        }
      }
      for (int Lq : {2, 4, 8}) {
        const unsigned gz = (unsigned)(nseg * ((n + Lq - 1) / Lq) * ((n + 15) / 16));
        for (int xw : {8, 32}) {
          char nm[32];
          snprintf(nm, sizeof(nm), "zt%d_x%d", Lq, xw);
          if (Lq == 2) run(nm, [&] { k_zt<2, 16><<<gz, kT>>>(n, n, n, code8, dval, x, y, xw); }, true);
          if (Lq == 4) run(nm, [&] { k_zt<4, 16><<<gz, kT>>>(n, n, n, code8, dval, x, y, xw); }, true);
          if (Lq == 8) run(nm, [&] { k_zt<8, 16><<<gz, kT>>>(n, n, n, code8, dval, x, y, xw); }, true);
        }
      }
    }
    run("dpair2", [&] { k_dpair<2, 8><<<g4, kT>>>((int32_t)N, code8, ddelta, dval, 7, x, y); }, true);

    run("noxg4", [&] { k_noxg<4><<<g4, kT>>>((int32_t)N, code8, ddelta, dval, 7, x, y); }, false);
    if (g4 % 64 == 0) {
      run("basex4_w8", [&] { k_basex<4><<<g4, kT>>>((int32_t)N, code8, ddelta, dval, 7, x, y, 8); }, true);
      }
  }
  printf("}}\n");
  return 0;
}
