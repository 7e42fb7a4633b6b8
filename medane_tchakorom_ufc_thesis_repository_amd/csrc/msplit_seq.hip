// msplit_seq.hip -- the parity reduction order, MSP_REDUCE_SEQ (include/msplit.h).
//
// PETSc's Seq kernels form every reduction as one running sum with the
// elements in index order:
//   VecDot_Seq / VecNorm_Seq (NORM_2)  BLASdot = f2cblaslapack ddot (the
//                                      reference's --download-f2cblaslapack,
//                                      config/petsc/arch-linux-mpich-g5k-opt.py);
//                                      its unroll-by-5 body is evaluated left to
//                                      right, i.e. still sequential
//   VecMDot_Seq                        per vector, sequential
//   MatMultTranspose_SeqDense          dgemv 'T': per column, sequential
//   MatNorm_SeqDense NORM_FROBENIUS    a plain sum of squares over the
//                                      column-major array (BLASnrm2 only under
//                                      PETSC_USE_REAL___FP16), then sqrt
// and the reference's outer LSQR runs on one rank over the whole of R
// (SMSM-global.c:136, comm_jacobi_block with one process per block), so its
// sums run across the row blocks in block order.  oracle/oracle.c's
// ORC_REDUCE_SEQ restates exactly this: s = fl(s + p_i), s_0 = +0.0, in index
// order, p_i = x_i * (y_i * sy) (or x_i * x_i).
//
// Results go out in the DBR partial layout -- partial[v*nchunks + 0] = the
// sum, the other chunks +0.0 -- so the unchanged stage 2 (or the fused GMRES
// norm/Hessenberg update) folds them to exactly the sequential sum: x + (+0.0)
// == x for every x a sum of products starting at +0.0 can produce.
//
// Two engines compute the same bits.
//
// The serial engine (k_seq_stage1; MSPLIT_SEQ_ENGINE=serial): the products are
// formed by the whole workgroup into LDS, and one lane adds them in order
// while the other waves form the next tile.  16.7 M terms cost ~56 ms: one
// dependent f64 add per term.
//
// The exact parallel engine (default, mspi_seq_stage1).  While the running
// sum s stays inside one binade [2^e, 2^(e+1)) of one sign, every double it can
// take is M * u, u = 2^(e-52), M an integer in [2^52, 2^53), and fl(s + p)
// = (M + inc) * u with inc = floor(p/u) + [frac(p/u) > 1/2], a tie (frac ==
// 1/2) rounding to the even M.  So a run of terms acts on M as an integer
// translation whose only dependence on M is M's parity (through ties; after a
// tie M is even whatever it was), valid while every exact sum stays >= 2^e and
// every rounded one < 2^(e+1).  A run's "transducer" is therefore, per input
// parity, the offset D, the lowest exact sum LO and the highest result HI
// (all in units of u), and transducers of one binade compose associatively.
// Three passes build and apply them:
//   1. approximate chunk sums (the DBR stage 1) and their exclusive prefix --
//      a guess of s at each 4096-term segment, used only to pick the binade;
//   2. k_seqx_trans: per 64-term sub-segment the transducer in the binade its
//      guessed start lies in (integer arithmetic on the terms' bits, exact),
//      and per segment their composition (BAD where the subs disagree);
//   3. k_seqx_ripwalk, one workgroup per sum (round 5): from s = +0.0, the
//      maps of a window of 64 segments applied in order as a ripple through
//      the wave (lane j adds its map's offset to lane j-1's previous result,
//      DPP wave_shr:1, one verdict per lane at the end), up to the first that
//      does not apply at the actual s; that segment's 64 sub maps likewise;
//      a sub that does not apply is added term by term by the f64 add (the
//      one term that leaves the binade, ties, zeros, subnormals and
//      non-finite values included), and the ripple resumes after it.
//      k_seqx_walk (MSPLIT_SEQ_WALK=scan, rounds 4-5) composes the window's
//      maps in a wave scan and applies subs one record at a time instead.
// Every step either is the f64 add or provably equals it, so the result is the
// sequential sum bit for bit whatever the guesses were; the guesses only
// decide how often the walk descends.  GMRES's dots at 256^3 descend into at
// most a few hundred of 4096 segments, and add ~1400 of 262144 subs serially.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>

#include "msplit_ctx.hpp"

namespace {

constexpr int kT = 256;      // threads per workgroup
constexpr int kTile = 2048;  // products per LDS tile

__device__ __forceinline__ bool stopped(const int* stop) { return stop && *stop; }

// One segment: x[i] * (y[i] * sy) (y == nullptr: x[i] * x[i]), added to acc in
// index order.  Wave 0 lane 0 sums; waves 1..3 form the next tile meanwhile.
__device__ double seq_segment(const double* __restrict__ x, const double* __restrict__ y, double sy, int64_t n,
                              double acc, double (*buf)[kTile]) {
  const int t = threadIdx.x;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  auto fill = [&](int64_t tile, double* dst, int t0, int nt) {
    const int64_t base = tile * kTile;
    const int cnt = (int)((n - base) < kTile ? (n - base) : kTile);
    for (int i = t0; i < cnt; i += nt) {
      const double xi = x[base + i];
      dst[i] = y ? xi * (y[base + i] * sy) : xi * xi;
    }
  };
  if (ntiles > 0) fill(0, buf[0], t, kT);
  __syncthreads();
  for (int64_t tile = 0; tile < ntiles; ++tile) {
    if (t >= 64) {
      if (tile + 1 < ntiles) fill(tile + 1, buf[(tile + 1) & 1], t - 64, kT - 64);
    } else if (t == 0) {
      const double* p = buf[tile & 1];
      const int64_t base = tile * kTile;
      const int cnt = (int)((n - base) < kTile ? (n - base) : kTile);
      int i = 0;
      for (; i + 32 <= cnt; i += 32) {
        double q[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) q[u] = p[i + u];
#pragma unroll
        for (int u = 0; u < 32; ++u) acc = acc + q[u];
      }
      for (; i < cnt; ++i) acc = acc + p[i];
    }
    __syncthreads();
  }
  return acc;
}

// Workgroup v: w . V_v (self: w . w) in sequential order, written in the DBR
// partial layout of row v.
__global__ __launch_bounds__(kT) void k_seq_stage1(const double* __restrict__ w, Vecs V, int64_t n, int self,
                                                   double* __restrict__ partial, int64_t nchunks,
                                                   const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double buf[2][kTile];
  const int v = blockIdx.x;
  const double* y = self ? nullptr : (V.base ? V.base + (int64_t)v * V.stride : V.p[v]);
  const double sy = (!self && V.scale) ? V.scale[v] : 1.0;
  const double acc = seq_segment(w, y, sy, n, 0.0, buf);
  double* row = partial + (int64_t)v * nchunks;
  for (int64_t c = threadIdx.x; c < nchunks; c += kT) row[c] = c == 0 ? acc : 0.0;
}

// Chained sums over the row blocks of one process (LSQR): workgroup j sums
// column_j . y over segment 0, then segment 1, ... (frob: one workgroup, the
// squares of column 0 over all segments, then column 1, ...).
__global__ __launch_bounds__(kT) void k_seq_chain(mspi_seq_segs sg, int ncol, int frob, double* __restrict__ out,
                                                  int m, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double buf[2][kTile];
  const int j = blockIdx.x;
  double acc = 0.0;
  const int j0 = frob ? 0 : j, j1 = frob ? ncol : j + 1;
  for (int jj = j0; jj < j1; ++jj)
    for (int k = 0; k < sg.nseg; ++k) {
      const double* x = sg.x[k] + (int64_t)jj * sg.ldx[k];
      acc = seq_segment(x, frob ? nullptr : sg.y[k], 1.0, sg.n[k], acc, buf);
    }
  if (threadIdx.x != 0) return;
  // only the last block's slot carries the sum: a block-order sum of the slots is the chain
  if (frob) {
    for (int k = 0; k < sg.nseg; ++k)
      for (int jj = 0; jj < ncol; ++jj) out[k * m + jj] = (k == sg.nseg - 1 && jj == ncol - 1) ? acc : 0.0;
  } else {
    for (int k = 0; k < sg.nseg; ++k) out[k * m + j] = k == sg.nseg - 1 ? acc : 0.0;
  }
}


// ------------------------------------------------------------ exact parallel engine
constexpr int kSeg = MSK_DBR_CHUNK;  // one segment = one DBR chunk (its partial is the guess)
constexpr int kSub = 64;             // terms per sub-segment (one per lane in the walk)
constexpr int kSubs = kSeg / kSub;
constexpr int kPer = kSeg / kT;      // contiguous terms per thread in k_seqx_trans
constexpr double kM0 = 4503599627370496.0, kM1 = 9007199254740992.0;  // 2^52, 2^53
constexpr double kLim = 4503599627370496.0, kBig = 1152921504606846976.0;  // 2^52 (a valid run's offsets are below), 2^60
constexpr uint64_t kFrac = (uint64_t(1) << 52) - 1;
constexpr uint32_t F_NEG = 1, F_BAD = 2, F_ZERO = 4, F_NZERO = 8;

// A run of terms as a map of the state M (s = +-M * 2^(e-52)): for input parity pi, M -> M + d[pi], valid iff
// M + lo[pi] >= 2^52 (every exact sum >= 2^e) and M + hi[pi] < 2^53 (every result < 2^(e+1)).  F_ZERO: every term
// is +-0 (identity; F_NZERO: all -0.0, so a -0.0 state stays -0.0); F_BAD: not a translation of one binade.
// The offsets are integers held in f64: exact below 2^53, and a valid run's are below 2^52 in magnitude (a sum that
// leaves that range marks the run BAD); +-2^60 stand for "no bound" and stay beyond 2^53 whatever is added to them.
struct alignas(16) Tr {  // scalar fields, no arrays: a select between two of them must not become a private index
  double d0, d1, lo0, lo1, hi0, hi1;
  int32_t e;
  uint32_t fl;
  int64_t pad;
};
static_assert(sizeof(Tr) == 64, "Tr is one 64-byte record");

__device__ __forceinline__ Tr tr_ident() {
  Tr t;
  t.d0 = t.d1 = 0.0;
  t.lo0 = t.lo1 = kBig;
  t.hi0 = t.hi1 = -kBig;
  t.e = 0;
  t.fl = F_ZERO | F_NZERO;
  t.pad = 0;
  return t;
}

__device__ __forceinline__ Tr tr_bad() {
  Tr t = tr_ident();
  t.fl = F_BAD;
  return t;
}

// p / 2^(e-52), sign-flipped when the state is negative, as q = floor and the fraction's class c (0: < 1/2,
// 1: == 1/2, 2: > 1/2); false for a non-finite p or |p| >= 2^(e+1).  In f64: a = |p| * 2^(52-e) is exact (ldexp;
// an underflow only loses bits far below 1/2), its floor and fraction are exact, and the class is read from the
// fraction of |p|'s scaled value, never from 1 - f (which can round onto 1/2).  tests/test_seq_engine_math.py
// holds it to the integer decomposition of p's bits.
__device__ __forceinline__ bool decomp_f(double p, int e, uint32_t sneg, double& q, int& c) {
  q = 0.0;
  c = 0;
  if (!isfinite(p)) return false;
  const double a = ldexp(fabs(p), 52 - e);
  if (a >= 9007199254740992.0) return false;  // |p| >= 2^(e+1)
  const double qa = floor(a), fa = a - qa;
  const bool neg = (signbit(p) ? 1u : 0u) != sneg;
  if (!neg) {
    q = qa;
    c = fa > 0.5 ? 2 : (fa == 0.5 ? 1 : 0);
  } else if (fa == 0.0) {
    q = -qa;
  } else {
    q = -qa - 1.0;
    c = fa < 0.5 ? 2 : (fa == 0.5 ? 1 : 0);
  }
  return true;
}

// field by field (a select of whole records becomes a private-memory copy)
__device__ __forceinline__ Tr tr_sel(bool c, const Tr& a, const Tr& b) {
  Tr r;
  r.d0 = c ? a.d0 : b.d0;
  r.d1 = c ? a.d1 : b.d1;
  r.lo0 = c ? a.lo0 : b.lo0;
  r.lo1 = c ? a.lo1 : b.lo1;
  r.hi0 = c ? a.hi0 : b.hi0;
  r.hi1 = c ? a.hi1 : b.hi1;
  r.e = c ? a.e : b.e;
  r.fl = c ? a.fl : b.fl;
  r.pad = 0;
  return r;
}

__device__ __forceinline__ double dbl(int lo, int hi) {
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ Tr tr_load(const Tr* p) {
  const int4* q = reinterpret_cast<const int4*>(p);
  const int4 a = q[0], b = q[1], c = q[2], d = q[3];
  Tr r;
  r.d0 = dbl(a.x, a.y);
  r.d1 = dbl(a.z, a.w);
  r.lo0 = dbl(b.x, b.y);
  r.lo1 = dbl(b.z, b.w);
  r.hi0 = dbl(c.x, c.y);
  r.hi1 = dbl(c.z, c.w);
  r.e = d.x;
  r.fl = (uint32_t)d.y;
  r.pad = 0;
  return r;
}

// c ? x1 : x0 as integer arithmetic on the bit patterns: a select of two loaded fields would be folded into a
// select of their addresses, and the record would go to private memory
__device__ __forceinline__ int64_t pick(bool c, int64_t x1, int64_t x0) { return x0 + (c ? x1 - x0 : 0); }
__device__ __forceinline__ double pickd(bool c, double x1, double x0) {
  return __longlong_as_double(pick(c, __double_as_longlong(x1), __double_as_longlong(x0)));
}

__device__ __forceinline__ double clampb(double v) { return fmin(fmax(v, -kBig), kBig); }

// an integer-valued f64 below 2^53 is odd
__device__ __forceinline__ bool odd(double x) {
  const double h = 0.5 * x;
  return h != floor(h);
}

// a, then b
__device__ __forceinline__ Tr tr_comb(const Tr& a, const Tr& b) {
  if (a.fl & F_ZERO) {
    Tr r = b;
    if (!(a.fl & F_NZERO)) r.fl &= ~F_NZERO;
    return r;
  }
  if (b.fl & F_ZERO) return a;
  Tr r;
  r.e = a.e;
  r.pad = 0;
  r.fl = ((a.fl | b.fl) & F_BAD) | (a.fl & F_NEG);
  if (a.e != b.e || ((a.fl ^ b.fl) & F_NEG)) r.fl |= F_BAD;
  // input parity 0 leaves a with parity (a.d0 & 1), input parity 1 with ((1 + a.d1) & 1)
  const bool q0 = odd(a.d0), q1 = !odd(a.d1);
  double d0 = a.d0 + pickd(q0, b.d1, b.d0), d1 = a.d1 + pickd(q1, b.d1, b.d0);
  r.lo0 = clampb(fmin(a.lo0, a.d0 + pickd(q0, b.lo1, b.lo0)));
  r.lo1 = clampb(fmin(a.lo1, a.d1 + pickd(q1, b.lo1, b.lo0)));
  r.hi0 = clampb(fmax(a.hi0, a.d0 + pickd(q0, b.hi1, b.hi0)));
  r.hi1 = clampb(fmax(a.hi1, a.d1 + pickd(q1, b.hi1, b.hi0)));
  if (fabs(d0) > kLim || fabs(d1) > kLim) {
    r.fl |= F_BAD;
    d0 = d1 = 0.0;
  }
  r.d0 = d0;
  r.d1 = d1;
  return r;
}

// s after the run, or false when the run is not known to be a translation at s
__device__ __forceinline__ bool tr_apply(const Tr& t, double s, double& out) {
  if (t.fl & F_ZERO) {
    out = s == 0.0 ? ((signbit(s) && (t.fl & F_NZERO)) ? -0.0 : 0.0) : s;
    return true;
  }
  if (t.fl & F_BAD) return false;
  const uint64_t b = (uint64_t)__double_as_longlong(s);
  const int E = (int)((b >> 52) & 0x7ff);
  if (E == 0 || E == 0x7ff) return false;
  if (E - 1023 != t.e || (uint32_t)(b >> 63) != (t.fl & F_NEG)) return false;
  const bool od = (b & 1) != 0;  // M's parity is its last fraction bit
  // M in [2^52, 2^53) as an f64: exponent 1075 over M's own fraction bits (no integer conversion)
  const double Md = __longlong_as_double((long long)((b & kFrac) | (uint64_t(0x433) << 52)));
  if (Md + pickd(od, t.lo1, t.lo0) < kM0 || Md + pickd(od, t.hi1, t.hi0) >= kM1) return false;
  const double Mn = Md + pickd(od, t.d1, t.d0);  // an integer in [2^52, 2^53): its fraction bits are M - 2^52
  out = __longlong_as_double((long long)((b & ~kFrac) | ((uint64_t)__double_as_longlong(Mn) & kFrac)));
  return true;
}

// tr_apply for a wave-uniform s and a per-lane map, without branches: every lane applies its own map to the same s
// (the walk's one-record applies: lane j's verdict comes from a ballot and its result from one readlane, instead of
// fourteen readlanes of lane j's record into scalar registers and a scalar apply).  Same verdict and result as
// tr_apply wherever that returns true.
__device__ __forceinline__ bool tr_apply_v(const Tr& t, double s, double& out) {
  const uint64_t b = (uint64_t)__double_as_longlong(s);
  const int E = (int)((b >> 52) & 0x7ff);
  const bool od = (b & 1) != 0;
  const double Md = __longlong_as_double((long long)((b & kFrac) | (uint64_t(0x433) << 52)));
  const bool inb = E != 0 && E != 0x7ff && E - 1023 == t.e && (uint32_t)(b >> 63) == (t.fl & F_NEG);
  const bool rng = Md + pickd(od, t.lo1, t.lo0) >= kM0 && Md + pickd(od, t.hi1, t.hi0) < kM1;
  const double Mn = Md + pickd(od, t.d1, t.d0);
  const double ot = __longlong_as_double((long long)((b & ~kFrac) | ((uint64_t)__double_as_longlong(Mn) & kFrac)));
  const double oz = s == 0.0 ? ((signbit(s) && (t.fl & F_NZERO)) ? -0.0 : 0.0) : s;
  const bool z = (t.fl & F_ZERO) != 0;
  out = z ? oz : ot;
  return z || (!(t.fl & F_BAD) && inb && rng);
}

// A map prepared for the one-record applies of the walk (round 5): in its binade e (u = 2^(e-52)) the map is valid at
// s iff |s| = M u lies in [L_p, H_p) -- L_p = max(2^52, 2^52 - lo_p) u, H_p = min(2^53, 2^53 - hi_p) u, every product
// exact (an integer below 2^61 times a power of two) -- and s has the map's sign; then |s| + d_p u is exact (its M + d
// lies in [2^52, 2^53)), so the result is one f64 add: a dozen mostly independent instructions where tr_apply_v
// decodes s's bits and rebuilds the result's.  BAD maps take L = +inf (never valid); zero maps the identity rule.
struct Prep {
  double L0, L1, H0, H1, D0, D1;
  uint32_t fl;
};

__device__ __forceinline__ Prep prep_of(const Tr& t) {
  Prep p;
  const int sh = t.e - 52;
  p.L0 = ldexp(fmax(kM0, kM0 - t.lo0), sh);
  p.L1 = ldexp(fmax(kM0, kM0 - t.lo1), sh);
  p.H0 = ldexp(fmin(kM1, kM1 - t.hi0), sh);
  p.H1 = ldexp(fmin(kM1, kM1 - t.hi1), sh);
  p.D0 = ldexp(t.d0, sh);
  p.D1 = ldexp(t.d1, sh);
  const bool bad = (t.fl & F_BAD) != 0;
  p.L0 = bad ? INFINITY : p.L0;
  p.L1 = bad ? INFINITY : p.L1;
  p.fl = t.fl;
  return p;
}

// tr_apply_v's verdict and result wherever that returns true (every lane its own prepared map at the same s)
__device__ __forceinline__ bool prep_apply(const Prep& p, double s, double& out) {
  const uint64_t b = (uint64_t)__double_as_longlong(s);
  const bool od = (b & 1) != 0;
  const bool neg = (b >> 63) != 0;
  const double a = fabs(s);
  const double L = pickd(od, p.L1, p.L0), H = pickd(od, p.H1, p.H0), D = pickd(od, p.D1, p.D0);
  const bool ok = a >= L && a < H && neg == ((p.fl & F_NEG) != 0);
  const double m = a + D;
  const double ot = neg ? -m : m;
  const double oz = s == 0.0 ? ((signbit(s) && (p.fl & F_NZERO)) ? -0.0 : 0.0) : s;
  const bool z = (p.fl & F_ZERO) != 0;
  out = z ? oz : ot;
  return z || ok;
}

__device__ __forceinline__ Tr shfl_xor_tr(const Tr& t, int m) {
  Tr r;
  r.d0 = __shfl_xor(t.d0, m);
  r.d1 = __shfl_xor(t.d1, m);
  r.lo0 = __shfl_xor(t.lo0, m);
  r.lo1 = __shfl_xor(t.lo1, m);
  r.hi0 = __shfl_xor(t.hi0, m);
  r.hi1 = __shfl_xor(t.hi1, m);
  r.e = __shfl_xor(t.e, m);
  r.fl = __shfl_xor(t.fl, m);
  r.pad = 0;
  return r;
}

__device__ __forceinline__ Tr shfl_down_tr(const Tr& t, int o) {
  Tr r;
  r.d0 = __shfl_down(t.d0, o);
  r.d1 = __shfl_down(t.d1, o);
  r.lo0 = __shfl_down(t.lo0, o);
  r.lo1 = __shfl_down(t.lo1, o);
  r.hi0 = __shfl_down(t.hi0, o);
  r.hi1 = __shfl_down(t.hi1, o);
  r.e = __shfl_down(t.e, o);
  r.fl = __shfl_down(t.fl, o);
  r.pad = 0;
  return r;
}

__device__ __forceinline__ Tr shfl_up_tr(const Tr& t, int o) {
  Tr r;
  r.d0 = __shfl_up(t.d0, o);
  r.d1 = __shfl_up(t.d1, o);
  r.lo0 = __shfl_up(t.lo0, o);
  r.lo1 = __shfl_up(t.lo1, o);
  r.hi0 = __shfl_up(t.hi0, o);
  r.hi1 = __shfl_up(t.hi1, o);
  r.e = __shfl_up(t.e, o);
  r.fl = __shfl_up(t.fl, o);
  r.pad = 0;
  return r;
}

// a wave-uniform copy of lane l's value (v_readlane into scalar registers: no LDS round trip)
__device__ __forceinline__ int64_t rl64(int64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double rld(double x, int l) { return __longlong_as_double(rl64(__double_as_longlong(x), l)); }
__device__ __forceinline__ const double* vec_row(const Vecs& V, int v) {
  return V.base ? V.base + (int64_t)v * V.stride : V.p[v];
}

// Row v of a (nv rows of K approximate chunk sums) -> its exclusive prefix: the guessed s at each segment start.
// Any order: a guess only picks the binade the transducers are built in.
__global__ __launch_bounds__(kT) void k_seqx_prefix(double* __restrict__ a, int64_t K, const double* __restrict__ acc_in,
                                                    const int* __restrict__ stop) {
  if (stopped(stop)) return;
  __shared__ double sh[kT];
  double* row = a + (int64_t)blockIdx.x * K;
  const int t = threadIdx.x;
  const int64_t per = (K + kT - 1) / kT, lo = min<int64_t>((int64_t)t * per, K), hi = min<int64_t>(lo + per, K);
  double sum = 0.0;
  for (int64_t i = lo; i < hi; ++i) sum += row[i];
  sh[t] = sum;
  __syncthreads();
  if (t == 0) {
    double run = acc_in ? acc_in[blockIdx.x] : 0.0;  // a chained sum starts where the previous piece ended
    for (int i = 0; i < kT; ++i) {
      const double v = sh[i];
      sh[i] = run;
      run += v;
    }
  }
  __syncthreads();
  double run = sh[t];
  for (int64_t i = lo; i < hi; ++i) {
    const double v = row[i];
    row[i] = run;
    run += v;
  }
}

// One segment's transducers for one sum, from its products the caller has staged in sp (thread t's term i at l + l/16,
// l = t + 256 i) and g0, the guessed sum at the segment's start: thread t's run of 16 terms, four threads to a
// sub-segment (sub_out[0..63]), the waves' trees and thread 0's composition to the segment (*seg_out).  Begins
// with a barrier.  cnt: thread t's terms inside n.
__device__ __forceinline__ void trans_segment(double* sp, double* ssum, Tr* str, double g0, int cnt,
                                              Tr* __restrict__ sub_out, Tr* __restrict__ seg_out) {
  const int t = threadIdx.x, lane = t & 63, j = t >> 2;
  __syncthreads();
  // the thread's 16 terms are read from LDS in each pass rather than held (three passes at most: the sum, track 0,
  // and track 1 where a tie needs it), which keeps the kernel at three waves per SIMD
  const double* mine = sp + t * (kPer + 1);
  double ps = 0.0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) ps += mine[i];
  ps += __shfl_xor(ps, 1);
  ps += __shfl_xor(ps, 2);
  if ((t & 3) == 0) ssum[j] = ps;
  __syncthreads();
  if (t < kSubs) {  // exclusive prefix of the sub sums (wave 0)
    const double a = ssum[t];
    double incl = a;
#pragma unroll
    for (int o = 1; o < kSubs; o <<= 1) {
      const double u = __shfl_up(incl, o);
      if (t >= o) incl += u;
    }
    ssum[t] = incl - a;
  }
  __syncthreads();
  const double G = g0 + ssum[j];
  const uint64_t gb = (uint64_t)__double_as_longlong(G);
  const int GE = (int)((gb >> 52) & 0x7ff);
  const bool gok = GE != 0 && GE != 0x7ff;
  const int e = GE - 1023;
  const uint32_t sneg = (uint32_t)(gb >> 63);
  // the lane's run, in f64 arithmetic on integer values (exact below 2^53; a run that leaves that range cannot
  // be valid and is marked BAD): every term decomposed (decomp_f) and input parity 0's track advanced in one pass;
  // parity 1's differs only through ties, so it is the same track unless the run holds one (then a second pass)
  Tr a = tr_ident();
  bool bad = false, tie = false;
  const double big = kBig;
  double d0 = 0.0, lo0 = big, hi0 = -big;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    if (i < cnt) {
      const double p = mine[i];
      const uint64_t b = (uint64_t)__double_as_longlong(p);
      if ((b << 1) == 0) {
        if (!(b >> 63)) a.fl &= ~F_NZERO;
      } else {
        if (a.fl & F_ZERO) {
          a.fl = sneg ? F_NEG : 0u;
          a.e = e;
        }
        double q = 0.0;
        int c = 0;
        if (!gok || !decomp_f(p, e, sneg, q, c)) bad = true;
        const double x = d0 + q;
        lo0 = fmin(lo0, x);
        d0 = x + (c == 2 ? 1.0 : 0.0) + (c == 1 ? x - 2.0 * floor(0.5 * x) : 0.0);  // a tie rounds to even
        hi0 = fmax(hi0, d0);
        tie |= c == 1;
      }
    }
  }
  if (!(a.fl & F_ZERO)) {
    double d1 = d0, lo1 = lo0, hi1 = hi0;
    if (tie) {
      d1 = 0.0;
      lo1 = big;
      hi1 = -big;
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        if (i < cnt) {
          const double p = mine[i];
          if (((uint64_t)__double_as_longlong(p) << 1) == 0) continue;
          double q = 0.0;
          int c = 0;
          if (gok) (void)decomp_f(p, e, sneg, q, c);
          const double x = d1 + q;
          lo1 = fmin(lo1, x);
          d1 = x + (c == 2 ? 1.0 : 0.0) + (c == 1 ? (x + 1.0) - 2.0 * floor(0.5 * (x + 1.0)) : 0.0);
          hi1 = fmax(hi1, d1);
        }
      }
    }
    const double lim = 4503599627370496.0;  // 2^52: every offset of a valid run is below this
    if (bad || fabs(d0) > lim || fabs(d1) > lim || (lo0 < big && fabs(lo0) > lim) ||
        (lo1 < big && fabs(lo1) > lim) || (hi0 > -big && fabs(hi0) > lim) || (hi1 > -big && fabs(hi1) > lim)) {
      a.fl |= F_BAD;
    } else {
      a.d0 = d0;
      a.d1 = d1;
      a.lo0 = lo0;
      a.lo1 = lo1;
      a.hi0 = hi0;
      a.hi1 = hi1;
    }
  }
  Tr o = shfl_xor_tr(a, 1);
  if ((t & 1) == 0) a = tr_comb(a, o);
  o = shfl_xor_tr(a, 2);
  if ((t & 3) == 0) {
    a = tr_comb(a, o);
    sub_out[j] = a;
  }
#pragma unroll
  for (int s = 4; s < 64; s <<= 1) {  // each wave: the ordered tree over its 16 subs (leaders 0, 4, .., 60)
    const Tr u = shfl_down_tr(a, s);
    if ((lane & (2 * s - 1)) == 0) a = tr_comb(a, u);
  }
  if (lane == 0) str[t >> 6] = a;
  __syncthreads();
  // no barrier after it: every read of sp and ssum is behind the barrier above, and str is next written three
  // barriers into the next sum, which thread 0 joins after this read
  if (t == 0) *seg_out = tr_comb(tr_comb(str[0], str[1]), tr_comb(str[2], str[3]));
}

// Workgroup k: segment k of every sum.  Thread t holds terms 16t..16t+15 of the segment (the products staged
// through LDS from coalesced loads); four threads make a sub-segment's transducer, wave 0 composes the 64 subs.
template <bool PF>
__device__ __forceinline__ void trans_block(int64_t k, const double* __restrict__ w, const Vecs& V, int nv, int64_t n,
                                            int self, const double* __restrict__ pre, Tr* __restrict__ segT,
                                            Tr* __restrict__ subT, int64_t K, double* sp, double* ssum, Tr* str) {
  const int t = threadIdx.x;
  const int64_t c0 = k * kSeg;
  const int cnt = (int)max<int64_t>(0, min<int64_t>(kPer, n - (c0 + (int64_t)kPer * t)));
  // sum v's w and y values, loaded one sum ahead (their round trip overlaps sum v - 1's transducers); w is the same
  // for every sum and re-read from the L2 each time rather than held, which keeps the kernel's registers down
  double wn[kPer], yn[kPer];
#define MSK_SEQX_LOAD(v_)                                        \
  do {                                                           \
    const double* y_ = self ? nullptr : vec_row(V, (v_));        \
    _Pragma("unroll") for (int i = 0; i < kPer; ++i) {           \
      const int64_t g = min<int64_t>(c0 + t + i * kT, n - 1);    \
      wn[i] = w[g];                                              \
      yn[i] = y_ ? y_[g] : 0.0;                                  \
    }                                                            \
  } while (0)
  if (PF) MSK_SEQX_LOAD(0);
  for (int v = 0; v < nv; ++v) {
    if (!PF) MSK_SEQX_LOAD(v);  // no loads in flight across the transducers: fewer registers, more waves
    const double sy = (!self && V.scale) ? V.scale[v] : 1.0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int64_t g = c0 + t + i * kT;
      const int l = t + i * kT;
      double p = 0.0;
      if (g < n) p = self ? wn[i] * wn[i] : wn[i] * (yn[i] * sy);
      sp[l + l / kPer] = p;
    }
    if (PF && v + 1 < nv) MSK_SEQX_LOAD(v + 1);
    trans_segment(sp, ssum, str, pre[(int64_t)v * K + k], cnt, subT + ((int64_t)v * K + k) * kSubs,
                  segT + (int64_t)v * K + k);
  }
#undef MSK_SEQX_LOAD
}

constexpr int kSpTrans = kSeg + kSeg / kPer;  // products, one pad slot per 16: thread t's run at 17t

// ready != nullptr (round 6, the overlapped launch): after its records, the workgroup publishes ready[k] = epoch for
// the walk that runs concurrently on the context's stream (ripwalk_sum's wait_ready).
// PF: the next sum's loads in flight during this sum's transducers (two waves per SIMD); else three waves per SIMD
template <bool PF>
__global__ __launch_bounds__(kT, PF ? 2 : 3) void k_seqx_trans(const double* __restrict__ w, Vecs V, int nv, int64_t n,
                                                   int self, const double* __restrict__ pre, Tr* __restrict__ segT,
                                                   Tr* __restrict__ subT, int64_t K, const int* __restrict__ stop,
                                                   uint32_t* ready, uint32_t epoch) {
  if (stopped(stop)) return;
  __shared__ double sp[kSpTrans];
  __shared__ double ssum[kSubs];
  __shared__ Tr str[kT / 64];
  trans_block<PF>(blockIdx.x, w, V, nv, n, self, pre, segT, subT, K, sp, ssum, str);
  if (!ready) return;
  __threadfence();  // every thread's records, at agent scope, before the flag
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(ready + blockIdx.x, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// Apply the longest prefix of the lanes' runs (lane order) that is valid at s; returns its length.
__device__ __forceinline__ int tr_walk(Tr t, double& s, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const Tr u = shfl_up_tr(t, o);
    if (lane >= o) t = tr_comb(u, t);
  }
  double out = 0.0;
  const bool ok = tr_apply(t, s, out);
  const uint64_t bad = __ballot(!ok);
  const int f = bad ? __builtin_ctzll(bad) : 64;
  const double sn = rld(out, f > 0 ? f - 1 : 0);
  if (f > 0) s = sn;
  return f;
}

constexpr int kWalkT = 256;  // four waves walk one sum redundantly; all four fill a descended segment's terms

// Segment k's terms into LDS (every thread of the workgroup, coalesced), products formed as the serial engine's.
// Every load is issued before the first product is formed (indices clamped into [0, n), the products past n are
// +0.0), so a thread waits for memory once, not once per term (the loop of rounds 3-4 waited 16 times, 12 us a
// segment).  fill_load issues the loads into registers, fill_store forms the products into LDS: work placed between
// the two overlaps the loads.
constexpr int kFillR = kSeg / kWalkT;
struct Fill {
  double a[kFillR], b[kFillR];
};
__device__ __forceinline__ void fill_load(Fill& f, const double* __restrict__ w, const double* __restrict__ y,
                                          int64_t n, int64_t k) {
  const int t = threadIdx.x;
#pragma unroll
  for (int r = 0; r < kFillR; ++r) f.a[r] = w[min<int64_t>(k * kSeg + t + r * kWalkT, n - 1)];
  if (y) {
#pragma unroll
    for (int r = 0; r < kFillR; ++r) f.b[r] = y[min<int64_t>(k * kSeg + t + r * kWalkT, n - 1)];
  }
}
__device__ __forceinline__ void fill_store(const Fill& f, double* sp, bool self, double sy, int64_t n, int64_t k) {
  const int t = threadIdx.x;
#pragma unroll
  for (int r = 0; r < kFillR; ++r) {
    const bool in = k * kSeg + t + r * kWalkT < n;
    sp[t + r * kWalkT] = in ? (self ? f.a[r] * f.a[r] : f.a[r] * (f.b[r] * sy)) : 0.0;
  }
}
__device__ __forceinline__ void fill_segment(double* sp, const double* __restrict__ w, const double* __restrict__ y,
                                             double sy, int64_t n, int64_t k) {
  Fill f;
  fill_load(f, w, y, n, k);
  fill_store(f, sp, y == nullptr, sy, n, k);
}

// Wave-uniform: s after the terms [i0, i1) of the LDS segment, added in order by the f64 add (lane 0; broadcast).
__device__ __forceinline__ double serial_terms(const double* sp, int i0, int i1, double s, int lane) {
  double a = s;
  if (lane == 0) {
    if (i1 - i0 == kSub) {  // a whole sub-segment: all 64 terms in registers first, then the dependent adds
      double2 q[kSub / 2];
#pragma unroll
      for (int u = 0; u < kSub / 2; ++u) q[u] = *reinterpret_cast<const double2*>(sp + i0 + 2 * u);
#pragma unroll
      for (int u = 0; u < kSub / 2; ++u) {
        a = a + q[u].x;
        a = a + q[u].y;
      }
    } else {
      for (int i = i0; i < i1; ++i) a = a + sp[i];
    }
  }
  return rld(a, 0);
}

// Workgroup v: sum v, from +0.0.  Windows of 64 segment transducers are composed in a wave scan and the longest
// prefix valid at s applied; a segment that does not apply is taken sub-segment by sub-segment (each lane applies
// its own sub's transducer to s, the failing ones' terms are added by the f64 add from LDS); after a descended
// segment the next one is tried on its own first, so runs of failing segments cost no scans.  All four waves
// compute the same s (identical inputs and operations), so every decision is uniform across the workgroup.
__global__ __launch_bounds__(kWalkT) void k_seqx_walk(const double* __restrict__ w, Vecs V, int64_t n, int self,
                                                      const Tr* __restrict__ segT, const Tr* __restrict__ subT,
                                                      int64_t K, const double* __restrict__ acc_in,
                                                      double* __restrict__ partial, int64_t nchunks,
                                                      const int* __restrict__ stop, int64_t* __restrict__ stats,
                                                      int prep) {
  if (stopped(stop)) return;
  __shared__ double sp[kSeg];
  const int v = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const double* y = self ? nullptr : vec_row(V, v);
  const double sy = (!self && V.scale) ? V.scale[v] : 1.0;
  int64_t n_scan = 0, n_segdesc = 0, n_subser = 0, n_single = 0, n_fbad = 0, n_fstate = 0, n_fguess = 0, n_frange = 0;
  int64_t c_scan = 0, c_single = 0, c_serial = 0, c_wait = 0, c_all = stats ? wall_clock64() : 0;  // 100 MHz ticks
  int64_t c_win = 0, c_subld = 0, c_fill = 0;  // stats only: memory waits made explicit (s_waitcnt 0) to time them
#define TICK(acc, stmt)                     \
  do {                                      \
    const int64_t t0_ = stats ? wall_clock64() : 0; \
    stmt;                                   \
    if (stats) acc += wall_clock64() - t0_; \
  } while (0)
  double s = acc_in ? acc_in[v] : 0.0;
  for (int64_t kb = 0; kb < K; kb += 64) {
    const bool in = kb + lane < K;
    const int64_t tw0 = stats ? wall_clock64() : 0;
    const Tr tw = tr_load(segT + (int64_t)v * K + (in ? kb + lane : 0));
    const Tr tv = tr_sel(in, tw, tr_bad());
    const Prep pv = prep_of(tv);
    if (stats) {
      __builtin_amdgcn_s_waitcnt(0);
      c_win += wall_clock64() - tw0;
    }
    int f0 = 0;
    bool scan = true;
    while (f0 < 64 && kb + f0 < K) {
      int f;
      if (scan) {
        TICK(c_scan, f = tr_walk(tr_sel(lane < f0, tr_ident(), tv), s, lane));
        ++n_scan;
      } else {  // the segment after a descended one, on its own
        double sn = 0.0;
        const bool ok = prep ? prep_apply(pv, s, sn) : tr_apply_v(tv, s, sn);  // every lane its own segment's map at
                                                                                  // s; lane f0's is the one
        const bool mine = ((__ballot(ok) >> f0) & 1) != 0;
        ++n_single;
        if (mine) {
          s = rld(sn, f0);
          f0 += 1;
          scan = true;
          continue;
        }
        f = f0;
      }
      if (f >= 64 || kb + f >= K) break;
      // segment kb + f does not apply at s: its sub-segments.  Its terms go to LDS now (the loads overlap the
      // scan over its subs, which skips the leading ones that apply); after the first failing sub, each sub is
      // tried on its own (lane j applies its map to s) and the failing ones are added term by term.
      const int64_t k = kb + f;
      ++n_segdesc;
      const int64_t tl0 = stats ? wall_clock64() : 0;
      const Tr u = tr_load(subT + ((int64_t)v * K + k) * kSubs + lane);
      const Prep pu = prep_of(u);
      if (stats) {
        __builtin_amdgcn_s_waitcnt(0);
        c_subld += wall_clock64() - tl0;
      }
      const int64_t tf0 = stats ? wall_clock64() : 0;
      __syncthreads();  // the previous segment's LDS reads are done
      fill_segment(sp, w, y, sy, n, k);
      if (stats) {
        __builtin_amdgcn_s_waitcnt(0);
        c_fill += wall_clock64() - tf0;
      }
      int j;
      TICK(c_scan, j = tr_walk(u, s, lane));
      ++n_scan;
      TICK(c_wait, __syncthreads());
      while (j < kSubs) {
        if (stats) {  // why this sub-segment did not apply (a diagnostic)
          const uint64_t sb = (uint64_t)__double_as_longlong(s);
          const int E = (int)((sb >> 52) & 0x7ff);
          const uint32_t ufl = __shfl(u.fl, j);
          const int ue = __shfl(u.e, j);
          if (ufl & F_BAD) ++n_fbad;
          else if (E == 0 || E == 0x7ff) ++n_fstate;
          else if (E - 1023 != ue || (uint32_t)(sb >> 63) != (ufl & F_NEG)) ++n_fguess;
          else ++n_frange;
        }
        const int64_t c0 = k * kSeg + (int64_t)j * kSub;
        const int i1 = (int)max<int64_t>(0, min<int64_t>(kSub, n - c0));
        TICK(c_serial, s = serial_terms(sp, j * kSub, j * kSub + i1, s, lane));
        ++n_subser;
        const int64_t t1 = stats ? wall_clock64() : 0;
        for (++j; j < kSubs; ++j) {
          double sn = 0.0;
          const bool ok = prep ? prep_apply(pu, s, sn) : tr_apply_v(u, s, sn);  // every lane its own sub's map at s;
                                                                                  // lane j's is the one
          ++n_single;
          if (!((__ballot(ok) >> j) & 1)) break;
          s = rld(sn, j);
        }
        if (stats) c_single += wall_clock64() - t1;
      }
      f0 = f + 1;
      scan = false;
    }
  }
#undef TICK
  if (t < 64)
    for (int64_t c = lane; c < nchunks; c += 64) partial[(int64_t)v * nchunks + c] = c == 0 ? s : 0.0;
  if (stats && t == 0) {
    stats[v * 8 + 0] = n_scan;
    stats[v * 8 + 1] = n_segdesc;
    stats[v * 8 + 2] = n_single;
    stats[v * 8 + 3] = n_subser;
    stats[v * 8 + 4] = n_fbad;
    stats[v * 8 + 5] = n_fstate;
    stats[v * 8 + 6] = n_fguess;
    stats[v * 8 + 7] = n_frange;
    stats[8 * MSK_MAX_GROUP + v * 8 + 0] = c_scan;
    stats[8 * MSK_MAX_GROUP + v * 8 + 1] = c_single;
    stats[8 * MSK_MAX_GROUP + v * 8 + 2] = c_serial;
    stats[8 * MSK_MAX_GROUP + v * 8 + 3] = c_wait;
    stats[8 * MSK_MAX_GROUP + v * 8 + 4] = wall_clock64() - c_all;
    stats[8 * MSK_MAX_GROUP + v * 8 + 5] = c_win;
    stats[8 * MSK_MAX_GROUP + v * 8 + 6] = c_subld;
    stats[8 * MSK_MAX_GROUP + v * 8 + 7] = c_fill;
  }
}

// ------------------------------------------------------------ the ripple walk (round 5)
// A prepared map in its one-add form: where it applies, s -> s + SD_p with SD_p = +-D_p carrying the map's sign (s
// has that sign, and |s| + D_p is exact, so s + SD_p is the same double); a zero map adds -0.0 when all its terms are
// -0.0 and +0.0 otherwise, which is its identity rule on every s, +-0.0 included.  Its validity is prep_valid.
struct Rip {
  double sd0, sd1;
};
__device__ __forceinline__ Rip rip_of(const Prep& p) {
  const bool z = (p.fl & F_ZERO) != 0, ng = (p.fl & F_NEG) != 0;
  const double zr = (p.fl & F_NZERO) ? -0.0 : 0.0;
  Rip r;
  r.sd0 = z ? zr : (ng ? -p.D0 : p.D0);
  r.sd1 = z ? zr : (ng ? -p.D1 : p.D1);
  return r;
}
// prep_apply's verdict
__device__ __forceinline__ bool prep_valid(const Prep& p, double s) {
  const uint64_t b = (uint64_t)__double_as_longlong(s);
  const bool od = (b & 1) != 0, neg = (b >> 63) != 0;
  const double a = fabs(s);
  const double L = pickd(od, p.L1, p.L0), H = pickd(od, p.H1, p.H0);
  return (p.fl & F_ZERO) != 0 || (a >= L && a < H && neg == ((p.fl & F_NEG) != 0));
}

// lane l gets lane l - 1's x; lane 0 keeps its own (the same DPP move with x as the "old" operand: no copy of s)
__device__ __forceinline__ double shr1_own(double x) {
  const int64_t b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, 0x138, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), 0x138, 0xf, 0xf, false);
  return __longlong_as_double((int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// The lanes' maps j0, j0 + 1, .. applied in order from s, R steps of a ripple through the wave: each step every lane
// adds its SD to its left neighbour's previous result (lanes below j0 are the identity), so after step i lanes j0 ..
// j0 + i hold the sequential results wherever every map before theirs applied -- one f64 add and two DPP moves a
// step (wave_shr:1, lane 0 keeping its own value), plus a parity select where a map holds a tie (TIES).  Lane 0 has
// no left neighbour: below j0 it is an identity lane holding s; as map j0 = 0 (J0) it reads s at step 0 and then
// turns into the identity, holding its result.  Then one verdict per lane at its true input: returns the first lane
// in [j0, j0 + r) whose map does not apply (j0 + r if all do), s advanced to that lane's input.
template <int R, bool TIES, bool J0>
__device__ __forceinline__ int ripple(const Prep& p, const Rip& q, double& s, int j0, int r, int lane) {
  const bool idn = lane < j0, frz = J0 && lane == 0;
  const double a0 = idn ? -0.0 : q.sd0, a1 = idn ? -0.0 : q.sd1;  // step 0
  const double b0 = frz ? -0.0 : a0, b1 = frz ? -0.0 : a1;        // steps 1 ..
  double in = s;
  double out = in + (TIES ? pickd(((uint32_t)__double_as_longlong(in) & 1u) != 0, a1, a0) : a0);
#pragma unroll
  for (int i = 1; i < R; ++i) {
    in = shr1_own(out);
    out = in + (TIES ? pickd(((uint32_t)__double_as_longlong(in) & 1u) != 0, b1, b0) : b0);
  }
  const bool ok = idn || prep_valid(p, frz ? s : in);
  const uint64_t bad = __ballot(!ok) & (~uint64_t(0) << j0);
  const int f = min(bad ? __builtin_ctzll(bad) : 64, j0 + r);
  if (f > j0) s = rld(out, f - 1);
  return f;
}

// The maps from lane j on, ripple after ripple, up to the first that does not apply or lim; returns its lane.
// ties: some lane's map depends on the state's parity (sd0 != sd1), wave-uniform.
template <int R, bool TIES>
__device__ __forceinline__ int ripple_run_t(const Prep& p, const Rip& q, double& s, int j, int lim, int lane,
                                            int64_t& calls) {
  while (j < lim) {
    const int r = min(R, lim - j);
    const int f = j == 0 ? ripple<R, TIES, true>(p, q, s, j, r, lane) : ripple<R, TIES, false>(p, q, s, j, r, lane);
    ++calls;
    if (f < j + r) return f;
    j = f;
  }
  return lim;
}
template <int R>
__device__ __forceinline__ int ripple_run(const Prep& p, const Rip& q, bool ties, double& s, int j, int lim, int lane,
                                          int64_t& calls) {
  return ties ? ripple_run_t<R, true>(p, q, s, j, lim, lane, calls)
              : ripple_run_t<R, false>(p, q, s, j, lim, lane, calls);
}
__device__ __forceinline__ int ripple_runw(int w, const Prep& p, const Rip& q, bool ties, double& s, int j, int lim,
                                           int lane, int64_t& calls) {
  switch (w) {
    case 4: return ripple_run<4>(p, q, ties, s, j, lim, lane, calls);
    case 8: return ripple_run<8>(p, q, ties, s, j, lim, lane, calls);
    case 32: return ripple_run<32>(p, q, ties, s, j, lim, lane, calls);
    default: return ripple_run<16>(p, q, ties, s, j, lim, lane, calls);
  }
}
// some lane's map of this set depends on the parity of the state (a tie in its run)
__device__ __forceinline__ bool any_ties(const Rip& q) {
  return __ballot(__double_as_longlong(q.sd0) != __double_as_longlong(q.sd1)) != 0;
}

// The overlapped builds (seqx_core, round 6): segment k's records are read only once its builder has published
// ready[k] = epoch (an agent-scope release behind the records; the acquire here orders the wave's later loads of
// them).  Lane l waits for segment k0 + l.  A wait that outlasts 4 s gives up: the sum then comes out NaN, a loud
// failure instead of a hang.
// How long a wait of the overlapped walk spins before it gives up (100 MHz ticks): 4 s; MSPLIT_SEQ_SPIN_TICKS sets it
// (tests: 0 makes every wait that is not already satisfied give up, which exercises the retry launch)
__device__ int64_t g_seq_spin_ticks = 400000000;

__device__ __forceinline__ bool wait_ready(uint32_t* ready, uint32_t epoch, int64_t k0, int64_t K, int lane) {
  if (!ready || k0 >= K) return true;
  uint32_t* f = ready + min<int64_t>(k0 + lane, K - 1);
  bool ok = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == epoch;
  const int64_t t0 = wall_clock64();
  while (__ballot(!ok)) {
    if (wall_clock64() - t0 > g_seq_spin_ticks) return false;
    __builtin_amdgcn_s_sleep(2);
    if (!ok) ok = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == epoch;
  }
  return true;
}

// Workgroup v: sum v, from +0.0, every map applied by ripples: the window of 64 segment maps up to the first that
// does not apply; that segment's sub maps likewise (its terms' loads in flight meanwhile); a sub that does not
// apply is added term by term from LDS, and the ripple resumes after it.  rw: the ripple width over segments and a
// descended segment's first subs; rs: after a serially added sub.  All four waves compute the same s.
__device__ __forceinline__ void ripwalk_sum(int v, const double* __restrict__ w, const Vecs& V, int64_t n, int self,
                                            const Tr* __restrict__ segT, const Tr* __restrict__ subT, int64_t K,
                                            const double* __restrict__ acc_in, double* __restrict__ partial,
                                            int64_t nchunks, int64_t* __restrict__ stats, int rw, int rs, int pf,
                                            double* sp, uint32_t* ready = nullptr, uint32_t epoch = 0,
                                            uint32_t* fail = nullptr) {
  const int t = threadIdx.x, lane = t & 63;
  const double* y = self ? nullptr : vec_row(V, v);
  const double sy = (!self && V.scale) ? V.scale[v] : 1.0;
  int64_t n_win = 0, n_segdesc = 0, n_rip = 0, n_subser = 0;
  int64_t c_win = 0, c_rip = 0, c_serial = 0, c_fill = 0, c_all = stats ? wall_clock64() : 0;  // 100 MHz ticks
#define TICK(acc, stmt)                             \
  do {                                              \
    const int64_t t0_ = stats ? wall_clock64() : 0; \
    stmt;                                           \
    if (stats) acc += wall_clock64() - t0_;         \
  } while (0)
  // pf: the next segment the walk will descend into is predicted -- a BAD segment map never applies, so the walk
  // stops at every one -- and its terms and sub record are loaded while the walk works on the segments before it
  // (fp / tp hold segment kp; a descent into any other segment loads its own into them).  The next window's segment
  // records are likewise loaded one window ahead.
  Fill fp;
  Tr tp = tr_bad();
  int64_t kp = -1;
  int64_t n_hit = 0, n_miss = 0;
  double s = acc_in ? acc_in[v] : 0.0;
  bool live = wait_ready(ready, epoch, 0, K, lane);
  Tr twn = tr_load(segT + (int64_t)v * K + min<int64_t>(lane, K - 1));
  for (int64_t kb = 0; kb < K && live; kb += 64) {
    const int lim = (int)min<int64_t>(64, K - kb);
    const bool in = lane < lim;
    const Tr tw = twn;
    if (kb + 64 < K) {
      live = wait_ready(ready, epoch, kb + 64, K, lane);  // the overlapped builds: the next window is built
      twn = tr_load(segT + (int64_t)v * K + min<int64_t>(kb + 64 + lane, K - 1));
    }
    const Prep pv = prep_of(tr_sel(in, tw, tr_bad()));
    const Rip qv = rip_of(pv);
    const bool tv = any_ties(qv);
    const uint64_t badm = __ballot(in && (pv.fl & F_BAD) != 0);  // the window's segments the walk must descend into
    if (pf && kp < kb && badm) {
      kp = kb + __builtin_ctzll(badm);
      fill_load(fp, w, y, n, kp);
      tp = tr_load(subT + ((int64_t)v * K + kp) * kSubs + lane);
    }
    for (int f = 0;;) {
      TICK(c_win, f = ripple_runw(rw, pv, qv, tv, s, f, lim, lane, n_win));
      if (f >= lim) break;
      const int64_t k = kb + f;  // segment k does not apply at s: its sub maps
      ++n_segdesc;
      const int64_t tf0 = stats ? wall_clock64() : 0;
      if (k != kp) {  // not the predicted one (a map that only fails at the actual s): load it now
        fill_load(fp, w, y, n, k);
        tp = tr_load(subT + ((int64_t)v * K + k) * kSubs + lane);
        kp = k;
        ++n_miss;
      } else {
        ++n_hit;
      }
      const Prep pu = prep_of(tp);
      const Rip qu = rip_of(pu);
      const bool tu = any_ties(qu);
      int j;
      TICK(c_rip, j = ripple_runw(rw, pu, qu, tu, s, 0, kSubs, lane, n_rip));
      if (j < kSubs) {
        __syncthreads();  // the previous segment's LDS reads are done
        fill_store(fp, sp, self != 0, sy, n, k);
        __syncthreads();
      }
      if (pf) {  // the next BAD segment of this window, while this one's subs are walked
        const uint64_t m = f < 63 ? badm & (~uint64_t(0) << (f + 1)) : 0;
        if (m) {
          kp = kb + __builtin_ctzll(m);
          fill_load(fp, w, y, n, kp);
          tp = tr_load(subT + ((int64_t)v * K + kp) * kSubs + lane);
        }
      }
      if (stats) c_fill += wall_clock64() - tf0;
      while (j < kSubs) {
        const int64_t c0 = k * kSeg + (int64_t)j * kSub;
        const int i1 = (int)max<int64_t>(0, min<int64_t>(kSub, n - c0));
        TICK(c_serial, s = serial_terms(sp, j * kSub, j * kSub + i1, s, lane));
        ++n_subser;
        TICK(c_rip, j = ripple_runw(rs, pu, qu, tu, s, j + 1, kSubs, lane, n_rip));
      }
      ++f;
    }
  }
#undef TICK
  if (!live) s = __builtin_nan("");  // a builder never published: no result (the retry launch redoes it)
  if (!live && fail && t == 0) fail[0] = epoch;
  if (t < 64)
    for (int64_t c = lane; c < nchunks; c += 64) partial[(int64_t)v * nchunks + c] = c == 0 ? s : 0.0;
  if (stats && t == 0) {
    stats[v * 8 + 0] = n_win;
    stats[v * 8 + 1] = n_segdesc;
    stats[v * 8 + 2] = n_rip;
    stats[v * 8 + 3] = n_subser;
    stats[v * 8 + 4] = n_hit;
    stats[v * 8 + 5] = n_miss;
    stats[v * 8 + 6] = stats[v * 8 + 7] = 0;
    stats[8 * MSK_MAX_GROUP + v * 8 + 0] = c_win;
    stats[8 * MSK_MAX_GROUP + v * 8 + 1] = c_rip;
    stats[8 * MSK_MAX_GROUP + v * 8 + 2] = c_serial;
    stats[8 * MSK_MAX_GROUP + v * 8 + 3] = 0;
    stats[8 * MSK_MAX_GROUP + v * 8 + 4] = wall_clock64() - c_all;
    stats[8 * MSK_MAX_GROUP + v * 8 + 5] = 0;
    stats[8 * MSK_MAX_GROUP + v * 8 + 6] = 0;
    stats[8 * MSK_MAX_GROUP + v * 8 + 7] = c_fill;
  }
}

__global__ __launch_bounds__(kWalkT) void k_seqx_ripwalk(const double* __restrict__ w, Vecs V, int64_t n, int self,
                                                         const Tr* __restrict__ segT, const Tr* __restrict__ subT,
                                                         int64_t K, const double* __restrict__ acc_in,
                                                         double* __restrict__ partial, int64_t nchunks,
                                                         const int* __restrict__ stop, int64_t* __restrict__ stats,
                                                         int rw, int rs, int pf, uint32_t* ready, uint32_t epoch,
                                                         uint32_t* fail, uint32_t guard) {
  if (stopped(stop)) return;
  if (guard && fail[0] != guard) return;  // the retry launch: only when this call's overlapped walk gave up
  __shared__ double sp[kSeg];
  ripwalk_sum(blockIdx.x, w, V, n, self, segT, subT, K, acc_in, partial, nchunks, stats, rw, rs, pf, sp, ready,
              epoch, fail);
}

// ------------------------------------------------------------ the ripple walk with filler waves (round 6)
// ripwalk_sum's four waves all walk, and all four fill a descended segment's terms: the walk stops at each fill and
// waits out its loads (a third of a PETSc-order step's walk time, profiles/r06/seq_pc/).  Here wave 0 walks alone
// and waves 1-3 fill: in walk order, each BAD segment's products and its 64 sub records go into a ring of kRing LDS
// slots, as far ahead of the walk as the ring allows.  A BAD segment never applies, so the walk descends into every
// one of them, in order, and finds it filled; a segment that fails only at the actual s (rare: 3 % of descents) is
// read by the walk itself, sub record and failing subs' terms.  The sums are the same bits: the same maps, the
// same products (formed as fill_store forms them), the same adds.
//
// Hand-off through LDS: a filler wave stores its part of a slot, then one add of its lane 0 to the slot's counter
// (workgroup-scope release, so the wave's LDS stores come first); the wave whose add completes the count publishes
// the slot's segment (release).  The walk polls for that segment (acquire) and only then reads the slot.  A slot is
// refilled only once the walk has moved past its segment (walk_pos, published by the walk before it looks for a
// slot), so the segment it reads is never rewritten under it.  Every wait gives up after 4 s: the sum then comes out
// NaN and the fillers stop.
constexpr int kRing = 3;
constexpr int64_t kRingSpin = 400000000;  // 4 s of 100 MHz ticks: a ring wait that outlasts it gives up
constexpr int kFillW = 3;
constexpr int kFillT = kFillW * 64;
constexpr int kFillPer = (kSeg + kFillT - 1) / kFillT;
struct alignas(16) RingSlot {
  double p[kSeg];
  Tr sub[kSubs];
};
struct RingCtl {
  int32_t seg[kRing];  // the segment a slot holds (published), -1: none yet
  int32_t cnt[kRing];  // filler waves done with the slot's current fill
  int32_t walk_pos;    // the walk is at this segment or past it: slots holding earlier ones are free
  int32_t done;        // the walk has finished (or given up): the fillers stop
};
__device__ __forceinline__ int32_t lds_acq(int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_rel(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The filler waves' loop: BAD segments in order into the ring.  ft: thread index among the fillers.
__device__ __forceinline__ void fill_ring(int v, const double* __restrict__ w, const double* __restrict__ y, double sy,
                                          int64_t n, int self, const Tr* __restrict__ segT,
                                          const Tr* __restrict__ subT, int64_t K, RingSlot* ring, RingCtl* ctl,
                                          uint32_t* ready, uint32_t epoch) {
  const int t = threadIdx.x, lane = t & 63, ft = t - 64;
  const bool recs = t < 128;  // wave 1 also moves the slot's sub records
  int32_t pk0 = -1, pk1 = -1, pk2 = -1;  // the segments of the last kRing fills (the oldest first)
  int u = 0;
  for (int64_t kb = 0; kb < K; kb += 64) {
    if (!wait_ready(ready, epoch, kb, K, lane)) return;
    const int64_t kl = kb + lane;
    const uint32_t fl = kl < K ? segT[(int64_t)v * K + kl].fl : 0u;
    uint64_t badm = __ballot((fl & F_BAD) != 0);
    while (badm) {
      const int32_t k = (int32_t)(kb + __builtin_ctzll(badm));
      badm &= badm - 1;
      const int slot = u % kRing;
      // the slot's previous segment (pk0) published by every filler wave, and passed by the walk
      const int64_t t0 = wall_clock64();
      for (;;) {
        if (lds_acq(&ctl->done)) return;
        if (lds_acq(&ctl->seg[slot]) == pk0 && pk0 < lds_acq(&ctl->walk_pos)) break;
        if (wall_clock64() - t0 > kRingSpin) return;
        __builtin_amdgcn_s_sleep(1);
      }
      RingSlot* S = ring + slot;
      double a[kFillPer], b[kFillPer];
      const int64_t c0 = (int64_t)k * kSeg;
#pragma unroll
      for (int r = 0; r < kFillPer; ++r) {
        const int i = ft + r * kFillT;
        const int64_t g = min<int64_t>(c0 + min(i, kSeg - 1), n - 1);
        a[r] = w[g];
        b[r] = y ? y[g] : 0.0;
      }
      Tr tr;
      if (recs) tr = tr_load(subT + ((int64_t)v * K + k) * kSubs + lane);
#pragma unroll
      for (int r = 0; r < kFillPer; ++r) {
        const int i = ft + r * kFillT;
        if (i < kSeg) S->p[i] = c0 + i < n ? (self ? a[r] * a[r] : a[r] * (b[r] * sy)) : 0.0;
      }
      if (recs) S->sub[lane] = tr;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) {
        const int32_t old = __hip_atomic_fetch_add(&ctl->cnt[slot], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == kFillW - 1) {  // the last of the filler waves: the slot is whole
          __hip_atomic_store(&ctl->cnt[slot], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          lds_rel(&ctl->seg[slot], k);
        }
      }
      pk0 = pk1;
      pk1 = pk2;
      pk2 = k;
      ++u;
    }
  }
}

// Wave 0: sum v, as ripwalk_sum (the same ripples, the same serial adds), its descended segments from the ring.
__device__ __forceinline__ void ripwalk_pc_walk(int v, const double* __restrict__ w, const double* __restrict__ y,
                                                double sy, int64_t n, int self, const Tr* __restrict__ segT,
                                                const Tr* __restrict__ subT, int64_t K,
                                                const double* __restrict__ acc_in, double* __restrict__ partial,
                                                int64_t nchunks, int64_t* __restrict__ stats, int rw, int rs,
                                                RingSlot* ring, RingCtl* ctl, double* sp1, uint32_t* ready,
                                                uint32_t epoch, uint32_t* fail) {
  const int lane = threadIdx.x & 63;
  int64_t n_win = 0, n_segdesc = 0, n_rip = 0, n_subser = 0, n_hit = 0, n_miss = 0, n_badsub = 0, n_guess = 0;
  int64_t c_win = 0, c_rip = 0, c_serial = 0, c_fill = 0, c_wait = 0, c_all = stats ? wall_clock64() : 0;
#define TICK(acc, stmt)                             \
  do {                                              \
    const int64_t t0_ = stats ? wall_clock64() : 0; \
    stmt;                                           \
    if (stats) acc += wall_clock64() - t0_;         \
  } while (0)
  double s = acc_in ? acc_in[v] : 0.0;
  bool live;
  TICK(c_wait, live = wait_ready(ready, epoch, 0, K, lane));
  Tr twn = tr_load(segT + (int64_t)v * K + min<int64_t>(lane, K - 1));
  for (int64_t kb = 0; kb < K && live; kb += 64) {
    if (lane == 0) lds_rel(&ctl->walk_pos, (int32_t)kb);
    const int lim = (int)min<int64_t>(64, K - kb);
    const bool in = lane < lim;
    const Tr tw = twn;
    if (kb + 64 < K) {
      TICK(c_wait, live = wait_ready(ready, epoch, kb + 64, K, lane));
      twn = tr_load(segT + (int64_t)v * K + min<int64_t>(kb + 64 + lane, K - 1));
    }
    const Prep pv = prep_of(tr_sel(in, tw, tr_bad()));
    const Rip qv = rip_of(pv);
    const bool tv = any_ties(qv);
    const uint64_t badm = __ballot(in && (pv.fl & F_BAD) != 0);
    for (int f = 0; live;) {
      TICK(c_win, f = ripple_runw(rw, pv, qv, tv, s, f, lim, lane, n_win));
      if (f >= lim) break;
      const int32_t k = (int32_t)(kb + f);
      ++n_segdesc;
      if (lane == 0) lds_rel(&ctl->walk_pos, k);
      const int64_t tf0 = stats ? wall_clock64() : 0;
      int slot = -1;
      Tr tp;
      if ((badm >> f) & 1) {  // the fillers bring it
        const int64_t t0 = wall_clock64();
        while (slot < 0) {
#pragma unroll
          for (int q = 0; q < kRing; ++q)
            if (lds_acq(&ctl->seg[q]) == k) slot = q;
          if (slot >= 0) break;
          if (wall_clock64() - t0 > kRingSpin) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if (slot < 0) {
          live = false;
          break;
        }
        tp = ring[slot].sub[lane];
        ++n_hit;
      } else {  // a map that only fails at the actual s
        tp = tr_load(subT + ((int64_t)v * K + k) * kSubs + lane);
        ++n_miss;
      }
      if (stats) c_fill += wall_clock64() - tf0;
      const Prep pu = prep_of(tp);
      const Rip qu = rip_of(pu);
      const bool tu = any_ties(qu);
      int j;
      TICK(c_rip, j = ripple_runw(rw, pu, qu, tu, s, 0, kSubs, lane, n_rip));
      while (j < kSubs) {
        const int64_t c0 = (int64_t)k * kSeg + (int64_t)j * kSub;
        const int i1 = (int)max<int64_t>(0, min<int64_t>(kSub, n - c0));
        if (stats) {  // why sub j failed: a BAD record, s outside the record's binade (the guess), or inside it
          const uint32_t fj = (uint32_t)__builtin_amdgcn_readlane((int)tp.fl, j);
          const int ej = __builtin_amdgcn_readlane(tp.e, j);
          const uint64_t sb = (uint64_t)__double_as_longlong(s);
          const int es = (int)((sb >> 52) & 0x7ff) - 1023;
          if (fj & F_BAD) ++n_badsub;
          else if (!(fj & F_ZERO) && (es != ej || (uint32_t)(sb >> 63) != (fj & F_NEG))) ++n_guess;
        }
        if (slot >= 0) {
          TICK(c_serial, s = serial_terms(ring[slot].p, j * kSub, j * kSub + i1, s, lane));
        } else {  // this sub's terms, formed as fill_store forms them
          const int64_t g = min<int64_t>(c0 + lane, n - 1);
          const double a = w[g], b = y ? y[g] : 0.0;
          sp1[lane] = c0 + lane < n ? (self ? a * a : a * (b * sy)) : 0.0;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          TICK(c_serial, s = serial_terms(sp1, 0, i1, s, lane));
          __builtin_amdgcn_wave_barrier();  // lane 0's reads before the next sub's stores
        }
        ++n_subser;
        TICK(c_rip, j = ripple_runw(rs, pu, qu, tu, s, j + 1, kSubs, lane, n_rip));
      }
      ++f;
    }
  }
#undef TICK
  if (lane == 0) lds_rel(&ctl->done, 1);
  if (!live) s = __builtin_nan("");  // a builder never published (the retry launch redoes the sum)
  if (!live && fail && lane == 0) fail[0] = epoch;
  for (int64_t c = lane; c < nchunks; c += 64) partial[(int64_t)v * nchunks + c] = c == 0 ? s : 0.0;
  if (stats && lane == 0) {
    stats[v * 8 + 0] = n_win;
    stats[v * 8 + 1] = n_segdesc;
    stats[v * 8 + 2] = n_rip;
    stats[v * 8 + 3] = n_subser;
    stats[v * 8 + 4] = n_hit;
    stats[v * 8 + 5] = n_miss;
    stats[v * 8 + 6] = n_badsub;
    stats[v * 8 + 7] = n_guess;
    stats[8 * MSK_MAX_GROUP + v * 8 + 0] = c_win;
    stats[8 * MSK_MAX_GROUP + v * 8 + 1] = c_rip;
    stats[8 * MSK_MAX_GROUP + v * 8 + 2] = c_serial;
    stats[8 * MSK_MAX_GROUP + v * 8 + 3] = c_wait;
    stats[8 * MSK_MAX_GROUP + v * 8 + 4] = wall_clock64() - c_all;
    stats[8 * MSK_MAX_GROUP + v * 8 + 5] = 0;
    stats[8 * MSK_MAX_GROUP + v * 8 + 6] = 0;
    stats[8 * MSK_MAX_GROUP + v * 8 + 7] = c_fill;
  }
}

__global__ __launch_bounds__(kWalkT) void k_seqx_ripwalk_pc(const double* __restrict__ w, Vecs V, int64_t n, int self,
                                                            const Tr* __restrict__ segT, const Tr* __restrict__ subT,
                                                            int64_t K, const double* __restrict__ acc_in,
                                                            double* __restrict__ partial, int64_t nchunks,
                                                            const int* __restrict__ stop, int64_t* __restrict__ stats,
                                                            int rw, int rs, uint32_t* ready, uint32_t epoch,
                                                            uint32_t* fail, uint32_t guard) {
  static_assert(kWalkT == 64 + kFillT, "one walking wave and the filler waves");
  if (stopped(stop)) return;
  if (guard && fail[0] != guard) return;  // the retry launch: only when this call's overlapped walk gave up
  __shared__ RingSlot ring[kRing];
  __shared__ RingCtl ctl;
  __shared__ double sp1[kSub];
  const int t = threadIdx.x, v = blockIdx.x;
  if (t < kRing) {
    ctl.seg[t] = -1;
    ctl.cnt[t] = 0;
  }
  if (t == 0) {
    ctl.walk_pos = 0;
    ctl.done = 0;
  }
  __syncthreads();
  const double* y = self ? nullptr : vec_row(V, v);
  const double sy = (!self && V.scale) ? V.scale[v] : 1.0;
  if (t < 64)
    ripwalk_pc_walk(v, w, y, sy, n, self, segT, subT, K, acc_in, partial, nchunks, stats, rw, rs, ring, &ctl, sp1,
                    ready, epoch, fail);
  else
    fill_ring(v, w, y, sy, n, self, segT, subT, K, ring, &ctl, ready, epoch);
}


}  // namespace

extern "C" int msk_seq_stage1(const double* w, const Vecs* V, int nv, int64_t n, int self, double* partial,
                              int64_t nchunks, const int* stop, hipStream_t s) {
  if (nv < 1 || nv > MSK_MAX_GROUP || (self && nv != 1) || nchunks < 1) return (int)hipErrorInvalidValue;
  k_seq_stage1<<<dim3(nv), dim3(kT), 0, s>>>(w, *V, n, self, partial, nchunks, stop);
  return (int)hipGetLastError();
}

extern "C" int mspi_reduce_seq(const msp_ctx* c) { return c->reduce == MSP_REDUCE_SEQ; }

// Which engine takes a PETSc-order sum of n terms: MSPLIT_SEQ_ENGINE=serial / parallel forces one, else the parallel
// engine from min_n terms on.  Below that its four launches and the per-segment transducers cost more than the
// serial adds save (a dot is 53 us parallel against 23 us serial at n = 1024), and where the engines meet depends on
// how often the sum changes binade (below).
static bool parallel_engine(int64_t n, int64_t min_n) {
  const char* eng = getenv("MSPLIT_SEQ_ENGINE");
  if (eng && (eng[0] == 's' || eng[0] == 'S')) return false;
  if (eng && (eng[0] == 'p' || eng[0] == 'P')) return n > 0;
  return n >= min_n;
}
// profiles/r05/seq_crossover/ (tools/seq_crossover.py, random data: the hardest sums): a norm's running sum only grows,
// so it leaves its binade log2(n) times and the parallel engine wins from 8 K terms (65 K: 73 against 315 us); a
// random dot hovers near zero and wins from ~100 K; an MDot of 30 random sums costs its slowest walk, about the
// serial time up to 1 M.
constexpr int64_t kParMinNorm = int64_t(1) << 13;   // a norm (sum of squares)
constexpr int64_t kParMinDot = int64_t(1) << 17;    // one dot
constexpr int64_t kParMinSum = int64_t(1) << 19;    // an MDot
constexpr int64_t kParMinChain = int64_t(1) << 17;  // an LSQR chain: its total length per sum

// The overlapped builds' two streams, made on first use: the walks on the first kSeqWalkCUs compute units, the
// builds on the others (CU masks), so that no build wave shares a CU with a walk -- a walk is a chain of dependent
// ripple steps, and co-resident build waves took its issue slots (the SMSM block in PETSc's order: +6 % with both
// streams on every CU); plus the events that order them with the context's stream.  Nonzero: no such streams.
constexpr int kSeqWalkCUs = 32;  // >= MSK_MAX_GROUP: one CU per walked sum
static int seq_aux(msp_ctx* c) {
  if (c->seq_aux) return 0;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
      ncu < 2 * kSeqWalkCUs || ncu > 1024)
    return 1;
  uint32_t mw[32] = {0}, mb[32] = {0};
  const int words = (ncu + 31) / 32;
  for (int i = 0; i < ncu; ++i) (i < kSeqWalkCUs ? mw : mb)[i / 32] |= 1u << (i % 32);
  hipStream_t sw = nullptr, sb = nullptr;
  if (hipExtStreamCreateWithCUMask(&sw, (uint32_t)words, mw) != hipSuccess) return 1;
  if (hipExtStreamCreateWithCUMask(&sb, (uint32_t)words, mb) != hipSuccess) {
    (void)hipStreamDestroy(sw);
    return 1;
  }
  for (auto& e : c->seq_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      (void)hipStreamDestroy(sw);
      (void)hipStreamDestroy(sb);
      return 1;
    }
  c->seq_walk = sw;
  c->seq_aux = sb;
  return 0;
}

// The parallel engine: nv sums of n terms w[i] * (V_v[i] * sy_v) (self: w[i] * w[i]), each from acc_in[v] (device;
// nullptr: +0.0), into partial's DBR layout.  n > 0.
static int seqx_core(msp_ctx* c, const double* w, const Vecs* V, int nv, int64_t n, int self, const double* acc_in,
                     double* partial, int64_t nchunks, const int* stop) {
  const int64_t K = (n + kSeg - 1) / kSeg;
  if (nv < 1 || nv > MSK_MAX_GROUP || (self && nv != 1) || nchunks < 1 || K < 1) return (int)hipErrorInvalidValue;
  const int64_t need = (int64_t)nv * K * ((int64_t)sizeof(Tr) * (kSubs + 1) + (int64_t)sizeof(double));
  if (need > c->seqbuf_cap) {
    if (hipStreamSynchronize(c->stream) != hipSuccess) return (int)hipErrorUnknown;
    if (c->seqbuf) (void)hipFree(c->seqbuf);
    c->seqbuf = nullptr;
    c->seqbuf_cap = 0;
    const hipError_t e = hipMalloc(&c->seqbuf, (size_t)need);
    if (e != hipSuccess) return (int)e;
    c->seqbuf_cap = need;
  }
  if (K > c->seqready_cap) {  // the overlapped builds' ready words: a buffer of their own, zeroed, so that no word ever
                              // held anything but an earlier launch's epoch (every launch takes a new, nonzero one)
    if (hipStreamSynchronize(c->stream) != hipSuccess) return (int)hipErrorUnknown;
    if (c->seqready) (void)hipFree(c->seqready);
    c->seqready = nullptr;
    c->seqready_cap = 0;
    hipError_t e = hipMalloc((void**)&c->seqready, (size_t)(K + 1) * sizeof(uint32_t));  // + the retry flag
    if (e != hipSuccess) return (int)e;
    if ((e = hipMemsetAsync(c->seqready, 0, (size_t)(K + 1) * sizeof(uint32_t), c->stream)) != hipSuccess) return (int)e;
    c->seqready_cap = K;
  }
  Tr* subT = static_cast<Tr*>(c->seqbuf);
  Tr* segT = subT + (int64_t)nv * K * kSubs;
  double* pre = reinterpret_cast<double*>(segT + (int64_t)nv * K);
  uint32_t* ready = c->seqready;
  uint32_t* fail = c->seqready + c->seqready_cap;  // an overlapped walk that gave up writes its epoch here
  const int rc = msk_dot_stage1(w, V, nv, n, pre, K, self, stop, c->stream);
  if (rc) return rc;
  k_seqx_prefix<<<dim3(nv), dim3(kT), 0, c->stream>>>(pre, K, acc_in, stop);
  // MSPLIT_SEQ_STATS=1: per-sum walk counters on stderr (a diagnostic; its buffer lives for this call only)
  const char* st = getenv("MSPLIT_SEQ_STATS");
  int64_t* dstats = nullptr;
  if (st && st[0] == '1' && hipMalloc((void**)&dstats, 16 * MSK_MAX_GROUP * sizeof(int64_t)) != hipSuccess)
    dstats = nullptr;
  // MSPLIT_SEQ_PREP=0: the one-record applies decode s's bits (tr_apply_v, round 4) instead of the prepared maps
  static const int prep = [] {
    const char* e = getenv("MSPLIT_SEQ_PREP");
    return e && e[0] == '0' ? 0 : 1;
  }();
  // MSPLIT_SEQ_WALK=scan: the walk of rounds 4-5 (wave scans of composed transducers and one-record applies) instead
  // of the ripple walk; MSPLIT_SEQ_RIPPLE_W / MSPLIT_SEQ_RIPPLE: the ripple widths (4, 8, 16, 32) over segments and
  // after a serially added sub.  Read per call (tests vary them); a getenv is nothing next to a walk.
  const char* wk = getenv("MSPLIT_SEQ_WALK");
  const char* rwe = getenv("MSPLIT_SEQ_RIPPLE_W");
  const char* rse = getenv("MSPLIT_SEQ_RIPPLE");
  const char* pfe = getenv("MSPLIT_SEQ_PREFETCH");  // 0: a descended segment's loads start at the descent
  const int rw = rwe ? atoi(rwe) : 16, rs = rse ? atoi(rse) : 8, pf = pfe && pfe[0] == '0' ? 0 : 1;
  const bool ripwalk = !(wk && wk[0] == 's');
  // MSPLIT_SEQ_FILLERS=0: every wave of the walk's workgroup walks and fills (round 5) instead of filler waves
  // MSPLIT_SEQ_TRANS_PF=1: the transducer build loads the next sum's terms during this sum's maps (round 5)
  const char* tpe = getenv("MSPLIT_SEQ_TRANS_PF");
  auto trans_kernel = tpe && tpe[0] == '1' ? k_seqx_trans<true> : k_seqx_trans<false>;
  const char* fle = getenv("MSPLIT_SEQ_FILLERS");
  const bool fillers = !(fle && fle[0] == '0');
  auto launch_walk = [&](hipStream_t st, uint32_t* rdy, uint32_t ep, uint32_t* fl, uint32_t guard) {
    if (fillers)
      k_seqx_ripwalk_pc<<<dim3(nv), dim3(kWalkT), 0, st>>>(w, *V, n, self, segT, subT, K, acc_in, partial, nchunks,
                                                           stop, dstats, rw, rs, rdy, ep, fl, guard);
    else
      k_seqx_ripwalk<<<dim3(nv), dim3(kWalkT), 0, st>>>(w, *V, n, self, segT, subT, K, acc_in, partial, nchunks, stop,
                                                        dstats, rw, rs, pf, rdy, ep, fl, guard);
  };
  // The transducer builds and the walk run on two streams of their own (seq_aux: disjoint compute units) while the
  // walk follows the builds (round 6): it waits per window of 64 segments for their builders' ready words
  // (ripwalk_sum's wait_ready), so the builds -- about a fifth of a PETSc-order GMRES step -- overlap the walks.
  // The builds are enqueued first, so two streams that share one hardware queue still make progress (the walk then
  // starts after them).
  // MSPLIT_SEQ_OVERLAP=0: one stream, the builds before the walk (rounds 4-5).
  const char* ove = getenv("MSPLIT_SEQ_OVERLAP");
  // only where walks are long next to their builds: MDots (several sums, each hovering near zero); a norm's walk
  // (one sum that only grows) or a single dot would just wait for its builds
  const bool overlap = ripwalk && !(ove && ove[0] == '0') && (ove && ove[0] == '2' ? true : nv >= 2 && !self) &&
                       seq_aux(c) == 0;
  if (overlap) {
    if (++c->seq_epoch == 0) c->seq_epoch = 1;  // 0 is the words' initial value
    const char* spe = getenv("MSPLIT_SEQ_SPIN_TICKS");
    const int64_t ticks = spe ? atoll(spe) : 400000000;
    if (ticks != c->seq_spin) {  // ordered before the walk by the stream and seq_ev[0]
      c->seq_spin = ticks;
      if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_seq_spin_ticks), &c->seq_spin, sizeof(int64_t), 0,
                                 hipMemcpyHostToDevice, c->stream) != hipSuccess ||
          hipStreamSynchronize(c->stream) != hipSuccess)
        return (int)hipErrorUnknown;
    }
    if (hipEventRecord(c->seq_ev[0], c->stream) != hipSuccess ||
        hipStreamWaitEvent(c->seq_aux, c->seq_ev[0], 0) != hipSuccess ||
        hipStreamWaitEvent(c->seq_walk, c->seq_ev[0], 0) != hipSuccess)
      return (int)hipErrorUnknown;
    trans_kernel<<<dim3((unsigned)K), dim3(kT), 0, c->seq_aux>>>(w, *V, nv, n, self, pre, segT, subT, K, stop, ready,
                                                                 c->seq_epoch);
    launch_walk(c->seq_walk, ready, c->seq_epoch, fail, 0);
    if (hipEventRecord(c->seq_ev[1], c->seq_aux) != hipSuccess ||
        hipEventRecord(c->seq_ev[2], c->seq_walk) != hipSuccess ||
        hipStreamWaitEvent(c->stream, c->seq_ev[1], 0) != hipSuccess ||  // the next call reuses the records
        hipStreamWaitEvent(c->stream, c->seq_ev[2], 0) != hipSuccess)    // and reads the sums
      return (int)hipErrorUnknown;
    // The overlap needs the builds and the walk resident together.  Where they are not (a profiler that serialises
    // dispatches, another process holding the GPU's queues), the walk's waits give up after 4 s and it leaves its
    // epoch in *fail; this launch, behind both on the context's stream, then walks the now complete records again.
    // Otherwise every workgroup of it returns at once.
    launch_walk(c->stream, nullptr, 0, fail, c->seq_epoch);
  } else {
    trans_kernel<<<dim3((unsigned)K), dim3(kT), 0, c->stream>>>(w, *V, nv, n, self, pre, segT, subT, K, stop,
                                                                nullptr, 0);
    if (!ripwalk)
      k_seqx_walk<<<dim3(nv), dim3(kWalkT), 0, c->stream>>>(w, *V, n, self, segT, subT, K, acc_in, partial, nchunks,
                                                            stop, dstats, prep);
    else
      launch_walk(c->stream, nullptr, 0, nullptr, 0);
  }
  if (dstats) {
    int64_t h[16 * MSK_MAX_GROUP];
    if (hipMemcpyAsync(h, dstats, sizeof(h), hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
        hipStreamSynchronize(c->stream) == hipSuccess)
      for (int v = 0; v < nv; ++v)
        fprintf(stderr,
                ripwalk ? "seqx n=%lld nv=%d v=%d win_rip=%lld seg_desc=%lld sub_rip=%lld sub_serial=%lld pf_hit=%lld "
                          "pf_miss=%lld f_guess=%lld f_range=%lld us_scan=%lld us_single=%lld us_serial=%lld us_wait=%lld "
                          "us_all=%lld us_win=%lld us_subld=%lld us_fill=%lld\n"
                        : "seqx n=%lld nv=%d v=%d scans=%lld seg_desc=%lld single=%lld sub_serial=%lld f_bad=%lld f_state=%lld "
                "f_guess=%lld f_range=%lld us_scan=%lld us_single=%lld us_serial=%lld us_wait=%lld us_all=%lld "
                "us_win=%lld us_subld=%lld us_fill=%lld\n",
                (long long)n, nv, v, (long long)h[8 * v], (long long)h[8 * v + 1], (long long)h[8 * v + 2],
                (long long)h[8 * v + 3], (long long)h[8 * v + 4], (long long)h[8 * v + 5], (long long)h[8 * v + 6],
                (long long)h[8 * v + 7], (long long)h[256 + 8 * v] / 100, (long long)h[256 + 8 * v + 1] / 100,
                (long long)h[256 + 8 * v + 2] / 100, (long long)h[256 + 8 * v + 3] / 100,
                (long long)h[256 + 8 * v + 4] / 100, (long long)h[256 + 8 * v + 5] / 100,
                (long long)h[256 + 8 * v + 6] / 100, (long long)h[256 + 8 * v + 7] / 100);
    (void)hipFree(dstats);
  }
  return (int)hipGetLastError();
}

// MSP_REDUCE_SEQ's stage 1: the exact parallel engine, or the serial one (parallel_engine decides).
int mspi_seq_stage1(msp_ctx* c, const double* w, const Vecs* V, int nv, int64_t n, int self, double* partial,
                    int64_t nchunks, const int* stop) {
  if (!parallel_engine(n, self ? kParMinNorm : nv == 1 ? kParMinDot : kParMinSum))
    return msk_seq_stage1(w, V, nv, n, self, partial, nchunks, stop, c->stream);
  return seqx_core(c, w, V, nv, n, self, nullptr, partial, nchunks, stop);
}


namespace {
// the chain's result in the block partial layout: only the last block's slot carries it (a block-order sum of the
// slots is the chain); frob: one sum, carried by the last block's last column
__global__ void k_seqx_chain_out(const double* __restrict__ res, int ncol, int frob, int nseg, double* __restrict__ out,
                                 int m, const int* __restrict__ stop) {
  if (stopped(stop)) return;
  for (int i = threadIdx.x; i < nseg * ncol; i += blockDim.x) {
    const int k = i / ncol, j = i % ncol;
    const bool last = k == nseg - 1 && (!frob || j == ncol - 1);
    out[(int64_t)k * m + j] = last ? res[frob ? 0 : j] : 0.0;
  }
}

__global__ void k_seqx_copy(const double* __restrict__ a, double* __restrict__ b, int n) {
  if ((int)threadIdx.x < n) b[threadIdx.x] = a ? a[threadIdx.x] : 0.0;
}
}  // namespace

static int seqx_piece(msp_ctx* c, const double* w, const Vecs* V, int nv, int64_t n, int self, const double* acc,
                      double* res, const int* stop) {
  if (n > 0) return seqx_core(c, w, V, nv, n, self, acc, res, 1, stop);
  k_seqx_copy<<<1, MSK_MAX_GROUP, 0, c->stream>>>(acc, res, nv);  // an empty piece leaves the sums as they were
  return (int)hipGetLastError();
}

// The LSQR sums chained across the row blocks of one process (the reference's LSQR over all of R on one rank,
// SMSM-global.c:136): column j . y summed over block 0, then block 1, ... as one sequential sum; frob: the squares
// of column 0 over all blocks, then column 1, ...  The parallel engine runs piece by piece, each starting from the
// previous piece's exact result (or the serial engine: parallel_engine on the chain's length per sum).
extern "C" int mspi_seq_chain(msp_ctx* c, const mspi_seq_segs* sg, int ncol, int frob, double* out, int m,
                              const int* stop) {
  ARGCHK(sg && out && sg->nseg >= 1 && sg->nseg <= MSPI_SEQ_MAXSEG && ncol >= 1 && ncol <= m && ncol <= MSK_MAX_GROUP,
         MSP_ERR_ARG_OUTOFRANGE, "sequential chain over %d segments, %d columns", sg ? sg->nseg : -1, ncol);
  int64_t total = 0;
  for (int k = 0; k < sg->nseg; ++k) total += sg->n[k];
  if (!parallel_engine(frob ? total * ncol : total, kParMinChain)) {
    k_seq_chain<<<dim3(frob ? 1 : ncol), dim3(kT), 0, c->stream>>>(*sg, ncol, frob, out, m, stop);
    KCHK((int)hipGetLastError());
    return MSP_SUCCESS;
  }
  if (!c->seqacc) HIPCHK(hipMalloc((void**)&c->seqacc, 2 * MSK_MAX_GROUP * sizeof(double)));
  double* buf[2] = {c->seqacc, c->seqacc + MSK_MAX_GROUP};
  const double* acc = nullptr;  // +0.0
  int cur = 0;
  if (frob) {
    for (int j = 0; j < ncol; ++j)
      for (int k = 0; k < sg->nseg; ++k) {
        Vecs none = {};
        KCHK(seqx_piece(c, sg->x[k] + (int64_t)j * sg->ldx[k], &none, 1, sg->n[k], 1, acc, buf[cur], stop));
        acc = buf[cur];
        cur ^= 1;
      }
  } else {
    for (int k = 0; k < sg->nseg; ++k) {
      Vecs cols = {};  // column j of block k: x[k] + j*ldx[k]; its products with y[k] are the serial engine's
      cols.base = sg->x[k];
      cols.stride = sg->ldx[k];
      KCHK(seqx_piece(c, sg->y[k], &cols, ncol, sg->n[k], 0, acc, buf[cur], stop));
      acc = buf[cur];
      cur ^= 1;
    }
  }
  k_seqx_chain_out<<<1, 256, 0, c->stream>>>(acc, ncol, frob, sg->nseg, out, m, stop);
  KCHK((int)hipGetLastError());
  return MSP_SUCCESS;
}
