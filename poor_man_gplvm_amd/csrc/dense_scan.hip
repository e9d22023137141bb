// Dense log-domain forward filter / backward smoother for arbitrary continuous
// kernels, gfx950.
//
// The banded scans (fb_kernels.h) need the continuous kernel as a Toeplitz band of
// <= 32 bins held in fp32 linear space.  Everything else runs here, in the
// reference's own log-domain formulation:
//   filter   decoder.py:151-172   a[d',i] = LSE_d(post[d,i] + logA[d,d'])
//                                 prior[0,j] = LSE_i(a[0,i] + logK0[i,j]),  prior[1,j] = LSE_i a[1,i] - log L
//                                 post = prior + s*ll - c,  c = LSE(prior + s*ll)
//   smoother decoder.py:200-226   alpha-beta form: beta_{t-1}[d,i] = LSE_{d'}(logA[d,d'] +
//                                 LSE_j(logK[d',i,j] + v_t[d',j])),  v_t = s*ll_t + beta_t - V_t
//   chunks   decoder.py:258-332
// with logK0 an arbitrary (L, L) matrix: custom_transition_kernel
// (gp_kernel.py:30-34, 61-66), RBF kernels wider than the band limit, and the
// latent-only model (decoder_latentonly.py:33-224: dynamics pinned to A = [[1,0],[1,0]]),
// whose far latent moves carry weights like exp(-1000) that only log space holds.
//
// Layout: one 256-thread workgroup per chain; thread t owns the states j = t + 256 k
// (k < JD), so for a fixed i the reads of logK0[i, j] (forward) or logK0^T[j, i]
// (backward) are coalesced.  Chunk parallelism, boundary verification and the
// relaxation rounds follow fb_kernels.h; states and the Hilbert metric are in log space.
#include <math.h>

#include "pmg_common.h"
#include "pmg_math64.h"

#pragma clang fp contract(on)

namespace pmg {

constexpr int kDNT = 256;                 // threads per chain
constexpr int kDNW = kDNT / 64;
constexpr int kDCtlStride = 16;
enum { kDRepairs = 0, kDRounds = 1, kDErr = 2, kDPending = 4, kDArrive = 5, kDChanged = 6 };
constexpr uint64_t kDSpinTicks = 200000000ull;  // 2 s of the 100 MHz real-time clock
constexpr int kDMaxSeg = 512;
constexpr float kNegBig = -3.0e38f;       // finite "minus infinity" for online LSE

struct DenseParams {
  const float* delta;
  const float* phi;
  const double* m;
  int64_t T;
  int L, nblk, Lp;   // Lp = 256 * JD, the state stride
  const float* K;    // (L, L) logK0 [i_prev][j_next], f32 hi part
  const float* KT;   // (L, L) logK0^T [j_next][i_prev]
  const float* Klo;  // f32 residuals logK0 - K (hi + lo carries far weights like -2500 to ~1e-10)
  const float* KTlo;
  float lA00, lA01, lA10, lA11;
  float logL;
  float s;
  double s_d;
  int C, B, M;
  float tol;
  // forward
  float* alpha;      // (T, 2, L) linear, may be null
  double* log_alpha;  // (T, 2, L) log, f64
  double* logc;
  double* chunk_logz;
  double* logz;
  double* s_in;     // chunk boundary states (f64: far components are compared to ~tol)
  double* s_out;
  // backward
  const double* log_alpha_in;
  float* P;
  float* gamma;
  float* log_gamma;
  float* rho;
  double* log_rho;
  double* b_in;
  double* b_first;
  int* flags;
  int* ctl;
  double* seg_end;
  int* seg_chg;
  int G, S;
  uint64_t spin;
  const double* ll64;  // (T, L) f64 ll (exact decodes) or null: e from (delta, phi)  // grid-barrier spin bound (kDSpinTicks unless a debug override)
};

// Precision: the O(L^2) inner loop runs in f32 on arguments taken relative to the
// step's maximum (so the dominant terms are computed near 0 and round like the
// linear-space scans), while the chain state, every LSE's max + log(sum) and the
// normaliser are f64: an f32 log value near -10 would carry ~5e-7 absolute rounding per
// step, ~10x the linear scans' relative rounding, which a slowly forgetting chain
// accumulates past the 1e-5 parity bar.

// log(exp(a) + exp(b)) in f64 (the small term's exp in f32 is exact to ~1e-7 of itself)
// exp_acc (pmg_common.h) for arguments that may be -inf: below -120 the f32 result is 0
// anyway, and the clamp keeps the error term finite
__device__ __forceinline__ float exp_lg(float x) { return exp_acc(fmaxf(x, -120.f)); }

__device__ __forceinline__ double lse2d(double a, double b) {
  const double m = fmax(a, b);
  if (m == -INFINITY) return -INFINITY;
  const float t = exp_lg((float)(fmin(a, b) - m));
  return m + log1p((double)t);
}

// online (max, scaled sum) pair over f32 arguments: value = m + log(s)
struct Lse {
  float m, s;
  __device__ Lse() : m(kNegBig), s(0.f) {}
  __device__ void add(float x) {
    if (x > m) {
      s = s * __expf(m - x) + 1.f;
      m = x;
    } else {
      s += __expf(x - m);
    }
  }
  __device__ void merge(float m2, float s2) {
    if (m2 > m) {
      s = s * __expf(m - m2) + s2;
      m = m2;
    } else {
      s += s2 * __expf(m2 - m);
    }
  }
  __device__ double value() const { return s > 0.f ? (double)m + log((double)s) : -INFINITY; }
};

__device__ __forceinline__ double shfl_xor_d(double v, int o) {
  const int lo = __shfl_xor(__double2loint(v), o, 64);
  const int hi = __shfl_xor(__double2hiint(v), o, 64);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double block_max_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, shfl_xor_d(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int k = 1; k < kDNW; ++k) r = fmax(r, red[k]);
  return r;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int k = 0; k < kDNW; ++k) r += red[k];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int k = 1; k < kDNW; ++k) r = fmaxf(r, red[k]);
  return r;
}

__device__ __forceinline__ float block_min(float v, float* red) { return -block_max(-v, red); }

template <int JD>
struct DenseShared {
  float vec[2][kDNT * JD];   // the broadcast operand of the mat-vec (double-buffered by step),
  float veclo[2][kDNT * JD]; // as an f32 hi + lo pair of the f64 value
  double redd[8][kDNW];      // f64 reduction scratch, rotated over call sites
  float red[8][2 * kDNW];    // f32 reduction scratch, rotated over call sites
};

// reduction-slot rotation shared by a chain's call sites (a slot is reused only after
// 4 more barriers, so no extra barrier guards it)
template <int JD>
struct Slots {
  int rs = 0;
  __device__ float* f(DenseShared<JD>& sh) {
    float* r = sh.red[rs];
    rs = (rs + 1) & 7;
    return r;
  }
  __device__ double* d(DenseShared<JD>& sh) {
    double* r = sh.redd[rs];
    rs = (rs + 1) & 7;
    return r;
  }
};

// LSE over the workgroup of n values per thread (f64 in, f64 out): exact max, f32 sum
// of the exps relative to it, f64 log
template <int JD, int NV>
__device__ double block_lse_d(const double* v, DenseShared<JD>& sh, Slots<JD>& sl) {
  double m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NV; ++k) m = fmax(m, v[k]);
  const double M = block_max_d(m, sl.d(sh));
  if (M == -INFINITY) return -INFINITY;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) s += exp_lg((float)(v[k] - M));
  const float S = block_sum(s, sl.f(sh));
  return M + log((double)S);
}

// log emission e[t, j] = s*delta[t, j] + phi[t, j/32] = s*(ll[t, j] - m[t])
// With ll64 (exact decodes): e = s * (ll[t, j] - m[t]) from the unsplit f64 ll (the
// backward pass drops the per-step constant s*m[t]: its normalisation absorbs it).
template <int JD>
__device__ __forceinline__ void emis(const DenseParams& p, int64_t t, double e[JD]) {
#pragma unroll
  for (int k = 0; k < JD; ++k) {
    const int j = threadIdx.x + kDNT * k;
    if (p.ll64)
      e[k] = j < p.L ? p.s_d * (p.ll64[t * p.L + j] - (p.m ? p.m[t] : 0.0)) : -INFINITY;
    else
      e[k] = j < p.L ? (double)p.s * (double)p.delta[t * p.L + j] + (double)p.phi[t * p.nblk + (j >> 5)]
                     : -INFINITY;
  }
}

// the mat-vec operand v (f64, <= 0 after the shift) as an f32 hi + lo pair
__device__ __forceinline__ void put_vec(float* hi, float* lo, int i, double v) {
  const float h = (float)v;
  hi[i] = h;
  lo[i] = (float)(v - (double)h);
}

// per own output j: LSE_i(vec[i] + K[i, j]), both operands as f32 hi + lo pairs, f32
// inner loop with an online max.  Each term is exp((s - m) + ((err + vlo) + klo)) with
// s = vhi + khi rounded, err its exact rounding error (two-sum) and m the running max
// (an earlier s): for the terms that matter s - m is exact (Sterbenz), so a term whose
// operands are both far below the peak (vec ~ -1000, K ~ -1000, ulp 6e-5) keeps its
// f64 value to ~1e-7 -- the joint rows of latents the posterior never visits are ratios
// of exactly such terms.  Value in f64.
__device__ __forceinline__ double matvec_lse(const float* vec, const float* veclo, const float* col,
                                             const float* clo, int L) {
  Lse l;
  int i = 0;
  for (; i + 8 <= L; i += 8) {
    float kh[8], kl[8], sv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      kh[q] = col[(size_t)(i + q) * L];
      kl[q] = clo[(size_t)(i + q) * L];
      sv[q] = vec[i + q] + kh[q];
    }
    float bm = sv[0];
#pragma unroll
    for (int q = 1; q < 8; ++q) bm = fmaxf(bm, sv[q]);
    if (bm > l.m) {
      l.s *= exp_lg(l.m - bm);
      l.m = bm;
    }
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float vh = vec[i + q];
      const float bb = sv[q] - vh;
      const float err = (vh - (sv[q] - bb)) + (kh[q] - bb);
      acc += exp_lg((sv[q] - l.m) + ((err + veclo[i + q]) + kl[q]));
    }
    l.s += acc;
  }
  for (; i < L; ++i) {
    const float kh = col[(size_t)i * L], kl = clo[(size_t)i * L];
    const float vh = vec[i];
    const float x = vh + kh;
    if (x > l.m) {
      l.s *= exp_lg(l.m - x);
      l.m = x;
    }
    const float bb = x - vh;
    const float err = (vh - (x - bb)) + (kh - bb);
    l.s += exp_lg((x - l.m) + ((err + veclo[i]) + kl));
  }
  return l.value();
}

// ---------------------------------------------------------------------------
// forward chain
// ---------------------------------------------------------------------------
template <int JD>
struct DFwd {
  double x0[JD], x1[JD];  // log filter state (normalised: LSE = 0), f64
  Slots<JD> sl;

  __device__ void init_uniform(const DenseParams& p) {
    const double u = -log(2.0 * (double)p.L);   // log(1/(D L)), decoder.py:181
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      x0[k] = x1[k] = j < p.L ? u : -INFINITY;
    }
  }
  __device__ void normalise(DenseShared<JD>& sh) {
    double v[2 * JD];
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      v[k] = x0[k];
      v[JD + k] = x1[k];
    }
    const double z = block_lse_d<JD, 2 * JD>(v, sh, sl);
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      x0[k] -= z;
      x1[k] -= z;
    }
  }
  __device__ void load(const DenseParams& p, const double* src, DenseShared<JD>& sh) {
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      x0[k] = j < p.L ? src[j] : -INFINITY;
      x1[k] = j < p.L ? src[p.Lp + j] : -INFINITY;
    }
    normalise(sh);
  }
  __device__ void save(const DenseParams& p, double* dst) const {
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      if (j < p.L) {
        dst[j] = x0[k];
        dst[p.Lp + j] = x1[k];
      }
    }
  }
  // one step with log emission e; returns the log normaliser c
  __device__ double step(const DenseParams& p, DenseShared<JD>& sh, int buf, const double e[JD]) {
    float* vec = sh.vec[buf];
    float* veclo = sh.veclo[buf];
    double a0[JD], a1[JD], am = -INFINITY;
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      a0[k] = lse2d(x0[k] + p.lA00, x1[k] + p.lA10);
      a1[k] = lse2d(x0[k] + p.lA01, x1[k] + p.lA11);
      am = fmax(am, a0[k]);
    }
    const double A = block_max_d(am, sl.d(sh));          // shift of the continuous operand
#pragma unroll
    for (int k = 0; k < JD; ++k) put_vec(vec, veclo, threadIdx.x + kDNT * k, a0[k] - A);
    const double jump = block_lse_d<JD, JD>(a1, sh, sl) - (double)p.logL;   // barriers: vec visible
    double x[2 * JD];
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      const double pr = j < p.L ? A + matvec_lse(vec, veclo, p.K + j, p.Klo + j, p.L) : -INFINITY;
      x[k] = pr + e[k];
      x[JD + k] = jump + e[k];
    }
    const double c = block_lse_d<JD, 2 * JD>(x, sh, sl);
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      x0[k] = x[k] - c;
      x1[k] = x[JD + k] - c;
    }
    return c;
  }
  __device__ void write_out(const DenseParams& p, int64_t t) const {
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      if (j < p.L) {
        const size_t o = (size_t)t * 2 * p.L + j;
        p.log_alpha[o] = x0[k];
        p.log_alpha[o + p.L] = x1[k];
        if (p.alpha) {
          p.alpha[o] = (float)exp(x0[k]);
          p.alpha[o + p.L] = (float)exp(x1[k]);
        }
      }
    }
  }
};

// run steps [t_a, t_b); OUT: write outputs, return sum of logc
template <int JD, bool OUT>
__device__ double dfwd_run(const DenseParams& p, DFwd<JD>& st, DenseShared<JD>& sh, int64_t t_a, int64_t t_b) {
  double lz = 0.0;
  for (int64_t t = t_a; t < t_b; ++t) {
    double e[JD];
    emis<JD>(p, t, e);
    const double c = st.step(p, sh, (int)(t & 1), e);
    if constexpr (OUT) {
      st.write_out(p, t);
      const double lc = c + p.s_d * p.m[t];
      if (threadIdx.x == 0) p.logc[t] = lc;
      lz += lc;
    }
  }
  return lz;
}

template <int JD>
__global__ void __launch_bounds__(kDNT) k_dense_forward(DenseParams p) {
  __shared__ DenseShared<JD> sh;
  const int c = blockIdx.x;
  if (c >= p.M) return;
  const size_t SZ = (size_t)2 * p.Lp;
  const int64_t t_c = (int64_t)c * p.C;
  const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
  int64_t t0 = c == 0 ? 0 : t_c - p.B;
  if (t0 < 0) t0 = 0;
  DFwd<JD> st;
  st.init_uniform(p);
  dfwd_run<JD, false>(p, st, sh, t0, t_c);
  if (c > 0) st.save(p, p.s_in + (size_t)c * SZ);
  const double lz = dfwd_run<JD, true>(p, st, sh, t_c, t_e);
  st.save(p, p.s_out + (size_t)c * SZ);
  if (threadIdx.x == 0) p.chunk_logz[c] = lz;
}

// ---------------------------------------------------------------------------
// Boundary distance of the dense scans (one wave).  Unlike the banded scans'
// thresholded Hilbert metric, EVERY component counts: without a jump state (the
// latent-only model) a component far below the peak (e^-150) can still dominate a
// later far move whose weight from the peak is e^-2500, so "negligible" components
// are not negligible here.  Both states are shifted by their max (scale-free);
// components below -1e19 on both sides (masked latents, empty dynamics) are skipped;
// one side only is a failure.  Down to kDFar below the max (1e-13 relative: below the
// outputs' 1e-12 atol) the tolerance is tol itself; further down it grows by kDRel per
// unit of |log value| (the states are f64 and the mat-vec keeps far terms to ~1e-7
// absolute, so the slack is only a guard against f64 rounding of huge logs; round 2
// needed 1e-6 with f32 states, which let far components of a boundary differ by 1e-3).
// Returns max(|a - b| - kDRel * max(0, max(|a|, |b|) - kDFar)), compared against tol.
// ---------------------------------------------------------------------------
constexpr double kDRel = 1e-10;
constexpr double kDFar = 30.0;
constexpr double kDEmpty = -1e19;

__device__ __forceinline__ double dense_comp(double a, double b) {
  const bool ea = a < kDEmpty, eb = b < kDEmpty;
  if (ea && eb) return 0.0;
  if (ea != eb) return INFINITY;
  return fabs(a - b) - kDRel * fmax(0.0, fmax(fabs(a), fabs(b)) - kDFar);
}

__device__ float dense_hilbert(const double* x, const double* y, int L, int Lp, const float* w) {
  (void)w;
  const int lane = threadIdx.x & 63;
  double xm = -INFINITY, ym = -INFINITY;
  for (int i = lane; i < 2 * L; i += 64) {
    const int d = i >= L, j = i - d * L;
    xm = fmax(xm, x[d * Lp + j]);
    ym = fmax(ym, y[d * Lp + j]);
  }
  xm = wave_max_f64(xm);
  ym = wave_max_f64(ym);
  if (!(xm > kDEmpty) || !(ym > kDEmpty)) return INFINITY;
  double dev = 0.0;
  for (int i = lane; i < 2 * L; i += 64) {
    const int d = i >= L, j = i - d * L;
    dev = fmax(dev, dense_comp(x[d * Lp + j] - xm, y[d * Lp + j] - ym));
  }
  return (float)wave_max_f64(dev);
}

// flags[c] = dist(x[c], y[c + off]) > tol; a failing boundary snapshots y into x
__global__ void __launch_bounds__(256) k_dense_verify(double* __restrict__ x, const double* __restrict__ y, int first,
                                                      int last, int off, int L, int Lp, float tol,
                                                      int* __restrict__ flags, const float* __restrict__ w, int C,
                                                      int* __restrict__ pending) {
  const int c = first + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c > last) return;
  const size_t SZ = (size_t)2 * Lp;
  const double* yc = y + (size_t)(c + off) * SZ;
  double* xc = x + (size_t)c * SZ;
  const float* wc = w ? w + (size_t)(c + 1) * C * 2 * L : nullptr;
  const float d = dense_hilbert(xc, yc, L, Lp, wc);
  const bool bad = !(d <= tol);
  if ((threadIdx.x & 63) == 0) {
    flags[c] = bad ? 1 : 0;
    if (bad) atomicAdd(pending, 1);
  }
  if (bad)
    for (int i = threadIdx.x & 63; i < (int)SZ; i += 64) xc[i] = yc[i];
}

// ---------------------------------------------------------------------------
// relaxation plumbing at workgroup granularity (fb_kernels.h protocol)
// ---------------------------------------------------------------------------
__device__ bool dense_barrier(int* ctl, int target, int* okword, uint64_t spin) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctl + kDArrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(ctl + kDArrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__hip_atomic_load(ctl + kDErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
          __builtin_amdgcn_s_memrealtime() - t0 > spin) {
        __hip_atomic_store(ctl + kDErr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *okword = ok;
  }
  __syncthreads();
  const int ok = *okword;
  __syncthreads();
  return ok != 0;
}

__device__ __forceinline__ void dense_publish(const DenseParams& p, int k, int s, bool changed) {
  if (threadIdx.x == 0) {
    p.seg_chg[(k & 1) * p.S + s] = changed ? 1 : 0;
    if (changed) __hip_atomic_fetch_add(p.ctl + kDChanged + k % 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 0) __hip_atomic_store(p.ctl + kDChanged + (k + 1) % 3, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ int dense_ctl(int* ctl, int w, int* word) {
  if (threadIdx.x == 0) *word = __hip_atomic_load(ctl + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int v = *word;
  __syncthreads();
  return v;
}

// first (DIR > 0) / last (DIR < 0) flagged index in [lo, hi), or -1 (whole block)
template <int DIR>
__device__ int dense_find_flag(const int* flags, int lo, int hi) {
  for (int q = 0; q < hi - lo; q += kDNT) {
    const int idx = DIR > 0 ? lo + q + (int)threadIdx.x : hi - 1 - q - (int)threadIdx.x;
    const bool f = (DIR > 0 ? idx < hi : idx >= lo) && flags[idx] != 0;
    const int hit = __syncthreads_or(f);
    if (hit) {
      __shared__ int best;
      if (threadIdx.x == 0) best = DIR > 0 ? 0x7fffffff : -1;
      __syncthreads();
      if (f) {
        if (DIR > 0) atomicMin(&best, idx);
        else atomicMax(&best, idx);
      }
      __syncthreads();
      const int r = best;
      __syncthreads();
      return r;
    }
  }
  return -1;
}

// Hilbert distance between a register state and a state in memory (whole block):
// per-thread partial max/min, block reductions
template <int JD>
__device__ float dense_hilbert_reg(const DenseParams& p, DenseShared<JD>& sh, Slots<JD>& sl, const double x0[JD],
                                   const double x1[JD], const double* y) {
  double xm = -INFINITY, ym = -INFINITY;
  double a[2 * JD], b[2 * JD];
#pragma unroll
  for (int k = 0; k < JD; ++k) {
    const int j = threadIdx.x + kDNT * k;
    const bool in = j < p.L;
    a[k] = in ? x0[k] : -INFINITY;
    a[JD + k] = in ? x1[k] : -INFINITY;
    b[k] = in ? y[j] : -INFINITY;
    b[JD + k] = in ? y[p.Lp + j] : -INFINITY;
  }
#pragma unroll
  for (int k = 0; k < 2 * JD; ++k) {
    xm = fmax(xm, a[k]);
    ym = fmax(ym, b[k]);
  }
  xm = block_max_d(xm, sl.d(sh));
  ym = block_max_d(ym, sl.d(sh));
  if (!(xm > kDEmpty) || !(ym > kDEmpty)) return INFINITY;
  double dev = 0.0;
#pragma unroll
  for (int k = 0; k < 2 * JD; ++k) {
    const int j = threadIdx.x + kDNT * (k % JD);
    if (j < p.L) dev = fmax(dev, dense_comp(a[k] - xm, b[k] - ym));
  }
  return (float)block_max_d(dev, sl.d(sh));
}

template <int JD>
__device__ bool dfwd_segment(const DenseParams& p, DFwd<JD>& st, DenseShared<JD>& sh, int c0, int b,
                             const int* flg, int& nrep, int* stop = nullptr) {
  const size_t SZ = (size_t)2 * p.Lp;
  for (int c = c0; c < b; ++c) {
    const int64_t t_c = (int64_t)c * p.C;
    const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
    st.save(p, p.s_in + (size_t)c * SZ);
    const double lz = dfwd_run<JD, true>(p, st, sh, t_c, t_e);
    if (threadIdx.x == 0) p.chunk_logz[c] = lz;
    ++nrep;
    double* so = p.s_out + (size_t)c * SZ;
    const float d = dense_hilbert_reg<JD>(p, sh, st.sl, st.x0, st.x1, so);
    __syncthreads();
    st.save(p, so);
    if (d <= p.tol && (c + 1 >= b || !(flg && flg[c + 1]))) {
      if (stop) *stop = c;
      return false;
    }
  }
  return true;
}

template <int JD>
__global__ void __launch_bounds__(kDNT) k_dense_forward_relax(DenseParams p) {
  __shared__ DenseShared<JD> sh;
  __shared__ int word;
  const size_t SZ = (size_t)2 * p.Lp;
  const int s = blockIdx.x;
  int nrep = 0, rounds = 0;
  if (dense_ctl(p.ctl, kDPending, &word) > 0) {
    const int a = s * p.G;
    const int b = a + p.G < p.M ? a + p.G : p.M;
    DFwd<JD> st;
    bool changed = false;
    // round 0: every flagged boundary of the segment (see forward_relax in fb_kernels.h)
    int c0 = dense_find_flag<1>(p.flags, a > 1 ? a : 1, b);
    while (c0 >= 0) {
      st.load(p, p.s_in + (size_t)c0 * SZ, sh);
      int stop = b;
      changed = dfwd_segment<JD>(p, st, sh, c0, b, p.flags, nrep, &stop);
      if (changed) break;
      c0 = stop + 2 < b ? dense_find_flag<1>(p.flags, stop + 2, b) : -1;
    }
    for (int k = 0;; ++k) {
      if (changed) st.save(p, p.seg_end + ((size_t)(k & 1) * p.S + s) * SZ);
      dense_publish(p, k, s, changed);
      ++rounds;
      if (!dense_barrier(p.ctl, (k + 1) * p.S, &word, p.spin)) break;
      if (dense_ctl(p.ctl, kDChanged + k % 3, &word) == 0) break;
      changed = false;
      if (s > 0 && p.seg_chg[(k & 1) * p.S + s - 1]) {
        const double* X = p.seg_end + ((size_t)(k & 1) * p.S + s - 1) * SZ;
        if (threadIdx.x < 64) {
          const float d = dense_hilbert(X, p.s_in + (size_t)a * SZ, p.L, p.Lp, nullptr);
          if (threadIdx.x == 0) word = !(d <= p.tol);
        }
        __syncthreads();
        const int redo = word;
        __syncthreads();
        if (redo) {
          st.load(p, X, sh);
          changed = dfwd_segment<JD>(p, st, sh, a, b, nullptr, nrep);
        }
      }
    }
  }
  if (threadIdx.x == 0 && nrep) atomicAdd(p.ctl + kDRepairs, nrep);
  if (s == 0 && threadIdx.x < 64) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < p.M; i += 64) acc += p.chunk_logz[i];
    acc = wave_sum_f64(acc);
    if (threadIdx.x == 0) {
      p.logz[0] = acc;
      p.ctl[kDRounds] = rounds;
    }
  }
}

// ---------------------------------------------------------------------------
// backward chain (log beta, alpha-beta smoothing)
// ---------------------------------------------------------------------------
template <int JD>
struct DBwd {
  double b0[JD], b1[JD];  // log beta at the current time (f64)
  Slots<JD> sl;

  __device__ void init_ones(const DenseParams& p) {
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      b0[k] = b1[k] = j < p.L ? 0.0 : -INFINITY;
    }
  }
  __device__ void load(const DenseParams& p, const double* src) {
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      b0[k] = j < p.L ? src[j] : -INFINITY;
      b1[k] = j < p.L ? src[p.Lp + j] : -INFINITY;
    }
  }
  __device__ void save(const DenseParams& p, double* dst) const {
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      if (j < p.L) {
        dst[j] = b0[k];
        dst[p.Lp + j] = b1[k];
      }
    }
  }
  // beta_t -> beta_{t-1} with log emission e_t; v (the normalised e*beta) kept
  __device__ void step_back(const DenseParams& p, DenseShared<JD>& sh, int buf, const double e[JD], double v0[JD],
                            double v1[JD]) {
    double u[2 * JD];
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      u[k] = e[k] + b0[k];
      u[JD + k] = e[k] + b1[k];
    }
    const double V = block_lse_d<JD, 2 * JD>(u, sh, sl);
    double vm = -INFINITY;
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      v0[k] = u[k] - V;
      v1[k] = u[JD + k] - V;
      vm = fmax(vm, v0[k]);
    }
    const double A = block_max_d(vm, sl.d(sh));
    float* vec = sh.vec[buf];
    float* veclo = sh.veclo[buf];
#pragma unroll
    for (int k = 0; k < JD; ++k) put_vec(vec, veclo, threadIdx.x + kDNT * k, v0[k] - A);
    const double w1 = block_lse_d<JD, JD>(v1, sh, sl) - (double)p.logL;   // barriers: vec visible
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int i = threadIdx.x + kDNT * k;
      if (i < p.L) {
        const double w0 = A + matvec_lse(vec, veclo, p.KT + i, p.KTlo + i, p.L);   // KT[j][i] = logK0[i][j]
        b0[k] = lse2d(p.lA00 + w0, p.lA01 + w1);
        b1[k] = lse2d(p.lA10 + w0, p.lA11 + w1);
      } else {
        b0[k] = b1[k] = -INFINITY;
      }
    }
  }
};

// output steps t = t_e-1 .. t_c; on entry st = beta_{t_e-1}, (vp0, vp1) = v_{t_e}
// (has_prev false at the sequence end); on exit st = beta_{t_c}
template <int JD>
__device__ void dbwd_out(const DenseParams& p, DBwd<JD>& st, DenseShared<JD>& sh, int64_t t_c, int64_t t_e,
                         double vp0[JD], double vp1[JD], bool has_prev) {
  for (int64_t t = t_e - 1; t >= t_c; --t) {
    double la[2 * JD];
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      const size_t o = (size_t)t * 2 * p.L + j;
      la[k] = j < p.L ? p.log_alpha_in[o] + st.b0[k] : -INFINITY;
      la[JD + k] = j < p.L ? p.log_alpha_in[o + p.L] + st.b1[k] : -INFINITY;
    }
    const double G = block_lse_d<JD, 2 * JD>(la, sh, st.sl);
#pragma unroll
    for (int k = 0; k < JD; ++k) {
      const int j = threadIdx.x + kDNT * k;
      if (j < p.L) {
        const size_t o = (size_t)t * 2 * p.L + j;
        const double g0 = la[k] - G, g1 = la[JD + k] - G;
        const double e0 = exp(g0), e1 = exp(g1);
        if (p.P) p.P[(size_t)t * p.L + j] = (float)(e0 + e1);
        if (p.gamma) {
          p.gamma[o] = (float)e0;
          p.gamma[o + p.L] = (float)e1;
        }
        if (p.log_gamma) {
          p.log_gamma[o] = (float)g0;
          p.log_gamma[o + p.L] = (float)g1;
        }
        if (has_prev && t + 1 < p.T) {   // rho_{t+1} = v_{t+1} / sum(alpha_t beta_t)
          const size_t o1 = (size_t)(t + 1) * 2 * p.L + j;
          if (p.rho) {
            p.rho[o1] = (float)exp(vp0[k] - G);
            p.rho[o1 + p.L] = (float)exp(vp1[k] - G);
          }
          if (p.log_rho) {
            p.log_rho[o1] = vp0[k] - G;
            p.log_rho[o1 + p.L] = vp1[k] - G;
          }
        }
      }
    }
    if (t != t_c) {
      double e[JD];
      emis<JD>(p, t, e);
      st.step_back(p, sh, (int)(t & 1), e, vp0, vp1);
      has_prev = true;
    }
  }
}

template <int JD>
__global__ void __launch_bounds__(kDNT) k_dense_backward(DenseParams p) {
  __shared__ DenseShared<JD> sh;
  const int c = blockIdx.x;
  if (c >= p.M) return;
  const size_t SZ = (size_t)2 * p.Lp;
  const int64_t t_c = (int64_t)c * p.C;
  const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
  DBwd<JD> st;
  st.init_ones(p);
  double vp0[JD], vp1[JD];
#pragma unroll
  for (int k = 0; k < JD; ++k) vp0[k] = vp1[k] = -INFINITY;
  bool has_prev = false;
  if (c < p.M - 1) {
    int64_t t_w = t_e + p.B;
    if (t_w > p.T - 1) t_w = p.T - 1;
    for (int64_t t = t_w; t >= t_e + 1; --t) {   // warm-up: beta guess (ones) at t_w
      double e[JD], v0[JD], v1[JD];
      emis<JD>(p, t, e);
      st.step_back(p, sh, (int)(t & 1), e, v0, v1);
    }
    st.save(p, p.b_in + (size_t)c * SZ);           // beta_{t_e}: the start the verify checks
    double e[JD];
    emis<JD>(p, t_e, e);
    st.step_back(p, sh, (int)(t_e & 1), e, vp0, vp1);
    has_prev = true;
  }
  dbwd_out<JD>(p, st, sh, t_c, t_e, vp0, vp1, has_prev);
  st.save(p, p.b_first + (size_t)c * SZ);
}

template <int JD>
__device__ bool dbwd_segment(const DenseParams& p, DBwd<JD>& st, DenseShared<JD>& sh, int c0, int a,
                             const int* flg, int& nrep, int* stop = nullptr) {
  const size_t SZ = (size_t)2 * p.Lp;
  for (int c = c0; c >= a; --c) {
    const int64_t t_c = (int64_t)c * p.C;
    const int64_t t_e = t_c + p.C;
    st.save(p, p.b_in + (size_t)c * SZ);
    double vp0[JD], vp1[JD], e[JD];
    emis<JD>(p, t_e, e);
    st.step_back(p, sh, (int)(t_e & 1), e, vp0, vp1);
    dbwd_out<JD>(p, st, sh, t_c, t_e, vp0, vp1, true);
    ++nrep;
    double* bf = p.b_first + (size_t)c * SZ;
    const float d = dense_hilbert_reg<JD>(p, sh, st.sl, st.b0, st.b1, bf);
    __syncthreads();
    st.save(p, bf);
    if (d <= p.tol && (c == a || !(flg && flg[c - 1]))) {
      if (stop) *stop = c;
      return false;
    }
  }
  return true;
}

template <int JD>
__global__ void __launch_bounds__(kDNT) k_dense_backward_relax(DenseParams p) {
  __shared__ DenseShared<JD> sh;
  __shared__ int word;
  const size_t SZ = (size_t)2 * p.Lp;
  const int s = blockIdx.x;
  int nrep = 0, rounds = 0;
  if (dense_ctl(p.ctl, kDPending, &word) > 0) {
    const int a = s * p.G;
    const int b = a + p.G < p.M ? a + p.G : p.M;
    const int top = b < p.M - 1 ? b : p.M - 1;
    DBwd<JD> st;
    bool changed = false;
    int c0 = dense_find_flag<-1>(p.flags, a, top);
    while (c0 >= 0) {
      st.load(p, p.b_in + (size_t)c0 * SZ);
      int stop = a;
      changed = dbwd_segment<JD>(p, st, sh, c0, a, p.flags, nrep, &stop);
      if (changed) break;
      c0 = stop - 1 > a ? dense_find_flag<-1>(p.flags, a, stop - 1) : -1;
    }
    for (int k = 0;; ++k) {
      if (changed) st.save(p, p.seg_end + ((size_t)(k & 1) * p.S + s) * SZ);
      dense_publish(p, k, s, changed);
      ++rounds;
      if (!dense_barrier(p.ctl, (k + 1) * p.S, &word, p.spin)) break;
      if (dense_ctl(p.ctl, kDChanged + k % 3, &word) == 0) break;
      changed = false;
      if (s + 1 < p.S && p.seg_chg[(k & 1) * p.S + s + 1]) {
        const double* X = p.seg_end + ((size_t)(k & 1) * p.S + s + 1) * SZ;
        if (threadIdx.x < 64) {
          const float d = dense_hilbert(p.b_in + (size_t)(b - 1) * SZ, X, p.L, p.Lp, nullptr);
          if (threadIdx.x == 0) word = !(d <= p.tol);
        }
        __syncthreads();
        const int redo = word;
        __syncthreads();
        if (redo) {
          st.load(p, X);
          changed = dbwd_segment<JD>(p, st, sh, b - 1, a, nullptr, nrep);
        }
      }
    }
  }
  if (threadIdx.x == 0) {
    if (nrep) atomicAdd(p.ctl + kDRepairs, nrep);
    if (s == 0) p.ctl[kDRounds] = rounds;
  }
}

// ---------------------------------------------------------------------------
// Pairwise joint in log space (decode only):
//   logS[x, x'] = LSE_{t < T-1} (log_alpha_t[x] + log_rho_{t+1}[x']),  x = (d, i),
// so that log joint = logA + logK + logS (decoder.py:215-221 accumulates the same sum
// with logaddexp).  The linear T-contraction (pmg_joint_accumulate) cannot hold it
// when a far move makes rho ~ e^{+1000} against K ~ e^{-1000} (latent-only chains).
//
// Blocked form (round 5): per 64 x 64 tile of (x, x') and per block of kJB time steps,
// the block's log values are shifted by their row maxima mx_x and column maxima my_x'
// (over the block's steps), exponentiated ONCE per (row, step) and (column, step) in
// f64, and the block sum s = sum_t e^{la_t[x] - mx_x} e^{lr_t[x'] - my_x'} is a plain
// f64 contraction (16 FMAs per step per thread); it is folded into the entry's running
// (m, sum) pair at reference mx_x + my_x'.  That is 128 exps per step per tile instead of
// 4096.  Every product is <= 1 and the row's and column's largest are 1, so s loses
// nothing unless the row's and the column's peaks inside the block are more than ~650
// nats apart in the product: a block sum below 1e-280 is recomputed for that entry term
// by term in log space (the per-pair form of round 4), so no entry's value depends on
// the range of f64.  The time axis is split over gridDim.z workgroups (occupancy); their
// (m, sum) partials are combined in split order by k_joint_log_combine.
// ---------------------------------------------------------------------------
constexpr int kJT = 64, kJB = 64;
constexpr int kJointSplits = 8;   // time splits of the joint (workspace partials)

__device__ __forceinline__ void lse_fold(double& m, double& sm, double r, double s) {
  if (!(s > 0.0)) return;
  if (r > m) {
    sm = (m > -INFINITY) ? fma(sm, exp_neg64(m - r), s) : s;
    m = r;
  } else {
    sm = fma(s, exp_neg64(r - m), sm);
  }
}

__global__ void __launch_bounds__(256) k_joint_log(const double* __restrict__ la, const double* __restrict__ lr,
                                                   int64_t T, int L2, int64_t steps_per_split,
                                                   double* __restrict__ part, double* __restrict__ logS) {
  __shared__ double ea[kJB][kJT], eb[kJB][kJT];   // log values, then their shifted exps
  __shared__ double mx[kJT], my[kJT];
  const int x0 = blockIdx.x * kJT, y0 = blockIdx.y * kJT;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t ta = (int64_t)blockIdx.z * steps_per_split;
  int64_t tb = ta + steps_per_split;
  if (tb > T - 1) tb = T - 1;
  double m[4][4], sm[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      m[a][b] = -INFINITY;
      sm[a][b] = 0.0;
    }
  for (int64_t t0 = ta; t0 < tb; t0 += kJB) {
    for (int k = threadIdx.x; k < kJB * kJT; k += 256) {
      const int tt = k / kJT, c = k % kJT;
      const int64_t t = t0 + tt;
      const bool ok = t < tb;
      ea[tt][c] = (ok && x0 + c < L2) ? la[t * L2 + x0 + c] : -INFINITY;
      eb[tt][c] = (ok && y0 + c < L2) ? lr[(t + 1) * L2 + y0 + c] : -INFINITY;
    }
    __syncthreads();
    {   // row / column maxima over the block: two threads per column
      const int col = threadIdx.x >> 1, half = threadIdx.x & 1;
      double v = -INFINITY;
      if (col < kJT) {
        for (int tt = half; tt < kJB; tt += 2) v = fmax(v, ea[tt][col]);
      } else {
        for (int tt = half; tt < kJB; tt += 2) v = fmax(v, eb[tt][col - kJT]);
      }
      v = fmax(v, __shfl_xor(v, 1, 64));
      if (half == 0) {
        if (col < kJT) mx[col] = v;
        else my[col - kJT] = v;
      }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kJB * kJT; k += 256) {
      const int tt = k / kJT, c = k % kJT;
      const double ma = mx[c], mb = my[c];
      ea[tt][c] = ma > -INFINITY ? exp_neg64(ea[tt][c] - ma) : 0.0;
      eb[tt][c] = mb > -INFINITY ? exp_neg64(eb[tt][c] - mb) : 0.0;
    }
    __syncthreads();
    double s[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) s[a][b] = 0.0;
    for (int tt = 0; tt < kJB; ++tt) {
      double av[4], rv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) av[a] = ea[tt][ty * 4 + a];
#pragma unroll
      for (int b = 0; b < 4; ++b) rv[b] = eb[tt][tx * 4 + b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) s[a][b] = fma(av[a], rv[b], s[a][b]);
    }
    bool redo = false;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const double r = mx[ty * 4 + a] + my[tx * 4 + b];
        if (!(r > -INFINITY)) continue;                 // a masked row or column: no terms
        if (s[a][b] >= 1e-280) lse_fold(m[a][b], sm[a][b], r, s[a][b]);
        else redo = true;
      }
    if (redo) {
      // term by term in log space for the entries whose block sum left f64's range (the
      // rows' and columns' peaks far apart inside the block); the logs from global memory
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int x = x0 + ty * 4 + a, y = y0 + tx * 4 + b;
          const double r = mx[ty * 4 + a] + my[tx * 4 + b];
          if (!(r > -INFINITY) || s[a][b] >= 1e-280 || x >= L2 || y >= L2) continue;
          const int64_t te = t0 + kJB < tb ? t0 + kJB : tb;
          double bm = -INFINITY;
          for (int64_t t = t0; t < te; ++t) bm = fmax(bm, la[t * L2 + x] + lr[(t + 1) * L2 + y]);
          if (!(bm > -INFINITY)) continue;
          double bs = 0.0;
          for (int64_t t = t0; t < te; ++t) bs += exp_neg64((la[t * L2 + x] + lr[(t + 1) * L2 + y]) - bm);
          lse_fold(m[a][b], sm[a][b], bm, bs);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int x = x0 + ty * 4 + a, y = y0 + tx * 4 + b;
      if (x >= L2 || y >= L2) continue;
      if (part) {
        double* q = part + ((size_t)blockIdx.z * L2 * L2 + (size_t)x * L2 + y) * 2;
        q[0] = m[a][b];
        q[1] = sm[a][b];
      } else {
        logS[(size_t)x * L2 + y] = sm[a][b] > 0.0 ? m[a][b] + log(sm[a][b]) : -INFINITY;
      }
    }
}

// the splits' (m, sum) partials of every entry, folded in split order
__global__ void k_joint_log_combine(const double* __restrict__ part, int nsplit, int64_t n, double* __restrict__ logS) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double m = -INFINITY, sm = 0.0;
  for (int z = 0; z < nsplit; ++z) {
    const double* q = part + ((size_t)z * n + i) * 2;
    lse_fold(m, sm, q[0], q[1]);
  }
  logS[i] = sm > 0.0 ? m + log(sm) : -INFINITY;
}

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
struct DenseWork {
  int* ctl;
  double *s_in, *s_out, *b_in, *b_first;
  double* chunk_logz;
  int* flags;
  double* seg_end;
  int* seg_chg;
};

// latents per thread: JD = 8 carries L in (1024, 2048], which the banded scans do not hold
static int dense_jd(int L) {
  return L <= 256 ? 1 : L <= 512 ? 2 : L <= 1024 ? 4 : L <= 2048 ? 8 : L <= 4096 ? 16 : -1;
}

static DenseWork carve_dense(void* ws, int64_t T, int Lp, int C, size_t* total = nullptr) {
  const int64_t M = (T + C - 1) / C;
  Carver c(ws);
  DenseWork w;
  w.ctl = c.take<int>(64);
  w.s_in = c.take<double>((size_t)M * 2 * Lp);
  w.s_out = c.take<double>((size_t)M * 2 * Lp);
  w.b_in = c.take<double>((size_t)M * 2 * Lp);
  w.b_first = c.take<double>((size_t)M * 2 * Lp);
  w.chunk_logz = c.take<double>(M);
  w.flags = c.take<int>(M);
  w.seg_end = c.take<double>((size_t)2 * kDMaxSeg * 2 * Lp);
  w.seg_chg = c.take<int>(2 * kDMaxSeg);
  if (total) *total = c.off + 256;
  return w;
}

static int dense_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 64;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 64;
  return n;
}

static int dense_params(DenseParams& p, const pmg_dense_transition* tr, int64_t T, int C, int B, double s,
                        double tol) {
  PMG_REQUIRE(tr && tr->L > 0 && tr->logK && tr->logKT && tr->logK_lo && tr->logKT_lo,
              "pmg dense scan: bad transition");
  PMG_REQUIRE(T > 0 && C > 0 && B >= 0, "pmg dense scan: T=%lld chunk=%d warmup=%d", (long long)T, C, B);
  const int JD = dense_jd(tr->L);
  PMG_REQUIRE(JD > 0, "pmg dense scan: L=%d > 4096 unsupported", tr->L);
  memset(&p, 0, sizeof(p));
  p.T = T;
  p.L = tr->L;
  p.nblk = (int)(round_up(tr->L, 32) / 32);
  p.Lp = kDNT * JD;
  p.K = tr->logK;
  p.KT = tr->logKT;
  p.Klo = tr->logK_lo;
  p.KTlo = tr->logKT_lo;
  p.lA00 = tr->logA[0];
  p.lA01 = tr->logA[1];
  p.lA10 = tr->logA[2];
  p.lA11 = tr->logA[3];
  p.logL = logf((float)tr->L);
  p.s = (float)s;
  p.s_d = s;
  p.C = C;
  p.B = B;
  p.M = (int)((T + C - 1) / C);
  p.tol = (float)tol;
  int S = dense_cus();
  if (S > kDMaxSeg) S = kDMaxSeg;
  if (S > p.M) S = p.M;
  p.G = (p.M + S - 1) / S;
  p.S = (p.M + p.G - 1) / p.G;
  p.spin = spin_ticks(kDSpinTicks);
  return PMG_OK;
}

typedef void (*dense_kernel_t)(DenseParams);

static void dense_kernels(int JD, dense_kernel_t* f, dense_kernel_t* fr, dense_kernel_t* b, dense_kernel_t* br) {
  switch (JD) {
    case 1: *f = k_dense_forward<1>; *fr = k_dense_forward_relax<1>; *b = k_dense_backward<1>; *br = k_dense_backward_relax<1>; break;
    case 2: *f = k_dense_forward<2>; *fr = k_dense_forward_relax<2>; *b = k_dense_backward<2>; *br = k_dense_backward_relax<2>; break;
    case 4: *f = k_dense_forward<4>; *fr = k_dense_forward_relax<4>; *b = k_dense_backward<4>; *br = k_dense_backward_relax<4>; break;
    case 8: *f = k_dense_forward<8>; *fr = k_dense_forward_relax<8>; *b = k_dense_backward<8>; *br = k_dense_backward_relax<8>; break;
    default: *f = k_dense_forward<16>; *fr = k_dense_forward_relax<16>; *b = k_dense_backward<16>; *br = k_dense_backward_relax<16>; break;
  }
}

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_dense_workspace_size(int64_t T, int32_t L, int32_t chunk) {
  const int JD = dense_jd(L);
  if (JD < 0 || chunk <= 0 || T <= 0) return 0;
  size_t total = 0;
  carve_dense(nullptr, T, kDNT * JD, chunk, &total);
  return total;
}

int32_t pmg_dense_lpad(int32_t L) {
  const int JD = dense_jd(L);
  return JD < 0 ? 0 : kDNT * JD;
}

double* pmg_dense_state(void* workspace, int64_t T, int32_t L, int32_t chunk, int32_t which, int64_t c) {
  const int JD = dense_jd(L);
  if (!workspace || JD < 0 || chunk <= 0 || T <= 0) return nullptr;
  const int64_t M = (T + chunk - 1) / chunk;
  if (c < 0 || c >= M) return nullptr;
  DenseWork w = carve_dense(workspace, T, kDNT * JD, chunk);
  double* base = nullptr;
  switch (which) {
    case PMG_STATE_FWD_IN: base = w.s_in; break;
    case PMG_STATE_FWD_OUT: base = w.s_out; break;
    case PMG_STATE_BWD_IN: base = w.b_in; break;
    case PMG_STATE_BWD_FIRST: base = w.b_first; break;
    default: return nullptr;
  }
  return base + (size_t)c * 2 * (kDNT * JD);
}

static int dense_forward_impl(const float* delta, const float* phi, const double* ll64, const double* m, int64_t T,
                              const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                              double tol, float* alpha, double* log_alpha, double* logc, double* logz,
                              void* workspace, size_t workspace_bytes, void* stream, int phase) {
  DenseParams p;
  int rc = dense_params(p, tr, T, chunk, warmup, likelihood_scale, tol);
  if (rc) return rc;
  PMG_REQUIRE(delta && phi && m && log_alpha && logc && logz && workspace, "pmg_dense_forward: null");
  PMG_REQUIRE(workspace_bytes >= pmg_dense_workspace_size(T, tr->L, chunk), "pmg_dense_forward: workspace too small");
  hipStream_t st = as_stream(stream);
  DenseWork w = carve_dense(workspace, T, p.Lp, chunk);
  p.delta = delta;
  p.phi = phi;
  p.ll64 = ll64;
  p.m = m;
  p.alpha = alpha;
  p.log_alpha = log_alpha;
  p.logc = logc;
  p.logz = logz;
  p.chunk_logz = w.chunk_logz;
  p.s_in = w.s_in;
  p.s_out = w.s_out;
  p.flags = w.flags;
  p.ctl = w.ctl;
  p.seg_end = w.seg_end;
  p.seg_chg = w.seg_chg;
  dense_kernel_t kf, kfr, kb, kbr;
  dense_kernels(p.Lp / kDNT, &kf, &kfr, &kb, &kbr);
  // per-pass words: repair / round counters at the main pass (a later phase-2 call, the
  // time-shard carry hand-off, adds its repairs to them), the relaxation protocol words
  // before each relaxation; the timeout word (kDErr) is sticky until the host reads it
  if (phase & 1) {
    PMG_HIP(hipMemsetAsync(p.ctl, 0, kDErr * sizeof(int), st));
    hipLaunchKernelGGL(kf, dim3(p.M), dim3(kDNT), 0, st, p);
    PMG_LAUNCH_CHECK();
  }
  if (phase & 2) {
    PMG_HIP(hipMemsetAsync(p.ctl + kDErr + 1, 0, (16 - kDErr - 1) * sizeof(int), st));
    if (p.M > 1) {
      hipLaunchKernelGGL(k_dense_verify, dim3((p.M - 1 + 3) / 4), dim3(256), 0, st, w.s_in, (const double*)w.s_out,
                         1, p.M - 1, -1, p.L, p.Lp, p.tol, w.flags, (const float*)nullptr, 0, p.ctl + kDPending);
      PMG_LAUNCH_CHECK();
    }
    PMG_HIP(launch_persistent(kfr, dim3(p.S), dim3(kDNT), 0, st, p));
  }
  return PMG_OK;
}

int pmg_dense_forward(const float* delta, const float* phi, const double* ll64, const double* m, int64_t T,
                      const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                      double tol, float* alpha, double* log_alpha, double* logc, double* logz, void* workspace,
                      size_t workspace_bytes, void* stream) {
  return dense_forward_impl(delta, phi, ll64, m, T, tr, likelihood_scale, chunk, warmup, tol, alpha, log_alpha, logc,
                            logz, workspace, workspace_bytes, stream, 3);
}

int pmg_dense_forward_phase(const float* delta, const float* phi, const double* ll64, const double* m, int64_t T,
                            const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                            double tol, float* alpha, double* log_alpha, double* logc, double* logz, void* workspace,
                            size_t workspace_bytes, void* stream, int32_t phase) {
  PMG_REQUIRE(phase >= 1 && phase <= 3, "pmg_dense_forward_phase: phase %d", phase);
  return dense_forward_impl(delta, phi, ll64, m, T, tr, likelihood_scale, chunk, warmup, tol, alpha, log_alpha, logc,
                            logz, workspace, workspace_bytes, stream, phase);
}

static int dense_backward_impl(const float* delta, const float* phi, const double* ll64, const double* log_alpha,
                               int64_t T, const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk,
                               int32_t warmup, double tol, float* P, float* gamma, float* log_gamma, float* rho,
                               double* log_rho, void* workspace, size_t workspace_bytes, void* stream, int phase) {
  DenseParams p;
  int rc = dense_params(p, tr, T, chunk, warmup, likelihood_scale, tol);
  if (rc) return rc;
  PMG_REQUIRE(delta && phi && log_alpha && workspace, "pmg_dense_backward: null");
  PMG_REQUIRE(workspace_bytes >= pmg_dense_workspace_size(T, tr->L, chunk), "pmg_dense_backward: workspace too small");
  hipStream_t st = as_stream(stream);
  DenseWork w = carve_dense(workspace, T, p.Lp, chunk);
  p.delta = delta;
  p.phi = phi;
  p.ll64 = ll64;
  p.log_alpha_in = log_alpha;
  p.P = P;
  p.gamma = gamma;
  p.log_gamma = log_gamma;
  p.rho = rho;
  p.log_rho = log_rho;
  p.b_in = w.b_in;
  p.b_first = w.b_first;
  p.flags = w.flags;
  p.ctl = w.ctl + kDCtlStride;
  p.seg_end = w.seg_end;
  p.seg_chg = w.seg_chg;
  dense_kernel_t kf, kfr, kb, kbr;
  dense_kernels(p.Lp / kDNT, &kf, &kfr, &kb, &kbr);
  // per-pass words as dense_forward_impl
  if (phase & 1) {
    PMG_HIP(hipMemsetAsync(p.ctl, 0, kDErr * sizeof(int), st));
    hipLaunchKernelGGL(kb, dim3(p.M), dim3(kDNT), 0, st, p);
    PMG_LAUNCH_CHECK();
  }
  if ((phase & 2) && p.M > 1) {
    PMG_HIP(hipMemsetAsync(p.ctl + kDErr + 1, 0, (16 - kDErr - 1) * sizeof(int), st));
    hipLaunchKernelGGL(k_dense_verify, dim3((p.M - 1 + 3) / 4), dim3(256), 0, st, w.b_in, (const double*)w.b_first, 0,
                       p.M - 2, 1, p.L, p.Lp, p.tol, w.flags, (const float*)nullptr, p.C, p.ctl + kDPending);
    PMG_LAUNCH_CHECK();
    PMG_HIP(launch_persistent(kbr, dim3(p.S), dim3(kDNT), 0, st, p));
  }
  return PMG_OK;
}

int pmg_dense_backward(const float* delta, const float* phi, const double* ll64, const double* log_alpha, int64_t T,
                       const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                       double tol, float* P, float* gamma, float* log_gamma, float* rho, double* log_rho,
                       void* workspace, size_t workspace_bytes, void* stream) {
  return dense_backward_impl(delta, phi, ll64, log_alpha, T, tr, likelihood_scale, chunk, warmup, tol, P, gamma,
                             log_gamma, rho, log_rho, workspace, workspace_bytes, stream, 3);
}

int pmg_dense_backward_phase(const float* delta, const float* phi, const double* ll64, const double* log_alpha,
                             int64_t T, const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk,
                             int32_t warmup, double tol, float* P, float* gamma, float* log_gamma, float* rho,
                             double* log_rho, void* workspace, size_t workspace_bytes, void* stream, int32_t phase) {
  PMG_REQUIRE(phase >= 1 && phase <= 3, "pmg_dense_backward_phase: phase %d", phase);
  return dense_backward_impl(delta, phi, ll64, log_alpha, T, tr, likelihood_scale, chunk, warmup, tol, P, gamma,
                             log_gamma, rho, log_rho, workspace, workspace_bytes, stream, phase);
}

// time splits of the joint: enough workgroups to fill the chip (one 64 x 64 tile each),
// each split at least a few blocks long; 1 (no workspace partials) when the tiles alone fill it
static int joint_log_splits(int64_t T, int32_t L) {
  const int L2 = 2 * L;
  const int64_t tiles = (int64_t)((L2 + kJT - 1) / kJT) * ((L2 + kJT - 1) / kJT);
  int nsplit = 1;
  while (nsplit < kJointSplits && tiles * nsplit < 1024 && (T - 1) / (2 * nsplit) >= 4 * kJB) nsplit *= 2;
  return nsplit;
}

// the partials of the splits (two f64 per entry and split), or 0 when the joint runs unsplit
size_t pmg_joint_log_workspace_size(int64_t T, int32_t L) {
  if (T <= 0 || L <= 0) return 0;
  const int nsplit = joint_log_splits(T, L);
  if (nsplit == 1) return 0;
  const int64_t n = (int64_t)(2 * L) * (2 * L);
  return (size_t)nsplit * (size_t)n * 2 * sizeof(double) + 256;
}

int pmg_joint_log_accumulate_ws(const double* log_alpha, const double* log_rho, int64_t T, int32_t L, double* logS,
                                void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(log_alpha && log_rho && logS && T > 0 && L > 0, "pmg_joint_log_accumulate: bad argument");
  const int L2 = 2 * L;
  const int64_t n = (int64_t)L2 * L2;
  // split in time only with a workspace of the size pmg_joint_log_workspace_size asks for
  int nsplit = 1;
  if (workspace) {
    PMG_REQUIRE(workspace_bytes >= pmg_joint_log_workspace_size(T, L), "pmg_joint_log_accumulate: workspace too small");
    nsplit = joint_log_splits(T, L);
  }
  const int64_t per = ((T - 1 + nsplit - 1) / nsplit + kJB - 1) / kJB * kJB;
  dim3 grid((L2 + kJT - 1) / kJT, (L2 + kJT - 1) / kJT, nsplit);
  double* part = nsplit > 1 ? static_cast<double*>(workspace) : nullptr;
  hipLaunchKernelGGL(k_joint_log, grid, dim3(256), 0, as_stream(stream), log_alpha, log_rho, T, L2, per > 0 ? per : kJB,
                     part, logS);
  PMG_LAUNCH_CHECK();
  if (part) {
    hipLaunchKernelGGL(k_joint_log_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), part,
                       nsplit, n, logS);
    PMG_LAUNCH_CHECK();
  }
  return PMG_OK;
}

int pmg_joint_log_accumulate(const double* log_alpha, const double* log_rho, int64_t T, int32_t L, double* logS,
                             void* stream) {
  return pmg_joint_log_accumulate_ws(log_alpha, log_rho, T, L, logS, nullptr, 0, stream);
}

}  // extern "C"
