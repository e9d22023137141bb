// Time-parallel forward filter / backward smoother over the joint
// (dynamics x latent) state of the jump GPLVM, gfx950.
//
// Reference (log-domain, strictly sequential lax.scan):
//   filter_one_step   decoder.py:151-172   prior = LSE_i(LSE_d(post+logA)+logK); post = prior+s*ll - c
//   smooth_one_step   decoder.py:200-226   acausal_t = LSE_{d',j}(logK+logA+(acausal_{t+1}-prior_{t+1})+post_t)
//   chunk driver      decoder.py:258-332   carries (post[-1], logZ) forward, (acausal[0], joint) backward
//
// MI355X design:
//   * linear space with per-step normalisation (exact up to fp32 rounding; states
//     below ~1e-38 of the total flush to 0 -- probability-space outputs unchanged);
//   * the continuous kernel is a row-normalised Toeplitz band K0[i,j] = g[|i-j|]/Z_i
//     (exactly zero beyond |i-j| = band in the reference's f32), applied
//     as a 1-D convolution through a per-wave LDS line; the jump kernel is rank-1
//     (a wave reduction); the 2x2 dynamics mix is elementwise;
//   * one wave per time chunk; each chunk starts from a uniform guess `warmup`
//     steps early (HMM forgetting), then every chunk boundary is verified in the
//     Hilbert projective metric (max-min of log ratios, a contraction of positive
//     linear maps, so a boundary error <= tol bounds every later output's relative
//     error by tol) and chunks that fail are recomputed exactly from their
//     predecessor's state by a single-wave repair pass (rare; sequential only over
//     consecutive failures);
//   * the smoother uses the equivalent alpha-beta form gamma_t ~ alpha_t * beta_t
//     with beta_{T-1} = 1 (the reference's RTS seed acausal_{T-1} = post_{T-1}), so
//     the backward pass needs only alpha_t and the emission -- no stored priors.
//
// Emission input: e[t,l] = exp(s*delta[t,l] + phi[t,l/32]) = exp(s*(ll[t,l] - m[t])).
#pragma once
#include <stdlib.h>

#include "pmg_common.h"

// Contract a*b+c only inside one expression (the explicit fmaf calls).  Chunk
// boundaries coalesce bitwise only if every unrolled copy of a step (the PF-deep row
// rings) rounds identically; hipcc's default cross-statement contraction lets the
// scheduler fuse differently per copy.
#pragma clang fp contract(on)

namespace pmg {

constexpr int kMaxBand = 32;
constexpr int kFixRounds = 2;  // parallel repair rounds before the sequential fallback
// Emission / alpha rows are prefetched this many steps ahead on the chunk-parallel
// kernels: with ~2 waves per SIMD the step's VALU work (~0.3 us) cannot cover an HBM
// round trip (~2 us), so the row ring, not other waves, hides the latency.
constexpr int kPfFwd = 4;
constexpr int kPfBwdWarm = 4;
constexpr int kPfBwdOut = 2;

struct FBParams {
  const float* delta;
  const float* phi;
  const double* m;
  int64_t T;
  int L;
  int nblk;
  const float* invz;
  float g[kMaxBand + 1];
  float A00, A01, A10, A11;
  float invL;
  float s;
  double s_d;
  int C, B, M;
  float tol;
  // forward
  float* alpha;
  double* logc;
  double* chunk_logz;
  float* s_in;
  float* s_out;
  // backward
  const float* alpha_in;
  float* P;
  float* gamma;
  float* rho;
  float* b_in;
  float* b_first;
  int* flags;
  int* repairs;
  int Lpad;  // 64*J
};

// ---------------------------------------------------------------------------
// per-lane helpers (lane owns latents j0 .. j0+J-1, j0 = lane*J)
// ---------------------------------------------------------------------------
template <int J>
__device__ __forceinline__ void load_row(const float* __restrict__ row, int L, int j0, float v[J]) {
  if ((L & 3) == 0 && (J & 3) == 0 && j0 + J <= L) {
#pragma unroll
    for (int j = 0; j < J; j += 4) {
      float4 q = *reinterpret_cast<const float4*>(row + j0 + j);
      v[j] = q.x; v[j + 1] = q.y; v[j + 2] = q.z; v[j + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = (j0 + j < L) ? row[j0 + j] : 0.f;
  }
}

template <int J>
__device__ __forceinline__ void store_row(float* __restrict__ row, int L, int j0, const float v[J]) {
  if ((L & 3) == 0 && (J & 3) == 0 && j0 + J <= L) {
#pragma unroll
    for (int j = 0; j < J; j += 4)
      *reinterpret_cast<float4*>(row + j0 + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (j0 + j < L) row[j0 + j] = v[j];
  }
}

// raw emission operands for one time step
template <int J>
struct EmRaw {
  float d[J];
  float ph;
};

template <int J>
__device__ __forceinline__ void em_load(const FBParams& p, int64_t t, int j0, EmRaw<J>& r) {
  load_row<J>(p.delta + t * p.L, p.L, j0, r.d);
  const int b = j0 >> 5;
  r.ph = (b < p.nblk) ? p.phi[t * p.nblk + b] : 0.f;
}

template <int J>
__device__ __forceinline__ void em_exp(const FBParams& p, int j0, const EmRaw<J>& r, float e[J]) {
#pragma unroll
  for (int j = 0; j < J; ++j) e[j] = (j0 + j < p.L) ? exp_acc(fmaf(p.s, r.d[j], r.ph)) : 0.f;
}

// out[j] = sum_{k=-WP..WP} g[|k|] * in[j+k]  over the whole latent line (zero halo)
// Multi-wave teams: through an LDS line (one barrier each side).
template <int J, int WP>
__device__ __forceinline__ void band_conv_lds(const FBParams& p, float* lds, int j0, const float in[J],
                                              float out[J]) {
#pragma unroll
  for (int j = 0; j < J; ++j) lds[WP + j0 + j] = in[j];
  __syncthreads();
  float win[J + 2 * WP];
#pragma unroll
  for (int k = 0; k < J + 2 * WP; ++k) win[k] = lds[j0 + k];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    float acc = p.g[0] * win[j + WP];
#pragma unroll
    for (int k = 1; k <= WP; ++k) acc = fmaf(p.g[k], win[j + WP - k] + win[j + WP + k], acc);
    out[j] = acc;
  }
  __syncthreads();
}

// One wave holds the whole line (lane l owns latents lJ .. lJ+J-1): the halo comes
// from the neighbouring lanes through wavefront-shift DPP moves (wave_shr:1 /
// wave_shl:1; the lanes past either end read 0), so the step touches no LDS.  The
// contiguous-block LDS exchange it replaces ran into 8-way bank conflicts (lane
// stride J words).  Only the entries inside the band are moved: J + 1 per side at
// J = 8, WP = 9.
__device__ __forceinline__ float wave_shr1(float v) {  // lane i <- lane i-1 (lane 0 <- 0)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_shl1(float v) {  // lane i <- lane i+1 (lane 63 <- 0)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
}

template <int J, int WP>
__device__ __forceinline__ void band_conv_dpp(const FBParams& p, const float in[J], float out[J]) {
  constexpr int NL = (WP + J - 1) / J;  // neighbour lanes on each side
  constexpr int C = NL * J;             // window index of this lane's first latent
  float win[J + 2 * C];
#pragma unroll
  for (int i = 0; i < J; ++i) win[C + i] = in[i];
  // left: block k (lane l-k) local i sits at window C - kJ + i; needed iff kJ - i <= WP
#pragma unroll
  for (int k = 1; k <= NL; ++k)
#pragma unroll
    for (int i = 0; i < J; ++i) {
      if (k * J - i <= WP) win[C - k * J + i] = wave_shr1(win[C - (k - 1) * J + i]);
      else win[C - k * J + i] = 0.f;
    }
  // right: block k (lane l+k) local i at window C + kJ + i; needed iff kJ + i - (J-1) <= WP
#pragma unroll
  for (int k = 1; k <= NL; ++k)
#pragma unroll
    for (int i = 0; i < J; ++i) {
      if (k * J + i - (J - 1) <= WP) win[C + k * J + i] = wave_shl1(win[C + (k - 1) * J + i]);
      else win[C + k * J + i] = 0.f;
    }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    float acc = p.g[0] * win[C + j];
#pragma unroll
    for (int k = 1; k <= WP; ++k) acc = fmaf(p.g[k], win[C + j - k] + win[C + j + k], acc);
    out[j] = acc;
  }
}

template <int J, int WP, class Team>
__device__ __forceinline__ void band_conv(const FBParams& p, float* lds, int j0, const float in[J],
                                          float out[J]) {
  if constexpr (Team::NW == 1) {
    (void)lds;
    (void)j0;
    band_conv_dpp<J, WP>(p, in, out);
  } else {
    band_conv_lds<J, WP>(p, lds, j0, in, out);
  }
}

// ---------------------------------------------------------------------------
// Teams: the threads that carry ONE chain.  The chunk-parallel kernels use one wave
// per chunk (DPP reductions, no block barriers); the sequential repair of a long
// cascade uses NW waves on the same chain (wave DPP + LDS partials behind a block
// barrier; the scratch is double-buffered so one barrier per reduction suffices).
// Thread t owns latents j0 = t*J .. t*J+J-1 in both cases.
// ---------------------------------------------------------------------------
struct WaveTeam {
  static constexpr int NW = 1;
  __device__ explicit WaveTeam(float*) {}
  __device__ void sum2(float& a, float& b) { wave_sum2(a, b); }
  __device__ float sum(float a) { return wave_sum(a); }
  __device__ float vmax(float a) { return wave_max_shfl(a); }
  __device__ float vmin(float a) { return wave_min_shfl(a); }
  __device__ bool any(bool b) { return __ballot(b) != 0ull; }
};

template <int NW_>
struct BlockTeam {
  static constexpr int NW = NW_;
  float* red;  // LDS scratch, 2 x 2 x NW floats
  int buf = 0;
  __device__ explicit BlockTeam(float* r) : red(r) {}
  __device__ float* slot() {
    float* r = red + buf * 2 * NW;
    buf ^= 1;
    return r;
  }
  __device__ void sum2(float& a, float& b) {
    wave_sum2(a, b);
    float* r = slot();
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      r[w] = a;
      r[NW + w] = b;
    }
    __syncthreads();
    float A = 0.f, B = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      A += r[i];
      B += r[NW + i];
    }
    a = A;
    b = B;
  }
  __device__ float sum(float a) {
    float b = 0.f;
    sum2(a, b);
    return a;
  }
  __device__ float vmax(float a) {
    a = wave_max_shfl(a);
    float* r = slot();
    if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = a;
    __syncthreads();
    float m = r[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) m = fmaxf(m, r[i]);
    return m;
  }
  __device__ float vmin(float a) { return -vmax(-a); }
  __device__ bool any(bool b) { return vmax(__ballot(b) ? 1.f : 0.f) > 0.f; }
};

// Hilbert projective distance between two non-negative (2, Lpad) states held in
// memory; components below 1e-30 of the max on both sides are ignored, a
// component significant (> 1e-20) on one side only counts as a failure.
__device__ __forceinline__ float hilbert_dist(const float* __restrict__ x, const float* __restrict__ y, int n,
                              const float* __restrict__ w = nullptr, int L = 0, int Lpad = 0) {
  const int lane = threadIdx.x & 63;
  // every operand is fetched up front (n = 2*Lpad <= 2048: at most 32 per lane) so the
  // wave pays one memory round trip, not one per strided pass
  constexpr int kMaxPer = 2 * 1024 / 64;
  float xv[kMaxPer], yv[kMaxPer];
#pragma unroll
  for (int q = 0; q < kMaxPer; ++q) {
    const int i = lane + 64 * q;
    float wi = 0.f;
    if (i < n) {
      wi = 1.f;
      if (w) {  // optional weights w in the (2, L) alpha-row layout for state index i = d*Lpad + j
        const int d = i >= Lpad ? 1 : 0, j = i - d * Lpad;
        wi = j < L ? w[d * L + j] : 0.f;
      }
    }
    xv[q] = i < n ? x[i] * wi : 0.f;
    yv[q] = i < n ? y[i] * wi : 0.f;
  }
  float xm = 0.f, ym = 0.f;
#pragma unroll
  for (int q = 0; q < kMaxPer; ++q) {
    xm = fmaxf(xm, xv[q]);
    ym = fmaxf(ym, yv[q]);
  }
  xm = wave_max_shfl(xm);
  ym = wave_max_shfl(ym);
  if (!(xm > 0.f) || !(ym > 0.f)) return INFINITY;
  const float ix = 1.f / xm, iy = 1.f / ym;
  // unweighted (state space): ratios of components above 1e-30 of the max, a component
  // above 1e-20 on one side only fails.  Weighted (posterior space, |posterior| <= 1):
  // components below 1e-14 move no output by more than 1e-14 absolute (parity atol is
  // 1e-12); above it the ratio spread bounds the relative error.
  const float lo_thr = w ? 1e-14f : 1e-30f, hi_thr = w ? 1e-12f : 1e-20f;
  float lo = INFINITY, hi = -INFINITY;
  int bad = 0;
#pragma unroll
  for (int q = 0; q < kMaxPer; ++q) {
    const float a = xv[q] * ix, b = yv[q] * iy;
    if (a > lo_thr && b > lo_thr) {
      const float r = __logf(a) - __logf(b);
      lo = fminf(lo, r);
      hi = fmaxf(hi, r);
    } else if (fmaxf(a, b) > hi_thr) {
      bad = 1;
    }
  }
  lo = wave_min_shfl(lo);
  hi = wave_max_shfl(hi);
  if (__ballot(bad)) return INFINITY;
  if (hi < lo) return 0.f;
  return hi - lo;
}

// same metric, x held in registers with the (2, Lpad) lane layout, y in memory
template <int J, class Team>
__device__ float hilbert_reg(Team& tm, const float x0[J], const float x1[J], const float* __restrict__ y,
                             int Lpad, int j0) {
  float xm = 0.f, ym = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    xm = fmaxf(xm, fmaxf(x0[j], x1[j]));
    ym = fmaxf(ym, fmaxf(y[j0 + j], y[Lpad + j0 + j]));
  }
  xm = tm.vmax(xm);
  ym = tm.vmax(ym);
  if (!(xm > 0.f) || !(ym > 0.f)) return INFINITY;
  const float ix = 1.f / xm, iy = 1.f / ym;
  float lo = INFINITY, hi = -INFINITY;
  int bad = 0;
#pragma unroll
  for (int j = 0; j < 2 * J; ++j) {
    const float a = (j < J ? x0[j] : x1[j - J]) * ix;
    const float b = (j < J ? y[j0 + j] : y[Lpad + j0 + j - J]) * iy;
    if (a > 1e-30f && b > 1e-30f) {
      const float r = __logf(a) - __logf(b);
      lo = fminf(lo, r);
      hi = fmaxf(hi, r);
    } else if (fmaxf(a, b) > 1e-20f) {
      bad = 1;
    }
  }
  lo = tm.vmin(lo);
  hi = tm.vmax(hi);
  if (tm.any(bad != 0)) return INFINITY;
  if (hi < lo) return 0.f;
  return hi - lo;
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int J, int WP, class Team = WaveTeam>
struct Fwd {
  float p0[J], p1[J];
  float P0, P1;  // sum of p0, p1 (wave-uniform)

  __device__ void init_uniform(const FBParams& p, int j0) {
    const float u = 0.5f * p.invL;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      p0[j] = (j0 + j < p.L) ? u : 0.f;
      p1[j] = p0[j];
    }
    P0 = 0.5f;
    P1 = 0.5f;
  }
  __device__ void load_state(Team& tm, const FBParams& p, const float* src, int j0) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      p0[j] = src[j0 + j];
      p1[j] = src[p.Lpad + j0 + j];
    }
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      a += p0[j];
      b += p1[j];
    }
    tm.sum2(a, b);
    const float inv = 1.f / (a + b);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      p0[j] *= inv;
      p1[j] *= inv;
    }
    P0 = a * inv;
    P1 = b * inv;
  }
  __device__ void save_state(const FBParams& p, float* dst, int j0) const {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      dst[j0 + j] = p0[j];
      dst[p.Lpad + j0 + j] = p1[j];
    }
  }
  // one filter step with emission e; returns the normaliser S
  __device__ float step(Team& tm, const FBParams& p, float* lds, int j0, const float invz[J],
                        const float e[J]) {
    float a0[J];
#pragma unroll
    for (int j = 0; j < J; ++j) a0[j] = fmaf(p0[j], p.A00, p1[j] * p.A10) * invz[j];
    const float jump = fmaf(p.A01, P0, p.A11 * P1) * p.invL;
    float pr0[J];
    band_conv<J, WP, Team>(p, lds, j0, a0, pr0);
    float U0 = 0.f, U1 = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      p0[j] = pr0[j] * e[j];
      p1[j] = jump * e[j];
      U0 += p0[j];
      U1 += p1[j];
    }
    tm.sum2(U0, U1);
    const float S = U0 + U1;
    const float inv = 1.f / S;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      p0[j] *= inv;
      p1[j] *= inv;
    }
    P0 = U0 * inv;
    P1 = U1 * inv;
    return S;
  }
};

// run forward from t0 (state initialised) to t_e; writes outputs for t >= t_c and the
// state at t_c-1 into s_in_dst (if given)
template <int J, int WP, class Team, int PF = 1>
__device__ double fwd_run(Team& tm, const FBParams& p, Fwd<J, WP, Team>& st, float* lds, int j0,
                          const float invz[J], int64_t t0, int64_t t_c, int64_t t_e, float* s_in_dst) {
  double logz = 0.0;
  if (t0 >= t_e) return 0.0;
  // emission rows PF steps ahead (the sequential repair chain is latency-bound; the
  // chunk-parallel kernels hide latency across waves and use PF = 1)
  // the row reference m[t] of logc rides in the same ring: a load consumed in its own
  // step would make the compiler drain every outstanding load (s_waitcnt vmcnt(0))
  EmRaw<J> ring[PF];
  double mr[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (t0 + q < t_e) {
      em_load<J>(p, t0 + q, j0, ring[q]);
      mr[q] = p.m[t0 + q];
    }
  for (int64_t tb = t0; tb < t_e; tb += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t t = tb + q;
      if (t < t_e) {
        float e[J];
        em_exp<J>(p, j0, ring[q], e);
        const double mt = mr[q];
        if (t + PF < t_e) {
          em_load<J>(p, t + PF, j0, ring[q]);
          mr[q] = p.m[t + PF];
        }
        const float S = st.step(tm, p, lds, j0, invz, e);
        if (t >= t_c) {
          float* arow = p.alpha + t * 2 * (int64_t)p.L;
          store_row<J>(arow, p.L, j0, st.p0);
          store_row<J>(arow + p.L, p.L, j0, st.p1);
          const double lc = (double)__logf(S) + p.s_d * mt;
          if (threadIdx.x == 0) p.logc[t] = lc;
          logz += lc;
        } else if (t == t_c - 1 && s_in_dst) {
          st.save_state(p, s_in_dst, j0);
        }
      }
    }
  }
  return logz;
}

#define PMG_FB_PROLOGUE_T(JJ, NWW)                                      \
  __shared__ __attribute__((aligned(16))) float lds[64 * (NWW) * (JJ) + 2 * WP + 4 * (NWW)]; \
  float* team_red = lds + 64 * (NWW) * (JJ) + 2 * WP;                   \
  const int lane = threadIdx.x & 63;                                    \
  (void)lane;                                                           \
  const int j0 = threadIdx.x * (JJ);                                    \
  for (int k = threadIdx.x; k < 64 * (NWW) * (JJ) + 2 * WP; k += 64 * (NWW)) lds[k] = 0.f; \
  __syncthreads();                                                      \
  float invz[JJ];                                                       \
  _Pragma("unroll") for (int j = 0; j < (JJ); ++j) invz[j] = (j0 + j < p.L) ? p.invz[j0 + j] : 0.f; \
  const size_t SZ = (size_t)2 * p.Lpad;                                 \
  (void)SZ;                                                             \
  (void)team_red;

#define PMG_FB_PROLOGUE                                                 \
  __shared__ __attribute__((aligned(16))) float lds[64 * J + 2 * WP];  \
  const int lane = threadIdx.x & 63;                                    \
  const int j0 = lane * J;                                              \
  WaveTeam tm(nullptr);                                                 \
  for (int k = lane; k < 64 * J + 2 * WP; k += 64) lds[k] = 0.f;        \
  __syncthreads();                                                      \
  float invz[J];                                                        \
  _Pragma("unroll") for (int j = 0; j < J; ++j) invz[j] = (j0 + j < p.L) ? p.invz[j0 + j] : 0.f; \
  const size_t SZ = (size_t)2 * p.Lpad;                                 \
  (void)SZ;

// ---------------------------------------------------------------------------
// Chunk-parallel streaming path (one wave per chain).  Every row access is a raw
// buffer load/store through a per-row resource (num_records = row bytes), so lanes
// past L read 0 / drop their writes without exec masking, and the step loop is
// straight-line: the rows of the next PF steps stay in flight across steps (the
// waitcnt pass only sees one in-order vmcnt stream; any divergent load or store in
// the loop would make it drain the ring).  VEC: L % 4 == 0 (16-byte row accesses).
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int J, bool VEC>
__device__ __forceinline__ void bload_row(const float* row, int L, int j0, float v[J]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(row, (uint32_t)L * 4u);
  if constexpr (VEC) {
#pragma unroll
    for (int j = 0; j < J; j += 4) {
      const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, (j0 + j) * 4, 0, 0);
      v[j] = __uint_as_float(q.x);
      v[j + 1] = __uint_as_float(q.y);
      v[j + 2] = __uint_as_float(q.z);
      v[j + 3] = __uint_as_float(q.w);
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (j0 + j) * 4, 0, 0));
  }
}

template <int J, bool VEC>
__device__ __forceinline__ void bstore_row(float* row, int L, int j0, const float v[J]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(row, (uint32_t)L * 4u);
  if constexpr (VEC) {
#pragma unroll
    for (int j = 0; j < J; j += 4) {
      u32x4 q;
      q.x = __float_as_uint(v[j]);
      q.y = __float_as_uint(v[j + 1]);
      q.z = __float_as_uint(v[j + 2]);
      q.w = __float_as_uint(v[j + 3]);
      __builtin_amdgcn_raw_buffer_store_b128(q, rs, (j0 + j) * 4, 0, 0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[j]), rs, (j0 + j) * 4, 0, 0);
  }
}

// one f64 per step written by lane 0 only (the other lanes' offsets are out of range)
__device__ __forceinline__ void bstore_f64_lane0(double* base, int64_t t, double v) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(base + t, 8u);
  const int off = (threadIdx.x & 63) == 0 ? 0 : 64;
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)u, rs, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)(u >> 32), rs, off + 4, 0, 0);
}

template <int J, bool VEC>
__device__ __forceinline__ void bem_load(const FBParams& p, int64_t t, int j0, EmRaw<J>& r) {
  bload_row<J, VEC>(p.delta + t * p.L, p.L, j0, r.d);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(p.phi + t * p.nblk, (uint32_t)p.nblk * 4u);
  r.ph = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (j0 >> 5) * 4, 0, 0));
}

// forward steps t in [t_a, t_b): OUT writes alpha / logc and returns sum logc
template <int J, int WP, int PF, bool VEC, bool OUT>
__device__ __forceinline__ double fwd_stream(const FBParams& p, Fwd<J, WP>& st, int j0, const float invz[J],
                                             int64_t t_a, int64_t t_b) {
  WaveTeam tm(nullptr);
  double logz = 0.0;
  if (t_a >= t_b) return 0.0;
  const int64_t last = t_b - 1;
  EmRaw<J> ring[PF];
  double mr[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int64_t tl = t_a + q < last ? t_a + q : last;
    bem_load<J, VEC>(p, tl, j0, ring[q]);
    if constexpr (OUT) mr[q] = p.m[tl];
  }
  auto body = [&](int q, int64_t t, bool refill) {
    float e[J];
    em_exp<J>(p, j0, ring[q], e);
    double mt = 0.0;
    if constexpr (OUT) mt = mr[q];
    if (refill) {
      const int64_t tl = t + PF < last ? t + PF : last;
      bem_load<J, VEC>(p, tl, j0, ring[q]);
      if constexpr (OUT) mr[q] = p.m[tl];
    }
    const float S = st.step(tm, p, nullptr, j0, invz, e);
    if constexpr (OUT) {
      float* arow = p.alpha + t * 2 * (int64_t)p.L;
      bstore_row<J, VEC>(arow, p.L, j0, st.p0);
      bstore_row<J, VEC>(arow + p.L, p.L, j0, st.p1);
      const double lc = (double)__logf(S) + p.s_d * mt;
      bstore_f64_lane0(p.logc, t, lc);
      logz += lc;
    }
  };
  int64_t tb = t_a;
  for (; tb + PF <= t_b; tb += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) body(q, tb + q, true);
  }
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (tb + q < t_b) body(q, tb + q, false);
  return logz;
}

template <int J, int WP, bool VEC>
__device__ __forceinline__ void forward_chunk(const FBParams& p, int c, int j0, const float invz[J], bool fix) {
  const size_t SZ = (size_t)2 * p.Lpad;
  const int64_t t_c = (int64_t)c * p.C;
  const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
  Fwd<J, WP> st;
  float* sin = p.s_in + (size_t)c * SZ;
  if (fix) {
    WaveTeam tm(nullptr);
    st.load_state(tm, p, sin, j0);
  } else {
    int64_t t0 = (c == 0) ? 0 : t_c - p.B;
    if (t0 < 0) t0 = 0;
    st.init_uniform(p, j0);
    fwd_stream<J, WP, kPfFwd, VEC, false>(p, st, j0, invz, t0, t_c);
    if (c > 0) st.save_state(p, sin, j0);  // the restart state of a later repair (the guess if no warm-up)
  }
  const double lz = fwd_stream<J, WP, kPfFwd, VEC, true>(p, st, j0, invz, t_c, t_e);
  st.save_state(p, p.s_out + (size_t)c * SZ, j0);
  if ((threadIdx.x & 63) == 0) {
    p.chunk_logz[c] = lz;
    if (fix) atomicAdd(&p.repairs[0], 1);
  }
}

#define PMG_FB_LANE_SETUP                                               \
  const int lane = threadIdx.x & 63;                                    \
  const int j0 = lane * J;                                              \
  float invz[J];                                                        \
  _Pragma("unroll") for (int j = 0; j < J; ++j) invz[j] = (j0 + j < p.L) ? p.invz[j0 + j] : 0.f;

// speculative pass: chunk c starts `B` steps early from a uniform guess
template <int J, int WP>
__global__ void __launch_bounds__(64) k_forward(FBParams p) {
  const int c = blockIdx.x;
  if (c >= p.M) return;
  PMG_FB_LANE_SETUP
  if constexpr (J % 4 == 0) {
    if ((p.L & 3) == 0) {
      forward_chunk<J, WP, true>(p, c, j0, invz, false);
      return;
    }
  }
  forward_chunk<J, WP, false>(p, c, j0, invz, false);
}

// parallel repair round: every flagged chunk restarts from its snapshot s_in[c]
template <int J, int WP>
__global__ void __launch_bounds__(64) k_forward_fix(FBParams p) {
  const int c = blockIdx.x;
  if (c >= p.M || c == 0 || p.flags[c] == 0) return;
  PMG_FB_LANE_SETUP
  if constexpr (J % 4 == 0) {
    if ((p.L & 3) == 0) {
      forward_chunk<J, WP, true>(p, c, j0, invz, true);
      return;
    }
  }
  forward_chunk<J, WP, false>(p, c, j0, invz, true);
}

// sequential fallback for whatever is still flagged after the parallel rounds.  A long
// cascade (slowly forgetting chain, e.g. the flat tuning of the first EM iterations)
// is latency-critical, so NW waves carry the one chain (J/NW latents per thread).
template <int J> constexpr int repair_nw() { return J >= 8 ? 8 : J; }

template <int J, int WP>
__global__ void __launch_bounds__(64 * repair_nw<J>()) k_forward_repair(FBParams p) {
  constexpr int NW = repair_nw<J>(), JB = J / NW;
  PMG_FB_PROLOGUE_T(JB, NW)
  BlockTeam<NW> tm(team_red);
  int repairs = 0;
  bool changed = false;
  int c = 1;
  Fwd<JB, WP, BlockTeam<NW>> st;
  while (c < p.M) {
    if (!changed) {  // jump to the next flagged chunk, 64 flags at a time (every wave alike)
      int found = -1;
      for (int base = c; base < p.M && found < 0; base += 64) {
        const int idx = base + lane;
        const bool f = idx < p.M && p.flags[idx] != 0;
        const unsigned long long bal = __ballot(f);
        if (bal) found = base + (int)__builtin_ctzll(bal);
      }
      if (found < 0) break;
      c = found;
      st.load_state(tm, p, p.s_out + (size_t)(c - 1) * SZ, j0);
    }
    const int64_t t_c = (int64_t)c * p.C;
    const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
    st.save_state(p, p.s_in + (size_t)c * SZ, j0);
    const double lz = fwd_run<JB, WP, BlockTeam<NW>, 16 / JB>(tm, p, st, lds, j0, invz, t_c, t_c, t_e, (float*)nullptr);
    float* sout = p.s_out + (size_t)c * SZ;
    const float d = hilbert_reg<JB>(tm, st.p0, st.p1, sout, p.Lpad, j0);
    changed = !(d <= p.tol);
    __syncthreads();  // every wave has read sout before it is overwritten
    st.save_state(p, sout, j0);
    if (threadIdx.x == 0) p.chunk_logz[c] = lz;
    __threadfence();
    __syncthreads();
    ++repairs;
    ++c;
  }
  if (threadIdx.x == 0) p.repairs[0] += repairs;
}

// ---------------------------------------------------------------------------
// backward (beta recursion).  Every step back uses the same arithmetic
//   v = e_t * beta_t / sum(e_t * beta_t),  beta_{t-1} = Trans(v)
// on the warm-up and on the output path, so two chunks that have converged to
// the same beta produce bit-identical continuations (as the forward does).
// ---------------------------------------------------------------------------
template <int J, int WP, class Team = WaveTeam>
struct Bwd {
  float b0[J], b1[J];  // beta at the current time

  __device__ void init_ones(const FBParams& p, int j0) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      b0[j] = (j0 + j < p.L) ? 1.f : 0.f;
      b1[j] = b0[j];
    }
  }
  __device__ void load_state(const FBParams& p, const float* src, int j0) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      b0[j] = src[j0 + j];
      b1[j] = src[p.Lpad + j0 + j];
    }
  }
  __device__ void save_state(const FBParams& p, float* dst, int j0) const {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      dst[j0 + j] = b0[j];
      dst[p.Lpad + j0 + j] = b1[j];
    }
  }
  // v = e*beta scaled by 1/(V0+V1) (returned in v0/v1); beta <- Trans(v)
  __device__ void step_back(const FBParams& p, float* lds, int j0, const float invz[J],
                            const float e[J], float V0, float V1, float v0[J], float v1[J]) {
    const float sc = 1.f / (V0 + V1);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      v0[j] = e[j] * b0[j] * sc;
      v1[j] = e[j] * b1[j] * sc;
    }
    float w0[J];
    band_conv<J, WP, Team>(p, lds, j0, v0, w0);
    const float w1 = V1 * sc * p.invL;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const float c0 = w0[j] * invz[j];
      const float real = (j0 + j < p.L) ? 1.f : 0.f;
      b0[j] = fmaf(p.A00, c0, p.A01 * w1) * real;
      b1[j] = fmaf(p.A10, c0, p.A11 * w1) * real;
    }
  }
};

// one plain backward step at time t (beta_t -> beta_{t-1}); v kept in (v0, v1)
template <int J, int WP, class Team>
__device__ __forceinline__ void bwd_plain(Team& tm, const FBParams& p, Bwd<J, WP, Team>& st, float* lds,
                                          int j0, const float invz[J], int64_t t, float v0[J], float v1[J]) {
  EmRaw<J> r;
  em_load<J>(p, t, j0, r);
  float e[J];
  em_exp<J>(p, j0, r, e);
  float V0 = 0.f, V1 = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    V0 += e[j] * st.b0[j];
    V1 += e[j] * st.b1[j];
  }
  tm.sum2(V0, V1);
  st.step_back(p, lds, j0, invz, e, V0, V1, v0, v1);
}

// plain backward steps t = t_hi .. t_lo (descending) with the emission rows PF steps
// ahead in a register ring (the warm-up of the chunk-parallel pass)
template <int J, int WP, class Team, int PF>
__device__ __forceinline__ void bwd_warm(Team& tm, const FBParams& p, Bwd<J, WP, Team>& st, float* lds,
                                         int j0, const float invz[J], int64_t t_hi, int64_t t_lo) {
  if (t_hi < t_lo) return;
  EmRaw<J> ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (t_hi - q >= t_lo) em_load<J>(p, t_hi - q, j0, ring[q]);
  for (int64_t tb = t_hi; tb >= t_lo; tb -= PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t t = tb - q;
      if (t >= t_lo) {
        float e[J];
        em_exp<J>(p, j0, ring[q], e);
        if (t - PF >= t_lo) em_load<J>(p, t - PF, j0, ring[q]);
        float V0 = 0.f, V1 = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
          V0 += e[j] * st.b0[j];
          V1 += e[j] * st.b1[j];
        }
        tm.sum2(V0, V1);
        float v0[J], v1[J];
        st.step_back(p, lds, j0, invz, e, V0, V1, v0, v1);
      }
    }
  }
}

// output steps t = t_e-1 .. t_c.  On entry st holds beta_{t_e-1} and (vp0, vp1) the v that
// produced it (has_prev false at the sequence end).  On exit st holds beta_{t_c}.
// RHO: also write the joint partner rho (decode); the EM path drops vp0/vp1.
template <int J>
struct BwdRow {
  EmRaw<J> em;
  float a0[J], a1[J];
};

template <int J>
__device__ __forceinline__ void bwd_row_load(const FBParams& p, int64_t t, int j0, BwdRow<J>& r) {
  em_load<J>(p, t, j0, r.em);
  const float* arow = p.alpha_in + t * 2 * (int64_t)p.L;
  load_row<J>(arow, p.L, j0, r.a0);
  load_row<J>(arow + p.L, p.L, j0, r.a1);
}

template <int J, int WP, class Team, int PF, bool RHO>
__device__ void bwd_out(Team& tm, const FBParams& p, Bwd<J, WP, Team>& st, float* lds, int j0,
                        const float invz[J], int64_t t_c, int64_t t_e, float vp0[J], float vp1[J],
                        bool has_prev) {
  const int64_t L = p.L;
  BwdRow<J> ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (t_e - 1 - q >= t_c) bwd_row_load<J>(p, t_e - 1 - q, j0, ring[q]);
  for (int64_t tb = t_e - 1; tb >= t_c; tb -= PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t t = tb - q;
      if (t >= t_c) {
        float a0[J], a1[J], e[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
          a0[j] = ring[q].a0[j];
          a1[j] = ring[q].a1[j];
        }
        em_exp<J>(p, j0, ring[q].em, e);
        if (t - PF >= t_c) bwd_row_load<J>(p, t - PF, j0, ring[q]);
        float G = 0.f, V0 = 0.f, V1 = 0.f;
#pragma unroll
        for (int j = 0; j < J; ++j) {
          a0[j] *= st.b0[j];
          a1[j] *= st.b1[j];
          G += a0[j] + a1[j];
          V0 += e[j] * st.b0[j];
          V1 += e[j] * st.b1[j];
        }
        tm.sum2(V0, V1);
        G = tm.sum(G);
        const float iG = 1.f / G;
        float pp[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
          a0[j] *= iG;
          a1[j] *= iG;
          pp[j] = a0[j] + a1[j];
        }
        if (p.P) store_row<J>(p.P + t * L, p.L, j0, pp);
        if (p.gamma) {
          store_row<J>(p.gamma + t * 2 * L, p.L, j0, a0);
          store_row<J>(p.gamma + t * 2 * L + L, p.L, j0, a1);
        }
        if constexpr (RHO) {
          if (p.rho && has_prev && t + 1 < p.T) {  // rho_{t+1} = v_{t+1} / sum(alpha_t * beta_t)
            float r0[J], r1[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
              r0[j] = vp0[j] * iG;
              r1[j] = vp1[j] * iG;
            }
            store_row<J>(p.rho + (t + 1) * 2 * L, p.L, j0, r0);
            store_row<J>(p.rho + (t + 1) * 2 * L + L, p.L, j0, r1);
          }
        }
        if (t != t_c) {
          st.step_back(p, lds, j0, invz, e, V0, V1, vp0, vp1);
          has_prev = true;
        }
      }
    }
  }
}

// ---- chunk-parallel streaming backward (buffer IO, straight-line step loops) ----
// plain steps t = t_hi .. t_lo (descending), emission rows PF steps ahead
template <int J, int WP, int PF, bool VEC>
__device__ __forceinline__ void bwd_stream_warm(const FBParams& p, Bwd<J, WP>& st, int j0, const float invz[J],
                                                int64_t t_hi, int64_t t_lo) {
  WaveTeam tm(nullptr);
  if (t_hi < t_lo) return;
  EmRaw<J> ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) bem_load<J, VEC>(p, t_hi - q > t_lo ? t_hi - q : t_lo, j0, ring[q]);
  auto body = [&](int q, int64_t t, bool refill) {
    float e[J];
    em_exp<J>(p, j0, ring[q], e);
    if (refill) bem_load<J, VEC>(p, t - PF > t_lo ? t - PF : t_lo, j0, ring[q]);
    float V0 = 0.f, V1 = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      V0 += e[j] * st.b0[j];
      V1 += e[j] * st.b1[j];
    }
    tm.sum2(V0, V1);
    float v0[J], v1[J];
    st.step_back(p, nullptr, j0, invz, e, V0, V1, v0, v1);
  };
  int64_t tb = t_hi;
  for (; tb - (PF - 1) >= t_lo; tb -= PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) body(q, tb - q, true);
  }
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (tb - q >= t_lo) body(q, tb - q, false);
}

template <int J>
struct BRow {
  EmRaw<J> em;
  float a0[J], a1[J];
};

template <int J, bool VEC>
__device__ __forceinline__ void brow_load(const FBParams& p, int64_t t, int j0, BRow<J>& r) {
  bem_load<J, VEC>(p, t, j0, r.em);
  const float* arow = p.alpha_in + t * 2 * (int64_t)p.L;
  bload_row<J, VEC>(arow, p.L, j0, r.a0);
  bload_row<J, VEC>(arow + p.L, p.L, j0, r.a1);
}

// output steps t = t_e-1 .. t_c; on entry st = beta_{t_e-1}, on exit beta_{t_c}.
// MODE 0 (EM): P only.  MODE 1: P / gamma / rho as given (decode, repair).
template <int J, int WP, int PF, bool VEC, int MODE>
__device__ __forceinline__ void bwd_stream_out(const FBParams& p, Bwd<J, WP>& st, int j0, const float invz[J],
                                               int64_t t_c, int64_t t_e, float vp0[J], float vp1[J],
                                               bool has_prev) {
  WaveTeam tm(nullptr);
  if (t_e - 1 < t_c) return;
  const int64_t L = p.L;
  BRow<J> ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) brow_load<J, VEC>(p, t_e - 1 - q > t_c ? t_e - 1 - q : t_c, j0, ring[q]);
  auto body = [&](int q, int64_t t, bool refill) {
    float a0[J], a1[J], e[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      a0[j] = ring[q].a0[j];
      a1[j] = ring[q].a1[j];
    }
    em_exp<J>(p, j0, ring[q].em, e);
    if (refill) brow_load<J, VEC>(p, t - PF > t_c ? t - PF : t_c, j0, ring[q]);
    float G = 0.f, V0 = 0.f, V1 = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      a0[j] *= st.b0[j];
      a1[j] *= st.b1[j];
      G += a0[j] + a1[j];
      V0 += e[j] * st.b0[j];
      V1 += e[j] * st.b1[j];
    }
    tm.sum2(V0, V1);
    G = tm.sum(G);
    const float iG = 1.f / G;
    float pp[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      a0[j] *= iG;
      a1[j] *= iG;
      pp[j] = a0[j] + a1[j];
    }
    if constexpr (MODE == 0) {
      bstore_row<J, VEC>(p.P + t * L, p.L, j0, pp);
    } else {
      if (p.P) bstore_row<J, VEC>(p.P + t * L, p.L, j0, pp);
      if (p.gamma) {
        bstore_row<J, VEC>(p.gamma + t * 2 * L, p.L, j0, a0);
        bstore_row<J, VEC>(p.gamma + t * 2 * L + L, p.L, j0, a1);
      }
      if (p.rho && has_prev && t + 1 < p.T) {  // rho_{t+1} = v_{t+1} / sum(alpha_t * beta_t)
        float r0[J], r1[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
          r0[j] = vp0[j] * iG;
          r1[j] = vp1[j] * iG;
        }
        bstore_row<J, VEC>(p.rho + (t + 1) * 2 * L, p.L, j0, r0);
        bstore_row<J, VEC>(p.rho + (t + 1) * 2 * L + L, p.L, j0, r1);
      }
    }
    if (t != t_c) {
      st.step_back(p, nullptr, j0, invz, e, V0, V1, vp0, vp1);
      has_prev = true;
    }
  };
  int64_t tb = t_e - 1;
  for (; tb - (PF - 1) >= t_c; tb -= PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) body(q, tb - q, true);
  }
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (tb - q >= t_c) body(q, tb - q, false);
}

template <int J, int WP, bool VEC, int MODE>
__device__ __forceinline__ void backward_chunk(const FBParams& p, int c, int j0, const float invz[J], bool fix) {
  WaveTeam tm(nullptr);
  const size_t SZ = (size_t)2 * p.Lpad;
  const int64_t t_c = (int64_t)c * p.C;
  const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
  Bwd<J, WP> st;
  float vp0[J], vp1[J];
#pragma unroll
  for (int j = 0; j < J; ++j) vp0[j] = vp1[j] = 0.f;
  bool has_prev = false;
  if (fix) {
    st.load_state(p, p.b_in + (size_t)c * SZ, j0);
    bwd_plain(tm, p, st, nullptr, j0, invz, t_e, vp0, vp1);
    has_prev = true;
  } else {
    st.init_ones(p, j0);
    if (c < p.M - 1) {
      int64_t t_w = t_e + p.B;  // beta guess (ones) at t_w, exact when t_w is the last bin
      if (t_w > p.T - 1) t_w = p.T - 1;
      bwd_stream_warm<J, WP, kPfBwdWarm, VEC>(p, st, j0, invz, t_w, t_e + 1);
      st.save_state(p, p.b_in + (size_t)c * SZ, j0);            // beta_{t_e}
      bwd_plain(tm, p, st, nullptr, j0, invz, t_e, vp0, vp1);   // -> beta_{t_e-1}
      has_prev = true;
    }
  }
  bwd_stream_out<J, WP, kPfBwdOut, VEC, MODE>(p, st, j0, invz, t_c, t_e, vp0, vp1, has_prev);
  st.save_state(p, p.b_first + (size_t)c * SZ, j0);
  if (fix && (threadIdx.x & 63) == 0) atomicAdd(&p.repairs[1], 1);
}

#define PMG_BWD_DISPATCH(MODE, FIX)                                     \
  if constexpr (J % 4 == 0) {                                           \
    if ((p.L & 3) == 0) {                                               \
      backward_chunk<J, WP, true, MODE>(p, c, j0, invz, FIX);           \
      return;                                                           \
    }                                                                   \
  }                                                                     \
  backward_chunk<J, WP, false, MODE>(p, c, j0, invz, FIX);

// speculative pass, EM outputs (P only)
template <int J, int WP>
__global__ void __launch_bounds__(64) k_backward(FBParams p) {
  const int c = blockIdx.x;
  if (c >= p.M) return;
  PMG_FB_LANE_SETUP
  PMG_BWD_DISPATCH(0, false)
}

// speculative pass, decode outputs (P / gamma / rho as given)
template <int J, int WP>
__global__ void __launch_bounds__(64) k_backward_full(FBParams p) {
  const int c = blockIdx.x;
  if (c >= p.M) return;
  PMG_FB_LANE_SETUP
  PMG_BWD_DISPATCH(1, false)
}

// parallel repair round: flagged chunk c restarts from its snapshot b_in[c] = beta_{t_e}
template <int J, int WP>
__global__ void __launch_bounds__(64) k_backward_fix(FBParams p) {
  const int c = blockIdx.x;
  if (c >= p.M - 1 || p.flags[c] == 0) return;
  PMG_FB_LANE_SETUP
  PMG_BWD_DISPATCH(1, true)
}

// sequential fallback (descending chunks), NW waves on the one chain
template <int J, int WP>
__global__ void __launch_bounds__(64 * repair_nw<J>()) k_backward_repair(FBParams p) {
  constexpr int NW = repair_nw<J>(), JB = J / NW;
  PMG_FB_PROLOGUE_T(JB, NW)
  BlockTeam<NW> tm(team_red);
  int repairs = 0;
  bool changed = false;
  int c = p.M - 2;
  while (c >= 0) {
    if (!changed) {
      int found = -1;
      for (int top = c; top >= 0 && found < 0; top -= 64) {
        const int idx = top - lane;
        const bool f = idx >= 0 && p.flags[idx] != 0;
        const unsigned long long bal = __ballot(f);
        if (bal) found = top - (int)__builtin_ctzll(bal);
      }
      if (found < 0) break;
      c = found;
    }
    const int64_t t_c = (int64_t)c * p.C;
    const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
    Bwd<JB, WP, BlockTeam<NW>> st;
    st.load_state(p, p.b_first + (size_t)(c + 1) * SZ, j0);
    st.save_state(p, p.b_in + (size_t)c * SZ, j0);
    float vp0[JB], vp1[JB];
    bwd_plain(tm, p, st, lds, j0, invz, t_e, vp0, vp1);
    bwd_out<JB, WP, BlockTeam<NW>, 16 / JB, true>(tm, p, st, lds, j0, invz, t_c, t_e, vp0, vp1, true);
    float* bf = p.b_first + (size_t)c * SZ;
    const float d = hilbert_reg<JB>(tm, st.b0, st.b1, bf, p.Lpad, j0);
    changed = !(d <= p.tol);
    __syncthreads();  // every wave has read bf before it is overwritten
    st.save_state(p, bf, j0);
    __threadfence();
    __syncthreads();
    ++repairs;
    --c;
  }
  if (threadIdx.x == 0) p.repairs[1] += repairs;
}

typedef void (*fb_kernel_t)(FBParams);

// the kernels of one (J, WP) instance (fb_inst_j*.hip)
struct FBKernelSet {
  fb_kernel_t forward, forward_fix, forward_repair;
  fb_kernel_t backward, backward_full, backward_fix, backward_repair;
};

bool fb_set_j1(int WP, FBKernelSet* k);
bool fb_set_j2(int WP, FBKernelSet* k);
bool fb_set_j4(int WP, FBKernelSet* k);
bool fb_set_j8(int WP, FBKernelSet* k);
bool fb_set_j16(int WP, FBKernelSet* k);

template <int J, int WP>
inline void fb_fill(FBKernelSet* k) {
  k->forward = k_forward<J, WP>;
  k->forward_fix = k_forward_fix<J, WP>;
  k->forward_repair = k_forward_repair<J, WP>;
  k->backward = k_backward<J, WP>;
  k->backward_full = k_backward_full<J, WP>;
  k->backward_fix = k_backward_fix<J, WP>;
  k->backward_repair = k_backward_repair<J, WP>;
}

// one instance file per J
#define PMG_FB_INSTANCES(JJ)                          \
  bool fb_set_j##JJ(int WP, FBKernelSet* k) {         \
    switch (WP) {                                     \
      case 5: fb_fill<JJ, 5>(k); return true;         \
      case 9: fb_fill<JJ, 9>(k); return true;         \
      case 13: fb_fill<JJ, 13>(k); return true;       \
      case 17: fb_fill<JJ, 17>(k); return true;       \
      case 25: fb_fill<JJ, 25>(k); return true;       \
      case 32: fb_fill<JJ, 32>(k); return true;       \
      default: return false;                          \
    }                                                 \
  }

}  // namespace pmg
