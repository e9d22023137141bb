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
//     as a 1-D convolution across the lanes of one wave (DPP shifts); the jump kernel
//     is rank-1 (a wave reduction); the 2x2 dynamics mix is elementwise;
//   * main pass: one wave per time chunk; each chunk starts from a uniform guess
//     `warmup` steps early (HMM forgetting);
//   * every chunk boundary is then verified in the Hilbert projective metric (max-min
//     of log ratios; positive linear maps contract it, so a boundary error <= tol
//     bounds every later output's relative error by tol), and the chunks behind a
//     failing boundary are recomputed by a persistent RELAXATION kernel: one wave per
//     segment of G consecutive chunks (<= one workgroup per CU, all co-resident),
//     rounds separated by a grid barrier.  In a round a segment recomputes its chunks
//     sequentially from its first inconsistent boundary (stopping as soon as a
//     recomputed state coalesces with the old one); a segment whose end state moved
//     hands it to its right neighbour for the next round.  The rounds end when no
//     segment end moved, i.e. every boundary verifies.  A slowly forgetting chain (the
//     nearly flat tuning of the first EM iterations) thus costs ~(forgetting length)
//     sequential steps, not T;
//   * the smoother uses the equivalent alpha-beta form gamma_t ~ alpha_t * beta_t
//     with beta_{T-1} = 1 (the reference's RTS seed acausal_{T-1} = post_{T-1}), so
//     the backward pass needs only alpha_t and the emission -- no stored priors.
//
// Emission input: e[t,l] = exp(s*delta[t,l] + phi[t,l/32]) = exp(s*(ll[t,l] - m[t])).
#pragma once
#include <stdlib.h>

#include <type_traits>

#include "pmg_common.h"

// Contract a*b+c only inside one expression (the explicit fmaf calls).  Chunk
// boundaries coalesce bitwise only if every unrolled copy of a step (the PF-deep row
// rings) rounds identically; hipcc's default cross-statement contraction lets the
// scheduler fuse differently per copy.
#pragma clang fp contract(on)

namespace pmg {

constexpr int kMaxBand = 32;
// Emission / alpha rows are prefetched this many steps ahead on the chunk-parallel
// kernels: with ~2 waves per SIMD the step's VALU work (~0.3 us) cannot cover an HBM
// round trip (~2 us), so the row ring, not other waves, hides the latency.
// The forward's alpha (d = 0) rows are stored non-temporally (nt) for L <= 512 (J <= 8):
// with them out of the caches the C3 backward pass, which reads delta + alpha, ran 11-16 us
// faster and the forward 2-5 us slower; at L = 1024 (J = 16, the C4 shard) the forward ran
// 25 % slower with them, so J = 16 keeps the default policy (profiles/r05_ab_experiments.txt
// item 18).  0 = the default policy everywhere (A/B builds).
#ifndef PMG_ALPHA_AUX
#define PMG_ALPHA_AUX 2
#endif
#ifndef PMG_PF_FWD
#define PMG_PF_FWD 4
#endif
#ifndef PMG_PF_BWD_WARM
#define PMG_PF_BWD_WARM 4
#endif
#ifndef PMG_PF_BWD_OUT
#define PMG_PF_BWD_OUT 2
#endif
constexpr int kPfFwd = PMG_PF_FWD;
constexpr int kPfBwdWarm = PMG_PF_BWD_WARM;
constexpr int kPfBwdOut = PMG_PF_BWD_OUT;
// the relaxation kernel runs <= 1 wave per CU: a deeper ring covers the latency alone,
// as deep as the registers allow (a backward row is 3J floats).  J = 8 forward: 4, not 8
// (with the EM relaxation's A1-free loop, the 4-deep ring was 7 % faster on the first
// E-step of a fit, profiles/r05_ab_experiments.txt item 7)
template <int J> constexpr int pf_relax_fwd() { return J >= 8 ? 4 : 8; }
template <int J> constexpr int pf_relax_bwd() { return J >= 16 ? 2 : (J >= 8 ? 4 : 8); }

// Control words at the start of the scan workspace (int32), one block per direction
// (forward at word 0, backward at word kCtlStride):
//   +0 chunks recomputed, +1 relaxation rounds   (zeroed by the main pass)
//   +2 timeout flag: sticky -- set by a relaxation whose grid barrier timed out, left
//      set by later calls (whose relaxations then fail fast), cleared by the host after
//      it has read it (DeviceEM.scan_status)
//   +3 warm-up of the next main pass (adaptive scans; written by the relaxation kernel)
//   +4 boundaries flagged by k_verify, +5 barrier arrivals,
//   +6..+8 segment-end changes of rounds k % 3, +9 relaxation exits
// Words 4..9 are zero between calls: the workspace starts zero-filled and the last
// relaxation wave to exit clears them, so no call needs a host memset.
enum {
  kCtlRepairs = 0,
  kCtlRounds = 1,
  kCtlErr = 2,
  kCtlWarm = 3,
  kCtlPending = 4,
  kCtlArrive = 5,
  kCtlChanged = 6,
  kCtlExit = 9,
  kCtlStride = 16,
};
constexpr uint64_t kSpinTicks = 200000000ull;          // 2 s of the 100 MHz real-time clock
constexpr int kRelaxMaxSeg = 512;                      // segment-state slots in the workspace
// Adaptive warm-up (FBParams::adapt): when more than 1/kCascadeFrac of a pass's
// boundaries failed (a slowly mixing chain: the nearly flat tuning of the first EM
// iterations), the next main pass of that direction warms up kLongWarm steps instead
// of B, which leaves mostly noise-level boundary failures (~1 chunk of repair each)
// instead of a relaxation cascade over whole segments.  Decided on the device, so
// no host sync and identical decisions however far the host runs ahead.
constexpr int kLongWarm = 256;
constexpr int kCascadeFrac = 8;

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
  double* logz;
  float* s_in;
  float* s_out;
  // per step (jump mass, 1/S) of the forward (T x 2 f32, in the workspace): alpha's d = 1
  // row is jump * e_t / S, so the backward rebuilds it bit-exactly from e_t and these
  float* jsc;
  uint32_t a1_bytes;  // bytes of alpha's d = 1 rows the forward stores (4 L, or 0: omitted)
  uint32_t a0_bytes;  // bytes of alpha's d = 0 rows the forward stores (4 L, or 0: logZ-only passes)
  // backward
  const float* alpha_in;  // only the d = 0 rows are read
  float* w_first;         // per chunk: alpha at its first step, (2, Lpad) (boundary weights)
  float* P;
  uint16_t* Pq;         // PMG_PHASE_P_BF16X3: P as bf16 planes hi / mid / lo, plane k at Pq + k pq_stride
  int64_t pq_stride;    // T ldd
  float* gamma;
  float* rho;
  float* b_in;
  float* b_first;
  int* flags;
  int* ctl;       // this direction's control block
  uint64_t spin;  // grid-barrier spin bound (real-time clock ticks; kSpinTicks unless a debug override)
  // relaxation: segments of G chunks, S segments; end states double-buffered by round
  float* seg_end;  // [2][S][2*Lpad]
  int* seg_chg;    // [2][S]
  int G, S;
  int Lpad;  // 64*J
  // adaptive warm-up (kCtlWarm): main pass uses max(B, ctl[kCtlWarm]); relaxation writes it
  int adapt;
  // row strides: delta and P (floats; L, or R L when R restarts' latents are stacked
  // side by side), phi (nblk or R nblk), m (1 or R)
  int ldd, ldphi, ldm;
  // batched restarts (blockIdx.y = restart r): per-restart offsets of the stacked inputs
  // (delta / P: r L floats, phi: r nblk, m: r), of the sequence outputs (alpha / gamma:
  // r T 2L, logc: r T, logz: r) and of the restart's own workspace slab (r ws_stride bytes)
  int64_t ws_stride;
};

// this restart's view of the parameters (identity for blockIdx.y = 0)
__device__ __forceinline__ FBParams batch_view(const FBParams& p0) {
  FBParams p = p0;
  const int r = blockIdx.y;
  if (r == 0) return p;
  const int64_t seq = (int64_t)r * p.T;
  p.delta += (int64_t)r * p.L;
  if (p.P) p.P += (int64_t)r * p.L;
  if (p.Pq) p.Pq += (int64_t)r * p.L;
  p.phi += (int64_t)r * p.nblk;
  p.m += r;
  if (p.alpha) p.alpha += seq * 2 * p.L;
  if (p.alpha_in) p.alpha_in += seq * 2 * p.L;
  if (p.gamma) p.gamma += seq * 2 * p.L;
  if (p.logc) p.logc += seq;
  if (p.logz) p.logz += r;
  const int64_t o = (int64_t)r * p.ws_stride;
  auto mv = [o](auto*& q) {
    typedef std::remove_reference_t<decltype(q)> ptr_t;
    if (q) q = reinterpret_cast<ptr_t>(reinterpret_cast<uintptr_t>(q) + (uintptr_t)o);
  };
  mv(p.jsc); mv(p.chunk_logz); mv(p.s_in); mv(p.s_out); mv(p.w_first); mv(p.b_in); mv(p.b_first);
  mv(p.flags); mv(p.ctl); mv(p.seg_end); mv(p.seg_chg);
  return p;
}

// this main pass's warm-up: B, or the longer one the last relaxation of this direction
// asked for (adaptive scans)
__device__ __forceinline__ int64_t main_warmup(const FBParams& p) {
  if (!p.adapt) return p.B;
  const int w = __builtin_amdgcn_readfirstlane(p.ctl[kCtlWarm]);
  return w > p.B ? w : p.B;
}

// the relaxation's warm-up decision for the next main pass (s == 0, lane 0)
__device__ __forceinline__ void relax_warm_decision(const FBParams& p, int pending) {
  if (p.adapt) p.ctl[kCtlWarm] = (pending * kCascadeFrac > p.M) ? kLongWarm : 0;
}

// ---------------------------------------------------------------------------
// per-lane helpers (lane owns latents j0 .. j0+J-1, j0 = lane*J)
// ---------------------------------------------------------------------------
// One lane's J values of a streamed row, held as 4-wide vectors: a row-ring slot is then
// a few 128-bit values that its buffer loads fill in place (as J separate floats hipcc
// re-pairs them for the packed math and copies every refill into the slot's registers,
// each copy waiting for its load).
typedef float f4v __attribute__((ext_vector_type(4)));
template <int J>
struct RowV {
  f4v q[(J + 3) / 4];
  __device__ __forceinline__ float operator[](int j) const { return q[j >> 2][j & 3]; }
  __device__ __forceinline__ void set(int j, float x) { q[j >> 2][j & 3] = x; }
};

template <int J>
__device__ __forceinline__ void load_row(const float* __restrict__ row, int L, int j0, RowV<J>& v) {
  if ((L & 3) == 0 && (J & 3) == 0 && j0 + J <= L) {
#pragma unroll
    for (int j = 0; j < J; j += 4) v.q[j >> 2] = *reinterpret_cast<const f4v*>(row + j0 + j);
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) v.set(j, (j0 + j < L) ? row[j0 + j] : 0.f);
  }
}

// raw emission operands for one time step
template <int J>
struct EmRaw {
  RowV<J> d;
  float ph;
};

template <int J>
__device__ __forceinline__ void em_load(const FBParams& p, int64_t t, int j0, EmRaw<J>& r) {
  load_row<J>(p.delta + t * p.ldd, p.L, j0, r.d);
  const int b = j0 >> 5;
  r.ph = (b < p.nblk) ? p.phi[t * p.ldphi + b] : 0.f;
}

// exp_acc on an aligned element pair (j, j + 1) as packed math: the pairing is the one the
// row slot's 128-bit loads deliver, so hipcc does not re-pair (copy) the loaded values
typedef float f2x __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2x exp_acc2(f2x x) {
  constexpr float kL2E = 1.44269502162933349609375f;
  constexpr float kL2E_lo = 1.925963033500011e-08f;
  const f2x y = x * (f2x){kL2E, kL2E};
  f2x err = __builtin_elementwise_fma(x, (f2x){kL2E, kL2E}, -y);
  err = __builtin_elementwise_fma(x, (f2x){kL2E_lo, kL2E_lo}, err);
  const f2x r = {__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
  return __builtin_elementwise_fma(r, err * (f2x){0.693147180559945309f, 0.693147180559945309f}, r);
}

// FULL: every lane's latents are < L (L == Lpad), so no lane-validity select
template <int J, bool FULL = false>
__device__ __forceinline__ void em_exp(const FBParams& p, int j0, const EmRaw<J>& r, float e[J]) {
  if constexpr (FULL && (J % 2) == 0) {
#pragma unroll
    for (int j = 0; j < J; j += 2) {
      const f2x d = {r.d[j], r.d[j + 1]};
      const f2x x = __builtin_elementwise_fma((f2x){p.s, p.s}, d, (f2x){r.ph, r.ph});
      const f2x v = exp_acc2(x);
      e[j] = v.x;
      e[j + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) e[j] = (FULL || j0 + j < p.L) ? exp_acc(fmaf(p.s, r.d[j], r.ph)) : 0.f;
  }
}

// One wave holds the whole line (lane l owns latents lJ .. lJ+J-1): the halo comes
// from the neighbouring lanes through wavefront-shift DPP moves (wave_shr:1 /
// wave_shl:1; the lanes past either end read 0), so the step touches no LDS.  The
// contiguous-block LDS exchange it replaces ran into 8-way bank conflicts (lane
// stride J words).  Only the entries inside the band are moved: J + 1 per side at
// J = 8, WP = 9.
// bound_ctrl: the lane without a source reads 0 (no 'old' operand to initialise)
__device__ __forceinline__ float wave_shr1(float v) {  // lane i <- lane i-1 (lane 0 <- 0)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float wave_shl1(float v) {  // lane i <- lane i+1 (lane 63 <- 0)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}

// the same shifts with the incoming lane (lane 0 / lane 63) taking `in0` instead of 0:
// DPP with bound_ctrl off leaves a lane whose source is out of range at its old value
__device__ __forceinline__ float wave_shr1_in(float v, float in0) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(in0), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_shl1_in(float v, float in63) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(in63), __float_as_int(v), 0x130, 0xf, 0xf, false));
}

// ---------------------------------------------------------------------------
// Several waves per chain (NW > 1): wave w of the chain's workgroup owns latents
// (64 w + lane) J .. + J - 1, so the (2, Lpad) state layout is the one-wave layout at
// J' = NW J.  Per exchange each wave writes its line (the band convolution's input) and
// its wave-reduced partial sums to LDS, one s_barrier, then reads its neighbours' edge
// latents (the halo of the DPP shifts) and every wave's partials, summed in wave order so
// all waves hold bit-identical totals.  Two LDS slots alternate between exchanges: a
// wave writes slot s again only after the barrier of the next exchange, which its
// neighbours pass only once their reads of slot s have returned (the LDS-only release
// before each barrier waits lgkmcnt(0), nothing else: the row rings stay in flight).
// Line slots 0 and NW + 1 of each LDS slot stay zero: the halo past the line's ends.
// ---------------------------------------------------------------------------
template <int NW, int J>
struct ChainX {
  static constexpr int kLine = 64 * J;
  static constexpr int kSlot = (NW + 2) * kLine + NW * 4;   // lines + [NW][4] partial sums
  int w;      // this wave's index in the chain (wave-uniform)
  int par;    // LDS slot of the next exchange
  float* lds;

  __device__ __forceinline__ void init() {
    lds = nullptr;
    w = 0;
    par = 0;
    if constexpr (NW > 1) {
      __shared__ float buf[2 * kSlot];
      lds = buf;
      w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
      for (int s = 0; s < 2; ++s)
        for (int i = threadIdx.x; i < kLine; i += 64 * NW) {
          buf[s * kSlot + i] = 0.f;
          buf[s * kSlot + (NW + 1) * kLine + i] = 0.f;
        }
      barrier();
    }
  }
  __device__ __forceinline__ static void barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  // one exchange: `line` (this lane's J values, may be null) and NS wave-uniform partial
  // sums in; the neighbours' edge values (NL lanes x J each side, lin: left neighbour's
  // lanes 64-NL..63, rin: right neighbour's lanes 0..NL-1; zero past the line) and the
  // chain's totals out
  template <int NL, int NS>
  __device__ __forceinline__ void exchange(const float* line, float* lin, float* rin, float* sums) {
    static_assert(NW > 1 && NS <= 4 && NL <= 64, "chain exchange");
    float* s = lds + par * kSlot;
    const int lane = threadIdx.x & 63;
    if (line) {
      float* my = s + (w + 1) * kLine + lane * J;
#pragma unroll
      for (int j = 0; j < J; ++j) my[j] = line[j];
    }
    if (NS > 0 && lane == 0) {
#pragma unroll
      for (int k = 0; k < NS; ++k) s[(NW + 2) * kLine + w * 4 + k] = sums[k];
    }
    barrier();
    if (line) {
      const float* ln = s + w * kLine + kLine - NL * J;    // wave w-1 (or the zero slot)
      const float* rn = s + (w + 2) * kLine;               // wave w+1 (or the zero slot)
#pragma unroll
      for (int q = 0; q < NL * J; ++q) {
        lin[q] = ln[q];
        rin[q] = rn[q];
      }
    }
    if constexpr (NS > 0) {
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        float t = 0.f;
#pragma unroll
        for (int v = 0; v < NW; ++v) t += s[(NW + 2) * kLine + v * 4 + k];
        sums[k] = t;
      }
    }
    par ^= 1;
  }
};

// out[j] = sum_{k=-WP..WP} g[|k|] * in[j+k]  over the whole latent line (zero halo).
// NW > 1: the lanes at the wave's ends take their neighbours' values from lin / rin
// (ChainX::exchange), so the line spans the chain's NW waves.
template <int J, int WP, int NW = 1>
__device__ __forceinline__ void band_conv(const FBParams& p, const float in[J], float out[J],
                                          const float* lin = nullptr, const float* rin = nullptr) {
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
      if (k * J - i > WP) win[C - k * J + i] = 0.f;
      else if constexpr (NW > 1) win[C - k * J + i] = wave_shr1_in(win[C - (k - 1) * J + i], lin[(NL - k) * J + i]);
      else win[C - k * J + i] = wave_shr1(win[C - (k - 1) * J + i]);
    }
  // right: block k (lane l+k) local i at window C + kJ + i; needed iff kJ + i - (J-1) <= WP
#pragma unroll
  for (int k = 1; k <= NL; ++k)
#pragma unroll
    for (int i = 0; i < J; ++i) {
      if (k * J + i - (J - 1) > WP) win[C + k * J + i] = 0.f;
      else if constexpr (NW > 1) win[C + k * J + i] = wave_shl1_in(win[C + (k - 1) * J + i], rin[(k - 1) * J + i]);
      else win[C + k * J + i] = wave_shl1(win[C + (k - 1) * J + i]);
    }
  if constexpr ((J & 1) == 0) {
    // output pairs (j, j+1) on packed math (v_pk_fma_f32 / v_pk_add_f32): per lane the
    // same IEEE operations as the scalar form below, so identical bits.  For even taps
    // k both window pairs are register-aligned (one packed add); for odd k the two
    // sums are formed by scalar adds straight into an aligned pair.
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 acc[J / 2];
#pragma unroll
    for (int jp = 0; jp < J / 2; ++jp) {
      const f2 c = {win[C + 2 * jp], win[C + 2 * jp + 1]};
      acc[jp] = (f2){p.g[0], p.g[0]} * c;
    }
#pragma unroll
    for (int k = 1; k <= WP; ++k) {
      const f2 gk = {p.g[k], p.g[k]};
#pragma unroll
      for (int jp = 0; jp < J / 2; ++jp) {
        const int a = C + 2 * jp - k, b = C + 2 * jp + k;
        f2 sm;
        if ((k & 1) == 0) {
          const f2 l = {win[a], win[a + 1]}, r = {win[b], win[b + 1]};
          sm = l + r;
        } else {
          sm.x = win[a] + win[b];
          sm.y = win[a + 1] + win[b + 1];
        }
        acc[jp] = __builtin_elementwise_fma(gk, sm, acc[jp]);
      }
    }
#pragma unroll
    for (int jp = 0; jp < J / 2; ++jp) {
      out[2 * jp] = acc[jp].x;
      out[2 * jp + 1] = acc[jp].y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      float acc = p.g[0] * win[C + j];
#pragma unroll
      for (int k = 1; k <= WP; ++k) acc = fmaf(p.g[k], win[C + j - k] + win[C + j + k], acc);
      out[j] = acc;
    }
  }
}

// reductions over one chain: the wave's sum, then (NW > 1) the waves' partials in wave
// order through the chain's LDS exchange
template <int NW, int J>
__device__ __forceinline__ void chain_sum2(ChainX<NW, J>& x, float& a, float& b) {
  wave_sum2(a, b);
  if constexpr (NW > 1) {
    float s[2] = {a, b};
    x.template exchange<0, 2>(nullptr, nullptr, nullptr, s);
    a = s[0];
    b = s[1];
  }
}

// ---------------------------------------------------------------------------
// Hilbert projective distance between two non-negative (2, Lpad) states.
// Unweighted (state space): components below 1e-30 of the max on both sides are
// ignored, a component above 1e-20 on one side only counts as a failure.  Weighted by
// w (alpha at the boundary in a (2, Lw) layout -- the scans pass the (2, Lpad) rows of
// w_first, entries past L zero; backward boundaries compare the POSTERIOR,
// |posterior| <= 1): components below 1e-14 move no output by more than 1e-14
// absolute (parity atol 1e-12); above it the ratio spread bounds the relative error.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float hilbert_finish(float lo, float hi, int bad) {
  lo = wave_min_shfl(lo);
  hi = wave_max_shfl(hi);
  if (__ballot(bad)) return INFINITY;
  if (hi < lo) return 0.f;
  return hi - lo;
}

// both states in memory (one wave), n = 2 Lpad floats, optional weights w[i] in the same
// (2, Lpad) layout.  Every operand is fetched up front with branch-free 16-byte buffer
// loads (lanes past n read 0), so the wave pays one memory round trip: the predicated
// scalar loads this replaces were serialised by their branches (k_verify spent 80 % of
// its ~20 us waiting on memory).
__device__ __forceinline__ float hilbert_dist(const float* __restrict__ x, const float* __restrict__ y, int n,
                                              const float* __restrict__ w = nullptr) {
  const int lane = threadIdx.x & 63;
  constexpr int kQ = 2 * 1024 / 256;  // float4 loads per lane for n <= 2048
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), (short)0, n * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(y), (short)0, n * 4, 0x00020000);
  const bool weighted = w != nullptr;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(weighted ? w : x), (short)0, n * 4, 0x00020000);
  float xv[4 * kQ], yv[4 * kQ];
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const int off = (lane + 64 * q) * 16;
    const u4 a = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
    const u4 b = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
    xv[4 * q] = __uint_as_float(a.x); xv[4 * q + 1] = __uint_as_float(a.y);
    xv[4 * q + 2] = __uint_as_float(a.z); xv[4 * q + 3] = __uint_as_float(a.w);
    yv[4 * q] = __uint_as_float(b.x); yv[4 * q + 1] = __uint_as_float(b.y);
    yv[4 * q + 2] = __uint_as_float(b.z); yv[4 * q + 3] = __uint_as_float(b.w);
    const u4 c = __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0);  // no branch: selects below
    const float wc[4] = {__uint_as_float(c.x), __uint_as_float(c.y), __uint_as_float(c.z), __uint_as_float(c.w)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float f = weighted ? wc[k] : 1.f;
      xv[4 * q + k] *= f;
      yv[4 * q + k] *= f;
    }
  }
  float xm = 0.f, ym = 0.f;
#pragma unroll
  for (int q = 0; q < 4 * kQ; ++q) {
    xm = fmaxf(xm, xv[q]);
    ym = fmaxf(ym, yv[q]);
  }
  xm = wave_max_shfl(xm);
  ym = wave_max_shfl(ym);
  if (!(xm > 0.f) || !(ym > 0.f)) return INFINITY;
  const float ix = 1.f / xm, iy = 1.f / ym;
  const float lo_thr = weighted ? 1e-14f : 1e-30f, hi_thr = weighted ? 1e-12f : 1e-20f;
  float lo = INFINITY, hi = -INFINITY;
  int bad = 0;
#pragma unroll
  for (int q = 0; q < 4 * kQ; ++q) {
    const float a = xv[q] * ix, b = yv[q] * iy;
    if (a > lo_thr && b > lo_thr) {
      const float r = __logf(a * __builtin_amdgcn_rcpf(b));  // log of the ratio: see hilbert_reg
      lo = fminf(lo, r);
      hi = fmaxf(hi, r);
    } else if (fmaxf(a, b) > hi_thr) {
      bad = 1;
    }
  }
  return hilbert_finish(lo, hi, bad);
}

// same metric, x held in registers in the (2, Lpad) lane layout, y in memory;
// optional weights w in a (2, L) layout (L = Lpad for w_first rows)
template <int J>
__device__ __forceinline__ float hilbert_reg(const float x0[J], const float x1[J], const float* __restrict__ y, int Lpad, int j0,
                             const float* __restrict__ w = nullptr, int L = 0) {
  float a[2 * J], b[2 * J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    float w0 = 1.f, w1 = 1.f;
    if (w) {
      w0 = j0 + j < L ? w[j0 + j] : 0.f;
      w1 = j0 + j < L ? w[L + j0 + j] : 0.f;
    }
    a[j] = x0[j] * w0;
    a[J + j] = x1[j] * w1;
    b[j] = y[j0 + j] * w0;
    b[J + j] = y[Lpad + j0 + j] * w1;
  }
  float xm = 0.f, ym = 0.f;
#pragma unroll
  for (int j = 0; j < 2 * J; ++j) {
    xm = fmaxf(xm, a[j]);
    ym = fmaxf(ym, b[j]);
  }
  xm = wave_max_shfl(xm);
  ym = wave_max_shfl(ym);
  if (!(xm > 0.f) || !(ym > 0.f)) return INFINITY;
  const float ix = 1.f / xm, iy = 1.f / ym;
  const float lo_thr = w ? 1e-14f : 1e-30f, hi_thr = w ? 1e-12f : 1e-20f;
  float lo = INFINITY, hi = -INFINITY;
  int bad = 0;
#pragma unroll
  for (int j = 0; j < 2 * J; ++j) {
    const float u = a[j] * ix, v = b[j] * iy;
    if (u > lo_thr && v > lo_thr) {
      // log of the ratio, not a difference of logs: for components near 1e-20 the log is
      // ~46, whose f32 ulp (3.8e-6) exceeds the tolerance, so two states 1 ulp apart
      // (the unnormalised scans store q * iS) would never read as converged
      const float r = __logf(u * __builtin_amdgcn_rcpf(v));
      lo = fminf(lo, r);
      hi = fmaxf(hi, r);
    } else if (fmaxf(u, v) > hi_thr) {
      bad = 1;
    }
  }
  return hilbert_finish(lo, hi, bad);
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// The state is held unnormalised: alpha_t = (q0 * iS, (jmp * ep) * iS), with ep the
// step's emission row and (jmp, iS) its jump mass and 1/S.  The next step folds iS into
// its scalar coefficients, so no per-element normalisation or d = 1 row is formed on
// the recursion (only where alpha is stored); the backward rebuilds alpha's d = 1 row
// from (e, jmp, iS) exactly as written here.
template <int J, int WP, int NW = 1>
struct Fwd {
  static constexpr int NL = (WP + J - 1) / J;
  float q0[J], ep[J];
  float P0, P1;  // normalised sums of the d = 0 / d = 1 parts (wave-uniform)
  float jmp, iS; // the last step's jump mass and 1/S
  ChainX<NW, J> x;

  __device__ void init_uniform(const FBParams& p, int j0) {
    x.init();
    const float u = 0.5f * p.invL;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      q0[j] = (j0 + j < p.L) ? u : 0.f;
      ep[j] = q0[j];
    }
    jmp = 1.f;
    iS = 1.f;
    P0 = 0.5f;
    P1 = 0.5f;
  }
  __device__ void load_state(const FBParams& p, const float* src, int j0) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      q0[j] = src[j0 + j];
      ep[j] = src[p.Lpad + j0 + j];
    }
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      a += q0[j];
      b += ep[j];
    }
    chain_sum2(x, a, b);
    const float inv = rcp_nr(a + b);
    jmp = 1.f;
    iS = inv;
    P0 = a * inv;
    P1 = b * inv;
  }
  // the normalised (2, Lpad) state
  __device__ void save_state(const FBParams& p, float* dst, int j0) const {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      dst[j0 + j] = q0[j] * iS;
      dst[p.Lpad + j0 + j] = (jmp * ep[j]) * iS;
    }
  }
  // one filter step with emission e; returns the normaliser S
  __device__ float step(const FBParams& p, int j0, const float invz[J], const float e[J]) {
    const float c0 = p.A00 * iS, c1 = (p.A10 * jmp) * iS;
    float a0[J];
#pragma unroll
    for (int j = 0; j < J; ++j) a0[j] = fmaf(q0[j], c0, ep[j] * c1) * invz[j];
    const float jump = fmaf(p.A01, P0, p.A11 * P1) * p.invL;
    float pr0[J];
    if constexpr (NW > 1) {
      float lin[NL * J], rin[NL * J];
      x.template exchange<NL, 0>(a0, lin, rin, nullptr);
      band_conv<J, WP, NW>(p, a0, pr0, lin, rin);
    } else {
      band_conv<J, WP>(p, a0, pr0);
    }
    float U0 = 0.f, E = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      q0[j] = pr0[j] * e[j];
      ep[j] = e[j];
      U0 += q0[j];
      E += e[j];
    }
    chain_sum2(x, U0, E);
    const float U1 = jump * E;
    const float S = U0 + U1;
    const float inv = rcp_nr(S);
    P0 = U0 * inv;
    P1 = U1 * inv;
    jmp = jump;
    iS = inv;
    return S;
  }
};

// ---------------------------------------------------------------------------
// Streaming step loops (one wave per chain).  Every row access is a raw buffer
// load/store through a per-row resource (num_records = row bytes), so lanes past L
// read 0 / drop their writes without exec masking, and the step loop is
// straight-line: the rows of the next PF steps stay in flight across steps (the
// waitcnt pass only sees one in-order vmcnt stream; any divergent load or store in
// the loop would make it drain the ring).  VEC: L % 4 == 0 (16-byte row accesses).
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int J, int VEC>
__device__ __forceinline__ void bload_row(const float* row, int L, int j0, RowV<J>& v) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(row, (uint32_t)L * 4u);
  if constexpr (VEC) {
#pragma unroll
    for (int j = 0; j < J; j += 4)
      v.q[j >> 2] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (j0 + j) * 4, 0, 0));
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) v.set(j, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (j0 + j) * 4, 0, 0)));
  }
}

// bytes: the row's extent (lanes past it drop their stores; 0 = the row is not written)
template <int J, int VEC, int AUX = 0>
__device__ __forceinline__ void bstore_row_n(float* row, uint32_t bytes, int j0, const float v[J]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(row, bytes);
  if constexpr (VEC) {
#pragma unroll
    for (int j = 0; j < J; j += 4) {
      u32x4 q;
      q.x = __float_as_uint(v[j]);
      q.y = __float_as_uint(v[j + 1]);
      q.z = __float_as_uint(v[j + 2]);
      q.w = __float_as_uint(v[j + 3]);
      __builtin_amdgcn_raw_buffer_store_b128(q, rs, (j0 + j) * 4, 0, AUX);
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[j]), rs, (j0 + j) * 4, 0, AUX);
  }
}

template <int J, int VEC>
__device__ __forceinline__ void bstore_row(float* row, int L, int j0, const float v[J]) {
  bstore_row_n<J, VEC>(row, (uint32_t)L * 4u, j0, v);
}

// row t of P as three bf16 planes (PMG_PHASE_P_BF16X3): the exact split of each value
// (split3_pair), the lane's J values as J / 2 dwords per plane
template <int J, int VEC>
__device__ __forceinline__ void bstore_planes(const FBParams& p, int64_t t, int j0, const float v[J]) {
  const uint32_t bytes = (uint32_t)p.L * 2u;
  if constexpr (VEC) {   // J % 4 == 0, L % 4 == 0: 8-byte aligned runs
    uint32_t w[3][J / 2];
#pragma unroll
    for (int i = 0; i < J / 2; ++i) split3_pair(v[2 * i], v[2 * i + 1], w[0][i], w[1][i], w[2][i]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(p.Pq + k * p.pq_stride + t * p.ldd, bytes);
      if constexpr (J == 4) {
        const u32x2 q = {w[k][0], w[k][1]};
        __builtin_amdgcn_raw_buffer_store_b64(q, rs, j0 * 2, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < J / 2; i += 4) {
          const u32x4 q = {w[k][i], w[k][i + 1], w[k][i + 2], w[k][i + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(q, rs, (j0 + 2 * i) * 2, 0, 0);
        }
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      uint32_t hw, mw, lw;
      split3_pair(v[j], 0.f, hw, mw, lw);
      const uint32_t w3[3] = {hw, mw, lw};
#pragma unroll
      for (int k = 0; k < 3; ++k)
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(w3[k] & 0xFFFFu),
                                             rsrc_of(p.Pq + k * p.pq_stride + t * p.ldd, bytes), (j0 + j) * 2, 0, 0);
    }
  }
}

// two f32 per step (x at 2t, y at 2t + 1) written by lane 0 only
__device__ __forceinline__ void bstore_pair_lane0(float* base, int64_t t, float x, float y) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(base + 2 * t, 8u);
  const int off = threadIdx.x == 0 ? 0 : 64;   // one store per chain (every wave of it holds the value)
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), rs, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), rs, off + 4, 0, 0);
}

// one f64 per step written by lane 0 only (the other lanes' offsets are out of range)
__device__ __forceinline__ void bstore_f64_lane0(double* base, int64_t t, double v) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(base + t, 8u);
  const int off = threadIdx.x == 0 ? 0 : 64;
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)u, rs, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)(u >> 32), rs, off + 4, 0, 0);
}

// Ordering point without instructions: `v` counts as rewritten once `dep` (a value of the
// step before) exists, so the emission arithmetic of a ring slot is not hoisted above the
// previous step.  Without it hipcc evaluates the exp arguments of every slot of the ring
// at the loop head, which makes it wait for all of them -- and for every store issued
// since (s_waitcnt vmcnt(0) once per ring cycle).
__device__ __forceinline__ void order_after(float& v, float dep) { asm volatile("" : "+v"(v) : "v"(dep)); }

// The values derived from a ring slot exist before the slot's refill is issued: the old
// and the new contents of the slot are then never live together, so the refill loads
// straight into the slot's registers.  Otherwise hipcc hoists the refill, loads into
// other registers and copies them into the slot before the loop's back edge -- and a copy
// of a loaded register waits for the load (s_waitcnt vmcnt(0) inside the ring cycle).
template <int J>
__device__ __forceinline__ void slot_consumed(const float v[J]) {
#pragma unroll
  for (int j = 0; j < J; ++j) asm volatile("" ::"v"(v[j]));
  asm volatile("" ::: "memory");
}

template <int J, int VEC>
__device__ __forceinline__ void bem_load(const FBParams& p, int64_t t, int j0, EmRaw<J>& r) {
  bload_row<J, VEC>(p.delta + t * p.ldd, p.L, j0, r.d);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(p.phi + t * p.ldphi, (uint32_t)p.nblk * 4u);
  r.ph = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (j0 >> 5) * 4, 0, 0));
}

// forward steps t in [t_a, t_b): OUT writes alpha / logc and returns sum logc; A1: also
// alpha's d = 1 rows (p.a1_bytes of them; the EM passes omit them).  MLDS: the row
// references m_t come from sm (LDS, indexed t - t_a), else from a register ring
template <int J, int WP, int PF, int VEC, bool OUT, bool A1, bool MLDS, int NW>
__device__ __forceinline__ double fwd_stream_piece(const FBParams& p, Fwd<J, WP, NW>& st, int j0, const float invz[J],
                                                   int64_t t_a, int64_t t_b, const double* sm) {
  double logz = 0.0;
  if (t_a >= t_b) return 0.0;
  const int64_t last = t_b - 1;
  EmRaw<J> ring[PF];
  double mr[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const int64_t tl = t_a + q < last ? t_a + q : last;
    bem_load<J, VEC>(p, tl, j0, ring[q]);
    if constexpr (OUT && !MLDS) mr[q] = p.m[tl * p.ldm];
  }
  auto body = [&](int q, int64_t t, bool refill) {
    float e[J];
    order_after(ring[q].ph, st.q0[0]);
    em_exp<J, VEC == 2>(p, j0, ring[q], e);
    double mt = 0.0;
    if constexpr (OUT && MLDS) mt = sm[t - t_a];
    if constexpr (OUT && !MLDS) mt = mr[q];
    slot_consumed<J>(e);
    if (refill) {
      const int64_t tl = t + PF < last ? t + PF : last;
      bem_load<J, VEC>(p, tl, j0, ring[q]);
      if constexpr (OUT && !MLDS) mr[q] = p.m[tl * p.ldm];
    }
    const float S = st.step(p, j0, invz, e);
    if constexpr (OUT) {
      float* arow = p.alpha + t * 2 * (int64_t)p.L;
      float a0[J];
#pragma unroll
      for (int j = 0; j < J; ++j) a0[j] = st.q0[j] * st.iS;
      bstore_row_n<J, VEC, (J <= 8 ? PMG_ALPHA_AUX : 0)>(arow, p.a0_bytes, j0, a0);
      if constexpr (A1) {   // alpha's d = 1 row, as the backward rebuilds it
        float a1[J];
#pragma unroll
        for (int j = 0; j < J; ++j) a1[j] = (st.jmp * st.ep[j]) * st.iS;
        bstore_row_n<J, VEC>(arow + p.L, p.a1_bytes, j0, a1);
      }
      bstore_pair_lane0(p.jsc, t, st.jmp, st.iS);
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

// The relaxation's output steps take the row references m_t from wave-local LDS, filled
// per piece of <= kMPiece steps before the piece's step loop: there a plain global load of
// m in the loop rotated through registers that the back-edge copied into the ring after a
// vmcnt(0), i.e. behind every store of the ring cycle (profiles/r05_ab_experiments.txt
// item 11).  The main passes keep the register ring, whose loops have no such drain and
// whose waits the LDS form would tighten.
#ifndef PMG_RELAX_MLDS
#define PMG_RELAX_MLDS true
#endif
constexpr int kMPiece = 512;
template <int J, int WP, int PF, int VEC, bool OUT, bool A1 = true, bool MLDS = false, int NW>
__device__ __forceinline__ double fwd_stream(const FBParams& p, Fwd<J, WP, NW>& st, int j0, const float invz[J],
                                             int64_t t_a, int64_t t_b) {
  if constexpr (OUT && MLDS) {
    // one copy per wave (each wave of a chain fills its own): no barrier, only the waits
    __shared__ double sm_all[NW * kMPiece];
    double* sm = sm_all + (threadIdx.x >> 6) * kMPiece;
    const int lane = threadIdx.x & 63;
    double logz = 0.0;
    for (int64_t ta = t_a; ta < t_b; ta += kMPiece) {
      const int64_t tz = ta + kMPiece < t_b ? ta + kMPiece : t_b;
      for (int64_t t = ta + lane; t < tz; t += 64) sm[t - ta] = p.m[t * p.ldm];
      __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) lgkmcnt(0): the piece's m is in LDS
      logz += fwd_stream_piece<J, WP, PF, VEC, OUT, A1, true, NW>(p, st, j0, invz, ta, tz, sm);
    }
    return logz;
  }
  return fwd_stream_piece<J, WP, PF, VEC, OUT, A1, false, NW>(p, st, j0, invz, t_a, t_b, nullptr);
}

#define PMG_FB_LANE_SETUP                                               \
  const int lane = threadIdx.x & 63;                                    \
  const int j0 = (int)threadIdx.x * J;  /* wave w of a chain: lanes 64 w .. */ \
  float invz[J];                                                        \
  _Pragma("unroll") for (int j = 0; j < J; ++j) invz[j] = (j0 + j < p.L) ? p.invz[j0 + j] : 0.f;

// speculative pass: chunk c starts `B` steps early from a uniform guess
template <int J, int WP, int VEC, bool A1, int NW = 1>
__device__ __forceinline__ void forward_chunk(const FBParams& p, int c, int j0, const float invz[J]) {
  const size_t SZ = (size_t)2 * p.Lpad;
  const int64_t t_c = (int64_t)c * p.C;
  const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
  Fwd<J, WP, NW> st;
  int64_t t0 = (c == 0) ? 0 : t_c - main_warmup(p);
  if (t0 < 0) t0 = 0;
  st.init_uniform(p, j0);
  fwd_stream<J, WP, kPfFwd, VEC, false>(p, st, j0, invz, t0, t_c);
  if (c > 0) st.save_state(p, p.s_in + (size_t)c * SZ, j0);  // the start k_verify checks
  // the row references m_t from LDS (filled once per chunk), as in the relaxation: a
  // register ring of them makes hipcc rotate it on the loop's back edge behind a vmcnt(0)
  const double lz = fwd_stream<J, WP, kPfFwd, VEC, true, A1, true>(p, st, j0, invz, t_c, t_e);
  st.save_state(p, p.s_out + (size_t)c * SZ, j0);
  if (threadIdx.x == 0) p.chunk_logz[c] = lz;
}

// the main pass clears the per-call words (the relaxation kernels run after it)
__device__ __forceinline__ void main_pass_reset(const FBParams& p) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.ctl[kCtlRepairs] = 0;
    p.ctl[kCtlRounds] = 0;
  }
}

// NW waves per chain (workgroup of 64 NW threads): J latents per lane, Lpad = 64 NW J
template <int J, int WP, int NW = 1>
__global__ void __launch_bounds__(64 * NW) k_forward(FBParams p_arg) {
  const FBParams p = batch_view(p_arg);
  const int c = blockIdx.x;
  if (c >= p.M) return;
  main_pass_reset(p);
  PMG_FB_LANE_SETUP
  (void)lane;
  const bool a1 = p.a1_bytes != 0;   // decode passes store alpha's d = 1 rows, EM passes do not
  if constexpr (J % 4 == 0) {
    if ((p.L & 3) == 0) {
      // VEC 2: L == Lpad, no lane-validity selects in the step loops (the EM shapes)
      if (a1) forward_chunk<J, WP, 1, true, NW>(p, c, j0, invz);
      else if (p.L == p.Lpad) forward_chunk<J, WP, 2, false, NW>(p, c, j0, invz);
      else forward_chunk<J, WP, 1, false, NW>(p, c, j0, invz);
      return;
    }
  }
  if (a1) forward_chunk<J, WP, false, true, NW>(p, c, j0, invz);
  else forward_chunk<J, WP, false, false, NW>(p, c, j0, invz);
}

// ---------------------------------------------------------------------------
// relaxation-kernel plumbing
// ---------------------------------------------------------------------------
// Grid barrier of the S co-resident single-wave workgroups (a monotone arrival
// counter): drain this wave's stores, agent-scope release, arrive, relaxed poll,
// agent-scope acquire.  The spin is bounded (kSpinTicks of the real-time clock, or
// another wave's timeout): on expiry the timeout word is set and false returned.
__device__ __forceinline__ bool relax_barrier(int* ctl, int target, uint64_t spin) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ok = 1;
  if ((threadIdx.x & 63) == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctl + kCtlArrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(ctl + kCtlArrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__hip_atomic_load(ctl + kCtlErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
          __builtin_amdgcn_s_memrealtime() - t0 > spin) {
        __hip_atomic_store(ctl + kCtlErr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  return __builtin_amdgcn_readfirstlane(ok) != 0;
}

// After the rounds: the last wave to leave clears the relaxation words for the next
// call (every wave has finished polling them before it counts its exit).
__device__ __forceinline__ void relax_exit(const FBParams& p) {
  if ((threadIdx.x & 63) == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const int old = __hip_atomic_fetch_add(p.ctl + kCtlExit, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == p.S - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (int w = kCtlPending; w <= kCtlExit; ++w)
        __hip_atomic_store(p.ctl + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ int ctl_load(int* ctl, int w) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Per-round change counters rotate over 3 slots: round k counts into slot k % 3 and
// every wave reads it after barrier k (so all take the same exit decision); wave 0
// zeroes slot (k+1) % 3 during round k -- its last readers passed barrier k-1, its
// next writers start after barrier k.
__device__ __forceinline__ void relax_publish(const FBParams& p, int k, int s, bool changed) {
  if ((threadIdx.x & 63) == 0) {
    p.seg_chg[(k & 1) * p.S + s] = changed ? 1 : 0;
    if (changed) __hip_atomic_fetch_add(p.ctl + kCtlChanged + k % 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 0) __hip_atomic_store(p.ctl + kCtlChanged + (k + 1) % 3, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// first (lowest, DIR > 0) or last (highest, DIR < 0) flagged index in [lo, hi), or -1
template <int DIR>
__device__ __forceinline__ int find_flag(const int* flags, int lo, int hi) {
  const int lane = threadIdx.x & 63;
  if constexpr (DIR > 0) {
    for (int base = lo; base < hi; base += 64) {
      const int idx = base + lane;
      const unsigned long long bal = __ballot(idx < hi && flags[idx] != 0);
      if (bal) return base + (int)__builtin_ctzll(bal);
    }
  } else {
    for (int top = hi - 1; top >= lo; top -= 64) {
      const int idx = top - lane;
      const unsigned long long bal = __ballot(idx >= lo && flags[idx] != 0);
      if (bal) return top - (int)__builtin_ctzll(bal);
    }
  }
  return -1;
}

// f64 sum of x[0..n) in one fixed order (lane-strided partials, then the wave butterfly)
// The loads of 8 strides are issued before their adds (same summation order): the
// plain loop waited one memory round trip per stride (~8 us for M = 2048 at C3).
__device__ __forceinline__ double wave_sum_fixed(const double* x, int n) {
  const int lane = threadIdx.x & 63;
  double a = 0.0;
  int i = lane;
  for (; i + 7 * 64 < n; i += 8 * 64) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = x[i + 64 * q];
#pragma unroll
    for (int q = 0; q < 8; ++q) a += v[q];
  }
  for (; i < n; i += 64) a += x[i];
  return wave_sum_f64(a);
}

// ---------------------------------------------------------------------------
// forward relaxation
// ---------------------------------------------------------------------------
// recompute chunks c0 .. b-1 from st (the filter state at c0*C - 1).  After chunk c,
// if its new end state is within tol of the old s_out[c] and boundary c+1 is not
// flagged (flg, round 0 only), the chunks up to the next flagged boundary are
// consistent: stop (*stop = c).  Returns true iff the segment's end state (chunk b-1)
// moved.
template <int J, int WP, int VEC, bool A1 = true>
__device__ __forceinline__ bool fwd_segment(const FBParams& p, Fwd<J, WP>& st, int c0, int b, int j0, const float invz[J],
                            const int* flg, int& nrep, int* stop = nullptr) {
  const size_t SZ = (size_t)2 * p.Lpad;
  for (int c = c0; c < b; ++c) {
    const int64_t t_c = (int64_t)c * p.C;
    const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
    st.save_state(p, p.s_in + (size_t)c * SZ, j0);
    const double lz = fwd_stream<J, WP, pf_relax_fwd<J>(), VEC, true, A1, PMG_RELAX_MLDS>(p, st, j0, invz, t_c, t_e);
    if ((threadIdx.x & 63) == 0) p.chunk_logz[c] = lz;
    ++nrep;
    float* so = p.s_out + (size_t)c * SZ;
    float x1[J];  // the d = 1 part on the d = 0 part's scale (the metric is scale-free)
#pragma unroll
    for (int j = 0; j < J; ++j) x1[j] = st.jmp * st.ep[j];
    const float d = hilbert_reg<J>(st.q0, x1, so, p.Lpad, j0);  // each lane reads only its own slots
    st.save_state(p, so, j0);
    if (d <= p.tol && (c + 1 >= b || !(flg && flg[c + 1]))) {
      if (stop) *stop = c;
      return false;
    }
  }
  return true;
}

template <int J, int WP, int VEC, bool A1 = true>
__device__ __forceinline__ void forward_relax(const FBParams& p, int j0, const float invz[J]) {
  const size_t SZ = (size_t)2 * p.Lpad;
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int a = s * p.G;
  const int b = a + p.G < p.M ? a + p.G : p.M;
  int nrep = 0, rounds = 0;
  const int pending = ctl_load(p.ctl, kCtlPending);
  if (pending > 0) {
    Fwd<J, WP> st;
    bool changed = false;
    // round 0: every boundary the verification flagged (it stored the carry into s_in),
    // in order; a pass that settles before the segment end resumes at the next flag
    int c0 = find_flag<1>(p.flags, a > 1 ? a : 1, b);
    while (c0 >= 0) {
      st.load_state(p, p.s_in + (size_t)c0 * SZ, j0);
      int stop = b;
      changed = fwd_segment<J, WP, VEC, A1>(p, st, c0, b, j0, invz, p.flags, nrep, &stop);
      if (changed) break;                                  // ran through to the segment end
      c0 = stop + 2 < b ? find_flag<1>(p.flags, stop + 2, b) : -1;
    }
    for (int k = 0;; ++k) {
      if (changed) st.save_state(p, p.seg_end + ((size_t)(k & 1) * p.S + s) * SZ, j0);
      relax_publish(p, k, s, changed);
      ++rounds;
      if (!relax_barrier(p.ctl, (k + 1) * p.S, p.spin)) break;
      if (ctl_load(p.ctl, kCtlChanged + k % 3) == 0) break;  // no segment end moved: all verified
      // round k+1: re-verify the first boundary against the left neighbour's new end state
      changed = false;
      if (s > 0 && p.seg_chg[(k & 1) * p.S + s - 1]) {
        const float* X = p.seg_end + ((size_t)(k & 1) * p.S + s - 1) * SZ;
        const float d = hilbert_dist(X, p.s_in + (size_t)a * SZ, (int)SZ);
        if (!(d <= p.tol)) {
          st.load_state(p, X, j0);
          changed = fwd_segment<J, WP, VEC, A1>(p, st, a, b, j0, invz, nullptr, nrep);
        }
      }
    }
    relax_exit(p);
  }
  if (lane == 0 && nrep) atomicAdd(p.ctl + kCtlRepairs, nrep);
  if (s == 0) {  // after the last barrier's acquire (or with no repair at all)
    const double lz = wave_sum_fixed(p.chunk_logz, p.M);
    if (lane == 0) {
      p.logz[0] = lz;
      p.ctl[kCtlRounds] = rounds;
      relax_warm_decision(p, pending);
    }
  }
}

template <int J, int WP>
__global__ void __launch_bounds__(64) k_forward_relax(FBParams p_arg) {
  const FBParams p = batch_view(p_arg);
  PMG_FB_LANE_SETUP
  (void)lane;
  if constexpr (J % 4 == 0) {
    if ((p.L & 3) == 0) {
      // the EM passes store no d = 1 rows of alpha (a1_bytes = 0): no a1 row formed either
      if (p.a1_bytes == 0) {
        if (p.L == p.Lpad) forward_relax<J, WP, 2, false>(p, j0, invz);
        else forward_relax<J, WP, 1, false>(p, j0, invz);
      } else {
        forward_relax<J, WP, 1>(p, j0, invz);
      }
      return;
    }
  }
  forward_relax<J, WP, false>(p, j0, invz);
}

// ---------------------------------------------------------------------------
// backward (beta recursion).  Every step back uses the same arithmetic
//   v = e_t * beta_t / sum(e_t * beta_t),  beta_{t-1} = Trans(v)
// on the warm-up and on the output path, so two chunks that have converged to
// the same beta produce bit-identical continuations (as the forward does).
// ---------------------------------------------------------------------------
template <int J, int WP, int NW = 1>
struct Bwd {
  static constexpr int NL = (WP + J - 1) / J;
  float b0[J], b1[J];  // beta at the current time
  ChainX<NW, J> x;
  float hl[NW > 1 ? NL * J : 1], hr[NW > 1 ? NL * J : 1];  // this step's halo of e * beta0 (NW > 1)

  __device__ void init_ones(const FBParams& p, int j0) {
    x.init();
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
  // the step's chain-wide sums (V0, V1 and, G != null, the output pass's G) and, NW > 1,
  // the halo of eb0 for step_back's band convolution: one LDS exchange per step
  __device__ __forceinline__ void sums(const float eb0[J], float& V0, float& V1, float* G) {
    if (G) {
      wave_sum2(V0, V1);
      *G = wave_sum(*G);
    } else {
      wave_sum2(V0, V1);
    }
    if constexpr (NW > 1) {
      if (G) {
        float t[3] = {V0, V1, *G};
        x.template exchange<NL, 3>(eb0, hl, hr, t);
        V0 = t[0];
        V1 = t[1];
        *G = t[2];
      } else {
        float t[2] = {V0, V1};
        x.template exchange<NL, 2>(eb0, hl, hr, t);
        V0 = t[0];
        V1 = t[1];
      }
    }
  }
  // beta <- Trans(v), v = e*beta / (V0+V1), given eb0 = e*b0 and eb1 = e*b1 (V0, V1
  // their chain sums, from sums()): the scale 1/(V0+V1) rides on the scalar coefficients.
  // KEEP_V: also return v (the joint partner rho of the decode / relaxation passes).
  // Lanes past L get beta != 0 but every consumer weights beta by e or alpha, which are
  // 0 there.
  template <bool KEEP_V>
  __device__ void step_back(const FBParams& p, const float invz[J], const float eb0[J], const float eb1[J],
                            float V0, float V1, float v0[J], float v1[J]) {
    const float sc = rcp_nr(V0 + V1);
    if constexpr (KEEP_V) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        v0[j] = eb0[j] * sc;
        v1[j] = eb1[j] * sc;
      }
    }
    float w0[J];
    if constexpr (NW > 1) band_conv<J, WP, NW>(p, eb0, w0, hl, hr);
    else band_conv<J, WP>(p, eb0, w0);
    const float w1 = V1 * sc * p.invL;
    const float a00 = p.A00 * sc, a10 = p.A10 * sc, c01 = p.A01 * w1, c11 = p.A11 * w1;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const float c0 = w0[j] * invz[j];
      b0[j] = fmaf(a00, c0, c01);
      b1[j] = fmaf(a10, c0, c11);
    }
  }
};

// eb = e * beta per dynamics state and their (lane-local) sums
template <int J, int WP, int NW>
__device__ __forceinline__ void e_beta(const Bwd<J, WP, NW>& st, const float e[J], float eb0[J], float eb1[J], float& V0,
                                       float& V1) {
  V0 = 0.f;
  V1 = 0.f;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    eb0[j] = e[j] * st.b0[j];
    eb1[j] = e[j] * st.b1[j];
    V0 += eb0[j];
    V1 += eb1[j];
  }
}

// one plain backward step at time t (beta_t -> beta_{t-1}); v kept in (v0, v1)
template <int J, int WP, int NW>
__device__ __forceinline__ void bwd_plain(const FBParams& p, Bwd<J, WP, NW>& st, int j0, const float invz[J],
                                          int64_t t, float v0[J], float v1[J]) {
  EmRaw<J> r;
  em_load<J>(p, t, j0, r);
  float e[J], eb0[J], eb1[J], V0, V1;
  em_exp<J>(p, j0, r, e);
  e_beta(st, e, eb0, eb1, V0, V1);
  st.sums(eb0, V0, V1, nullptr);
  st.template step_back<true>(p, invz, eb0, eb1, V0, V1, v0, v1);
}

// plain steps t = t_hi .. t_lo (descending), emission rows PF steps ahead
template <int J, int WP, int PF, int VEC, int NW>
__device__ __forceinline__ void bwd_stream_warm(const FBParams& p, Bwd<J, WP, NW>& st, int j0, const float invz[J],
                                                int64_t t_hi, int64_t t_lo) {
  if (t_hi < t_lo) return;
  EmRaw<J> ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) bem_load<J, VEC>(p, t_hi - q > t_lo ? t_hi - q : t_lo, j0, ring[q]);
  auto body = [&](int q, int64_t t, bool refill) {
    float e[J];
    order_after(ring[q].ph, st.b0[0]);
    em_exp<J, VEC == 2>(p, j0, ring[q], e);
    slot_consumed<J>(e);
    if (refill) bem_load<J, VEC>(p, t - PF > t_lo ? t - PF : t_lo, j0, ring[q]);
    float eb0[J], eb1[J], V0, V1;
    e_beta(st, e, eb0, eb1, V0, V1);
    st.sums(eb0, V0, V1, nullptr);
    st.template step_back<false>(p, invz, eb0, eb1, V0, V1, nullptr, nullptr);
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

typedef float f2v_t __attribute__((ext_vector_type(2)));
template <int J>
struct BRow {
  EmRaw<J> em;
  RowV<J> a0;
  f2v_t jj;  // the forward's (jump, 1/S) of this step
};

template <int J, int VEC>
__device__ __forceinline__ void brow_load(const FBParams& p, int64_t t, int j0, BRow<J>& r) {
  bem_load<J, VEC>(p, t, j0, r.em);
  bload_row<J, VEC>(p.alpha_in + t * 2 * (int64_t)p.L, p.L, j0, r.a0);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(p.jsc + 2 * t, 8u);
  r.jj = __builtin_bit_cast(f2v_t, __builtin_amdgcn_raw_buffer_load_b64(rs, 0, 0, 0));
}

// alpha_t's d = 1 row as the forward formed it: (jump * e) * (1/S)
template <int J>
__device__ __forceinline__ void alpha1_row(float js, float ji, const float e[J], float a1[J]) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    a1[j] = js * e[j];
    a1[j] *= ji;
  }
}

// the boundary weights of chunk c: alpha at its first step t_c, (2, Lpad) layout
template <int J, int VEC>
__device__ __forceinline__ void store_weights(const FBParams& p, int64_t t_c, int j0, float* dst) {
  BRow<J> r;
  brow_load<J, VEC>(p, t_c, j0, r);
  float e[J], a1[J];
  em_exp<J, VEC == 2>(p, j0, r.em, e);
  alpha1_row<J>(r.jj.x, r.jj.y, e, a1);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    dst[j0 + j] = r.a0[j];
    dst[p.Lpad + j0 + j] = a1[j];
  }
}

// output steps t = t_e-1 .. t_c; on entry st = beta_{t_e-1} and (vp0, vp1) the v that
// produced it (has_prev false at the sequence end), on exit beta_{t_c}.
// MODE 0 (EM): P only.  MODE 1: P / gamma / rho as given (decode, relaxation).
template <int J, int WP, int PF, int VEC, int MODE, int NW>
__device__ __forceinline__ void bwd_stream_out(const FBParams& p, Bwd<J, WP, NW>& st, int j0, const float invz[J],
                                               int64_t t_c, int64_t t_e, float vp0[J], float vp1[J],
                                               bool has_prev) {
  if (t_e - 1 < t_c) return;
  const int64_t L = p.L;
  BRow<J> ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) brow_load<J, VEC>(p, t_e - 1 - q > t_c ? t_e - 1 - q : t_c, j0, ring[q]);
  auto body = [&](int q, int64_t t, bool refill) {
    float a0[J], a1[J], e[J], eb0[J], eb1[J], pp[J], V0, V1;
    order_after(ring[q].em.ph, st.b0[0]);
    em_exp<J, VEC == 2>(p, j0, ring[q].em, e);
#pragma unroll
    for (int j = 0; j < J; ++j) a0[j] = ring[q].a0[j];
    const float js = ring[q].jj.x, ji = ring[q].jj.y;
    e_beta(st, e, eb0, eb1, V0, V1);
    float G = 0.f;
    if constexpr (MODE == 0) {
      // gamma_t summed over d, unnormalised: alpha0 beta0 + (js ji) e beta1
      const float jj = js * ji;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        pp[j] = fmaf(a0[j], st.b0[j], jj * eb1[j]);
        G += pp[j];
      }
      slot_consumed<J>(pp);
      slot_consumed<J>(eb0);
    } else {
      alpha1_row<J>(js, ji, e, a1);
#pragma unroll
      for (int j = 0; j < J; ++j) {
        a0[j] *= st.b0[j];
        a1[j] *= st.b1[j];
        G += a0[j] + a1[j];
      }
      slot_consumed<J>(a0);
      slot_consumed<J>(a1);
      slot_consumed<J>(eb0);
    }
    if (refill) brow_load<J, VEC>(p, t - PF > t_c ? t - PF : t_c, j0, ring[q]);
    st.sums(eb0, V0, V1, &G);
    const float iG = rcp_nr(G);
    if constexpr (MODE == 0) {
#pragma unroll
      for (int j = 0; j < J; ++j) pp[j] *= iG;
      if constexpr (VEC == 2) {   // dispatched only without planes: no branch in the step loop
        bstore_row<J, VEC>(p.P + t * p.ldd, p.L, j0, pp);
      } else {
        if (p.Pq) bstore_planes<J, VEC>(p, t, j0, pp);
        else bstore_row<J, VEC>(p.P + t * p.ldd, p.L, j0, pp);
      }
    } else {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        a0[j] *= iG;
        a1[j] *= iG;
        pp[j] = a0[j] + a1[j];
      }
      if (p.P) bstore_row<J, VEC>(p.P + t * p.ldd, p.L, j0, pp);
      if (p.Pq) bstore_planes<J, VEC>(p, t, j0, pp);
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
      st.template step_back<MODE != 0>(p, invz, eb0, eb1, V0, V1, vp0, vp1);
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

// speculative pass: beta guess (ones) `B` steps after the chunk, warmed up backwards
template <int J, int WP, int VEC, int MODE, int NW = 1>
__device__ __forceinline__ void backward_chunk(const FBParams& p, int c, int j0, const float invz[J]) {
  const size_t SZ = (size_t)2 * p.Lpad;
  const int64_t t_c = (int64_t)c * p.C;
  const int64_t t_e = t_c + p.C < p.T ? t_c + p.C : p.T;
  Bwd<J, WP, NW> st;
  float vp0[J], vp1[J];
#pragma unroll
  for (int j = 0; j < J; ++j) vp0[j] = vp1[j] = 0.f;
  bool has_prev = false;
  st.init_ones(p, j0);
  if (c < p.M - 1) {
    int64_t t_w = t_e + main_warmup(p);  // beta guess (ones) at t_w, exact when t_w is the last bin
    if (t_w > p.T - 1) t_w = p.T - 1;
    bwd_stream_warm<J, WP, kPfBwdWarm, VEC>(p, st, j0, invz, t_w, t_e + 1);
    st.save_state(p, p.b_in + (size_t)c * SZ, j0);  // beta_{t_e}: the start k_verify checks
    bwd_plain(p, st, j0, invz, t_e, vp0, vp1);       // -> beta_{t_e-1}
    has_prev = true;
  }
  bwd_stream_out<J, WP, kPfBwdOut, VEC, MODE>(p, st, j0, invz, t_c, t_e, vp0, vp1, has_prev);
  st.save_state(p, p.b_first + (size_t)c * SZ, j0);
  store_weights<J, VEC>(p, t_c, j0, p.w_first + (size_t)c * SZ);
}

#define PMG_BWD_DISPATCH(MODE)                                          \
  if constexpr (J % 4 == 0) {                                           \
    if ((p.L & 3) == 0) {                                               \
      if (MODE == 0 && p.L == p.Lpad && !p.Pq)                          \
        backward_chunk<J, WP, 2, MODE, NW>(p, c, j0, invz);             \
      else                                                              \
        backward_chunk<J, WP, 1, MODE, NW>(p, c, j0, invz);             \
      return;                                                           \
    }                                                                   \
  }                                                                     \
  backward_chunk<J, WP, false, MODE, NW>(p, c, j0, invz);

// speculative pass, EM outputs (P only); NW waves per chain as k_forward
template <int J, int WP, int NW = 1>
__global__ void __launch_bounds__(64 * NW) k_backward(FBParams p_arg) {
  const FBParams p = batch_view(p_arg);
  const int c = blockIdx.x;
  if (c >= p.M) return;
  main_pass_reset(p);
  PMG_FB_LANE_SETUP
  (void)lane;
  PMG_BWD_DISPATCH(0)
}

// speculative pass, decode outputs (P / gamma / rho as given)
template <int J, int WP, int NW = 1>
__global__ void __launch_bounds__(64 * NW) k_backward_full(FBParams p_arg) {
  const FBParams p = batch_view(p_arg);
  const int c = blockIdx.x;
  if (c >= p.M) return;
  main_pass_reset(p);
  PMG_FB_LANE_SETUP
  (void)lane;
  PMG_BWD_DISPATCH(1)
}

// ---------------------------------------------------------------------------
// backward relaxation (chunks in descending order; a segment's "left" neighbour in
// the data flow is the segment above it)
// ---------------------------------------------------------------------------
// recompute chunks c0, c0-1, .., a from st (beta at (c0+1)*C).  After chunk c, if its
// new beta at c*C is within tol of the old b_first[c] (weighted by alpha at c*C, the
// boundary metric of k_verify) and boundary c-1 is not flagged, stop.  Returns true
// iff the segment's end state (b_first[a]) moved; otherwise *stop = the chunk it
// settled at.
template <int J, int WP, int VEC, int MODE = 1>
__device__ __forceinline__ bool bwd_segment(const FBParams& p, Bwd<J, WP>& st, int c0, int a, int j0, const float invz[J],
                            const int* flg, int& nrep, int* stop = nullptr) {
  const size_t SZ = (size_t)2 * p.Lpad;
  for (int c = c0; c >= a; --c) {
    const int64_t t_c = (int64_t)c * p.C;
    const int64_t t_e = t_c + p.C;  // c <= M-2: a whole chunk with a successor
    st.save_state(p, p.b_in + (size_t)c * SZ, j0);
    float vp0[J], vp1[J];
    bwd_plain(p, st, j0, invz, t_e, vp0, vp1);
    bwd_stream_out<J, WP, pf_relax_bwd<J>(), VEC, MODE>(p, st, j0, invz, t_c, t_e, vp0, vp1, true);
    ++nrep;
    float* bf = p.b_first + (size_t)c * SZ;
    const float d = hilbert_reg<J>(st.b0, st.b1, bf, p.Lpad, j0, p.w_first + (size_t)c * SZ, p.Lpad);
    st.save_state(p, bf, j0);
    if (d <= p.tol && (c == a || !(flg && flg[c - 1]))) {
      if (stop) *stop = c;
      return false;
    }
  }
  return true;
}

template <int J, int WP, int VEC, int MODE = 1>
__device__ __forceinline__ void backward_relax(const FBParams& p, int j0, const float invz[J]) {
  const size_t SZ = (size_t)2 * p.Lpad;
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int a = s * p.G;
  const int b = a + p.G < p.M ? a + p.G : p.M;
  const int top = b < p.M - 1 ? b : p.M - 1;  // boundaries c <= M-2 have a successor
  int nrep = 0, rounds = 0;
  const int pending = ctl_load(p.ctl, kCtlPending);
  if (pending > 0) {
    Bwd<J, WP> st;
    bool changed = false;
    // round 0: every flagged boundary, top down (see forward_relax)
    int c0 = find_flag<-1>(p.flags, a, top);
    while (c0 >= 0) {
      st.load_state(p, p.b_in + (size_t)c0 * SZ, j0);
      int stop = a;
      changed = bwd_segment<J, WP, VEC, MODE>(p, st, c0, a, j0, invz, p.flags, nrep, &stop);
      if (changed) break;
      c0 = stop - 1 > a ? find_flag<-1>(p.flags, a, stop - 1) : -1;
    }
    for (int k = 0;; ++k) {
      if (changed) st.save_state(p, p.seg_end + ((size_t)(k & 1) * p.S + s) * SZ, j0);
      relax_publish(p, k, s, changed);
      ++rounds;
      if (!relax_barrier(p.ctl, (k + 1) * p.S, p.spin)) break;
      if (ctl_load(p.ctl, kCtlChanged + k % 3) == 0) break;
      changed = false;
      if (s + 1 < p.S && p.seg_chg[(k & 1) * p.S + s + 1]) {
        const float* X = p.seg_end + ((size_t)(k & 1) * p.S + s + 1) * SZ;
        const float* w = p.w_first + (size_t)b * SZ;
        const float d = hilbert_dist(p.b_in + (size_t)(b - 1) * SZ, X, (int)SZ, w);
        if (!(d <= p.tol)) {
          st.load_state(p, X, j0);
          changed = bwd_segment<J, WP, VEC, MODE>(p, st, b - 1, a, j0, invz, nullptr, nrep);
        }
      }
    }
    relax_exit(p);
  }
  if (lane == 0) {
    if (nrep) atomicAdd(p.ctl + kCtlRepairs, nrep);
    if (s == 0) {
      p.ctl[kCtlRounds] = rounds;
      relax_warm_decision(p, pending);
    }
  }
}

template <int J, int WP>
__global__ void __launch_bounds__(64) k_backward_relax(FBParams p_arg) {
  const FBParams p = batch_view(p_arg);
  PMG_FB_LANE_SETUP
  (void)lane;
  if constexpr (J % 4 == 0) {
    if ((p.L & 3) == 0) {
      // EM passes (P only): the main pass's P arithmetic (MODE 0: P bit-identical to a
      // main pass from the same beta), no gamma / rho rows, no v kept
      if (!p.gamma && !p.rho) {
        if (p.L == p.Lpad && !p.Pq) backward_relax<J, WP, 2, 0>(p, j0, invz);
        else backward_relax<J, WP, 1, 0>(p, j0, invz);
      } else {
        backward_relax<J, WP, 1>(p, j0, invz);
      }
      return;
    }
  }
  backward_relax<J, WP, false>(p, j0, invz);
}

typedef void (*fb_kernel_t)(FBParams);

// the kernels of one (J, WP) instance (fb_inst_j*.hip); forward2 / backward2: the main
// passes with each chain on two waves of J / 2 latents per lane (same state layout,
// Lpad = 64 J), compiled for J = 8 and 16 (null elsewhere)
struct FBKernelSet {
  fb_kernel_t forward, forward_relax;
  fb_kernel_t backward, backward_full, backward_relax;
  fb_kernel_t forward2, backward2;
};

template <int J, int WP>
inline void fb_fill(FBKernelSet* k) {
  k->forward = k_forward<J, WP>;
  k->forward_relax = k_forward_relax<J, WP>;
  k->backward = k_backward<J, WP>;
  k->backward_full = k_backward_full<J, WP>;
  k->backward_relax = k_backward_relax<J, WP>;
  k->forward2 = nullptr;
  k->backward2 = nullptr;
  if constexpr (J == 8 || J == 16) {
    k->forward2 = k_forward<J / 2, WP, 2>;
    k->backward2 = k_backward<J / 2, WP, 2>;
  }
}

// one (J, WP) instance fb_set_j<J>_w<WP>, defined in the fb_inst_j*_w*.hip unit that lists it
#define PMG_FB_WPS(X, JJ) X(JJ, 5) X(JJ, 9) X(JJ, 13) X(JJ, 17) X(JJ, 25) X(JJ, 32)
#define PMG_FB_ALL(X) PMG_FB_WPS(X, 1) PMG_FB_WPS(X, 2) PMG_FB_WPS(X, 4) PMG_FB_WPS(X, 8) PMG_FB_WPS(X, 16)
#define PMG_FB_DECL(JJ, WPP) void fb_set_j##JJ##_w##WPP(FBKernelSet* k);
PMG_FB_ALL(PMG_FB_DECL)
#define PMG_FB_INST(JJ, WPP) \
  void fb_set_j##JJ##_w##WPP(FBKernelSet* k) { fb_fill<JJ, WPP>(k); }

}  // namespace pmg
