// Adam M-step for the Poisson tuning weights, one persistent launch on gfx950.
//
// Reference: fit_tuning_helper.make_adam_runner.run (fit_tuning_helper.py:133-194)
//   on poisson_m_step_objective (fit_tuning_helper.py:63-81):
//     f = softplus(B W)   (L,N)
//     loss = -sum[xlogy(y_w, f+1e-20) - f t_w] - sum norm.logpdf(W; 0, sd)
//     grad = -B^T[(y_w/(f+1e-20) - t_w) * sigmoid(B W)] + W/sd^2
//   optax 0.2.2 adam (b1 .9, b2 .999, eps 1e-8, eps_root 0), state carried across EM
//   iterations, and the while-loop stop rule
//     i < maxiter-1 and (i < 5 or |loss - loss_prev| / max(|loss|, 1e-8) > tol).
//
// MI355X design: the objective separates over neurons except for the scalar loss
// the stop rule reads.  Workgroups own disjoint neuron columns (one workgroup per
// CU, all co-resident), keep the basis in registers once (a 2-D block per thread,
// see "Basis layout" below), run Adam on their own columns in f64 and publish a
// f64 partial loss / squared gradient norm per iteration.  Instead of a grid
// barrier per iteration, every workgroup runs LAG iterations ahead and decides
// "stop after body j" from the globally summed partials of iteration j (summed in
// the same fixed order by every workgroup, hence identical decisions); a small
// ring of (W, mu, nu) states lets it return exactly the state after body j+1.
#include <stdio.h>
#include <stdlib.h>

#include "pmg_common.h"
#include "pmg_math64.h"

namespace pmg {

// In-loop workgroup barrier that waits only for LDS traffic (lgkmcnt), so the
// decision pipeline's global loads stay in flight across it (a __syncthreads()
// would drain vmcnt, cdna_hip_programming.md "Pipelining across barriers").
#define PMG_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

#ifndef PMG_ADAM_SP_OCML
#define PMG_ADAM_SP_OCML 0
#endif

constexpr int kLag = 4;                 // bodies a workgroup runs ahead of the decision
constexpr int kRing = kLag + 2;
constexpr int kSMax = 4;                // neurons per workgroup
constexpr int kThreads = 512;           // L <= 512
constexpr int kPartPerLane = 4;         // G <= 256 workgroups -> 4 partials per lane
constexpr int kBiasLds = 1024;          // bias corrections held in LDS (bodies)
constexpr int kXSlots = 512;            // exchange slots per workgroup (NB S <= 512 elements)
constexpr uint64_t kAdamSpinTicks = 200000000ull;   // 2 s of the 100 MHz real-time clock

struct AdamParams {
  double* W;
  double* mu;
  double* nu;
  int64_t* count;
  const float* basis;
  const double* yw;
  const double* tw;
  int L, NB, N, S, G, ng, LG;
  double lr, b1, b2, eps, eps_root, prior_std, tol;
  int maxiter;
  double* stats;
  double* loss_hist;
  double* err_hist;
  const double* bias;         // [2][maxiter] 1/(1 - b1^(count0+k+1)), 1/(1 - b2^(count0+k+1))
  unsigned long long* lpart;  // [maxiter + kLag + 2][G] f64 bits, pre-filled with kSentinel
  unsigned long long* gpart;  // [..][G]
  int* timeout;               // sticky: word 0 of the workspace, shared by all restarts,
                              // set by a bounded wait that gave up; read and cleared only
                              // by pmg_mstep_adam_status (never by a launch)
  uint64_t spin;              // bound of those waits (real-time clock ticks, spin_ticks)
  // row blocks (L > 512): workgroup g = rb Gg + gg owns rows [rb 32 A, (rb + 1) 32 A) of
  // neuron group gg; the RB row blocks of a group swap their B^T G partials every body
  int RB, Gg;
  float* xbuf;                // [2][G][kXSlots] partial B^T G (body parity)
  int* xflag;                 // [G][kNW] bodies published per wave (monotone, zeroed per launch)
  long long* prof;            // optional (PMG_ADAM_PROF): s_memtime stamps of WG 0, bodies < 64
  // batched restarts (blockIdx.y = restart r of this launch): per-restart strides of the
  // operands (elements) and of the restart's workspace slab (bytes)
  int64_t rs_W, rs_yw, rs_ws;
  int rs_tw, rs_hist;
};

// restart r's view of the parameters (identity for blockIdx.y = 0)
__device__ __forceinline__ AdamParams adam_view(const AdamParams& p0) {
  AdamParams p = p0;
  const int64_t r = blockIdx.y;
  if (r == 0) return p;
  p.W += r * p.rs_W;
  p.mu += r * p.rs_W;
  p.nu += r * p.rs_W;
  p.count += r;
  p.yw += r * p.rs_yw;
  p.tw += r * p.rs_tw;
  p.stats += 4 * r;
  p.loss_hist += r * p.rs_hist;
  p.err_hist += r * p.rs_hist;
  // byte offsets as pointer arithmetic (not integer round trips): the compiler keeps the
  // kernel arguments' global address space and emits global / buffer accesses, not flat
  // ones (a flat store also counts in lgkmcnt, so every LDS barrier would wait for it)
  const int64_t o = r * p.rs_ws;
  p.bias = reinterpret_cast<const double*>(reinterpret_cast<const char*>(p.bias) + o);
  p.lpart = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(p.lpart) + o);
  p.gpart = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(p.gpart) + o);
  p.prof = nullptr;
  return p;
}

#define PMG_ADAM_STAMP(k, i)                                                   \
  if (p.prof && g == 0 && tid == 0 && (k) < 64) p.prof[(k) * 16 + (i)] = __builtin_amdgcn_s_memtime();

// signalling NaN with a payload: no arithmetic result has this bit pattern
constexpr unsigned long long kSentinel = 0x7FF4DEADBEEF0001ull;

__device__ __forceinline__ void st_sc1(unsigned long long* p, double v) {
  __hip_atomic_store(p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_bits(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void load_parts(const AdamParams& p, int j, int lane,
                                           unsigned long long* lv) {
#pragma unroll
  for (int q = 0; q < kPartPerLane; ++q) {
    const int gi = lane + 64 * q;
    lv[q] = gi < p.G ? ld_bits(&p.lpart[(size_t)j * p.G + gi]) : 0ull;
  }
}

// the one summation order of a body's partials (decision, histories): lane-strided
// sums in q order, then the f64 butterfly of wave_sum_f64
__device__ __forceinline__ double sum_parts(const unsigned long long* lv) {
  double a = 0.0;
#pragma unroll
  for (int q = 0; q < kPartPerLane; ++q) a += __longlong_as_double((long long)lv[q]);
  return wave_sum_f64(a);
}

__global__ void k_fill_u64(unsigned long long* __restrict__ x, size_t n, unsigned long long v) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) x[i] = v;
}

// Launch prologue: sentinel-fill both partial arrays, zero the outputs the loop fills
// sparsely (histories, stats: no host memsets), and tabulate the bias
// corrections of every body from the Adam step count, c_k = 1 / (1 - b^(count0 + k + 1)).
// A closed form per body (not a running product) gives the same bits however the loop
// is split into launches (the speculative batches of the neuron-sharded M-step).
__global__ void k_adam_prologue(AdamParams p_arg, size_t n) {
  const AdamParams p = adam_view(p_arg);
  unsigned long long* __restrict__ lpart = p.lpart;
  unsigned long long* __restrict__ gpart = p.gpart;
  const int64_t* __restrict__ count = p.count;
  const double b1 = p.b1, b2 = p.b2;
  const int maxiter = p.maxiter > 1 ? p.maxiter : 1;
  double* __restrict__ bias = const_cast<double*>(p.bias);
  double* __restrict__ loss_hist = p.loss_hist;
  double* __restrict__ err_hist = p.err_hist;
  double* __restrict__ stats = p.stats;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t q = i; q < n; q += stride) {
    lpart[q] = kSentinel;
    gpart[q] = kSentinel;
  }
  const double c0 = (double)count[0];
  for (size_t k = i; k < (size_t)maxiter; k += stride) {
    bias[k] = 1.0 / (1.0 - pow(b1, c0 + (double)k + 1.0));
    bias[maxiter + k] = 1.0 / (1.0 - pow(b2, c0 + (double)k + 1.0));
    loss_hist[k] = 0.0;
    err_hist[k] = 0.0;
  }
  if (i < 4) stats[i] = 0.0;
  if (p.xflag)
    for (size_t q = i; q < (size_t)p.G * 8; q += stride) p.xflag[q] = 0;
}

// ---------------------------------------------------------------------------
// Basis layout: ONE register-resident copy, as a 2-D block per thread.  The 512 threads
// form 32 l-blocks (4 per wave: the 16-lane DPP rows) x 16 q-blocks (lane & 15); thread
// (lb, qb) holds B[lb*A + i, qb*BC + k] for i < A = Lp/32, k < BC = ceil(NB/16).
//   f = B W  : per-thread partial sums over its BC columns for its A rows, then a
//              16-lane DPP reduce-scatter (lane j gets row bitrev(j)): every row's F
//              ends on one lane, which evaluates softplus / sigmoid and G for it;
//   B^T G    : G of the block's rows is broadcast through wave-local LDS, each thread
//              forms its BC column partials over its A rows, lanes with the same q-block
//              are summed over the 4 DPP rows (shfl_xor 16, 32) and over the 8 waves
//              (LDS, fixed order) by the element-update threads.
// Everything but the G broadcast and the cross-wave sum stays in registers.
// ---------------------------------------------------------------------------
constexpr int kNW = kThreads / 64;          // waves
// The decision pipeline runs on wave kCtl before barrier 1: waves w and w + 4 share a
// SIMD and the older one (w < 4) is issued first, so it ends phases A+B ~1,500 ticks
// before its partner and waits at barrier 1 -- the decision fills that wait instead of
// holding barrier 2 open after the element update (round 4: the last wave, after it).
constexpr int kCtl = 3;
constexpr int kRefresh = 16;
typedef float f2v __attribute__((ext_vector_type(2)));   // row pairs: v_pk_fma_f32 operands

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// lower lanes of the pairing: a + partner(a); upper lanes: b + partner(b) (two fused
// DPP adds and one select: no select on the DPP source)
template <int CTRL, typename T>
__device__ __forceinline__ T pair_add(T a, T b, bool upper) {
  T sa, sb;
  if constexpr (sizeof(T) == 8) {
    sa = a + dpp_d<CTRL>(a);
    sb = b + dpp_d<CTRL>(b);
  } else {
    sa = a + dpp_f<CTRL>(a);
    sb = b + dpp_f<CTRL>(b);
  }
  return upper ? sb : sa;
}

// v + v(lane ^ 16), v + v(lane ^ 32): permlane swaps (VALU, no LDS round trip)
__device__ __forceinline__ float add_xor16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// 1/x in f64 from v_rcp_f64 and two Newton steps (x > 0, finite)
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  r = fma(r, fma(-x, r, 1.0), r);
  return r;
}
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_t(T v) {
  if constexpr (sizeof(T) == 8) return dpp_d<CTRL>(v);
  else return dpp_f<CTRL>(v);
}

// x[A] per lane -> sum over the 16 lanes of the DPP row of x[idx], idx = the lane's row
// slot (scatter_slot).  Four stages on lane bits 3, 2, 1, 0 (row_ror:8, row_half_mirror,
// quad_perm [2,3,0,1], quad_perm [1,0,3,2]): the first 4 - log2(A) are plain butterflies
// (lanes differing in those bits end with the same sums), each later one halves the
// vector, the lane keeping the even (lower lanes) or odd (upper lanes) entries, so the
// index bits are read from the lane bits in reverse order.
template <int A, typename T>
__device__ __forceinline__ T reduce_scatter16(T* x) {
  const int lane = threadIdx.x & 63;
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  if constexpr (A == 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = pair_add<0x128>(x[2 * i], x[2 * i + 1], b3);
  } else {
#pragma unroll
    for (int i = 0; i < A; ++i) x[i] = x[i] + dpp_t<0x128>(x[i]);
  }
  if constexpr (A >= 8) {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = pair_add<0x141>(x[2 * i], x[2 * i + 1], b2);
  } else {
#pragma unroll
    for (int i = 0; i < A; ++i) x[i] = x[i] + dpp_t<0x141>(x[i]);
  }
  if constexpr (A >= 4) {
#pragma unroll
    for (int i = 0; i < 2; ++i) x[i] = pair_add<0x4E>(x[2 * i], x[2 * i + 1], b1);
  } else {
#pragma unroll
    for (int i = 0; i < A; ++i) x[i] = x[i] + dpp_t<0x4E>(x[i]);
  }
  return pair_add<0xB1>(x[0], x[1], b0);
}

// the row slot of a lane after reduce_scatter16<A>: index bits from lane bits 3..(4-log2 A)
template <int A>
__device__ __forceinline__ int scatter_slot(int lane) {
  const int j = lane & 15;
  const int r4 = ((j & 1) << 3) | ((j & 2) << 1) | ((j & 4) >> 1) | ((j & 8) >> 3);   // bitrev4
  return A == 16 ? r4 : A == 8 ? (r4 >> 1) : (r4 >> 2);   // lanes j < A (j & 8 == 0 ...) own the slots
}

template <int A, int BC, int SP>
__global__ void __launch_bounds__(kThreads) k_adam(AdamParams p_arg) {
  const AdamParams p = adam_view(p_arg);
  constexpr int BCP = (BC + 3) & ~3;                                   // padded q-block (b128 reads)
  constexpr int QS = 16 * BCP;                                         // padded columns per neuron
  __shared__ __attribute__((aligned(16))) double sW[kSMax * QS];       // W_k (f64), [s][qb][BCP]
  __shared__ __attribute__((aligned(16))) float sD[kSMax * QS];        // W_k - W_{k-1}
  // G of every row, row pairs interleaved per neuron: [l/2][s][l&1], so one b64 / b128 read
  // of a pair is the (even row, odd row) operand of the packed FMAs with no register moves
  __shared__ __attribute__((aligned(16))) float sG[32 * A * SP];
  __shared__ float sPart[kNW * SP * 16 * BC];                          // per-wave B^T G, [w][s][q]
  __shared__ double sSum[2 * kNW];
  __shared__ int sCtl[4];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave index: uniform (SGPR)
  const bool ctl = wid == kCtl;                        // runs the decision pipeline
  const int g = blockIdx.x;
  const int rb = g / p.Gg, gg = g - rb * p.Gg;         // row block, neuron group
  const int r0 = rb * 32 * A;                          // first row of this workgroup
  const int n0 = gg * p.S;
  const int S = (p.N - n0) < p.S ? (p.N - n0) : p.S;  // neurons owned (<= SP)
  const int L = p.L, NB = p.NB;
  const double sd = p.prior_std, isd2 = 1.0 / (sd * sd);
  // the prior's normaliser, read from LDS in the update (a register held across the loop
  // is one the allocator would rather spill)
  __shared__ double sLconst;
  if (threadIdx.x == 0) sLconst = log(sd) + 0.5 * log(2.0 * M_PI);

  // ---- thread roles ------------------------------------------------------------
  const int lb = wid * 4 + (lane >> 4);                // l-block (rows lb*A ..)
  const int qb = lane & 15;                            // q-block (cols qb*BC ..)
  const int slot = scatter_slot<A>(lane);
  const int lrow = r0 + lb * A + slot;                 // the row this lane evaluates
  const bool owner = (lane & 15) < A;                  // one lane per row slot
  const bool is_row = owner && lrow < L;
  // element (q, s) of the Adam update
  const int eq = tid / SP, es = tid % SP;
  const bool is_el = eq < NB && es < S;

  // ---- one-time loads -------------------------------------------------------
  // the thread's basis block as row pairs (rows 2i, 2i+1): both contractions run on
  // packed FMAs (v_pk_fma_f32), two rows per instruction
  f2v bb[A / 2][BC];
#pragma unroll
  for (int i = 0; i < A / 2; ++i)
#pragma unroll
    for (int k = 0; k < BC; ++k) {
      const int l = r0 + lb * A + 2 * i, q = qb * BC + k;
      bb[i][k].x = (l < L && q < NB) ? p.basis[(size_t)l * NB + q] : 0.f;
      bb[i][k].y = (l + 1 < L && q < NB) ? p.basis[(size_t)(l + 1) * NB + q] : 0.f;
    }
  // per-thread constants and the running F of the lane's row live in LDS, not in
  // registers (each read once per slot per body): the kernel sits at the 256-VGPR cap
  // and every register spilled instead costs a scratch reload + vmcnt wait per body
  __shared__ double sYw[SP][kThreads];
  __shared__ double sTw[kThreads];
  __shared__ double sF[SP][kThreads];
  __shared__ __attribute__((aligned(16))) double sLog[kMathTab];      // softplus_tab's log + exp tables
  for (int q = tid; q < kLogTab + kExpTab; q += blockDim.x) math_tab_entry(q, sLog);
#pragma unroll
  for (int s = 0; s < SP; ++s) {
    sYw[s][tid] = (is_row && s < S) ? p.yw[(size_t)lrow * p.N + n0 + s] : 0.0;
    sF[s][tid] = 0.0;
  }
  sTw[tid] = is_row ? p.tw[lrow] : 0.0;
  for (int q = tid; q < kSMax * QS; q += blockDim.x) {
    sW[q] = 0.0;
    sD[q] = 0.f;
  }
  for (int q = tid; q < 32 * A * SP; q += blockDim.x) sG[q] = 0.f;
  if (tid < 4) sCtl[tid] = 0;
  // element state (W, mu, nu) of this thread's weight, and its ring of the last kRing
  // states in LDS (each slot written and read by its own thread: no barrier, no HBM)
  double w_cur = 0.0, mu_cur = 0.0, nu_cur = 0.0;
  constexpr int RS = 16 * BC * SP;                     // ring slab per state: NB <= 16 BC columns
  __shared__ double sRing[kRing * 3 * RS];
  const int e = eq * SP + es;
  const int ewo = es * QS + (eq / BC) * BCP + eq % BC; // this element's sW / sD slot
  __syncthreads();
  if (is_el) {
    const size_t o = (size_t)eq * p.N + n0 + es;
    w_cur = p.W[o];
    mu_cur = p.mu[o];
    nu_cur = p.nu[o];
    sW[ewo] = w_cur;
    sRing[(0 * 3 + 0) * RS + e] = w_cur;
    sRing[(0 * 3 + 1) * RS + e] = mu_cur;
    sRing[(0 * 3 + 2) * RS + e] = nu_cur;
  }
  const int64_t count0 = p.count[0];
  // the bias-correction table of the first kBiasLds bodies in LDS (uniform reads, no
  // memory wait inside the loop); later bodies read it from the workspace
  const int mi = p.maxiter > 1 ? p.maxiter : 1;
  __shared__ double sBias[2 * kBiasLds];
  const double* bias2 = p.bias + mi;
  for (int q = tid; q < kBiasLds && q < mi; q += blockDim.x) {
    sBias[q] = p.bias[q];
    sBias[kBiasLds + q] = p.bias[mi + q];
  }
  __syncthreads();

  // control-wave state
  double loss_prev = 0.0, loss0 = 0.0;
  int dj = 0;                              // next body to decide
  unsigned long long lv0[kPartPerLane];    // body dj loss partials (in flight)
  unsigned long long lv1[kPartPerLane];    // body dj+1
  bool issued0 = false, issued1 = false;
  double fin_loss = 0.0;
  const int maxiter = p.maxiter;
  const bool eval_only = maxiter <= 1;

  for (int k = 0;; ++k) {
    // ---- phase A: F = B W_k on the lane's row, softplus, loss, G -----------------
    PMG_ADAM_STAMP(k, 0)
    double lpart = 0.0;
    const bool exact = (k % kRefresh) == 0;
    // one neuron slot at a time (slots s >= S carry zeros and write G = 0); the
    // scheduling barrier keeps one slot's A-row partials live at a time
#pragma unroll
    for (int s = 0; s < SP; ++s) {
      double F;
      if (exact) {
        double x[A];
#pragma unroll
        for (int i = 0; i < A; ++i) x[i] = 0.0;
#pragma unroll
        for (int k4 = 0; k4 < BC; ++k4) {
          const double w = sW[s * QS + qb * BCP + k4];
#pragma unroll
          for (int i = 0; i < A / 2; ++i) {
            x[2 * i] = fma((double)bb[i][k4].x, w, x[2 * i]);
            x[2 * i + 1] = fma((double)bb[i][k4].y, w, x[2 * i + 1]);
          }
        }
        F = reduce_scatter16<A>(x);
      } else {
        float dw[BCP];
#pragma unroll
        for (int k4 = 0; k4 < BCP; k4 += 4) {
          const float4 v = *reinterpret_cast<const float4*>(&sD[s * QS + qb * BCP + k4]);
          dw[k4] = v.x;
          dw[k4 + 1] = v.y;
          dw[k4 + 2] = v.z;
          dw[k4 + 3] = v.w;
        }
        float x[A];
#pragma unroll
        for (int i = 0; i < A / 2; ++i) {
          f2v a = {0.f, 0.f};
#pragma unroll
          for (int k4 = 0; k4 < BC; ++k4) a = __builtin_elementwise_fma(bb[i][k4], (f2v){dw[k4], dw[k4]}, a);
          x[2 * i] = a.x;
          x[2 * i + 1] = a.y;
        }
        F = sF[s][tid] + (double)reduce_scatter16<A>(x);
      }
      sF[s][tid] = F;
      const double ywd = sYw[s][tid], twd = sTw[tid];
      // softplus / sigmoid in f32 at Fh = f32(F), corrected to first order in the
      // exact residual r = F - Fh (|r| <= 2^-24 |F|): f = softplus(Fh) + sigmoid(Fh) r
      const float Fh = (float)F;
      const double r = F - (double)Fh;
      const bool live = is_row && s < S;
#if PMG_ADAM_SP_OCML
      // round-3 form (A/B builds only): OCML log1pf / expf and a second f64 reciprocal
      const float f32 = fmaxf(Fh, 0.f) + log1pf(expf(-fabsf(Fh)));
      const float sg = 1.f / (1.f + expf(-Fh));
      const double fd = (double)f32 + (double)sg * r;
      const float gv = live ? (float)((ywd * rcp_nr(fd + 1e-20) - twd) * (double)sg) : 0.f;
      if (owner) sG[((lb * A + slot) >> 1) * 2 * SP + 2 * s + (slot & 1)] = gv;
      const double xl = (ywd != 0.0) ? ywd * ((double)logf(f32 + 1e-20f) + (double)sg * r * rcp_nr((double)f32)) : 0.0;
#else
      // softplus and its log to a few f64 ulps (pmg_math64.h, table log): the loss feeds
      // the stop rule, which compares consecutive losses to 1e-6 relative, so it must not
      // carry f32 rounding (a few-ulp f32 softplus moved a stop decision by one body).
      // The sigmoid (f32) only scales G = y_w / f - t_w, which cancels near the optimum
      // and so is formed in f64 before its f32 rounding.
      (void)Fh;
      (void)r;
      const SoftplusT sp = softplus_tab(F, sLog);
      const double fd = sp.f;
      const float gv = live ? (float)(ywd * rcp_nr(fd + 1e-20) - twd) * sp.sg : 0.f;
      if (owner) sG[((lb * A + slot) >> 1) * 2 * SP + 2 * s + (slot & 1)] = gv;
      const double xl = (ywd != 0.0) ? ywd * sp.logf : 0.0;
#endif
      lpart -= live ? xl - fd * twd : 0.0;
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- phase B: B^T G partials (G of the block from wave-local LDS) ---------------
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's G stores are visible
    // packed over row pairs: acc.x sums the even rows, acc.y the odd ones
    f2v gacc[SP][BC];
#pragma unroll
    for (int s = 0; s < SP; ++s)
#pragma unroll
      for (int k4 = 0; k4 < BC; ++k4) gacc[s][k4] = (f2v){0.f, 0.f};
#pragma unroll
    for (int i = 0; i < A / 2; ++i) {
      f2v gl[SP];                                      // (G[2i][s], G[2i+1][s])
      const float* src = &sG[(lb * A / 2 + i) * 2 * SP];
#pragma unroll
      for (int s = 0; s < SP; ++s) gl[s] = *reinterpret_cast<const f2v*>(src + 2 * s);
#pragma unroll
      for (int s = 0; s < SP; ++s)
#pragma unroll
        for (int k4 = 0; k4 < BC; ++k4) gacc[s][k4] = __builtin_elementwise_fma(bb[i][k4], gl[s], gacc[s][k4]);
    }
    float gp[SP][BC];
#pragma unroll
    for (int s = 0; s < SP; ++s)
#pragma unroll
      for (int k4 = 0; k4 < BC; ++k4) gp[s][k4] = gacc[s][k4].x + gacc[s][k4].y;
#pragma unroll
    for (int s = 0; s < SP; ++s)
#pragma unroll
      for (int k4 = 0; k4 < BC; ++k4) {
        gp[s][k4] = add_xor32(add_xor16(gp[s][k4]));
      }
    if (lane < 16) {
#pragma unroll
      for (int s = 0; s < SP; ++s)
#pragma unroll
        for (int k4 = 0; k4 < BC; ++k4) sPart[(wid * SP + s) * 16 * BC + qb * BC + k4] = gp[s][k4];
    }
    if (p.prof && g == 0 && tid == kCtl * 64 && k < 64) p.prof[k * 16 + 5] = __builtin_amdgcn_s_memtime();
    if (ctl && k > 0) {
      // ---- decision pipeline (control wave) over bodies dj .. k-1 ---------------
      // Partials are pre-filled with a signalling-NaN sentinel (never produced by
      // arithmetic) and each is written once by one 8-byte atomic store, so a load
      // returns either the sentinel (not published yet) or the final value.  Loads
      // for bodies dj and dj+1 are kept in flight across bodies; the wave blocks
      // (bounded spin) only when the pipeline is kLag bodies behind.
      const int last = k - 1;                // latest body this workgroup has published
      for (int rep = 0; rep < 2; ++rep) {
        const bool must = eval_only || (last - dj) >= kLag;
        if (!issued0 || dj > last) break;
        bool ok = true;
#pragma unroll
        for (int q = 0; q < kPartPerLane; ++q) ok &= (lv0[q] != kSentinel);
        ok = __all(ok);
        if (p.prof && g == 0 && lane == 0 && k < 64 && rep == 0) p.prof[k * 16 + 8] = __builtin_amdgcn_s_memtime();
        if (!ok && must) {  // blocking re-poll of body dj
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (!ok) {
            __builtin_amdgcn_s_sleep(1);
            load_parts(p, dj, lane, lv0);
            ok = true;
#pragma unroll
            for (int q = 0; q < kPartPerLane; ++q) ok &= (lv0[q] != kSentinel);
            ok = __all(ok);
            if (p.prof && g == 0 && lane == 0 && k < 64) p.prof[k * 16 + 7] += 1;
            if (__builtin_amdgcn_s_memrealtime() - t0 > p.spin) {
              if (lane == 0) {
                atomicOr(p.timeout, 1);
                sCtl[2] = 1;
              }
              break;
            }
          }
          if (!ok) break;
        }
        if (!ok) {  // not published yet: re-issue, try next body
          load_parts(p, dj, lane, lv0);
          break;
        }
        const double loss = sum_parts(lv0);
        if (p.prof && g == 0 && lane == 0 && k < 64 && rep == 0) p.prof[k * 16 + 9] = __builtin_amdgcn_s_memtime();
        const int j = dj;
        if (j == 0) {
          loss0 = loss;
          loss_prev = loss;
        }
        bool cont;
        if (eval_only) {
          cont = false;
        } else {
          const double rel = fabs(loss - loss_prev) / fmax(fabs(loss), 1e-8);
          // tol < 0: no early stop (the speculative batches of the neuron-sharded M-step),
          // also not on a NaN loss, whose rel compares false
          cont = (j + 1 < maxiter - 1) && ((j + 1 < 5) || p.tol < 0.0 || (rel > p.tol));
        }
        loss_prev = loss;
        ++dj;
        if (!cont) {
          fin_loss = loss;
          if (lane == 0) sCtl[0] = 1, sCtl[1] = j;
          break;
        }
#pragma unroll
        for (int q = 0; q < kPartPerLane; ++q) lv0[q] = lv1[q];
        issued0 = issued1;
        issued1 = false;
      }
      if (p.prof && g == 0 && lane == 0 && k < 64) p.prof[k * 16 + 10] = __builtin_amdgcn_s_memtime();
      if (!sCtl[0]) {  // keep bodies dj and dj+1 in flight (both <= last)
        if (!issued0 && dj <= last) {
          load_parts(p, dj, lane, lv0);
          issued0 = true;
        }
        if (!issued1 && dj + 1 <= last) {
          load_parts(p, dj + 1, lane, lv1);
          issued1 = true;
        }
      }
    }
    if (p.prof && g == 0 && tid == kCtl * 64 && k < 64) p.prof[k * 16 + 6] = __builtin_amdgcn_s_memtime();
    PMG_ADAM_STAMP(k, 1)
    PMG_LDS_BARRIER();
    PMG_ADAM_STAMP(k, 2)
    // ---- Adam element update ------------------------------------------------------
    double gsq = 0.0;
    float gsum = 0.f;
    // the element's LDS indices re-derived here from an opaque copy of tid (a few VALU
    // per body) instead of being held across the loop: at the 256-VGPR cap the
    // allocator would spill them, and each scratch reload waits on vmcnt
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int eq_ = tq / SP, es_ = tq % SP;
    const int e_ = eq_ * SP + es_;
    const int ewo_ = es_ * QS + (eq_ / BC) * BCP + eq_ % BC;
    if (is_el) {
#pragma unroll
      for (int w = 0; w < kNW; ++w) gsum += sPart[(w * SP + es_) * 16 * BC + eq_];
    }
    // (row blocks exist only with A = 8, L in (512, 1024]: the other instances carry no
    // exchange code, which would cost them registers)
    if (A == 8 && p.RB > 1 && wid * 64 < NB * SP) {
      // row blocks: this workgroup's partial B^T G (its rows) to the other row blocks of
      // the group, theirs back; every block sums the RB partials in block order, so all
      // of them run the identical update.  Message passing per wave: the data as
      // agent-scope (sc1, cache-bypassing) stores, vmcnt(0) so they are performed, then the
      // flag = bodies published; the partner polls the flag, then reads the data with sc1
      // loads.  Data and flags never sit in the non-coherent L2, so no agent-scope fence
      // (an XCD-wide L2 writeback / invalidate per wave and body) is needed.  Two body-
      // parity buffers suffice: a block publishes body k + 2 only after every partner has
      // published body k + 1, i.e. after each has read its body-k partials.
      float* xb = p.xbuf + (size_t)(k & 1) * p.G * kXSlots;
      if (is_el) __hip_atomic_store(&xb[(size_t)g * kXSlots + e_], gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&p.xflag[g * kNW + wid], k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      float tot = 0.f;
      for (int rr = 0; rr < p.RB; ++rr) {
        const int gp = rr * p.Gg + gg;
        if (rr != rb) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&p.xflag[gp * kNW + wid], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT)) < k + 1) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > p.spin) {
              if (lane == 0) {
                atomicOr(p.timeout, 1);
                sCtl[2] = 1;
              }
              break;
            }
          }
          asm volatile("" ::: "memory");
        }
        const float v = rr == rb ? gsum
                                 : (is_el ? __hip_atomic_load(&xb[(size_t)gp * kXSlots + e_], __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT)
                                          : 0.f);
        tot += v;
      }
      gsum = tot;
    }
    if (is_el) {
      const double gr = -(double)gsum + w_cur * isd2;
      // the prior and |g|^2 terms once per neuron group (row block 0)
      gsq = rb == 0 ? gr * gr : 0.0;
      lpart += rb == 0 ? 0.5 * w_cur * w_cur * isd2 + sLconst : 0.0;
      const double w_old = w_cur;
      if (!eval_only) {  // optax 0.2.2 scale_by_adam + scale(-lr)
        const double mu = (1.0 - p.b1) * gr + p.b1 * mu_cur;
        const double nu = (1.0 - p.b2) * gr * gr + p.b2 * nu_cur;
        // this body's bias corrections (uniform); bodies run ahead of the decision past
        // maxiter are discarded
        const int kb = __builtin_amdgcn_readfirstlane(k < mi ? k : mi - 1);
        double c1, c2;
        if (kb < kBiasLds) {
          c1 = sBias[kb];
          c2 = sBias[kBiasLds + kb];
        } else {
          c1 = p.bias[kb];
          c2 = bias2[kb];
        }
        const double mh = mu * c1;
        const double nh = nu * c2;
        w_cur = w_cur - p.lr * (mh * rcp_nr(sqrt(nh + p.eps_root) + p.eps));
        mu_cur = mu;
        nu_cur = nu;
      }
      const int ns = (k + 1) % kRing;
      sW[ewo_] = w_cur;
      sD[ewo_] = (float)(w_cur - w_old);
      sRing[(ns * 3 + 0) * RS + e_] = w_cur;
      sRing[(ns * 3 + 1) * RS + e_] = mu_cur;
      sRing[(ns * 3 + 2) * RS + e_] = nu_cur;
    }
    lpart = wave_sum_f64(lpart);
    gsq = wave_sum_f64(gsq);
    if (lane == 0) {
      sSum[wid] = lpart;
      sSum[kNW + wid] = gsq;
    }
    PMG_ADAM_STAMP(k, 3)
    PMG_LDS_BARRIER();
    if (sCtl[0] || sCtl[2]) break;
    if (tid == 0) {
      double a = 0.0, b = 0.0;
      for (int q = 0; q < kNW; ++q) {
        a += sSum[q];
        b += sSum[kNW + q];
      }
      st_sc1(&p.lpart[(size_t)k * p.G + g], a);
      st_sc1(&p.gpart[(size_t)k * p.G + g], b);
    }
    PMG_ADAM_STAMP(k, 4)
  }
  // Row blocks: the blocks of a group learn the stop at bodies up to kLag apart (each
  // control wave decides as soon as the partials are there), so a block that leaves
  // first releases its partners: a flag no body index reaches.  They finish their (at
  // most kLag) speculative bodies past the stop on stale partials, which the ring
  // discards: the state written below is the one after the stop body.
  if (A == 8 && p.RB > 1 && wid * 64 < NB * SP && lane == 0)
    __hip_atomic_store(&p.xflag[g * kNW + wid], 0x7fffffff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int stop_j = sCtl[1];
  // ---- write the state after body stop_j (W_{stop_j+1}) from the ring ---------
  const int fs = eval_only ? (1 % kRing) : ((stop_j + 1) % kRing);
  if (is_el && !sCtl[2]) {
    const size_t o = (size_t)eq * p.N + n0 + es;
    p.W[o] = sRing[(fs * 3 + 0) * RS + e];
    p.mu[o] = sRing[(fs * 3 + 1) * RS + e];
    p.nu[o] = sRing[(fs * 3 + 2) * RS + e];
  }
  if (g == 0 && ctl && lane == 0 && !sCtl[2]) {
    const int n_iter = eval_only ? 1 : stop_j + 2;
    p.stats[0] = (double)n_iter;
    p.stats[1] = fin_loss;
    p.stats[3] = loss0;
    p.count[0] = count0 + (eval_only ? 0 : (stop_j + 1));
  }
  // ---- histories (fit_tuning_helper.py:147-149, :175-176), entries i = g, g + G, ... ----
  // loss_hist[0] = loss of body 0, loss_hist[i] = loss of body i - 1; the same for the
  // gradient norm; final_error = the norm of the last body.  Summed in the decision's
  // order (load_parts / sum_parts).  Every body <= stop_j has all its loss partials (the
  // decision read them); its |g|^2 partials were stored right after them and are polled
  // until they have landed.
  if (ctl && !sCtl[2]) {
    const int n_iter = eval_only ? 1 : stop_j + 2;
    for (int i = g; i < n_iter; i += p.G) {
      const int j = i == 0 ? 0 : i - 1;
      unsigned long long lv[kPartPerLane], gv[kPartPerLane];
      load_parts(p, j, lane, lv);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      bool ok = false;
      while (!ok) {
#pragma unroll
        for (int q = 0; q < kPartPerLane; ++q) {
          const int gi = lane + 64 * q;
          gv[q] = gi < p.G ? ld_bits(&p.gpart[(size_t)j * p.G + gi]) : 0ull;
        }
        ok = true;
#pragma unroll
        for (int q = 0; q < kPartPerLane; ++q) ok &= (gv[q] != kSentinel) && (lv[q] != kSentinel);
        ok = __all(ok);
        if (!ok) {
          load_parts(p, j, lane, lv);
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > p.spin) {
            if (lane == 0) atomicOr(p.timeout, 1);
            break;
          }
        }
      }
      if (!ok) break;
      const double loss = sum_parts(lv);
      const double err = sqrt(sum_parts(gv));
      if (lane == 0) {
        p.loss_hist[i] = loss;
        p.err_hist[i] = err;
        if (i == n_iter - 1) p.stats[2] = err;
      }
    }
  }
}

struct AdamWork {
  unsigned long long* lpart;
  unsigned long long* gpart;
  double* bias;
  int* timeout;
  float* xbuf;
  int* xflag;
};

static int num_cus();

// G <= #CUs workgroups (all co-resident): the partial arrays and the row-block exchange
// are sized for #CUs, so one size serves every row-block split of a shape
static size_t adam_ws(int G, int maxiter, AdamWork* w, void* base) {
  const int cus = num_cus();
  const size_t Gw = (size_t)(G > cus ? G : cus);
  Carver c(base);
  AdamWork ww;
  ww.timeout = c.take<int>(64);
  ww.lpart = c.take<unsigned long long>(((size_t)maxiter + kLag + 2) * Gw);
  ww.gpart = c.take<unsigned long long>(((size_t)maxiter + kLag + 2) * Gw);
  ww.bias = c.take<double>(2 * (size_t)maxiter);
  ww.xbuf = c.take<float>(2 * Gw * kXSlots);
  ww.xflag = c.take<int>(Gw * kNW);
  if (w) *w = ww;
  return c.off + 256;
}

typedef void (*adam_kernel_t)(AdamParams);

struct AdamKernel {
  adam_kernel_t fn;
  size_t lds;
};

template <int A, int BC>
static AdamKernel pick_sp(int S) {
  if (S <= 1) return {k_adam<A, BC, 1>, 0};
  if (S <= 2) return {k_adam<A, BC, 2>, 0};
  if constexpr (16 * BC * 4 <= kThreads) return {k_adam<A, BC, 4>, 0};   // NB S <= 512
  return {nullptr, 0};
}

template <int A>
static AdamKernel pick_bc(int NB, int S) {
  if constexpr (A == 8) {    // row-block split (L > 512, BASELINE C4: NB = 154)
    if (NB > 128 && NB <= 160) return pick_sp<A, 10>(S);
  }
  if (NB <= 32) return pick_sp<A, 2>(S);
  if (NB <= 48) return pick_sp<A, 3>(S);
  if (NB <= 64) return pick_sp<A, 4>(S);
  if (NB <= 80) return pick_sp<A, 5>(S);
  if (NB <= 96) return pick_sp<A, 6>(S);
  if (NB <= 128) return pick_sp<A, 8>(S);
  return {nullptr, 0};
}

// rows per l-block A = ceil(L / 32) rounded up to 4 / 8 / 16; L in (512, 1024]: row blocks
// of 256 rows (A = 8), adam_row_blocks
static AdamKernel pick_adam(int NB, int L, int S) {
  if (L <= 128) return pick_bc<4>(NB, S);
  if (L <= 256) return pick_bc<8>(NB, S);
  if (L <= 512) return pick_bc<16>(NB, S);
  if (L <= 1024) return pick_bc<8>(NB, S);
  return {nullptr, 0};
}

static int adam_row_blocks(int L) { return L <= 512 ? 1 : (L + 255) / 256; }

static int num_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
  return cus > 0 ? cus : 256;
}

// RB row blocks x Gg neuron groups of S neurons, G = RB Gg <= #CUs
static void adam_geometry(int N, int L, int NB, int& S, int& G, int& ng, int& LG, int* RBo = nullptr,
                          int* Ggo = nullptr) {
  const int cus = num_cus();
  const int RB = adam_row_blocks(L);
  const int gmax = cus / RB > 0 ? cus / RB : 1;
  S = (N + gmax - 1) / gmax;
  if (S < 1) S = 1;
  if (S == 3) S = 4;
  const int Gg = (N + S - 1) / S;
  G = RB * Gg;
  if (RBo) *RBo = RB;
  if (Ggo) *Ggo = Gg;
  ng = kThreads / NB;
  if (ng < 1) ng = 1;
  LG = (L + ng - 1) / ng;
}

// R restarts: Rg of them per launch, each on G workgroups of S neurons, with Rg G <= #CUs
// (one 512-thread workgroup per CU: every workgroup of a launch is resident).  S grows
// (up to kSMax, while the kernel still fits) so that more restarts share a launch.
static void adam_batch_geometry(int N, int L, int NB, int R, int& S, int& G, int& ng, int& LG, int& Rg) {
  adam_geometry(N, L, NB, S, G, ng, LG);
  const int cus = num_cus();
  if (R > 1) {
    int want = (int)(((int64_t)R * N + cus - 1) / cus);
    if (want == 3) want = 4;
    for (int s = want < kSMax ? want : kSMax; s > S; s = (s == 4 ? 2 : s - 1)) {
      AdamKernel k = pick_adam(NB, L, s);
      if (NB * s <= kThreads && k.fn != nullptr && k.lds <= 160 * 1024) {
        S = s;
        G = (N + S - 1) / S;
        break;
      }
    }
  }
  Rg = cus / G;
  if (Rg < 1) Rg = 1;
  if (Rg > R) Rg = R;
}

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_mstep_workspace_size(int32_t N, int32_t maxiter) {
  int S, G, ng, LG;
  adam_geometry(N, 512, 1, S, G, ng, LG);
  return adam_ws(G, maxiter > 1 ? maxiter : 1, nullptr, nullptr);
}

int pmg_mstep_adam_supported(int32_t L, int32_t NB, int32_t N) {
  if (L <= 0 || L > 2 * kThreads || NB <= 0 || N <= 0) return 0;
  int S, G, ng, LG;
  adam_geometry(N, L, NB, S, G, ng, LG);
  if (S > kSMax || NB * S > kThreads || G > num_cus()) return 0;
  AdamKernel kern = pick_adam(NB, L, S);
  return (kern.fn != nullptr && kern.lds <= 160 * 1024) ? 1 : 0;
}

// R restarts (R = 1: the plain call): restarts r0 .. r0+Rg-1 of each launch are its
// blockIdx.y; every restart has its own workspace slab of `slab` bytes.
static int adam_run(double* W, double* mu, double* nu, int64_t* count, const float* basis, const double* yw,
                    const double* tw, int L, int NB, int N, int R, const pmg_adam_cfg* cfg, double* stats,
                    double* loss_hist, double* err_hist, void* workspace, size_t workspace_bytes, hipStream_t st) {
  PMG_REQUIRE(cfg && W && mu && nu && count && basis && yw && tw && stats && loss_hist && err_hist && workspace,
              "pmg_mstep_adam: null argument");
  PMG_REQUIRE(L > 0 && L <= 2 * kThreads, "pmg_mstep_adam: L=%d must be in [1, %d]", L, 2 * kThreads);
  PMG_REQUIRE(NB > 0 && N > 0 && R >= 1 && R <= 65535, "pmg_mstep_adam: bad shape");
  PMG_REQUIRE(R == 1 || L <= kThreads, "pmg_mstep_adam: batched restarts need L <= %d", kThreads);
  int S, G, ng, LG, Rg;
  adam_batch_geometry(N, L, NB, R, S, G, ng, LG, Rg);
  int RB = 1, Gg = G;
  if (R == 1) adam_geometry(N, L, NB, S, G, ng, LG, &RB, &Gg);
  PMG_REQUIRE(G <= num_cus(), "pmg_mstep_adam: %d workgroups (%d row blocks) exceed the %d CUs", G, RB, num_cus());
  PMG_REQUIRE(S <= kSMax, "pmg_mstep_adam: N=%d needs %d neurons per workgroup (> %d)", N, S, kSMax);
  PMG_REQUIRE(NB * S <= kThreads, "pmg_mstep_adam: NB*S=%d > %d", NB * S, kThreads);
  AdamKernel kern = pick_adam(NB, L, S);
  PMG_REQUIRE(kern.fn != nullptr && kern.lds <= 160 * 1024,
              "pmg_mstep_adam: NB=%d unsupported (basis must fit registers + 160 KiB LDS)", NB);
  const int maxiter = cfg->maxiter > 1 ? cfg->maxiter : 1;
  const size_t slab = (adam_ws(G, maxiter, nullptr, nullptr) + 255) & ~(size_t)255;
  PMG_REQUIRE(workspace_bytes >= (R == 1 ? adam_ws(G, maxiter, nullptr, nullptr) : (size_t)R * slab),
              "pmg_mstep_adam: workspace too small");
  AdamWork w;
  adam_ws(G, maxiter, &w, workspace);
  AdamParams p;
  memset(&p, 0, sizeof(p));
  p.W = W;
  p.mu = mu;
  p.nu = nu;
  p.count = count;
  p.basis = basis;
  p.yw = yw;
  p.tw = tw;
  p.L = L;
  p.NB = NB;
  p.N = N;
  p.S = S;
  p.G = G;
  p.ng = ng;
  p.LG = LG;
  p.lr = cfg->lr;
  p.b1 = cfg->b1;
  p.b2 = cfg->b2;
  p.eps = cfg->eps;
  p.eps_root = cfg->eps_root;
  p.prior_std = cfg->prior_std;
  p.tol = cfg->tol;
  p.maxiter = cfg->maxiter;
  p.stats = stats;
  p.loss_hist = loss_hist;
  p.err_hist = err_hist;
  p.lpart = w.lpart;
  p.gpart = w.gpart;
  p.timeout = w.timeout;
  p.spin = spin_ticks(kAdamSpinTicks);
  p.bias = w.bias;
  p.rs_W = (int64_t)NB * N;
  p.rs_yw = (int64_t)L * N;
  p.rs_tw = L;
  p.rs_hist = maxiter;
  p.rs_ws = (int64_t)slab;
  p.RB = RB;
  p.Gg = Gg;
  p.xbuf = RB > 1 ? w.xbuf : nullptr;
  p.xflag = RB > 1 ? w.xflag : nullptr;
  static long long* prof_buf = nullptr;   // debug: per-phase stamps (PMG_ADAM_PROF set)
  const bool prof = getenv("PMG_ADAM_PROF") != nullptr;
  if (prof) {
    if (!prof_buf) PMG_HIP(hipMalloc(&prof_buf, 64 * 16 * sizeof(long long)));
    PMG_HIP(hipMemsetAsync(prof_buf, 0, 64 * 16 * sizeof(long long), st));
    p.prof = prof_buf;
  } else {
    p.prof = nullptr;
  }
  const size_t n = ((size_t)maxiter + kLag + 2) * G;
  for (int r0 = 0; r0 < R; r0 += Rg) {
    const int rg = R - r0 < Rg ? R - r0 : Rg;
    AdamParams q = p;   // restart r0's pointers
    q.W += r0 * p.rs_W;
    q.mu += r0 * p.rs_W;
    q.nu += r0 * p.rs_W;
    q.count += r0;
    q.yw += r0 * p.rs_yw;
    q.tw += (int64_t)r0 * p.rs_tw;
    q.stats += 4 * (int64_t)r0;
    q.loss_hist += (int64_t)r0 * p.rs_hist;
    q.err_hist += (int64_t)r0 * p.rs_hist;
    const size_t o = (size_t)r0 * slab;
    q.bias = reinterpret_cast<const double*>(reinterpret_cast<char*>(w.bias) + o);
    q.lpart = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.lpart) + o);
    q.gpart = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(w.gpart) + o);
    hipLaunchKernelGGL(k_adam_prologue, dim3(256, rg), dim3(256), 0, st, q, n);
    PMG_LAUNCH_CHECK();
    // rg x G workgroups, at most one per CU (adam_batch_geometry): all co-resident
    PMG_HIP(launch_persistent(kern.fn, dim3(G, rg), dim3(kThreads), kern.lds, st, q));
  }
  if (prof) {
    long long h[64 * 16];
    PMG_HIP(hipMemcpyAsync(h, prof_buf, sizeof(h), hipMemcpyDeviceToHost, st));
    PMG_HIP(hipStreamSynchronize(st));
    double acc[6] = {0, 0, 0, 0, 0, 0};
    double acc6 = 0, acc7 = 0, acc8 = 0;
    int n6 = 0, n7 = 0, n8 = 0;
    long long spins = 0;
    int cnt = 0;
    for (int k = 8; k + 1 < 64; ++k) {   // skip the pipeline fill
      if (h[k * 16 + 4] == 0 || h[(k + 1) * 16] == 0) break;
      for (int i = 0; i < 4; ++i) acc[i] += (double)(h[k * 16 + i + 1] - h[k * 16 + i]);
      acc[4] += (double)(h[(k + 1) * 16] - h[k * 16 + 4]);
      acc[5] += (double)(h[k * 16 + 6] - h[k * 16 + 5]);
      if (h[k * 16 + 8]) acc6 += (double)(h[k * 16 + 8] - h[k * 16 + 5]), ++n6;
      if (h[k * 16 + 9]) acc7 += (double)(h[k * 16 + 9] - h[k * 16 + 8]), ++n7;
      if (h[k * 16 + 10]) acc8 += (double)(h[k * 16 + 6] - h[k * 16 + 10]), ++n8;
      spins += h[k * 16 + 7];
      ++cnt;
    }
    if (cnt > 0)
      fprintf(stderr, "[pmg adam prof] bodies=%d ticks/body: rows %.0f | bar1 %.0f | update %.0f | "
              "sums+bar2+publish %.0f | loop %.0f | decision (ctl wave) %.0f, blocking polls %lld\n", cnt,
              acc[0] / cnt, acc[1] / cnt, acc[2] / cnt, acc[3] / cnt, acc[4] / cnt, acc[5] / cnt, spins);
    if (cnt > 0)
      fprintf(stderr, "[pmg adam prof] decision: to first check %.0f (%d) | first sum %.0f (%d) | after loop %.0f (%d)\n",
              n6 ? acc6 / n6 : 0.0, n6, n7 ? acc7 / n7 : 0.0, n7, n8 ? acc8 / n8 : 0.0, n8);
  }
  return PMG_OK;
}

int pmg_mstep_adam(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                   const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                   const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                   void* workspace, size_t workspace_bytes, void* stream) {
  return adam_run(W, mu, nu, count, basis, yw, tw, L, NB, N, 1, cfg, stats, loss_hist, err_hist, workspace,
                  workspace_bytes, as_stream(stream));
}

int pmg_mstep_adam_status(void* workspace, int32_t* timed_out, void* stream) {
  PMG_REQUIRE(workspace && timed_out, "pmg_mstep_adam_status: null argument");
  hipStream_t st = as_stream(stream);
  int32_t h = 0;
  PMG_HIP(hipMemcpyAsync(&h, workspace, sizeof(h), hipMemcpyDeviceToHost, st));
  PMG_HIP(hipStreamSynchronize(st));
  if (h != 0) PMG_HIP(hipMemsetAsync(workspace, 0, sizeof(h), st));
  *timed_out = h != 0;
  return PMG_OK;
}

size_t pmg_mstep_batched_workspace_size(int32_t L, int32_t NB, int32_t N, int32_t R, int32_t maxiter) {
  if (L <= 0 || NB <= 0 || N <= 0 || R < 1) return 0;
  int S, G, ng, LG, Rg;
  adam_batch_geometry(N, L, NB, R, S, G, ng, LG, Rg);
  const size_t one = adam_ws(G, maxiter > 1 ? maxiter : 1, nullptr, nullptr);
  return R == 1 ? one : (size_t)R * ((one + 255) & ~(size_t)255);
}

int pmg_mstep_adam_batched_supported(int32_t L, int32_t NB, int32_t N, int32_t R) {
  if (L <= 0 || L > kThreads || NB <= 0 || N <= 0 || R < 1) return 0;
  int S, G, ng, LG, Rg;
  adam_batch_geometry(N, L, NB, R, S, G, ng, LG, Rg);
  if (S > kSMax || NB * S > kThreads) return 0;
  AdamKernel kern = pick_adam(NB, L, S);
  return (kern.fn != nullptr && kern.lds <= 160 * 1024) ? 1 : 0;
}

int pmg_mstep_adam_batched(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                           const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N, int32_t R,
                           const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                           void* workspace, size_t workspace_bytes, void* stream) {
  return adam_run(W, mu, nu, count, basis, yw, tw, L, NB, N, R, cfg, stats, loss_hist, err_hist, workspace,
                  workspace_bytes, as_stream(stream));
}

}  // extern "C"
