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
// CU, all co-resident), keep the basis in registers twice (row-major for f = B W,
// column groups for B^T G), run Adam on their own columns in f64 and publish a
// f64 partial loss / squared gradient norm per iteration.  Instead of a grid
// barrier per iteration, every workgroup runs LAG iterations ahead and decides
// "stop after body j" from the globally summed partials of iteration j (summed in
// the same fixed order by every workgroup, hence identical decisions); a small
// ring of (W, mu, nu) states lets it return exactly the state after body j+1.
#include <stdio.h>
#include <stdlib.h>

#include "pmg_common.h"

namespace pmg {

// In-loop workgroup barrier that waits only for LDS traffic (lgkmcnt), so the
// decision pipeline's global loads stay in flight across it (a __syncthreads()
// would drain vmcnt, cdna_hip_programming.md "Pipelining across barriers").
#define PMG_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

constexpr int kLag = 4;                 // bodies a workgroup runs ahead of the decision
constexpr int kRing = kLag + 2;
constexpr int kSMax = 4;                // neurons per workgroup
constexpr int kThreads = 512;           // L <= 512
constexpr int kPartPerLane = 4;         // G <= 256 workgroups -> 4 partials per lane

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
  unsigned long long* lpart;  // [maxiter + kLag + 2][G] f64 bits, pre-filled with kSentinel
  unsigned long long* gpart;  // [..][G]
  double* ring;               // [G][kRing][3][NBM*4] (W, mu, nu) after each body
  int* timeout;
  long long* prof;            // optional (PMG_ADAM_PROF): s_memtime stamps of WG 0, bodies < 64
};

#define PMG_ADAM_STAMP(k, i)                                                   \
  if (p.prof && g == 0 && tid == 0 && (k) < 64) p.prof[(k) * 8 + (i)] = __builtin_amdgcn_s_memtime();

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

// ---------------------------------------------------------------------------
// Wave transpose-reduce: 64 per-lane values x[0..63] -> lane l returns
// sum over the 64 lanes of x[bitrev6(l)].  Six butterfly stages (lane bit 5..0:
// permlane32_swap, permlane16_swap, DPP row_ror:8, row_half_mirror,
// quad_perm[2,3,0,1], quad_perm[1,0,3,2]); at every stage the lower half of each
// lane group keeps the even register of a pair and the upper half the odd one, so
// each stage halves the registers: ~140 instructions for 64 sums.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float f_of(unsigned u) { return __uint_as_float(u); }
__device__ __forceinline__ unsigned u_of(float f) { return __float_as_uint(f); }

template <int CTRL>
__device__ __forceinline__ float dpp_pair_add(float a, float b, bool upper) {
  // lower lanes: a + partner(a); upper lanes: b + partner(b)
  const float x = upper ? b : a;
  const float y = upper ? a : b;
  return x + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(y), CTRL, 0xf, 0xf, false));
}

__device__ __forceinline__ int bitrev5(int l) {
  return ((l & 1) << 4) | ((l & 2) << 2) | (l & 4) | ((l & 8) >> 2) | ((l & 16) >> 4);
}

// 32 values x_i = a[i/S]*b[i%S] (generated on the fly, pairwise, to keep register
// pressure at 16 + 2): stages on lane bits 4..0 inside each 32-lane half, then the
// two halves are added (permlane32_swap of a register with itself).  Lane l returns
// the 64-lane sum of x[bitrev5(l & 31)].
template <int SP, int C0, int R>
__device__ __forceinline__ float wave_products_reduce32(const float* brow, const float* gr) {
  const int lane = threadIdx.x & 63;
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int v0 = C0 + 2 * i, v1 = v0 + 1;
    const float p0 = (v0 < R) ? brow[v0 / SP] * gr[v0 % SP] : 0.f;
    const float p1 = (v1 < R) ? brow[v1 / SP] * gr[v1 % SP] : 0.f;
    auto r = __builtin_amdgcn_permlane16_swap(u_of(p0), u_of(p1), false, false);
    x[i] = f_of(r[0]) + f_of(r[1]);
  }
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = dpp_pair_add<0x128>(x[2 * i], x[2 * i + 1], b3);  // row_ror:8
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = dpp_pair_add<0x141>(x[2 * i], x[2 * i + 1], b2);  // row_half_mirror
#pragma unroll
  for (int i = 0; i < 2; ++i) x[i] = dpp_pair_add<0x4E>(x[2 * i], x[2 * i + 1], b1);   // quad_perm 2,3,0,1
  const float v = dpp_pair_add<0xB1>(x[0], x[1], b0);                                  // quad_perm 1,0,3,2
  auto r = __builtin_amdgcn_permlane32_swap(u_of(v), u_of(v), false, false);
  return f_of(r[0]) + f_of(r[1]);
}

// products brow[q]*g for q in [C0, R) (one neuron), reduced over the wave, written to
// sred[(QOFF + q) * 4] (the caller offsets sred by the neuron slot)
template <int C0, int R, int QOFF>
struct ChunkLoop {
  static __device__ __forceinline__ void run(const float* brow, float g, float* sred, int lane) {
    const float gg[1] = {g};
    const float red = wave_products_reduce32<1, C0, R>(brow, gg);
    const int v = C0 + bitrev5(lane & 31);
    if (lane < 32 && v < R) sred[(QOFF + v) * 4] = red;
    if constexpr (C0 + 32 < R) ChunkLoop<C0 + 32, R, QOFF>::run(brow, g, sred, lane);
  }
};

// Basis split: the first NBR columns of each row live in registers, the remaining
// NBM-NBR in an LDS row tile with a padded stride (stride = 16m+4 words: the 16
// lanes of a ds_read_b128 group land on distinct bank quads).
template <int NBM>
struct BasisSplit {
  static constexpr int NBR = NBM < 32 ? NBM : 32;
  static constexpr int NBL = NBM - NBR;               // multiple of 16
  static constexpr int STRIDE = NBL > 0 ? NBL + 4 : 4;
};

// Threads: thread = latent row (L <= 512).  Per body: rows (f, G, B^T G partials) |
// barrier | Adam element update (threads < NB*S, i.e. the first waves) while the LAST
// wave, which owns no weight, runs the stop-rule decision pipeline | barrier |
// publish.  The stop flag is seen by every wave right after the second barrier.
//
// f = softplus(F), F = B W_k, is needed to f64 accuracy (the factor y_w/f - t_w
// cancels near the optimum).  F is carried per (row, neuron) in f64 registers and
// advanced by the f32 product B (W_k - W_{k-1}) of the small Adam step (error ~1e-9
// per body), and recomputed exactly in f64 every kRefresh bodies.
constexpr int kNW = kThreads / 64;          // waves (the last one also runs the decision)
constexpr int kThreadsAll = kThreads;
constexpr int kRefresh = 16;

template <int NBM, int LGM, int SP>
__global__ void __launch_bounds__(kThreadsAll) k_adam(AdamParams p) {
  using BS = BasisSplit<NBM>;
  constexpr int NBR = BS::NBR, NBL = BS::NBL, STRIDE = BS::STRIDE;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sBl = smem;                                                   // [kThreads][STRIDE]
  double* sW = reinterpret_cast<double*>(sBl + kThreads * STRIDE);     // [4][NBM] W_k (f64)
  float* sD = reinterpret_cast<float*>(sW + NBM * kSMax);              // [4][NBM] W_k - W_{k-1}
  float* sRed = sD + NBM * kSMax;                                      // [kNW][NBM][4] partial B^T G
  double* sSum = reinterpret_cast<double*>(sRed + kNW * NBM * kSMax);  // [2][kNW]
  double* sYw = sSum + 2 * kNW;                                        // [kThreads][4]
  int* sCtl = reinterpret_cast<int*>(sYw + kThreads * kSMax);          // [4]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const bool ctl = wid == kNW - 1;                     // runs the decision pipeline
  const int g = blockIdx.x;
  const int n0 = g * p.S;
  const int S = (p.N - n0) < p.S ? (p.N - n0) : p.S;  // neurons owned
  const int L = p.L, NB = p.NB;
  const double sd = p.prior_std, isd2 = 1.0 / (sd * sd);
  const double lconst = log(sd) + 0.5 * log(2.0 * M_PI);

  // ---- one-time loads -------------------------------------------------------
  const bool is_row = tid < L;
  float brow[NBR];
#pragma unroll
  for (int k = 0; k < NBR; ++k) brow[k] = (is_row && k < NB) ? p.basis[(size_t)tid * NB + k] : 0.f;
  for (int k = 0; k < STRIDE; ++k) {
    const int q = NBR + k;
    sBl[tid * STRIDE + k] = (is_row && k < NBL && q < NB) ? p.basis[(size_t)tid * NB + q] : 0.f;
  }
  double twd = 0.0;
  for (int s = 0; s < kSMax; ++s)
      sYw[tid * kSMax + s] = (is_row && s < S) ? p.yw[(size_t)tid * p.N + n0 + s] : 0.0;
  if (is_row) twd = p.tw[tid];
  const int ek = tid % NB, en = tid / NB;
  const bool is_el = en < S;
  for (int q = tid; q < NBM * kSMax; q += blockDim.x) {
    sW[q] = 0.0;
    sD[q] = 0.f;
  }
  if (tid < 4) sCtl[tid] = 0;
  // element state (W, mu, nu) of this thread's weight, and its global ring
  double w_cur = 0.0, mu_cur = 0.0, nu_cur = 0.0;
  double* ring = p.ring + (size_t)g * kRing * 3 * NBM * kSMax;
  const int e = ek * kSMax + en;
  __syncthreads();
  if (is_el) {
    const size_t o = (size_t)ek * p.N + n0 + en;
    w_cur = p.W[o];
    mu_cur = p.mu[o];
    nu_cur = p.nu[o];
    sW[en * NBM + ek] = w_cur;
    ring[(0 * 3 + 0) * NBM * kSMax + e] = w_cur;
    ring[(0 * 3 + 1) * NBM * kSMax + e] = mu_cur;
    ring[(0 * 3 + 2) * NBM * kSMax + e] = nu_cur;
  }
  const int64_t count0 = p.count[0];
  double b1t = pow(p.b1, (double)count0), b2t = pow(p.b2, (double)count0);
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
  // running F of this row for neurons 0..3 (f64)
  double F0 = 0.0, F1 = 0.0, F2 = 0.0, F3 = 0.0;

  for (int k = 0;; ++k) {
    // ---- body k: evaluate at W_k ---------------------------------------------
    PMG_ADAM_STAMP(k, 0)
    double lpart = 0.0;
    {
      const bool exact = (k % kRefresh) == 0;
      // neurons one at a time (runtime loop, not unrolled: one neuron's registers live)
#pragma unroll 1
      for (int s = 0; s < S; ++s) {
        double F;
        if (exact) {
          F = 0.0;
#pragma unroll
          for (int q = 0; q < NBR; ++q) {
            asm volatile("" : "+v"(brow[q]));   // keep the f32->f64 conversion local
            F = fma((double)brow[q], sW[s * NBM + q], F);
          }
#pragma unroll 2
          for (int q4 = 0; q4 < NBL; q4 += 4) {
            const float4 b4 = *reinterpret_cast<const float4*>(&sBl[tid * STRIDE + q4]);
            F = fma((double)b4.x, sW[s * NBM + NBR + q4], F);
            F = fma((double)b4.y, sW[s * NBM + NBR + q4 + 1], F);
            F = fma((double)b4.z, sW[s * NBM + NBR + q4 + 2], F);
            F = fma((double)b4.w, sW[s * NBM + NBR + q4 + 3], F);
          }
        } else {
          float dF = 0.f;
#pragma unroll
          for (int q = 0; q < NBR; ++q) dF = fmaf(brow[q], sD[s * NBM + q], dF);
#pragma unroll
          for (int q4 = 0; q4 < NBL; q4 += 4) {
            const float4 b4 = *reinterpret_cast<const float4*>(&sBl[tid * STRIDE + q4]);
            const float4 d4 = *reinterpret_cast<const float4*>(&sD[s * NBM + NBR + q4]);
            dF = fmaf(b4.x, d4.x, dF);
            dF = fmaf(b4.y, d4.y, dF);
            dF = fmaf(b4.z, d4.z, dF);
            dF = fmaf(b4.w, d4.w, dF);
          }
          F = (s == 0 ? F0 : s == 1 ? F1 : s == 2 ? F2 : F3) + (double)dF;
        }
        F0 = s == 0 ? F : F0;
        F1 = s == 1 ? F : F1;
        F2 = s == 2 ? F : F2;
        F3 = s == 3 ? F : F3;
        const double ywd = is_row ? sYw[tid * kSMax + s] : 0.0;
        // softplus / sigmoid in f32 at Fh = f32(F), corrected to first order in the
        // exact residual r = F - Fh (|r| <= 2^-24 |F|): f = softplus(Fh) + sigmoid(Fh) r
        const float Fh = (float)F;
        const double r = F - (double)Fh;
        const float f32 = fmaxf(Fh, 0.f) + log1pf(expf(-fabsf(Fh)));
        const float sg = 1.f / (1.f + expf(-Fh));
        const double fd = (double)f32 + (double)sg * r;
        const float gr = is_row ? (float)((ywd / (fd + 1e-20) - twd) * (double)sg) : 0.f;
        if (is_row) {
          const double xl = (ywd != 0.0) ? ywd * ((double)logf(f32 + 1e-20f) + (double)sg * r / (double)f32) : 0.0;
          lpart -= xl - fd * twd;
        }
        // per-wave partial of B^T G for this neuron, 32 columns per chunk
        float* sr = &sRed[(wid * NBM) * kSMax] + s;
        ChunkLoop<0, NBR, 0>::run(brow, gr, sr, lane);
#pragma unroll
        for (int c0 = 0; c0 < NBL; c0 += 32) {
          float bl[32];
#pragma unroll
          for (int q4 = 0; q4 < 32; q4 += 4) {
            const float4 b4 = (c0 + q4 < NBL)
                                  ? *reinterpret_cast<const float4*>(&sBl[tid * STRIDE + c0 + q4])
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
            bl[q4] = b4.x;
            bl[q4 + 1] = b4.y;
            bl[q4 + 2] = b4.z;
            bl[q4 + 3] = b4.w;
          }
          const float gg[1] = {gr};
          const float red = wave_products_reduce32<1, 0, 32>(bl, gg);
          const int v = c0 + bitrev5(lane & 31);
          if (lane < 32 && v < NBL) sr[(NBR + v) * kSMax] = red;
        }
      }
    }
    PMG_ADAM_STAMP(k, 1)
    PMG_LDS_BARRIER();
    PMG_ADAM_STAMP(k, 2)
    double gsq = 0.0;
    b1t *= p.b1;
    b2t *= p.b2;
    if (is_el) {
      float gsum = 0.f;
      for (int q = 0; q < kNW; ++q) gsum += sRed[(q * NBM) * kSMax + e];
      const double gr = -(double)gsum + w_cur * isd2;
      gsq = gr * gr;
      lpart += 0.5 * w_cur * w_cur * isd2 + lconst;
      const double w_old = w_cur;
      if (!eval_only) {  // optax 0.2.2 scale_by_adam + scale(-lr)
        const double mu = (1.0 - p.b1) * gr + p.b1 * mu_cur;
        const double nu = (1.0 - p.b2) * gr * gr + p.b2 * nu_cur;
        const double mh = mu / (1.0 - b1t);
        const double nh = nu / (1.0 - b2t);
        w_cur = w_cur - p.lr * (mh / (sqrt(nh + p.eps_root) + p.eps));
        mu_cur = mu;
        nu_cur = nu;
      }
      const int ns = (k + 1) % kRing;
      ring[(ns * 3 + 0) * NBM * kSMax + e] = w_cur;
      ring[(ns * 3 + 1) * NBM * kSMax + e] = mu_cur;
      ring[(ns * 3 + 2) * NBM * kSMax + e] = nu_cur;
      sW[en * NBM + ek] = w_cur;
      sD[en * NBM + ek] = (float)(w_cur - w_old);
    }
    lpart = wave_sum_f64(lpart);
    gsq = wave_sum_f64(gsq);
    if (lane == 0) {
      sSum[wid] = lpart;
      sSum[kNW + wid] = gsq;
    }
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
        if (!ok && must) {  // blocking re-poll of body dj
          unsigned spins = 0;
          while (!ok) {
            __builtin_amdgcn_s_sleep(1);
            load_parts(p, dj, lane, lv0);
            ok = true;
#pragma unroll
            for (int q = 0; q < kPartPerLane; ++q) ok &= (lv0[q] != kSentinel);
            ok = __all(ok);
            if (++spins > (1u << 24)) {
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
          cont = (j + 1 < maxiter - 1) && ((j + 1 < 5) || (rel > p.tol));
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
  const int stop_j = sCtl[1];
  // ---- write the state after body stop_j (W_{stop_j+1}) from the ring ---------
  const int fs = eval_only ? (1 % kRing) : ((stop_j + 1) % kRing);
  if (is_el && !sCtl[2]) {
    const size_t o = (size_t)ek * p.N + n0 + en;
    p.W[o] = ring[(fs * 3 + 0) * NBM * kSMax + e];
    p.mu[o] = ring[(fs * 3 + 1) * NBM * kSMax + e];
    p.nu[o] = ring[(fs * 3 + 2) * NBM * kSMax + e];
  }
  if (g == 0 && ctl && lane == 0 && !sCtl[2]) {
    const int n_iter = eval_only ? 1 : stop_j + 2;
    p.stats[0] = (double)n_iter;
    p.stats[1] = fin_loss;
    p.stats[3] = loss0;
    p.count[0] = count0 + (eval_only ? 0 : (stop_j + 1));
  }
}

template <int NBM>
static size_t adam_lds_bytes() {
  using BS = BasisSplit<NBM>;
  return sizeof(float) * ((size_t)kThreads * BS::STRIDE + 2 * NBM * kSMax + NBM * kSMax +
                          kNW * NBM * kSMax) +
         sizeof(double) * (2 * kNW + kThreads * kSMax) + sizeof(int) * 4 + 64;
}

// Histories (fit_tuning_helper.py:147-149, :175-176) from the published partials, summed
// in the decision's order: loss_hist[0] = loss of body 0, loss_hist[j+1] = loss of body j
// (j + 1 < n_iter); the same for the gradient norm; final_error = norm of the last body.
__global__ void __launch_bounds__(64) k_adam_hist(AdamParams p) {
  const int lane = threadIdx.x;
  const int n_iter = (int)p.stats[0];
  if (n_iter <= 0) return;
  for (int i = blockIdx.x; i < n_iter; i += gridDim.x) {
    const int j = (i == 0) ? 0 : i - 1;
    unsigned long long lv[kPartPerLane], gv[kPartPerLane];
#pragma unroll
    for (int q = 0; q < kPartPerLane; ++q) {
      const int gi = lane + 64 * q;
      lv[q] = gi < p.G ? p.lpart[(size_t)j * p.G + gi] : 0ull;
      gv[q] = gi < p.G ? p.gpart[(size_t)j * p.G + gi] : 0ull;
    }
    const double loss = sum_parts(lv);
    const double err = sqrt(sum_parts(gv));
    if (lane == 0) {
      p.loss_hist[i] = loss;
      p.err_hist[i] = err;
      if (i == n_iter - 1) p.stats[2] = err;
    }
  }
}

struct AdamWork {
  double* ring;
  unsigned long long* lpart;
  unsigned long long* gpart;
  int* timeout;
};

static size_t adam_ws(int G, int maxiter, AdamWork* w, void* base) {
  Carver c(base);
  AdamWork ww;
  ww.timeout = c.take<int>(64);
  ww.ring = c.take<double>((size_t)G * kRing * 3 * 128 * kSMax);
  ww.lpart = c.take<unsigned long long>(((size_t)maxiter + kLag + 2) * G);
  ww.gpart = c.take<unsigned long long>(((size_t)maxiter + kLag + 2) * G);
  if (w) *w = ww;
  return c.off + 256;
}

typedef void (*adam_kernel_t)(AdamParams);

struct AdamKernel {
  adam_kernel_t fn;
  size_t lds;
};

template <int NBM>
static AdamKernel pick_sp(int SPn) {
  (void)SPn;  // neurons are looped at run time inside the kernel
  return {k_adam<NBM, NBM, 1>, adam_lds_bytes<NBM>()};
}

static AdamKernel pick_adam(int NB, int SPn) {
  if (NB <= 32) return pick_sp<32>(SPn);
  if (NB <= 48) return pick_sp<48>(SPn);
  if (NB <= 64) return pick_sp<64>(SPn);
  if (NB <= 80) return pick_sp<80>(SPn);
  if (NB <= 96) return pick_sp<96>(SPn);
  if (NB <= 112) return pick_sp<112>(SPn);
  if (NB <= 128) return pick_sp<128>(SPn);
  return {nullptr, 0};
}

static int num_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
  return cus > 0 ? cus : 256;
}

static void adam_geometry(int N, int L, int NB, int& S, int& G, int& ng, int& LG) {
  const int cus = num_cus();
  S = (N + cus - 1) / cus;
  if (S < 1) S = 1;
  if (S == 3) S = 4;
  G = (N + S - 1) / S;
  ng = kThreads / NB;
  if (ng < 1) ng = 1;
  LG = (L + ng - 1) / ng;
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
  if (L <= 0 || L > kThreads || NB <= 0 || N <= 0) return 0;
  int S, G, ng, LG;
  adam_geometry(N, L, NB, S, G, ng, LG);
  if (S > kSMax || NB * S > kThreads) return 0;
  AdamKernel kern = pick_adam(NB, S);
  return (kern.fn != nullptr && kern.lds <= 160 * 1024) ? 1 : 0;
}

int pmg_mstep_adam(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                   const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                   const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                   void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(cfg && W && mu && nu && count && basis && yw && tw && stats && loss_hist && err_hist &&
                  workspace,
              "pmg_mstep_adam: null argument");
  PMG_REQUIRE(L > 0 && L <= kThreads, "pmg_mstep_adam: L=%d must be in [1, %d]", L, kThreads);
  PMG_REQUIRE(NB > 0 && N > 0, "pmg_mstep_adam: bad shape");
  int S, G, ng, LG;
  adam_geometry(N, L, NB, S, G, ng, LG);
  PMG_REQUIRE(S <= kSMax, "pmg_mstep_adam: N=%d needs %d neurons per workgroup (> %d)", N, S, kSMax);
  PMG_REQUIRE(NB * S <= kThreads, "pmg_mstep_adam: NB*S=%d > %d", NB * S, kThreads);
  AdamKernel kern = pick_adam(NB, S);
  PMG_REQUIRE(kern.fn != nullptr && kern.lds <= 160 * 1024,
              "pmg_mstep_adam: NB=%d unsupported (basis must fit registers + 160 KiB LDS)", NB);
  const int maxiter = cfg->maxiter > 1 ? cfg->maxiter : 1;
  PMG_REQUIRE(workspace_bytes >= adam_ws(G, maxiter, nullptr, nullptr),
              "pmg_mstep_adam: workspace too small");
  hipStream_t st = as_stream(stream);
  AdamWork w;
  adam_ws(G, maxiter, &w, workspace);
  {
    const size_t n = ((size_t)maxiter + kLag + 2) * G;
    hipLaunchKernelGGL(k_fill_u64, dim3(256), dim3(256), 0, st, w.lpart, n, kSentinel);
    PMG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_fill_u64, dim3(256), dim3(256), 0, st, w.gpart, n, kSentinel);
    PMG_LAUNCH_CHECK();
  }
  PMG_HIP(hipMemsetAsync(w.timeout, 0, sizeof(int), st));
  PMG_HIP(hipMemsetAsync(loss_hist, 0, sizeof(double) * (size_t)maxiter, st));
  PMG_HIP(hipMemsetAsync(err_hist, 0, sizeof(double) * (size_t)maxiter, st));
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
  p.ring = w.ring;
  PMG_HIP(hipMemsetAsync(stats, 0, 4 * sizeof(double), st));
  if (kern.lds > 64 * 1024)
    PMG_HIP(hipFuncSetAttribute((const void*)kern.fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)kern.lds));
  static long long* prof_buf = nullptr;   // debug: per-phase stamps (PMG_ADAM_PROF set)
  const bool prof = getenv("PMG_ADAM_PROF") != nullptr;
  if (prof) {
    if (!prof_buf) PMG_HIP(hipMalloc(&prof_buf, 64 * 8 * sizeof(long long)));
    PMG_HIP(hipMemsetAsync(prof_buf, 0, 64 * 8 * sizeof(long long), st));
    p.prof = prof_buf;
  } else {
    p.prof = nullptr;
  }
  hipLaunchKernelGGL(kern.fn, dim3(G), dim3(kThreadsAll), kern.lds, st, p);
  PMG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_adam_hist, dim3(64), dim3(64), 0, st, p);
  PMG_LAUNCH_CHECK();
  if (prof) {
    long long h[64 * 8];
    PMG_HIP(hipMemcpyAsync(h, prof_buf, sizeof(h), hipMemcpyDeviceToHost, st));
    PMG_HIP(hipStreamSynchronize(st));
    double acc[5] = {0, 0, 0, 0, 0};
    int n = 0;
    for (int k = 8; k + 1 < 64; ++k) {   // skip the pipeline fill
      if (h[k * 8 + 4] == 0 || h[(k + 1) * 8] == 0) break;
      for (int i = 0; i < 4; ++i) acc[i] += (double)(h[k * 8 + i + 1] - h[k * 8 + i]);
      acc[4] += (double)(h[(k + 1) * 8] - h[k * 8 + 4]);
      ++n;
    }
    if (n > 0)
      fprintf(stderr, "[pmg adam prof] bodies=%d ticks/body: rows %.0f | bar1 %.0f | update %.0f | "
              "sums+bar2+publish %.0f | loop %.0f\n", n, acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n,
              acc[4] / n);
  }
  return PMG_OK;
}

}  // extern "C"
