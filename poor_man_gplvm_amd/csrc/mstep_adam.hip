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
#include "pmg_common.h"

namespace pmg {

constexpr int kLag = 2;
constexpr int kRing = kLag + 2;
constexpr int kSMax = 4;        // neurons per workgroup
constexpr int kThreads = 512;   // L <= 512

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
  unsigned* cnt;            // [maxiter]
  unsigned long long* lpart;  // [maxiter][G] f64 bits
  unsigned long long* gpart;  // [maxiter][G]
  int* timeout;
};

__device__ __forceinline__ void st_sc1(unsigned long long* p, double v) {
  __hip_atomic_store(p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const unsigned long long* p) {
  return __longlong_as_double((long long)__hip_atomic_load(const_cast<unsigned long long*>(p),
                                                           __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
}

template <int NBM, int LGM>
__global__ void __launch_bounds__(kThreads) k_adam(AdamParams p) {
  __shared__ float sW[NBM * kSMax];               // current W (f32) for f = B W
  __shared__ float sGr[kThreads * kSMax];         // G[l][n]
  __shared__ float sRed[kThreads * kSMax];        // group partials of B^T G
  __shared__ double sRing[kRing][3][NBM * kSMax]; // (W, mu, nu) after each body
  __shared__ double sSum[2][kThreads / 64];
  __shared__ int sCtl[4];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.x;
  const int n0 = g * p.S;
  const int S = (p.N - n0) < p.S ? (p.N - n0) : p.S;  // neurons owned
  const int L = p.L, NB = p.NB;
  const double sd = p.prior_std, isd2 = 1.0 / (sd * sd);
  const double lconst = log(sd) + 0.5 * log(2.0 * M_PI);

  // ---- one-time loads -------------------------------------------------------
  float brow[NBM];
  const bool is_row = tid < L;
#pragma unroll
  for (int k = 0; k < NBM; ++k) brow[k] = (is_row && k < NB) ? p.basis[(size_t)tid * NB + k] : 0.f;
  const int kk = tid % NB, grp = tid / NB;
  const bool is_col = grp < p.ng;
  const int lbeg = grp * p.LG;
  float bcol[LGM];
#pragma unroll
  for (int i = 0; i < LGM; ++i) {
    const int l = lbeg + i;
    bcol[i] = (is_col && i < p.LG && l < L) ? p.basis[(size_t)l * NB + kk] : 0.f;
  }
  float ywf[kSMax];
  double ywd[kSMax];
  double twd = 0.0;
#pragma unroll
  for (int s = 0; s < kSMax; ++s) {
    ywd[s] = (is_row && s < S) ? p.yw[(size_t)tid * p.N + n0 + s] : 0.0;
    ywf[s] = (float)ywd[s];
  }
  if (is_row) twd = p.tw[tid];
  const float twf = (float)twd;
  // element role: (ek, en) owns W[ek][n0+en]
  const int ek = tid % NB, en = tid / NB;
  const bool is_el = en < S;
  for (int q = tid; q < NBM * kSMax; q += blockDim.x) sW[q] = 0.f;
  if (tid < 4) sCtl[tid] = 0;
  __syncthreads();
  if (is_el) {
    const size_t o = (size_t)ek * p.N + n0 + en;
    sRing[0][0][ek * kSMax + en] = p.W[o];
    sRing[0][1][ek * kSMax + en] = p.mu[o];
    sRing[0][2][ek * kSMax + en] = p.nu[o];
    sW[ek * kSMax + en] = (float)p.W[o];
  }
  const int64_t count0 = p.count[0];
  __syncthreads();

  double loss_prev = 0.0, loss0 = 0.0;
  int next_j = 0;          // next body whose global loss is undecided
  int stop_j = -1;         // body after which the loop stops
  double fin_loss = 0.0, fin_err = 0.0;
  const int maxiter = p.maxiter;
  const bool eval_only = maxiter <= 1;

  for (int k = 0;; ++k) {
    const int slot = k % kRing;
    // ---- body k: evaluate at W_k ---------------------------------------------
    double lpart = 0.0;
    if (is_row) {
#pragma unroll
      for (int s = 0; s < kSMax; ++s) {
        if (s < S) {
          float F = 0.f;
#pragma unroll
          for (int q = 0; q < NBM; ++q) F = fmaf(brow[q], sW[q * kSMax + s], F);
          const float f = softplus_f(F);
          const float sg = sigmoid_f(F);
          sGr[tid * kSMax + s] = (ywf[s] / (f + 1e-20f) - twf) * sg;
          const double fd = (double)f;
          const double xl = (ywd[s] != 0.0) ? ywd[s] * log(fd + 1e-20) : 0.0;
          lpart -= xl - fd * twd;
        }
      }
    }
    __syncthreads();
    if (is_col) {
#pragma unroll
      for (int s = 0; s < kSMax; ++s) {
        if (s < S) {
          float acc = 0.f;
#pragma unroll
          for (int i = 0; i < LGM; ++i) {
            const int l = lbeg + i;
            if (i < p.LG && l < L) acc = fmaf(bcol[i], sGr[l * kSMax + s], acc);
          }
          sRed[(grp * NB + kk) * kSMax + s] = acc;
        }
      }
    }
    __syncthreads();
    double gsq = 0.0;
    if (is_el) {
      float gsum = 0.f;
      for (int q = 0; q < p.ng; ++q) gsum += sRed[(q * NB + ek) * kSMax + en];
      const int e = ek * kSMax + en;
      const double w = sRing[slot][0][e];
      const double gr = -(double)gsum + w * isd2;
      gsq = gr * gr;
      lpart += 0.5 * w * w * isd2 + lconst;
      // optax 0.2.2 scale_by_adam + scale(-lr)
      const double cnt = (double)(count0 + k + 1);
      const double mu = (1.0 - p.b1) * gr + p.b1 * sRing[slot][1][e];
      const double nu = (1.0 - p.b2) * gr * gr + p.b2 * sRing[slot][2][e];
      const double mh = mu / (1.0 - pow(p.b1, cnt));
      const double nh = nu / (1.0 - pow(p.b2, cnt));
      const double wn = w - p.lr * (mh / (sqrt(nh + p.eps_root) + p.eps));
      const int ns = (k + 1) % kRing;
      sRing[ns][0][e] = eval_only ? w : wn;
      sRing[ns][1][e] = eval_only ? sRing[slot][1][e] : mu;
      sRing[ns][2][e] = eval_only ? sRing[slot][2][e] : nu;
    }
    // block sums of the partial loss and squared gradient
    lpart = wave_sum_f64(lpart);
    gsq = wave_sum_f64(gsq);
    if (lane == 0) {
      sSum[0][wid] = lpart;
      sSum[1][wid] = gsq;
    }
    __syncthreads();
    if (tid == 0) {
      double a = 0.0, b = 0.0;
      for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
        a += sSum[0][q];
        b += sSum[1][q];
      }
      st_sc1(&p.lpart[(size_t)k * p.G + g], a);
      st_sc1(&p.gpart[(size_t)k * p.G + g], b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&p.cnt[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (is_el) sW[ek * kSMax + en] = (float)sRing[(k + 1) % kRing][0][ek * kSMax + en];
    __syncthreads();

    // ---- decide bodies whose partials are (or must be) complete --------------
    const int last_decidable = eval_only ? k : k - kLag;
    while (stop_j < 0 && next_j <= last_decidable && next_j < maxiter) {
      const int j = next_j;
      if (wid == 0) {
        if (lane == 0) {
          unsigned spins = 0;
          while (__hip_atomic_load(&p.cnt[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                 (unsigned)p.G) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 26)) {
              atomicOr(p.timeout, 1);
              sCtl[2] = 1;
              break;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double a = 0.0, b = 0.0;
        for (int q = lane; q < p.G; q += 64) {
          a += ld_sc1(&p.lpart[(size_t)j * p.G + q]);
          b += ld_sc1(&p.gpart[(size_t)j * p.G + q]);
        }
        a = wave_sum_f64(a);
        b = wave_sum_f64(b);
        if (lane == 0) {
          const double loss = a, err = sqrt(b);
          if (j == 0) {
            loss0 = loss;
            loss_prev = loss;
            if (g == 0) {
              p.loss_hist[0] = loss;
              p.err_hist[0] = err;
            }
          }
          bool cont;
          if (eval_only) {
            cont = false;
          } else {
            if (g == 0 && j + 1 < maxiter) {
              p.loss_hist[j + 1] = loss;
              p.err_hist[j + 1] = err;
            }
            const double rel = fabs(loss - loss_prev) / fmax(fabs(loss), 1e-8);
            cont = (j + 1 < maxiter - 1) && ((j + 1 < 5) || (rel > p.tol));
          }
          loss_prev = loss;
          sCtl[0] = cont ? 0 : 1;
          if (!cont) {
            fin_loss = loss;
            fin_err = err;
          }
        }
      }
      __syncthreads();
      if (sCtl[0]) stop_j = next_j;
      ++next_j;
      __syncthreads();
    }
    if (stop_j >= 0) break;
    if (sCtl[2]) break;  // a wait timed out (reported through p.timeout)
  }

  // ---- write the state after body stop_j (W_{stop_j+1}) -----------------------
  const int fs = eval_only ? (1 % kRing) : ((stop_j + 1) % kRing);
  if (is_el && stop_j >= 0) {
    const size_t o = (size_t)ek * p.N + n0 + en;
    const int e = ek * kSMax + en;
    p.W[o] = sRing[fs][0][e];
    p.mu[o] = sRing[fs][1][e];
    p.nu[o] = sRing[fs][2][e];
  }
  if (g == 0 && tid == 0 && stop_j >= 0) {
    const int n_iter = eval_only ? 1 : stop_j + 2;
    p.stats[0] = (double)n_iter;
    p.stats[1] = fin_loss;
    p.stats[2] = fin_err;
    p.stats[3] = loss0;
    p.count[0] = count0 + (eval_only ? 0 : (stop_j + 1));
  }
}

struct AdamWork {
  unsigned* cnt;
  unsigned long long* lpart;
  unsigned long long* gpart;
  int* timeout;
};

static size_t adam_ws(int G, int maxiter, AdamWork* w, void* base) {
  Carver c(base);
  AdamWork ww;
  ww.timeout = c.take<int>(64);
  ww.cnt = c.take<unsigned>((size_t)maxiter + kLag + 2);
  ww.lpart = c.take<unsigned long long>(((size_t)maxiter + kLag + 2) * G);
  ww.gpart = c.take<unsigned long long>(((size_t)maxiter + kLag + 2) * G);
  if (w) *w = ww;
  return c.off + 256;
}

typedef void (*adam_kernel_t)(AdamParams);

static adam_kernel_t pick_adam(int NB, int LG) {
  const int m = NB > LG ? NB : LG;
  if (m <= 32) return k_adam<32, 32>;
  if (m <= 64) return k_adam<64, 64>;
  if (m <= 96) return k_adam<96, 96>;
  if (m <= 128) return k_adam<128, 128>;
  return nullptr;
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
  adam_kernel_t kern = pick_adam(NB, LG);
  PMG_REQUIRE(kern != nullptr, "pmg_mstep_adam: NB=%d / row group %d > 128 unsupported", NB, LG);
  const int maxiter = cfg->maxiter > 1 ? cfg->maxiter : 1;
  PMG_REQUIRE(workspace_bytes >= adam_ws(G, maxiter, nullptr, nullptr),
              "pmg_mstep_adam: workspace too small");
  hipStream_t st = as_stream(stream);
  AdamWork w;
  adam_ws(G, maxiter, &w, workspace);
  PMG_HIP(hipMemsetAsync(w.cnt, 0, sizeof(unsigned) * ((size_t)maxiter + kLag + 2), st));
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
  p.cnt = w.cnt;
  p.lpart = w.lpart;
  p.gpart = w.gpart;
  p.timeout = w.timeout;
  hipLaunchKernelGGL(kern, dim3(G), dim3(kThreads), 0, st, p);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // extern "C"
