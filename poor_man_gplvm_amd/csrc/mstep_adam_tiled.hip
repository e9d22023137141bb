// Adam M-step for large shapes (L > 512 or NB > 128: BASELINE config C4, L = 1024,
// NB = 154), where the persistent one-launch kernel of mstep_adam.hip cannot hold a
// latent row per thread.  Same contract as pmg_mstep_adam: the whole
// fit_tuning_helper.make_adam_runner.run loop (fit_tuning_helper.py:133-194) on
// poisson_m_step_objective (:63-81) with optax 0.2.2 adam, the stop rule
//   i < maxiter-1 and (i < 5 or |loss-loss_prev|/max(|loss|,1e-8) > tol)
// decided on the device from fixed-order f64 sums (bit-identical on every rank of a
// time-sharded fit, which runs this loop replicated).
//
// One body = four launches on the caller's stream:
//   k_at_rows    F = B W (f64 LDS-tiled GEMM, 32 latents x 32 neurons per workgroup),
//                f = softplus(F), G = (y_w/(f+1e-20) - t_w) sigmoid(F) -> G (L,N) f64,
//                per-workgroup partial of sum[xlogy(y_w, f+1e-20) - f t_w]
//   k_at_grad    partial B^T G over 8 slices of L (16 basis x 64 neurons per workgroup)
//   k_at_update  g = -B^T G + W/sd^2 (slices summed in order), partials of |g|^2 and
//                of the log prior at the evaluated W, then the optax update of
//                (W, mu, nu) in place (skipped on the initial evaluation)
//   k_at_ctrl    one workgroup: fixed-order sums -> loss, |g|; histories; stop decision
// Every kernel returns immediately once the decision is "stop", so the host enqueues
// bodies in batches of kBatch and reads the decision word once per batch.
#include <math.h>

#include "pmg_common.h"

namespace pmg {

constexpr int kAtBatch = 16;
// Small tiles on purpose: at C4 one body is ~160 M f64 FMAs per GEMM, too little to
// hide a global-load round trip inside a workgroup, so latency is hidden ACROSS
// workgroups (4-5 resident per CU); LDS reads are mostly broadcasts (cheap).
constexpr int kRowTM = 32, kRowTN = 32, kRowTK = 16;    // k_at_rows tile (4 outputs / thread)
constexpr int kGradTK = 16, kGradTN = 64, kGradTL = 32; // k_at_grad tile (4 outputs / thread)
constexpr int kGradSplit = 8;                           // split of the L reduction

struct AtCtrl {
  int active;   // 1 while the loop runs (the decision for the NEXT body)
  int i;        // optax loop counter of the reference
  int pad[2];
  double loss, loss_prev, err;
};

struct AtParams {
  double* W;
  double* mu;
  double* nu;
  int64_t* count;
  const float* basis;  // (L, NB)
  const double* yw;    // (L, N)
  const double* tw;    // (L)
  int L, NB, N;
  double lr, b1, b2, eps, eps_root, prior_std, tol;
  int maxiter;
  double* stats;
  double* loss_hist;
  double* err_hist;
  AtCtrl* ctrl;
  double* G;      // (L, N)
  double* gsplit; // [kGradSplit][NB][N] partial B^T G
  double* lpart;  // [gridRows]
  double* epart;  // [gridGrad]
  double* ppart;  // [gridGrad]
  int n_lpart, n_gpart;
};

__device__ __forceinline__ double at_sigmoid(double x) { return 1.0 / (1.0 + exp(-x)); }

// fixed-order block sum of one double per thread (NT threads)
template <int NT = 256>
__device__ __forceinline__ double block_sum(double v, double* sm) {
  sm[threadIdx.x] = v;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sm[threadIdx.x] += sm[threadIdx.x + o];
    __syncthreads();
  }
  const double r = sm[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(256) k_at_rows(AtParams p) {
  if (!p.ctrl->active) return;
  __shared__ double sB[kRowTK][kRowTM];
  __shared__ double sW[kRowTK][kRowTN];
  __shared__ double sm[256];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int n0 = blockIdx.x * kRowTN, l0 = blockIdx.y * kRowTM;
  double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  for (int k0 = 0; k0 < p.NB; k0 += kRowTK) {
    for (int e = threadIdx.x; e < kRowTK * kRowTM; e += 256) {
      const int l = e / kRowTK, k = e % kRowTK;   // consecutive threads walk k (contiguous in B)
      const int gl = l0 + l, gk = k0 + k;
      sB[k][l] = (gl < p.L && gk < p.NB) ? (double)p.basis[(size_t)gl * p.NB + gk] : 0.0;
    }
    for (int e = threadIdx.x; e < kRowTK * kRowTN; e += 256) {
      const int k = e / kRowTN, n = e % kRowTN;
      const int gk = k0 + k, gn = n0 + n;
      sW[k][n] = (gk < p.NB && gn < p.N) ? p.W[(size_t)gk * p.N + gn] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRowTK; ++k) {
      const double b0 = sB[k][ty], b1 = sB[k][ty + 16];
      const double w0 = sW[k][tx], w1 = sW[k][tx + 16];
      acc[0][0] = fma(b0, w0, acc[0][0]);
      acc[0][1] = fma(b0, w1, acc[0][1]);
      acc[1][0] = fma(b1, w0, acc[1][0]);
      acc[1][1] = fma(b1, w1, acc[1][1]);
    }
    __syncthreads();
  }
  double part = 0.0;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int l = l0 + ty + 16 * a;
    if (l >= p.L) continue;
    const double twl = p.tw[l];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int n = n0 + tx + 16 * c;
      if (n >= p.N) continue;
      const double F = acc[a][c];
      const double ex = exp(-fabs(F));                 // shared by softplus and sigmoid
      const double f = fmax(F, 0.0) + log1p(ex);        // jax softplus = logaddexp(F, 0)
      const double sg = F >= 0.0 ? 1.0 / (1.0 + ex) : ex / (1.0 + ex);
      const double fe = f + 1e-20;
      const double y = p.yw[(size_t)l * p.N + n];
      p.G[(size_t)l * p.N + n] = (y / fe - twl) * sg;
      part += (y == 0.0 ? 0.0 : y * log(fe)) - f * twl;
    }
  }
  const double s = block_sum(part, sm);
  if (threadIdx.x == 0) p.lpart[blockIdx.y * gridDim.x + blockIdx.x] = s;
}

// partial B^T G over one L-slice (blockIdx.z): 16 basis rows x 64 neurons per workgroup
__global__ void __launch_bounds__(256) k_at_grad(AtParams p) {
  if (!p.ctrl->active) return;
  __shared__ double sG[kGradTL][kGradTN];
  __shared__ double sB[kGradTL][kGradTK + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // ty: basis row, tx: 4 neurons
  const int n0 = blockIdx.x * kGradTN, k0 = blockIdx.y * kGradTK;
  const int span = (p.L + kGradSplit - 1) / kGradSplit;
  const int la = blockIdx.z * span, lb = min(p.L, la + span);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int l0 = la; l0 < lb; l0 += kGradTL) {
    for (int e = threadIdx.x; e < kGradTL * kGradTN; e += 256) {
      const int l = e / kGradTN, n = e % kGradTN;
      const int gl = l0 + l, gn = n0 + n;
      sG[l][n] = (gl < lb && gn < p.N) ? p.G[(size_t)gl * p.N + gn] : 0.0;
    }
    for (int e = threadIdx.x; e < kGradTL * kGradTK; e += 256) {
      const int l = e / kGradTK, k = e % kGradTK;
      const int gl = l0 + l, gk = k0 + k;
      sB[l][k] = (gl < lb && gk < p.NB) ? (double)p.basis[(size_t)gl * p.NB + gk] : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int l = 0; l < kGradTL; ++l) {
      const double b = sB[l][ty];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = fma(b, sG[l][tx + 16 * c], acc[c]);
    }
    __syncthreads();
  }
  const int k = k0 + ty;
  if (k >= p.NB) return;
  double* out = p.gsplit + ((size_t)blockIdx.z * p.NB + k) * p.N;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int n = n0 + tx + 16 * c;
    if (n < p.N) out[n] = acc[c];
  }
}

// g = -sum_z gsplit[z] + W/sd^2 (fixed order), |g|^2 and log-prior partials at the
// evaluated W, then the optax 0.2.2 update of (W, mu, nu) in place when `update`
__global__ void __launch_bounds__(256) k_at_update(AtParams p, int update) {
  if (!p.ctrl->active) return;
  __shared__ double sm[256];
  const size_t tot = (size_t)p.NB * p.N;
  const size_t o = (size_t)blockIdx.x * 256 + threadIdx.x;
  double e2 = 0.0, lpr = 0.0;
  if (o < tot) {
    double gs = 0.0;
#pragma unroll
    for (int z = 0; z < kGradSplit; ++z) gs += p.gsplit[(size_t)z * tot + o];
    const double sd = p.prior_std, isd2 = 1.0 / (sd * sd);
    const double w = p.W[o];
    const double g = -gs + w * isd2;
    e2 = g * g;
    const double zz = w / sd;
    lpr = -0.5 * zz * zz - log(sd) - 0.5 * log(2.0 * M_PI);
    if (update) {
      const int64_t cnt = *p.count + 1;
      const double bc1 = 1.0 - pow(p.b1, (double)cnt), bc2 = 1.0 - pow(p.b2, (double)cnt);
      const double m = (1.0 - p.b1) * g + p.b1 * p.mu[o];
      const double v = (1.0 - p.b2) * g * g + p.b2 * p.nu[o];
      p.mu[o] = m;
      p.nu[o] = v;
      p.W[o] = w + (-p.lr) * ((m / bc1) / (sqrt(v / bc2 + p.eps_root) + p.eps));
    }
  }
  const double se = block_sum(e2, sm);
  const double sp = block_sum(lpr, sm);
  if (threadIdx.x == 0) {
    p.epart[blockIdx.x] = se;
    p.ppart[blockIdx.x] = sp;
  }
}

__global__ void k_at_start(AtCtrl* c) {
  c->active = 1;
  c->i = 0;
}

// mode 0: initial evaluation (histories[0], loss_prev = loss); mode 1: after a body
__global__ void __launch_bounds__(256) k_at_ctrl(AtParams p, int mode) {
  AtCtrl* c = p.ctrl;
  if (!c->active) return;
  __shared__ double sm[256];
  double a = 0.0, b = 0.0, e = 0.0;
  for (int q = threadIdx.x; q < p.n_lpart; q += 256) a += p.lpart[q];
  for (int q = threadIdx.x; q < p.n_gpart; q += 256) {
    b += p.ppart[q];
    e += p.epart[q];
  }
  const double ll = block_sum(a, sm);
  const double lpr = block_sum(b, sm);
  const double e2 = block_sum(e, sm);
  if (threadIdx.x != 0) return;
  const double loss = -ll - lpr;
  const double err = sqrt(e2);
  int i = c->i;
  if (mode == 0) {
    c->loss = loss;
    c->loss_prev = loss;
    c->err = err;
    p.loss_hist[0] = loss;
    p.err_hist[0] = err;
  } else {
    i += 1;
    c->i = i;
    p.loss_hist[i] = loss;
    p.err_hist[i] = err;
    c->loss_prev = c->loss;
    c->loss = loss;
    c->err = err;
    *p.count += 1;
  }
  const double L0 = c->loss, Lp = c->loss_prev;
  // tol < 0: no early stop (speculative batches), also not on a NaN loss
  const bool go = (i < p.maxiter - 1) && (i < 5 || p.tol < 0.0 || fabs(L0 - Lp) / fmax(fabs(L0), 1e-8) > p.tol);
  p.stats[0] = (double)(i + 1);
  p.stats[1] = L0;
  p.stats[2] = c->err;
  c->active = go ? 1 : 0;
}

static size_t at_ws(int L, int NB, int N, AtParams* p, void* base) {
  const int gr = ((N + kRowTN - 1) / kRowTN) * ((L + kRowTM - 1) / kRowTM);
  const int gg = (int)(((size_t)NB * N + 255) / 256);
  Carver c(base);
  AtCtrl* ctrl = c.take<AtCtrl>(1);
  double* G = c.take<double>((size_t)L * N);
  double* gs = c.take<double>((size_t)kGradSplit * NB * N);
  double* lp = c.take<double>(gr);
  double* ep = c.take<double>(gg);
  double* pp = c.take<double>(gg);
  if (p) {
    p->ctrl = ctrl;
    p->G = G;
    p->gsplit = gs;
    p->lpart = lp;
    p->epart = ep;
    p->ppart = pp;
    p->n_lpart = gr;
    p->n_gpart = gg;
  }
  return c.off + 256;
}

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_mstep_tiled_workspace_size(int32_t L, int32_t NB, int32_t N) {
  if (L <= 0 || NB <= 0 || N <= 0) return 0;
  return at_ws(L, NB, N, nullptr, nullptr);
}

int pmg_mstep_adam_tiled(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                         const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                         const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                         void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(cfg && W && mu && nu && count && basis && yw && tw && stats && loss_hist && err_hist &&
                  workspace,
              "pmg_mstep_adam_tiled: null argument");
  PMG_REQUIRE(L > 0 && NB > 0 && N > 0, "pmg_mstep_adam_tiled: bad shape");
  PMG_REQUIRE(workspace_bytes >= at_ws(L, NB, N, nullptr, nullptr), "pmg_mstep_adam_tiled: workspace too small");
  hipStream_t st = as_stream(stream);
  AtParams p;
  memset(&p, 0, sizeof(p));
  at_ws(L, NB, N, &p, workspace);
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
  p.lr = cfg->lr;
  p.b1 = cfg->b1;
  p.b2 = cfg->b2;
  p.eps = cfg->eps;
  p.eps_root = cfg->eps_root;
  p.prior_std = cfg->prior_std;
  p.tol = cfg->tol;
  p.maxiter = cfg->maxiter > 1 ? cfg->maxiter : 1;
  p.stats = stats;
  p.loss_hist = loss_hist;
  p.err_hist = err_hist;
  PMG_HIP(hipMemsetAsync(loss_hist, 0, sizeof(double) * (size_t)p.maxiter, st));
  PMG_HIP(hipMemsetAsync(err_hist, 0, sizeof(double) * (size_t)p.maxiter, st));
  PMG_HIP(hipMemsetAsync(stats, 0, 4 * sizeof(double), st));
  const dim3 grow((N + kRowTN - 1) / kRowTN, (L + kRowTM - 1) / kRowTM);
  const dim3 ggrad((N + kGradTN - 1) / kGradTN, (NB + kGradTK - 1) / kGradTK, kGradSplit);
  const dim3 gupd((unsigned)(((size_t)NB * N + 255) / 256));
  hipLaunchKernelGGL(k_at_start, dim3(1), dim3(1), 0, st, p.ctrl);
  PMG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_at_rows, grow, dim3(256), 0, st, p);
  hipLaunchKernelGGL(k_at_grad, ggrad, dim3(256), 0, st, p);
  hipLaunchKernelGGL(k_at_update, gupd, dim3(256), 0, st, p, 0);
  hipLaunchKernelGGL(k_at_ctrl, dim3(1), dim3(256), 0, st, p, 0);
  PMG_LAUNCH_CHECK();
  int active = 1;
  for (int done = 0; done < p.maxiter - 1 && active;) {
    const int nb = (p.maxiter - 1 - done) < kAtBatch ? (p.maxiter - 1 - done) : kAtBatch;
    for (int b = 0; b < nb; ++b) {
      hipLaunchKernelGGL(k_at_rows, grow, dim3(256), 0, st, p);
      hipLaunchKernelGGL(k_at_grad, ggrad, dim3(256), 0, st, p);
      hipLaunchKernelGGL(k_at_update, gupd, dim3(256), 0, st, p, 1);
      hipLaunchKernelGGL(k_at_ctrl, dim3(1), dim3(256), 0, st, p, 1);
    }
    PMG_LAUNCH_CHECK();
    done += nb;
    PMG_HIP(hipMemcpyAsync(&active, &p.ctrl->active, sizeof(int), hipMemcpyDeviceToHost, st));
    PMG_HIP(hipStreamSynchronize(st));
  }
  return PMG_OK;
}

}  // extern "C"
