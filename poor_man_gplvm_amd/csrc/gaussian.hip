// Gaussian observation model (GaussianGPLVMJump1D, reference core.py:852-917):
//   tuning   = basis @ W                         fit_tuning_helper.get_tuning_linear (:12-17)
//   emission = sum_n m[t,n] norm.logpdf(y, tuning*dt, noise_std)
//                                                decoder.get_loglikelihood_ma_gaussian (:50-57)
//   M-step   = (B^T diag(t_w) B / s^2 + I / p^2) W = B^T y_w / s^2
//                                                fit_tuning_helper.gaussian_m_step_analytic (:44-61)
// The fwd-bwd scan and the sufficient statistics are the Poisson path's kernels: the
// emission writes the same (delta, rblk) split, so the scans do not know the model.
#include <math.h>

#include "pmg_common.h"

namespace pmg {

// tuning[l,n] = sum_b basis[l,b] W[b,n] (f64); one thread per (l, n), W row reads coalesced in n.
__global__ void __launch_bounds__(256) k_tuning_linear(const float* __restrict__ basis,
                                                       const double* __restrict__ W, int L, int NB, int N,
                                                       double* __restrict__ t64, float* __restrict__ t32) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int l = blockIdx.y;
  if (n >= N) return;
  const float* b = basis + (size_t)l * NB;
  double a = 0.0;
  for (int k = 0; k < NB; ++k) a = fma((double)b[k], W[(size_t)k * N + n], a);
  if (t64) t64[(size_t)l * N + n] = a;
  if (t32) t32[(size_t)l * N + n] = (float)a;
}

// ll[t,l] = sum_n m[t,n] (c0 - 0.5 ((y - mu) / s)^2),  mu = tuning dt,  c0 = -log(s) - 0.5 log(2 pi)
// (jax.scipy.stats.norm.logpdf), -1e20 where ma_latent == 0.  Expanded into two dense
// contractions over neurons plus a per-time-bin constant:
//   ll = q_t + (1/s^2) [(m*y) mu^T]_tl - (1/2s^2) [m (mu^2)^T]_tl,   q_t = sum_n m (c0 - y^2/2s^2)
// both contractions on the f64 MFMA (v_mfma_f64_16x16x4_f64, full f64: same numbers as an
// f64 dot product up to summation order).  Block = 4 waves, tile 64 time bins x 64 latents,
// neurons staged through LDS 32 at a time; wave w owns time rows 16w..16w+15 and all four
// 16-latent sub-tiles.  Operand maps (cdna_hip_programming.md, f64 16x16x4): A lane l =
// A[l&15][k=l>>4], B lane l = B[k=l>>4][l&15], D reg r of lane l = D[(l>>4)+4r][l&15].
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_emission_gaussian(
    const float* __restrict__ y, const float* __restrict__ ma, int ma_2d, const double* __restrict__ tuning,
    const uint8_t* __restrict__ ma_latent, double inv_s, double c0, double dt, const double* __restrict__ dt_t,
    int64_t T, int L, int N, int Lp, float* __restrict__ delta, double* __restrict__ rblk,
    double* __restrict__ ll64) {
  __shared__ float sY[64][33];     // y and m stay f32 (their f64 product is exact)
  __shared__ float sM[64][33];
  __shared__ double sTu[32][65];   // mu = tuning * dt (f64); mu^2 is formed at use
  __shared__ double sQs[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * 64;
  const int l0 = blockIdx.y * 64;
  const double inv_s2 = inv_s * inv_s;
  f64x4 acc_a[4], acc_b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    acc_a[s] = (f64x4){0.0, 0.0, 0.0, 0.0};
    acc_b[s] = (f64x4){0.0, 0.0, 0.0, 0.0};
  }
  double q[4] = {0, 0, 0, 0};
  const int ar = 16 * w + (lane & 15);   // A row (time) this lane feeds
  const int kq = lane >> 4;               // k index within a 4-step
  for (int n0 = 0; n0 < N; n0 += 32) {
    {   // thread -> (time row tt, 8 consecutive neurons); the q_t partial is summed in
        // registers and over the 4 lanes sharing a row (no LDS array, no division)
      const int tt = threadIdx.x >> 2, nb = (threadIdx.x & 3) * 8;
      const int64_t t = t0 + tt;
      double qp = 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = n0 + nb + i;
        double yv = 0.0, mv = 0.0;
        if (t < T && n < N) {
          yv = y[t * N + n];
          mv = ma ? (ma_2d ? ma[t * N + n] : ma[n]) : 1.0;
        }
        sY[tt][nb + i] = (float)yv;
        sM[tt][nb + i] = (float)mv;
        qp = fma(mv, fma(-0.5 * inv_s2 * yv, yv, c0), qp);
      }
      qp += __shfl_xor(qp, 1, 64);
      qp += __shfl_xor(qp, 2, 64);
      if ((threadIdx.x & 3) == 0) sQs[tt] = qp;
    }
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {   // n fastest: coalesced tuning rows
      const int nn = e & 31, ll = e >> 5;
      const int n = n0 + nn, l = l0 + ll;
      const double mu = (n < N && l < L) ? tuning[(size_t)l * N + n] * dt : 0.0;
      sTu[nn][ll] = mu;
    }
    __syncthreads();
#pragma unroll
    for (int k0 = 0; k0 < 32; k0 += 4) {
      const double bm = (double)sM[ar][k0 + kq];
      const double am = bm * (double)sY[ar][k0 + kq];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double mu = sTu[k0 + kq][16 * s + (lane & 15)];
        acc_a[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(am, mu, acc_a[s], 0, 0, 0);
        acc_b[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(bm, mu * mu, acc_b[s], 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] += sQs[16 * w + (lane >> 4) + 4 * r];
  }
  const int nblk = Lp >> 5;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t t = t0 + 16 * w + (lane >> 4) + 4 * r;
#pragma unroll
    for (int h = 0; h < 2; ++h) {          // 32-latent block = sub-tiles 2h, 2h+1
      double v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int s = 2 * h + u;
        const int l = l0 + 16 * s + (lane & 15);
        double x = -INFINITY;
        if (l < L && t < T) {
          // per-time-bin dt (decoder.py:73-85): mu = tuning dt_t, so the contractions (run
          // with dt = 1) scale by dt_t and dt_t^2
          const double d = dt_t ? dt_t[t] : 1.0;
          x = q[r] + inv_s2 * d * acc_a[s][r] - 0.5 * inv_s2 * (d * d) * acc_b[s][r];
          if (ma_latent && ma_latent[l] == 0) x = -1e20;
        }
        v[u] = x;
      }
      double mx = fmax(v[0], v[1]);
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
      if (t < T) {
        const int lb = l0 + 32 * h;
        if ((lane & 15) == 0 && lb < Lp) rblk[t * nblk + (lb >> 5)] = mx;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int l = lb + 16 * u + (lane & 15);
          if (l < L) delta[t * (int64_t)L + l] = (float)(v[u] - mx);
          if (ll64 && l < L) ll64[t * (int64_t)L + l] = v[u];
        }
      }
    }
  }
}

// Normal equations.  Column c < N:  R[d,c] = sum_l B[l,d] yw[l,c] / s^2   (the right-hand side)
//                    column N + b:  H[d,b] = sum_l B[l,d] tw[l] B[l,b] / s^2 + (d==b) / p^2
// One thread per output, written to ws as [NB][N + NB] (f64).
__global__ void __launch_bounds__(256) k_gauss_normal_eq(const float* __restrict__ basis,
                                                         const double* __restrict__ yw,
                                                         const double* __restrict__ tw, int L, int NB, int N,
                                                         double inv_s2, double inv_p2, double* __restrict__ ws) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int d = blockIdx.y;
  const int C = N + NB;
  if (c >= C) return;
  double a = 0.0;
  if (c < N) {
    for (int l = 0; l < L; ++l) a = fma((double)basis[(size_t)l * NB + d], yw[(size_t)l * N + c], a);
    a *= inv_s2;
  } else {
    const int b = c - N;
    for (int l = 0; l < L; ++l)
      a = fma((double)basis[(size_t)l * NB + d] * tw[l], (double)basis[(size_t)l * NB + b], a);
    a = a * inv_s2 + (d == b ? inv_p2 : 0.0);
  }
  ws[(size_t)d * C + c] = a;
}

__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }   // j <= i

// Cholesky of H (packed lower triangle in LDS, f64), then Linv = L^{-1} (row-major NB x NB,
// zero above the diagonal) by one column solve per thread.  One workgroup: NB^3/6 flops for
// the factor and NB^3/6 for the inverse, with no dependency chain longer than NB^2 per
// thread.  A non-positive pivot sets the (sticky) status word, which the host checks
// once per fit, and fills Linv with NaN, so W = NaN: a failed solve never leaves a
// plausible W built from an older inverse.
__global__ void __launch_bounds__(256) k_gauss_chol_inv(const double* __restrict__ ws, int NB, int N,
                                                        double* __restrict__ Linv, int* __restrict__ status,
                                                        int x_in_lds) {
  extern __shared__ double sA[];
  const int C = N + NB;
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB; e += 256) {
    const int i = e / NB, j = e % NB;
    if (j <= i) sA[tri(i, j)] = ws[(size_t)i * C + N + j];
  }
  __syncthreads();
  for (int k = 0; k < NB; ++k) {
    const double piv = sA[tri(k, k)];
    __syncthreads();
    if (!(piv > 0.0)) {   // uniform across the workgroup: every thread read the same pivot
      if (tid == 0) status[0] = 1;
      for (int e = tid; e < NB * NB; e += 256) Linv[e] = __builtin_nan("");
      return;
    }
    const double r = sqrt(piv);
    for (int i = k + 1 + tid; i < NB; i += 256) sA[tri(i, k)] /= r;
    if (tid == 0) sA[tri(k, k)] = r;
    __syncthreads();
    const int m = NB - k - 1;
    for (int e = tid; e < m * m; e += 256) {
      const int i = k + 1 + e / m, j = k + 1 + e % m;
      if (j <= i) sA[tri(i, j)] -= sA[tri(i, k)] * sA[tri(j, k)];
    }
    __syncthreads();
  }
  // the inverse is built in LDS when it fits next to the factor (NB <= 118), else in place
  // in global memory; a column's values are re-read by the thread that wrote them
  double* X = x_in_lds ? sA + NB * (NB + 1) / 2 : Linv;
  for (int j = tid; j < NB; j += 256) {   // column j of L^{-1}: L x = e_j
    for (int i = 0; i < j; ++i) X[(size_t)i * NB + j] = 0.0;
    for (int i = j; i < NB; ++i) {
      double v = (i == j) ? 1.0 : 0.0;
      for (int k = j; k < i; ++k) v -= sA[tri(i, k)] * X[(size_t)k * NB + j];
      X[(size_t)i * NB + j] = v / sA[tri(i, i)];
    }
  }
  if (x_in_lds) {
    __syncthreads();
    for (int e = tid; e < NB * NB; e += 256) Linv[e] = X[e];
  }
}

// Triangular products of the solve W = L^{-T} (L^{-1} R), one thread per output (d, n):
//   trans = 0:  out[d,n] = sum_{k<=d} Linv[d,k] X[k,n]
//   trans = 1:  out[d,n] = sum_{k>=d} Linv[k,d] X[k,n]
// X rows have stride ldx; Linv reads are uniform across the workgroup (same d).
__global__ void __launch_bounds__(256) k_gauss_tri_mm(const double* __restrict__ Linv,
                                                      const double* __restrict__ X, int64_t ldx, int NB, int N,
                                                      int trans, double* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int d = blockIdx.y;
  if (n >= N) return;
  double a = 0.0;
  if (!trans) {
    for (int k = 0; k <= d; ++k) a = fma(Linv[(size_t)d * NB + k], X[(size_t)k * ldx + n], a);
  } else {
    for (int k = d; k < NB; ++k) a = fma(Linv[(size_t)k * NB + d], X[(size_t)k * ldx + n], a);
  }
  out[(size_t)d * N + n] = a;
}

}  // namespace pmg

using namespace pmg;

extern "C" {

int pmg_tuning_linear(const float* basis, const double* W, int32_t L, int32_t NB, int32_t N, double* tuning64,
                      float* tuning32, void* stream) {
  PMG_REQUIRE(basis && W && L > 0 && NB > 0 && N > 0 && (tuning64 || tuning32), "pmg_tuning_linear: bad args");
  hipLaunchKernelGGL(k_tuning_linear, dim3((unsigned)((N + 255) / 256), (unsigned)L), dim3(256), 0,
                     as_stream(stream), basis, W, L, NB, N, tuning64, tuning32);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_gaussian(const float* y, const double* tuning64, const float* ma_neuron, int32_t ma_is_2d,
                          const uint8_t* ma_latent, double noise_std, double dt, int64_t T, int32_t L, int32_t N,
                          float* delta, double* rblk, double* ll64, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && y && tuning64 && delta && rblk, "pmg_emission_gaussian: bad args");
  PMG_REQUIRE(noise_std > 0.0, "pmg_emission_gaussian: noise_std must be > 0");
  const int Lp = (int)round_up(L, 32);
  const double c0 = -log(noise_std) - 0.5 * log(2.0 * M_PI);
  dim3 grid((unsigned)((T + 63) / 64), (unsigned)((L + 63) / 64));
  hipLaunchKernelGGL(k_emission_gaussian, grid, dim3(256), 0, as_stream(stream), y, ma_neuron, ma_is_2d, tuning64,
                     ma_latent, 1.0 / noise_std, c0, dt, nullptr, T, L, N, Lp, delta, rblk, ll64);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_gaussian_dt(const float* y, const double* tuning64, const float* ma_neuron, int32_t ma_is_2d,
                             const uint8_t* ma_latent, double noise_std, const double* dt_t, int64_t T, int32_t L,
                             int32_t N, float* delta, double* rblk, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && y && tuning64 && dt_t && delta && rblk,
              "pmg_emission_gaussian_dt: bad args");
  PMG_REQUIRE(noise_std > 0.0, "pmg_emission_gaussian_dt: noise_std must be > 0");
  const int Lp = (int)round_up(L, 32);
  const double c0 = -log(noise_std) - 0.5 * log(2.0 * M_PI);
  dim3 grid((unsigned)((T + 63) / 64), (unsigned)((L + 63) / 64));
  hipLaunchKernelGGL(k_emission_gaussian, grid, dim3(256), 0, as_stream(stream), y, ma_neuron, ma_is_2d, tuning64,
                     ma_latent, 1.0 / noise_std, c0, 1.0, dt_t, T, L, N, Lp, delta, rblk, nullptr);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

size_t pmg_gaussian_mstep_workspace_size(int32_t NB, int32_t N) {
  // [R | H] (NB x (N+NB)), Linv (NB x NB), Z = Linv R (NB x N)
  return ((size_t)NB * (size_t)(N + NB) + (size_t)NB * NB + (size_t)NB * N) * sizeof(double) + 256;
}

int pmg_gaussian_mstep(const float* basis, const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                       double noise_std, double prior_std, double* W, int32_t* status, void* workspace,
                       size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(basis && yw && tw && W && status && workspace && L > 0 && NB > 0 && N > 0,
              "pmg_gaussian_mstep: bad args");
  PMG_REQUIRE(noise_std > 0.0 && prior_std > 0.0, "pmg_gaussian_mstep: noise_std and prior_std must be > 0");
  const size_t lds = (size_t)NB * (NB + 1) / 2 * sizeof(double);
  PMG_REQUIRE(lds <= 160 * 1024, "pmg_gaussian_mstep: NB=%d too large (packed factor must fit 160 KiB LDS)", NB);
  PMG_REQUIRE(workspace_bytes >= pmg_gaussian_mstep_workspace_size(NB, N), "pmg_gaussian_mstep: workspace too small");
  hipStream_t st = as_stream(stream);
  double* ws = reinterpret_cast<double*>(workspace);
  hipLaunchKernelGGL(k_gauss_normal_eq, dim3((unsigned)((N + NB + 255) / 256), (unsigned)NB), dim3(256), 0, st,
                     basis, yw, tw, L, NB, N, 1.0 / (noise_std * noise_std), 1.0 / (prior_std * prior_std), ws);
  PMG_LAUNCH_CHECK();
  double* Linv = ws + (size_t)NB * (N + NB);
  double* Z = Linv + (size_t)NB * NB;
  const size_t lds_x = lds + (size_t)NB * NB * sizeof(double);
  const int x_in_lds = lds_x <= 160 * 1024 ? 1 : 0;
  const size_t lds_use = x_in_lds ? lds_x : lds;
  if (lds_use > 64 * 1024)
    PMG_HIP(hipFuncSetAttribute((const void*)k_gauss_chol_inv, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds_use));
  hipLaunchKernelGGL(k_gauss_chol_inv, dim3(1), dim3(256), lds_use, st, ws, NB, N, Linv, status, x_in_lds);
  PMG_LAUNCH_CHECK();
  const dim3 g((unsigned)((N + 255) / 256), (unsigned)NB);
  hipLaunchKernelGGL(k_gauss_tri_mm, g, dim3(256), 0, st, Linv, ws, (int64_t)(N + NB), NB, N, 0, Z);
  PMG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_gauss_tri_mm, g, dim3(256), 0, st, Linv, Z, (int64_t)N, NB, N, 1, W);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // extern "C"
