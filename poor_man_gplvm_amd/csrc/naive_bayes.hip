// Naive-Bayes decoding (no temporal prior): decoder.get_naive_bayes_ma_chunk
// (decoder.py:106-149) -> get_naive_bayes_ma (:88-102) -> the per-time-dt emission
// get_loglikelihood_ma_all_changing_dt (:73-85), then a logsumexp normalisation per
// time bin.  A constant dt goes through the exact int8 emission (emission.hip);
// this file holds the per-time-dt emission and the row normalisation.
#include <math.h>

#include "pmg_common.h"

namespace pmg {

// ll[t,l] = sum_n m[t,n] (xlogy(y, lam) - lam) - gconst[t],  lam = tuning[l,n] dt[t] + 1e-20
// (log lam depends on t: one log per (t, l, n), as in the reference).  Output split as the
// other emissions: delta = ll - r[t, l/32] (f32), rblk = 32-latent block max (f64).
// Block: 256 threads = 16 time bins x 64 latents; thread (ty, tx) owns latent l0+tx and
// time bins t0+4ty .. +3.
__global__ void __launch_bounds__(256) k_emission_dt(
    const float* __restrict__ y, const float* __restrict__ ma, int ma_2d,
    const double* __restrict__ tuning, const double* __restrict__ dt, const double* __restrict__ gconst,
    const uint8_t* __restrict__ ma_latent, int64_t T, int L, int N, int Lp,
    float* __restrict__ delta, double* __restrict__ rblk) {
  __shared__ double sY[16][33];
  __shared__ double sM[16][33];
  __shared__ double sTu[32][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * 16;
  const int l0 = blockIdx.y * 64;
  double dts[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t t = t0 + ty * 4 + j;
    dts[j] = t < T ? dt[t] : 1.0;
  }
  double a[4] = {0, 0, 0, 0};
  for (int n0 = 0; n0 < N; n0 += 32) {
    for (int e = threadIdx.x; e < 16 * 32; e += 256) {
      const int tt = e / 32, nn = e % 32;
      const int64_t t = t0 + tt;
      const int n = n0 + nn;
      double yv = 0.0, mv = 0.0;
      if (t < T && n < N) {
        yv = y[t * N + n];
        mv = ma ? (ma_2d ? ma[t * N + n] : ma[n]) : 1.0;
      }
      sY[tt][nn] = yv;
      sM[tt][nn] = mv;
    }
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int nn = e / 64, ll = e % 64;
      const int n = n0 + nn, l = l0 + ll;
      sTu[nn][ll] = (n < N && l < L) ? tuning[(size_t)l * N + n] : 0.0;
    }
    __syncthreads();
    for (int nn = 0; nn < 32 && n0 + nn < N; ++nn) {
      const double tu = sTu[nn][tx];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double lam = tu * dts[j] + 1e-20;
        const double yv = sY[ty * 4 + j][nn];
        const double xl = yv == 0.0 ? 0.0 : yv * log(lam);   // jax xlogy
        a[j] = fma(sM[ty * 4 + j][nn], xl - lam, a[j]);
      }
    }
    __syncthreads();
  }
  const int l = l0 + tx;
  const int nblk = Lp >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t t = t0 + ty * 4 + j;
    double v = -INFINITY;
    if (l < L && t < T) {
      v = a[j] - gconst[t];
      if (ma_latent && ma_latent[l] == 0) v = -1e20;
    }
    double mx = v;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if (t < T) {
      if ((tx & 31) == 0 && l < Lp) rblk[t * nblk + (l >> 5)] = mx;
      if (l < L) delta[t * (int64_t)L + l] = (float)(v - mx);
    }
  }
}

// one wave per time bin: lse_t = logsumexp_l ll[t,l] (f64), log_post = ll - lse (f32)
__global__ void __launch_bounds__(256) k_nb_normalize(const float* __restrict__ delta,
                                                      const double* __restrict__ rblk, int64_t T, int L,
                                                      int nblk, float* __restrict__ log_post,
                                                      double* __restrict__ log_marg) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const double* rb = rblk + t * nblk;
  double m = -INFINITY;
  for (int b = lane; b < nblk; b += 64) m = fmax(m, rb[b]);
  for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  const float* dr = delta + t * (int64_t)L;
  double s = 0.0;
  for (int l = lane; l < L; l += 64) s += exp((double)dr[l] + rb[l >> 5] - m);
  s = wave_sum_f64(s);
  const double lse = m + log(s);
  float* out = log_post + t * (int64_t)L;
  for (int l = lane; l < L; l += 64) out[l] = (float)((double)dr[l] + rb[l >> 5] - lse);
  if (lane == 0) log_marg[t] = lse;
}

}  // namespace pmg

using namespace pmg;

extern "C" {

int pmg_emission_poisson_dt(const float* y, const double* gconst, const double* tuning64,
                            const float* ma_neuron, int32_t ma_is_2d, const uint8_t* ma_latent,
                            const double* dt_t, int64_t T, int32_t L, int32_t N, float* delta,
                            double* rblk, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && y && gconst && tuning64 && dt_t && delta && rblk,
              "pmg_emission_poisson_dt: bad args");
  const int Lp = (int)round_up(L, 32);
  dim3 grid((unsigned)((T + 15) / 16), (unsigned)((L + 63) / 64));
  hipLaunchKernelGGL(k_emission_dt, grid, dim3(256), 0, as_stream(stream), y, ma_neuron, ma_is_2d,
                     tuning64, dt_t, gconst, ma_latent, T, L, N, Lp, delta, rblk);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_naive_bayes_normalize(const float* delta, const double* rblk, int64_t T, int32_t L,
                              float* log_post, double* log_marginal_l, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && delta && rblk && log_post && log_marginal_l,
              "pmg_naive_bayes_normalize: bad args");
  const int nblk = (int)(round_up(L, 32) / 32);
  hipLaunchKernelGGL(k_nb_normalize, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, as_stream(stream), delta,
                     rblk, T, L, nblk, log_post, log_marginal_l);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // extern "C"
