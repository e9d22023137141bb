// Poisson emission log-likelihood on gfx950.
//
// Replaces decoder.get_loglikelihood_ma_poisson (decoder.py:30-48) vmapped over
// time by get_loglikelihood_ma_all (decoder.py:60-71):
//     ll[t,l] = sum_n m[t,n] (xlogy(y[t,n], lam[l,n]) - lam[l,n] - gammaln(y[t,n]+1))
//     lam = tuning*dt + 1e-20,   ll[:, ma_latent == 0] = -1e20
// i.e. a dense (T x N).(N x L) contraction  Y.log(lam)^T  plus a per-latent and a
// per-time constant.
//
// Precision: the posterior depends on differences ll[t,l]-ll[t,l'] of sums of ~N
// terms of size O(1-10); fp32 accumulation would cost ~1e-5 absolute.  The fast
// path is therefore EXACT integer arithmetic: y (0..127) as int8 and log(lam) as a
// 2^-24 fixed-point number split into 4 balanced base-256 int8 digits; the digit
// GEMMs run on v_mfma_i32_32x32x32_i8 with exact int32 accumulation and are
// recombined in int64 (quantisation error <= 2^-25 per log(lam)).  Anything the
// integer path cannot represent (non-integer / >127 counts, weighted or 2-D masks)
// goes through the f64 kernel at the bottom.
//
// Output format (both paths): delta[t,l] = f32(ll[t,l] - r[t,b]) with
// r[t,b] = max over the 32-latent block b (f64), so an fp32 consumer recovers
// exp(s*(ll - max_l ll)) = exp(s*delta + phi) with 1-ulp accuracy near the max.
#include "pmg_common.h"

namespace pmg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr double kQScale = 16777216.0;  // 2^24
constexpr double kQInv = 1.0 / 16777216.0;

// One wave per latent row: log(lam) -> 4 int8 digits, lamsum = sum_n m_n lam.
__global__ void __launch_bounds__(256) k_rates_prepare(
    const double* __restrict__ tuning, int L, int N, const float* __restrict__ ma, double dt,
    int Lp, int Kp, int8_t* __restrict__ qd, double* __restrict__ lamsum, int* __restrict__ bad) {
  const int lane = threadIdx.x & 63;
  const int l = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (l >= Lp) return;
  const size_t plane = (size_t)Lp * Kp;
  double ls = 0.0;
  int flag = 0;
  for (int n = lane; n < Kp; n += 64) {
    int8_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
    if (l < L && n < N) {
      const double lam = tuning[(size_t)l * N + n] * dt + 1e-20;
      const double lg = log(lam);
      if (!(fabs(lg) < 60.0)) flag = 1;
      long long q = llrint(lg * kQScale);
      long long r0 = ((q + 128) & 255) - 128;
      q = (q - r0) >> 8;
      long long r1 = ((q + 128) & 255) - 128;
      q = (q - r1) >> 8;
      long long r2 = ((q + 128) & 255) - 128;
      q = (q - r2) >> 8;
      d0 = (int8_t)r0;
      d1 = (int8_t)r1;
      d2 = (int8_t)r2;
      d3 = (int8_t)q;  // |q| <= 64 for |lg| < 60
      const float m = ma ? ma[n] : 1.f;
      ls += (double)m * lam;
    }
    const size_t o = (size_t)l * Kp + n;
    qd[o] = d0;
    qd[plane + o] = d1;
    qd[2 * plane + o] = d2;
    qd[3 * plane + o] = d3;
  }
  ls = wave_sum_f64(ls);
  if (lane == 0) lamsum[l] = ls;
  if (__ballot(flag)) {
    if (lane == 0) atomicOr(bad, 1);
  }
}

// Wave tile: 32 latents (MFMA rows, A = digits of log lam) x 64 time bins
// (2 x 32 MFMA columns, B = y^T) x 4 digits: 8 v16i accumulators.
// A fragment: lane (r = lane&31, h = lane>>5) holds A[row r][k0+16h .. +15];
// B fragment: lane holds B[k0+16h .. +15][col r].  The same (h, element) -> k
// assignment on both operands makes the K pairing consistent.
// C/D: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*h  (cdna_hip_programming §3).
__global__ void __launch_bounds__(256) k_emission_i8(
    const int8_t* __restrict__ yq, const int8_t* __restrict__ qd,
    const double* __restrict__ lamsum, const double* __restrict__ gconst,
    const uint8_t* __restrict__ ma_latent, int64_t T, int L, int Lp, int Kp, int nLB,
    int64_t nTB, float* __restrict__ delta, double* __restrict__ rblk) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (w >= (int64_t)nLB * nTB) return;
  const int lb = (int)(w % nLB);
  const int64_t tb = w / nLB;
  const int r = lane & 31, h = lane >> 5;
  const size_t plane = (size_t)Lp * Kp;

  const int8_t* a_ptr = qd + (size_t)(lb * 32 + r) * Kp + 16 * h;
  const int8_t* b_ptr0 = yq + (size_t)(tb * 64 + r) * Kp + 16 * h;
  const int8_t* b_ptr1 = b_ptr0 + (size_t)32 * Kp;

  v16i acc[4][2];
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    acc[d][0] = (v16i){0};
    acc[d][1] = (v16i){0};
  }
  for (int k0 = 0; k0 < Kp; k0 += 32) {
    const v4i b0 = *reinterpret_cast<const v4i*>(b_ptr0 + k0);
    const v4i b1 = *reinterpret_cast<const v4i*>(b_ptr1 + k0);
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const v4i a = *reinterpret_cast<const v4i*>(a_ptr + d * plane + k0);
      acc[d][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0, acc[d][0], 0, 0, 0);
      acc[d][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1, acc[d][1], 0, 0, 0);
    }
  }

  const int nblk = Lp >> 5;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int64_t t = tb * 64 + s * 32 + r;
    const bool tvalid = t < T;
    const double gc = tvalid ? gconst[t] : 0.0;
    double ll[16];
    double mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int l = lb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      long long q = (long long)acc[0][s][i] + ((long long)acc[1][s][i] << 8) +
                    ((long long)acc[2][s][i] << 16) + ((long long)acc[3][s][i] << 24);
      double v = (double)q * kQInv - lamsum[l] - gc;
      if (l < L) {
        if (ma_latent && ma_latent[l] == 0) v = -1e20;
        mx = fmax(mx, v);
      } else {
        v = -INFINITY;
      }
      ll[i] = v;
    }
    mx = fmax(mx, __shfl_xor(mx, 32, 64));
    if (tvalid) {
      if (h == 0) rblk[t * nblk + lb] = mx;
      float* drow = delta + t * (int64_t)L;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int l = lb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (l < L) drow[l] = (float)(ll[i] - mx);
      }
    }
  }
}

// Generic f64 emission: any y, weighted and/or 2-D neuron masks.
// Block: 256 threads = tile of 16 time bins x 64 latents; thread (ty, tx) owns
// latent l0+tx and time bins t0+4ty .. +3.
__global__ void __launch_bounds__(256) k_emission_f64(
    const float* __restrict__ y, const float* __restrict__ ma, int ma_2d,
    const double* __restrict__ tuning, double dt, const double* __restrict__ gconst,
    const uint8_t* __restrict__ ma_latent, int64_t T, int L, int N, int Lp,
    float* __restrict__ delta, double* __restrict__ rblk) {
  __shared__ double sYM[16][33];
  __shared__ double sM[16][33];
  __shared__ double sLG[32][65];
  __shared__ double sLA[32][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * 16;
  const int l0 = blockIdx.y * 64;
  double a1[4] = {0, 0, 0, 0}, a2[4] = {0, 0, 0, 0};
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
      sYM[tt][nn] = yv * mv;
      sM[tt][nn] = mv;
    }
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int nn = e / 64, ll = e % 64;
      const int n = n0 + nn, l = l0 + ll;
      double lam = 0.0, lg = 0.0;
      if (n < N && l < L) {
        lam = tuning[(size_t)l * N + n] * dt + 1e-20;
        lg = log(lam);
      }
      sLG[nn][ll] = lg;
      sLA[nn][ll] = lam;
    }
    __syncthreads();
#pragma unroll 4
    for (int nn = 0; nn < 32; ++nn) {
      const double lg = sLG[nn][tx], la = sLA[nn][tx];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a1[j] = fma(sYM[ty * 4 + j][nn], lg, a1[j]);
        a2[j] = fma(sM[ty * 4 + j][nn], la, a2[j]);
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
      v = a1[j] - a2[j] - gconst[t];
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

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_emission_workspace_size(int64_t T, int32_t L, int32_t N) {
  (void)T;
  const int64_t Lp = round_up(L, 32), Kp = round_up(N, 32);
  Carver c(nullptr);
  c.take<int8_t>(4 * Lp * Kp);
  c.take<double>(Lp);
  c.take<int>(4);
  return c.off + 256;
}

int pmg_emission_poisson(const int8_t* yq, const double* gconst, const double* tuning64,
                         const float* ma_neuron_1d, const uint8_t* ma_latent, double dt,
                         int64_t T, int32_t L, int32_t N, int32_t Kp, float* delta,
                         double* rblk, void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0, "pmg_emission_poisson: bad shape");
  PMG_REQUIRE(Kp == round_up(N, 32), "pmg_emission_poisson: Kp must be roundup(N,32)");
  PMG_REQUIRE(yq && gconst && tuning64 && delta && rblk && workspace, "pmg_emission_poisson: null");
  PMG_REQUIRE(workspace_bytes >= pmg_emission_workspace_size(T, L, N),
              "pmg_emission_poisson: workspace too small");
  hipStream_t st = as_stream(stream);
  const int Lp = (int)round_up(L, 32);
  Carver c(workspace);
  int8_t* qd = c.take<int8_t>(4 * (size_t)Lp * Kp);
  double* lamsum = c.take<double>(Lp);
  int* bad = c.take<int>(4);
  PMG_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_rates_prepare, dim3((Lp + 3) / 4), dim3(256), 0, st, tuning64, L, N,
                     ma_neuron_1d, dt, Lp, Kp, qd, lamsum, bad);
  PMG_LAUNCH_CHECK();
  const int nLB = Lp / 32;
  const int64_t nTB = (T + 63) / 64;
  const int64_t waves = nLB * nTB;
  hipLaunchKernelGGL(k_emission_i8, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, yq,
                     qd, lamsum, gconst, ma_latent, T, L, Lp, Kp, nLB, nTB, delta, rblk);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_poisson_f64(const float* y, const double* gconst, const double* tuning64,
                             const float* ma_neuron, int32_t ma_is_2d, const uint8_t* ma_latent,
                             double dt, int64_t T, int32_t L, int32_t N, float* delta,
                             double* rblk, void* workspace, size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && y && gconst && tuning64 && delta && rblk,
              "pmg_emission_poisson_f64: bad args");
  const int Lp = (int)round_up(L, 32);
  dim3 grid((unsigned)((T + 15) / 16), (unsigned)((L + 63) / 64));
  hipLaunchKernelGGL(k_emission_f64, grid, dim3(256), 0, as_stream(stream), y, ma_neuron,
                     ma_is_2d, tuning64, dt, gconst, ma_latent, T, L, N, Lp, delta, rblk);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // extern "C"
