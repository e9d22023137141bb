// Small elementwise / per-row kernels of the EM hot path and the ABI plumbing.
//   spikes preparation  (y handling of decoder.py:30-71, fit_tuning_helper.py:28-42)
//   tuning softplus     (fit_tuning_helper.py:19-25)
//   emission row reference, log-likelihood materialisation, exp / log maps
#include <stdarg.h>

#include "pmg_common.h"

namespace pmg {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// One wave per time row: y*ma -> int8 operand, gammaln constant, f32 copy with a
// ones column, integrality / mask flags.  The workgroups are persistent over rows
// (grid-stride), and each first tabulates lgamma(k + 1) for k = 0..127 in LDS: spike
// counts are almost always small integers, and one f64 lgamma per (t, n) was ~0.7 ms of
// a C3 fit's setup (T N = 5.1e7 evaluations); a table lookup is exact (the same device
// lgamma values), any other value still takes lgamma.  With N % 4 == 0 a lane handles 4
// neurons per pass (16-byte loads of y and the mask, one 4-byte int8 store, one 16-byte
// yext store); the gammaln sum keeps the per-lane order of the scalar form (lane l adds
// neurons l, l + 64, ...), so gconst is identical in both forms.
constexpr int kLgfN = 128;

__device__ __forceinline__ void spike_elem(float v, float m, const double* lgf, double& g, int& bad) {
  if (!(m == 0.f || m == 1.f)) bad |= PMG_YFLAG_MASK;
  const bool small_int = v >= 0.f && v <= 127.f && v == rintf(v);
  if (!small_int) bad |= PMG_YFLAG_NONINT;
  if (m != 0.f) g += (double)m * (small_int ? lgf[(int)v] : lgamma((double)v + 1.0));
}

__device__ __forceinline__ int8_t spike_q(float v, float m) {
  return (int8_t)(int)fminf(fmaxf(v * m, -128.f), 127.f);
}

__global__ void __launch_bounds__(256) k_spikes_prepare(
    const float* __restrict__ y, int64_t T, int N, const float* __restrict__ ma, int ma_2d,
    int8_t* __restrict__ yq, int Kp, double* __restrict__ gconst, float* __restrict__ yext,
    int Np, int* __restrict__ flags, int64_t Tp) {
  __shared__ double lgf[kLgfN];
  if (threadIdx.x < kLgfN) lgf[threadIdx.x] = lgamma((double)threadIdx.x + 1.0);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 6);
  const bool vec = (N & 3) == 0;   // Kp, Np are multiples of 32 / 64
  int bad = 0;
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < Tp; t += stride) {
    if (t >= T) {  // zero padding rows of the int8 operand
      for (int n = lane; n < Kp; n += 64) yq[t * Kp + n] = 0;
      continue;
    }
    const float* yr = y + t * (int64_t)N;
    const float* mr = ma ? (ma_2d ? ma + t * (int64_t)N : ma) : nullptr;
    float* er = yext + t * (int64_t)Np;
    int8_t* qr = yq + t * (int64_t)Kp;
    double g = 0.0;
    if (vec) {
      // neurons 4i .. 4i+3 for i = lane, lane + 64, ...: int8 operand and yext copy
      const int n4 = N >> 2;
      for (int i = lane; i < (Kp >> 2); i += 64) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f), m = make_float4(1.f, 1.f, 1.f, 1.f);
        if (i < n4) {
          v = reinterpret_cast<const float4*>(yr)[i];
          if (mr) m = reinterpret_cast<const float4*>(mr)[i];
          *reinterpret_cast<float4*>(er + 4 * i) = v;
        } else {
          v = make_float4(0.f, 0.f, 0.f, 0.f);
          m = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        char4 q;
        q.x = spike_q(v.x, m.x); q.y = spike_q(v.y, m.y); q.z = spike_q(v.z, m.z); q.w = spike_q(v.w, m.w);
        *reinterpret_cast<char4*>(qr + 4 * i) = q;
      }
      // gammaln sum in the scalar order (the values are re-read from L1 / L2)
      for (int n = lane; n < N; n += 64) spike_elem(yr[n], mr ? mr[n] : 1.f, lgf, g, bad);
      for (int n = N + lane; n < Np; n += 64) er[n] = (n == N) ? 1.f : 0.f;
    } else {
      for (int n = lane; n < Kp; n += 64) {
        float v = 0.f, m = 1.f;
        if (n < N) {
          v = yr[n];
          if (mr) m = mr[n];
          spike_elem(v, m, lgf, g, bad);
        }
        qr[n] = (n < N) ? spike_q(v, m) : (int8_t)0;
      }
      for (int n = lane; n < Np; n += 64) er[n] = (n < N) ? yr[n] : (n == N ? 1.f : 0.f);
    }
    g = wave_sum_f64(g);
    if (lane == 0) gconst[t] = g;
  }
  unsigned long long anybad = __ballot(bad != 0);
  if (anybad) {
    int b = bad;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) b |= __shfl_xor(b, o, 64);
    if (lane == 0) atomicOr(flags, b);
  }
}

// tuning[l, n] = softplus(sum_k B[l, k] W[k, n]) (fit_tuning_helper.py:19-25) in f64.
// A 64-thread workgroup owns 64 neurons x kTunRows latent rows: each W element is loaded
// once per row tile (the per-row form re-read W's 323 KB 512 times at C3, 165 MB of L2
// traffic for 2 MB of output), the tile's basis rows sit in LDS.  Larger tiles leave too
// few waves to hide the f64 softplus latency (tools/tuning_bench.py).  Every
// output keeps the round-4 summation order (four interleaved partial sums over k % 4,
// combined (a0 + a1) + (a2 + a3), the tail into a0), so the tuning is bit-identical.
// blockIdx.z = restart r of a batched fit: W (R, NB, N) -> rows r L + l of the stacked
// (R L, N) tuning.
constexpr int kTunRows = 2;   // C3: 12.6 (one row per workgroup) -> 9.1 us; 4 rows 10.9, 8 rows 16.6 (fewer waves)
constexpr int kTunKC = 256;   // basis columns staged in LDS per pass (a multiple of 4)
__global__ void __launch_bounds__(64) k_tuning_softplus(const float* __restrict__ basis, const double* __restrict__ W,
                                                        int L, int NB, int N, double* __restrict__ t64,
                                                        float* __restrict__ t32) {
  __shared__ float sB[kTunRows * kTunKC];
  const int n = blockIdx.x * 64 + threadIdx.x;
  const bool live = n < N;
  const int l0 = blockIdx.y * kTunRows;
  const int64_t r = blockIdx.z;
  W += r * NB * (int64_t)N;
  const int nr = L - l0 < kTunRows ? L - l0 : kTunRows;
  const int NB4 = NB & ~3;
  double a[kTunRows][4];
#pragma unroll
  for (int rr = 0; rr < kTunRows; ++rr) a[rr][0] = a[rr][1] = a[rr][2] = a[rr][3] = 0.0;
  for (int kc = 0; kc < NB; kc += kTunKC) {
    const int kw = NB - kc < kTunKC ? NB - kc : kTunKC;
    __syncthreads();   // the previous pass's reads are done
    for (int i = threadIdx.x; i < kTunRows * kw; i += 64) {
      const int rr = i / kw, k = i - rr * kw;
      sB[rr * kTunKC + k] = rr < nr ? basis[(int64_t)(l0 + rr) * NB + kc + k] : 0.f;
    }
    __syncthreads();
    if (live) {
      const int k4 = (NB4 - kc) < kw ? (NB4 - kc) : kw;   // this pass's columns of the k % 4 sums
      int k = 0;
      for (; k + 4 <= k4; k += 4) {
        double w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = W[(int64_t)(kc + k + j) * N + n];
#pragma unroll
        for (int rr = 0; rr < kTunRows; ++rr)
#pragma unroll
          for (int j = 0; j < 4; ++j) a[rr][j] = fma((double)sB[rr * kTunKC + k + j], w[j], a[rr][j]);
      }
      for (k = k4 > 0 ? k4 : 0; k < kw; ++k) {   // the NB % 4 tail (last pass only)
        const double w = W[(int64_t)(kc + k) * N + n];
#pragma unroll
        for (int rr = 0; rr < kTunRows; ++rr) a[rr][0] = fma((double)sB[rr * kTunKC + k], w, a[rr][0]);
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int rr = 0; rr < kTunRows; ++rr) {
    if (rr >= nr) break;
    const int64_t row = r * L + l0 + rr;
    const double f = softplus_d((a[rr][0] + a[rr][1]) + (a[rr][2] + a[rr][3]));
    if (t64) t64[row * N + n] = f;
    if (t32) t32[row * N + n] = (float)f;
  }
}

// Row references: per (t, group) the max over the group's nb = nblk / R blocks (R groups
// = batched restarts' stacked latents; R = 1: the whole row) -> m (T, R), and
// phi[t, b] = s (rblk[t, b] - m).  A (t, group) row occupies NBP = pow2 >= nb lanes, so a
// wave handles 64 / NBP rows with coalesced loads / stores and a segmented shuffle max
// (one thread per row, as before, read 16 strided f64 per thread: ~21 us at C3).
template <int NBP>
__global__ void __launch_bounds__(256) k_rowref(const double* __restrict__ rblk, int64_t T, int nblk, int R,
                                                double s, float* __restrict__ phi, double* __restrict__ m) {
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * (64 / NBP) + lane / NBP;
  const int b = lane % NBP;
  const int nb = nblk / R;
  const bool live = row < T * R && b < nb;
  // R == 1 (one model): no 64-bit division by R (a ~150-instruction sequence per lane)
  const int64_t t = !live ? 0 : R == 1 ? row : row / R;
  const int g = live && R != 1 ? (int)(row - t * R) : 0;
  const int64_t o = t * nblk + (int64_t)g * nb + b;
  const double v = live ? rblk[o] : -INFINITY;
  double mx = v;
#pragma unroll
  for (int d = 1; d < NBP; d <<= 1) mx = fmax(mx, __shfl_xor(mx, d, 64));
  if (mx == -INFINITY) mx = 0.0;  // cannot happen for L >= 1 (masked latents are -1e20)
  if (live) {
    phi[o] = (float)(s * (v - mx));
    if (b == 0) m[row] = mx;
  }
}

// rows of more than 64 blocks (L > 2048, the dense scans): one wave per (t, group) row,
// KB blocks per lane (lane, lane + 64, ...)
template <int KB>
__global__ void __launch_bounds__(256) k_rowref_wide(const double* __restrict__ rblk, int64_t T, int nblk, int R,
                                                     double s, float* __restrict__ phi, double* __restrict__ m) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int nb = nblk / R;
  const bool rlive = row < T * R;
  const int64_t t = !rlive ? 0 : R == 1 ? row : row / R;
  const int g = rlive && R != 1 ? (int)(row - t * R) : 0;
  const int64_t o0 = t * nblk + (int64_t)g * nb;
  double v[KB], mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const int b = lane + 64 * k;
    v[k] = rlive && b < nb ? rblk[o0 + b] : -INFINITY;
    mx = fmax(mx, v[k]);
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) mx = fmax(mx, __shfl_xor(mx, d, 64));
  if (mx == -INFINITY) mx = 0.0;
  if (rlive) {
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int b = lane + 64 * k;
      if (b < nb) phi[o0 + b] = (float)(s * (v[k] - mx));
    }
    if (lane == 0) m[row] = mx;
  }
}

static void launch_rowref(const double* rblk, int64_t T, int nblk, int R, double s, float* phi, double* m,
                          hipStream_t st) {
  const int nb = nblk / R;
  const int64_t rows = T * R;
#define PMG_RR(NBP)                                                                                  \
  if (nb <= NBP) {                                                                                   \
    const int64_t waves = (rows + (64 / NBP) - 1) / (64 / NBP);                                      \
    hipLaunchKernelGGL(k_rowref<NBP>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, rblk, T, nblk, R, s, \
                       phi, m);                                                                      \
    return;                                                                                          \
  }
  PMG_RR(1) PMG_RR(2) PMG_RR(4) PMG_RR(8) PMG_RR(16) PMG_RR(32) PMG_RR(64)
#undef PMG_RR
  hipLaunchKernelGGL(k_rowref_wide<2>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, rblk, T, nblk, R, s, phi, m);
}

__global__ void k_loglik(const float* __restrict__ delta, const double* __restrict__ rblk,
                         int64_t T, int L, int nblk, float* __restrict__ ll) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T * (int64_t)L) return;
  const int64_t t = i / L;
  const int l = (int)(i - t * L);
  ll[i] = (float)((double)delta[i] + rblk[t * nblk + (l >> 5)]);
}

__global__ void k_exp(const float* __restrict__ x, int64_t n, float* __restrict__ y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) y[i] = expf(x[i]);
}
__global__ void k_log(const float* __restrict__ x, int64_t n, float* __restrict__ y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) y[i] = logf(x[i]);
}

// The arrays a fit / decode returns from the posterior (T, 2, L) (core.py:696-712,
// decoder.py:300-315), in one pass over it: its log (logf, as k_log), the latent marginal
// plm (T, L) = g[t,0,l] + g[t,1,l] and the dynamics marginal pdm (T, 2) = sum_l g[t,d,l]
// (f64 sums rounded once).  One workgroup per row t (grid-stride); any output may be null.
__global__ void __launch_bounds__(256) k_posterior_outputs(const float* __restrict__ g, int64_t T, int L,
                                                           float* __restrict__ lg, float* __restrict__ plm,
                                                           float* __restrict__ pdm) {
  __shared__ double red[2][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
    const float* r = g + t * 2 * L;
    double s0 = 0.0, s1 = 0.0;
    for (int l = threadIdx.x; l < L; l += 256) {
      const float a = r[l], b = r[L + l];
      s0 += a;
      s1 += b;
      if (plm) plm[t * L + l] = a + b;
      if (lg) {
        lg[t * 2 * L + l] = logf(a);
        lg[t * 2 * L + L + l] = logf(b);
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
    }
    if (lane == 0) {
      red[0][wv] = s0;
      red[1][wv] = s1;
    }
    __syncthreads();
    if (pdm && threadIdx.x < 2)
      pdm[t * 2 + threadIdx.x] = (float)(red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] +
                                         red[threadIdx.x][3]);
    __syncthreads();
  }
}

// out[t, n] = y[(t - shift[n]) mod T, n]: np.roll of every neuron's column by its own
// shift (circular_shuffle_data, test.py:20-23).  A block walks rows t; its threads own
// neuron columns, so each thread's shift is read once and every row write is coalesced.
__global__ void __launch_bounds__(256) k_roll_columns(const float* __restrict__ y, int64_t T, int N,
                                                      const int64_t* __restrict__ shift,
                                                      float* __restrict__ out) {
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    int64_t s = shift[n] % T;
    if (s < 0) s += T;
    for (int64_t t = blockIdx.x; t < T; t += gridDim.x) {
      int64_t src = t - s;
      src += (src < 0) ? T : 0;
      out[t * N + n] = y[src * N + n];
    }
  }
}

}  // namespace pmg

using namespace pmg;

extern "C" {

int pmg_abi_version(void) { return PMG_ABI_VERSION; }
const char* pmg_last_error(void) { return g_err; }

int pmg_spikes_prepare(const float* y, int64_t T, int32_t N, const float* ma_neuron,
                       int32_t ma_is_2d, int8_t* yq_out, int32_t Kp, double* gconst_out,
                       float* yext_out, int32_t Np, int32_t* flags_out, void* stream) {
  PMG_REQUIRE(T > 0 && N > 0, "pmg_spikes_prepare: T=%lld N=%d", (long long)T, N);
  PMG_REQUIRE(Kp >= N && Kp % 32 == 0, "pmg_spikes_prepare: Kp=%d must be >= N and a multiple of 32", Kp);
  PMG_REQUIRE(Np >= N + 1 && Np % 64 == 0, "pmg_spikes_prepare: Np=%d must be >= N+1 and a multiple of 64", Np);
  PMG_REQUIRE(y && yq_out && gconst_out && yext_out && flags_out, "pmg_spikes_prepare: null pointer");
  hipStream_t st = as_stream(stream);
  PMG_HIP(hipMemsetAsync(flags_out, 0, sizeof(int32_t), st));
  const int64_t Tp = round_up(T, 64);
  const int waves = 4;
  int64_t blocks = (Tp + waves - 1) / waves;
  if (blocks > 2048) blocks = 2048;   // persistent over rows: the lgamma table once per workgroup
  dim3 grid((unsigned)blocks);
  hipLaunchKernelGGL(k_spikes_prepare, grid, dim3(64 * waves), 0, st, y, T, N, ma_neuron,
                     ma_is_2d, yq_out, Kp, gconst_out, yext_out, Np, flags_out, Tp);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_tuning_softplus(const float* basis, const double* W, int32_t L, int32_t NB, int32_t N,
                        double* tuning64, float* tuning32, void* stream) {
  return pmg_tuning_softplus_batched(basis, W, L, NB, N, 1, tuning64, tuning32, stream);
}

int pmg_tuning_softplus_batched(const float* basis, const double* W, int32_t L, int32_t NB, int32_t N, int32_t R,
                                double* tuning64, float* tuning32, void* stream) {
  PMG_REQUIRE(L > 0 && NB > 0 && N > 0 && R > 0 && R <= 65535 && basis && W, "pmg_tuning_softplus: bad args");
  dim3 grid((N + 63) / 64, (L + kTunRows - 1) / kTunRows, R);
  hipLaunchKernelGGL(k_tuning_softplus, grid, dim3(64), 0, as_stream(stream), basis, W, L, NB,
                     N, tuning64, tuning32);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_rowref(const double* rblk, int64_t T, int32_t nblk, double likelihood_scale,
                        float* phi, double* m, void* stream) {
  PMG_REQUIRE(T > 0 && nblk > 0 && rblk && phi && m, "pmg_emission_rowref: bad args");
  PMG_REQUIRE(nblk <= 128, "pmg_emission_rowref: nblk=%d > 128 (L > 4096)", nblk);
  launch_rowref(rblk, T, nblk, 1, likelihood_scale, phi, m, as_stream(stream));
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_rowref_batched(const double* rblk, int64_t T, int32_t nblk, int32_t R, double likelihood_scale,
                                float* phi, double* m, void* stream) {
  PMG_REQUIRE(T > 0 && nblk > 0 && R > 0 && nblk % R == 0 && rblk && phi && m,
              "pmg_emission_rowref_batched: bad args (nblk=%d, R=%d)", nblk, R);
  PMG_REQUIRE(nblk / R <= 128, "pmg_emission_rowref_batched: %d blocks per restart > 128", nblk / R);
  launch_rowref(rblk, T, nblk, R, likelihood_scale, phi, m, as_stream(stream));
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_loglik_materialize(const float* delta, const double* rblk, int64_t T, int32_t L,
                           float* ll, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && delta && rblk && ll, "pmg_loglik_materialize: bad args");
  const int64_t n = T * (int64_t)L;
  const int nblk = (int)(round_up(L, 32) / 32);
  hipLaunchKernelGGL(k_loglik, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), delta, rblk, T, L, nblk, ll);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_exp(const float* logp, int64_t n, float* p, void* stream) {
  PMG_REQUIRE(n >= 0, "pmg_exp: bad args");
  if (n == 0) return PMG_OK;
  PMG_REQUIRE(logp && p, "pmg_exp: null pointer");
  unsigned blocks = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  hipLaunchKernelGGL(k_exp, dim3(blocks), dim3(256), 0, as_stream(stream), logp, n, p);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_roll_columns(const float* y, int64_t T, int32_t N, const int64_t* shift, float* out, void* stream) {
  PMG_REQUIRE(T > 0 && N > 0 && y && shift && out && y != out, "pmg_roll_columns: bad args");
  const unsigned threads = (unsigned)(N >= 256 ? 256 : round_up(N, 64));
  const unsigned blocks = (unsigned)(T < 8192 ? T : 8192);
  hipLaunchKernelGGL(k_roll_columns, dim3(blocks), dim3(threads), 0, as_stream(stream), y, T, N, shift, out);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_log(const float* x, int64_t n, float* out, void* stream) {
  PMG_REQUIRE(n >= 0, "pmg_log: bad args");
  if (n == 0) return PMG_OK;
  PMG_REQUIRE(x && out, "pmg_log: null pointer");
  unsigned blocks = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  hipLaunchKernelGGL(k_log, dim3(blocks), dim3(256), 0, as_stream(stream), x, n, out);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_posterior_outputs(const float* gamma, int64_t T, int32_t L, float* log_out, float* plm, float* pdm,
                          void* stream) {
  PMG_REQUIRE(T >= 0 && L > 0 && (T == 0 || gamma), "pmg_posterior_outputs: bad args (T=%lld, L=%d)", (long long)T, L);
  if (T == 0 || (!log_out && !plm && !pdm)) return PMG_OK;
  const unsigned blocks = (unsigned)(T < 4096 ? T : 4096);
  hipLaunchKernelGGL(k_posterior_outputs, dim3(blocks), dim3(256), 0, as_stream(stream), gamma, T, L, log_out,
                     plm, pdm);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // extern "C"
