// Time contractions C[m,n] = sum_t A[t,m] * B[t+shift,n] on gfx950 fp32 MFMA.
//
//   * sufficient statistics, fit_tuning_helper.get_statistics (fit_tuning_helper.py:28-42):
//       y_w = P^T y (L,N), t_w = sum_t P (L)     A = P (T,L), B = [y | 1] (T,Np)
//   * pairwise joint for decode_latent (decoder.py:215-221 accumulated over the scan):
//       S = sum_{t<T-1} alpha_t (x) rho_{t+1}   A = alpha (T,2L), B = rho (T,2L), shift 1
//
// Both operands are time-major, which is exactly the per-lane layout of
// v_mfma_f32_32x32x2f32: lane (r = lane&31, h = lane>>5) supplies A[row r][k = h] and
// B[k = h][col r], i.e. 32 consecutive floats of one time row per half-wave --
// coalesced 128-B loads straight from HBM, no LDS transpose.
// Products are exact fp32 (the instruction is an fma chain); each wave flushes its
// fp32 accumulators into f64 registers every 128 time steps and writes one f64
// partial per K-slice; slices are summed in f64 in a fixed order.
#include "pmg_common.h"

namespace pmg {

typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kFlush = 128;  // time steps per fp32 accumulation segment

// wave tile 64 (m) x 64 (n); grid of waves (mt, nt, ks)
__global__ void __launch_bounds__(256) k_atb(const float* __restrict__ A, int64_t lda, int Mdim,
                                             const float* __restrict__ B, int64_t ldb, int Ndim,
                                             int shift, int64_t K, int64_t KT, int nMT, int nNT,
                                             int nKS, int Mp, int Npd, double* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (w >= (int64_t)nMT * nNT * nKS) return;
  const int mt = (int)(w % nMT);
  const int nt = (int)((w / nMT) % nNT);
  const int ks = (int)(w / ((int64_t)nMT * nNT));
  const int r = lane & 31, h = lane >> 5;
  const int m0 = mt * 64 + r, m1 = m0 + 32;
  const int n0 = nt * 64 + r, n1 = n0 + 32;
  const bool vm0 = m0 < Mdim, vm1 = m1 < Mdim, vn0 = n0 < Ndim, vn1 = n1 < Ndim;
  const int64_t kb = (int64_t)ks * KT;
  const int64_t ke = kb + KT < K ? kb + KT : K;

  double acc64[4][16];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc64[q][i] = 0.0;

  for (int64_t s0 = kb; s0 < ke; s0 += kFlush) {
    const int64_t s1 = s0 + kFlush < ke ? s0 + kFlush : ke;
    v16f c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0};
#pragma unroll 4
    for (int64_t t = s0; t < s1; t += 2) {
      const int64_t tt = t + h;
      const bool vt = tt < s1;
      const float* ar = A + tt * lda;
      const float* br = B + (tt + shift) * ldb;
      const float a0 = (vt && vm0) ? ar[m0] : 0.f;
      const float a1 = (vt && vm1) ? ar[m1] : 0.f;
      const float b0 = (vt && vn0) ? br[n0] : 0.f;
      const float b1 = (vt && vn1) ? br[n1] : 0.f;
      c00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, c00, 0, 0, 0);
      c01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, c01, 0, 0, 0);
      c10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, c10, 0, 0, 0);
      c11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, c11, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc64[0][i] += (double)c00[i];
      acc64[1][i] += (double)c01[i];
      acc64[2][i] += (double)c10[i];
      acc64[3][i] += (double)c11[i];
    }
  }
  // C/D layout: col = lane&31, row = (i&3) + 8*(i>>2) + 4*h
  double* pp = part + (size_t)ks * Mp * Npd;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int mi = q >> 1, ni = q & 1;
    const int col = nt * 64 + ni * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = mt * 64 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      pp[(size_t)row * Npd + col] = acc64[q][i];
    }
  }
}

__global__ void k_atb_reduce(const double* __restrict__ part, int nKS, int Mp, int Npd, int Mdim,
                             int Nout, int ld_out, double* __restrict__ out, int tcol,
                             double* __restrict__ tout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)Mdim * Npd;
  if (i >= total) return;
  const int m = (int)(i / Npd), n = (int)(i % Npd);
  const bool to_out = n < Nout, to_t = (tout != nullptr) && n == tcol;
  if (!to_out && !to_t) return;
  double s = 0.0;
  for (int k = 0; k < nKS; ++k) s += part[((size_t)k * Mp + m) * Npd + n];
  if (to_out) out[(size_t)m * ld_out + n] = s;
  if (to_t) tout[m] = s;
}

static int atb_geometry(int64_t K, int Mdim, int Ndim, int& nMT, int& nNT, int& nKS, int64_t& KT,
                        int& Mp, int& Npd) {
  nMT = (Mdim + 63) / 64;
  nNT = (Ndim + 63) / 64;
  Mp = nMT * 64;
  Npd = nNT * 64;
  // enough waves to fill the chip (~8 per CU), K-slices of whole flush segments
  const int64_t tiles = (int64_t)nMT * nNT;
  int64_t want = (2048 + tiles - 1) / tiles;
  if (want < 1) want = 1;
  KT = (K + want - 1) / want;
  KT = round_up(KT < kFlush ? kFlush : KT, kFlush);
  nKS = (int)((K + KT - 1) / KT);
  if (nKS < 1) nKS = 1;
  return 0;
}

static size_t atb_ws(int64_t K, int Mdim, int Ndim) {
  int nMT, nNT, nKS, Mp, Npd;
  int64_t KT;
  atb_geometry(K, Mdim, Ndim, nMT, nNT, nKS, KT, Mp, Npd);
  return (size_t)nKS * Mp * Npd * sizeof(double) + 256;
}

static int atb_run(const float* A, int64_t lda, int Mdim, const float* B, int64_t ldb, int Ndim,
                   int shift, int64_t K, double* out, int Nout, int ld_out, int tcol, double* tout,
                   void* ws, hipStream_t st) {
  int nMT, nNT, nKS, Mp, Npd;
  int64_t KT;
  atb_geometry(K, Mdim, Ndim, nMT, nNT, nKS, KT, Mp, Npd);
  double* part = reinterpret_cast<double*>(ws);
  const int64_t waves = (int64_t)nMT * nNT * nKS;
  hipLaunchKernelGGL(k_atb, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, A, lda, Mdim, B,
                     ldb, Ndim, shift, K, KT, nMT, nNT, nKS, Mp, Npd, part);
  PMG_LAUNCH_CHECK();
  const int64_t total = (int64_t)Mdim * Npd;
  hipLaunchKernelGGL(k_atb_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     (const double*)part, nKS, Mp, Npd, Mdim, Nout, ld_out, out, tcol, tout);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_suffstats_workspace_size(int64_t T, int32_t L, int32_t Np) {
  return atb_ws(T, L, Np);
}

int pmg_suffstats(const float* P, const float* yext, int64_t T, int32_t L, int32_t N, int32_t Np,
                  double* yw, double* tw, void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && Np >= N + 1 && Np % 64 == 0, "pmg_suffstats: bad shape");
  PMG_REQUIRE(P && yext && yw && tw && workspace, "pmg_suffstats: null");
  PMG_REQUIRE(workspace_bytes >= pmg_suffstats_workspace_size(T, L, Np),
              "pmg_suffstats: workspace too small");
  return atb_run(P, L, L, yext, Np, Np, 0, T, yw, N, N, N, tw, workspace, as_stream(stream));
}

size_t pmg_joint_workspace_size(int64_t T, int32_t L) {
  return atb_ws(T > 1 ? T - 1 : 1, 2 * L, 2 * L);
}

int pmg_joint_accumulate(const float* alpha, const float* rho, int64_t T, int32_t L, double* S,
                         void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && alpha && rho && S && workspace, "pmg_joint_accumulate: bad args");
  PMG_REQUIRE(workspace_bytes >= pmg_joint_workspace_size(T, L), "pmg_joint_accumulate: workspace");
  hipStream_t st = as_stream(stream);
  if (T < 2) {
    PMG_HIP(hipMemsetAsync(S, 0, sizeof(double) * 4 * (size_t)L * L, st));
    return PMG_OK;
  }
  return atb_run(alpha, 2 * (int64_t)L, 2 * L, rho, 2 * (int64_t)L, 2 * L, 1, T - 1, S, 2 * L,
                 2 * L, -1, nullptr, workspace, st);
}

}  // extern "C"
