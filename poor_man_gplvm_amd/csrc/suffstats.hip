// Time contractions C[m,n] = sum_t A[t,m] * B[t+shift,n] on gfx950 fp32 MFMA.
//
//   * sufficient statistics, fit_tuning_helper.get_statistics (fit_tuning_helper.py:28-42):
//       y_w = P^T y (L,N), t_w = sum_t P (L)     A = P (T,L), B = [y | 1] (T,Np)
//   * pairwise joint for decode_latent (decoder.py:215-221 accumulated over the scan):
//       S = sum_{t<T-1} alpha_t (x) rho_{t+1}   A = alpha (T,2L), B = rho (T,2L), shift 1
//
// Both operands are time-major, which is exactly the per-lane layout of
// v_mfma_f32_32x32x2f32: lane (r = lane&31, h = lane>>5) supplies A[row r][k = h] and
// B[k = h][col r], i.e. 32 consecutive floats of one time row per half-wave, so K-tiles
// are staged row-major in LDS (float4 global loads, no transpose) and read back with
// conflict-free ds_read_b32.
// Products are exact fp32 (the instruction is an fma chain); each wave flushes its
// fp32 accumulators into f64 registers every 128 time steps and writes one f64
// partial per K-slice; slices are summed in f64 in a fixed order.
#include "pmg_common.h"

namespace pmg {

typedef float v16f __attribute__((ext_vector_type(16)));

// PMG_SS_EARLY_LOAD: issue the next K-tile's loads right after the split that consumes
// the staged values, two MFMA blocks before the barrier (C3: 0.182 -> 0.167 ms)
#ifndef PMG_SS_EARLY_LOAD
#define PMG_SS_EARLY_LOAD 1
#endif
constexpr int kFlush = 128;  // time steps per fp32 accumulation segment

// Workgroup tile 128 (m) x 128 (n), 4 waves as 2 x 2 of 64 x 64 (2 x 2 MFMA tiles each).
// K (time) advances in tiles of KB rows staged through LDS: the next tile is loaded
// into registers (float4, coalesced) while the MFMAs consume the current one.
constexpr int KB = 32;
constexpr int TM = 128, TN = 128;

__global__ void __launch_bounds__(256) k_atb(const float* __restrict__ A, int64_t lda, int Mdim,
                                             const float* __restrict__ B, int64_t ldb, int Ndim,
                                             int shift, int64_t K, int64_t KT, int nMT, int nNT,
                                             int nKS, int Mp, int Npd, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sA[KB][TM];
  __shared__ __attribute__((aligned(16))) float sB[KB][TN];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int mt = blockIdx.x % nMT;
  const int nt = (blockIdx.x / nMT) % nNT;
  const int ks = blockIdx.x / (nMT * nNT);
  const int wm = wid & 1, wn = wid >> 1;
  const int r = lane & 31, h = lane >> 5;
  const int64_t kb = (int64_t)ks * KT;
  const int64_t ke = kb + KT < K ? kb + KT : K;

  // staging map: each thread moves 4 float4 of A and 4 of B per K-tile
  // element e = tid + 256*q (q < 4): row = e / 32, col4 = e % 32
  const bool vecA = (lda & 3) == 0 && (Mdim & 3) == 0;
  const bool vecB = (ldb & 3) == 0 && (Ndim & 3) == 0;
  float4 ra[4], rb[4];
  auto load_tile = [&](int64_t t0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      const int row = e >> 5, c4 = (e & 31) * 4;
      const int64_t t = t0 + row;
      const int m = mt * TM + c4, n = nt * TN + c4;
      float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
      if (t < ke) {
        const float* ar = A + t * lda;
        const float* br = B + (t + shift) * ldb;
        if (vecA && m + 3 < Mdim) {
          va = *reinterpret_cast<const float4*>(ar + m);
        } else {
          va.x = m < Mdim ? ar[m] : 0.f;
          va.y = m + 1 < Mdim ? ar[m + 1] : 0.f;
          va.z = m + 2 < Mdim ? ar[m + 2] : 0.f;
          va.w = m + 3 < Mdim ? ar[m + 3] : 0.f;
        }
        if (vecB && n + 3 < Ndim) {
          vb = *reinterpret_cast<const float4*>(br + n);
        } else {
          vb.x = n < Ndim ? br[n] : 0.f;
          vb.y = n + 1 < Ndim ? br[n + 1] : 0.f;
          vb.z = n + 2 < Ndim ? br[n + 2] : 0.f;
          vb.w = n + 3 < Ndim ? br[n + 3] : 0.f;
        }
      }
      ra[q] = va;
      rb[q] = vb;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      const int row = e >> 5, c4 = (e & 31) * 4;
      *reinterpret_cast<float4*>(&sA[row][c4]) = ra[q];
      *reinterpret_cast<float4*>(&sB[row][c4]) = rb[q];
    }
  };

  double acc64[4][16];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc64[q][i] = 0.0;
  v16f c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0};
  int rows_in_seg = 0;

  const int am0 = wm * 64 + r, am1 = am0 + 32;
  const int bn0 = wn * 64 + r, bn1 = bn0 + 32;
  if (kb < ke) load_tile(kb);
  for (int64_t t0 = kb; t0 < ke; t0 += KB) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (t0 + KB < ke) load_tile(t0 + KB);  // in flight during the MFMAs below
#pragma unroll
    for (int kk = 0; kk < KB; kk += 2) {
      const float a0 = sA[kk + h][am0], a1 = sA[kk + h][am1];
      const float b0 = sB[kk + h][bn0], b1 = sB[kk + h][bn1];
      c00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, c00, 0, 0, 0);
      c01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, c01, 0, 0, 0);
      c10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, c10, 0, 0, 0);
      c11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, c11, 0, 0, 0);
    }
    rows_in_seg += KB;
    if (rows_in_seg >= kFlush || t0 + KB >= ke) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        acc64[0][i] += (double)c00[i];
        acc64[1][i] += (double)c01[i];
        acc64[2][i] += (double)c10[i];
        acc64[3][i] += (double)c11[i];
        c00[i] = c01[i] = c10[i] = c11[i] = 0.f;
      }
      rows_in_seg = 0;
    }
  }
  // C/D layout: col = lane&31, row = (i&3) + 8*(i>>2) + 4*h
  double* pp = part + (size_t)ks * Mp * Npd;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int mi = q >> 1, ni = q & 1;
    const int col = nt * TN + wn * 64 + ni * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = mt * TM + wm * 64 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
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
  nMT = (Mdim + TM - 1) / TM;
  nNT = (Ndim + TN - 1) / TN;
  Mp = nMT * TM;
  Npd = nNT * TN;
  // ~2 workgroups per CU over 256 CUs, K-slices of whole flush segments
  const int64_t tiles = (int64_t)nMT * nNT;
  int64_t want = (512 + tiles - 1) / tiles;
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
  const int64_t wgs = (int64_t)nMT * nNT * nKS;
  hipLaunchKernelGGL(k_atb, dim3((unsigned)wgs), dim3(256), 0, st, A, lda, Mdim, B,
                     ldb, Ndim, shift, K, KT, nMT, nNT, nKS, Mp, Npd, part);
  PMG_LAUNCH_CHECK();
  const int64_t total = (int64_t)Mdim * Npd;
  hipLaunchKernelGGL(k_atb_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     (const double*)part, nKS, Mp, Npd, Mdim, Nout, ld_out, out, tcol, tout);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}


// ---------------------------------------------------------------------------------
// Sufficient statistics on bf16 MFMA, exact products (integer spikes 0..127).
//
// y is an integer <= 127, exact in bf16.  P (f32) is split by truncation into
// P = hi + mid + lo with each part exact in bf16 (hi takes the top 8 significant
// bits, mid the next 8, lo the last 8; both remainders are exact in f32), so
// y_w = sum_t (hi + mid + lo) y is three v_mfma_f32_32x32x16_bf16 per tile whose
// products are exact; accumulation is f32 inside a 128-step segment and f64 across
// segments (same as the f32 path), at the bf16 MFMA rate instead of the f32 one.
//
// Operand layout: lane (r, h) of the 32x32x16 MFMA holds A[m=r][t=8h..8h+7] and
// B[t=8h..8h+7][n=r], i.e. 8 consecutive TIME steps.  P is time-major, so the
// transpose happens on the LDS write (each thread gathers 32 time rows of one m
// column with coalesced dword loads and writes 16-byte runs of its LDS row); the
// spikes are pre-transposed once per data set to bf16 [Np][Tp].
// LDS rows are 64 + 8 bf16 (144 B): the 16-byte reads/writes of 16 consecutive
// rows land on distinct bank quads.
// ---------------------------------------------------------------------------------
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
constexpr int KB3 = 64, ROW3 = KB3 + 8;


// bijective XCD-grouping of workgroup ids (consecutive logical ids share an XCD)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Per K-tile (64 time steps) each wave issues 24 MFMAs (2 output tiles x 3 parts x 4
// k-steps) on the current LDS buffer and, in their shadow, splits the NEXT tile's
// staged P values (16 per thread) into the other buffer: the split arithmetic (VALU)
// and the MFMAs overlap inside each wave instead of alternating across a barrier.  P
// rows are fetched with one buffer descriptor per K-tile whose extent ends at the
// K-slice end, so rows past it read 0 without per-row clamps or selects.
__global__ void __launch_bounds__(512) k_ptb3(const float* __restrict__ P, int L,
                                              const uint16_t* __restrict__ Ybt, int64_t Tp, int Np,
                                              int64_t K, int64_t KT, int nMT, int nNT, int nKS,
                                              int Mp, int Npd, double* __restrict__ part,
                                              double* __restrict__ twpart) {
  // double-buffered operands: 2 x (3 x 128 x 72 + 128 x 72) x 2 B = 147456 B
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][3][TM][ROW3];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][TN][ROW3];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lb % nMT;
  const int nt = (lb / nMT) % nNT;
  const int ks = lb / (nMT * nNT);
  const int wm = wid & 3, wn = wid >> 2;       // wave tile: 32 m x 64 n
  const int r = lane & 31, h = lane >> 5;
  const int64_t kb = (int64_t)ks * KT;
  const int64_t ke = kb + KT < K ? kb + KT : K;

  // staging: A column m_l = tid & 127, time rows 16*tg .. 16*tg+15 of the K-tile (tg
  // wave-uniform); B row n_l = tid >> 2, time quarter hq = tid & 3 (16 bf16 = 2 x 16 B).
  // Rows m >= L / n >= N only feed output rows/columns the reduction drops.
  const int m_l = tid & 127, tg = tid >> 7;
  const int n_l = tid >> 2, hq = tid & 3;
  const int mg = mt * TM + m_l;
  const int ng = nt * TN + n_l;
  const int mgc = mg < L ? mg : L - 1;
  const uint32_t voffA = (uint32_t)(16 * tg * L + mgc) * 4u;
  const uint32_t rowB = (uint32_t)L * 4u;
  const uint16_t* yrow = Ybt + (size_t)(ng < Np ? ng : Np - 1) * Tp + 16 * hq;
  float ra[16];
  uint4 rb0, rb1;
#define PMG_SS_LOAD(t0_)                                                                     \
  {                                                                                          \
    const int64_t t0l = (t0_);                                                               \
    const int64_t nrow = ke - t0l < 0 ? 0 : (ke - t0l > KB3 ? KB3 : ke - t0l);               \
    const int64_t tbase = t0l < K ? t0l : 0;                                                 \
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(                     \
        const_cast<float*>(P + tbase * (int64_t)L), (short)0, (int)(nrow * L * 4), 0x00020000); \
    _Pragma("unroll") for (int i = 0; i < 16; ++i)                                           \
      ra[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voffA, i * rowB, 0));  \
    const int64_t tb = t0l < Tp - KB3 ? t0l : Tp - KB3;                                      \
    rb0 = *reinterpret_cast<const uint4*>(yrow + tb);                                        \
    rb1 = *reinterpret_cast<const uint4*>(yrow + tb + 8);                                    \
  }
  double tsum = 0.0;                 // t_w partial of column mg (f64)
  // split values 8q .. 8q+7 of the staged rows into buffer buf; t_w in f32 per 8, then f64
#define PMG_SS_SPLIT(buf, q)                                                              \
  {                                                                                       \
    uint32_t hw[4], mw[4], lw[4];                                                         \
    _Pragma("unroll") for (int j = 0; j < 4; ++j)                                         \
      split3_pair(ra[8 * (q) + 2 * j], ra[8 * (q) + 2 * j + 1], hw[j], mw[j], lw[j]);    \
    const float s8 = ((ra[8 * (q)] + ra[8 * (q) + 1]) + (ra[8 * (q) + 2] + ra[8 * (q) + 3])) + \
                     ((ra[8 * (q) + 4] + ra[8 * (q) + 5]) + (ra[8 * (q) + 6] + ra[8 * (q) + 7])); \
    tsum += (double)s8;                                                                   \
    const int c = 16 * tg + 8 * (q);                                                      \
    *reinterpret_cast<uint4*>(&sA[buf][0][m_l][c]) = make_uint4(hw[0], hw[1], hw[2], hw[3]); \
    *reinterpret_cast<uint4*>(&sA[buf][1][m_l][c]) = make_uint4(mw[0], mw[1], mw[2], mw[3]); \
    *reinterpret_cast<uint4*>(&sA[buf][2][m_l][c]) = make_uint4(lw[0], lw[1], lw[2], lw[3]); \
  }
#define PMG_SS_STORE_B(buf)                                                               \
  {                                                                                       \
    *reinterpret_cast<uint4*>(&sB[buf][n_l][16 * hq]) = rb0;                              \
    *reinterpret_cast<uint4*>(&sB[buf][n_l][16 * hq + 8]) = rb1;                          \
  }
  double acc64[2][16];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc64[q][i] = 0.0;
  v16f c0 = {0}, c1 = {0};
  const int am = wm * 32 + r;
  const int bn0 = wn * 64 + r, bn1 = bn0 + 32;
#define PMG_SS_MFMA_K(buf, kk)                                                             \
  {                                                                                       \
    const v8bf b0 = *reinterpret_cast<const v8bf*>(&sB[buf][bn0][(kk) + 8 * h]);          \
    const v8bf b1 = *reinterpret_cast<const v8bf*>(&sB[buf][bn1][(kk) + 8 * h]);          \
    _Pragma("unroll") for (int sp = 0; sp < 3; ++sp) {                                    \
      const v8bf a = *reinterpret_cast<const v8bf*>(&sA[buf][sp][am][(kk) + 8 * h]);      \
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, c0, 0, 0, 0);                   \
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, c1, 0, 0, 0);                   \
    }                                                                                     \
  }
// one K-tile: MFMAs on buffer cur, the staged next tile split into buffer nxt between
// them, then the loads of the tile after that (their latency spans a whole K-tile)
#if PMG_SS_EARLY_LOAD
// the next loads as soon as the staged values are consumed (a quarter tile earlier)
#define PMG_SS_TILE(cur, nxt, tload)                                                      \
  PMG_SS_MFMA_K(cur, 0)                                                                   \
  PMG_SS_SPLIT(nxt, 0)                                                                    \
  PMG_SS_MFMA_K(cur, 16)                                                                  \
  PMG_SS_SPLIT(nxt, 1)                                                                    \
  PMG_SS_STORE_B(nxt)                                                                     \
  PMG_SS_LOAD(tload)                                                                      \
  PMG_SS_MFMA_K(cur, 32)                                                                  \
  PMG_SS_MFMA_K(cur, 48)                                                                  \
  __syncthreads();
#else
#define PMG_SS_TILE(cur, nxt, tload)                                                      \
  PMG_SS_MFMA_K(cur, 0)                                                                   \
  PMG_SS_SPLIT(nxt, 0)                                                                    \
  PMG_SS_MFMA_K(cur, 16)                                                                  \
  PMG_SS_MFMA_K(cur, 32)                                                                  \
  PMG_SS_SPLIT(nxt, 1)                                                                    \
  PMG_SS_STORE_B(nxt)                                                                     \
  PMG_SS_MFMA_K(cur, 48)                                                                  \
  PMG_SS_LOAD(tload)                                                                      \
  __syncthreads();
#endif

  if (kb < ke) {
    PMG_SS_LOAD(kb)
    PMG_SS_SPLIT(0, 0)
    PMG_SS_SPLIT(0, 1)
    PMG_SS_STORE_B(0)
    PMG_SS_LOAD(kb + KB3)
    __syncthreads();
    for (int64_t t0 = kb; t0 < ke; t0 += 2 * KB3) {   // 2 tiles = one kFlush segment
      PMG_SS_TILE(0, 1, t0 + 2 * KB3)
      PMG_SS_TILE(1, 0, t0 + 3 * KB3)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        acc64[0][i] += (double)c0[i];
        acc64[1][i] += (double)c1[i];
        c0[i] = c1[i] = 0.f;
      }
    }
  }
  double* pp = part + (size_t)ks * Mp * Npd;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int col = nt * TN + wn * 64 + q * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = mt * TM + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      pp[(size_t)row * Npd + col] = acc64[q][i];
    }
  }
  if (nt == 0) twpart[((size_t)ks * 4 + tg) * Mp + mg] = tsum;
#undef PMG_SS_LOAD
#undef PMG_SS_SPLIT
#undef PMG_SS_STORE_B
#undef PMG_SS_MFMA_K
#undef PMG_SS_TILE
}

// ---------------------------------------------------------------------------------
// The same statistics from P already split into its three bf16 planes by the backward
// smoother (PMG_PHASE_P_BF16X3, [3][T][ldp] uint16): no split here, so the kernel is the
// three exact-product bf16 MFMA GEMMs plus their operand staging.
//   A planes: each K-tile (64 time rows x 128 latents x 3 planes, 48 KiB) is staged
//     row-major (one 16-byte chunk = 8 latents of one time row per load / ds_write_b128)
//     into 256-byte LDS rows with the XOR swizzle ch ^ ((row & 3) << 2 | (row >> 2) & 3)
//     (cdna_hip_programming.md T10 image (b)), and read back with ds_read_b64_tr_b16, which
//     hands every lane 4 consecutive TIME steps of one latent: two reads are the 8 time
//     steps lane (r, h) of the 32x32x16 MFMA A operand holds.
//   B (spikes): time-contiguous bf16 [Np][Tp] as in k_ptb3.
//   t_w: the workgroup of neuron tile nt sums P = (hi + mid) + lo (exact in f32) of the
//     K-tiles with index % nNT == nt, so the four neuron tiles of a latent tile share the
//     work; f32 within a kFlush segment, then f64.
// ---------------------------------------------------------------------------------
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t img_off(int row, int ch) {
  return 256u * row + 16u * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__global__ void __launch_bounds__(512) k_ptb3q(const uint16_t* __restrict__ Pq, int64_t pq_stride, int ldp,
                                               int L, const uint16_t* __restrict__ Ybt, int64_t Tp, int Np,
                                               int64_t K, int64_t KT, int nMT, int nNT, int nKS, int Mp,
                                               int Npd, double* __restrict__ part, double* __restrict__ twpart) {
  // 2 x 3 x 64 x 256 B (A planes) + 2 x 128 x 72 x 2 B (B) = 135168 B
  __shared__ __attribute__((aligned(16))) uint8_t sA[2][3][KB3 * 256];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][TN][ROW3];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = lb % nMT;
  const int nt = (lb / nMT) % nNT;
  const int ks = lb / (nMT * nNT);
  const int wm = wid & 3, wn = wid >> 2;       // wave tile: 32 m x 64 n
  const int r = lane & 31, h = lane >> 5;
  const int64_t kb = (int64_t)ks * KT;
  const int64_t ke = kb + KT < K ? kb + KT : K;

  // A staging: chunk ch (latents mt*128 + 8 ch ..) of time rows rw and rw + 32
  const int ch = tid & 15, rw = tid >> 4;
  const int col = mt * TM + 8 * ch;
  const bool col_ok = col + 8 <= ldp;          // chunks past the row feed only dropped outputs
  // per-lane offsets only (a lane-dependent soffset would be a waterfall loop): rows rw
  // and rw + 32; out-of-range chunks point past the descriptor (reads return 0)
  const uint32_t voffA = col_ok ? (uint32_t)(rw * ldp + col) * 2u : 0x80000000u;
  const uint32_t voffA2 = col_ok ? voffA + (uint32_t)(32 * ldp) * 2u : 0x80000000u;
  // B staging (as k_ptb3)
  const int n_l = tid >> 2, hq = tid & 3;
  const int ng = nt * TN + n_l;
  const uint16_t* yrow = Ybt + (size_t)(ng < Np ? ng : Np - 1) * Tp + 16 * hq;
  u32x4 qa[3][2];
  uint4 rb0, rb1;
  auto load = [&](int64_t t0) {
    const int64_t nrow = ke - t0 < 0 ? 0 : (ke - t0 > KB3 ? KB3 : ke - t0);
    const int64_t tbase = t0 < K ? t0 : 0;
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(Pq + sp * pq_stride + tbase * (int64_t)ldp), (short)0, (int)(nrow * ldp * 2),
          0x00020000);
      qa[sp][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, voffA, 0, 0);
      qa[sp][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, voffA2, 0, 0);
    }
    const int64_t tb = t0 < Tp - KB3 ? t0 : Tp - KB3;
    rb0 = *reinterpret_cast<const uint4*>(yrow + tb);
    rb1 = *reinterpret_cast<const uint4*>(yrow + tb + 8);
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
      *reinterpret_cast<u32x4*>(&sA[buf][sp][img_off(rw, ch)]) = qa[sp][0];
      *reinterpret_cast<u32x4*>(&sA[buf][sp][img_off(rw + 32, ch)]) = qa[sp][1];
    }
    *reinterpret_cast<uint4*>(&sB[buf][n_l][16 * hq]) = rb0;
    *reinterpret_cast<uint4*>(&sB[buf][n_l][16 * hq + 8]) = rb1;
  };
  // t_w of this thread's 8 latents over its two staged rows
  float tacc[8];
  double tsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) tacc[j] = 0.f, tsum[j] = 0.0;
  auto tw_add = [&]() {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t a = qa[0][hh][i], b = qa[1][hh][i], c = qa[2][hh][i];
        tacc[2 * i] += (bf16_lo(a) + bf16_lo(b)) + bf16_lo(c);
        tacc[2 * i + 1] += (bf16_hi(a) + bf16_hi(b)) + bf16_hi(c);
      }
  };
  auto tw_flush = [&]() {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      tsum[j] += (double)tacc[j];
      tacc[j] = 0.f;
    }
  };
  // the staged K-tile of global index ti: its rows join t_w if this neuron tile owns it;
  // f32 sums close at the end of every 2-tile (kFlush) segment of the GLOBAL tile grid, so
  // the rounding does not depend on where the K-slices start (nor on the latent count)
  auto tw_tile = [&](int64_t ti) {
    const int t32 = __builtin_amdgcn_readfirstlane((int)ti);   // tile indices < 2^31
    if (t32 % nNT == nt) tw_add();
    if (t32 & 1) tw_flush();
  };

  double acc64[2][16];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc64[q][i] = 0.0;
  v16f c0 = {0}, c1 = {0};
  const int bn0 = wn * 64 + r, bn1 = bn0 + 32;
  // transposed-read addresses of the A operand: lane 4q + p of 16-lane group g reads row
  // (kk + 8 (g >> 1) + q [+ 4]), latents wm*32 + 16 (g & 1) + 4p .. + 3
  const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int ach = wm * 4 + 2 * (g & 1) + (pp >> 1);
  const uint32_t abyte = 8u * (pp & 1);
  auto mfma_k = [&](int buf, int kk) {
    const v8bf b0 = *reinterpret_cast<const v8bf*>(&sB[buf][bn0][kk + 8 * h]);
    const v8bf b1 = *reinterpret_cast<const v8bf*>(&sB[buf][bn1][kk + 8 * h]);
    const int row0 = kk + 8 * (g >> 1) + qq;
#pragma unroll
    for (int sp = 0; sp < 3; ++sp) {
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(&sA[buf][sp][img_off(row0, ach) + abyte]));
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(&sA[buf][sp][img_off(row0 + 4, ach) + abyte]));
      const v8bf a = __builtin_bit_cast(v8bf, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, c1, 0, 0, 0);
    }
  };

  int64_t tile = kb / KB3;                       // global K-tile index (t_w ownership)
  if (kb < ke) {
    load(kb);
    store(0);
    tw_tile(tile);
    load(kb + KB3);
    __syncthreads();
    int cur = 0;
    for (int64_t t0 = kb; t0 < ke; t0 += KB3, ++tile) {
      mfma_k(cur, 0);
      mfma_k(cur, 16);
      store(cur ^ 1);                            // tile t0 + KB3 (loaded a tile ago)
      if (t0 + KB3 < ke) tw_tile(tile + 1);
      load(t0 + 2 * KB3);
      mfma_k(cur, 32);
      mfma_k(cur, 48);
      __syncthreads();
      cur ^= 1;
      if (((t0 - kb) / KB3) & 1) {              // every 2 K-tiles: one kFlush segment
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          acc64[0][i] += (double)c0[i];
          acc64[1][i] += (double)c1[i];
          c0[i] = c1[i] = 0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc64[0][i] += (double)c0[i];
      acc64[1][i] += (double)c1[i];
    }
    tw_flush();
  }
  double* pq = part + (size_t)ks * Mp * Npd;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int oc = nt * TN + wn * 64 + q * 32 + r;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = mt * TM + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      pq[(size_t)row * Npd + oc] = acc64[q][i];
    }
  }
  // t_w: the 32 row-threads of each chunk summed in row order, one partial per (ks, nt);
  // the A buffers are free (the loop ended on a barrier)
  double(*sTw)[TM / 8][8] = reinterpret_cast<double(*)[TM / 8][8]>(&sA[0][0][0]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) sTw[rw][ch][j] = tsum[j];
  __syncthreads();
  if (tid < TM) {
    const int c8 = tid >> 3, j = tid & 7;
    double t = 0.0;
    for (int q = 0; q < 32; ++q) t += sTw[q][c8][j];
    twpart[((size_t)ks * nNT + nt) * Mp + mt * TM + tid] = t;
  }
}

// t_w[m] = sum over the 4 nKS partial rows, in one fixed order: block = 64 latents x
// 16 k-groups (group g sums rows k = g, g + 16, ... in k order, coalesced over m), then
// the 16 group sums in g order through LDS.  (One thread per latent summing every row
// put L threads, i.e. 8 waves, on the whole chip: ~16 us at C3.)
constexpr int kTwM = 64, kTwG = 16;
__global__ void __launch_bounds__(kTwM * kTwG) k_tw_reduce(const double* __restrict__ twpart, int nKS, int Mp,
                                                           int L, double* __restrict__ tw) {
  __shared__ double sp[kTwG][kTwM];
  const int mi = threadIdx.x % kTwM, g = threadIdx.x / kTwM;
  const int m = blockIdx.x * kTwM + mi;
  double s = 0.0;
  if (m < L)
    for (int k = g; k < 4 * nKS; k += kTwG) s += twpart[(size_t)k * Mp + m];
  sp[g][mi] = s;
  __syncthreads();
  if (g == 0 && m < L) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kTwG; ++q) t += sp[q][mi];
    tw[m] = t;
  }
}

// y_w (k_atb_reduce's per-element sums) and t_w (k_tw_reduce's) in ONE launch of
// 1024-thread blocks: blocks [0, nA) reduce y_w elements, the rest t_w rows, each with the
// arithmetic and order of the two separate kernels (bit-identical); one launch fewer per
// EM iteration
__global__ void __launch_bounds__(kTwM * kTwG) k_ss_reduce(const double* __restrict__ part, int nKS, int Mp, int Npd,
                                                           int L, int N, double* __restrict__ yw,
                                                           const double* __restrict__ twpart, double* __restrict__ tw,
                                                           int nA) {
  if ((int)blockIdx.x < nA) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)L * Npd) return;
    const int m = (int)(i / Npd), n = (int)(i % Npd);
    if (n >= N) return;
    double s = 0.0;
    for (int k = 0; k < nKS; ++k) s += part[((size_t)k * Mp + m) * Npd + n];
    yw[(size_t)m * N + n] = s;
    return;
  }
  __shared__ double sp[kTwG][kTwM];
  const int mi = threadIdx.x % kTwM, g = threadIdx.x / kTwM;
  const int m = ((int)blockIdx.x - nA) * kTwM + mi;
  double s = 0.0;
  if (m < L)
    for (int k = g; k < 4 * nKS; k += kTwG) s += twpart[(size_t)k * Mp + m];
  sp[g][mi] = s;
  __syncthreads();
  if (g == 0 && m < L) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kTwG; ++q) t += sp[q][mi];
    tw[m] = t;
  }
}

// the same over `rows` partial rows (k_ptb3q: nKS x nNT)
__global__ void __launch_bounds__(kTwM * kTwG) k_tw_reduce_n(const double* __restrict__ twpart, int rows, int Mp,
                                                             int L, double* __restrict__ tw) {
  __shared__ double sp[kTwG][kTwM];
  const int mi = threadIdx.x % kTwM, g = threadIdx.x / kTwM;
  const int m = blockIdx.x * kTwM + mi;
  double s = 0.0;
  if (m < L)
    for (int k = g; k < rows; k += kTwG) s += twpart[(size_t)k * Mp + m];
  sp[g][mi] = s;
  __syncthreads();
  if (g == 0 && m < L) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kTwG; ++q) t += sp[q][mi];
    tw[m] = t;
  }
}

// yext (T, Np) f32 -> ybt (Np, Tp) bf16 bits (truncation; exact for integers <= 256),
// zero for t >= T.  64 x 64 tiles through LDS.
__global__ void __launch_bounds__(256) k_spikes_bf16t(const float* __restrict__ yext, int64_t T,
                                                      int Np, uint16_t* __restrict__ ybt, int64_t Tp) {
  __shared__ uint16_t tile[64][66];
  const int64_t t0 = (int64_t)blockIdx.x * 64;
  const int n0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t t = t0 + i;
    const int n = n0 + tx;
    const float v = (t < T && n < Np) ? yext[t * Np + n] : 0.f;
    tile[i][tx] = (uint16_t)(__float_as_uint(v) >> 16);
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int n = n0 + i;
    const int64_t t = t0 + tx;
    if (n < Np && t < Tp) ybt[(size_t)n * Tp + t] = tile[tx][i];
  }
}

static int device_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

// One workgroup per CU (the kernel runs at one wave per SIMD: 73.7 KB LDS, 406
// registers), all in ONE round: tiles x K-slices <= #CUs.
static int ptb3_geometry(int64_t K, int Mdim, int Ndim, int& nMT, int& nNT, int& nKS, int64_t& KT,
                         int& Mp, int& Npd) {
  nMT = (Mdim + TM - 1) / TM;
  nNT = (Ndim + TN - 1) / TN;
  Mp = nMT * TM;
  Npd = nNT * TN;
  const int64_t tiles = (int64_t)nMT * nNT;
  int64_t want = device_cus() / tiles;
  if (want < 1) want = 1;
  KT = (K + want - 1) / want;
  KT = round_up(KT < kFlush ? kFlush : KT, kFlush);
  nKS = (int)((K + KT - 1) / KT);
  if (nKS < 1) nKS = 1;
  return 0;
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

int pmg_spikes_bf16t(const float* yext, int64_t T, int32_t Np, uint16_t* ybt, int64_t Tp, void* stream) {
  PMG_REQUIRE(yext && ybt && T > 0 && Np > 0 && Tp == round_up(T, KB3), "pmg_spikes_bf16t: bad args");
  dim3 grid((unsigned)(Tp / 64), (unsigned)((Np + 63) / 64));
  hipLaunchKernelGGL(k_spikes_bf16t, grid, dim3(256), 0, as_stream(stream), yext, T, Np, ybt, Tp);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

size_t pmg_suffstats_bf16_workspace_size(int64_t T, int32_t L, int32_t N) {
  int nMT, nNT, nKS, Mp, Npd;
  int64_t KT;
  ptb3_geometry(T, L, N, nMT, nNT, nKS, KT, Mp, Npd);
  return (size_t)nKS * Mp * (Npd + 4) * sizeof(double) + 256;
}

int pmg_suffstats_bf16(const float* P, const uint16_t* ybt, int64_t T, int64_t Tp, int32_t L, int32_t N,
                       int32_t Np, double* yw, double* tw, void* workspace, size_t workspace_bytes,
                       void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && Np >= N + 1 && Np % 64 == 0 && Tp == round_up(T, KB3),
              "pmg_suffstats_bf16: bad shape");
  PMG_REQUIRE(P && ybt && yw && tw && workspace, "pmg_suffstats_bf16: null");
  PMG_REQUIRE(workspace_bytes >= pmg_suffstats_bf16_workspace_size(T, L, N),
              "pmg_suffstats_bf16: workspace too small");
  int nMT, nNT, nKS, Mp, Npd;
  int64_t KT;
  // the ones column of yext is not used: t_w comes from the staged P values
  ptb3_geometry(T, L, N, nMT, nNT, nKS, KT, Mp, Npd);
  double* part = reinterpret_cast<double*>(workspace);
  double* twpart = part + (size_t)nKS * Mp * Npd;
  hipStream_t st = as_stream(stream);
  const int64_t wgs = (int64_t)nMT * nNT * nKS;
  hipLaunchKernelGGL(k_ptb3, dim3((unsigned)wgs), dim3(512), 0, st, P, L, ybt, Tp, N, T, KT, nMT, nNT,
                     nKS, Mp, Npd, part, twpart);
  PMG_LAUNCH_CHECK();
  const int64_t total = (int64_t)L * Npd;
  const int nA = (int)((total + kTwM * kTwG - 1) / (kTwM * kTwG));
  const int nT = (L + kTwM - 1) / kTwM;
  hipLaunchKernelGGL(k_ss_reduce, dim3((unsigned)(nA + nT)), dim3(kTwM * kTwG), 0, st, (const double*)part, nKS,
                     Mp, Npd, L, N, yw, (const double*)twpart, tw, nA);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

size_t pmg_suffstats_bf16x3_workspace_size(int64_t T, int32_t L, int32_t N) {
  int nMT, nNT, nKS, Mp, Npd;
  int64_t KT;
  ptb3_geometry(T, L, N, nMT, nNT, nKS, KT, Mp, Npd);
  return (size_t)nKS * Mp * Npd * sizeof(double) + (size_t)nKS * nNT * Mp * sizeof(double) + 256;
}

int pmg_suffstats_bf16x3(const uint16_t* Pq, int64_t ldp, const uint16_t* ybt, int64_t T, int64_t Tp, int32_t L,
                         int32_t N, int32_t Np, double* yw, double* tw, void* workspace, size_t workspace_bytes,
                         void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && Np >= N + 1 && Np % 64 == 0 && Tp == round_up(T, KB3) && ldp >= L &&
                  ldp % 8 == 0,
              "pmg_suffstats_bf16x3: bad shape");
  PMG_REQUIRE(Pq && ybt && yw && tw && workspace, "pmg_suffstats_bf16x3: null");
  PMG_REQUIRE(workspace_bytes >= pmg_suffstats_bf16x3_workspace_size(T, L, N),
              "pmg_suffstats_bf16x3: workspace too small");
  PMG_REQUIRE(T * ldp * 2 < ((int64_t)1 << 31), "pmg_suffstats_bf16x3: planes of %lld elements exceed 2 GiB",
              (long long)(T * ldp));
  int nMT, nNT, nKS, Mp, Npd;
  int64_t KT;
  ptb3_geometry(T, L, N, nMT, nNT, nKS, KT, Mp, Npd);
  double* part = reinterpret_cast<double*>(workspace);
  double* twpart = part + (size_t)nKS * Mp * Npd;
  hipStream_t st = as_stream(stream);
  const int64_t wgs = (int64_t)nMT * nNT * nKS;
  hipLaunchKernelGGL(k_ptb3q, dim3((unsigned)wgs), dim3(512), 0, st, Pq, T * ldp, (int)ldp, L, ybt, Tp, N, T, KT,
                     nMT, nNT, nKS, Mp, Npd, part, twpart);
  PMG_LAUNCH_CHECK();
  const int64_t total = (int64_t)L * Npd;
  hipLaunchKernelGGL(k_atb_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     (const double*)part, nKS, Mp, Npd, L, N, N, yw, -1, (double*)nullptr);
  PMG_LAUNCH_CHECK();
  // the nKS x nNT partial rows, in the fixed order of k_tw_reduce (its 4 nKS rows: nNT = 4)
  hipLaunchKernelGGL(k_tw_reduce_n, dim3((unsigned)((L + kTwM - 1) / kTwM)), dim3(kTwM * kTwG), 0, st,
                     (const double*)twpart, nKS * nNT, Mp, L, tw);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
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
