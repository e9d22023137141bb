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
// 2^-32 fixed-point number split into 5 balanced base-256 int8 digits; the digit
// GEMMs run on v_mfma_i32_32x32x32_i8 with exact int32 accumulation and are
// recombined in int64 (quantisation error <= 2^-33 per log(lam), i.e. ll exact to
// ~1e-9 for any realistic spike count).  Anything the integer path cannot represent
// (non-integer / >127 counts, weighted or 2-D masks) goes through the f64 kernel at
// the bottom.
//
// Output format (both paths): delta[t,l] = f32(ll[t,l] - r[t,b]) with
// r[t,b] = max over the 32-latent block b (f64), so an fp32 consumer recovers
// exp(s*(ll - max_l ll)) = exp(s*delta + phi) with 1-ulp accuracy near the max.
#include "pmg_common.h"

namespace pmg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kDig = 5;
constexpr double kQScale = 4294967296.0;  // 2^32
constexpr double kQInv = 1.0 / 4294967296.0;

// One wave per latent row: log(lam) -> 5 int8 digits, lamsum = sum_n m_n lam.
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
    int8_t dg[kDig] = {0, 0, 0, 0, 0};
    if (l < L && n < N) {
      const double lam = tuning[(size_t)l * N + n] * dt + 1e-20;
      const double lg = log(lam);
      if (!(fabs(lg) < 60.0)) flag = 1;
      long long q = llrint(lg * kQScale);
#pragma unroll
      for (int d = 0; d < kDig - 1; ++d) {
        const long long rr = ((q + 128) & 255) - 128;
        dg[d] = (int8_t)rr;
        q = (q - rr) >> 8;
      }
      dg[kDig - 1] = (int8_t)q;  // |q| <= 61 for |lg| < 60
      const float m = ma ? ma[n] : 1.f;
      ls += (double)m * lam;
    }
    const size_t o = (size_t)l * Kp + n;
#pragma unroll
    for (int d = 0; d < kDig; ++d) qd[d * plane + o] = dg[d];
  }
  ls = wave_sum_f64(ls);
  if (lane == 0) lamsum[l] = ls;
  if (__ballot(flag)) {
    if (lane == 0) atomicOr(bad, 1);
  }
}

// Workgroup tile 128 time bins x 64 latents, 8 waves as 4 (time) x 2 (latent); each
// wave owns 32 t x 32 l for all 5 digits (5 v16i accumulators).  MFMA operand A = y
// (rows = time), B = digits (cols = latent), so C[t][l] rows leave as 128-byte
// coalesced stores.  K (neurons) advances in 128-byte chunks staged through
// double-buffered LDS (rows of 144 B: the 16-byte fragment reads of 16 consecutive
// rows hit distinct bank quads); the next chunk's global loads are in flight during
// the current chunk's MFMAs.
// Fragment map (i8 32x32x32): lane (r = lane&31, h = lane>>5) supplies
// A[row r][k = 16h .. 16h+15] and B[k = 16h ..][col r]; the same (h, byte) -> k
// assignment on both operands keeps the K pairing consistent.
// C/D: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*h.
constexpr int EL = 64, EKC = 64, EROW = EKC + 16;
// EKC = 64: the double-buffered stage (sY 20 KB + sQ 51 KB) lets two workgroups share a
// CU, so one workgroup's epilogue and first loads overlap the other's MFMAs (at 128 B
// chunks the 129 KB stage held the CU alone).  Rows of 80 B: 16 consecutive rows still
// start on distinct bank quads (5 is odd).
constexpr int ESEG = EKC / 16;                 // 16-byte segments per staged row
constexpr int EQSEG = kDig * EL * ESEG;        // digit segments per chunk (1280)

__device__ __forceinline__ int xcd_group(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// MT time fragments per wave: the workgroup tile is ET = 128 MT time bins x 64 latents and
// each wave 32 MT t x 32 l (5 MT accumulators).  MT = 2 halves the digit planes' L2 -> LDS
// traffic per output (each plane chunk feeds twice the MFMAs) and the LDS reads per MFMA
// (one B fragment per digit serves both A fragments): the digit planes are re-read once
// per time tile, so their traffic is T / ET x 5 Lp Kp bytes.
// MT = 1: 80 accumulator registers, <= 128 per lane so two workgroups share a CU (one's
// epilogue beside the other's MFMAs); MT = 2: 160, one workgroup per CU.
// LL: the f64 ll rows are written (exact decodes); the EM passes skip those stores.
template <int MT, bool LL>
__global__ void __launch_bounds__(512, MT == 1 ? 4 : 2) k_emission_i8(
    const int8_t* __restrict__ yq, const int8_t* __restrict__ qd,
    const double* __restrict__ lamsum, const double* __restrict__ gconst,
    const uint8_t* __restrict__ ma_latent, int64_t T, int64_t Tp, int L, int Lp, int Kp, int nLT,
    float* __restrict__ delta, double* __restrict__ rblk, double* __restrict__ ll64) {
  constexpr int ET = 128 * MT;
  __shared__ __attribute__((aligned(16))) int8_t sY[2][ET][EROW];
  __shared__ __attribute__((aligned(16))) int8_t sQ[2][kDig][EL][EROW];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int lb = xcd_group(blockIdx.x, gridDim.x);   // l-tiles of one t-tile share an XCD
  const int lt = lb % nLT;
  const int64_t tt = lb / nLT;
  const int64_t t0 = tt * ET;
  const int l0 = lt * EL;
  const int r = lane & 31, h = lane >> 5;
  const int wt = wid & 3, wl = wid >> 2;
  const size_t plane = (size_t)Lp * Kp;

  // branch-free staging loads (Kp is a multiple of EKC): rows past Tp / Lp are
  // clamped -- their outputs are never written.  One spike segment and up to three
  // digit segments per thread.
  const int ysr = tid / ESEG, ysc = (tid % ESEG) * 16;   // + 128 m for segment m < MT
  const int8_t* yrow[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    int64_t ty = t0 + ysr + 128 * m;
    ty = ty < Tp ? ty : Tp - 1;
    yrow[m] = yq + ty * Kp + ysc;
  }
  const int8_t* qsrc[3];
  int qdst[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    int sgi = tid + 512 * i;
    sgi = sgi < EQSEG ? sgi : EQSEG - 1;          // the third slot is partly idle
    const int d = sgi / (EL * ESEG), rem = sgi % (EL * ESEG);
    const int row = rem / ESEG, col = (rem % ESEG) * 16;
    int lq = l0 + row;
    lq = lq < Lp ? lq : Lp - 1;
    qsrc[i] = qd + d * plane + (size_t)lq * Kp + col;
    qdst[i] = (d * EL + row) * EROW + col;
  }
  const bool q2 = tid + 1024 < EQSEG;
#define PMG_EM_LOAD(k0)                                                      \
  _Pragma("unroll") for (int m = 0; m < MT; ++m) ry[m] = *reinterpret_cast<const uint4*>(yrow[m] + (k0)); \
  rq0 = *reinterpret_cast<const uint4*>(qsrc[0] + (k0));                    \
  rq1 = *reinterpret_cast<const uint4*>(qsrc[1] + (k0));                    \
  rq2 = *reinterpret_cast<const uint4*>(qsrc[2] + (k0));
#define PMG_EM_STORE(b)                                                      \
  _Pragma("unroll") for (int m = 0; m < MT; ++m) *reinterpret_cast<uint4*>(&sY[b][ysr + 128 * m][ysc]) = ry[m]; \
  *reinterpret_cast<uint4*>(&sQ[b][0][0][0] + qdst[0]) = rq0;               \
  *reinterpret_cast<uint4*>(&sQ[b][0][0][0] + qdst[1]) = rq1;               \
  if (q2) *reinterpret_cast<uint4*>(&sQ[b][0][0][0] + qdst[2]) = rq2;
  uint4 ry[MT], rq0, rq1, rq2;

  v16i acc[MT][kDig];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int d = 0; d < kDig; ++d) acc[m][d] = (v16i){0};
  const int nch = Kp / EKC;
  PMG_EM_LOAD(0)
  PMG_EM_STORE(0)
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    const bool more = ch + 1 < nch;
    if (more) {   // in flight during the MFMAs
      PMG_EM_LOAD((ch + 1) * EKC)
    }
#pragma unroll
    for (int ks = 0; ks < EKC; ks += 32) {
      v4i a[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) a[m] = *reinterpret_cast<const v4i*>(&sY[buf][wt * 32 * MT + 32 * m + r][ks + 16 * h]);
#pragma unroll
      for (int d = 0; d < kDig; ++d) {
        const v4i b = *reinterpret_cast<const v4i*>(&sQ[buf][d][wl * 32 + r][ks + 16 * h]);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][d] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[m], b, acc[m][d], 0, 0, 0);
      }
    }
    if (more) {
      PMG_EM_STORE(buf ^ 1)   // the other buffer was last read before the previous barrier
      __syncthreads();
    }
  }
#undef PMG_EM_LOAD
#undef PMG_EM_STORE

  // Epilogue: digit recombination in f64 (Horner over the 5 int32 accumulators; exact
  // while |ll| < 2^21, every partial an integer below 2^53), f64 ll, the 32-latent block
  // max, coalesced rows.  Straight-line over the 16 outputs of a lane: every global
  // access goes through a buffer descriptor bounded by the workgroup's last valid row, and
  // lanes that must not write (latents past L; all but lane 0 of a block for rblk) aim
  // past the bound, so the 16 DPP reductions interleave freely (no per-row branches).
  const int nblk = Lp >> 5;
  const int blk = (l0 >> 5) + wl;
  if (blk >= nblk) return;
  const int l = l0 + wl * 32 + r;
  const bool lvalid = l < L;
  const bool lmask = lvalid && ma_latent && ma_latent[l] == 0;
  const bool over = !lvalid || lmask;                   // ll replaced by a constant
  const double ov = lvalid ? -1e20 : -INFINITY;
  const double lsum = lamsum[l];                        // l < Lp here
  const int64_t nrow64 = T - t0 < ET ? T - t0 : ET;     // >= 1
  const int nrow = (int)nrow64;
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(delta + t0 * (int64_t)L, (short)0,
                                                                       nrow * L * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rblk + t0 * (int64_t)nblk, (short)0,
                                                                       nrow * nblk * 8, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(gconst + t0), (short)0,
                                                                       nrow * 8, 0x00020000);
  // optional f64 ll rows (exact decodes): num_records 0 drops every store when absent
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
      ll64 ? (void*)(ll64 + t0 * (int64_t)L) : (void*)delta, (short)0, ll64 ? nrow * L * 8 : 0, 0x00020000);
  const uint32_t kNoWrite = 0x80000000u;                // past any bound above
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int tr = wt * 32 * MT + 32 * m + 4 * h + (i & 3) + 8 * (i >> 2);   // row within the workgroup tile
    double q = (double)acc[m][kDig - 1][i];
#pragma unroll
    for (int d = kDig - 2; d >= 0; --d) q = fma(q, 256.0, (double)acc[m][d][i]);
    const uint32_t g0 = __builtin_amdgcn_raw_buffer_load_b32(rg, tr * 8, 0, 0);
    const uint32_t g1 = __builtin_amdgcn_raw_buffer_load_b32(rg, tr * 8 + 4, 0, 0);
    const double gc = __hiloint2double((int)g1, (int)g0);
    double v = q * kQInv - lsum - gc;
    v = over ? ov : v;
    const double mx = (double)half_max32((float)v);
    const float dv = (float)(v - mx);
    const uint32_t od = lvalid ? (uint32_t)(tr * L + l - l0 + l0) * 4u : kNoWrite;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dv), rd, od, 0, 0);
    if constexpr (LL) {
      const unsigned long long vu = (unsigned long long)__double_as_longlong(v);
      const uint32_t ol = lvalid ? 2u * od : kNoWrite;
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)vu, rl, ol, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(vu >> 32), rl, ol + 4, 0, 0);
    }
    const uint32_t orb = r == 0 ? (uint32_t)(tr * nblk + blk) * 8u : kNoWrite;
    const unsigned long long mu = (unsigned long long)__double_as_longlong(mx);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)mu, rr, orb, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(mu >> 32), rr, orb + 4, 0, 0);
  }
}

// Generic f64 emission: any y, weighted and/or 2-D neuron masks.
// Block: 256 threads = tile of 16 time bins x 64 latents; thread (ty, tx) owns
// latent l0+tx and time bins t0+4ty .. +3.
__global__ void __launch_bounds__(256) k_emission_f64(
    const float* __restrict__ y, const float* __restrict__ ma, int ma_2d,
    const double* __restrict__ tuning, double dt, const double* __restrict__ gconst,
    const uint8_t* __restrict__ ma_latent, int64_t T, int L, int N, int Lp,
    float* __restrict__ delta, double* __restrict__ rblk, double* __restrict__ ll64) {
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
      if (ll64 && l < L) ll64[t * (int64_t)L + l] = v;
    }
  }
}

// Latent mask applied to an unmasked emission (delta0, rblk0) in the format above:
// ll[:, ma_latent == 0] = -1e20 (decoder.py:46) and the 32-latent block references
// re-derived over the kept bins, exactly as the emission kernels derive them.  Blocks
// without a masked bin are copied bit for bit; in the others a kept bin's ll is
// recovered as delta0 + rblk0 in f64 (exact up to delta0's own f32 rounding).  One wave
// per (time bin, pair of 32-latent blocks); T * L * 8 bytes + rblk traffic per mask, no
// contraction: this is what lets log_marginal_masked run the emission GEMM once for all
// its masks (model_selection_helper.get_downsampled_lml, :243-260).
// R masks (rows of ma_latent) from one read of (delta0, rblk0): mask r is written at
// column r L of delta rows of ldo floats and column r nblk of rblk rows of ldr doubles
// (R = 1: the plain layout).
__global__ void __launch_bounds__(256) k_latent_mask_apply(
    const float* __restrict__ delta0, const double* __restrict__ rblk0, int64_t T, int L, int nblk,
    const uint8_t* __restrict__ ma_latent, int R, float* __restrict__ delta, double* __restrict__ rblk,
    int64_t ldo, int64_t ldr) {
  const int lane = threadIdx.x & 63;
  const int npair = (nblk + 1) >> 1;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (w >= T * npair) return;               // uniform per wave
  const int64_t t = w / npair;
  const int l = (int)(w - t * npair) * 64 + lane;
  const int blk = l >> 5;
  const bool bvalid = blk < nblk;
  const bool lvalid = l < L;
  const double r0 = bvalid ? rblk0[t * nblk + blk] : 0.0;
  const float d0 = lvalid ? delta0[t * (int64_t)L + l] : 0.f;
  const double v0 = (double)d0 + r0;
  for (int r = 0; r < R; ++r) {
    const bool msk = lvalid && ma_latent[(int64_t)r * L + l] == 0;
    double v = msk ? -1e20 : v0;
    v = lvalid ? v : -INFINITY;
    const float anym = half_max32(msk ? 1.f : 0.f);
    const double mx = (double)half_max32((float)v);
    if (bvalid) {
      float* drow = delta + t * ldo + (int64_t)r * L;
      double* rrow = rblk + t * ldr + (int64_t)r * nblk;
      if (anym > 0.f) {
        if ((lane & 31) == 0) rrow[blk] = mx;
        if (lvalid) drow[l] = (float)(v - mx);
      } else {
        if ((lane & 31) == 0) rrow[blk] = r0;
        if (lvalid) drow[l] = d0;
      }
    }
  }
}

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_emission_workspace_size(int64_t T, int32_t L, int32_t N) {
  (void)T;
  const int64_t Lp = round_up(L, 32), Kp = round_up(N, 128);
  Carver c(nullptr);
  c.take<int8_t>(kDig * Lp * Kp);
  c.take<double>(Lp);
  c.take<int>(4);
  return c.off + 256;
}

int32_t* pmg_emission_range_flag(void* workspace, int64_t T, int32_t L, int32_t N) {
  (void)T;
  if (!workspace || L <= 0 || N <= 0) return nullptr;
  const int64_t Lp = round_up(L, 32), Kp = round_up(N, 128);
  Carver c(workspace);
  c.take<int8_t>(kDig * Lp * Kp);
  c.take<double>(Lp);
  return c.take<int>(4);
}

int pmg_emission_poisson(const int8_t* yq, const double* gconst, const double* tuning64,
                         const float* ma_neuron_1d, const uint8_t* ma_latent, double dt,
                         int64_t T, int32_t L, int32_t N, int32_t Kp, float* delta,
                         double* rblk, double* ll64, void* workspace, size_t workspace_bytes, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && N > 0, "pmg_emission_poisson: bad shape");
  PMG_REQUIRE(Kp == round_up(N, 128), "pmg_emission_poisson: Kp must be roundup(N,128)");
  PMG_REQUIRE(yq && gconst && tuning64 && delta && rblk && workspace, "pmg_emission_poisson: null");
  PMG_REQUIRE(workspace_bytes >= pmg_emission_workspace_size(T, L, N),
              "pmg_emission_poisson: workspace too small");
  hipStream_t st = as_stream(stream);
  const int Lp = (int)round_up(L, 32);
  Carver c(workspace);
  int8_t* qd = c.take<int8_t>(kDig * (size_t)Lp * Kp);
  double* lamsum = c.take<double>(Lp);
  int* bad = c.take<int>(4);   // sticky range flag (zero-filled workspace; the caller clears it)
  hipLaunchKernelGGL(k_rates_prepare, dim3((Lp + 3) / 4), dim3(256), 0, st, tuning64, L, N,
                     ma_neuron_1d, dt, Lp, Kp, qd, lamsum, bad);
  PMG_LAUNCH_CHECK();
  const int nLT = (Lp + EL - 1) / EL;
  const int64_t Tp = round_up(T, 64);   // rows of yq (pmg_spikes_prepare zero-pads to Tp)
  // one time fragment per wave: two workgroups share a CU (one's epilogue beside the
  // other's MFMAs).  MT = 2 (PMG_EMISSION_MT=2, env: tests / A/B timing) halves the
  // digit-plane traffic but holds the CU alone: C3 emission 0.223 -> 0.284 ms, so it is
  // not the default.
  const char* mt_s = getenv("PMG_EMISSION_MT");
  const int MT = (mt_s && atoi(mt_s) == 2) ? 2 : 1;
  const int64_t ET = 128 * MT;
  const int64_t nTT = (T + ET - 1) / ET;
  auto kern = MT == 2 ? (ll64 ? k_emission_i8<2, true> : k_emission_i8<2, false>)
                      : (ll64 ? k_emission_i8<1, true> : k_emission_i8<1, false>);
  hipLaunchKernelGGL(kern, dim3((unsigned)(nLT * nTT)), dim3(512), 0, st, yq, qd, lamsum, gconst, ma_latent, T, Tp,
                     L, Lp, Kp, nLT, delta, rblk, ll64);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_poisson_f64(const float* y, const double* gconst, const double* tuning64,
                             const float* ma_neuron, int32_t ma_is_2d, const uint8_t* ma_latent,
                             double dt, int64_t T, int32_t L, int32_t N, float* delta,
                             double* rblk, double* ll64, void* workspace, size_t workspace_bytes, void* stream) {
  (void)workspace;
  (void)workspace_bytes;
  PMG_REQUIRE(T > 0 && L > 0 && N > 0 && y && gconst && tuning64 && delta && rblk,
              "pmg_emission_poisson_f64: bad args");
  const int Lp = (int)round_up(L, 32);
  dim3 grid((unsigned)((T + 15) / 16), (unsigned)((L + 63) / 64));
  hipLaunchKernelGGL(k_emission_f64, grid, dim3(256), 0, as_stream(stream), y, ma_neuron,
                     ma_is_2d, tuning64, dt, gconst, ma_latent, T, L, N, Lp, delta, rblk, ll64);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

int pmg_emission_latent_mask(const float* delta0, const double* rblk0, int64_t T, int32_t L,
                             const uint8_t* ma_latent, float* delta, double* rblk, void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && delta0 && rblk0 && ma_latent && delta && rblk,
              "pmg_emission_latent_mask: bad args");
  PMG_REQUIRE(delta0 != delta && rblk0 != rblk, "pmg_emission_latent_mask: in-place is not supported");
  const int nblk = (int)(round_up(L, 32) / 32);
  const int64_t waves = T * ((nblk + 1) / 2);
  hipLaunchKernelGGL(k_latent_mask_apply, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, as_stream(stream),
                     delta0, rblk0, T, L, nblk, ma_latent, 1, delta, rblk, (int64_t)L, (int64_t)nblk);
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

// R masks at once, R <= 64: one wave per (32-latent block pair, row group); every lane
// turns its latent's R mask bytes into one bit word once, then walks the wave's rows
// (stride gridDim.y), each row's (delta0, rblk0) read once for all R masks and the next
// row's prefetched.  Mask r's outputs are bit-identical to k_latent_mask_apply's.
__global__ void __launch_bounds__(256) k_latent_mask_apply_rows(
    const float* __restrict__ delta0, const double* __restrict__ rblk0, int64_t T, int L, int nblk,
    const uint8_t* __restrict__ ma_latent, int R, float* __restrict__ delta, double* __restrict__ rblk) {
  const int lane = threadIdx.x & 63;
  const int npair = (nblk + 1) >> 1;
  const int pw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);   // block pair
  if (pw >= npair) return;                  // uniform per wave
  const int l = pw * 64 + lane;
  const int blk = l >> 5;
  const bool bvalid = blk < nblk;
  const bool lvalid = l < L;
  uint64_t keep = 0;                        // bit r: latent l kept by mask r
  if (lvalid)
    for (int r = 0; r < R; ++r) keep |= (uint64_t)(ma_latent[(int64_t)r * L + l] != 0) << r;
  // bit r: latent l's 32-block has a bin mask r drops (else the block is copied as is)
  uint64_t bmask = 0;
  for (int r = 0; r < R; ++r)
    bmask |= (uint64_t)(half_max32((lvalid && !((keep >> r) & 1)) ? 1.f : 0.f) > 0.f) << r;
  const int64_t ldo = (int64_t)R * L, ldr = (int64_t)R * nblk;
  int64_t t = blockIdx.y;
  double r0 = 0.0;
  float d0 = 0.f;
  if (t < T) {
    r0 = bvalid ? rblk0[t * nblk + blk] : 0.0;
    d0 = lvalid ? delta0[t * (int64_t)L + l] : 0.f;
  }
  for (; t < T; t += gridDim.y) {
    const int64_t tn = t + gridDim.y;       // prefetch the next row
    double r1 = 0.0;
    float d1 = 0.f;
    if (tn < T) {
      r1 = bvalid ? rblk0[tn * nblk + blk] : 0.0;
      d1 = lvalid ? delta0[tn * (int64_t)L + l] : 0.f;
    }
    const double v0 = (double)d0 + r0;
    float* drow = delta + t * ldo;
    double* rrow = rblk + t * ldr;
#pragma unroll 4
    for (int r = 0; r < R; ++r) {
      const bool msk = lvalid && !((keep >> r) & 1);
      double v = msk ? -1e20 : v0;
      v = lvalid ? v : -INFINITY;
      const bool anym = (bmask >> r) & 1;
      const double mx = (double)half_max32((float)v);
      if (bvalid) {
        if (anym) {
          if ((lane & 31) == 0) rrow[(int64_t)r * nblk + blk] = mx;
          if (lvalid) drow[(int64_t)r * L + l] = (float)(v - mx);
        } else {
          if ((lane & 31) == 0) rrow[(int64_t)r * nblk + blk] = r0;
          if (lvalid) drow[(int64_t)r * L + l] = d0;
        }
      }
    }
    r0 = r1;
    d0 = d1;
  }
}

int pmg_emission_latent_mask_batched(const float* delta0, const double* rblk0, int64_t T, int32_t L,
                                     const uint8_t* ma_latent, int32_t R, float* delta, double* rblk,
                                     void* stream) {
  PMG_REQUIRE(T > 0 && L > 0 && R >= 1 && R <= 65535 && delta0 && rblk0 && ma_latent && delta && rblk,
              "pmg_emission_latent_mask_batched: bad args");
  PMG_REQUIRE(L % 32 == 0, "pmg_emission_latent_mask_batched: L %% 32 == 0 (L=%d)", L);
  PMG_REQUIRE(delta0 != delta && rblk0 != rblk, "pmg_emission_latent_mask_batched: in-place is not supported");
  const int nblk = L / 32;
  if (R <= 64) {
    // ~32 waves per CU in total: block pairs x row groups
    const int npair = (nblk + 1) / 2;
    const int64_t groups64 = (int64_t)(8192 + npair - 1) / npair;
    const unsigned groups = (unsigned)(groups64 < T ? groups64 : T);
    hipLaunchKernelGGL(k_latent_mask_apply_rows, dim3((unsigned)((npair + 3) / 4), groups), dim3(256), 0,
                       as_stream(stream), delta0, rblk0, T, L, nblk, ma_latent, R, delta, rblk);
  } else {
    const int64_t waves = T * ((nblk + 1) / 2);
    hipLaunchKernelGGL(k_latent_mask_apply, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, as_stream(stream),
                       delta0, rblk0, T, L, nblk, ma_latent, R, delta, rblk, (int64_t)R * L, (int64_t)R * nblk);
  }
  PMG_LAUNCH_CHECK();
  return PMG_OK;
}

}  // extern "C"
