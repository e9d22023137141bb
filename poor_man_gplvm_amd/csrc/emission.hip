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
// 2^-32 fixed-point number split into kDig = 5 balanced base-256 int8 digits; the digit
// GEMMs run on v_mfma_i32_32x32x32_i8 with exact int32 accumulation and are recombined
// exactly in f64 (quantisation error <= 2^-33 per log(lam), i.e. ll exact to ~1e-9 for
// any realistic spike count).  PMG_EMISSION_DIGITS=4 (A/B builds only) keeps 4 digits of
// a 2^-24 fixed point: 2^-25 per log(lam) is a FIXED error per (l, n), so it adds up
// coherently over a slowly mixing chain's memory (nearly flat tuning: 1.7e-5 relative on
// the posterior, test_flat_tuning_cascade) -- not kept.  Anything the integer path
// cannot represent (non-integer / >127 counts, weighted or 2-D masks) goes through the
// f64 kernel at the bottom.
//
// Output format (both paths): delta[t,l] = f32(ll[t,l] - r[t,b]) with
// r[t,b] = max over the 32-latent block b (f64), so an fp32 consumer recovers
// exp(s*(ll - max_l ll)) = exp(s*delta + phi) with 1-ulp accuracy near the max.
#include "pmg_common.h"

#include <vector>

namespace pmg {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));


#ifndef PMG_EMISSION_DIGITS
#define PMG_EMISSION_DIGITS 5
#endif
constexpr int kDig = PMG_EMISSION_DIGITS;
static_assert(kDig == 4 || kDig == 5, "4 or 5 digits");
#ifndef PMG_EMISSION_DIAG
#define PMG_EMISSION_DIAG 0   // timing diagnostics of k_emission_yreg (A/B builds only)
#endif
// 2^(8 (kDig - 1)): the top digit stays within int8 (|q| <= 61) for |log lam| < 60
constexpr double kQScale = kDig == 5 ? 4294967296.0 : 16777216.0;
constexpr double kQInv = 1.0 / kQScale;

// One 4-wave workgroup per latent row: log(lam) -> kDig int8 digits, lamsum = sum_n m_n lam,
// and the pipelined kernel's per-latent constant lconst = -lamsum (+inf: latent masked by
// ma_latent, -inf: padding row l >= L).  Wave w takes the neuron groups j = w, w + 4, ...
// (neurons n = 64 j + lane); the products m_n lam pass through LDS so wave 0 adds each
// lane's values in ascending j, the order of a one-wave-per-row loop.
constexpr int kRpBlk = 16;   // neuron groups per LDS round
__global__ void __launch_bounds__(256) k_rates_prepare(
    const double* __restrict__ tuning, int L, int N, const float* __restrict__ ma, double dt,
    int Lp, int Kp, int8_t* __restrict__ qd, double* __restrict__ lamsum, int* __restrict__ bad,
    const uint8_t* __restrict__ ma_latent, double* __restrict__ lconst) {
  __shared__ double sml[kRpBlk][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l = blockIdx.x;
  if (l >= Lp) return;                                      // uniform per workgroup
  const size_t plane = (size_t)Lp * Kp;
  const int nj = Kp / 64;
  double ls = 0.0;
  int flag = 0;
  for (int jb = 0; jb < nj; jb += kRpBlk) {
    for (int j = jb + w; j < nj && j < jb + kRpBlk; j += 4) {
      const int n = 64 * j + lane;
      int8_t dg[kDig] = {};
      double mlam = 0.0;
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
        mlam = (double)m * lam;
      }
      sml[j - jb][lane] = mlam;
      const size_t o = (size_t)l * Kp + n;
#pragma unroll
      for (int d = 0; d < kDig; ++d) qd[d * plane + o] = dg[d];
    }
    __syncthreads();
    if (w == 0 && l < L)
      for (int j = jb; j < nj && j < jb + kRpBlk; ++j)
        if (64 * j + lane < N) ls += sml[j - jb][lane];
    __syncthreads();
  }
  if (__syncthreads_or(flag)) {
    if (threadIdx.x == 0) atomicOr(bad, 1);
  }
  if (w == 0) {
    ls = wave_sum_f64(ls);
    if (lane == 0) {
      lamsum[l] = ls;
      lconst[l] = l >= L ? -INFINITY : (ma_latent && ma_latent[l] == 0) ? INFINITY : -ls;
    }
  }
}

// Workgroup tile 128 time bins x 64 latents, 8 waves as 4 (time) x 2 (latent); each
// wave owns 32 t x 32 l for all kDig digits (kDig v16i accumulators).  MFMA operand A = y
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
// each wave 32 MT t x 32 l (kDig MT accumulators).  MT = 2 halves the digit planes' L2 -> LDS
// traffic per output (each plane chunk feeds twice the MFMAs) and the LDS reads per MFMA
// (one B fragment per digit serves both A fragments): the digit planes are re-read once
// per time tile, so their traffic is T / ET x kDig Lp Kp bytes.
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
      __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)vu, (uint32_t)(vu >> 32)}, rl, ol, 0, 0);
    }
    const uint32_t orb = r == 0 ? (uint32_t)(tr * nblk + blk) * 8u : kNoWrite;
    const unsigned long long mu = (unsigned long long)__double_as_longlong(mx);
    __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)mu, (uint32_t)(mu >> 32)}, rr, orb, 0, 0);
  }
}

// ---------------------------------------------------------------------------------
// Pipelined form (the default): the same digit GEMM and epilogue, reorganised around
// the two limits measured on k_emission_i8 at C3 (r02/r03 PMC: MFMA busy 25 %, every
// K-chunk waited for its own L2 round trip behind a barrier, and the 128 x 64 tile
// moved 350 B from L2 per MFMA).
// - Tiles of 256 time bins x 64 latents (16 waves as 8 (time) x 2 (latent), each wave
//   32 t x 32 l x kDig digits; 5 digits): 225 B of staged operands per MFMA.
// - One 1024-thread workgroup per CU walks its own list of tiles (the 8 latent tiles of a
//   time tile on one XCD, so y rows are re-read from that XCD's L2).  The operands of
//   each 64-neuron chunk (y: 256 rows x 64 B, digits: 5 x 64 rows x 64 B = 36 KiB) stream
//   through a 4-slot LDS ring filled by LDS-DMA (buffer_load ... lds) three chunks ahead
//   -- across tile boundaries, so the next tile's first chunks load during this tile's
//   epilogue.  Each wave waits only for its own DMA pieces with a counted vmcnt, then one
//   barrier publishes the chunk (and retires the reads of the slot the new DMA refills).
// - The per-tile constants (gconst rows, lconst = -lamsum / +inf masked / -inf padding)
//   arrive by the same DMA into 4 per-tile slots, so the epilogue issues no vector loads
//   (a VGPR load would make hipcc drain the DMA queue with vmcnt(0)).
// - LDS image: lane-linear 1 KiB pieces of 16 rows x 64 B; a row's 16-B segment s sits
//   at s ^ ((row >> 2) & 3), applied on the DMA source address and on the read, so the
//   ds_read_b128 fragment reads of 16 consecutive rows hit 16 distinct bank quads.
// Bit-identical to k_emission_i8 (same integer accumulators, same f64 epilogue order).
constexpr int PT = 256, PL = 64, PK = 64;          // tile time bins, tile latents, neurons per chunk
constexpr int PNS = 4;                              // ring slots (3 chunks in flight)
constexpr int PY = PT * PK;                         // y bytes per chunk
constexpr int PSTAGE = PY + kDig * PL * PK;         // 36864 B per chunk
constexpr int PPIECES = PSTAGE / 1024;              // 36 DMA pieces per chunk
constexpr int PCONST = 3072;                        // per tile: 256 gconst + 64 (+64 pad) lconst doubles
constexpr int PLDS = PNS * PSTAGE + 4 * PCONST;     // 159744 B

typedef __attribute__((address_space(3))) void lds_void_t;

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 63] (the immediate must be a literal)
__device__ __forceinline__ void vm_wait_upto(int n) {
#define PMG_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define PMG_VMW8(k) PMG_VMW(k) PMG_VMW(k + 1) PMG_VMW(k + 2) PMG_VMW(k + 3) PMG_VMW(k + 4) PMG_VMW(k + 5) \
  PMG_VMW(k + 6) PMG_VMW(k + 7)
  switch (n) {
    PMG_VMW8(0) PMG_VMW8(8) PMG_VMW8(16) PMG_VMW8(24) PMG_VMW8(32) PMG_VMW8(40) PMG_VMW8(48) PMG_VMW8(56)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef PMG_VMW8
#undef PMG_VMW
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pipe_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)(bytes > 0 ? bytes : 0),
                                           0x00020000);
}

// k_emission_pipe's tile list and DMA issue (per workgroup / wave constants)
struct PipeCtx {
  const int8_t* yq;
  const int8_t* qd;
  const double* lconst;
  const double* gconst;
  int8_t* smem;
  int64_t T, Tp;
  int Lp, Kp, nLT, plane, rb, slot, nx, wid, lane, vlane;
  bool cwave;

  __device__ __forceinline__ void tile_of(int ti, int64_t& t0, int& l0) const {
    const int g = rb + slot + ti * nx;
    const int tt = g / nLT;
    t0 = (int64_t)tt * PT;
    l0 = (g - tt * nLT) * PL;
  }
  // DMA of chunk kc of tile ti into ring slot sl (and, for kc == 0, the tile's constants)
  __device__ __forceinline__ void issue(int ti, int kc, int sl) const {
    int64_t t0;
    int l0;
    tile_of(ti, t0, l0);
    int8_t* dst = smem + sl * PSTAGE;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int p = wid + 16 * j;
      if (p < PPIECES) {
        if (p < PT / 16) {
          const int64_t o = (t0 + 16 * p) * Kp + kc * PK;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(pipe_rsrc(yq + o, Tp * Kp - o), (lds_void_t*)(dst + p * 1024),
                                                   16, vlane, 0, 0, 0);
        } else {
          const int pp = p - PT / 16, d = pp >> 2, rg = pp & 3;
          const int o = (l0 + 16 * rg) * Kp + kc * PK;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(pipe_rsrc(qd + d * plane + o, (int64_t)plane - o),
                                                   (lds_void_t*)(dst + p * 1024), 16, vlane, 0, 0, 0);
        }
      }
    }
    if (cwave && kc == 0) {
      int8_t* cdst = smem + PNS * PSTAGE + (ti & 3) * PCONST + (wid - 4) * 1024;
      if (wid < 6) {
        const int64_t o = t0 + (wid - 4) * 128;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(pipe_rsrc(gconst + o, (T - o) * 8), (lds_void_t*)cdst, 16,
                                                 lane * 16, 0, 0, 0);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(pipe_rsrc(lconst + l0, (int64_t)(Lp - l0) * 8), (lds_void_t*)cdst,
                                                 16, (lane & 31) * 16, 0, 0, 0);
      }
    }
  }
};

template <bool LL>
__global__ void __launch_bounds__(1024) k_emission_pipe(
    const int8_t* __restrict__ yq, const int8_t* __restrict__ qd, const double* __restrict__ lconst,
    const double* __restrict__ gconst, int64_t T, int64_t Tp, int L, int Lp, int Kp, int nLT,
    int ntile, float* __restrict__ delta, double* __restrict__ rblk, double* __restrict__ ll64,
    unsigned long long* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) int8_t smem[PLDS];
  (void)stamps;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wt = wid & 7, wl = wid >> 3;
  const int r = lane & 31, h = lane >> 5;

  // this workgroup's tiles: XCD x owns the contiguous range [x n / 8, (x + 1) n / 8) of the
  // time-major tile order; its nx workgroups take every nx-th tile of it
  const int nwg = gridDim.x, nx = nwg >> 3;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int rb = (int)((int64_t)ntile * xcd / 8), re = (int)((int64_t)ntile * (xcd + 1) / 8);
  const int mine = re - rb > slot ? (re - rb - slot + nx - 1) / nx : 0;
  if (mine == 0) return;                                   // uniform per workgroup
  const int nch = Kp / PK;                                 // >= 2 (Kp % 128 == 0)
  const int S = mine * nch;                                // chunks this workgroup streams

  const int plane = Lp * Kp;
  // DMA lane map: lane i fills row i >> 2 of a 16-row piece, physical segment i & 3, i.e.
  // logical segment (i & 3) ^ ((i >> 4) & 3).  Every wave-uniform part of a piece's source
  // goes into its buffer descriptor (base and extent: rows past Tp / Lp / T read as 0), so
  // the only per-lane operand is this offset.
  const int vlane = (lane >> 2) * Kp + ((lane & 3) ^ ((lane >> 4) & 3)) * 16;
  // fragment reads: logical segment h (k-step 0) of row 32 w + r; k-step 1 (segment 2 + h)
  // is that address ^ 32
  const int lrow = r * PK + (h ^ ((r >> 2) & 3)) * 16;
  const int aoff = wt * 32 * PK + lrow;
  const int boff = PY + wl * 32 * PK + lrow;
  const int npieces_w = 2 + (wid < PPIECES - 32);          // pieces p = wid, wid + 16, wid + 32 < 36
  const bool cwave = wid >= 4 && wid < 7;                  // carries one per-tile constant piece

  PipeCtx cx{yq, qd, lconst, gconst, smem, T, Tp, Lp, Kp, nLT, plane, rb, slot, nx, wid, lane, vlane, cwave};

  // VMEM stores one epilogue issues (at least: 16 delta + 16 rblk (+16 ll) instructions);
  // they are younger than the DMA pieces of the following chunks, so counting them only
  // lowers the wait (vmcnt retires in issue order: MI355X_MICROARCH.md, s_waitcnt)
  constexpr int NST = LL ? 48 : 32;
  // DMA cursor (chunk x + 3 as (tile, chunk))
  int dti = 0, dkc = 0;
  for (int x = 0; x < 3 && x < S; ++x) {
    cx.issue(dti, dkc, x);
    if (++dkc == nch) { dkc = 0; ++dti; }
  }
  v16i acc[kDig];
  int ti = 0, kc = 0;
  for (int x = 0; x < S; ++x) {
    {
      // my DMA pieces of chunks x + 1, x + 2 and the stores of epilogues at x - 3 .. x - 1
      // may stay in flight
      int n = 0;
      if (x + 1 < S) n += npieces_w + (cwave && kc == nch - 1);
      if (x + 2 < S) n += npieces_w + (cwave && kc == nch - 2);
      n += NST * ((x >= 1 && kc == 0) + (x >= 2 && kc == 1 % nch) + (x >= 3 && kc == 2 % nch));
      vm_wait_upto(n < 63 ? n : 63);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (x + 3 < S) {
      cx.issue(dti, dkc, (x + 3) & (PNS - 1));
      if (++dkc == nch) { dkc = 0; ++dti; }
    }
    if (kc == 0) {
#pragma unroll
      for (int d = 0; d < kDig; ++d) acc[d] = (v16i){0};
    }
    const int sbo = (x & (PNS - 1)) * PSTAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int8_t* sa = smem + sbo + (aoff ^ (32 * ks));
      const int8_t* sq = smem + sbo + (boff ^ (32 * ks));
      const v4i a = *reinterpret_cast<const v4i*>(sa);
#pragma unroll
      for (int d = 0; d < kDig; ++d) {
        const v4i b = *reinterpret_cast<const v4i*>(sq + d * PL * PK);
        acc[d] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[d], 0, 0, 0);
      }
    }
    const int cur = ti;
    if (++kc < nch) {
      continue;
    }
    kc = 0;
    ++ti;

    // epilogue of tile cur (k_emission_i8's arithmetic, constants from the LDS slot)
    int64_t t0;
    int l0;
    cx.tile_of(cur, t0, l0);
    const int8_t* cs = smem + PNS * PSTAGE + (cur & 3) * PCONST;
    const int nblk = Lp >> 5;
    const int blk = (l0 >> 5) + wl;
    const int l = l0 + wl * 32 + r;
    const bool lvalid = l < L && blk < nblk;
    const double lc = *reinterpret_cast<const double*>(cs + 2048 + (wl * 32 + r) * 8);
    const int64_t nrow64 = T - t0 < PT ? T - t0 : PT;
    const int nrow = (int)nrow64;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(delta + t0 * (int64_t)L, (short)0,
                                                                         nrow * L * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rblk + t0 * (int64_t)nblk, (short)0,
                                                                         nrow * nblk * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
        LL ? (void*)(ll64 + t0 * (int64_t)L) : (void*)delta, (short)0, LL ? nrow * L * 8 : 0, 0x00020000);
    // per-lane row bases (row 32 wt + 4 h); row i of the accumulator adds the uniform
    // (i & 3) + 8 (i >> 2).  Lanes that must not write start past every bound.  The empty
    // asm keeps the 16 per-row offsets from being hoisted out of the chunk loop.
    const int trb = wt * 32 + 4 * h;
    uint32_t od0 = lvalid ? (uint32_t)(trb * L + l) * 4u : 0x80000000u;
    uint32_t ob0 = (r == 0 && blk < nblk) ? (uint32_t)(trb * nblk + blk) * 8u : 0x80000000u;
    uint32_t ol0 = lvalid ? (uint32_t)(trb * L + l) * 8u : 0x80000000u;
    int gco = trb * 8;
    asm volatile("" : "+v"(od0), "+v"(ob0), "+v"(gco));
    if constexpr (LL) asm volatile("" : "+v"(ol0));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ri = (i & 3) + 8 * (i >> 2);
      double q = (double)acc[kDig - 1][i];
#pragma unroll
      for (int d = kDig - 2; d >= 0; --d) q = fma(q, 256.0, (double)acc[d][i]);
      const double gc = *reinterpret_cast<const double*>(cs + gco + ri * 8);
      double v = q * kQInv + lc - gc;   // lc = -lamsum: (q / kQScale - lamsum) - gc as k_emission_i8
      v = v == INFINITY ? -1e20 : v;      // masked latent (lc = +inf); padding latents: -inf
      const double mx = (double)half_max32((float)v);
      const float dv = (float)(v - mx);
      const uint32_t od = od0 + (uint32_t)(ri * L) * 4u;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dv), rd, od, 0, 0);
      if constexpr (LL) {
        const unsigned long long vu = (unsigned long long)__double_as_longlong(v);
        const uint32_t ol = ol0 + (uint32_t)(ri * L) * 8u;
        __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)vu, (uint32_t)(vu >> 32)}, rl, ol, 0, 0);
      }
      const uint32_t ob = ob0 + (uint32_t)(ri * nblk) * 8u;
      const unsigned long long mu = (unsigned long long)__double_as_longlong(mx);
      __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)mu, (uint32_t)(mu >> 32)}, rr, ob, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------------
// Register-resident spikes (N <= 512): the traffic form.  Measured on k_emission_i8 and
// k_emission_pipe at C3, the operand delivery from L2 caps at ~6.6 TB/s chip-wide, so
// time follows the staged bytes per output: 21.9 B (128 x 64 tiles), 17.6 B (256 x 64).
// Here each wave keeps its 32 time bins' spikes for the WHOLE neuron range in VGPRs as
// MFMA A fragments (Kp / 8 registers, loaded once per time tile) and only the digit
// planes stream: a workgroup of 8 waves = 256 time bins walks 32-latent tiles, every
// 128-neuron chunk of the tile's 5 digit planes (20 KiB, full 128-B rows) arriving by
// LDS-DMA into a 5-slot ring four chunks ahead and read by all 8 waves.  Staged bytes
// per output: 5 Kp / 256 = 10 (+ spikes once per time tile) -> 563 MB at C3.
// - Work items (time tile, 32-latent tile) in time-major order, a contiguous range per
//   workgroup (one per CU, persistent): the spikes and gconst of a time tile are loaded
//   once per range segment.
// - LDS image: 8-row x 128-B pieces; row segment s sits at s ^ ((row >> 1) & 7) (DMA
//   source and read), so the ds_read_b128 B-fragment reads of 16 rows hit 16 distinct
//   bank quads.
// - Per-latent constants (lconst) live in LDS for the whole launch.
// - The MFMAs take the digit planes as the A operand and the spikes as B, so the output
//   tile is transposed: a lane holds ONE time row (its gconst in one register) and 16 of
//   the item's 32 latents, 4 runs of 4 consecutive ones.  The block max is then 15 register
//   maxima and one half-wave swap per row (it was a 5-step cross-lane reduction per output
//   row), and delta leaves as 16-B stores: emission 164 -> 140 us at C3.
// Bit-identical to k_emission_i8 (same int32 digit sums, same f64 epilogue).
#ifndef PMG_RBLK_PAIRS
#define PMG_RBLK_PAIRS 1   // 0: one 8-byte rblk store per item (round 4; A/B builds)
#endif
#ifndef PMG_RBLK_RUN
#define PMG_RBLK_RUN 4
#endif
constexpr int kRbRun = PMG_RBLK_RUN;   // 2 or 4 blocks per rblk run
constexpr int RT = 256, RLW = 32;                       // time bins, latents per work item
constexpr int RLC_MAX = 4096;                            // latents of the LDS lconst table
// chunk of CK neurons (128 or 256 B digit rows): ring slots and DMA pieces
template <int CK> struct YRing {
  static constexpr int NS = CK == 256 ? 3 : 5;           // 2 or 4 chunks in flight (120 / 100 KiB)
  static constexpr int STAGE = kDig * RLW * CK;          // 40960 / 20480 B
  static constexpr int PIECES = STAGE / 1024;            // 40 / 20 pieces (8 waves: 5 / 2-3 each)
  static constexpr int RPP = 1024 / CK;                  // digit rows per piece
  static constexpr int NSEG = CK / 16;                   // 16-B segments per row
};

// The epilogue of one 256 x 32 work item of k_emission_yreg (k_emission_i8's
// arithmetic) on the transposed tile: the MFMAs ran with the digit planes as the A operand, so
// lane (r, h) holds time row t0 + tr (tr = 32 wid + r) and, in register i = 4 g + e, latent
// l0 + 8 g + 4 h + e.  The block max over the item's 32 latents is a register max plus one
// half-wave swap, each group of 4 latents one 16-B delta store (and two of ll64).  Returns
// the block max (the caller writes rblk).
template <bool LL, bool MASK>
__device__ __forceinline__ double item_rows(const v16i (&acc)[kDig], const double* __restrict__ slc, int l0,
                                            int64_t t0, int64_t T, int L, int tr, int h, double gcv,
                                            float* __restrict__ delta, double* __restrict__ ll64) {
  const int nrow = (int)(T - t0 < RT ? T - t0 : RT);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(delta + t0 * (int64_t)L, (short)0,
                                                                       nrow * L * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
      LL ? (void*)(ll64 + t0 * (int64_t)L) : (void*)delta, (short)0, LL ? nrow * L * 8 : 0, 0x00020000);
  const bool tvalid = tr < nrow;
  double vv[16];
  float fm = -INFINITY;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const double* lcg = slc + l0 + 8 * g + 4 * h;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e;
      // digit pairs combine exactly in int32 first (|a0 + 256 a1| < 2^31 for Kp <= 512)
      const int lo = acc[0][i] + (acc[1][i] << 8);
      const int mid = acc[2][i] + (acc[3][i] << 8);
      double q;
      if constexpr (kDig == 5) q = fma(fma((double)acc[4][i], 65536.0, (double)mid), 65536.0, (double)lo);
      else q = fma((double)mid, 65536.0, (double)lo);
      double v = q * kQInv + lcg[e] - gcv;   // lc = -lamsum: (q / kQScale - lamsum) - gc
      if constexpr (MASK) v = v == INFINITY ? -1e20 : v;   // masked latent (lc = +inf)
      vv[i] = v;                                            // padding latents: lc = -inf
      fm = fmaxf(fm, (float)v);
    }
  }
  {
    const auto pr = __builtin_amdgcn_permlane32_swap(__float_as_int(fm), __float_as_int(fm), false, false);
    fm = fmaxf(__int_as_float((int)pr[0]), __int_as_float((int)pr[1]));
  }
  const double mx = (double)fm;
  const bool vec4 = (L & 3) == 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int lg = l0 + 8 * g + 4 * h;
    float dv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) dv[e] = (float)(vv[4 * g + e] - mx);
    if (vec4) {
      const uint32_t od = (tvalid && lg < L) ? (uint32_t)(tr * L + lg) * 4u : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(
          (v4u){__float_as_uint(dv[0]), __float_as_uint(dv[1]), __float_as_uint(dv[2]), __float_as_uint(dv[3])},
          rd, od, 0, 0);
      if constexpr (LL) {
        const uint32_t ol = (tvalid && lg < L) ? (uint32_t)(tr * L + lg) * 8u : 0x80000000u;
        const unsigned long long a0 = __double_as_longlong(vv[4 * g]), a1 = __double_as_longlong(vv[4 * g + 1]);
        const unsigned long long a2 = __double_as_longlong(vv[4 * g + 2]), a3 = __double_as_longlong(vv[4 * g + 3]);
        __builtin_amdgcn_raw_buffer_store_b128(
            (v4u){(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32)}, rl, ol, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(
            (v4u){(uint32_t)a2, (uint32_t)(a2 >> 32), (uint32_t)a3, (uint32_t)(a3 >> 32)}, rl,
            ol == 0x80000000u ? ol : ol + 16u, 0, 0);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = tvalid && lg + e < L;
        const uint32_t od = ok ? (uint32_t)(tr * L + lg + e) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dv[e]), rd, od, 0, 0);
        if constexpr (LL) {
          const uint32_t ol = ok ? (uint32_t)(tr * L + lg + e) * 8u : 0x80000000u;
          const unsigned long long vu = __double_as_longlong(vv[4 * g + e]);
          __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)vu, (uint32_t)(vu >> 32)}, rl, ol, 0, 0);
        }
      }
    }
  }
  return mx;
}

template <int CK, int KC, bool LL, bool MASK>
__global__ void __launch_bounds__(512) k_emission_yreg(
    const int8_t* __restrict__ yq, const int8_t* __restrict__ qd, const double* __restrict__ lconst,
    const double* __restrict__ gconst, int64_t T, int64_t Tp, int L, int Lp, int nitem,
    float* __restrict__ delta, double* __restrict__ rblk, double* __restrict__ ll64,
    unsigned long long* __restrict__ stamps) {
  constexpr int Kp = KC * CK;
  constexpr int RNS = YRing<CK>::NS, RSTAGE = YRing<CK>::STAGE, RPIECES = YRing<CK>::PIECES;
  constexpr int RPP = YRing<CK>::RPP, NSEG = YRing<CK>::NSEG;
  __shared__ __attribute__((aligned(16))) int8_t smem[RNS * RSTAGE + RLC_MAX * 8];
  (void)stamps;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int nLT = Lp / RLW;
  const int i0 = (int)((int64_t)nitem * blockIdx.x / gridDim.x);
  const int i1 = (int)((int64_t)nitem * (blockIdx.x + 1) / gridDim.x);
  const int mine = i1 - i0;
  if (mine <= 0) return;                                  // uniform per workgroup
  const int S = mine * KC;

  // per-latent constants for the launch (plain loads; no DMA is in flight yet)
  double* slc = reinterpret_cast<double*>(smem + RNS * RSTAGE);
  for (int l = tid; l < Lp; l += 512) slc[l] = lconst[l];
  __syncthreads();

  const int plane = Lp * Kp;
  // DMA lane map: lane i fills row i / NSEG of an RPP-row piece, physical segment i % NSEG,
  // i.e. logical segment (i % NSEG) ^ f(row) with f = (row >> 1) & 7 (128-B rows) or
  // row & 15 (256-B rows); for row = RPP pr + i / NSEG both read f = (4 pr + (i >> 4)) % NSEG,
  // so a lane needs one offset per pr % (NSEG / 4)
  int vl[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    vl[q] = (lane / NSEG) * Kp + (((lane % NSEG) ^ ((4 * q + (lane >> 4)) & (NSEG - 1))) * 16);
  // B fragment of k-step ks (logical segment 2 ks + h of row r): bb ^ (32 ks)
  const int fr = CK == 256 ? (r & 15) : ((r >> 1) & 7);
  const int bb = r * CK + ((h ^ fr) * 16);
  const int npw = RPIECES / 8 + (wid < RPIECES % 8);     // pieces p = wid + 8 j < RPIECES

#define PMG_YR_ISSUE(x_)                                                                           \
  {                                                                                                \
    const int xi = (x_) / KC, xc = (x_) - xi * KC;                                                 \
    const int it = i0 + xi;                                                                        \
    const int tt = it / nLT;                                                                       \
    const int l0 = (it - tt * nLT) * RLW;                                                          \
    int8_t* dst = smem + ((x_) % RNS) * RSTAGE;                                                    \
    _Pragma("unroll") for (int j = 0; j < (RPIECES + 7) / 8; ++j) {                                \
      const int p = wid + 8 * j;                                                                   \
      if (p < RPIECES) {                                                                           \
        const int d = p / (RLW / RPP), pr = p % (RLW / RPP);                                       \
        const int o = d * plane + (l0 + RPP * pr) * Kp + xc * CK;                                  \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(                                                  \
            __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(qd + o), (short)0, kDig * plane - o, \
                                              0x00020000),                                         \
            (lds_void_t*)(dst + p * 1024), 16, vl[pr & (NSEG / 4 - 1)], 0, 0, 0);                  \
      }                                                                                            \
    }                                                                                              \
  }
  for (int x = 0; x < RNS - 1 && x < S; ++x) PMG_YR_ISSUE(x)

  v4i ya[Kp / 32];                  // A fragments: y[t0 + 32 wid + r][32 ks + 16 h .. +16]
  double gcv = 0.0;                 // gconst of the lane's time row t0 + 32 wid + r
  // VMEM stores per epilogue, a lower bound over both store forms (4 x 16 B delta + 1 rblk
  // (+ 8 x 16 B ll) when L % 4 == 0, 16 + 1 (+ 16) otherwise): the counted waits below
  // must never assume more younger stores than were issued
  constexpr int NST = (LL ? 13 : 5) - (PMG_RBLK_PAIRS ? 1 : 0);   // a held rblk block stores nothing
  v16i acc[kDig];
  int cur_tt = -1;
#if PMG_RBLK_PAIRS
  unsigned long long rb_h0 = 0, rb_h1 = 0, rb_h2 = 0;   // held block maxima of the open run
  int rb_n = 0;                                          // (uniform) blocks held
#endif
  for (int xi = 0; xi < mine; ++xi) {
    const int it = i0 + xi;
    const int tt = it / nLT;
    const int l0 = (it - tt * nLT) * RLW;
    const int64_t t0 = (int64_t)tt * RT;
    if (tt != cur_tt) {
      // new time tile: this wave's 32 spike rows and its rows' gconst into registers, then
      // a full vmcnt drain (the pending DMA pieces retire with it; hipcc's own waits then
      // know the loads are done)
      int64_t ty = t0 + 32 * wid + r;
      ty = ty < Tp ? ty : Tp - 1;
      const int8_t* yrow = yq + ty * Kp + 16 * h;
#pragma unroll
      for (int ks = 0; ks < Kp / 32; ++ks) ya[ks] = *reinterpret_cast<const v4i*>(yrow + 32 * ks);
      {
        int64_t tg = t0 + 32 * wid + r;
        tg = tg < T ? tg : T - 1;
        gcv = gconst[tg];
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
      cur_tt = tt;
    }
#pragma unroll
    for (int d = 0; d < kDig; ++d) acc[d] = (v16i){0};
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int x = xi * KC + c;
      {
        // my DMA pieces of chunks x + 1 .. x + RNS - 2 and the stores of the epilogues at
        // chunks x - RNS + 1 .. x - 1 (younger than piece x) may stay in flight
        int n = 0;
#pragma unroll
        for (int j = 1; j <= RNS - 2; ++j) n += (x + j < S) ? npw : 0;
#pragma unroll
        for (int j = 1; j <= RNS - 1; ++j) n += (x - j >= 0 && ((x - j) % KC) == KC - 1) ? NST : 0;
        vm_wait_upto(n < 63 ? n : 63);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      const int8_t* sq = smem + (x % RNS) * RSTAGE;
      // B fragments one k-step ahead: the 5 reads of k-step ks + 1 are issued before ks's
      // MFMAs (the scheduling barriers keep them there; hipcc's own schedule waited on each
      // read right before its MFMA, 2 % of the kernel)
      v4i bq[2][kDig];
#pragma unroll
      for (int d = 0; d < kDig; ++d) bq[0][d] = *reinterpret_cast<const v4i*>(sq + d * RLW * CK + bb);
#pragma unroll
      for (int ks = 0; ks < CK / 32; ++ks) {
        if (ks + 1 < CK / 32) {
          const int bn = bb ^ (32 * (ks + 1));
#pragma unroll
          for (int d = 0; d < kDig; ++d) bq[(ks + 1) & 1][d] = *reinterpret_cast<const v4i*>(sq + d * RLW * CK + bn);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int d = 0; d < kDig; ++d) {
#if PMG_EMISSION_DIAG == 2
          // timing diagnostic (A/B builds only): the B reads without the MFMAs
          acc[d][0] += bq[ks & 1][d][0] ^ ya[(CK / 32) * c + ks][1];
#elif PMG_EMISSION_DIAG == 3
          // timing diagnostic (A/B builds only): neither the B reads nor the MFMAs
          acc[d][0] += ya[(CK / 32) * c + ks][1] + d;
#else
          acc[d] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bq[ks & 1][d], ya[(CK / 32) * c + ks], acc[d], 0, 0, 0);
#endif
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ks == 0) {
          // the next DMA behind the first k-step's MFMAs (their issue hides its SALU work)
          __builtin_amdgcn_sched_barrier(0);
          if (x + RNS - 1 < S) PMG_YR_ISSUE(x + RNS - 1)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }

#if PMG_EMISSION_DIAG == 1
    // timing diagnostic (A/B builds only, wrong results): the epilogue's stores without its
    // arithmetic (same store count, so the counted vmcnt waits stay as in the real kernel)
    {
      const int nrow = (int)(T - t0 < RT ? T - t0 : RT);
      const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(delta + t0 * (int64_t)L, (short)0,
                                                                           nrow * L * 4, 0x00020000);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rblk + t0 * (int64_t)(Lp >> 5), (short)0,
                                                                           nrow * (Lp >> 5) * 8, 0x00020000);
      const int tr = 32 * wid + r;
      int sacc = 0;
#pragma unroll
      for (int d = 0; d < kDig; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc += acc[d][i];
      const uint32_t sv = (uint32_t)sacc;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int lg = l0 + 8 * gq + 4 * h;
        const uint32_t od = (tr < nrow && lg < L) ? (uint32_t)(tr * L + lg) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128((v4u){sv, sv, sv, sv}, rd, od, 0, 0);
      }
      const uint32_t ob = (h == 0 && tr < nrow) ? (uint32_t)(tr * (Lp >> 5) + (l0 >> 5)) * 8u : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b64((u32x2){sv, sv}, rr, ob, 0, 0);
    }
    continue;
#endif
    // epilogue (item_rows), then the item's block maxima
    {
      const int nblk = Lp >> 5;
      const int blk = l0 >> 5;
      const int64_t nrow64 = T - t0 < RT ? T - t0 : RT;
      const int nrow = (int)nrow64;
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rblk + t0 * (int64_t)nblk, (short)0,
                                                                           nrow * nblk * 8, 0x00020000);
      const int tr = 32 * wid + r;
      const bool tvalid = tr < nrow;
      const double mx = item_rows<LL, MASK>(acc, slc, l0, t0, T, L, tr, h, gcv, delta, ll64);
      const unsigned long long mu = (unsigned long long)__double_as_longlong(mx);
#if PMG_RBLK_PAIRS
      // rblk in runs of up to kRbRun blocks: a block whose successor is this workgroup's next
      // item (same time tile) and does not end a run is held in registers and written with
      // the run, so each row's 8-byte block maxima reach memory in fewer, wider partial-line
      // writes (one 8-byte store per item before)
      if ((blk % kRbRun) != kRbRun - 1 && blk + 1 < nLT && xi + 1 < mine) {
        if (rb_n == 0) rb_h0 = mu;
        else if (rb_n == 1) rb_h1 = mu;
        else rb_h2 = mu;
        ++rb_n;
      } else if (rb_n > 0) {
        const uint32_t ob = (h == 0 && tvalid) ? (uint32_t)(tr * nblk + blk - rb_n) * 8u : 0x80000000u;
        if (rb_n == 1) {
          __builtin_amdgcn_raw_buffer_store_b128((v4u){(uint32_t)rb_h0, (uint32_t)(rb_h0 >> 32), (uint32_t)mu,
                                                       (uint32_t)(mu >> 32)}, rr, ob, 0, 0);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128((v4u){(uint32_t)rb_h0, (uint32_t)(rb_h0 >> 32), (uint32_t)rb_h1,
                                                       (uint32_t)(rb_h1 >> 32)}, rr, ob, 0, 0);
          const uint32_t ob2 = ob == 0x80000000u ? ob : ob + 16u;
          if (rb_n == 2)
            __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)mu, (uint32_t)(mu >> 32)}, rr, ob2, 0, 0);
          else
            __builtin_amdgcn_raw_buffer_store_b128((v4u){(uint32_t)rb_h2, (uint32_t)(rb_h2 >> 32), (uint32_t)mu,
                                                         (uint32_t)(mu >> 32)}, rr, ob2, 0, 0);
        }
        rb_n = 0;
      } else
#endif
      {
        const uint32_t ob = (h == 0 && tvalid) ? (uint32_t)(tr * nblk + blk) * 8u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)mu, (uint32_t)(mu >> 32)}, rr, ob, 0, 0);
      }
    }
  }
#undef PMG_YR_ISSUE
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
  c.take<double>(Lp);
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
  double* lconst = c.take<double>(Lp);
  hipLaunchKernelGGL(k_rates_prepare, dim3(Lp), dim3(256), 0, st, tuning64, L, N,
                     ma_neuron_1d, dt, Lp, Kp, qd, lamsum, bad, ma_latent, lconst);
  PMG_LAUNCH_CHECK();
  const int64_t Tp = round_up(T, 64);   // rows of yq (pmg_spikes_prepare zero-pads to Tp)
  // pipelined kernel unless PMG_EMISSION_PIPE=0 (env: tests / A/B timing); its 32-bit
  // offsets need the digit planes and a 256-row slab of y below 2^31 bytes
  const char* pipe_s = getenv("PMG_EMISSION_PIPE");
  // register-resident spikes for Kp <= 512 (PMG_EMISSION_PIPE=1 forces the 256 x 64 ring
  // kernel, 0 the original k_emission_i8)
  const bool yreg = !(pipe_s && (pipe_s[0] == '0' || pipe_s[0] == '1')) && Kp <= 512 && Lp <= RLC_MAX &&
                    (int64_t)kDig * Lp * Kp < (1ll << 31) && T < (1ll << 38);
  if (yreg) {
    const int nLT32 = Lp / RLW;
    const int64_t nitem64 = (T + RT - 1) / RT * nLT32;
    PMG_REQUIRE(nitem64 < (1ll << 30), "pmg_emission_poisson: too many tiles (%lld)", (long long)nitem64);
    const int nitem = (int)nitem64;
    int nwg = device_cu_count();
    if (nwg > nitem) nwg = nitem;
    unsigned long long* ystamps = nullptr;
#define PMG_YR_LAUNCH(CK, KC)                                                                               \
  {                                                                                                         \
    auto kern = ll64 ? (ma_latent ? k_emission_yreg<CK, KC, true, true> : k_emission_yreg<CK, KC, true, false>) \
                     : (ma_latent ? k_emission_yreg<CK, KC, false, true> : k_emission_yreg<CK, KC, false, false>); \
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(512), 0, st, yq, qd, lconst, gconst, T, Tp, L, Lp, nitem, \
                       delta, rblk, ll64, ystamps);                                                        \
  }
    // 256-neuron chunks where they divide Kp (fewer barriers per MFMA), else 128
    switch (Kp) {
      case 128: PMG_YR_LAUNCH(128, 1); break;
      case 256: PMG_YR_LAUNCH(256, 1); break;
      case 384: PMG_YR_LAUNCH(128, 3); break;
      default: PMG_YR_LAUNCH(256, 2); break;
    }
#undef PMG_YR_LAUNCH
    PMG_LAUNCH_CHECK();
    return PMG_OK;
  }
  const bool pipe = !(pipe_s && pipe_s[0] == '0') && (int64_t)kDig * Lp * Kp < (1ll << 31) &&
                    (int64_t)PT * Kp < (1ll << 31) && T < (1ll << 38);
  if (pipe) {
    const int nLTp = (Lp + PL - 1) / PL;
    const int64_t ntile64 = (T + PT - 1) / PT * nLTp;
    PMG_REQUIRE(ntile64 < (1ll << 30), "pmg_emission_poisson: too many tiles (%lld)", (long long)ntile64);
    const int ntile = (int)ntile64;
    int nwg = device_cu_count() & ~7;
    if (nwg < 8) nwg = 8;
    auto kern = ll64 ? k_emission_pipe<true> : k_emission_pipe<false>;
    unsigned long long* stamps = nullptr;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(1024), 0, st, yq, qd, lconst, gconst, T, Tp, L, Lp, Kp,
                       nLTp, ntile, delta, rblk, ll64, stamps);
    PMG_LAUNCH_CHECK();
    return PMG_OK;
  }
  const int nLT = (Lp + EL - 1) / EL;
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
