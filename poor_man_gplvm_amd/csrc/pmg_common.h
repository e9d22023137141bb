// Shared helpers for the gfx950 kernels of libpmg_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pmg.h"

namespace pmg {

// thread-local last error message (pmg_last_error)
void set_error(const char* fmt, ...);

#define PMG_HIP(call)                                                            \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) {                                                      \
      ::pmg::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call,                \
                       hipGetErrorString(e_));                                   \
      return PMG_EHIP;                                                           \
    }                                                                            \
  } while (0)

#define PMG_LAUNCH_CHECK()                                                       \
  do {                                                                           \
    hipError_t e_ = hipGetLastError();                                           \
    if (e_ != hipSuccess) {                                                      \
      ::pmg::set_error("%s:%d launch: %s", __FILE__, __LINE__,                   \
                       hipGetErrorString(e_));                                   \
      return PMG_EHIP;                                                           \
    }                                                                            \
  } while (0)

#define PMG_REQUIRE(cond, ...)                                                   \
  do {                                                                           \
    if (!(cond)) {                                                               \
      ::pmg::set_error(__VA_ARGS__);                                             \
      return PMG_EINVAL;                                                         \
    }                                                                            \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Spin bound of the persistent kernels' grid barriers, in 100 MHz real-time clock
// ticks: `def` (2 s) unless PMG_DEBUG_SPIN_TICKS overrides it (tests force a timeout
// with a tiny bound to check that the host raises on the sticky timeout word).
// Persistent kernels whose workgroups wait on one another (the relaxation kernels' grid
// barriers, the Adam loop's cross-workgroup decision pipeline) need every workgroup of
// the grid resident at once.  Every such launch first checks it against the occupancy
// query (blocks per CU x CUs, cached per kernel / block / LDS size) and fails with
// hipErrorCooperativeLaunchTooLarge instead of launching a grid that could never be
// co-resident.  PMG_COOP=1 (env) launches them with hipLaunchCooperativeKernel, which
// also holds the launch until the whole grid can be placed (measured at C3: +86 us per
// EM iteration over the five persistent launches, 890 -> 827 EM it/s, so it is opt-in;
// without it, a grid kept off part of the device by other work ends its bounded spins
// with PMG_ETIMEOUT rather than hanging).
static inline int device_cu_count() {
  static int ncu = 0;
  if (ncu <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

static inline bool coop_launch_enabled() {
  static int coop = -1;
  if (coop < 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess)
      v = 0;
    const char* e = getenv("PMG_COOP");
    coop = (v && e && *e && *e != '0') ? 1 : 0;
  }
  return coop == 1;
}

// blocks of kernel k (block threads, lds bytes) that fit one CU, cached
static inline int occupancy_per_cu(const void* k, int threads, size_t lds) {
  struct Entry { const void* k; int threads; size_t lds; int n; };
  static Entry cache[64];
  static int used = 0;
  for (int i = 0; i < used; ++i)
    if (cache[i].k == k && cache[i].threads == threads && cache[i].lds == lds) return cache[i].n;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, threads, lds) != hipSuccess) n = 0;
  if (used < 64) cache[used++] = Entry{k, threads, lds, n};
  return n;
}

template <typename P>
static inline hipError_t launch_persistent(void (*k)(P), dim3 grid, dim3 block, size_t lds, hipStream_t st, P p) {
  const void* kp = reinterpret_cast<const void*>(k);
  const int64_t blocks = (int64_t)grid.x * grid.y * grid.z;
  const int per_cu = occupancy_per_cu(kp, (int)(block.x * block.y * block.z), lds);
  if ((int64_t)per_cu * device_cu_count() < blocks) return hipErrorCooperativeLaunchTooLarge;
  if (!coop_launch_enabled()) {
    hipLaunchKernelGGL(k, grid, block, lds, st, p);
    return hipGetLastError();
  }
  void* args[] = {&p};
  return hipLaunchCooperativeKernel(kp, grid, block, args, (unsigned)lds, st);
}

static inline uint64_t spin_ticks(uint64_t def) {
  const char* e = getenv("PMG_DEBUG_SPIN_TICKS");
  if (!e || !*e) return def;
  return (uint64_t)strtoull(e, nullptr, 10);
}

// workspace carving: 256-byte aligned slices
struct Carver {
  char* base;
  size_t off;
  explicit Carver(void* b) : base(static_cast<char*>(b)), off(0) {}
  template <class T>
  T* take(size_t count) {
    off = (off + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
};

// ---------------------------------------------------------------------------
// wave64 reductions through DPP (row ops) + row_bcast, result broadcast from
// lane 63 with readlane (wave-uniform SGPR value).
// dpp_ctrl: quad_perm[1,0,3,2]=0xB1, quad_perm[2,3,0,1]=0x4E,
// row_half_mirror=0x141, row_mirror=0x140, row_bcast15=0x142, row_bcast31=0x143
// ---------------------------------------------------------------------------
template <int CTRL, int ROWMASK = 0xf, int BANKMASK = 0xf, bool BC = false>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, BANKMASK, BC));
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  v += dppf<0x142, 0xa>(v);
  v += dppf<0x143, 0xc>(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// two independent sums (interleaved for ILP)
__device__ __forceinline__ void wave_sum2(float& a, float& b) {
  a += dppf<0xB1>(a);
  b += dppf<0xB1>(b);
  a += dppf<0x4E>(a);
  b += dppf<0x4E>(b);
  a += dppf<0x141>(a);
  b += dppf<0x141>(b);
  a += dppf<0x140>(a);
  b += dppf<0x140>(b);
  a += dppf<0x142, 0xa>(a);
  b += dppf<0x142, 0xa>(b);
  a += dppf<0x143, 0xc>(a);
  b += dppf<0x143, 0xc>(b);
  a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), 63));
  b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b), 63));
}

// exp(x) to ~1 ulp: 2^(x log2 e) with the rounding error of the f32 product x*log2e
// (and log2e's own f32 residual) restored to first order; __expf drops that error,
// ~|x| * 6e-8 relative, which matters for |x| of a few units.
__device__ __forceinline__ float exp_acc(float x) {
  constexpr float kL2E = 1.44269502162933349609375f;   // f32(log2 e)
  constexpr float kL2E_lo = 1.925963033500011e-08f;    // log2 e - kL2E
  const float y = x * kL2E;
  float err = fmaf(x, kL2E, -y);
  err = fmaf(x, kL2E_lo, err);
  const float r = __builtin_amdgcn_exp2f(y);
  return fmaf(r, err * 0.693147180559945309f, r);
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  v = fmaxf(v, dppf<0x142, 0xa>(v));
  v = fmaxf(v, dppf<0x143, 0xc>(v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// 1/x to ~0.5 ulp: v_rcp_f32 (1 ulp) + one Newton step (2 FMAs) -- the IEEE division
// sequence costs ~10 instructions; the scans take one reciprocal per step
__device__ __forceinline__ float rcp_nr(float x) {
  const float r = __builtin_amdgcn_rcpf(x);
  return fmaf(r, fmaf(-x, r, 1.f), r);
}

// max over each 32-lane half of the wave, result in every lane of the half:
// quad_perm xor1 / xor2, row_half_mirror, row_mirror (16-lane row max), then
// permlane16_swap pairs rows 0<->1 and 2<->3.
__device__ __forceinline__ float half_max32(float v) {
  v = fmaxf(v, dppf<0xB1>(v));
  v = fmaxf(v, dppf<0x4E>(v));
  v = fmaxf(v, dppf<0x141>(v));
  v = fmaxf(v, dppf<0x140>(v));
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Exact 3-way bf16 split of a pair of f32 values, packed two per dword (value a in the
// low half): hi = the top 16 bits, mid / lo = those of the successive remainders (each
// remainder is exact in f32).  3 byte-permutes + 8 ALU ops per pair.
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t& hw, uint32_t& mw, uint32_t& lw) {
  const uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
  hw = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
  const float ra = a - __uint_as_float(ua & 0xFFFF0000u), rb = b - __uint_as_float(ub & 0xFFFF0000u);
  const uint32_t va = __float_as_uint(ra), vb = __float_as_uint(rb);
  mw = __builtin_amdgcn_perm(vb, va, 0x07060302u);
  const float sa = ra - __uint_as_float(va & 0xFFFF0000u), sb = rb - __uint_as_float(vb & 0xFFFF0000u);
  lw = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
}

// the f32 value of the bf16 halves of a dword (low half: element 2i, high half: 2i + 1)
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

// f64 DPP: both 32-bit halves moved by the same DPP control
template <int CTRL, int ROWMASK = 0xf, int BANKMASK = 0xf>
__device__ __forceinline__ double dppd(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWMASK, BANKMASK, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWMASK, BANKMASK, false);
  return __hiloint2double(hi, lo);
}

// f64 wave sum, same DPP stage pattern as wave_sum (no LDS round trips), result in
// every lane (readlane of lane 63)
__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dppd<0xB1>(v);
  v += dppd<0x4E>(v);
  v += dppd<0x141>(v);
  v += dppd<0x140>(v);
  v += dppd<0x142, 0xa>(v);
  v += dppd<0x143, 0xc>(v);
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  return __hiloint2double(hi, lo);
}
// f64 reductions via shuffles (used off the critical path)
__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_min_shfl(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max_shfl(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// jax.nn.softplus == logaddexp(x, 0)
__device__ __forceinline__ double softplus_d(double x) {
  return fmax(x, 0.0) + log1p(exp(-fabs(x)));
}
__device__ __forceinline__ float softplus_f(float x) {
  return fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoid_f(float x) {
  return 1.f / (1.f + __expf(-x));
}

}  // namespace pmg
