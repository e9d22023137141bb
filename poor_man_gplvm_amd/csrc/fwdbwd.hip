// Time-parallel forward filter / backward smoother: host dispatch, boundary
// verification and the C ABI.  The device code is in fb_kernels.h; its template
// instances are compiled per J in fb_inst_j*.hip.
#include "fb_kernels.h"

namespace pmg {

// boundary verification: flags[c] = hilbert(x[c], y[c + off]) > tol; a failing
// boundary also copies y[c + off] into x[c] (the restart state of the relaxation) and
// counts itself in *pending.
// Backward (w != nullptr): both betas are weighted by alpha at the boundary time
// t_e = (c+1) C (w[c+1], the (2, Lpad) w_first slot of chunk c+1), i.e. the POSTERIOR at
// t_e is compared.  An error of beta_{t_e}(j)
// reaches gamma_t(i), t < t_e, only through the joint P(x_t = i, x_{t_e} = j) <=
// gamma_{t_e}(j), so components with negligible posterior cannot move any output
// above ~1e-18 probability, while they are exactly the ones the chain forgets slowly.
// Batched restarts: blockIdx.y = restart, whose operands (all in its workspace slab) sit
// ws_stride bytes further per restart.
__global__ void __launch_bounds__(256) k_verify(float* __restrict__ x, const float* __restrict__ y,
                                                int first, int last, int off, int SZ, float tol,
                                                int* __restrict__ flags, const float* __restrict__ w,
                                                int Lpad, int* __restrict__ pending, int64_t ws_stride) {
  if (blockIdx.y) {
    const uintptr_t o = (uintptr_t)blockIdx.y * (uintptr_t)ws_stride;
    x = reinterpret_cast<float*>(reinterpret_cast<uintptr_t>(x) + o);
    y = reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(y) + o);
    flags = reinterpret_cast<int*>(reinterpret_cast<uintptr_t>(flags) + o);
    if (w) w = reinterpret_cast<const float*>(reinterpret_cast<uintptr_t>(w) + o);
    pending = reinterpret_cast<int*>(reinterpret_cast<uintptr_t>(pending) + o);
  }
  // wave-uniform (readfirstlane): the state pointers below feed scalar buffer descriptors
  const int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int c = first + wv;
  if (c > last) return;
  const float* yc = y + (size_t)(c + off) * SZ;
  float* xc = x + (size_t)c * SZ;
  const float* wc = w ? w + (size_t)(c + 1) * SZ : nullptr;
  const float d = hilbert_dist(xc, yc, SZ, wc);
  const bool bad = !(d <= tol);
  if ((threadIdx.x & 63) == 0) {
    flags[c] = bad ? 1 : 0;
    if (bad) atomicAdd(pending, 1);
  }
  if (bad)
    for (int i = threadIdx.x & 63; i < SZ; i += 64) xc[i] = yc[i];
}

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
struct FBWork {
  int* ctl;       // control words: forward block at 0, backward at kCtlStride
  float* jsc;     // (T, 2) the forward's per-step (jump, 1/S)
  float *s_in, *s_out, *b_in, *b_first, *w_first;
  double* chunk_logz;
  int* flags;
  float* seg_end;  // [2][kRelaxMaxSeg][2*Lpad]
  int* seg_chg;    // [2][kRelaxMaxSeg]
};

// workspace layout (the Python diagnostics mirror it): ctl[64] | jsc[2T] | s_in | s_out |
// b_in | b_first (M x 2 x Lpad f32 each) | chunk_logz[M] | flags[M] | seg_end | seg_chg |
// w_first (M x 2 x Lpad).  ctl and jsc sit before anything sized by the chunk, so the
// forward (chunk C) and the backward (chunk Cb) agree on them.  The workspace must be
// zero-filled before its first use: the kernels then keep the control words zero
// between calls.
static FBWork carve_fb(void* ws, int64_t T, int Lpad, int C, size_t* total = nullptr) {
  const int64_t M = (T + C - 1) / C;
  Carver c(ws);
  FBWork w;
  w.ctl = c.take<int>(64);
  w.jsc = c.take<float>((size_t)2 * T);
  w.s_in = c.take<float>((size_t)M * 2 * Lpad);
  w.s_out = c.take<float>((size_t)M * 2 * Lpad);
  w.b_in = c.take<float>((size_t)M * 2 * Lpad);
  w.b_first = c.take<float>((size_t)M * 2 * Lpad);
  w.chunk_logz = c.take<double>(M);
  w.flags = c.take<int>(M);
  w.seg_end = c.take<float>((size_t)2 * kRelaxMaxSeg * 2 * Lpad);
  w.seg_chg = c.take<int>(2 * kRelaxMaxSeg);
  w.w_first = c.take<float>((size_t)M * 2 * Lpad);
  if (total) *total = c.off + 256;
  return w;
}

// Relaxation segments: at most one single-wave workgroup per CU (so all are resident
// whatever else the device runs: 64 threads, no LDS), G chunks each.
static int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 64;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 64;
    cached[dev] = n;
  }
  return cached[dev];
}

static void relax_shape(FBParams& p) {
  int S = device_cus();
  if (S > kRelaxMaxSeg) S = kRelaxMaxSeg;
  if (S > p.M) S = p.M;
  if (S < 1) S = 1;
  p.G = (p.M + S - 1) / S;
  p.S = (p.M + p.G - 1) / p.G;
}

// PMG_DEBUG_NO_REPAIR (diagnostics): k_verify flags the boundaries into a dummy
// pending word, so the relaxation kernel repairs nothing (it only sums logZ).
static bool debug_no_repair() { return getenv("PMG_DEBUG_NO_REPAIR") != nullptr; }

static int pick_J(int L) {
  if (L <= 64) return 1;
  if (L <= 128) return 2;
  if (L <= 256) return 4;
  if (L <= 512) return 8;
  if (L <= 1024) return 16;
  return -1;
}
// band = ceil(8.31 mv): 5 (mv 0.5), 9 (mv 1, the default), 17 (mv 2), 25 (mv 3) are exact
static int pick_WP(int band) {
  if (band <= 5) return 5;
  if (band <= 9) return 9;
  if (band <= 13) return 13;
  if (band <= 17) return 17;
  if (band <= 25) return 25;
  if (band <= 32) return 32;
  return -1;
}

// kernel sets are instantiated per (J, WP) in fb_inst_j*_w*.hip (parallel builds)
static bool fb_set(int J, int WP, FBKernelSet* k) {
#define PMG_FB_CASE(JJ, WPP)      \
  if (J == JJ && WP == WPP) {     \
    fb_set_j##JJ##_w##WPP(k);     \
    return true;                  \
  }
  PMG_FB_ALL(PMG_FB_CASE)
#undef PMG_FB_CASE
  return false;
}

static int fill_params(FBParams& p, const pmg_transition* tr, int64_t T, int C, int B,
                       double s, double tol) {
  PMG_REQUIRE(tr && tr->L > 0 && tr->invz, "pmg fwd/bwd: bad transition");
  PMG_REQUIRE(tr->band >= 0 && tr->band <= kMaxBand,
              "pmg fwd/bwd: continuous-kernel band %d > %d unsupported (dense kernels: not yet)",
              tr->band, kMaxBand);
  PMG_REQUIRE(T > 0 && C > 0 && B >= 0, "pmg fwd/bwd: T=%lld chunk=%d warmup=%d", (long long)T, C, B);
  const int J = pick_J(tr->L);
  PMG_REQUIRE(J > 0, "pmg fwd/bwd: L=%d > 1024 unsupported", tr->L);
  memset(&p, 0, sizeof(p));
  p.T = T;
  p.L = tr->L;
  p.nblk = (int)(round_up(tr->L, 32) / 32);
  p.invz = tr->invz;
  p.A00 = tr->A[0];
  p.A01 = tr->A[1];
  p.A10 = tr->A[2];
  p.A11 = tr->A[3];
  p.invL = 1.f / (float)tr->L;
  p.s = (float)s;
  p.s_d = s;
  p.C = C;
  p.B = B;
  p.M = (int)((T + C - 1) / C);
  p.tol = (float)tol;
  p.Lpad = 64 * J;
  p.ldd = p.L;
  p.ldphi = p.nblk;
  p.ldm = 1;
  p.ws_stride = 0;
  p.adapt = 0;
  p.spin = spin_ticks(kSpinTicks);
  for (int k = 0; k <= kMaxBand; ++k) p.g[k] = (k <= tr->band) ? tr->g[k] : 0.f;
  return PMG_OK;
}

// R > 1: R restarts' latents stacked side by side in delta / phi / m (and P), each
// restart its own alpha / logc sequence and its own workspace slab of
// (workspace_bytes / R) rounded down to 256 bytes; blockIdx.y selects the restart.
// The relaxation runs <= #CUs / R segments per restart, so all R S waves stay resident.
static int batch_params(FBParams& p, int R, int64_t T, int chunk, size_t workspace_bytes, size_t* slab) {
  PMG_REQUIRE(R >= 1 && R <= 65535, "pmg scans: R=%d restarts", R);
  *slab = R == 1 ? workspace_bytes : (workspace_bytes / (size_t)R) & ~(size_t)255;
  PMG_REQUIRE(*slab >= pmg_fwdbwd_workspace_size(T, p.L, chunk), "pmg scans: workspace too small (%zu per restart)",
              *slab);
  if (R == 1) return PMG_OK;
  PMG_REQUIRE(p.L % 32 == 0, "pmg scans: batched restarts need L %% 32 == 0 (L=%d)", p.L);
  p.ldd = R * p.L;
  p.ldphi = R * p.nblk;
  p.ldm = R;
  p.ws_stride = (int64_t)*slab;
  int S = device_cus() / R;
  if (S < 1) S = 1;
  if (S > p.S) S = p.S;
  p.G = (p.M + S - 1) / S;
  p.S = (p.M + p.G - 1) / p.G;
  return PMG_OK;
}

// PMG_PHASE_SEGMENTS: an explicit relaxation segment count per sequence
static void requested_segments(FBParams& p, int phase, int R) {
  int S = (phase >> 16) & 0xfff;
  if (S <= 0) return;
  if (S > kRelaxMaxSeg) S = kRelaxMaxSeg;
  const int cap = 2 * device_cus() / (R > 1 ? R : 1);   // all R S single-wave groups co-resident
  if (S > cap) S = cap > 0 ? cap : 1;
  if (S > p.M) S = p.M;
  p.G = (p.M + S - 1) / S;
  p.S = (p.M + p.G - 1) / p.G;
}

}  // namespace pmg

using namespace pmg;

extern "C" {

size_t pmg_fwdbwd_workspace_size(int64_t T, int32_t L, int32_t chunk) {
  const int J = pick_J(L);
  if (J < 0 || chunk <= 0 || T <= 0) return 0;
  size_t total = 0;
  carve_fb(nullptr, T, 64 * J, chunk, &total);
  return total;
}

size_t pmg_fwdbwd_repair_counter_offset(int64_t T, int32_t L, int32_t chunk) {
  (void)T; (void)L; (void)chunk;
  return 0;  // int32 control blocks at the workspace start: forward words 0.., backward kCtlStride..
}

int32_t pmg_fwdbwd_lpad(int32_t L) {
  const int J = pick_J(L);
  return J < 0 ? 0 : 64 * J;
}

float* pmg_fwdbwd_state(void* workspace, int64_t T, int32_t L, int32_t chunk, int32_t which, int64_t c) {
  const int J = pick_J(L);
  if (!workspace || J < 0 || chunk <= 0 || T <= 0) return nullptr;
  const int64_t M = (T + chunk - 1) / chunk;
  if (c < 0 || c >= M) return nullptr;
  FBWork w = carve_fb(workspace, T, 64 * J, chunk);
  float* base = nullptr;
  switch (which) {
    case PMG_STATE_FWD_IN: base = w.s_in; break;
    case PMG_STATE_FWD_OUT: base = w.s_out; break;
    case PMG_STATE_BWD_IN: base = w.b_in; break;
    case PMG_STATE_BWD_FIRST: base = w.b_first; break;
    default: return nullptr;
  }
  return base + (size_t)c * 2 * (64 * J);
}

// phase bits: 1 = chunk-parallel main pass, 2 = boundary verification + relaxation
// (+ logZ), 4 = forward: alpha's d = 1 rows not written
static int forward_impl(const float* delta, const float* phi, const double* m, int64_t T,
                        const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                        int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                        void* workspace, size_t workspace_bytes, void* stream, int phase, int R = 1) {
  FBParams p;
  int rc = fill_params(p, tr, T, chunk, warmup, likelihood_scale, tol);
  if (rc) return rc;
  PMG_REQUIRE(delta && phi && m && alpha && logc && logz && workspace, "pmg_forward_filter: null");
  PMG_REQUIRE(workspace_bytes >= pmg_fwdbwd_workspace_size(T, tr->L, chunk),
              "pmg_forward_filter: workspace too small");
  hipStream_t st = as_stream(stream);
  FBWork w = carve_fb(workspace, T, p.Lpad, chunk);
  p.delta = delta;
  p.phi = phi;
  p.m = m;
  p.alpha = alpha;
  p.logc = logc;
  p.logz = logz;
  p.chunk_logz = w.chunk_logz;
  p.jsc = w.jsc;
  p.a1_bytes = (phase & (PMG_PHASE_NO_JUMP_ROWS | PMG_PHASE_NO_ALPHA)) ? 0u : (uint32_t)p.L * 4u;
  p.a0_bytes = (phase & PMG_PHASE_NO_ALPHA) ? 0u : (uint32_t)p.L * 4u;
  p.adapt = (phase & PMG_PHASE_ADAPTIVE_WARMUP) ? 1 : 0;
  p.s_in = w.s_in;
  p.s_out = w.s_out;
  p.flags = w.flags;
  p.ctl = w.ctl;
  p.seg_end = w.seg_end;
  p.seg_chg = w.seg_chg;
  relax_shape(p);
  size_t slab = 0;
  rc = batch_params(p, R, T, chunk, workspace_bytes, &slab);
  if (rc) return rc;
  requested_segments(p, phase, R);
  const int J = p.Lpad / 64, WP = pick_WP(tr->band);
  FBKernelSet ks;
  const bool have = fb_set(J, WP, &ks);
  PMG_REQUIRE(have && ks.forward && ks.forward_relax, "pmg_forward_filter: no kernel for J=%d WP=%d", J, WP);
  if (phase & 1) {
    const bool two = (phase & PMG_PHASE_TWO_WAVES) && ks.forward2;
    hipLaunchKernelGGL(two ? ks.forward2 : ks.forward, dim3(p.M, R), dim3(two ? 128 : 64), 0, st, p);
    PMG_LAUNCH_CHECK();
  }
  if (phase & 2) {
    if (p.M > 1) {
      int* pend = debug_no_repair() ? p.ctl + kCtlStride - 1 : p.ctl + kCtlPending;
      const int nver = p.M - 1;
      hipLaunchKernelGGL(k_verify, dim3((nver + 3) / 4, R), dim3(256), 0, st, w.s_in, (const float*)w.s_out, 1,
                         p.M - 1, -1, 2 * p.Lpad, p.tol, w.flags, (const float*)nullptr, p.Lpad, pend,
                         p.ws_stride);
      PMG_LAUNCH_CHECK();
    }
    PMG_HIP(launch_persistent(ks.forward_relax, dim3(p.S, R), dim3(64), 0, st, p));  // also sums logZ
  }
  return PMG_OK;
}

int pmg_forward_filter(const float* delta, const float* phi, const double* m, int64_t T,
                       const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                       int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                       void* workspace, size_t workspace_bytes, void* stream) {
  return forward_impl(delta, phi, m, T, tr, likelihood_scale, chunk, warmup, tol, alpha, logc, logz,
                      workspace, workspace_bytes, stream, 3);
}

int pmg_forward_filter_phase(const float* delta, const float* phi, const double* m, int64_t T,
                             const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                             int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                             void* workspace, size_t workspace_bytes, void* stream, int32_t phase) {
  PMG_REQUIRE((phase & 3) != 0 && (phase & ~(PMG_PHASE_FLAG_BITS & ~PMG_PHASE_P_BF16X3)) == 0,
              "pmg_forward_filter_phase: phase %d", phase);
  return forward_impl(delta, phi, m, T, tr, likelihood_scale, chunk, warmup, tol, alpha, logc, logz,
                      workspace, workspace_bytes, stream, phase);
}

static int backward_impl(const float* delta, const float* phi, const float* alpha, int64_t T,
                         const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                         int32_t warmup, double tol, float* P, float* gamma, float* rho,
                         void* workspace, size_t workspace_bytes, void* stream, int phase, int R = 1) {
  FBParams p;
  int rc = fill_params(p, tr, T, chunk, warmup, likelihood_scale, tol);
  if (rc) return rc;
  PMG_REQUIRE(delta && phi && alpha && workspace, "pmg_backward_smoother: null");
  PMG_REQUIRE(workspace_bytes >= pmg_fwdbwd_workspace_size(T, tr->L, chunk),
              "pmg_backward_smoother: workspace too small");
  PMG_REQUIRE(R == 1 || (P && !rho), "pmg_backward_smoother: batched restarts write P (and gamma), not rho");
  hipStream_t st = as_stream(stream);
  FBWork w = carve_fb(workspace, T, p.Lpad, chunk);
  p.delta = delta;
  p.phi = phi;
  p.alpha_in = alpha;
  p.jsc = w.jsc;
  p.w_first = w.w_first;
  if (phase & PMG_PHASE_P_BF16X3) {   // P is the bf16 planes [3][T][ldd]
    p.Pq = reinterpret_cast<uint16_t*>(P);
    p.P = nullptr;
  } else {
    p.P = P;
  }
  p.gamma = gamma;
  p.rho = rho;
  p.adapt = (phase & PMG_PHASE_ADAPTIVE_WARMUP) ? 1 : 0;
  p.b_in = w.b_in;
  p.b_first = w.b_first;
  p.flags = w.flags;
  p.ctl = w.ctl + kCtlStride;
  p.seg_end = w.seg_end;
  p.seg_chg = w.seg_chg;
  relax_shape(p);
  size_t slab = 0;
  rc = batch_params(p, R, T, chunk, workspace_bytes, &slab);
  if (rc) return rc;
  requested_segments(p, phase, R);
  p.pq_stride = T * (int64_t)p.ldd;
  const int J = p.Lpad / 64, WP = pick_WP(tr->band);
  FBKernelSet ks;
  const bool have = fb_set(J, WP, &ks);
  fb_kernel_t kb = !have ? nullptr : (rho || gamma || !P) ? ks.backward_full : ks.backward;
  PMG_REQUIRE(kb && ks.backward_relax, "pmg_backward_smoother: no kernel for J=%d WP=%d", J, WP);
  if (phase & 1) {
    const bool two = (phase & PMG_PHASE_TWO_WAVES) && kb == ks.backward && ks.backward2;   // EM (P-only) passes
    hipLaunchKernelGGL(two ? ks.backward2 : kb, dim3(p.M, R), dim3(two ? 128 : 64), 0, st, p);
    PMG_LAUNCH_CHECK();
  }
  if ((phase & 2) && p.M > 1) {
    int* pend = debug_no_repair() ? p.ctl + kCtlStride - 1 : p.ctl + kCtlPending;
    const int nver = p.M - 1;
    hipLaunchKernelGGL(k_verify, dim3((nver + 3) / 4, R), dim3(256), 0, st, w.b_in, (const float*)w.b_first, 0,
                       p.M - 2, 1, 2 * p.Lpad, p.tol, w.flags, (const float*)w.w_first, p.Lpad, pend, p.ws_stride);
    PMG_LAUNCH_CHECK();
    PMG_HIP(launch_persistent(ks.backward_relax, dim3(p.S, R), dim3(64), 0, st, p));
  }
  return PMG_OK;
}

int pmg_backward_smoother(const float* delta, const float* phi, const float* alpha, int64_t T,
                          const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                          int32_t warmup, double tol, float* P, float* gamma, float* rho,
                          void* workspace, size_t workspace_bytes, void* stream) {
  return backward_impl(delta, phi, alpha, T, tr, likelihood_scale, chunk, warmup, tol, P, gamma, rho,
                       workspace, workspace_bytes, stream, 3);
}

int pmg_backward_smoother_phase(const float* delta, const float* phi, const float* alpha, int64_t T,
                                const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                                int32_t warmup, double tol, float* P, float* gamma, float* rho,
                                void* workspace, size_t workspace_bytes, void* stream, int32_t phase) {
  PMG_REQUIRE((phase & 3) != 0 && (phase & ~(PMG_PHASE_FLAG_BITS & ~(PMG_PHASE_NO_JUMP_ROWS | PMG_PHASE_NO_ALPHA))) == 0,
              "pmg_backward_smoother_phase: phase %d", phase);
  return backward_impl(delta, phi, alpha, T, tr, likelihood_scale, chunk, warmup, tol, P, gamma, rho,
                       workspace, workspace_bytes, stream, phase);
}

size_t pmg_fwdbwd_batched_workspace_size(int64_t T, int32_t L, int32_t chunk, int32_t R) {
  const size_t one = pmg_fwdbwd_workspace_size(T, L, chunk);
  if (one == 0 || R < 1) return 0;
  return R == 1 ? one : (size_t)R * ((one + 255) & ~(size_t)255);
}

int pmg_forward_filter_batched(const float* delta, const float* phi, const double* m, int64_t T, int32_t R,
                               const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                               int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                               void* workspace, size_t workspace_bytes, void* stream, int32_t phase) {
  PMG_REQUIRE((phase & 3) != 0 && (phase & ~(PMG_PHASE_FLAG_BITS & ~PMG_PHASE_P_BF16X3)) == 0,
              "pmg_forward_filter_batched: phase %d", phase);
  return forward_impl(delta, phi, m, T, tr, likelihood_scale, chunk, warmup, tol, alpha, logc, logz,
                      workspace, workspace_bytes, stream, phase, R);
}

int pmg_backward_smoother_batched(const float* delta, const float* phi, const float* alpha, int64_t T, int32_t R,
                                  const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                                  int32_t warmup, double tol, float* P, float* gamma, void* workspace,
                                  size_t workspace_bytes, void* stream, int32_t phase) {
  PMG_REQUIRE((phase & 3) != 0 && (phase & ~(PMG_PHASE_FLAG_BITS & ~(PMG_PHASE_NO_JUMP_ROWS | PMG_PHASE_NO_ALPHA))) == 0,
              "pmg_backward_smoother_batched: phase %d", phase);
  return backward_impl(delta, phi, alpha, T, tr, likelihood_scale, chunk, warmup, tol, P, gamma, nullptr,
                       workspace, workspace_bytes, stream, phase, R);
}

}  // extern "C"
