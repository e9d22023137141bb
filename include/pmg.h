/*
 * pmg.h -- C ABI of libpmg_hip.so, the MI355X (gfx950) engine behind the
 * PoissonGPLVMJump1D EM hot path of poor-man-GPLVM.
 *
 * Conventions
 *   - every array argument is a DEVICE pointer allocated and owned by the
 *     caller (PyTorch in the Python host layer), row-major, no padding unless
 *     the parameter list says so;
 *   - `stream` is a hipStream_t passed as void* (0 = null stream); all work of
 *     one call is enqueued on that stream in order and nothing synchronises
 *     the host unless stated;
 *   - every entry point returns 0 (PMG_OK) or a negative PMG_E* code; the
 *     message of the last error on the calling thread is pmg_last_error();
 *   - no global device state: scratch space is a caller workspace whose size
 *     comes from the matching *_workspace_size query.
 *
 * Each entry point names the reference function it replaces
 * (/root/reference/poor_man_gplvm/..., file:line).
 *
 * Shapes: T time bins, N neurons, L latent bins, D = 2 dynamics
 * (0 continuous, 1 jump), NB basis columns (incl. bias).
 */
#ifndef PMG_H
#define PMG_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PMG_ABI_VERSION 2

#define PMG_OK 0
#define PMG_EINVAL (-1)       /* bad shape / argument */
#define PMG_EHIP (-2)         /* HIP runtime error */
#define PMG_EUNSUPPORTED (-3) /* configuration outside what the kernels implement */
#define PMG_ETIMEOUT (-4)     /* a bounded in-kernel spin gave up */

/* spike-preparation flags (written to *flags_out on the device) */
#define PMG_YFLAG_NONINT 1    /* some y is non-integer, negative or > 127: use the f64 emission */
#define PMG_YFLAG_MASK 2      /* ma_neuron is not 0/1 */

int pmg_abi_version(void);
const char* pmg_last_error(void);

/* ------------------------------------------------------------------ */
/* Spike preparation (once per fit).  Feeds the emission and the       */
/* sufficient statistics.  Replaces the per-call y handling of          */
/* decoder.get_loglikelihood_ma_all (decoder.py:60-71) and the y of     */
/* fit_tuning_helper.get_statistics (fit_tuning_helper.py:28-42).       */
/*   y        (T,N) f32 spike counts                                     */
/*   ma_neuron (N) f32 or (T,N) f32 (ma_is_2d) or NULL (all ones)        */
/*   yq_out   (Tp,Kp) int8, Tp = roundup(T,64), Kp = roundup(N,128):      */
/*            y*ma (zero padded), the integer emission operand           */
/*   gconst_out (T) f64: sum_n ma[t,n]*gammaln(y[t,n]+1)                 */
/*   yext_out (T,Np) f32, Np = roundup(N+1,64): y, then a ones column    */
/*            (t_w = sum_t P falls out of the same GEMM), zero padded    */
/*   flags_out (1) int32 device word, OR of PMG_YFLAG_*; zeroed here     */
int pmg_spikes_prepare(const float* y, int64_t T, int32_t N, const float* ma_neuron,
                       int32_t ma_is_2d, int8_t* yq_out, int32_t Kp, double* gconst_out,
                       float* yext_out, int32_t Np, int32_t* flags_out, void* stream);

/* ------------------------------------------------------------------ */
/* tuning = softplus(basis @ W)   -- fit_tuning_helper.py:19-25,        */
/* core.py:772-774.  basis (L,NB) f32, W (NB,N) f64;                     */
/* tuning64 (L,N) f64 and tuning32 (L,N) f32 (either may be NULL).       */
int pmg_tuning_softplus(const float* basis, const double* W, int32_t L, int32_t NB, int32_t N,
                        double* tuning64, float* tuning32, void* stream);
/* R restarts at once: W (R,NB,N) f64 -> tuning rows r*L + l of the stacked */
/* (R*L, N) outputs (the latents of the batched emission).       */
int pmg_tuning_softplus_batched(const float* basis, const double* W, int32_t L, int32_t NB, int32_t N, int32_t R,
                                double* tuning64, float* tuning32, void* stream);

/* ------------------------------------------------------------------ */
/* Poisson emission  -- decoder.get_loglikelihood_ma_poisson            */
/* (decoder.py:30-48) vmapped by get_loglikelihood_ma_all (:60-71):      */
/*   ll[t,l] = sum_n m[t,n]*(xlogy(y,lam) - lam - gammaln(y+1)),         */
/*   lam = tuning*dt + 1e-20, ll = -1e20 where ma_latent == 0.           */
/* Output is split for an fp32 consumer without losing precision:       */
/*   delta (T,L) f32 = ll - r[t, l/32],  rblk (T, Lp/32) f64 = max over   */
/*   the 32-latent block (Lp = roundup(L,32)).                           */
/* Integer path (flags == 0, 1-D or no mask): exact int8 MFMA            */
/* (v_mfma_i32_32x32x32_i8) on y and log(lam) in 5 balanced base-256     */
/* digits of a 2^-32 fixed point (5 digits).  Generic path: f64.         */
/* The workspace must be zero-filled before its first use: it holds a    */
/* sticky int32 range flag (pmg_emission_range_flag) that the integer    */
/* path ORs to 1 when some |log lam| >= 60 (outside the digit range);    */
/* the caller reads and clears it (no per-call memset).                  */
size_t pmg_emission_workspace_size(int64_t T, int32_t L, int32_t N);
int32_t* pmg_emission_range_flag(void* workspace, int64_t T, int32_t L, int32_t N);
/* ll64 (T,L) f64 (may be NULL): the unsplit ll as well, for consumers   */
/* that need it exact far below the block maximum (the exact decode's    */
/* dense scans: delta's f32 rounding is 3e-5 absolute at |delta| ~ 500). */
int pmg_emission_poisson(const int8_t* yq, const double* gconst, const double* tuning64,
                         const float* ma_neuron_1d, const uint8_t* ma_latent, double dt,
                         int64_t T, int32_t L, int32_t N, int32_t Kp, float* delta,
                         double* rblk, double* ll64, void* workspace, size_t workspace_bytes, void* stream);
/* Generic f64 emission (non-integer y, weighted or 2-D masks). y (T,N) f32. */
int pmg_emission_poisson_f64(const float* y, const double* gconst, const double* tuning64,
                             const float* ma_neuron, int32_t ma_is_2d, const uint8_t* ma_latent,
                             double dt, int64_t T, int32_t L, int32_t N, float* delta,
                             double* rblk, double* ll64, void* workspace, size_t workspace_bytes, void* stream);
/* Latent mask on an unmasked emission (any of the emissions above, run with ma_latent =   */
/* NULL): (delta, rblk) = the (delta0, rblk0) those kernels would produce with ma_latent   */
/* (ll[:, ma_latent == 0] = -1e20, decoder.py:46; block references over kept bins).  Used  */
/* by log_marginal_masked so that get_downsampled_lml's masks (model_selection_helper.py: */
/* 243-260) share one emission contraction.  Out of place.                                */
int pmg_emission_latent_mask(const float* delta0, const double* rblk0, int64_t T, int32_t L,
                             const uint8_t* ma_latent, float* delta, double* rblk, void* stream);
/* R masks at once (ma_latent (R, L) uint8, one row per mask), written side by side */
/* as R stacked latent sets: delta (T, R*L), rblk (T, R*nblk), nblk = ceil(L/32):   */
/* the layout of the batched scans (pmg_emission_rowref_batched, then              */
/* pmg_forward_filter_batched).  Mask r's columns equal pmg_emission_latent_mask's  */
/* output for ma_latent[r] bit for bit.  L % 32 == 0.                              */
int pmg_emission_latent_mask_batched(const float* delta0, const double* rblk0, int64_t T, int32_t L,
                                     const uint8_t* ma_latent, int32_t R, float* delta, double* rblk,
                                     void* stream);
/* Per-time reference: m[t] = max_b rblk[t,b], phi[t,b] = f32(s*(rblk[t,b]-m[t])) so that  */
/* exp(s*ll[t,l] - s*m[t]) = exp(s*delta[t,l] + phi[t,l/32]).                              */
int pmg_emission_rowref(const double* rblk, int64_t T, int32_t nblk, double likelihood_scale,
                        float* phi, double* m, void* stream);
/* Batched restarts (R restarts per GPU): rblk holds R restarts'  */
/* stacked latents, nblk = R * nblk_r; m (T, R) and phi (T, nblk) are taken  */
/* per restart (each restart's row reference is its own block maximum).      */
int pmg_emission_rowref_batched(const double* rblk, int64_t T, int32_t nblk, int32_t R, double likelihood_scale,
                                float* phi, double* m, void* stream);
/* ll (T,L) f32 = delta + rblk  (the log_likelihood_all output, decoder.py:307). */
int pmg_loglik_materialize(const float* delta, const double* rblk, int64_t T, int32_t L,
                           float* ll, void* stream);

/* Naive-Bayes decoding (no temporal prior) -- decoder.get_naive_bayes_ma_chunk   */
/* (decoder.py:106-149) / get_naive_bayes_ma (:88-102).                           */
/* Per-time dt emission, get_loglikelihood_ma_all_changing_dt (decoder.py:73-85):  */
/* lam = tuning*dt_t[t] + 1e-20, one log per (t, l, n) as in the reference, f64;   */
/* outputs split as pmg_emission_poisson (delta, rblk).  dt_t (T) f64.            */
int pmg_emission_poisson_dt(const float* y, const double* gconst, const double* tuning64,
                            const float* ma_neuron, int32_t ma_is_2d, const uint8_t* ma_latent,
                            const double* dt_t, int64_t T, int32_t L, int32_t N, float* delta,
                            double* rblk, void* stream);
/* Row normalisation of decoder.py:97-100: log_marginal_l[t] = logsumexp_l ll[t,l]  */
/* (f64), log_post (T,L) f32 = ll - log_marginal_l[t]; ll given as (delta, rblk).    */
int pmg_naive_bayes_normalize(const float* delta, const double* rblk, int64_t T, int32_t L,
                              float* log_post, double* log_marginal_l, void* stream);

/* ------------------------------------------------------------------ */
/* Gaussian observation model -- GaussianGPLVMJump1D (core.py:852-917).  */
/* tuning = basis @ W  (fit_tuning_helper.get_tuning_linear, :12-17).     */
int pmg_tuning_linear(const float* basis, const double* W, int32_t L, int32_t NB, int32_t N,
                      double* tuning64, float* tuning32, void* stream);
/* ll[t,l] = sum_n m[t,n] norm.logpdf(y[t,n], tuning[l,n]*dt, noise_std), -1e20   */
/* where ma_latent == 0 (decoder.get_loglikelihood_ma_gaussian, decoder.py:50-57). */
/* f64 accumulation; output split as pmg_emission_poisson (delta, rblk).           */
int pmg_emission_gaussian(const float* y, const double* tuning64, const float* ma_neuron, int32_t ma_is_2d,
                          const uint8_t* ma_latent, double noise_std, double dt, int64_t T, int32_t L,
                          int32_t N, float* delta, double* rblk, double* ll64, void* stream);
/* Per-time-bin dt (decoder.get_loglikelihood_ma_all_changing_dt with the Gaussian
 * observation model, decoder.py:73-85 -> :50-57): mu = tuning * dt_t[t]; dt_t (T) f64. */
int pmg_emission_gaussian_dt(const float* y, const double* tuning64, const float* ma_neuron, int32_t ma_is_2d,
                             const uint8_t* ma_latent, double noise_std, const double* dt_t, int64_t T, int32_t L,
                             int32_t N, float* delta, double* rblk, void* stream);
/* Analytic M-step, fit_tuning_helper.gaussian_m_step_analytic (:44-61):          */
/* W (NB,N) f64 = solve(B^T diag(t_w) B / s^2 + I / p^2, B^T y_w / s^2), Cholesky */
/* in f64 (H is SPD).  status (device int32) is sticky: set to 1 when a pivot was  */
/* not positive (W is then NaN), never cleared -- the caller zeroes it, e.g. once   */
/* per fit, and checks it after the last M-step.                                   */
size_t pmg_gaussian_mstep_workspace_size(int32_t NB, int32_t N);
int pmg_gaussian_mstep(const float* basis, const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                       double noise_std, double prior_std, double* W, int32_t* status, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ */
/* Transition description (gp_kernel.create_transition_prob_1d,         */
/* gp_kernel.py:42-89): continuous kernel K0[i,j] = g[|i-j|]*invz[i]     */
/* (row-normalised RBF, exactly zero beyond |i-j| > band in the f32       */
/* arithmetic the reference uses; band <= 32 here), jump kernel 1/L,     */
/* dynamics A[prev,next].                                                */
#define PMG_MAX_BAND 32
typedef struct pmg_transition {
  int32_t L;
  int32_t band;                 /* half-width W of the continuous kernel, <= PMG_MAX_BAND */
  float g[PMG_MAX_BAND + 1];    /* host values: g[k] = exp(-k^2/mv^2), k <= band */
  const float* invz;            /* (L) DEVICE f32: 1 / sum_j exp(-(i-j)^2/mv^2) */
  float A[4];                   /* host values A00 A01 A10 A11 */
} pmg_transition;

/* Chunked, time-parallel forward filter  -- decoder.filter_one_step    */
/* (decoder.py:151-172) scanned by filter_all_step (:174-187) over the   */
/* chunk loop of smooth_all_step_combined_ma_chunk (:283-304).           */
/*   chunk C steps per wave, warm-up B steps from a uniform guess, then   */
/*   boundary verification (Hilbert metric <= tol) and exact sequential  */
/*   repair of any chunk whose start state disagreed.                    */
/* outputs: alpha (T,2,L) f32 normalised filter posteriors;              */
/*          logc (T) f64 one-step predictive marginals (decoder.py:167); */
/*          logz (1) f64 = sum_t logc (decoder.py:169).                  */
/* The workspace must be ZERO-FILLED before its first use (one hipMemset);   */
/* the kernels keep its control words and counters zero between calls, so    */
/* the scans issue no memsets of their own.  One exception is STICKY: the    */
/* int32 timeout word at pmg_fwdbwd_repair_counter_offset + 4*2 (forward) /  */
/* + 4*(16+2) (backward) is set when a relaxation's bounded grid barrier     */
/* gave up (the call's outputs are then invalid) and stays set across later  */
/* calls (their relaxations fail fast) until the caller reads and clears it. */
/* PMG_DEBUG_SPIN_TICKS (env) overrides the 2 s spin bound (tests).          */
size_t pmg_fwdbwd_workspace_size(int64_t T, int32_t L, int32_t chunk);
int pmg_forward_filter(const float* delta, const float* phi, const double* m, int64_t T,
                       const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                       int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                       void* workspace, size_t workspace_bytes, void* stream);
/* Chunked, time-parallel backward smoother -- decoder.smooth_one_step   */
/* (decoder.py:200-226) / smooth_all_step (:230-256) / chunk loop        */
/* (:313-326), in the equivalent alpha-beta form                          */
/*   gamma_t = alpha_t * beta_t / sum,  beta_{T-1} = 1,                   */
/*   beta_t = Trans (e_{t+1} * beta_{t+1}).                               */
/* The call must run on the workspace of the forward call that produced   */
/* alpha: it reads only alpha's d = 0 rows and rebuilds the d = 1 rows     */
/* (jump * e_t / S_t, bit-exact) from per-step scalars that forward left   */
/* in the workspace.                                                       */
/* outputs (either may be NULL): P (T,L) f32 = sum_d gamma (the dynamics  */
/* marginal of core.py:668, exponentiated); gamma (T,2,L) f32.            */
/* rho (T,2,L) f32 (NULL = skip): rho_t = e_t*beta_t/N_{t-1} with         */
/* N_{t-1} = sum prior_t e_t beta_t, so that the pairwise joint is        */
/* sum_t alpha_t (x) (Trans .* rho_{t+1}) (decoder.py:215-221).           */
int pmg_backward_smoother(const float* delta, const float* phi, const float* alpha, int64_t T,
                          const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                          int32_t warmup, double tol, float* P, float* gamma, float* rho,
                          void* workspace, size_t workspace_bytes, void* stream);
/* The same two calls split in phases (1 = the chunk-parallel main pass,   */
/* 2 = boundary verification, repair rounds and, forward, the logZ sum;    */
/* 3 = both = the calls above).  Lets a caller time the main kernel alone. */
/* Forward only: OR PMG_PHASE_NO_JUMP_ROWS into phase to leave alpha's    */
/* d = 1 rows unwritten (their values are jump_t * e_t / S_t; the backward */
/* rebuilds them), for callers that read only P / logZ (an EM iteration). */
#define PMG_PHASE_NO_JUMP_ROWS 4
/* Forward only: OR PMG_PHASE_NO_ALPHA into both phase calls to write no alpha at */
/* all (logc / logZ only; no backward may follow on this workspace).  For the    */
/* log-marginal-only passes of model_selection_helper.get_downsampled_lml        */
/* (model_selection_helper.py:243-260, which reads log_marginal_final only).     */
#define PMG_PHASE_NO_ALPHA 16
/* Either direction: OR PMG_PHASE_ADAPTIVE_WARMUP into the phase-1 and the  */
/* phase-2 call of each E-step to let the device pick the warm-up: when    */
/* more than 1/8 of a pass's chunk boundaries failed verification (a slowly */
/* mixing chain), the next main pass of that direction on this workspace   */
/* warms up 256 steps instead of `warmup` (decided by the relaxation kernel, */
/* no host sync).  Phase-2 calls without it leave the decision unchanged.   */
#define PMG_PHASE_ADAPTIVE_WARMUP 8
/* Either direction, phase-2 calls: PMG_PHASE_SEGMENTS(S) (1 <= S <= 4095) sets  */
/* the relaxation's segment count per sequence (default 0: #CUs, or #CUs / R for */
/* R batched restarts).  The relaxation's repaired states depend on where its    */
/* segments end (each segment stops recomputing once a state settles within tol) */
/* so two calls agree bit for bit only on the same segment grid: a single fit    */
/* run with S = #CUs / R reproduces restart r of an R-restart batch.             */
#define PMG_PHASE_SEGMENTS(S) ((int32_t)((S) & 0xfff) << 16)
/* Backward only: OR PMG_PHASE_P_BF16X3 into both phase calls to write P as three */
/* bf16 planes instead of f32: P then points at uint16 [3][T][ldd] (ldd = L, or  */
/* R*L batched), plane k at P + k*T*ldd: hi = the top 16 bits of the f32 P value, */
/* mid / lo those of the successive remainders, so P = (hi + mid) + lo exactly in  */
/* f32.  They are the exact-product operands of pmg_suffstats_bf16x3 (the split  */
/* runs once per value here instead of once per neuron tile in the statistics).  */
#define PMG_PHASE_P_BF16X3 32
/* Either direction, phase-1 calls: PMG_PHASE_TWO_WAVES runs each chain of the main  */
/* pass on two waves (half the latents per lane, the band halo and the per-step sums */
/* exchanged through LDS) where that form is compiled (Lpad 512 / 1024, i.e. L in    */
/* (256, 1024]); elsewhere it is ignored.  Same outputs up to f32 summation order.   */
#define PMG_PHASE_TWO_WAVES 64
#define PMG_PHASE_FLAG_BITS \
  (7 | PMG_PHASE_ADAPTIVE_WARMUP | PMG_PHASE_NO_ALPHA | PMG_PHASE_P_BF16X3 | PMG_PHASE_TWO_WAVES | (0xfff << 16))
int pmg_forward_filter_phase(const float* delta, const float* phi, const double* m, int64_t T,
                             const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                             int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                             void* workspace, size_t workspace_bytes, void* stream, int32_t phase);
int pmg_backward_smoother_phase(const float* delta, const float* phi, const float* alpha, int64_t T,
                                const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                                int32_t warmup, double tol, float* P, float* gamma, float* rho,
                                void* workspace, size_t workspace_bytes, void* stream, int32_t phase);
/* number of chunks repaired by the last forward / backward call on this  */
/* workspace (device int32 pair at a fixed offset; host reads it lazily). */
size_t pmg_fwdbwd_repair_counter_offset(int64_t T, int32_t L, int32_t chunk);

/* Chunk-boundary states of the two scans inside a pmg_fwdbwd workspace, so that a  */
/* caller can stitch scans that run on different devices (time shards: the carries */
/* of the chunk loop, decoder.py:283-304 forward / :313-326 backward, handed from  */
/* one shard to the next).  Each state is 2 x Lpad f32 (d = 0 row at [0, L), d = 1  */
/* row at [Lpad, Lpad + L), Lpad = pmg_fwdbwd_lpad(L)), unnormalised (the scans and */
/* the boundary check are scale-free).  For chunk c of a workspace sized for         */
/* (T, L, chunk):                                                                   */
/*   FWD_IN    restart state of chunk c (filter state at c*chunk - 1)               */
/*   FWD_OUT   filter state at the last step of chunk c                              */
/*   BWD_IN    restart beta at the first step after chunk c                          */
/*   BWD_FIRST beta at the first step of chunk c                                     */
/* Writing FWD_OUT[c-1] (BWD_FIRST[c+1]) and re-running phase 2 of the forward        */
/* (backward) call re-verifies chunk c against the new carry and repairs it and its */
/* successors exactly as for an interior boundary.  Returns NULL on a bad argument. */
#define PMG_STATE_FWD_IN 0
#define PMG_STATE_FWD_OUT 1
#define PMG_STATE_BWD_IN 2
#define PMG_STATE_BWD_FIRST 3
int32_t pmg_fwdbwd_lpad(int32_t L);
float* pmg_fwdbwd_state(void* workspace, int64_t T, int32_t L, int32_t chunk, int32_t which, int64_t c);

/* Batched restarts (R independent fits of one recording on one GPU,          */
/* model_selection_helper.py:53-59; SURVEY 8(e): 8 restarts per GPU at C5).    */
/* The R restarts' latents are stacked side by side: delta (T, R*L),          */
/* phi (T, R*nblk_r), m (T, R) (pmg_emission_poisson over the (R*L, N) tuning, */
/* then pmg_emission_rowref_batched), P (T, R*L) (so pmg_suffstats_bf16 over   */
/* R*L latents gives every restart's y_w / t_w in one GEMM).  Each restart has */
/* its own sequence outputs alpha (R,T,2,L), logc (R,T), logz (R) and its own  */
/* workspace slab (workspace_bytes / R, 256-byte aligned; size it with         */
/* pmg_fwdbwd_batched_workspace_size at the smaller of the two chunks, zero-   */
/* filled once).  One launch per pass covers every restart (blockIdx.y); the   */
/* phases are those of the _phase calls; the backward writes P and, if         */
/* non-NULL, gamma (R,T,2,L).  Requires L % 32 == 0.                           */
size_t pmg_fwdbwd_batched_workspace_size(int64_t T, int32_t L, int32_t chunk, int32_t R);
int pmg_forward_filter_batched(const float* delta, const float* phi, const double* m, int64_t T, int32_t R,
                               const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                               int32_t warmup, double tol, float* alpha, double* logc, double* logz,
                               void* workspace, size_t workspace_bytes, void* stream, int32_t phase);
int pmg_backward_smoother_batched(const float* delta, const float* phi, const float* alpha, int64_t T, int32_t R,
                                  const pmg_transition* tr, double likelihood_scale, int32_t chunk,
                                  int32_t warmup, double tol, float* P, float* gamma, void* workspace,
                                  size_t workspace_bytes, void* stream, int32_t phase);

/* ------------------------------------------------------------------ */
/* Dense log-domain scans: any continuous kernel (custom_transition_kernel,  */
/* gp_kernel.py:30-34 and 61-66; RBF kernels wider than PMG_MAX_BAND; the     */
/* latent-only model of decoder_latentonly.py:33-224 with A = [[1,0],[1,0]]). */
/* The reference's own log-space recursion (decoder.py:151-226):               */
/*   prior[0,j] = LSE_i(LSE_d(post[d,i] + logA[d,0]) + logK0[i,j]),            */
/*   prior[1,j] = LSE_i(LSE_d(post[d,i] + logA[d,1])) - log L,                  */
/* with the chunk parallelism, boundary verification (Hilbert metric in log    */
/* space) and relaxation of the banded scans.  Emission input as              */
/* pmg_forward_filter (delta, phi, m).                                         */
typedef struct pmg_dense_transition {
  int32_t L;
  const float* logK;    /* (L, L) DEVICE f32 log continuous kernel [i_prev][j_next] */
  const float* logKT;   /* (L, L) DEVICE f32 its transpose [j_next][i_prev]          */
  const float* logK_lo; /* (L, L) DEVICE f32 residual logK0 - logK (0 where -inf):   */
  const float* logKT_lo;/*   hi + lo keeps far weights (-2500) to ~1e-10; transpose  */
  float logA[4];        /* host values logA00 logA01 logA10 logA11 (-inf allowed)    */
} pmg_dense_transition;
size_t pmg_dense_workspace_size(int64_t T, int32_t L, int32_t chunk);
/* outputs: log_alpha (T,2,L) F64 log filter posteriors (required: the backward */
/* pass reads it; f64 because entries far below the row maximum, e.g. -1000,    */
/* would carry 6e-5 absolute rounding in f32 and the joint of rarely visited     */
/* states is a ratio of such terms); alpha (T,2,L) f32 = exp(log_alpha) (may be */
/* NULL); logc, logz as pmg_forward_filter.                                     */
/* ll64 (T,L) f64 or NULL: the emission's unsplit ll (pmg_emission_poisson's ll64)  */
/* instead of (delta, phi) -- exact far below the block maxima (exact decodes).       */
int pmg_dense_forward(const float* delta, const float* phi, const double* ll64, const double* m, int64_t T,
                      const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                      double tol, float* alpha, double* log_alpha, double* logc, double* logz, void* workspace,
                      size_t workspace_bytes, void* stream);
/* outputs (each may be NULL): P (T,L), gamma (T,2,L), log_gamma (T,2,L) (exact   */
/* log posteriors, the reference's log_acausal_posterior_all), rho (T,2,L) as      */
/* pmg_backward_smoother, log_rho (T,2,L) F64 = log(rho) (no overflow).            */
int pmg_dense_backward(const float* delta, const float* phi, const double* ll64, const double* log_alpha, int64_t T,
                       const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                       double tol, float* P, float* gamma, float* log_gamma, float* rho, double* log_rho,
                       void* workspace, size_t workspace_bytes, void* stream);
/* Phase-split forms (time shards of one recording): phase 1 = the      */
/* chunk-parallel main pass (it also zeroes the repair / round counters), 2 = boundary */
/* verification + relaxation (+ logZ); a phase-2 call after a boundary slot was        */
/* overwritten (pmg_dense_state: the neighbour shard's carry) re-verifies and repairs   */
/* from there, adding its repairs to the counters.  pmg_dense_state returns the f64     */
/* log state slot (2 x pmg_dense_lpad(L) values, [d][j]) of chunk c, `which` as        */
/* pmg_fwdbwd_state; null on bad arguments.                                             */
int32_t pmg_dense_lpad(int32_t L);
double* pmg_dense_state(void* workspace, int64_t T, int32_t L, int32_t chunk, int32_t which, int64_t c);
int pmg_dense_forward_phase(const float* delta, const float* phi, const double* ll64, const double* m, int64_t T,
                            const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk, int32_t warmup,
                            double tol, float* alpha, double* log_alpha, double* logc, double* logz, void* workspace,
                            size_t workspace_bytes, void* stream, int32_t phase);
int pmg_dense_backward_phase(const float* delta, const float* phi, const double* ll64, const double* log_alpha,
                             int64_t T, const pmg_dense_transition* tr, double likelihood_scale, int32_t chunk,
                             int32_t warmup, double tol, float* P, float* gamma, float* log_gamma, float* rho,
                             double* log_rho, void* workspace, size_t workspace_bytes, void* stream, int32_t phase);
/* Pairwise joint in log space (decode, dense scans): logS (2L x 2L) f64 =           */
/* LSE_{t<T-1} log_alpha_t[x] + log_rho_{t+1}[x'], x = (d,i) (f64 inputs, f64 online  */
/* sum); the caller forms the log joint logA[d,d'] + logK[d',i,j] + logS               */
/* (decoder.py:215-221).  Every entry is finite wherever the reference's is.           */
int pmg_joint_log_accumulate(const double* log_alpha, const double* log_rho, int64_t T, int32_t L, double* logS,
                             void* stream);
/* The same with a caller-owned workspace of pmg_joint_log_workspace_size bytes, which  */
/* lets the time axis split over more workgroups (their (max, sum) partials are folded  */
/* in split order).  The size is 0 when the 64 x 64 output tiles alone fill the chip   */
/* (e.g. L >= 1024): the joint then runs unsplit and needs no workspace (pass NULL).  Per block of 64 steps the logs are shifted by their row / column  */
/* maxima and exponentiated once per (row, step), the block sum is an f64 contraction, */
/* and an entry whose block sum leaves f64's range is summed term by term in log space. */
size_t pmg_joint_log_workspace_size(int64_t T, int32_t L);
int pmg_joint_log_accumulate_ws(const double* log_alpha, const double* log_rho, int64_t T, int32_t L, double* logS,
                                void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ */
/* Sufficient statistics -- fit_tuning_helper.get_statistics             */
/* (fit_tuning_helper.py:28-42): y_w = P^T y (L,N), t_w = sum_t P (L).    */
/* P (T,L) f32 probabilities; yext from pmg_spikes_prepare.  fp32 MFMA    */
/* (v_mfma_f32_32x32x2f32) over K-slices, slices summed in f64.           */
size_t pmg_suffstats_workspace_size(int64_t T, int32_t L, int32_t Np);
int pmg_suffstats(const float* P, const float* yext, int64_t T, int32_t L, int32_t N, int32_t Np,
                  double* yw, double* tw, void* workspace, size_t workspace_bytes, void* stream);
/* Same statistics on bf16 MFMA with exact products, for integer spikes   */
/* 0..127 (pmg_spikes_prepare flags without PMG_YFLAG_NONINT): P is split */
/* exactly as hi+mid+lo bf16 (3 x v_mfma_f32_32x32x16_bf16), y is exact.   */
/* ybt = spikes transposed to bf16 [Np][Tp], Tp = round_up(T, 64), from    */
/* pmg_spikes_bf16t (once per data set).  t_w is summed from P in f64.     */
int pmg_spikes_bf16t(const float* yext, int64_t T, int32_t Np, uint16_t* ybt, int64_t Tp, void* stream);
size_t pmg_suffstats_bf16_workspace_size(int64_t T, int32_t L, int32_t N);
int pmg_suffstats_bf16(const float* P, const uint16_t* ybt, int64_t T, int64_t Tp, int32_t L, int32_t N,
                       int32_t Np, double* yw, double* tw, void* workspace, size_t workspace_bytes,
                       void* stream);
/* P = exp(logp) elementwise (the first M-step's exp at fit_tuning_helper.py:38). */
int pmg_exp(const float* logp, int64_t n, float* p, void* stream);
/* out = log(x) elementwise (log-space outputs; log(0) = -inf). */
int pmg_log(const float* x, int64_t n, float* out, void* stream);
/* The returned arrays of a posterior gamma (T, 2, L) f32 in one pass: log_out (T, 2, L) =
 * logf(gamma) (as pmg_log), plm (T, L) = gamma[t,0,l] + gamma[t,1,l] (posterior_latent_marg)
 * and pdm (T, 2) = sum_l gamma[t,d,l] (posterior_dynamics_marg, f64 sum rounded once) --
 * core.py:696-712 / decoder.py:300-315 form them with jnp sums.  Any output may be NULL. */
int pmg_posterior_outputs(const float* gamma, int64_t T, int32_t L, float* log_out, float* plm, float* pdm,
                          void* stream);
/* out[t, n] = y[(t - shift[n]) mod T, n] for y, out (T, N) row-major f32, shift (N,) int64
 * (device): every neuron's column rolled by its own shift, the np.roll of
 * test.circular_shuffle_data (reference poor_man_gplvm/test.py:10-24).  y != out. */
int pmg_roll_columns(const float* y, int64_t T, int32_t N, const int64_t* shift, float* out, void* stream);

/* ------------------------------------------------------------------ */
/* Adam M-step -- fit_tuning_helper.make_adam_runner.run                 */
/* (fit_tuning_helper.py:133-194) on poisson_m_step_objective            */
/* (:63-81) with optax 0.2.2 adam; one persistent launch, neurons        */
/* partitioned over workgroups, the stop rule                             */
/*   i < maxiter-1 and (i < 5 or |loss-loss_prev|/max(|loss|,1e-8) > tol) */
/* decided from globally summed f64 losses (fixed summation order).      */
/*   W, mu, nu (NB,N) f64 in/out; count (1) int64 in/out (optax count).  */
/*   stats (4) f64 out: n_iter, final_loss, final_error, unused.          */
/*   loss_hist, err_hist (maxiter) f64 out (zeros past n_iter).           */
/*   tol < 0: the loop never stops before maxiter (not even on a NaN loss,  */
/*   whose relative change compares false): the speculative batches of the */
/*   neuron-sharded M-step apply the stop rule on the host.                */
typedef struct pmg_adam_cfg {
  double lr, b1, b2, eps, eps_root;
  double prior_std;
  double tol;
  int32_t maxiter;
} pmg_adam_cfg;
size_t pmg_mstep_workspace_size(int32_t N, int32_t maxiter);
/* 1 when pmg_mstep_adam holds this (L, NB, N) shape (basis in registers + LDS, */
/* L <= 512), else 0: the caller then uses pmg_mstep_adam_tiled.               */
int pmg_mstep_adam_supported(int32_t L, int32_t NB, int32_t N);
int pmg_mstep_adam(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                   const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                   const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                   void* workspace, size_t workspace_bytes, void* stream);
/* Workgroups of the persistent launch wait on one another (the lagged stop      */
/* decision, the row-block B^T G exchange) in waits bounded by 2 s of the real-    */
/* time clock.  A wait that gives up sets the sticky int32 word 0 of the workspace */
/* and the launch's W / mu / nu / stats are then invalid.  No launch clears it:    */
/* allocate the workspace zeroed and read it with pmg_mstep_adam_status, which      */
/* syncs the stream, sets *timed_out (0/1) and clears the word (also the batched    */
/* call's workspace: every restart shares word 0).                                 */
int pmg_mstep_adam_status(void* workspace, int32_t* timed_out, void* stream);
/* R restarts' M-steps (batched restarts): W, mu, nu (R,NB,N),  */
/* count (R), yw (R*L, N) and tw (R*L) (the stacked suff-stats), stats (R,4), */
/* loss_hist / err_hist (R, max(maxiter,1)).  Each restart runs its own loop */
/* and stop rule (bit-identical to R pmg_mstep_adam calls); several restarts */
/* share one persistent launch (blockIdx.y) with up to 4 neurons per        */
/* workgroup, so R loops cost ~R * N / (4 * #CUs) launches instead of R.     */
size_t pmg_mstep_batched_workspace_size(int32_t L, int32_t NB, int32_t N, int32_t R, int32_t maxiter);
int pmg_mstep_adam_batched_supported(int32_t L, int32_t NB, int32_t N, int32_t R);
int pmg_mstep_adam_batched(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                           const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N, int32_t R,
                           const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                           void* workspace, size_t workspace_bytes, void* stream);

/* Same loop and outputs for shapes the persistent kernel does not hold          */
/* (L > 512 or NB > 128, e.g. BASELINE C4: L = 1024, NB = 154): per body an f64    */
/* LDS-tiled F = B W + gradient-factor kernel, an f64 B^T G + optax-update kernel  */
/* and a one-workgroup decision kernel (fixed-order sums); bodies are enqueued in */
/* batches of 16 and the host reads the decision word once per batch (this call   */
/* synchronises the stream).  Workspace: pmg_mstep_tiled_workspace_size.           */
size_t pmg_mstep_tiled_workspace_size(int32_t L, int32_t NB, int32_t N);
int pmg_mstep_adam_tiled(double* W, double* mu, double* nu, int64_t* count, const float* basis,
                         const double* yw, const double* tw, int32_t L, int32_t NB, int32_t N,
                         const pmg_adam_cfg* cfg, double* stats, double* loss_hist, double* err_hist,
                         void* workspace, size_t workspace_bytes, void* stream);

/* Sufficient statistics from P's bf16 planes (PMG_PHASE_P_BF16X3 output):       */
/* Pq uint16 [3][T][ldp] (ldp >= L, ldp % 8 == 0: the row stride of the planes,    */
/* R*L for stacked restarts with L = R*L), ybt as pmg_suffstats_bf16.  The same    */
/* exact-product bf16 MFMA GEMMs as pmg_suffstats_bf16 without the split (which   */
/* the backward did once per value); t_w from (hi + mid) + lo.  Replaces           */
/* fit_tuning_helper.get_statistics (fit_tuning_helper.py:28-42).                  */
size_t pmg_suffstats_bf16x3_workspace_size(int64_t T, int32_t L, int32_t N);
int pmg_suffstats_bf16x3(const uint16_t* Pq, int64_t ldp, const uint16_t* ybt, int64_t T, int64_t Tp, int32_t L,
                         int32_t N, int32_t Np, double* yw, double* tw, void* workspace, size_t workspace_bytes,
                         void* stream);

/* ------------------------------------------------------------------ */
/* Pairwise joint (decode only) -- the logaddexp accumulation of         */
/* decoder.smooth_one_step (decoder.py:215-221) as a T-contraction:       */
/*   S[x,x'] = sum_{t<T-1} alpha_t[x] * rho_{t+1}[x'],  x = (d,i)          */
/* (2L x 2L f64); the caller forms joint = A[d,d'] K[d',i,j] S.            */
size_t pmg_joint_workspace_size(int64_t T, int32_t L);
int pmg_joint_accumulate(const float* alpha, const float* rho, int64_t T, int32_t L, double* S,
                         void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ */
/* Page-locked HOST buffers for the arrays a fit returns (the host       */
/* arrays of core.run_em's result dict, core.py:696-712).  The pages are */
/* mapped, first-touched by `threads` host threads in parallel (as       */
/* transparent huge pages if `huge`), then registered with HIP, so a     */
/* device->host copy into them runs at full PCIe rate.  Host-only: no    */
/* stream, no device work; safe to call from a side thread while the     */
/* device computes.  Free with pmg_host_free(ptr, bytes).                */
int pmg_host_alloc(size_t bytes, int32_t threads, int32_t huge, void** out);
int pmg_host_free(void* ptr, size_t bytes);
/* device -> host copy into such a buffer, enqueued on `stream`               */
int pmg_copy_d2h(void* dst, const void* src, size_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PMG_H */
