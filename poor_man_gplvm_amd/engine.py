"""Device-resident EM engine for PoissonGPLVMJump1D on one MI355X.

Orchestrates the native kernels of ``libpmg_hip.so`` for one fit:

    M-step   pmg_suffstats  -> pmg_mstep_adam            (core.py:802-827)
    tuning   pmg_tuning_softplus                          (core.py:664, :772)
    E-step   pmg_emission_poisson -> pmg_emission_rowref
             -> pmg_forward_filter -> pmg_backward_smoother  (core.py:666 -> decoder.py:258-332)
             P = sum_d gamma feeds the next M-step          (core.py:668)

All tensors live on the GPU (torch allocations, torch's current stream); the host
only reads back per-iteration scalars at the end of a fit and the posteriors the
caller asks for.  There is no CPU fallback: a missing library or an unsupported
configuration raises.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as nat
from .gp_kernel import BandedTransition, DenseTransition, banded_transition


def _ru(x, m):
    return (int(x) + m - 1) // m * m


@dataclass
class AdamConfig:
    lr: float = 0.01
    maxiter: int = 1000
    tol: float = 1e-6
    prior_std: float = 1.0
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    eps_root: float = 0.0

    def to_c(self):
        return nat.AdamCfg(self.lr, self.b1, self.b2, self.eps, self.eps_root, self.prior_std,
                           self.tol, int(self.maxiter))


@dataclass
class ScanConfig:
    """Time-parallel scan parameters (see fwdbwd.hip)."""
    chunk: int | None = None     # time steps per chunk (None: ~2048 chunks)
    warmup: int = 48             # forgetting warm-up before each chunk (initial value)
    tol: float = 3e-6            # Hilbert-metric boundary tolerance.  A posterior's relative
                                 # error is bounded by the forward + backward boundary
                                 # distances, so 2 x tol stays inside the 1e-5 parity bar.
                                 # In slowly mixing regimes (the flat tuning of the first EM
                                 # iterations) two f32 chains of one filter settle 1.4e-6
                                 # (median) to 7.6e-6 (q99) apart and never coalesce bitwise
                                 # (profiles/r02_diag_cascade_c3.log, measured with a difference
                                 # of f32 logs, which overstates distances between tiny
                                 # components; the kernels now take the log of the ratio);
                                 # boundaries that fail on that noise alone cost a short
                                 # relaxation, not a rescan of T
    adaptive: bool = False       # per pass: double the warm-up when >1% of chunks needed
                                 # repair, halve it after two E-steps with <=0.1%.  Off by
                                 # default: the relaxation kernel absorbs the cascades of the
                                 # first EM iterations, and a doubled warm-up taxes every
                                 # later main pass (C3: 0.19 -> 0.36 ms forward at 192 steps)
    max_warmup: int = 1024
    min_warmup: int = 16
    chunk_bwd: int | None = None  # backward chunk (None: = chunk if set, else 2x the default)
    device_adaptive: bool = True  # PMG_PHASE_ADAPTIVE_WARMUP: after a pass where > 1/8 of the chunk
                                  # boundaries failed (the first EM iterations), the next main pass
                                  # of that direction warms up 256 steps (device-side decision)
    relax_segments: int = 0       # relaxation segments per sequence (0: #CUs, or #CUs / R for R
                                  # batched restarts; PMG_PHASE_SEGMENTS).  The repaired states depend
                                  # on the segment grid, so a single fit with #CUs / R segments
                                  # reproduces restart r of an R-restart batch bit for bit
    two_waves: bool = False       # PMG_PHASE_TWO_WAVES: the main passes run each chain on two waves
                                  # (L in (256, 1024]; half the latents per lane, LDS halo exchange)
    decode_exact: bool = True     # decode_latent / _decode_latent (the calls that return the pairwise
                                  # joint) run the dense log-domain scans with the full kernel: every
                                  # row of p_transition_* is then the reference's conditional, also for
                                  # latents the posterior never visits (their linear-space counts
                                  # underflow, and the far kernel entries the band drops decide them).
                                  # False: the banded linear-space scans (faster; those rows fall back
                                  # to the prior transition, core.JOINT_COUNT_FLOOR)

    def chunk_for(self, T):
        if self.chunk:
            return int(self.chunk)
        return max(32, int(math.ceil(T / 2048)))

    def chunk_dense_for(self, T):
        """Chunk of the dense log-domain scans: one 256-thread workgroup per chain and
        ~13 us per step at L = 512, so ~2 chains per CU and a warm-up that is small
        next to the chunk."""
        if self.chunk:
            return int(self.chunk)
        return max(64, int(math.ceil(T / 512)))

    def chunk_bwd_for(self, T):
        """The backward pass runs at ~1 wave per SIMD with twice the forward chunk: its
        per-step work is larger and its warm-up is then amortised over more output
        steps (C3 sweep, profiles/r01_c3_chunk_sweep.txt)."""
        if self.chunk_bwd:
            return int(self.chunk_bwd)
        if self.chunk:
            return int(self.chunk)
        return 2 * self.chunk_for(T)


def planes_ok(T, ld):
    """pmg_suffstats_bf16x3's operand bounds: ld % 8 == 0 and planes below 2 GiB."""
    return ld % 8 == 0 and T * ld * 2 < (1 << 31)


def default_device():
    if not torch.cuda.is_available():
        raise nat.NativeError("poor_man_gplvm_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


class SpikeData:
    """Spike counts prepared once per fit (pmg_spikes_prepare)."""

    def __init__(self, y, ma_neuron=None, device=None):
        """y: (n_time, n_neuron) host array, or a float32 device tensor (used in place)."""
        dev = device or default_device()
        if isinstance(y, torch.Tensor):
            if y.device.type != 'cuda' or y.dtype != torch.float32 or not y.is_contiguous():
                raise ValueError("a tensor y must be a contiguous float32 device tensor")
        else:
            y = np.asarray(y)
        if y.ndim != 2:
            raise ValueError(f"y must be (n_time, n_neuron), got {tuple(y.shape)}")
        self.T, self.N = int(y.shape[0]), int(y.shape[1])
        self.device = dev
        self.y = y if isinstance(y, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(y, dtype=np.float32),
                                                                       device=dev)
        self.Kp = _ru(self.N, 128)
        self.Np = _ru(self.N + 1, 64)
        self.Tp = _ru(self.T, 64)
        self.ma_2d = False
        self.ma = None
        if ma_neuron is not None:
            ma = np.asarray(ma_neuron, dtype=np.float32)
            if ma.ndim == 2:
                if ma.shape != (self.T, self.N):
                    raise ValueError(f"2-D ma_neuron must be {(self.T, self.N)}, got {ma.shape}")
                self.ma_2d = True
            elif ma.shape != (self.N,):
                raise ValueError(f"ma_neuron must be ({self.N},) or ({self.T},{self.N}), got {ma.shape}")
            if not (ma.ndim == 1 and np.all(ma == 1.0)):
                self.ma = torch.as_tensor(np.ascontiguousarray(ma), device=dev)
        self.yq = torch.empty((self.Tp, self.Kp), dtype=torch.int8, device=dev)
        self.gconst = torch.empty(self.T, dtype=torch.float64, device=dev)
        self.yext = torch.empty((self.T, self.Np), dtype=torch.float32, device=dev)
        self._flags = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ybt = None
        self._prepare()
        self.flags = int(self._flags.item())
        # exact int8 path: integer counts in [0,127], 0/1 mask, no per-time mask
        self.int_path = self.flags == 0 and not self.ma_2d
        # integer counts are exact in bf16: suff-stats on the bf16 MFMA (exact products)
        if not (self.flags & 1):
            self.ybt = torch.empty((self.Np, self.Tp), dtype=torch.int16, device=dev)
            self._transpose()

    def _prepare(self):
        nat.check(nat.load().pmg_spikes_prepare(nat.ptr(self.y), self.T, self.N, nat.ptr(self.ma),
                                                int(self.ma_2d), nat.ptr(self.yq), self.Kp,
                                                nat.ptr(self.gconst), nat.ptr(self.yext), self.Np,
                                                nat.ptr(self._flags), nat.stream_handle()),
                  "pmg_spikes_prepare")

    def _transpose(self):
        nat.check(nat.load().pmg_spikes_bf16t(nat.ptr(self.yext), self.T, self.Np, nat.ptr(self.ybt), self.Tp,
                                              nat.stream_handle()), "pmg_spikes_bf16t")

    def refresh(self):
        """Re-derive the prepared forms after self.y was rewritten in place on the device
        with the same multiset of counts per neuron (a permutation in time, such as
        pmg_roll_columns): the int8 / bf16 eligibility flags cannot change, so this
        stays on the stream without a host sync."""
        self._prepare()
        if self.ybt is not None:
            self._transpose()


class KernelTimer:
    """Per-call HIP event pairs on the current stream (torch.cuda.Event records on
    torch's current stream, the stream every native call is enqueued on)."""

    def __init__(self):
        self.events = {}

    def __call__(self, name):
        return _TimedSection(self, name)

    def summary(self):
        """{name: (calls, mean ms)} -- synchronises."""
        torch.cuda.synchronize()
        out = {}
        for k, evs in self.events.items():
            ms = [a.elapsed_time(b) for a, b in evs]
            out[k] = (len(ms), float(np.mean(ms)) if ms else 0.0)
        return out

    def reset(self):
        self.events = {}


class _TimedSection:
    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.a.record()

    def __exit__(self, *exc):
        b = torch.cuda.Event(enable_timing=True)
        b.record()
        self.timer.events.setdefault(self.name, []).append((self.a, b))
        return False


class _NoTimer:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_TIMER = _NoTimer()


class DeviceEM:
    """One fit's device state: spikes, basis, transition, workspaces, buffers."""

    def __init__(self, spikes: SpikeData, L: int, basis=None, scan: ScanConfig | None = None):
        self.lib = nat.load()
        self.sp = spikes
        self.dev = spikes.device
        self.T, self.N, self.L = spikes.T, spikes.N, int(L)
        self.scan = scan or ScanConfig()
        self.C = self.scan.chunk_for(self.T)
        self.Cb = self.scan.chunk_bwd_for(self.T)
        self.nblk = _ru(self.L, 32) // 32
        T, L, N, dev = self.T, self.L, self.N, self.dev
        f32, f64 = torch.float32, torch.float64
        self.basis = None
        if basis is not None:
            b = np.ascontiguousarray(basis, dtype=np.float32)
            if b.shape[0] != L:
                raise ValueError("basis must have n_latent_bin rows")
            self.NB = int(b.shape[1])
            self.basis = torch.as_tensor(b, device=dev)
        self.delta = torch.empty((T, L), dtype=f32, device=dev)
        self.rblk = torch.empty((T, self.nblk), dtype=f64, device=dev)
        self.phi = torch.empty((T, self.nblk), dtype=f32, device=dev)
        self.mref = torch.empty(T, dtype=f64, device=dev)
        self.alpha = torch.empty((T, 2, L), dtype=f32, device=dev)
        self.logc = torch.empty(T, dtype=f64, device=dev)
        self._P = torch.empty((T, L), dtype=f32, device=dev)
        # integer spikes: the backward writes P as its three exact bf16 planes, the operands
        # of the statistics GEMMs (PMG_PHASE_P_BF16X3), instead of f32 P
        self.use_planes = bool(self.PLANES and spikes.ybt is not None and planes_ok(T, L))
        self.Pq = torch.empty((3, T, L), dtype=torch.int16, device=dev) if self.use_planes else None
        self._p_fresh = 'f32'       # which of _P / Pq holds the current posterior marginal
        self.tuning64 = torch.empty((L, N), dtype=f64, device=dev)
        self.tuning32 = torch.empty((L, N), dtype=f32, device=dev)
        self.yw = torch.empty((L, N), dtype=f64, device=dev)
        self.tw = torch.empty(L, dtype=f64, device=dev)
        # zero-filled once: it holds the emission's sticky range flag (include/pmg.h)
        self.ws_em = torch.zeros(int(self.lib.pmg_emission_workspace_size(T, L, N)), dtype=torch.uint8, device=dev)
        self._em_flag = _flag_view(self.lib, self.ws_em, T, L, N)
        # zero-filled once (include/pmg.h): the scan kernels keep its control words zero
        self.ws_fb = torch.zeros(int(self.lib.pmg_fwdbwd_workspace_size(T, L, min(self.C, self.Cb))),
                                 dtype=torch.uint8, device=dev)
        ss_bytes = (max(self.lib.pmg_suffstats_bf16_workspace_size(T, L, N),
                        self.lib.pmg_suffstats_bf16x3_workspace_size(T, L, N) if self.use_planes else 0)
                    if spikes.ybt is not None
                    else self.lib.pmg_suffstats_workspace_size(T, L, spikes.Np))
        self.ws_ss = torch.empty(int(ss_bytes), dtype=torch.uint8, device=dev)
        if self.ws_fb.numel() == 0 and L <= 1024:
            raise nat.NativeError(f"pmg_fwdbwd_workspace_size(T={T}, L={L}) returned 0")
        # L > 1024: only the dense log-domain scans (set_transition refuses a banded one)
        self.ws_ad = AdamWorkspace(self.lib, self.dev)
        self.warm = [int(self.scan.warmup), int(self.scan.warmup)]   # forward, backward
        self._clean = [0, 0]
        self._rep_host = torch.zeros(nat.CTL_WORDS, dtype=torch.int32).pin_memory()
        self._rep_evt = None
        self.timer = None       # optional KernelTimer (bench): per-call HIP events
        self._tr = None
        self._tr_c = None
        self._invz = None
        self.dense = False          # transition held by the dense log-domain scans
        self.ws_dense = None
        self.log_alpha = None       # (T, 2, L) f64 log filter state (dense scans)
        self.ll64 = None            # (T, L) f64 unsplit ll (dense scans; None: not written)
        self.alpha_bits = 0         # phase bits of the last forward (PHASE_NO_JUMP_ROWS or 0)
        # device-side adaptive warm-up across the E-steps of ONE fit (run_em sets it; a
        # decode is a single E-step whose result must not depend on earlier calls)
        self.adaptive = False
        self.ma_latent = None
        # Gaussian observation model (GaussianGPLVMJump1D): when noise_std is set, the
        # emission, tuning and M-step dispatch to gaussian.hip; the scans are shared.
        self.noise_std = None
        self.gauss_prior_std = 1.0
        self._gstatus = None
        self._ws_gm = None

    # P as three bf16 planes between the backward and the statistics: bit-identical
    # statistics, measured slower at C3 (6 B written per cell instead of 4: k_backward
    # 180 -> 195 us, statistics 169 -> 176 us), so off by default
    PLANES = False

    @property
    def P(self):
        """(T, L) f32 posterior marginal sum_d gamma.  When the last backward wrote the bf16
        planes, they are recombined here, exactly ((hi + mid) + lo in f32).  The buffer is
        handed out for reading or writing, so the next M-step reads it, not the planes."""
        if self._p_fresh == 'planes':
            q = self.Pq.to(torch.int32) << 16
            f = q.view(torch.float32)
            torch.add(f[0], f[1], out=self._P)
            self._P.add_(f[2])
        self._p_fresh = 'f32'
        return self._P

    @P.setter
    def P(self, v):
        self._P = v
        self._p_fresh = 'f32'

    def _t(self, name):
        return self.timer(name) if self.timer is not None else _NO_TIMER

    def _seg_bits(self):
        """PMG_PHASE_SEGMENTS of ScanConfig.relax_segments (0: the library default)."""
        return nat.phase_segments(self.scan.relax_segments)

    def _tw_bits(self):
        return nat.PHASE_TWO_WAVES if self.scan.two_waves else 0

    # ------------------------------------------------------------------ setup
    def set_transition(self, tr):
        if tr.L != self.L:
            raise ValueError("transition size mismatch")
        if isinstance(tr, DenseTransition):
            self._set_dense(tr)
            return
        if self.L > 1024:
            raise nat.NativeError(f"n_latent_bin={self.L}: the banded scans hold L <= 1024; pass a DenseTransition "
                                  "(gp_kernel.make_transition / dense_transition)")
        self.dense = False
        self._tr = tr
        self._invz = torch.as_tensor(tr.invz, device=self.dev)
        c = nat.Transition()
        c.L = tr.L
        c.band = tr.band
        for k in range(tr.band + 1):
            c.g[k] = float(tr.g[k])
        c.invz = nat.ptr(self._invz)
        A = tr.A.astype(np.float32)
        c.A[0], c.A[1], c.A[2], c.A[3] = float(A[0, 0]), float(A[0, 1]), float(A[1, 0]), float(A[1, 1])
        self._tr_c = c

    def _set_dense(self, tr: DenseTransition):
        """Dense log-domain scans (dense_scan.hip): logK0 and its transpose on the device."""
        self.dense = True
        self._tr = tr
        lk64 = np.asarray(tr.logK0, dtype=np.float64)
        lk = lk64.astype(np.float32)
        with np.errstate(invalid='ignore'):
            lo = np.where(np.isfinite(lk), lk64 - lk.astype(np.float64), 0.0).astype(np.float32)
        self._dK = torch.as_tensor(np.ascontiguousarray(lk), device=self.dev)
        self._dKT = torch.as_tensor(np.ascontiguousarray(lk.T), device=self.dev)
        self._dKlo = torch.as_tensor(np.ascontiguousarray(lo), device=self.dev)
        self._dKTlo = torch.as_tensor(np.ascontiguousarray(lo.T), device=self.dev)
        c = nat.DenseTransition()
        c.L = self.L
        c.logK = nat.ptr(self._dK)
        c.logKT = nat.ptr(self._dKT)
        c.logK_lo = nat.ptr(self._dKlo)
        c.logKT_lo = nat.ptr(self._dKTlo)
        la = tr.logA.astype(np.float32)
        c.logA[0], c.logA[1], c.logA[2], c.logA[3] = (float(la[0, 0]), float(la[0, 1]), float(la[1, 0]),
                                                      float(la[1, 1]))
        self._tr_d = c
        self.Cd = self.scan.chunk_dense_for(self.T)
        need = int(self.lib.pmg_dense_workspace_size(self.T, self.L, self.Cd))
        if need == 0:
            raise nat.NativeError(f"n_latent_bin={self.L} unsupported by the dense scans (max 4096)")
        if self.ws_dense is None or self.ws_dense.numel() < need:
            # zero-filled: it holds the sticky relaxation timeout words (include/pmg.h)
            self.ws_dense = torch.zeros(need, dtype=torch.uint8, device=self.dev)
        if self.log_alpha is None:
            self.log_alpha = torch.empty((self.T, 2, self.L), dtype=torch.float64, device=self.dev)
        if self.ll64 is None:   # the emission writes the unsplit f64 ll for the dense scans
            self.ll64 = torch.empty((self.T, self.L), dtype=torch.float64, device=self.dev)

    def set_ma_latent(self, ma_latent):
        if ma_latent is None:
            self.ma_latent = None
            return
        m = np.asarray(ma_latent)
        if m.shape != (self.L,):
            raise ValueError(f"ma_latent must have shape ({self.L},)")
        if np.all(m != 0):
            self.ma_latent = None
        else:
            self.ma_latent = torch.as_tensor((m != 0).astype(np.uint8), device=self.dev)

    def set_log_posterior(self, log_post):
        """P = exp(log_posterior) (T, L) for the first M-step (fit_tuning_helper.py:38)."""
        lp = torch.as_tensor(np.ascontiguousarray(log_post, dtype=np.float32), device=self.dev)
        if tuple(lp.shape) != (self.T, self.L):
            raise ValueError(f"log_posterior must be {(self.T, self.L)}")
        nat.check(self.lib.pmg_exp(nat.ptr(lp), lp.numel(), nat.ptr(self._P), nat.stream_handle()), "pmg_exp")
        self._p_fresh = 'f32'

    # ------------------------------------------------------------------ M-step
    def m_step(self, W, mu, nu, count, cfg: AdamConfig, stats_out, lh_out, eh_out):
        """Sufficient statistics of self.P, then the Adam loop; W/mu/nu/count in place."""
        sh = nat.stream_handle()
        with self._t('suffstats'):
          if self._p_fresh == 'planes':
            nat.check(self.lib.pmg_suffstats_bf16x3(nat.ptr(self.Pq), self.L, nat.ptr(self.sp.ybt), self.T,
                                                    self.sp.Tp, self.L, self.N, self.sp.Np, nat.ptr(self.yw),
                                                    nat.ptr(self.tw), nat.ptr(self.ws_ss), self.ws_ss.numel(), sh),
                      "pmg_suffstats_bf16x3")
          elif self.sp.ybt is not None:
            nat.check(self.lib.pmg_suffstats_bf16(nat.ptr(self.P), nat.ptr(self.sp.ybt), self.T, self.sp.Tp,
                                                  self.L, self.N, self.sp.Np, nat.ptr(self.yw), nat.ptr(self.tw),
                                                  nat.ptr(self.ws_ss), self.ws_ss.numel(), sh),
                      "pmg_suffstats_bf16")
          else:
            nat.check(self.lib.pmg_suffstats(nat.ptr(self.P), nat.ptr(self.sp.yext), self.T, self.L, self.N,
                                             self.sp.Np, nat.ptr(self.yw), nat.ptr(self.tw),
                                             nat.ptr(self.ws_ss), self.ws_ss.numel(), sh), "pmg_suffstats")
        if self.noise_std is not None:
            self.gaussian_m_step(W)
            return
        self.adam(W, mu, nu, count, cfg, stats_out, lh_out, eh_out)

    def gaussian_m_step(self, W):
        """Analytic M-step of the Gaussian model (fit_tuning_helper.py:44-61) from the
        current y_w, t_w; W (NB, N) f64 overwritten.  A non-SPD system sets the sticky
        status word (and W = NaN), checked by gaussian_status() (no host sync here)."""
        need = int(self.lib.pmg_gaussian_mstep_workspace_size(self.NB, self.N))
        if self._ws_gm is None or self._ws_gm.numel() < need:
            self._ws_gm = torch.empty(need, dtype=torch.uint8, device=self.dev)
        if self._gstatus is None:
            self._gstatus = torch.zeros(1, dtype=torch.int32, device=self.dev)
        with self._t('mstep_gaussian'):
          nat.check(self.lib.pmg_gaussian_mstep(nat.ptr(self.basis), nat.ptr(self.yw), nat.ptr(self.tw), self.L,
                                                self.NB, self.N, float(self.noise_std), float(self.gauss_prior_std),
                                                nat.ptr(W), nat.ptr(self._gstatus), nat.ptr(self._ws_gm),
                                                self._ws_gm.numel(), nat.stream_handle()), "pmg_gaussian_mstep")

    def gaussian_status(self):
        """Raise if any Gaussian M-step since the last check met a non-positive pivot
        (device read: syncs); the sticky word is cleared for the next fit."""
        if self._gstatus is not None:
            bad = int(self._gstatus.item()) != 0
            self._gstatus.zero_()
            if bad:
                raise nat.NativeError("pmg_gaussian_mstep: normal-equation matrix is not positive definite")

    # shapes the persistent one-launch Adam kernel holds (the basis block in registers;
    # L in (512, 1024] as 256-row blocks of one neuron group exchanging their B^T G partials
    # each body, which needs row blocks x neuron groups <= #CUs, pmg_mstep_adam_supported);
    # the others use the tiled per-body kernels
    PERSISTENT_MAX_L, PERSISTENT_MAX_NB = 1024, 160

    def adam(self, W, mu, nu, count, cfg: AdamConfig, stats_out, lh_out, eh_out, yw=None):
        """The Adam loop on W (NB, n) f64 with sufficient statistics yw (L, n) (default:
        this engine's y_w, n = N); a column slice of the neurons when given (the
        neuron-sharded M-step of timeshard.py)."""
        if self.basis is None:
            raise ValueError("no basis")
        yw = self.yw if yw is None else yw
        n = int(W.shape[1])
        if tuple(yw.shape) != (self.L, n) or not yw.is_contiguous() or not W.is_contiguous():
            raise ValueError(f"adam: W {tuple(W.shape)} / yw {tuple(yw.shape)} mismatch")
        tiled = (self.L > self.PERSISTENT_MAX_L or self.NB > self.PERSISTENT_MAX_NB
                 or not self.lib.pmg_mstep_adam_supported(self.L, self.NB, n))
        if tiled:
            blocks = self._adam_blocks(n)
            if blocks is not None:
                with self._t('mstep_adam'):     # one section per M-step, whatever the launches
                    self._adam_blocked(W, mu, nu, count, cfg, stats_out, lh_out, eh_out, yw, blocks)
                return
        with self._t('mstep_adam'):
            self._adam_launch(W, mu, nu, count, cfg, stats_out, lh_out, eh_out, yw, tiled)

    # neuron blocks of the persistent kernel on one GPU (see _adam_blocked); False: the tiled
    # kernels for every shape one launch cannot hold
    ADAM_BLOCKED = True
    # the blocked loop's launches double from 16 up to this many bodies: each launch round
    # trip (host stop rule, snapshot) costs ~0.8 ms at C4 against ~34 us per body of kernel
    ADAM_BLOCKED_MAX_BATCH = 64

    def _adam_blocks(self, n):
        """The fewest contiguous neuron blocks that the persistent kernel holds one launch
        each, when all n neurons in one launch need more workgroups than there are CUs (e.g.
        C4's N = L = 1024 on one GPU: 4 row blocks x 256 neuron groups); None if no split
        up to 16 blocks fits or the shape is beyond the persistent kernel anyway."""
        if (not self.ADAM_BLOCKED or self.L > self.PERSISTENT_MAX_L or self.NB > self.PERSISTENT_MAX_NB
                or n < 2):
            return None
        from .timeshard import neuron_bounds
        for k in range(2, min(16, n) + 1):
            bounds = neuron_bounds(n, k)
            if all(self.lib.pmg_mstep_adam_supported(self.L, self.NB, b - a) for a, b in bounds):
                return bounds
        return None

    def _adam_blocked(self, W, mu, nu, count, cfg: AdamConfig, stats_out, lh_out, eh_out, yw, blocks):
        """One Adam M-step as neuron blocks of the persistent kernel on this GPU: the
        speculative loop of the neuron-sharded time shards (timeshard.speculative_adam:
        launches of 16, 32, then 64 bodies per block (ADAM_BLOCKED_MAX_BATCH) with the local
        stop rule off, one snapshot copy per launch round, the reference's stop rule
        on the blocks' summed loss partials, replay up to the stopping body), with the blocks
        in place of ranks.  The per-element arithmetic does not depend on the neuron
        partition, so W, mu, nu equal one launch's (test_neuron_sharded_adam_bit_identical);
        in place of the tiled f64 kernels (~97 us per body at C4) each body costs the blocks'
        persistent bodies."""
        from .timeshard import SPEC_BATCH, speculative_adam
        mi = max(int(cfg.maxiter), 1)
        mb = self.ADAM_BLOCKED_MAX_BATCH
        # every block's (W, mu, nu) as views of ONE flat buffer and the counts of one tensor,
        # so a snapshot / restore is one copy each (not four per block)
        NB = W.shape[0]
        flat = torch.empty(3 * NB * W.shape[1], dtype=W.dtype, device=W.device)
        cnts = count.repeat(len(blocks)).contiguous()
        sl, off = [], 0
        for i, (a, b) in enumerate(blocks):
            n_b = NB * (b - a)
            d = dict(yw=yw[:, a:b].contiguous(), count=cnts[i:i + 1])
            for k, src in (('W', W), ('mu', mu), ('nu', nu)):
                v = flat[off:off + n_b].view(NB, b - a)
                v.copy_(src[:, a:b])
                d[k] = v
                off += n_b
            sl.append(d)
        hl = max(mi, mb + 1) + 1
        hist = torch.zeros((len(sl), 4 + 2 * hl), dtype=torch.float64, device=self.dev)

        def run(kmax):
            c = AdamConfig(lr=cfg.lr, maxiter=kmax, tol=-1.0, prior_std=cfg.prior_std, b1=cfg.b1, b2=cfg.b2,
                           eps=cfg.eps, eps_root=cfg.eps_root)
            k = int(kmax)
            if k > hl:
                raise ValueError(f"blocked Adam launch of {k} bodies > history slots {hl}")
            for i, d in enumerate(sl):
                h = hist[i]
                self._adam_launch(d['W'], d['mu'], d['nu'], d['count'], c, h[:4], h[4:4 + hl], h[4 + hl:],
                                  d['yw'], False)
            sel = torch.cat([hist[:, :1], hist[:, 4:4 + k], hist[:, 4 + hl:4 + hl + k]], dim=1).cpu().numpy()
            return [(int(r[0]), r[1:1 + int(r[0])], r[1 + k:1 + k + int(r[0])]) for r in sel]

        def snapshot():
            return flat.clone(), cnts.clone()

        def restore(snap):
            flat.copy_(snap[0])
            cnts.copy_(snap[1])

        res = speculative_adam(run, snapshot, restore, lambda x: np.asarray(x, np.float64), int(cfg.maxiter),
                               float(cfg.tol), batch=SPEC_BATCH, max_batch=mb)
        for (a, b), d in zip(blocks, sl):
            W[:, a:b].copy_(d['W'])
            mu[:, a:b].copy_(d['mu'])
            nu[:, a:b].copy_(d['nu'])
        count.copy_(sl[0]['count'])
        n = int(res['n_iter'])
        stats_out.copy_(torch.tensor([n, res['final_loss'], res['final_error'], res['loss0']], dtype=torch.float64))
        k = min(n, lh_out.shape[-1])
        lh_out.zero_()
        eh_out.zero_()
        lh_out[:k].copy_(torch.as_tensor(res['loss_history'][:k]))
        eh_out[:k].copy_(torch.as_tensor(res['error_history'][:k]))

    def _adam_launch(self, W, mu, nu, count, cfg: AdamConfig, stats_out, lh_out, eh_out, yw, tiled):
        n = int(W.shape[1])
        need = int(self.lib.pmg_mstep_tiled_workspace_size(self.L, self.NB, n) if tiled
                   else self.lib.pmg_mstep_workspace_size(n, int(cfg.maxiter)))
        ws = self.ws_ad.get(need, tiled)
        c = cfg.to_c()
        fn = self.lib.pmg_mstep_adam_tiled if tiled else self.lib.pmg_mstep_adam
        nat.check(fn(nat.ptr(W), nat.ptr(mu), nat.ptr(nu), nat.ptr(count),
                     nat.ptr(self.basis), nat.ptr(yw), nat.ptr(self.tw),
                     self.L, self.NB, n, ctypes.byref(c), nat.ptr(stats_out),
                     nat.ptr(lh_out), nat.ptr(eh_out), nat.ptr(ws),
                     ws.numel(), nat.stream_handle()),
                  "pmg_mstep_adam_tiled" if tiled else "pmg_mstep_adam")

    def compute_tuning(self, W):
        if self.noise_std is not None:
            with self._t('tuning_linear'):
              nat.check(self.lib.pmg_tuning_linear(nat.ptr(self.basis), nat.ptr(W), self.L, self.NB, self.N,
                                                   nat.ptr(self.tuning64), nat.ptr(self.tuning32),
                                                   nat.stream_handle()), "pmg_tuning_linear")
            return
        with self._t('tuning_softplus'):
          nat.check(self.lib.pmg_tuning_softplus(nat.ptr(self.basis), nat.ptr(W), self.L, self.NB, self.N,
                                               nat.ptr(self.tuning64), nat.ptr(self.tuning32),
                                               nat.stream_handle()), "pmg_tuning_softplus")

    def set_tuning(self, tuning):
        t = np.ascontiguousarray(tuning, dtype=np.float64)
        if t.shape != (self.L, self.N):
            raise ValueError(f"tuning must be {(self.L, self.N)}")
        self.tuning64.copy_(torch.as_tensor(t, device=self.dev))
        self.tuning32.copy_(self.tuning64.to(torch.float32))

    # ------------------------------------------------------------------ E-step
    def emission(self, likelihood_scale=1.0, dt=1.0):
        sp, sh = self.sp, nat.stream_handle()
        with self._t('emission'):
          self._emission_call(sp, sh, dt)
        with self._t('emission_rowref'):
          nat.check(self.lib.pmg_emission_rowref(nat.ptr(self.rblk), self.T, self.nblk, float(likelihood_scale),
                                                 nat.ptr(self.phi), nat.ptr(self.mref), sh), "pmg_emission_rowref")

    def emission_unmasked(self, dt=1.0):
        """The emission contraction without a latent mask into fresh (delta0, rblk0)
        buffers, to be masked per use by emission_from."""
        saved, self.ma_latent = self.ma_latent, None
        try:
            with self._t('emission'):
                self._emission_call(self.sp, nat.stream_handle(), dt)
        finally:
            self.ma_latent = saved
        return self.delta.clone(), self.rblk.clone()

    def emission_from(self, delta0, rblk0, ma_latent_u8, likelihood_scale=1.0):
        """(delta, rblk) = (delta0, rblk0) under the latent mask ma_latent_u8 ((L,) uint8
        device tensor; pmg_emission_latent_mask), then the row reference."""
        if tuple(ma_latent_u8.shape) != (self.L,) or ma_latent_u8.dtype != torch.uint8:
            raise ValueError(f"ma_latent_u8 must be a ({self.L},) uint8 tensor")
        # the f64 ll the dense scans prefer when present is the UNMASKED one
        # (emission_unmasked): drop it, so the masked (delta, rblk) are what the scans read
        self.ll64 = None
        sh = nat.stream_handle()
        with self._t('emission_mask'):
            nat.check(self.lib.pmg_emission_latent_mask(nat.ptr(delta0), nat.ptr(rblk0), self.T, self.L,
                                                        nat.ptr(ma_latent_u8), nat.ptr(self.delta),
                                                        nat.ptr(self.rblk), sh), "pmg_emission_latent_mask")
        with self._t('emission_rowref'):
            nat.check(self.lib.pmg_emission_rowref(nat.ptr(self.rblk), self.T, self.nblk, float(likelihood_scale),
                                                   nat.ptr(self.phi), nat.ptr(self.mref), sh), "pmg_emission_rowref")

    # masks per batched forward launch (log-marginal passes; ~13 device bytes per (t, l) each)
    MASK_BATCH_MAX = 16
    MASK_BATCH_BYTES = 16 << 30

    def mask_batch_size(self, R):
        per = 13 * self.T * self.L
        return int(max(1, min(R, self.MASK_BATCH_MAX, self.MASK_BATCH_BYTES // max(per, 1))))

    def masked_chunk(self):
        """Forward chunk of the log-marginal mask passes (independent of the batch size)."""
        return max(32, int(math.ceil(self.MASK_BATCH_MAX * self.T / 2048)))

    def masked_segments(self):
        """Relaxation segments per mask of the log-marginal passes (independent of the batch
        size; all MASK_BATCH_MAX masks' segments are co-resident)."""
        if self.scan.relax_segments:
            return int(self.scan.relax_segments)
        cus = torch.cuda.get_device_properties(self.dev).multi_processor_count
        return max(1, cus // self.MASK_BATCH_MAX)

    def masked_logz_batched(self, delta0, rblk0, masks_u8, likelihood_scale, logz_out):
        """log_marginal_final of the forward filter under each of R latent masks
        (masks_u8 (R, L) uint8 device tensor) in ONE pass per stage: the R masked
        emissions are written side by side as R stacked latent sets
        (pmg_emission_latent_mask_batched), one row reference per mask
        (pmg_emission_rowref_batched) and one chunk-parallel forward launch covers every
        mask (pmg_forward_filter_batched, blockIdx.y = mask, no alpha written:
        PMG_PHASE_NO_ALPHA).  The chunk and the relaxation segment grid are pinned to
        the largest batch (MASK_BATCH_MAX masks: chunk ceil(16 T / 2048), #CUs / 16
        segments per mask), so a mask's logZ does not depend on how many masks share
        its batch, on the rank count that dealt them, or on the memory budget; it equals
        a single-mask forward on that chunk and segment grid bit for bit.
        Banded transitions, L % 32 == 0."""
        R = int(masks_u8.shape[0])
        T, L, dev = self.T, self.L, self.dev
        if self.dense or L % 32:
            raise nat.NativeError("batched masks need the banded scans and n_latent_bin % 32 == 0")
        nb = self.nblk
        sc = self.scan
        C = int(sc.chunk) if sc.chunk else self.masked_chunk()
        key = (R, C)
        if getattr(self, '_mb_key', None) != key:
            f32, f64 = torch.float32, torch.float64
            self._mb = dict(delta=torch.empty((T, R * L), dtype=f32, device=dev),
                            rblk=torch.empty((T, R * nb), dtype=f64, device=dev),
                            phi=torch.empty((T, R * nb), dtype=f32, device=dev),
                            mref=torch.empty((T, R), dtype=f64, device=dev),
                            logc=torch.empty((R, T), dtype=f64, device=dev),
                            ws=torch.zeros(int(self.lib.pmg_fwdbwd_batched_workspace_size(T, L, C, R)),
                                           dtype=torch.uint8, device=dev))
            self._mb_key = key
        b = self._mb
        sh = nat.stream_handle()
        with self._t('emission_mask'):
            nat.check(self.lib.pmg_emission_latent_mask_batched(nat.ptr(delta0), nat.ptr(rblk0), T, L,
                                                                nat.ptr(masks_u8), R, nat.ptr(b['delta']),
                                                                nat.ptr(b['rblk']), sh),
                      "pmg_emission_latent_mask_batched")
        with self._t('emission_rowref'):
            nat.check(self.lib.pmg_emission_rowref_batched(nat.ptr(b['rblk']), T, R * nb, R, float(likelihood_scale),
                                                           nat.ptr(b['phi']), nat.ptr(b['mref']), sh),
                      "pmg_emission_rowref_batched")
        # no alpha is written (PMG_PHASE_NO_ALPHA); the kernels only need a valid pointer
        args = (nat.ptr(b['delta']), nat.ptr(b['phi']), nat.ptr(b['mref']), T, R, ctypes.byref(self._tr_c),
                float(likelihood_scale), C, int(sc.warmup), float(sc.tol), nat.ptr(self.alpha),
                nat.ptr(b['logc']), nat.ptr(logz_out), nat.ptr(b['ws']), b['ws'].numel(), sh)
        with self._t('forward_filter'):
            nat.check(self.lib.pmg_forward_filter_batched(*args, 1 | nat.PHASE_NO_ALPHA), "pmg_forward_filter_batched")
        with self._t('forward_repair'):
            nat.check(self.lib.pmg_forward_filter_batched(
                *args, 2 | nat.PHASE_NO_ALPHA | nat.phase_segments(self.masked_segments())),
                "pmg_forward_filter_batched")
        w = b['ws']
        slab = (w.numel() // R) & ~255 if R > 1 else w.numel()
        views = [w[r * slab:r * slab + 4 * nat.CTL_WORDS].view(torch.int32) for r in range(R)]
        host = torch.stack(views).cpu().numpy()   # one read of every mask's sticky timeout words
        for r in range(R):
            _raise_on_timeout(views[r], host[r], "masked forward relaxation")

    def _emission_call(self, sp, sh, dt):
        if self.noise_std is not None:
            nat.check(self.lib.pmg_emission_gaussian(nat.ptr(sp.y), nat.ptr(self.tuning64), nat.ptr(sp.ma),
                                                     int(sp.ma_2d), nat.ptr(self.ma_latent), float(self.noise_std),
                                                     float(dt), self.T, self.L, self.N, nat.ptr(self.delta),
                                                     nat.ptr(self.rblk), nat.ptr(self.ll64), sh),
                      "pmg_emission_gaussian")
        elif sp.int_path:
            ma1 = sp.ma if (sp.ma is not None and not sp.ma_2d) else None
            nat.check(self.lib.pmg_emission_poisson(nat.ptr(sp.yq), nat.ptr(sp.gconst), nat.ptr(self.tuning64),
                                                    nat.ptr(ma1), nat.ptr(self.ma_latent), float(dt), self.T,
                                                    self.L, self.N, sp.Kp, nat.ptr(self.delta),
                                                    nat.ptr(self.rblk), nat.ptr(self.ll64), nat.ptr(self.ws_em),
                                                    self.ws_em.numel(), sh), "pmg_emission_poisson")
        else:
            nat.check(self.lib.pmg_emission_poisson_f64(nat.ptr(sp.y), nat.ptr(sp.gconst), nat.ptr(self.tuning64),
                                                        nat.ptr(sp.ma), int(sp.ma_2d), nat.ptr(self.ma_latent),
                                                        float(dt), self.T, self.L, self.N, nat.ptr(self.delta),
                                                        nat.ptr(self.rblk), nat.ptr(self.ll64), nat.ptr(self.ws_em),
                                                        self.ws_em.numel(), sh), "pmg_emission_poisson_f64")

    def _adapt_warmup(self):
        """Adaptive warm-up from the previous E-step's repair counters, read without a
        host sync (pinned async copy + event query)."""
        if not self.scan.adaptive or self._rep_evt is None or not self._rep_evt.query():
            return
        Ms = ((self.T + self.C - 1) // self.C, (self.T + self.Cb - 1) // self.Cb)
        ctl = self._rep_host.tolist()
        for i, r in enumerate((ctl[nat.CTL_FWD + nat.CTL_REPAIRS], ctl[nat.CTL_BWD + nat.CTL_REPAIRS])):
            M = Ms[i]
            if r > max(1, M // 100):
                self.warm[i] = min(self.scan.max_warmup, 2 * self.warm[i])
                self._clean[i] = 0
            elif r <= M // 1000:
                self._clean[i] += 1
                if self._clean[i] >= 2 and self.warm[i] > self.scan.min_warmup:
                    self.warm[i] = max(self.scan.min_warmup, self.warm[i] // 2)
                    self._clean[i] = 0
            else:
                self._clean[i] = 0
        self._rep_evt = None

    def ctl_words(self):
        """The scans' int32 control words (device view; see fb_kernels.h kCtl*; the dense
        scans use the same layout in their own workspace)."""
        ws = self.ws_dense if self.dense else self.ws_fb
        return ws[:4 * nat.CTL_WORDS].view(torch.int32)

    def reset_adaptive(self):
        """Start of a fit: forget the adaptive warm-up decisions of earlier E-steps (the
        kCtlWarm words of both directions)."""
        w = self.ws_fb[:4 * nat.CTL_WORDS].view(torch.int32)
        w[nat.CTL_FWD + nat.CTL_WARM] = 0
        w[nat.CTL_BWD + nat.CTL_WARM] = 0

    def emission_status(self):
        """Raise if an integer-path emission since the last check met |log lam| >= 60
        (outside the exact digit range; device read: syncs), then clear the flag."""
        _check_emission_flag(self._em_flag)

    def _snapshot_repairs(self):
        self._rep_host.copy_(self.ctl_words(), non_blocking=True)
        self._rep_evt = torch.cuda.Event()
        self._rep_evt.record()

    def forward(self, likelihood_scale, logz_out, keep_alpha=True):
        """keep_alpha False: alpha's d = 1 rows are not written (the backward call rebuilds
        them from per-step scalars; callers that read only P / logZ skip 4 T L bytes)."""
        if self.dense:
            with self._t('forward_filter'):      # main pass + verify + relaxation + logZ
                nat.check(self.lib.pmg_dense_forward(
                    nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.ll64), nat.ptr(self.mref), self.T,
                    ctypes.byref(self._tr_d),
                    float(likelihood_scale), self.Cd, int(self.warm[0]), float(self.scan.tol),
                    nat.ptr(self.alpha), nat.ptr(self.log_alpha), nat.ptr(self.logc), nat.ptr(logz_out),
                    nat.ptr(self.ws_dense), self.ws_dense.numel(), nat.stream_handle()), "pmg_dense_forward")
            return
        self._adapt_warmup()
        sc = self.scan
        args = (nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.mref), self.T, ctypes.byref(self._tr_c),
                float(likelihood_scale), self.C, int(self.warm[0]), float(sc.tol), nat.ptr(self.alpha),
                nat.ptr(self.logc), nat.ptr(logz_out), nat.ptr(self.ws_fb), self.ws_fb.numel(),
                nat.stream_handle())
        self.alpha_bits = 0 if keep_alpha else nat.PHASE_NO_JUMP_ROWS
        ad = nat.PHASE_ADAPTIVE_WARMUP if (sc.device_adaptive and self.adaptive) else 0
        with self._t('forward_filter'):          # main chunk-parallel pass (k_forward)
            nat.check(self.lib.pmg_forward_filter_phase(*args, 1 | ad | self.alpha_bits | self._tw_bits()), "pmg_forward_filter")
        with self._t('forward_repair'):          # verify / relaxation / logZ
            nat.check(self.lib.pmg_forward_filter_phase(*args, 2 | ad | self.alpha_bits | self._seg_bits()),
                      "pmg_forward_filter")

    def backward(self, likelihood_scale, P=True, gamma=None, rho=None, log_gamma=None):
        """rho: the joint partner; with the dense scans it is written as log(rho), f64
        (see joint_log)."""
        if self.dense:
            with self._t('backward_smoother'):
                nat.check(self.lib.pmg_dense_backward(
                    nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.ll64), nat.ptr(self.log_alpha), self.T,
                    ctypes.byref(self._tr_d),
                    float(likelihood_scale), self.Cd, int(self.warm[1]), float(self.scan.tol),
                    nat.ptr(self._P) if P else None, nat.ptr(gamma), nat.ptr(log_gamma), None, nat.ptr(rho),
                    nat.ptr(self.ws_dense), self.ws_dense.numel(), nat.stream_handle()), "pmg_dense_backward")
            if P:
                self._p_fresh = 'f32'
            return
        if log_gamma is not None:
            raise ValueError("log_gamma is produced by the dense scans only")
        sc = self.scan
        planes = bool(P) and self.use_planes
        pout = (nat.ptr(self.Pq) if planes else nat.ptr(self._P)) if P else None
        args = (nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.alpha), self.T, ctypes.byref(self._tr_c),
                float(likelihood_scale), self.Cb, int(self.warm[1]), float(sc.tol),
                pout, nat.ptr(gamma), nat.ptr(rho), nat.ptr(self.ws_fb),
                self.ws_fb.numel(), nat.stream_handle())
        ad = (nat.PHASE_ADAPTIVE_WARMUP if (sc.device_adaptive and self.adaptive) else 0) | \
            (nat.PHASE_P_BF16X3 if planes else 0)
        if P:
            self._p_fresh = 'planes' if planes else 'f32'
        with self._t('backward_smoother'):       # main chunk-parallel pass (k_backward)
            nat.check(self.lib.pmg_backward_smoother_phase(*args, 1 | ad | self._tw_bits()), "pmg_backward_smoother")
        with self._t('backward_repair'):         # verify / relaxation
            nat.check(self.lib.pmg_backward_smoother_phase(*args, 2 | ad | self._seg_bits()), "pmg_backward_smoother")

    def e_step(self, likelihood_scale, logz_out, gamma=None, rho=None, log_gamma=None, keep_alpha=None):
        """keep_alpha (default: whenever a posterior output is requested): write alpha in full."""
        if keep_alpha is None:
            keep_alpha = gamma is not None or rho is not None or log_gamma is not None
        self.emission(likelihood_scale)
        self.forward(likelihood_scale, logz_out, keep_alpha)
        self.backward(likelihood_scale, True, gamma, rho, log_gamma)
        if self.scan.adaptive:      # host-side adaptation reads the counters without a sync
            self._snapshot_repairs()

    def repairs(self):
        """(forward, backward) chunks recomputed by the last scans' relaxation (device
        read: syncs).  Raises if a relaxation kernel's bounded grid barrier timed out
        since the last check (the sticky timeout words; cleared here)."""
        w = self.ctl_words()
        r = w.cpu().numpy()
        _raise_on_timeout(w, r, "scan relaxation")
        return int(r[nat.CTL_FWD + nat.CTL_REPAIRS]), int(r[nat.CTL_BWD + nat.CTL_REPAIRS])

    def scan_status(self):
        """Raise if any scan relaxation since the last check timed out in its bounded grid
        barrier (its outputs are invalid); the sticky timeout words are cleared.  Device
        read: syncs."""
        w = self.ctl_words()
        _raise_on_timeout(w, w.cpu().numpy(), "scan relaxation")

    def adam_status(self):
        """Raise if a persistent Adam launch since the last check timed out in a
        cross-workgroup wait (sticky word, cleared here; syncs)."""
        self.ws_ad.status()

    def check_status(self):
        """Every sticky device error of the calls since the last check: the scans' and
        the Adam loop's timeout words and (integer-path Poisson emission) the digit-range
        flag."""
        self.scan_status()
        self.adam_status()
        if self.noise_std is None:
            self.emission_status()

    def relax_rounds(self):
        """(forward, backward) relaxation rounds of the last scans (device read: syncs)."""
        r = self.ctl_words().cpu().numpy()
        return int(r[nat.CTL_FWD + nat.CTL_ROUNDS]), int(r[nat.CTL_BWD + nat.CTL_ROUNDS])

    def loglik(self):
        ll = torch.empty((self.T, self.L), dtype=torch.float32, device=self.dev)
        nat.check(self.lib.pmg_loglik_materialize(nat.ptr(self.delta), nat.ptr(self.rblk), self.T, self.L,
                                                  nat.ptr(ll), nat.stream_handle()), "pmg_loglik_materialize")
        return ll

    def joint_log(self, log_rho):
        """Dense scans: log S[x,x'] = LSE_t log alpha_t[x] + log rho_{t+1}[x'] (2L x 2L, f64)."""
        S = torch.empty((2 * self.L, 2 * self.L), dtype=torch.float64, device=self.dev)
        # split partials only when the tiles alone leave the chip idle (size 0 otherwise, e.g. L >= 1024)
        nws = int(self.lib.pmg_joint_log_workspace_size(self.T, self.L))
        ws = torch.empty(nws, dtype=torch.uint8, device=self.dev) if nws else None
        with self._t('joint_log'):
            nat.check(self.lib.pmg_joint_log_accumulate_ws(nat.ptr(self.log_alpha), nat.ptr(log_rho), self.T, self.L,
                                                           nat.ptr(S), nat.ptr(ws) if nws else None, nws,
                                                           nat.stream_handle()),
                      "pmg_joint_log_accumulate")
        return S

    def joint(self, rho):
        """S[x,x'] = sum_t alpha_t[x] rho_{t+1}[x'] (2L x 2L, f64)."""
        ws = torch.empty(int(self.lib.pmg_joint_workspace_size(self.T, self.L)), dtype=torch.uint8, device=self.dev)
        S = torch.empty((2 * self.L, 2 * self.L), dtype=torch.float64, device=self.dev)
        with self._t('joint'):
            nat.check(self.lib.pmg_joint_accumulate(nat.ptr(self.alpha), nat.ptr(rho), self.T, self.L, nat.ptr(S),
                                                    nat.ptr(ws), ws.numel(), nat.stream_handle()),
                      "pmg_joint_accumulate")
        return S


def _raise_on_timeout(words, host, what):
    """words: a (CTL_WORDS,) int32 device view of a scan control block pair; host: its
    values.  A set timeout word is cleared (it is sticky on the device) and raised."""
    bad = [d for d in (nat.CTL_FWD, nat.CTL_BWD) if host[d + nat.CTL_ERR]]
    if bad:
        for d in bad:
            words[d + nat.CTL_ERR] = 0
        raise nat.NativeError(f"{what}: grid barrier timed out (results of the calls since the last check are "
                              "invalid)")


class AdamWorkspace:
    """Workspaces of the Adam M-step.  The persistent kernels' (pmg_mstep_adam,
    _batched) starts with the sticky timeout word of their bounded cross-workgroup waits,
    so it is allocated zeroed and its word is read (and cleared) by status(); it is
    checked before a larger one replaces it.  The tiled kernels get their own buffer."""

    def __init__(self, lib, dev):
        self.lib, self.dev = lib, dev
        self.persistent = None
        self.tiled = None

    def get(self, need, tiled):
        if tiled:
            if self.tiled is None or self.tiled.numel() < need:
                self.tiled = torch.empty(need, dtype=torch.uint8, device=self.dev)
            return self.tiled
        if self.persistent is None or self.persistent.numel() < need:
            self.status()
            self.persistent = torch.zeros(max(need, 256), dtype=torch.uint8, device=self.dev)
        return self.persistent

    def status(self):
        """Raise if a persistent Adam launch since the last check gave up a bounded wait
        on another workgroup (its W / mu / nu are then invalid).  Syncs the stream."""
        if self.persistent is None:
            return
        flag = ctypes.c_int32(0)
        nat.check(self.lib.pmg_mstep_adam_status(nat.ptr(self.persistent), ctypes.byref(flag),
                                                 nat.stream_handle()), "pmg_mstep_adam_status")
        if flag.value:
            raise nat.NativeError("pmg_mstep_adam: a cross-workgroup wait timed out; the M-step result is invalid")


def _flag_view(lib, ws, T, L, N):
    """The emission workspace's int32 range flag as a (1,) device view."""
    off = int(lib.pmg_emission_range_flag(ctypes.c_void_p(ws.data_ptr()), T, L, N)) - ws.data_ptr()
    return ws[off:off + 4].view(torch.int32)


def _check_emission_flag(flag):
    bad = int(flag.item()) != 0
    flag.zero_()
    if bad:
        raise nat.NativeError("pmg_emission_poisson: |log(tuning*dt)| >= 60 somewhere -- outside the exact "
                              "int8-digit range (the emission of that E-step is invalid)")


def log_of(x: torch.Tensor) -> torch.Tensor:
    """Elementwise log on the device (pmg_log); log(0) = -inf."""
    out = torch.empty_like(x)
    nat.check(nat.load().pmg_log(nat.ptr(x), x.numel(), nat.ptr(out), nat.stream_handle()), "pmg_log")
    return out


def posterior_outputs(gamma: torch.Tensor, log: bool = True):
    """(log gamma or None, posterior_latent_marg (T, L), posterior_dynamics_marg (T, 2)) of a
    posterior (T, 2, L) f32, in one device pass (pmg_posterior_outputs)."""
    if gamma.dim() != 3 or gamma.shape[1] != 2 or gamma.dtype != torch.float32:
        raise ValueError("posterior_outputs: expected a (T, 2, L) float32 tensor")
    T, _, L = gamma.shape
    lg = torch.empty_like(gamma) if log else None
    plm = torch.empty((T, L), dtype=torch.float32, device=gamma.device)
    pdm = torch.empty((T, 2), dtype=torch.float32, device=gamma.device)
    nat.check(nat.load().pmg_posterior_outputs(nat.ptr(gamma), T, L, nat.ptr(lg), nat.ptr(plm), nat.ptr(pdm),
                                               nat.stream_handle()), "pmg_posterior_outputs")
    return lg, plm, pdm


class RestartBatchEM:
    """R independent EM restarts of one recording on one GPU (model_selection_helper.py:53-59:
    the restarts differ only in their posterior init; SURVEY 8(e): 8 restarts per GPU at C5).

    The restarts' latents are stacked side by side, so the dense stages run once for all
    of them:
      * tuning: pmg_tuning_softplus_batched, W (R, NB, N) -> the (R L, N) tuning;
      * emission: ONE int8-MFMA contraction of y (T, N) against R L latents -> delta
        (T, R L), then pmg_emission_rowref_batched (each restart its own row reference);
      * scans: pmg_forward_filter_batched / pmg_backward_smoother_batched, one launch per
        pass with blockIdx.y = restart (each restart its own alpha (T, 2, L), logc, logZ
        and workspace slab), writing P (T, R L);
      * sufficient statistics: ONE bf16-MFMA GEMM over the R L latents -> y_w (R L, N),
        t_w (R L), whose row blocks are the restarts' statistics;
      * Adam: pmg_mstep_adam_batched, several restarts per persistent launch (each its
        own loop and stop rule, bit-identical to separate fits); the tiled kernels run
        once per restart where the persistent one cannot hold the shape.
    Chunks are sized so the R restarts together run ~2048 chains (R x longer chunks than
    one restart alone: the warm-up is amortised over R x more output steps).
    Banded transitions only; L % 32 == 0; Poisson observation model."""

    def __init__(self, spikes: SpikeData, L: int, basis, R: int, scan: ScanConfig | None = None):
        self.lib = nat.load()
        self.sp = spikes
        self.dev = spikes.device
        self.R = int(R)
        self.T, self.N, self.L = spikes.T, spikes.N, int(L)
        if self.R < 1:
            raise ValueError("R >= 1 restarts")
        if self.L % 32:
            raise nat.NativeError(f"batched restarts need n_latent_bin % 32 == 0 (got {self.L})")
        self.scan = scan or ScanConfig()
        T, L, N, R, dev = self.T, self.L, self.N, self.R, self.dev
        RT = R * T
        self.C = self.scan.chunk if self.scan.chunk else max(32, int(math.ceil(RT / 2048)))
        self.Cb = self.scan.chunk_bwd or (self.scan.chunk if self.scan.chunk else 2 * self.C)
        b = np.ascontiguousarray(basis, dtype=np.float32)
        if b.shape[0] != L:
            raise ValueError("basis must have n_latent_bin rows")
        self.NB = int(b.shape[1])
        self.basis = torch.as_tensor(b, device=dev)
        LA = R * L
        self.nblk = L // 32
        f32, f64 = torch.float32, torch.float64
        self.delta = torch.empty((T, LA), dtype=f32, device=dev)
        self.rblk = torch.empty((T, R * self.nblk), dtype=f64, device=dev)
        self.phi = torch.empty((T, R * self.nblk), dtype=f32, device=dev)
        self.mref = torch.empty((T, R), dtype=f64, device=dev)
        self.alpha = torch.empty((R, T, 2, L), dtype=f32, device=dev)
        self.logc = torch.empty((R, T), dtype=f64, device=dev)
        self._P = torch.empty((T, LA), dtype=f32, device=dev)
        # as DeviceEM: P as its exact bf16 planes between the backward and the statistics.
        # The gate here is the stacked width R L, a lone restart's is L, so near the 2 GiB
        # plane bound a batch can take the f32-P path where the lone restart takes the
        # planes.  The two paths give y_w bit for bit (the planes are the exact split of
        # the same f32 P that k_ptb3 splits in-kernel) and t_w to ~1e-8 (f32 group sums over
        # different time groupings; test_backward_planes_bit_identical,
        # test_suffstats_vs_numpy), inside the restart-equivalence bar of 1e-6
        # (tests/test_gpu_restarts.py).  PLANES is off by default in both engines.
        self.use_planes = bool(self.PLANES and spikes.ybt is not None and planes_ok(T, LA))
        self.Pq = torch.empty((3, T, LA), dtype=torch.int16, device=dev) if self.use_planes else None
        self._p_fresh = 'f32'
        self.tuning64 = torch.empty((LA, N), dtype=f64, device=dev)
        self.tuning32 = torch.empty((LA, N), dtype=f32, device=dev)
        self.yw = torch.empty((LA, N), dtype=f64, device=dev)
        self.tw = torch.empty(LA, dtype=f64, device=dev)
        self.ws_em = torch.zeros(int(self.lib.pmg_emission_workspace_size(T, LA, N)), dtype=torch.uint8, device=dev)
        self._em_flag = _flag_view(self.lib, self.ws_em, T, LA, N)
        fb = int(self.lib.pmg_fwdbwd_batched_workspace_size(T, L, min(self.C, self.Cb), R))
        if fb == 0:
            raise nat.NativeError(f"n_latent_bin={L} unsupported by the scan kernels (max 1024)")
        self.ws_fb = torch.zeros(fb, dtype=torch.uint8, device=dev)    # zero-filled once (include/pmg.h)
        self.slab = (fb // R) & ~255 if R > 1 else fb
        ss_bytes = (max(self.lib.pmg_suffstats_bf16_workspace_size(T, LA, N),
                        self.lib.pmg_suffstats_bf16x3_workspace_size(T, LA, N) if self.use_planes else 0)
                    if spikes.ybt is not None
                    else self.lib.pmg_suffstats_workspace_size(T, LA, spikes.Np))
        self.ws_ss = torch.empty(int(ss_bytes), dtype=torch.uint8, device=dev)
        self.ws_ad = AdamWorkspace(self.lib, self.dev)
        self.warm = [int(self.scan.warmup), int(self.scan.warmup)]
        self.timer = None
        self._tr_c = None
        self.ma_latent = None

    _t = DeviceEM._t
    _seg_bits = DeviceEM._seg_bits
    _tw_bits = DeviceEM._tw_bits
    PLANES = False
    P = DeviceEM.P

    def set_transition(self, tr):
        if isinstance(tr, DenseTransition):
            raise NotImplementedError("batched restarts run the banded scans only")
        DeviceEM.set_transition(self, tr)

    def set_ma_latent(self, ma_latent):
        if ma_latent is None:
            self.ma_latent = None
            return
        m = np.asarray(ma_latent)
        if m.shape != (self.L,):
            raise ValueError(f"ma_latent must have shape ({self.L},)")
        self.ma_latent = None if np.all(m != 0) else torch.as_tensor(
            np.tile((m != 0).astype(np.uint8), self.R), device=self.dev)

    def set_log_posterior(self, log_posts):
        """P[:, r L:(r+1) L] = exp(log_posts[r]) for the first M-step; log_posts (R, T, L)."""
        lp = torch.as_tensor(np.ascontiguousarray(log_posts, dtype=np.float32), device=self.dev)
        if tuple(lp.shape) != (self.R, self.T, self.L):
            raise ValueError(f"log_posteriors must be {(self.R, self.T, self.L)}")
        stacked = lp.permute(1, 0, 2).contiguous()       # (T, R, L) = the stacked layout
        nat.check(self.lib.pmg_exp(nat.ptr(stacked), stacked.numel(), nat.ptr(self._P), nat.stream_handle()),
                  "pmg_exp")
        self._p_fresh = 'f32'

    # ------------------------------------------------------------------ M-step
    def m_step(self, W, mu, nu, count, cfg: AdamConfig, stats_out, lh_out, eh_out):
        """W, mu, nu (R, NB, N) f64, count (R,) int64; stats_out (R, 4), lh/eh (R, maxiter)."""
        sh = nat.stream_handle()
        T, LA, N = self.T, self.R * self.L, self.N
        with self._t('suffstats'):
            if self._p_fresh == 'planes':
                nat.check(self.lib.pmg_suffstats_bf16x3(nat.ptr(self.Pq), LA, nat.ptr(self.sp.ybt), T, self.sp.Tp,
                                                        LA, N, self.sp.Np, nat.ptr(self.yw), nat.ptr(self.tw),
                                                        nat.ptr(self.ws_ss), self.ws_ss.numel(), sh),
                          "pmg_suffstats_bf16x3")
            elif self.sp.ybt is not None:
                nat.check(self.lib.pmg_suffstats_bf16(nat.ptr(self.P), nat.ptr(self.sp.ybt), T, self.sp.Tp, LA, N,
                                                      self.sp.Np, nat.ptr(self.yw), nat.ptr(self.tw),
                                                      nat.ptr(self.ws_ss), self.ws_ss.numel(), sh),
                          "pmg_suffstats_bf16")
            else:
                nat.check(self.lib.pmg_suffstats(nat.ptr(self.P), nat.ptr(self.sp.yext), T, LA, N, self.sp.Np,
                                                 nat.ptr(self.yw), nat.ptr(self.tw), nat.ptr(self.ws_ss),
                                                 self.ws_ss.numel(), sh), "pmg_suffstats")
        L, NB, R = self.L, self.NB, self.R
        batched = (L <= DeviceEM.PERSISTENT_MAX_L and NB <= DeviceEM.PERSISTENT_MAX_NB
                   and bool(self.lib.pmg_mstep_adam_batched_supported(L, NB, N, R)))
        tiled = not batched and (L > DeviceEM.PERSISTENT_MAX_L or NB > DeviceEM.PERSISTENT_MAX_NB
                                 or not self.lib.pmg_mstep_adam_supported(L, NB, N))
        if batched:
            need = int(self.lib.pmg_mstep_batched_workspace_size(L, NB, N, R, int(cfg.maxiter)))
        else:
            need = int(self.lib.pmg_mstep_tiled_workspace_size(L, NB, N) if tiled
                       else self.lib.pmg_mstep_workspace_size(N, int(cfg.maxiter)))
        ws = self.ws_ad.get(need, tiled)
        c = cfg.to_c()
        if batched:     # several restarts per persistent launch, each its own loop and stop rule
            with self._t('mstep_adam'):
                nat.check(self.lib.pmg_mstep_adam_batched(
                    nat.ptr(W), nat.ptr(mu), nat.ptr(nu), nat.ptr(count), nat.ptr(self.basis), nat.ptr(self.yw),
                    nat.ptr(self.tw), L, NB, N, R, ctypes.byref(c), nat.ptr(stats_out), nat.ptr(lh_out),
                    nat.ptr(eh_out), nat.ptr(ws), ws.numel(), sh), "pmg_mstep_adam_batched")
            return
        fn = self.lib.pmg_mstep_adam_tiled if tiled else self.lib.pmg_mstep_adam
        with self._t('mstep_adam'):
            for r in range(self.R):
                nat.check(fn(nat.ptr(W[r]), nat.ptr(mu[r]), nat.ptr(nu[r]), nat.ptr(count[r:r + 1]),
                             nat.ptr(self.basis), nat.ptr(self.yw[r * L:(r + 1) * L]),
                             nat.ptr(self.tw[r * L:(r + 1) * L]), L, NB, N, ctypes.byref(c),
                             nat.ptr(stats_out[r]), nat.ptr(lh_out[r]), nat.ptr(eh_out[r]),
                             nat.ptr(ws), ws.numel(), sh),
                          "pmg_mstep_adam_tiled" if tiled else "pmg_mstep_adam")

    def compute_tuning(self, W):
        with self._t('tuning_softplus'):
            nat.check(self.lib.pmg_tuning_softplus_batched(nat.ptr(self.basis), nat.ptr(W), self.L, self.NB, self.N,
                                                           self.R, nat.ptr(self.tuning64), nat.ptr(self.tuning32),
                                                           nat.stream_handle()), "pmg_tuning_softplus_batched")

    # ------------------------------------------------------------------ E-step
    def emission(self, likelihood_scale=1.0):
        sp, sh = self.sp, nat.stream_handle()
        T, LA, N = self.T, self.R * self.L, self.N
        with self._t('emission'):
            if sp.int_path:
                ma1 = sp.ma if (sp.ma is not None and not sp.ma_2d) else None
                nat.check(self.lib.pmg_emission_poisson(nat.ptr(sp.yq), nat.ptr(sp.gconst), nat.ptr(self.tuning64),
                                                        nat.ptr(ma1), nat.ptr(self.ma_latent), 1.0, T, LA, N, sp.Kp,
                                                        nat.ptr(self.delta), nat.ptr(self.rblk), None, nat.ptr(self.ws_em),
                                                        self.ws_em.numel(), sh), "pmg_emission_poisson")
            else:
                nat.check(self.lib.pmg_emission_poisson_f64(nat.ptr(sp.y), nat.ptr(sp.gconst), nat.ptr(self.tuning64),
                                                            nat.ptr(sp.ma), int(sp.ma_2d), nat.ptr(self.ma_latent),
                                                            1.0, T, LA, N, nat.ptr(self.delta), nat.ptr(self.rblk),
                                                            None, nat.ptr(self.ws_em), self.ws_em.numel(), sh),
                          "pmg_emission_poisson_f64")
        with self._t('emission_rowref'):
            nat.check(self.lib.pmg_emission_rowref_batched(nat.ptr(self.rblk), T, self.R * self.nblk, self.R,
                                                           float(likelihood_scale), nat.ptr(self.phi),
                                                           nat.ptr(self.mref), sh), "pmg_emission_rowref_batched")

    def forward(self, likelihood_scale, logz_out, keep_alpha=True):
        """logz_out: (R,) f64 device tensor."""
        bits = (0 if keep_alpha else nat.PHASE_NO_JUMP_ROWS) | (nat.PHASE_ADAPTIVE_WARMUP if self.scan.device_adaptive
                                                                  else 0)   # RestartBatchEM: always one fit
        args = (nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.mref), self.T, self.R,
                ctypes.byref(self._tr_c), float(likelihood_scale), self.C, int(self.warm[0]), float(self.scan.tol),
                nat.ptr(self.alpha), nat.ptr(self.logc), nat.ptr(logz_out), nat.ptr(self.ws_fb),
                self.ws_fb.numel(), nat.stream_handle())
        with self._t('forward_filter'):
            nat.check(self.lib.pmg_forward_filter_batched(*args, 1 | bits | self._tw_bits()), "pmg_forward_filter_batched")
        with self._t('forward_repair'):
            nat.check(self.lib.pmg_forward_filter_batched(*args, 2 | bits | self._seg_bits()),
                      "pmg_forward_filter_batched")

    def backward(self, likelihood_scale, gamma=None):
        """gamma: optional (R, T, 2, L) f32 posterior output."""
        planes = self.use_planes
        args = (nat.ptr(self.delta), nat.ptr(self.phi), nat.ptr(self.alpha), self.T, self.R,
                ctypes.byref(self._tr_c), float(likelihood_scale), self.Cb, int(self.warm[1]), float(self.scan.tol),
                nat.ptr(self.Pq) if planes else nat.ptr(self._P), nat.ptr(gamma), nat.ptr(self.ws_fb),
                self.ws_fb.numel(), nat.stream_handle())
        ad = (nat.PHASE_ADAPTIVE_WARMUP if self.scan.device_adaptive else 0) | (nat.PHASE_P_BF16X3 if planes else 0)
        self._p_fresh = 'planes' if planes else 'f32'
        with self._t('backward_smoother'):
            nat.check(self.lib.pmg_backward_smoother_batched(*args, 1 | ad | self._tw_bits()), "pmg_backward_smoother_batched")
        with self._t('backward_repair'):
            nat.check(self.lib.pmg_backward_smoother_batched(*args, 2 | ad | self._seg_bits()),
                      "pmg_backward_smoother_batched")

    def e_step(self, likelihood_scale, logz_out, gamma=None):
        self.emission(likelihood_scale)
        self.forward(likelihood_scale, logz_out, keep_alpha=gamma is not None)
        self.backward(likelihood_scale, gamma)

    def emission_status(self):
        _check_emission_flag(self._em_flag)

    def ctl_words(self, r):
        """Restart r's scan control words (device view)."""
        return self.ws_fb[r * self.slab:r * self.slab + 4 * nat.CTL_WORDS].view(torch.int32)

    def reset_adaptive(self):
        """Start of a fit: forget earlier adaptive warm-up decisions (every restart)."""
        for r in range(self.R):
            w = self.ctl_words(r)
            w[nat.CTL_FWD + nat.CTL_WARM] = 0
            w[nat.CTL_BWD + nat.CTL_WARM] = 0

    def repairs(self):
        """[(forward, backward) chunks recomputed] per restart (device read: syncs)."""
        out = []
        for r in range(self.R):
            words = self.ctl_words(r)
            w = words.cpu().numpy()
            _raise_on_timeout(words, w, f"scan relaxation (restart {r})")
            out.append((int(w[nat.CTL_FWD + nat.CTL_REPAIRS]), int(w[nat.CTL_BWD + nat.CTL_REPAIRS])))
        return out
