"""PoissonGPLVMJump1D on MI355X: the reference's public API over the native engine.

Mirrors poor_man_gplvm.core (reference core.py:376-849): the constructor
(:381-420), fit_em (:829-849 -> :592-713), decode_latent (:454-497),
m_step (:802-827), _decode_latent (:777-786), get_tuning (:772-774),
init_latent_posterior (:571-583), sample / sample_latent / sample_y
(:526-569, :795-800), predict_expected_rate (:716-733) -- same argument names,
defaults and returned dict keys.  Differences that cannot be avoided without JAX:
  * random draws (W init, posterior init, sampling) use numpy's PCG64 instead of
    jax threefry; ``key`` may be an int, a numpy Generator or any array (hashed);
  * arrays come back as numpy (the reference mixes jax and numpy arrays);
  * log-space posteriors are log of the fp32 probabilities (-inf where a state's
    probability underflows; the reference keeps very negative finite logs there);
  * ``n_time_per_chunk`` is accepted and ignored (the reference uses it only to
    bound XLA memory; the math does not depend on it, decoder.py:258-332);
  * pynapple TsdFrame inputs are accepted when pynapple is importable.
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch

from . import _native as nat
from .engine import (AdamConfig, DeviceEM, RestartBatchEM, ScanConfig, SpikeData, default_device, log_of,
                     posterior_outputs)
from .gp_kernel import (DenseTransition, banded_transition, create_transition_prob_1d, dense_transition,
                        generate_basis, make_transition, transition_from_log_kernels)

try:  # optional, as in the reference's TsdFrame handling
    import pynapple as nap  # type: ignore
except Exception:  # pragma: no cover - pynapple is not installed in this image
    nap = None


def _is_tsd(y):
    return nap is not None and isinstance(y, nap.TsdFrame)


def _rng(key):
    if isinstance(key, np.random.Generator):
        return key
    if key is None:
        return np.random.default_rng(0)
    if isinstance(key, (int, np.integer)):
        return np.random.default_rng(int(key))
    a = np.ascontiguousarray(np.asarray(key))
    return np.random.default_rng(zlib.crc32(a.tobytes()))


def _np(t):
    return t.detach().cpu().numpy()


_NP_DTYPE = {torch.float32: np.float32, torch.float64: np.float64, torch.int64: np.int64,
             torch.int32: np.int32}


class _PinnedCopies:
    """Device -> host copies of the arrays a fit returns, into page-locked buffers
    (`_native.host_array`: PCIe DMA at full rate instead of the staged pageable path),
    issued without a host sync.  The large buffers are reserved up front on a helper
    thread (the allocation is a C call that holds no Python lock, so it runs while the
    host enqueues the EM iterations); copies of intermediate results (the save_every
    snapshots) run on a side stream beside the remaining iterations.  finish()
    synchronises and returns; the buffers are the numpy arrays handed to the caller."""

    # page-locked bytes reserved ahead of the loop for snapshots; further snapshots get
    # their buffer when they are submitted (a small save_every must not pin n_iter copies
    # of (T, 2, L) up front)
    RESERVE_BYTES = 2 << 30

    def __init__(self, dev):
        from concurrent.futures import ThreadPoolExecutor
        self.dev = dev
        self.side = torch.cuda.Stream(dev)
        self.items = []
        self.reserved = {}
        self.pool = ThreadPoolExecutor(max_workers=1)

    def reserve_upto(self, key, shape, count, dtype=torch.float32):
        """reserve() up to `count` buffers, within RESERVE_BYTES."""
        nbytes = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
        for _ in range(min(int(count), max(1, self.RESERVE_BYTES // max(nbytes, 1)))):
            self.reserve(key, shape, dtype)

    def reserve(self, key, shape, dtype=torch.float32):
        """Start allocating a host buffer for a later submit(..., key=key)."""
        self.reserved.setdefault(key, []).append(
            self.pool.submit(nat.host_array, tuple(shape), _NP_DTYPE[dtype]))

    def submit(self, t, key=None, side=False):
        """Copy device tensor t (not written again before finish) to a pinned buffer.
        The caller may drop t at once: a side-stream copy records its use on the side
        stream, so the caching allocator frees the memory only after the copy (same-stream
        copies are ordered before any later use of the memory anyway)."""
        t = t.contiguous()
        cur = torch.cuda.current_stream(self.dev)
        if side:
            self.side.wait_stream(cur)
            t.record_stream(self.side)
        st = self.side if side else cur
        nbytes = t.numel() * t.element_size()
        q = self.reserved.get(key)
        host = q.pop(0).result() if q else nat.host_array(tuple(t.shape), _NP_DTYPE[t.dtype])
        if host.shape != tuple(t.shape) or host.dtype != _NP_DTYPE[t.dtype]:
            raise ValueError("reserved host buffer does not match the tensor")
        if nbytes:   # an empty tensor (e.g. run_em(n_iter=0)'s histories) has nothing to copy
            nat.check(nat.load().pmg_copy_d2h(host.ctypes.data, t.data_ptr(), nbytes, st.cuda_stream),
                      "pmg_copy_d2h")
        self.items.append(host)
        return host

    def finish(self):
        torch.cuda.current_stream(self.dev).synchronize()
        self.side.synchronize()
        self.pool.shutdown(wait=False)
        return self.items


class PoissonGPLVMJump1D:
    """Poisson GPLVM with a smooth 1-d latent and jump dynamics (core.py:746)."""

    def __init__(self, n_neuron, n_latent_bin=100, tuning_lengthscale=1., param_prior_std=1.,
                 movement_variance=1., explained_variance_threshold_basis=0.999, rng_init_int=123,
                 w_init_variance=1., w_init_mean=0., p_move_to_jump=0.01, p_jump_to_move=0.01,
                 basis_type='rbf', custom_tuning_kernel=None, custom_transition_kernel=None,
                 smoothness_penalty=0., scan_config: ScanConfig | None = None):
        self.n_latent_bin = int(n_latent_bin)
        self.tuning_lengthscale = tuning_lengthscale
        self.param_prior_std = param_prior_std
        self.movement_variance = movement_variance
        self.p_move_to_jump = p_move_to_jump
        self.p_jump_to_move = p_jump_to_move
        self.explained_variance_threshold_basis = explained_variance_threshold_basis
        self.rng_init_int = rng_init_int
        self.n_neuron = int(n_neuron)
        self.possible_latent_bin = np.arange(self.n_latent_bin)
        self.possible_dynamics = np.arange(2)
        self.w_init_variance = w_init_variance
        self.w_init_mean = w_init_mean
        self.custom_transition_kernel = custom_transition_kernel
        self.basis_type = basis_type
        self.tuning_basis = generate_basis(tuning_lengthscale, self.n_latent_bin,
                                           explained_variance_threshold_basis, include_bias=True,
                                           basis_type=basis_type, custom_kernel=custom_tuning_kernel)
        self.n_basis = self.tuning_basis.shape[1]
        self.smoothness_penalty = smoothness_penalty
        self.ma_neuron_default = np.ones(self.n_neuron)
        self.ma_latent_default = np.ones(self.n_latent_bin)
        self.scan_config = scan_config or ScanConfig()
        self.adam_runner = None          # kept for attribute parity (core.py:841)
        self.opt_state_init_fun = None
        self.initialize_params(_rng(rng_init_int))

    # ------------------------------------------------------------------ params
    def initialize_params(self, key):
        """core.py:429-437 (numpy RNG)."""
        rng = _rng(key)
        W = rng.normal(size=(self.n_basis, self.n_neuron)) * math.sqrt(self.w_init_variance) + self.w_init_mean
        self.params = W.astype(np.float32)
        self._tuning = None   # softplus(basis @ W), computed on the device on first use
        return self.params, self.tuning if torch.cuda.is_available() else None

    @property
    def tuning(self):
        """(n_latent_bin, n_neuron) tuning curves (core.py:434, lazily on the device)."""
        if self._tuning is None:
            self._tuning = self.get_tuning(self.params, {}, self.tuning_basis)
        return self._tuning

    @tuning.setter
    def tuning(self, value):
        self._tuning = None if value is None else np.asarray(value, np.float32)

    def get_tuning(self, params, hyperparam, tuning_basis):
        """fit_tuning_helper.get_tuning_softplus (fit_tuning_helper.py:19-25), on device."""
        B = np.asarray(tuning_basis, np.float32)
        W = np.asarray(params, np.float64)
        dev = default_device()
        lib = nat.load()
        bt = torch.as_tensor(np.ascontiguousarray(B), device=dev)
        wt = torch.as_tensor(np.ascontiguousarray(W), device=dev)
        out = torch.empty((B.shape[0], W.shape[1]), dtype=torch.float32, device=dev)
        nat.check(lib.pmg_tuning_softplus(nat.ptr(bt), nat.ptr(wt), B.shape[0], B.shape[1], W.shape[1],
                                          None, nat.ptr(out), nat.stream_handle()), "pmg_tuning_softplus")
        return _np(out)

    def init_latent_posterior(self, T, key, random_scale=0.1):
        """core.py:571-583: U(0,1)*scale, row-normalised, log (numpy RNG)."""
        u = _rng(key).random((T, self.n_latent_bin))
        post = u * random_scale
        post = post / post.sum(axis=1, keepdims=True)
        with np.errstate(divide='ignore'):
            lp = np.log(post)
        lp = np.where(lp == -np.inf, -1e40, lp)
        return lp.astype(np.float32), post.astype(np.float32)

    # ------------------------------------------------------------------ transitions
    def _transition(self, movement_variance, p_move_to_jump, p_jump_to_move):
        """gp_kernel.py:42-89 in device form: the banded linear-space scans when the
        continuous kernel is a <= 32-bin RBF band, else the dense log-domain scans
        (custom_transition_kernel, wide movement_variance)."""
        return make_transition(self.n_latent_bin, movement_variance, p_move_to_jump, p_jump_to_move,
                               custom_kernel=self.custom_transition_kernel)

    # ------------------------------------------------------------------ M-step
    def m_step(self, param_curr, y, log_posterior_curr, tuning_basis, hyperparam, opt_state_curr=None):
        """core.py:802-827: sufficient statistics + Adam (one device launch each).
        opt_state_curr: dict(mu, nu, count) as returned in the result (None = fresh)."""
        hp = dict(hyperparam)
        y = np.asarray(y)
        sp = SpikeData(y, None)
        B = np.asarray(tuning_basis, np.float32)
        eng = DeviceEM(sp, B.shape[0], basis=B, scan=self.scan_config)
        eng.set_log_posterior(log_posterior_curr)
        cfg = AdamConfig(lr=getattr(self, '_m_step_step_size', 0.01),
                         maxiter=getattr(self, '_m_step_maxiter', 1000),
                         tol=getattr(self, '_m_step_tol', 1e-6),
                         prior_std=hp.get('param_prior_std', self.param_prior_std))
        dev = eng.dev
        W = torch.as_tensor(np.asarray(param_curr, np.float64), device=dev).contiguous()
        st = opt_state_curr or {'mu': np.zeros(W.shape), 'nu': np.zeros(W.shape), 'count': 0}
        mu = torch.as_tensor(np.asarray(st['mu'], np.float64), device=dev).contiguous()
        nu = torch.as_tensor(np.asarray(st['nu'], np.float64), device=dev).contiguous()
        cnt = torch.tensor([int(st['count'])], dtype=torch.int64, device=dev)
        stats = torch.zeros(4, dtype=torch.float64, device=dev)
        lh = torch.zeros(max(cfg.maxiter, 1), dtype=torch.float64, device=dev)
        eh = torch.zeros_like(lh)
        eng.m_step(W, mu, nu, cnt, cfg, stats, lh, eh)
        s = _np(stats)
        n = int(s[0])
        return {'params': _np(W).astype(np.float32),
                'opt_state': {'mu': _np(mu), 'nu': _np(nu), 'count': int(_np(cnt)[0])},
                'n_iter': n, 'final_loss': float(s[1]), 'final_error': float(s[2]),
                'loss_history': _np(lh)[:n], 'error_history': _np(eh)[:n]}

    # ------------------------------------------------------------------ E-step
    def _decode_latent(self, y, tuning, hyperparam, log_latent_transition_kernel_l,
                       log_dynamics_transition_kernel, ma_neuron, ma_latent=None, likelihood_scale=1.,
                       n_time_per_chunk=10000):
        """core.py:777-786 -> decoder.smooth_all_step_combined_ma_chunk (decoder.py:258-332).
        The scan runs with the log kernels passed in (their device form, see
        _scan_transition) and the joint's log-space outputs are assembled from them.
        Returns the reference's 6-tuple (numpy)."""
        res = self._run_decode(y, tuning, hyperparam, ma_neuron, ma_latent, likelihood_scale, joint=True,
                               logK=log_latent_transition_kernel_l, logA=log_dynamics_transition_kernel)
        return (res['log_posterior_all'], res['log_marginal_final'], res['log_causal_posterior_all'],
                res['log_one_step_predictive_marginals_all'], res['log_accumulated_joint'],
                res['log_likelihood_all'])

    def _check_latent_mask(self, tr, ma_latent):
        """Hook for models without a jump state (PoissonGPLVM1D)."""

    def _observation(self, eng, hyperparam):
        """Hook: the Gaussian model switches the engine's emission here."""

    def _scan_transition(self, mv, pmj, pjm, logK=None, logA=None, exact=None):
        """Device transition for a decode scan: this model's own (hyper-parameters), or,
        when log kernels are passed (the _decode_latent arguments), the device form of
        exactly those kernels.  Kernels equal to the model's own (1e-6) keep its
        transition bit for bit.  With scan_config.decode_exact (default) the decode runs
        the dense log-domain scans with the whole kernel (exact joint rows for every
        latent, see ScanConfig.decode_exact)."""
        tr = self._transition(mv, pmj, pjm)
        if exact is None:
            exact = bool(getattr(self.scan_config, 'decode_exact', False))
        if exact and not isinstance(tr, DenseTransition):
            tr = dense_transition(self.n_latent_bin, mv, pmj, pjm, self.custom_transition_kernel)
        if logK is None or logA is None:
            return tr
        lk = np.asarray(logK, np.float64)
        la = np.asarray(logA, np.float64)
        L = self.n_latent_bin
        if lk.shape == (2, L, L) and la.shape == (2, 2):
            _, lk_m, _, la_m = create_transition_prob_1d(L, mv, pmj, pjm, self.custom_transition_kernel)
            with np.errstate(invalid='ignore'):
                same = (np.allclose(np.exp(lk), np.exp(lk_m), rtol=1e-6, atol=1e-300)
                        and np.allclose(np.exp(la), np.exp(la_m), rtol=1e-6, atol=1e-12))
            if same:
                return tr
        return transition_from_log_kernels(lk, la, force_dense=exact or isinstance(tr, DenseTransition))

    def _run_decode(self, y, tuning, hyperparam, ma_neuron, ma_latent, likelihood_scale, joint=True,
                    logK=None, logA=None):
        eng = self._decode_engine(y, tuning, hyperparam, ma_neuron, ma_latent, logK, logA)
        return self._decode_on(eng, hyperparam, ma_latent, likelihood_scale, joint, logK, logA)

    def _decode_engine(self, y, tuning, hyperparam, ma_neuron, ma_latent, logK=None, logA=None, exact=None):
        """Device state of a decode: spikes uploaded and prepared, transition, masks and
        tuning set (reusable across decodes of spike trains of the same shape).  exact:
        the dense log-domain scans (None: ScanConfig.decode_exact)."""
        mv = hyperparam.get('movement_variance', self.movement_variance)
        pmj = hyperparam.get('p_move_to_jump', self.p_move_to_jump)
        pjm = hyperparam.get('p_jump_to_move', self.p_jump_to_move)
        ma = None if ma_neuron is None else np.asarray(ma_neuron, np.float32)
        tr = self._scan_transition(mv, pmj, pjm, logK, logA, exact)
        self._check_latent_mask(tr, ma_latent)
        sp = SpikeData(y if isinstance(y, torch.Tensor) else np.asarray(y), ma)
        eng = DeviceEM(sp, self.n_latent_bin, scan=self.scan_config)
        self._observation(eng, hyperparam)
        eng.set_transition(tr)
        eng.set_ma_latent(ma_latent)
        eng.set_tuning(np.asarray(tuning))
        return eng

    def _decode_on(self, eng, hyperparam, ma_latent, likelihood_scale, joint=True, logK=None, logA=None):
        """One smoother pass (emission, forward, backward, joint) over eng's current spikes."""
        mv = hyperparam.get('movement_variance', self.movement_variance)
        pmj = hyperparam.get('p_move_to_jump', self.p_move_to_jump)
        pjm = hyperparam.get('p_jump_to_move', self.p_jump_to_move)
        dev = eng.dev
        T, L = eng.T, self.n_latent_bin
        # the (T, 2, L) / (T, L) results go to page-locked host buffers, allocated on a
        # helper thread while the device runs the scans (as run_em's)
        cp = _PinnedCopies(dev)
        for key, shape in (('lpost', (T, 2, L)), ('lcaus', (T, 2, L)), ('gamma', (T, 2, L)), ('ll', (T, L)),
                           ('plm', (T, L))):
            cp.reserve(key, shape)
        logz = torch.zeros(1, dtype=torch.float64, device=dev)
        gamma = torch.empty((T, 2, L), dtype=torch.float32, device=dev)
        rho = (torch.zeros((T, 2, L), dtype=torch.float64 if eng.dense else torch.float32, device=dev)
               if joint else None)
        lgam = torch.empty((T, 2, L), dtype=torch.float32, device=dev) if eng.dense else None
        eng.e_step(likelihood_scale, logz, gamma=gamma, rho=rho, log_gamma=lgam)
        eng.check_status()
        ml = None if ma_latent is None else np.asarray(ma_latent).astype(bool)
        # the log-domain scans hold the exact log posteriors (f64 causal ones, cast on the device)
        lg, plm, pdm = posterior_outputs(gamma, log=not eng.dense)
        h_lpost = cp.submit(lgam if eng.dense else lg, key='lpost')
        h_lcaus = cp.submit(eng.log_alpha.to(torch.float32) if eng.dense else log_of(eng.alpha), key='lcaus')
        h_gamma = cp.submit(gamma, key='gamma')
        h_plm = cp.submit(plm, key='plm')
        h_pdm = cp.submit(pdm)
        h_logc = cp.submit(eng.logc.to(torch.float32))
        h_ll = cp.submit(eng.loglik(), key='ll')
        h_lz = cp.submit(logz)
        if joint:
            h_S = cp.submit(eng.joint_log(rho) if eng.dense else eng.joint(rho))
        cp.finish()
        out = {
            'log_posterior_all': _masked_log(h_lpost, ml),
            'log_marginal_final': float(h_lz[0]),
            'posterior_all': h_gamma,
            'log_causal_posterior_all': _masked_log(h_lcaus, ml),
            'log_one_step_predictive_marginals_all': h_logc,
            'log_likelihood_all': h_ll,
            '_posterior_latent_marg': h_plm,      # sums over d / l formed on the device
            '_posterior_dynamics_marg': h_pdm,
        }
        if joint:
            if logK is None or logA is None:
                _, logK, _, logA = create_transition_prob_1d(L, mv, pmj, pjm, self.custom_transition_kernel)
            logK = np.asarray(logK, np.float64)
            logA = np.asarray(logA, np.float64)
            if eng.dense:   # rho holds log(rho): the joint is accumulated in log space
                logS4 = h_S.reshape(2, L, 2, L).transpose(0, 2, 1, 3)
                with np.errstate(invalid='ignore'):
                    lj = np.asarray(logA, np.float64)[:, :, None, None] + logK[None] + logS4
                lj = np.where(np.isnan(lj), -np.inf, lj)
            else:
                S4 = h_S.reshape(2, L, 2, L).transpose(0, 2, 1, 3)        # [d, d', i, j]
                lj = log_joint_from_counts(S4, logK, logA, ml)
            out['log_accumulated_joint'] = lj
        return out

    # ------------------------------------------------------------------ decode
    def decode_latent(self, y, tuning=None, hyperparam={}, ma_neuron=None, ma_latent=None,
                      likelihood_scale=1., n_time_per_chunk=10000, t_l=None):
        """core.py:454-497 (+ decoder.compute_transition_posterior_prob, decoder.py:334-375)."""
        if _is_tsd(y):
            t_l = y.t
            y = y.d
        if tuning is None:
            tuning = self.tuning
        if ma_neuron is None:
            ma_neuron = self.ma_neuron_default
        if ma_latent is None:
            ma_latent = self.ma_latent_default
        hp, logK, logA = self._dynamics_decode_args(hyperparam)
        r = self._run_decode(y, tuning, hp, ma_neuron, ma_latent, likelihood_scale, joint=True, logK=logK,
                             logA=logA)
        return self._decode_result(r, t_l)

    def _decode_hp(self, hyperparam):
        """Hook: the hyper-parameters a public decode call adds (the Gaussian model's noise_std)."""
        return dict(hyperparam)

    def _dynamics_decode_args(self, hyperparam):
        """Hook: (hyperparam, logK, logA) of decode_latent's smoother; None kernels = the
        model's own transition for these hyper-parameters."""
        return dict(hyperparam), None, None

    def decode_marginals(self, y, tuning=None, hyperparam={}, ma_neuron=None, ma_latent=None,
                         likelihood_scale=1.):
        """The part of decode_latent that model evaluation reads (model_selection_helper.py:
        89-97): log_marginal_final, log_one_step_predictive_marginals_all and
        posterior_dynamics_marg, from the banded linear-space scans without the pairwise
        joint (the dense log-domain scans of ScanConfig.decode_exact only matter for the
        transition rows of latents the posterior never visits).  The same values as
        decode_latent's within the scans' 1e-5 parity bar; not part of the reference API."""
        if _is_tsd(y):
            y = y.d
        tuning = self.tuning if tuning is None else tuning
        ma_neuron = self.ma_neuron_default if ma_neuron is None else ma_neuron
        ma_latent = self.ma_latent_default if ma_latent is None else ma_latent
        hp, logK, logA = self._dynamics_decode_args(hyperparam)
        eng = self._decode_engine(y, tuning, hp, ma_neuron, ma_latent, logK, logA, exact=False)
        logz = torch.zeros(1, dtype=torch.float64, device=eng.dev)
        gamma = torch.empty((eng.T, 2, self.n_latent_bin), dtype=torch.float32, device=eng.dev)
        lgam = torch.empty_like(gamma) if eng.dense else None
        eng.e_step(likelihood_scale, logz, gamma=gamma, log_gamma=lgam)
        eng.check_status()
        return {'log_marginal_final': float(_np(logz)[0]),
                'log_one_step_predictive_marginals_all': _np(eng.logc).astype(np.float32),
                'posterior_dynamics_marg': _np(posterior_outputs(gamma, log=False)[2])}

    def _decode_result(self, r, t_l=None):
        """decode_latent's returned dict from a _decode_on result (core.py:477-497)."""
        posterior_all = r['posterior_all']
        plm = r['_posterior_latent_marg'] if '_posterior_latent_marg' in r else posterior_all.sum(axis=1)
        pdm = r['_posterior_dynamics_marg'] if '_posterior_dynamics_marg' in r else posterior_all.sum(axis=2)
        if t_l is not None and nap is not None:
            plm = nap.TsdFrame(d=plm, t=t_l)
            pdm = nap.TsdFrame(d=pdm, t=t_l)
        res = {'log_posterior_all': r['log_posterior_all'],
               'log_marginal_final': r['log_marginal_final'],
               'posterior_all': posterior_all,
               'posterior_latent_marg': plm,
               'posterior_dynamics_marg': pdm,
               'log_one_step_predictive_marginals_all': r['log_one_step_predictive_marginals_all'],
               'log_likelihood_all': r['log_likelihood_all']}
        res.update(compute_transition_posterior_prob(r['log_accumulated_joint']))
        return res

    def decode_latent_naive_bayes(self, y, tuning=None, hyperparam={}, ma_neuron=None, ma_latent=None,
                                  likelihood_scale=1., n_time_per_chunk=10000, dt_l=1., t_l=None):
        """core.py:788-792 -> core.py:499-524 -> decoder.get_naive_bayes_ma_chunk
        (decoder.py:106-149): per-time-bin posterior without temporal prior.
        A constant dt uses the exact int8 emission; a per-time dt_l the f64 per-bin
        kernel (pmg_emission_poisson_dt); the logsumexp normalisation is
        pmg_naive_bayes_normalize.  likelihood_scale and n_time_per_chunk are accepted
        and unused, as in the reference."""
        if _is_tsd(y):
            t_l = y.t
            y = y.d
        if tuning is None:
            tuning = self.tuning
        if ma_neuron is None:
            ma_neuron = self.ma_neuron_default
        if ma_latent is None:
            ma_latent = self.ma_latent_default
        eng = self._nb_engine(y, tuning, hyperparam, ma_neuron, ma_latent)
        return self._nb_on(eng, dt_l, t_l)

    def _nb_engine(self, y, tuning, hyperparam, ma_neuron, ma_latent):
        """Device state of a naive-Bayes decode (spikes, masks, tuning; no transition)."""
        ma = None if ma_neuron is None else np.asarray(ma_neuron, np.float32)
        sp = SpikeData(y if isinstance(y, torch.Tensor) else np.asarray(y), ma)
        eng = DeviceEM(sp, self.n_latent_bin, scan=self.scan_config)
        self._observation(eng, hyperparam)
        eng.set_ma_latent(ma_latent)
        eng.set_tuning(np.asarray(tuning))
        return eng

    def _nb_on(self, eng, dt_l, t_l=None, n_split=1):
        """decode_latent_naive_bayes over eng's current spikes.  n_split > 1: the spikes
        are n_split equal-length recordings stacked in time (the batched shuffles of
        test.shuffle_and_decode); dt_l is one recording's and a list of per-recording
        result dicts is returned.  Every output row depends on its own time bin only, so
        each dict equals the decode of that recording alone bit for bit."""
        sp = eng.sp
        T = sp.T
        if n_split > 1:
            if T % n_split:
                raise ValueError("stacked recordings must have equal length")
            dt = np.tile(np.broadcast_to(np.asarray(dt_l, np.float64), (T // n_split,)), n_split)
        else:
            dt = np.broadcast_to(np.asarray(dt_l, np.float64), (T,))
        dev, L = eng.dev, self.n_latent_bin
        lib, sh = eng.lib, nat.stream_handle()
        if np.all(dt == dt[0]):
            eng._emission_call(sp, sh, float(dt[0]))
        elif eng.noise_std is not None:
            dtt = torch.as_tensor(np.array(dt, dtype=np.float64), device=dev)
            nat.check(lib.pmg_emission_gaussian_dt(nat.ptr(sp.y), nat.ptr(eng.tuning64), nat.ptr(sp.ma),
                                                   int(sp.ma_2d), nat.ptr(eng.ma_latent), float(eng.noise_std),
                                                   nat.ptr(dtt), T, L, sp.N, nat.ptr(eng.delta), nat.ptr(eng.rblk),
                                                   sh), "pmg_emission_gaussian_dt")
        else:
            dtt = torch.as_tensor(np.array(dt, dtype=np.float64), device=dev)
            nat.check(lib.pmg_emission_poisson_dt(nat.ptr(sp.y), nat.ptr(sp.gconst), nat.ptr(eng.tuning64),
                                                  nat.ptr(sp.ma), int(sp.ma_2d), nat.ptr(eng.ma_latent),
                                                  nat.ptr(dtt), T, L, sp.N, nat.ptr(eng.delta), nat.ptr(eng.rblk),
                                                  sh), "pmg_emission_poisson_dt")
        log_post = torch.empty((T, L), dtype=torch.float32, device=dev)
        lml = torch.empty(T, dtype=torch.float64, device=dev)
        nat.check(lib.pmg_naive_bayes_normalize(nat.ptr(eng.delta), nat.ptr(eng.rblk), T, L, nat.ptr(log_post),
                                                nat.ptr(lml), sh), "pmg_naive_bayes_normalize")
        if eng.noise_std is None:
            eng.emission_status()
        lp = _np(log_post)
        pl = np.exp(lp)       # host exp: cheaper than a second (T, L) device-to-host copy
        lml_h = _np(lml)
        ll = _np(eng.loglik())
        if n_split > 1:
            Ts = T // n_split
            return [_nb_dict(lp[r * Ts:(r + 1) * Ts], pl[r * Ts:(r + 1) * Ts], lml_h[r * Ts:(r + 1) * Ts],
                             ll[r * Ts:(r + 1) * Ts], t_l) for r in range(n_split)]
        return _nb_dict(lp, pl, lml_h, ll, t_l)

    def log_marginal_masked(self, y, ma_latent_l, tuning=None, hyperparam={}, ma_neuron=None,
                            likelihood_scale=1.):
        """log_marginal_final of decode_latent(y, ma_latent=m) for every mask m in
        ma_latent_l ((R, L) or a list), as an (R,) float64 array.

        This is the inner loop of model_selection_helper.get_downsampled_lml
        (model_selection_helper.py:243-260), which reads nothing from each decode
        but log_marginal_final.  So the spikes are uploaded once, the transition and
        tuning are set once, the emission contraction runs once (unmasked), and each
        mask runs only pmg_emission_latent_mask (masked bins to -1e20, block
        references re-derived), the row reference and the forward filter (logZ is
        the filter's sum_t c_t, decoder.py:151-187).  The backward pass, the joint
        and the host copies of (T, D, L) tensors are skipped.  Every logZ stays on
        the device until one copy at the end.  With the banded scans and L % 32 == 0
        the masks run batched (DeviceEM.masked_logz_batched): one stacked mask
        launch, one row-reference launch and one forward launch per group of masks,
        no alpha written."""
        if _is_tsd(y):
            y = y.d
        if tuning is None:
            tuning = self.tuning
        if ma_neuron is None:
            ma_neuron = self.ma_neuron_default
        masks = np.asarray(ma_latent_l)
        if masks.ndim != 2 or masks.shape[1] != self.n_latent_bin:
            raise ValueError(f"ma_latent_l must have shape (R, {self.n_latent_bin})")
        if not np.all(masks.any(axis=1)):
            raise ValueError("every latent mask must keep at least one latent bin")
        mv = hyperparam.get('movement_variance', self.movement_variance)
        pmj = hyperparam.get('p_move_to_jump', self.p_move_to_jump)
        pjm = hyperparam.get('p_jump_to_move', self.p_jump_to_move)
        ma = None if ma_neuron is None else np.asarray(ma_neuron, np.float32)
        tr = self._transition(mv, pmj, pjm)
        for m in masks:
            self._check_latent_mask(tr, m)
        eng = DeviceEM(SpikeData(np.asarray(y), ma), self.n_latent_bin, scan=self.scan_config)
        self._observation(eng, hyperparam)
        eng.set_transition(tr)
        eng.ll64 = None     # the masks edit (delta, rblk) only; logZ needs no far-state ll
        eng.set_tuning(np.asarray(tuning))
        logz = torch.zeros(len(masks), dtype=torch.float64, device=eng.dev)
        eng.set_ma_latent(None)
        delta0, rblk0 = eng.emission_unmasked()
        mu8 = torch.as_tensor((masks != 0).astype(np.uint8), device=eng.dev)
        R = len(masks)
        if not eng.dense and self.n_latent_bin % 32 == 0:
            # batched: Rg masks per pass (stacked masked emissions, one forward launch)
            Rg = eng.mask_batch_size(R)
            for r0 in range(0, R, Rg):
                r1 = min(R, r0 + Rg)
                eng.masked_logz_batched(delta0, rblk0, mu8[r0:r1], likelihood_scale, logz[r0:r1])
        else:
            for r in range(R):
                eng.emission_from(delta0, rblk0, mu8[r], likelihood_scale)
                eng.forward(likelihood_scale, logz[r:r + 1])
        eng.check_status()
        return _np(logz).astype(np.float64)

    # ------------------------------------------------------------------ EM
    def fit_em(self, y, hyperparam={}, key=0, n_iter=20, log_posterior_init=None, ma_neuron=None,
               ma_latent=None, n_time_per_chunk=10000, dt=1., likelihood_scale=1., save_every=None,
               m_step_step_size=0.01, m_step_maxiter=1000, m_step_tol=1e-6,
               posterior_init_kwargs={'random_scale': 0.1}, verboase=True, **kwargs):
        """core.py:829-849 + core.py:592-713: n_iter x (M-step, E-step) on the GPU."""
        hp = dict(hyperparam)
        hp['param_prior_std'] = hp.get('param_prior_std', self.param_prior_std)
        hp['smoothness_penalty'] = hp.get('smoothness_penalty', self.smoothness_penalty)
        y_in = y
        if _is_tsd(y):
            y = y.d
        y = np.asarray(y)
        T = y.shape[0]
        tuning_lengthscale = hp.get('tuning_lengthscale', self.tuning_lengthscale)
        movement_variance = hp.get('movement_variance', self.movement_variance)
        p_move_to_jump = hp.get('p_move_to_jump', self.p_move_to_jump)
        p_jump_to_move = hp.get('p_jump_to_move', self.p_jump_to_move)
        self.tuning_lengthscale = tuning_lengthscale
        self.movement_variance = movement_variance
        self.p_move_to_jump = p_move_to_jump
        self.p_jump_to_move = p_jump_to_move
        self._m_step_step_size, self._m_step_maxiter, self._m_step_tol = m_step_step_size, m_step_maxiter, m_step_tol
        if save_every is None:
            save_every = n_iter
        # the host-side log kernels the model keeps (core.py:683-684) are formed on a helper
        # thread while the device runs the fit
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=1)
        log_kernels = pool.submit(create_transition_prob_1d, self.n_latent_bin, movement_variance, p_move_to_jump,
                                  p_jump_to_move, self.custom_transition_kernel)
        pool.shutdown(wait=False)
        if ma_neuron is None:
            ma_neuron = self.ma_neuron_default
        if ma_latent is None:
            ma_latent = self.ma_latent_default
        if 'tuning_lengthscale' in hyperparam:                            # core.py:635-638
            tuning_basis = generate_basis(tuning_lengthscale, self.n_latent_bin,
                                          self.explained_variance_threshold_basis, include_bias=True)
        else:
            tuning_basis = self.tuning_basis
        if log_posterior_init is None:
            log_posterior_init, _ = self.init_latent_posterior(T, key, **posterior_init_kwargs)

        res, info = run_em(y, self.params, tuning_basis, log_posterior_init, n_iter=n_iter,
                     transition=self._transition(movement_variance, p_move_to_jump, p_jump_to_move),
                     ma_neuron=ma_neuron, ma_latent=ma_latent, likelihood_scale=likelihood_scale,
                     save_every=save_every,
                     adam=AdamConfig(lr=m_step_step_size, maxiter=m_step_maxiter, tol=m_step_tol,
                                     prior_std=hp['param_prior_std']),
                     scan=self.scan_config, noise_std=getattr(self, '_fit_noise_std', None))
        _, log_latent_transition_kernel_l, _, log_dynamics_transition_kernel = log_kernels.result()
        self.params = res['params']
        self.tuning = res['tuning']
        self.fit_info = info
        self.log_marginal_final = res['log_marginal']
        self.log_latent_transition_kernel_l = log_latent_transition_kernel_l
        self.log_dynamics_transition_kernel = log_dynamics_transition_kernel
        self.tuning_basis = tuning_basis
        if _is_tsd(y_in):
            res['posterior_latent_marg'] = nap.TsdFrame(d=res['posterior_latent_marg'], t=y_in.t)
            res['posterior_dynamics_marg'] = nap.TsdFrame(d=res['posterior_dynamics_marg'], t=y_in.t)
        res['log_posterior_init'] = log_posterior_init
        return res

    # ------------------------------------------------------------------ misc API
    def predict_expected_rate(self, post_latent_marg, tuning=None):
        """core.py:716-733: rate[t,n] = sum_p tuning[p,n] post[t,p]."""
        if tuning is None:
            tuning = self.tuning
        pv = post_latent_marg.d if _is_tsd(post_latent_marg) else post_latent_marg
        rate = np.einsum('pn,tp->tn', np.asarray(tuning), np.asarray(pv))
        if _is_tsd(post_latent_marg):
            rate = nap.TsdFrame(d=rate, t=post_latent_marg.t)
        return rate

    def sample_latent(self, T, key=0, movement_variance=1, p_move_to_jump=0.01, p_jump_to_move=0.01,
                      init_dynamics=None, init_latent=None):
        """core.py:526-555 with a numpy RNG: dynamics from A[prev], then latent from K[dyn][prev]."""
        rng = _rng(key)
        K, _, A, _ = create_transition_prob_1d(self.n_latent_bin, movement_variance, p_move_to_jump, p_jump_to_move)
        d = int(rng.integers(2)) if init_dynamics is None else int(init_dynamics)
        l = int(rng.integers(self.n_latent_bin)) if init_latent is None else int(init_latent)
        out = np.empty((T, 2), np.int32)
        cA = np.cumsum(A, 1)
        cK = np.cumsum(K, 2)
        u = rng.random((T, 2))
        for t in range(T):
            d = int(min(np.searchsorted(cA[d], u[t, 0] * cA[d, -1], side='right'), 1))
            l = int(min(np.searchsorted(cK[d, l], u[t, 1] * cK[d, l, -1], side='right'), self.n_latent_bin - 1))
            out[t] = (d, l)
        return out

    def sample_y(self, latent_l, hyperparam={}, tuning=None, dt=1., key=10):
        """core.py:795-800: Poisson(tuning[latent] * dt)."""
        if tuning is None:
            tuning = self.tuning
        return _rng(key).poisson(np.asarray(tuning, np.float64)[np.asarray(latent_l)] * dt)

    def sample(self, T, hyperparam={}, key=0, init_dynamics=None, init_latent=None, dt=1., tuning=None):
        """core.py:558-569."""
        rng = _rng(key)
        k1, k2 = int(rng.integers(2 ** 31)), int(rng.integers(2 ** 31))
        mv = hyperparam.get('movement_variance', self.movement_variance)
        pmj = hyperparam.get('p_move_to_jump', self.p_move_to_jump)
        pjm = hyperparam.get('p_jump_to_move', self.p_jump_to_move)
        latent_l = self.sample_latent(T, k1, mv, pmj, pjm, init_dynamics, init_latent)
        y_l = self.sample_y(latent_l[:, 1], hyperparam, tuning, dt, k2)
        return latent_l, y_l

    def __getstate__(self):
        """core.py:757-767: picklable (no device state is held between calls)."""
        state = self.__dict__.copy()
        state['adam_runner'] = None
        state['opt_state_init_fun'] = None
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)


# Floor of the linear joint count S: pairs (x, x') whose every alpha_t[x] rho_{t+1}[x']
# product underflowed fp32 (states the posterior never visits) get log S = log(1e-300)
# instead of -inf.  The reference's log-domain accumulation (decoder.py:215-221) keeps a
# finite, very negative value there; the floor keeps log_joint_* finite, and a row with
# no mass at all normalises to the prior transition A[d,d'] K[d',i,:] (its reference
# value when the smoothed ratio is flat) instead of NaN.  Probability-space outputs
# differ from the reference by < 1e-290 there.
JOINT_COUNT_FLOOR = 1e-300


def log_joint_from_counts(S4, logK, logA, ml=None):
    """log accumulated joint [d, d', i, j] = logA + logK + log S, where S = sum_t
    alpha_t (x) rho_{t+1} is the device's linear-space joint count (decoder.py:215-221
    accumulates the same quantity with logaddexp).  Never -inf / NaN (see
    JOINT_COUNT_FLOOR); masked latents keep the reference's -1e20 sentinel sums."""
    S4 = np.asarray(S4, np.float64)
    zero = ~(S4 > JOINT_COUNT_FLOOR)
    logS = np.log(np.where(zero, JOINT_COUNT_FLOOR, S4))
    if ml is not None and not ml.all():
        # decoder.py:215 in log space carries ll = -1e20 (core.py:59-60) into every
        # joint entry that starts or ends in a masked latent; those entries are exact
        # zeros of S here.  Restore the sentinel sums so normalised transition rows
        # match the reference's arithmetic.
        nm = (~ml).astype(np.float64)
        sent = -1e20 * (nm[:, None] + nm[None, :])
        logS = np.where(zero & (sent < 0.0), sent[None, None], logS)
    return np.asarray(logA, np.float64)[:, :, None, None] + np.asarray(logK, np.float64)[None] + logS


def _nb_dict(lp, posterior_latent, lml_h, ll, t_l=None):
    """decode_latent_naive_bayes's returned dict (core.py:499-524)."""
    if t_l is not None and nap is not None:
        posterior_latent = nap.TsdFrame(d=posterior_latent, t=t_l)
    return {'log_posterior_latent': lp,
            'log_marginal_l': lml_h.astype(np.float32),
            'log_marginal_total': float(lml_h.sum()),
            'posterior_latent': posterior_latent,
            'll_per_pos_l': ll}


def _masked_log(logp, ml):
    """Masked latents carry ll = -1e20 in the reference (core.py:59-60), so their
    log posteriors are -1e20 (absorbed in float32), not log(0) = -inf."""
    if ml is not None and not ml.all():
        logp[..., ~ml] = np.float32(-1e20)
    return logp


def compute_transition_posterior_prob(log_accumulated_joint_total):
    """decoder.py:334-375 on the host (f64), keys in jax's sorted pytree order."""
    from scipy.special import logsumexp
    lj = np.asarray(log_accumulated_joint_total, np.float64)
    ljf = lj - logsumexp(lj)
    ljl = logsumexp(ljf, axis=(0, 1))
    ljd = logsumexp(ljf, axis=(2, 3))
    ltl = ljl - logsumexp(ljl, axis=1, keepdims=True)
    ltd = ljd - logsumexp(ljd, axis=1, keepdims=True)
    ltf = ljf - logsumexp(ljf, axis=(1, 3), keepdims=True)
    r = {'p_joint_full': np.exp(ljf), 'p_joint_latent': np.exp(ljl), 'p_joint_dynamics': np.exp(ljd),
         'p_transition_full': np.exp(ltf), 'p_transition_latent': np.exp(ltl),
         'p_transition_dynamics': np.exp(ltd), 'log_joint_full': ljf, 'log_joint_latent': ljl,
         'log_joint_dynamics': ljd, 'log_transition_full': ltf, 'log_transition_latent': ltl,
         'log_transition_dynamics': ltd}
    return {k: r[k].astype(np.float32) for k in sorted(r)}


def _m_step_res(s, lhn, ehn, n_iter):
    """m_step_res_l of the fit_em dict (core.py:655-658, histories trimmed to n_iter as
    core.py:819-826) from the device's per-iteration (n_iter, final_loss, final_error)
    stats and the padded loss / error histories."""
    out = {'params': [], 'opt_state': [], 'n_iter': [], 'final_loss': [], 'final_error': [],
           'loss_history': [], 'error_history': []}
    for i in range(n_iter):
        n = int(s[i, 0])
        out['n_iter'].append(n)
        out['final_loss'].append(float(s[i, 1]))
        out['final_error'].append(float(s[i, 2]))
        out['loss_history'].append(lhn[i, :n].copy())
        out['error_history'].append(ehn[i, :n].copy())
    return out


def run_em(y, params, basis, log_posterior_init, n_iter, transition, ma_neuron=None, ma_latent=None,
           likelihood_scale=1.0, save_every=None, adam: AdamConfig | None = None,
           scan: ScanConfig | None = None, opt_state=None, timing=None, noise_std=None):
    """The EM loop of core.py:650-676 on one GPU; returns the fit_em dict (core.py:696-712).
    noise_std: Gaussian observation model (analytic M-step, linear tuning; adam.prior_std
    is the parameter prior) instead of the Poisson one.
    `timing`, if a list, receives per-iteration wall-clock seconds (bench)."""
    if int(n_iter) < 1:
        # the reference's fit_em defines tuning / log_posterior_all inside its loop and
        # fails after a 0-iteration loop (core.py:650-681); never return an unset posterior
        raise ValueError(f"n_iter must be >= 1 (got {n_iter})")
    adam = adam or AdamConfig()
    y = np.asarray(y)
    T = y.shape[0]
    B = np.asarray(basis, np.float32)
    L = B.shape[0]
    if save_every is None:
        save_every = n_iter
    ma = None if ma_neuron is None else np.asarray(ma_neuron, np.float32)
    dev = default_device()
    # the returned arrays go to the host through pinned buffers without host syncs inside
    # the loop: snapshots on a side stream beside the later iterations (their device
    # copies are fresh tensors), the final arrays after the loop.  The large buffers are
    # allocated on a helper thread from here on, beside the uploads and the loop.
    cp = _PinnedCopies(dev)
    n_saved = len(range(0, n_iter, save_every))
    cp.reserve_upto('snap', (T, 2, L), n_saved)
    for key, shape in (('post', (T, 2, L)), ('lpf', (T, 2, L)), ('plm', (T, L))):
        cp.reserve(key, shape)
    sp = SpikeData(y, ma)
    eng = DeviceEM(sp, L, basis=B, scan=scan)
    eng.adaptive = True          # adaptive warm-up across this fit's E-steps
    eng.set_transition(transition)
    eng.set_ma_latent(ma_latent)
    if noise_std is not None:
        eng.noise_std, eng.gauss_prior_std = float(noise_std), float(adam.prior_std)
    mlat = None if ma_latent is None else np.asarray(ma_latent).astype(bool)
    eng.set_log_posterior(log_posterior_init)
    dev = eng.dev
    W = torch.as_tensor(np.asarray(params, np.float64), device=dev).contiguous()
    if opt_state is None:
        mu = torch.zeros_like(W)
        nu = torch.zeros_like(W)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    else:
        mu = torch.as_tensor(np.asarray(opt_state['mu'], np.float64), device=dev).contiguous()
        nu = torch.as_tensor(np.asarray(opt_state['nu'], np.float64), device=dev).contiguous()
        cnt = torch.tensor([int(opt_state['count'])], dtype=torch.int64, device=dev)
    mi = max(int(adam.maxiter), 1)
    stats = torch.zeros((n_iter, 4), dtype=torch.float64, device=dev)
    lh = torch.zeros((n_iter, mi), dtype=torch.float64, device=dev)
    eh = torch.zeros((n_iter, mi), dtype=torch.float64, device=dev)
    logz = torch.zeros(max(n_iter, 1), dtype=torch.float64, device=dev)
    gamma = torch.empty((T, 2, L), dtype=torch.float32, device=dev)
    lgam = torch.empty((T, 2, L), dtype=torch.float32, device=dev) if eng.dense else None

    def log_post_dev():
        return lgam.clone() if eng.dense else log_of(gamma)
    saved_dev = []      # (i, log posterior, W f32, tuning) pinned host buffers per snapshot
    saved_idx = []
    import time
    for i in range(n_iter):
        t0 = time.perf_counter() if timing is not None else 0.0
        eng.m_step(W, mu, nu, cnt, adam, stats[i], lh[i], eh[i])
        eng.compute_tuning(W)
        want_gamma = (i == n_iter - 1) or (i % save_every == 0)
        eng.e_step(likelihood_scale, logz[i:i + 1], gamma=gamma if want_gamma else None,
                   log_gamma=lgam if want_gamma else None)
        if i % save_every == 0:
            # the (T, 2, L) log posterior (a fresh tensor) on the side stream; W and the
            # tuning (written again by the next iterations) on this stream, W as f64 (cast
            # on the host: no cast kernel)
            saved_dev.append((cp.submit(log_post_dev(), key='snap', side=True), cp.submit(W),
                              cp.submit(eng.tuning32)))
            saved_idx.append(i)
        if timing is not None:
            torch.cuda.synchronize()
            timing.append(time.perf_counter() - t0)
    # final arrays: the sums over d and l on the device (posterior_latent_marg /
    # posterior_dynamics_marg), every copy queued behind the last E-step
    lg, plm, pdm = posterior_outputs(gamma, log=not eng.dense)
    h_post = cp.submit(gamma, key='post')
    h_lpf = cp.submit(lgam if eng.dense else lg, key='lpf')
    h_plm = cp.submit(plm, key='plm')
    h_pdm = cp.submit(pdm)
    h_W = cp.submit(W)
    h_tun = cp.submit(eng.tuning32)
    h_st, h_lh, h_eh, h_lz = cp.submit(stats), cp.submit(lh), cp.submit(eh), cp.submit(logz)
    cp.finish()
    lz = h_lz
    saved = {'log_posterior_all_saved': [_masked_log(a, mlat) for a, _, _ in saved_dev],
             'params_saved': [b.astype(np.float32) for _, b, _ in saved_dev],
             'tuning_saved': [c for _, _, c in saved_dev],
             'iter_saved': list(saved_idx),
             'log_marginal_saved': [float(lz[i]) for i in saved_idx]}
    m_step_res_l = _m_step_res(h_st, h_lh, h_eh, n_iter)
    posterior = h_post
    res = {'log_posterior_all_saved': saved['log_posterior_all_saved'],
           'log_posterior_init': log_posterior_init,
           'params_saved': saved['params_saved'],
           'tuning_saved': saved['tuning_saved'],
           'iter_saved': saved['iter_saved'],
           'params': h_W.astype(np.float32),
           'tuning': h_tun,
           'log_posterior_final': _masked_log(h_lpf, mlat),
           'log_marginal': float(lz[n_iter - 1]),
           'log_marginal_l': [float(v) for v in lz[:n_iter]],
           'log_marginal_saved': saved['log_marginal_saved'],
           'posterior': posterior,
           'posterior_latent_marg': h_plm,
           'posterior_dynamics_marg': h_pdm,
           'm_step_res_l': m_step_res_l}
    if noise_std is not None:
        eng.gaussian_status()
        res['m_step_res_l'] = {'params': [], 'opt_state': []}      # core.py:655-658 with m_step core.py:898-904
    else:
        eng.emission_status()
        eng.adam_status()
    info = {'opt_state': {'mu': _np(mu), 'nu': _np(nu), 'count': int(_np(cnt)[0])},
            'params64': _np(W), 'repairs': eng.repairs(), 'chunk': eng.C}
    return res, info


def run_em_restarts(y, params, basis, log_posterior_inits, n_iter, transition, ma_neuron=None, ma_latent=None,
                    likelihood_scale=1.0, save_every=None, adam: AdamConfig | None = None,
                    scan: ScanConfig | None = None, timing=None):
    """R restarts of the Poisson EM loop (core.py:650-676) batched on one GPU
    (engine.RestartBatchEM); returns [(fit_em dict, info)] per restart, each the same as
    run_em would return for that restart alone.  params: (NB, N) shared initial W or
    (R, NB, N); log_posterior_inits: (R, T, L).  The restart loop this replaces is
    model_selection_helper.py:53-59 (one fit_em per key)."""
    adam = adam or AdamConfig()
    y = np.asarray(y)
    lpi = np.asarray(log_posterior_inits, np.float32)
    R, T, L = lpi.shape
    B = np.asarray(basis, np.float32)
    if B.shape[0] != L or y.shape[0] != T:
        raise ValueError("log_posterior_inits must be (R, n_time, n_latent_bin)")
    if save_every is None:
        save_every = n_iter
    ma = None if ma_neuron is None else np.asarray(ma_neuron, np.float32)
    sp = SpikeData(y, ma)
    eng = RestartBatchEM(sp, L, B, R, scan=scan)
    eng.set_transition(transition)
    eng.set_ma_latent(ma_latent)
    mlat = None if ma_latent is None else np.asarray(ma_latent).astype(bool)
    eng.set_log_posterior(lpi)
    dev = eng.dev
    W0 = np.asarray(params, np.float64)
    W = torch.as_tensor(np.ascontiguousarray(np.broadcast_to(W0, (R,) + W0.shape[-2:])), device=dev).contiguous()
    mu = torch.zeros_like(W)
    nu = torch.zeros_like(W)
    cnt = torch.zeros(R, dtype=torch.int64, device=dev)
    mi = max(int(adam.maxiter), 1)
    stats = torch.zeros((n_iter, R, 4), dtype=torch.float64, device=dev)
    lh = torch.zeros((n_iter, R, mi), dtype=torch.float64, device=dev)
    eh = torch.zeros((n_iter, R, mi), dtype=torch.float64, device=dev)
    logz = torch.zeros((max(n_iter, 1), R), dtype=torch.float64, device=dev)
    gamma = torch.empty((R, T, 2, L), dtype=torch.float32, device=dev)
    saved = [{'log_posterior_all_saved': [], 'params_saved': [], 'tuning_saved': [], 'iter_saved': []}
             for _ in range(R)]
    saved_idx = []

    def log_post(r):
        return _masked_log(_np(log_of(gamma[r])), mlat)
    import time
    for i in range(n_iter):
        t0 = time.perf_counter() if timing is not None else 0.0
        eng.m_step(W, mu, nu, cnt, adam, stats[i], lh[i], eh[i])
        eng.compute_tuning(W)
        want_gamma = (i == n_iter - 1) or (i % save_every == 0)
        eng.e_step(likelihood_scale, logz[i], gamma=gamma if want_gamma else None)
        if i % save_every == 0:
            for r in range(R):
                saved[r]['log_posterior_all_saved'].append(log_post(r))
                saved[r]['params_saved'].append(_np(W[r]).astype(np.float32))
                saved[r]['tuning_saved'].append(_np(eng.tuning32[r * L:(r + 1) * L]))
                saved[r]['iter_saved'].append(i)
            saved_idx.append(i)
        if timing is not None:
            torch.cuda.synchronize()
            timing.append(time.perf_counter() - t0)
    lz = _np(logz)
    st, lhn, ehn = _np(stats), _np(lh), _np(eh)
    repairs = eng.repairs()
    eng.emission_status()
    eng.ws_ad.status()
    out = []
    for r in range(R):
        posterior = _np(gamma[r])
        res = {'log_posterior_all_saved': saved[r]['log_posterior_all_saved'],
               'log_posterior_init': lpi[r],
               'params_saved': saved[r]['params_saved'],
               'tuning_saved': saved[r]['tuning_saved'],
               'iter_saved': saved[r]['iter_saved'],
               'params': _np(W[r]).astype(np.float32),
               'tuning': _np(eng.tuning32[r * L:(r + 1) * L]),
               'log_posterior_final': log_post(r),
               'log_marginal': float(lz[n_iter - 1, r]) if n_iter else float('nan'),
               'log_marginal_l': [float(v) for v in lz[:n_iter, r]],
               'log_marginal_saved': [float(lz[i, r]) for i in saved_idx],
               'posterior': posterior,
               'posterior_latent_marg': posterior.sum(axis=1),
               'posterior_dynamics_marg': posterior.sum(axis=2),
               'm_step_res_l': _m_step_res(st[:, r], lhn[:, r], ehn[:, r], n_iter)}
        info = {'opt_state': {'mu': _np(mu[r]), 'nu': _np(nu[r]), 'count': int(_np(cnt)[r])},
                'params64': _np(W[r]), 'repairs': repairs[r], 'chunk': eng.C, 'batched_restarts': R}
        out.append((res, info))
    return out


def fit_em_restarts(models, y, keys, hyperparam={}, n_iter=20, ma_neuron=None, ma_latent=None,
                    likelihood_scale=1., save_every=None, m_step_step_size=0.01, m_step_maxiter=1000,
                    m_step_tol=1e-6, posterior_init_kwargs={'random_scale': 0.1}, **kwargs):
    """models[r].fit_em(y, hyperparam, key=keys[r], ...) for every r, run as ONE batched
    fit on the GPU (run_em_restarts) when the models allow it: the same exact class
    PoissonGPLVMJump1D, identical configuration and initial params, a banded transition
    and n_latent_bin % 32 == 0.  Otherwise the fits run one after another.  Each model
    ends in the state its own fit_em would leave (params, tuning, kernels, basis)."""
    models = list(models)
    keys = list(keys)
    if len(models) != len(keys):
        raise ValueError("one key per model")
    fit_kw = dict(n_iter=n_iter, ma_neuron=ma_neuron, ma_latent=ma_latent, likelihood_scale=likelihood_scale,
                  save_every=save_every, m_step_step_size=m_step_step_size, m_step_maxiter=m_step_maxiter,
                  m_step_tol=m_step_tol, posterior_init_kwargs=posterior_init_kwargs, **kwargs)
    if len(models) < 2 or not _restarts_batchable(models, hyperparam):
        return [m.fit_em(y, hyperparam=hyperparam, key=k, **fit_kw) for m, k in zip(models, keys)]
    m0 = models[0]
    y_in = y
    y = np.asarray(y.d if _is_tsd(y) else y)
    T = y.shape[0]
    hp = dict(hyperparam)
    prior_std = hp.get('param_prior_std', m0.param_prior_std)
    mv = hp.get('movement_variance', m0.movement_variance)
    pmj = hp.get('p_move_to_jump', m0.p_move_to_jump)
    pjm = hp.get('p_jump_to_move', m0.p_jump_to_move)
    ls = hp.get('tuning_lengthscale', m0.tuning_lengthscale)
    tuning_basis = (generate_basis(ls, m0.n_latent_bin, m0.explained_variance_threshold_basis, include_bias=True)
                    if 'tuning_lengthscale' in hyperparam else m0.tuning_basis)
    if ma_neuron is None:
        ma_neuron = m0.ma_neuron_default
    if ma_latent is None:
        ma_latent = m0.ma_latent_default
    lp_given = kwargs.get('log_posterior_init')
    if lp_given is not None:   # fit_em(log_posterior_init=...) starts every restart there
        lpi = np.stack([np.asarray(lp_given, np.float32)] * len(models))
    else:
        lpi = np.stack([m.init_latent_posterior(T, k, **posterior_init_kwargs)[0] for m, k in zip(models, keys)])
    outs = run_em_restarts(y, m0.params, tuning_basis, lpi, n_iter=n_iter,
                           transition=m0._transition(mv, pmj, pjm), ma_neuron=ma_neuron, ma_latent=ma_latent,
                           likelihood_scale=likelihood_scale, save_every=save_every,
                           adam=AdamConfig(lr=m_step_step_size, maxiter=m_step_maxiter, tol=m_step_tol,
                                           prior_std=prior_std), scan=m0.scan_config)
    _, lk, _, la = create_transition_prob_1d(m0.n_latent_bin, mv, pmj, pjm, m0.custom_transition_kernel)
    results = []
    for m, (res, info) in zip(models, outs):
        m.tuning_lengthscale, m.movement_variance, m.p_move_to_jump, m.p_jump_to_move = ls, mv, pmj, pjm
        m._m_step_step_size, m._m_step_maxiter, m._m_step_tol = m_step_step_size, m_step_maxiter, m_step_tol
        m.params = res['params']
        m.tuning = res['tuning']
        m.fit_info = info
        m.log_marginal_final = res['log_marginal']
        m.log_latent_transition_kernel_l = lk
        m.log_dynamics_transition_kernel = la
        m.tuning_basis = tuning_basis
        if _is_tsd(y_in):
            res['posterior_latent_marg'] = nap.TsdFrame(d=res['posterior_latent_marg'], t=y_in.t)
            res['posterior_dynamics_marg'] = nap.TsdFrame(d=res['posterior_dynamics_marg'], t=y_in.t)
        results.append(res)
    return results


def _restarts_batchable(models, hyperparam):
    """run_em_restarts holds these fits: exact PoissonGPLVMJump1D models with identical
    configuration and initial params, a banded transition and n_latent_bin % 32 == 0."""
    m0 = models[0]
    if any(type(m) is not PoissonGPLVMJump1D for m in models):
        return False
    if m0.n_latent_bin % 32 or m0.custom_transition_kernel is not None:
        return False
    keys = ('n_neuron', 'n_latent_bin', 'tuning_lengthscale', 'param_prior_std', 'movement_variance',
            'p_move_to_jump', 'p_jump_to_move', 'smoothness_penalty')
    for m in models[1:]:
        if any(np.any(np.asarray(getattr(m, k, None)) != np.asarray(getattr(m0, k, None))) for k in keys):
            return False
        if not np.array_equal(np.asarray(m.params), np.asarray(m0.params)):
            return False
        if not np.array_equal(np.asarray(m.tuning_basis), np.asarray(m0.tuning_basis)):
            return False
    mv = hyperparam.get('movement_variance', m0.movement_variance)
    pmj = hyperparam.get('p_move_to_jump', m0.p_move_to_jump)
    pjm = hyperparam.get('p_jump_to_move', m0.p_jump_to_move)
    return not isinstance(m0._transition(mv, pmj, pjm), DenseTransition)


class GaussianGPLVMJump1D(PoissonGPLVMJump1D):
    """Gaussian GPLVM with jumps (core.py:852-917): tuning = basis @ W
    (fit_tuning_helper.get_tuning_linear, :12-17), y ~ N(tuning[latent] * dt, noise_std),
    analytic M-step (gaussian_m_step_analytic, fit_tuning_helper.py:44-61; no optimiser
    state).  Same jump dynamics, scans, sufficient statistics and result dicts as the
    Poisson model; the emission, tuning and M-step run in gaussian.hip."""

    def __init__(self, n_neuron, noise_std=0.5, **kwargs):
        super().__init__(n_neuron, **kwargs)
        self.noise_std = noise_std

    def _observation(self, eng, hyperparam):
        eng.noise_std = float(hyperparam.get('noise_std', self.noise_std))
        eng.gauss_prior_std = float(hyperparam.get('param_prior_std', self.param_prior_std))

    def get_tuning(self, params, hyperparam, tuning_basis):
        """fit_tuning_helper.get_tuning_linear (:12-17), on the device (f64)."""
        B = np.asarray(tuning_basis, np.float32)
        W = np.asarray(params, np.float64)
        dev = default_device()
        lib = nat.load()
        bt = torch.as_tensor(np.ascontiguousarray(B), device=dev)
        wt = torch.as_tensor(np.ascontiguousarray(W), device=dev)
        out = torch.empty((B.shape[0], W.shape[1]), dtype=torch.float32, device=dev)
        nat.check(lib.pmg_tuning_linear(nat.ptr(bt), nat.ptr(wt), B.shape[0], B.shape[1], W.shape[1],
                                        None, nat.ptr(out), nat.stream_handle()), "pmg_tuning_linear")
        return _np(out)

    def m_step(self, param_curr, y, log_posterior_curr, tuning_basis, hyperparam, opt_state_curr=None):
        """core.py:898-904: suff-stats then the analytic solve; {'params', 'opt_state': None}."""
        y = np.asarray(y)
        B = np.asarray(tuning_basis, np.float32)
        eng = DeviceEM(SpikeData(y, None), B.shape[0], basis=B, scan=self.scan_config)
        self._observation(eng, hyperparam)
        eng.set_log_posterior(log_posterior_curr)
        W = torch.zeros((B.shape[1], y.shape[1]), dtype=torch.float64, device=eng.dev)
        eng.m_step(W, None, None, None, None, None, None, None)
        eng.gaussian_status()
        return {'params': _np(W).astype(np.float32), 'opt_state': None}

    def fit_em(self, y, hyperparam={}, key=0, n_iter=20, log_posterior_init=None, ma_neuron=None,
               ma_latent=None, n_time_per_chunk=10000, dt=1., likelihood_scale=1., save_every=None, **kwargs):
        """core.py:905-917 over AbstractGPLVMJump1D.fit_em (core.py:592-713)."""
        hp = dict(hyperparam)
        hp['noise_std'] = hp.get('noise_std', self.noise_std)
        hp['param_prior_std'] = hp.get('param_prior_std', self.param_prior_std)
        self._fit_noise_std = hp['noise_std']
        try:
            return super().fit_em(y, hyperparam=hp, key=key, n_iter=n_iter, log_posterior_init=log_posterior_init,
                                  ma_neuron=ma_neuron, ma_latent=ma_latent, n_time_per_chunk=n_time_per_chunk,
                                  dt=dt, likelihood_scale=likelihood_scale, save_every=save_every, **kwargs)
        finally:
            self._fit_noise_std = None

    def _decode_hp(self, hyperparam):
        hp = dict(hyperparam)
        hp['noise_std'] = hp.get('noise_std', self.noise_std)
        return hp

    def decode_latent(self, y, tuning=None, hyperparam={}, **kwargs):
        """core.py:879-882: noise_std from hyperparam or the model."""
        hp = dict(hyperparam)
        hp['noise_std'] = hp.get('noise_std', self.noise_std)
        return super().decode_latent(y, tuning=tuning, hyperparam=hp, **kwargs)

    def decode_latent_naive_bayes(self, y, tuning=None, hyperparam={}, **kwargs):
        """core.py:884-887: the naive-Bayes decoder with the Gaussian emission
        (constant dt; pmg_emission_gaussian + pmg_naive_bayes_normalize)."""
        hp = dict(hyperparam)
        hp['noise_std'] = hp.get('noise_std', self.noise_std)
        return super().decode_latent_naive_bayes(y, tuning=tuning, hyperparam=hp, **kwargs)

    def sample_y(self, latent_l, hyperparam={}, tuning=None, dt=1., key=10):
        """core.py:889-896: N(tuning[latent] * dt, noise_std * sqrt(dt))."""
        if tuning is None:
            tuning = self.tuning
        s = hyperparam.get('noise_std', self.noise_std) * math.sqrt(dt)
        rate = np.asarray(tuning, np.float64)[np.asarray(latent_l)] * dt
        return _rng(key).normal(size=rate.shape) * s + rate


class PoissonGPLVM1D(PoissonGPLVMJump1D):
    """Poisson GPLVM with a smooth 1-d latent and no dynamics (core.py:919-1019 over
    AbstractGPLVM1D, core.py:76-375; decoder_latentonly.py).

    The latent-only chain is the jump engine with the dynamics pinned to
    A = [[1, 0], [1, 0]] (p_move_to_jump = 0, p_jump_to_move = 1): starting from the
    uniform (d, l) state, the continuous prior is K^T (1/L) exactly as
    filter_all_step_latent starts from log(1/L) (decoder_latentonly.py:66-68), the jump
    state's prior is exactly 0 at every step, and every latent-only quantity (filter,
    smoother, logZ, one-step marginals, pairwise joint) is the d = 0 block of the jump
    engine's.  basis_type 'rbf' with smoothness_penalty = 0 (the default objective
    poisson_m_step_objective); the b-spline smoothness objective is not implemented."""

    def __init__(self, n_neuron, n_latent_bin=100, tuning_lengthscale=5., param_prior_std=1.,
                 movement_variance=1., explained_variance_threshold_basis=0.999, rng_init_int=123,
                 w_init_variance=1., w_init_mean=0., basis_type='rbf', custom_tuning_kernel=None,
                 custom_transition_kernel=None, smoothness_penalty=0., scan_config: ScanConfig | None = None):
        if basis_type != 'rbf' or smoothness_penalty != 0.:
            raise NotImplementedError("PoissonGPLVM1D: only basis_type='rbf' with smoothness_penalty=0 "
                                      "(poisson_m_step_objective) is implemented")
        super().__init__(n_neuron, n_latent_bin=n_latent_bin, tuning_lengthscale=tuning_lengthscale,
                         param_prior_std=param_prior_std, movement_variance=movement_variance,
                         explained_variance_threshold_basis=explained_variance_threshold_basis,
                         rng_init_int=rng_init_int, w_init_variance=w_init_variance, w_init_mean=w_init_mean,
                         p_move_to_jump=0.0, p_jump_to_move=1.0, basis_type=basis_type,
                         custom_tuning_kernel=custom_tuning_kernel,
                         custom_transition_kernel=custom_transition_kernel,
                         smoothness_penalty=smoothness_penalty, scan_config=scan_config)
        del self.possible_dynamics

    def _transition(self, movement_variance, p_move_to_jump=0.0, p_jump_to_move=1.0):
        """Always the dense log-domain scans: without a jump state the only way between
        distant latents is the continuous kernel itself, with weights like
        exp(-d^2/mv^2) far below the fp32 / f64 range that the reference's log-space
        recursion (decoder_latentonly.py:33-123) keeps exactly."""
        return dense_transition(self.n_latent_bin, movement_variance, 0.0, 1.0, self.custom_transition_kernel)

    def _check_latent_mask(self, tr, ma_latent):
        """Masks with wide gaps are exact on the dense log-domain scans: nothing to check."""

    def _decode_latent(self, y, tuning, hyperparam, log_latent_transition_kernel, ma_neuron, ma_latent=None,
                       likelihood_scale=1., n_time_per_chunk=10000):
        """core.py:943-953 -> decoder_latentonly.smooth_all_step_combined_ma_chunk_latent
        (decoder_latentonly.py:156-224) with the (L, L) log kernel passed in.  Returns the
        latent-only 6-tuple: log_acausal (T, L), log marginal, log_causal (T, L),
        one-step predictive marginals (T,), log joint (L, L), log likelihood (T, L)."""
        lk = np.asarray(log_latent_transition_kernel, np.float64)
        L = self.n_latent_bin
        if lk.shape != (L, L):
            raise ValueError(f"log_latent_transition_kernel must be ({L}, {L})")
        hp = dict(hyperparam)
        hp['p_move_to_jump'], hp['p_jump_to_move'] = 0.0, 1.0
        logK = np.stack([lk, np.full((L, L), -math.log(L))])
        with np.errstate(divide='ignore'):
            logA = np.log(np.array([[1.0, 0.0], [1.0, 0.0]]))
        r = self._run_decode(y, tuning, hp, ma_neuron, ma_latent, likelihood_scale, joint=True, logK=logK,
                             logA=logA)
        return (r['log_posterior_all'][:, 0], r['log_marginal_final'], r['log_causal_posterior_all'][:, 0],
                r['log_one_step_predictive_marginals_all'], r['log_accumulated_joint'][0, 0],
                r['log_likelihood_all'])

    def init_latent_posterior(self, T, key, random_scale=0.1):
        """core.py:241-251: (1/L + U(0,1)*scale), row-normalised, log (numpy RNG)."""
        L = self.n_latent_bin
        post = np.ones((T, L)) / L + _rng(key).random((T, L)) * random_scale
        post = post / post.sum(axis=1, keepdims=True)
        with np.errstate(divide='ignore'):
            lp = np.log(post)
        lp = np.where(lp == -np.inf, -1e40, lp)
        return lp.astype(np.float32), post.astype(np.float32)

    def decode_latent(self, y, tuning=None, hyperparam={}, ma_neuron=None, ma_latent=None,
                      likelihood_scale=1., n_time_per_chunk=10000, t_l=None):
        """core.py:136-177 + decoder_latentonly.compute_transition_posterior_prob_latent
        (decoder_latentonly.py:227-252)."""
        if _is_tsd(y):
            t_l = y.t
            y = y.d
        if tuning is None:
            tuning = self.tuning
        if ma_neuron is None:
            ma_neuron = self.ma_neuron_default
        if ma_latent is None:
            ma_latent = self.ma_latent_default
        hp, logK, logA = self._dynamics_decode_args(hyperparam)
        r = self._run_decode(y, tuning, hp, ma_neuron, ma_latent, likelihood_scale, joint=True, logK=logK, logA=logA)
        return self._decode_result(r, t_l)

    def _dynamics_decode_args(self, hyperparam):
        hp = dict(hyperparam)
        hp['p_move_to_jump'], hp['p_jump_to_move'] = 0.0, 1.0
        mv = hp.get('movement_variance', self.movement_variance)
        _, logK, _, logA = create_transition_prob_1d(self.n_latent_bin, mv, 0.0, 1.0, self.custom_transition_kernel)
        return hp, logK, logA

    def _decode_result(self, r, t_l=None):
        """decode_latent's latent-only dict (core.py:160-177)."""
        posterior_all = r['posterior_all'][:, 0]
        if t_l is not None and nap is not None:
            posterior_all = nap.TsdFrame(d=posterior_all, t=t_l)
        res = {'log_posterior_all': r['log_posterior_all'][:, 0],
               'log_marginal_final': r['log_marginal_final'],
               'posterior_all': posterior_all,
               'log_one_step_predictive_marginals_all': r['log_one_step_predictive_marginals_all'],
               'log_likelihood_all': r['log_likelihood_all']}
        res.update(compute_transition_posterior_prob_latent(r['log_accumulated_joint'][0, 0]))
        return res

    def fit_em(self, y, hyperparam={}, key=0, n_iter=20, log_posterior_init=None, ma_neuron=None,
               ma_latent=None, n_time_per_chunk=10000, dt=1., likelihood_scale=1., save_every=None,
               m_step_step_size=0.01, m_step_maxiter=1000, m_step_tol=1e-6,
               posterior_init_kwargs={'random_scale': 0.1}, verboase=True, **kwargs):
        """core.py:1000-1019 + AbstractGPLVM1D.fit_em (core.py:259-375): returns its 13 keys."""
        hp = dict(hyperparam)
        hp['p_move_to_jump'], hp['p_jump_to_move'] = 0.0, 1.0
        self._check_latent_mask(self._transition(hp.get('movement_variance', self.movement_variance)), ma_latent)
        r = super().fit_em(y, hyperparam=hp, key=key, n_iter=n_iter, log_posterior_init=log_posterior_init,
                           ma_neuron=ma_neuron, ma_latent=ma_latent, n_time_per_chunk=n_time_per_chunk, dt=dt,
                           likelihood_scale=likelihood_scale, save_every=save_every,
                           m_step_step_size=m_step_step_size, m_step_maxiter=m_step_maxiter,
                           m_step_tol=m_step_tol, posterior_init_kwargs=posterior_init_kwargs, verboase=verboase)
        del self.log_latent_transition_kernel_l, self.log_dynamics_transition_kernel
        self.log_latent_transition_kernel = create_transition_prob_1d(
            self.n_latent_bin, self.movement_variance, 0.0, 1.0, self.custom_transition_kernel)[1][0]
        posterior = r['posterior'][:, 0]
        if _is_tsd(y):
            posterior = nap.TsdFrame(d=posterior, t=y.t)
        return {'log_posterior_all_saved': [lp[:, 0] for lp in r['log_posterior_all_saved']],
                'log_posterior_init': r['log_posterior_init'],
                'params_saved': r['params_saved'],
                'tuning_saved': r['tuning_saved'],
                'iter_saved': r['iter_saved'],
                'params': r['params'],
                'tuning': r['tuning'],
                'log_posterior_final': r['log_posterior_final'][:, 0],
                'log_marginal': r['log_marginal'],
                'log_marginal_l': r['log_marginal_l'],
                'log_marginal_saved': r['log_marginal_saved'],
                'posterior': posterior,
                'm_step_res_l': r['m_step_res_l']}

    def sample_latent(self, T, key=0, movement_variance=1, init_latent=None):
        """core.py:209-229 with a numpy RNG: latent from K[prev]."""
        rng = _rng(key)
        K, _ = create_transition_prob_1d(self.n_latent_bin, movement_variance, 0.0, 1.0)[:2]
        cK = np.cumsum(K[0], 1)
        l = int(rng.integers(self.n_latent_bin)) if init_latent is None else int(init_latent)
        out = np.empty(T, np.int32)
        u = rng.random(T)
        for t in range(T):
            l = int(min(np.searchsorted(cK[l], u[t] * cK[l, -1], side='right'), self.n_latent_bin - 1))
            out[t] = l
        return out

    def sample(self, T, hyperparam={}, key=0, init_latent=None, dt=1., tuning=None):
        """core.py:231-239."""
        rng = _rng(key)
        k1, k2 = int(rng.integers(2 ** 31)), int(rng.integers(2 ** 31))
        mv = hyperparam.get('movement_variance', self.movement_variance)
        latent_l = self.sample_latent(T, k1, mv, init_latent)
        return latent_l, self.sample_y(latent_l, hyperparam, tuning, dt, k2)


class GaussianGPLVM1D(GaussianGPLVMJump1D, PoissonGPLVM1D):
    """Gaussian GPLVM with a latent-only chain (core.py:1022-1090): the Gaussian
    observation model (emission, linear tuning, analytic M-step) of
    GaussianGPLVMJump1D on PoissonGPLVM1D's pinned-dynamics engine (latent-only
    outputs, uniform 1/L start, band-limited continuous kernel)."""

    def __init__(self, n_neuron, noise_std=0.5, **kwargs):
        super().__init__(n_neuron, noise_std=noise_std, **kwargs)


def compute_transition_posterior_prob_latent(log_accumulated_joint_total):
    """decoder_latentonly.py:227-252 on the host (f64): normalised joint and
    row-conditional transition of the latent-only model, keys in jax's sorted order."""
    from scipy.special import logsumexp
    lj = np.asarray(log_accumulated_joint_total, np.float64)
    lj = lj - logsumexp(lj)
    lt = lj - logsumexp(lj, axis=1, keepdims=True)
    r = {'p_joint_latent': np.exp(lj), 'p_transition_latent': np.exp(lt),
         'log_joint_latent': lj, 'log_transition_latent': lt}
    return {k: r[k].astype(np.float32) for k in sorted(r)}
