"""CPU oracle: float64 numpy restatement of the reference's PoissonGPLVMJump1D EM hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product package (``poor_man_gplvm_amd``)
never imports it.

PARITY UNPINNED (against the reference's own outputs): the reference is a JAX
program (jax/jaxlib 0.4.26 + optax 0.2.2) and JAX is not installable in this
image; the reference ships no golden vectors or known-answer tests for this
path (its only test file, ``tests/test_basic.py:6``, imports a class that does
not exist).  This restatement is instead pinned by
  * brute-force path enumeration of tiny HMMs (``oracle/brute.py``), which
    computes posteriors, pairwise joints and the log marginal by summing over
    every (dynamics, latent) path -- an independent, exact check of the
    filter / smoother / chunk-carry logic;
  * hand-derived optax-0.2.2 Adam steps and finite-difference gradients of the
    M-step objective (tests/test_oracle_*.py);
  * the API facts the reference's own notebooks record (dict key order of
    ``decode_latent``, ``ripple-type-GPLVM-tunings.ipynb`` cell 25).

Every function cites the reference file:line it restates.  Arithmetic is
float64 and follows the reference's log-domain formulation exactly (dense
logsumexp over the full L x L kernels, joint accumulated with logaddexp) --
this is also the algorithm the CPU baseline times.

``working_precision(np.float32)`` runs the same restatement in float32, the
reference's own arithmetic type (all arrays fp32, no x64 anywhere in the
reference): a *reference-mimic* used by the tests to measure the reference's
own rounding noise against the float64 answer.
"""
from __future__ import annotations

import contextlib
import math

import numpy as np
from scipy.special import gammaln, logsumexp, xlogy

__all__ = [
    "rbf_kernel_matrix", "generate_basis", "create_transition_prob_1d",
    "get_tuning_softplus", "softplus", "loglikelihood_poisson_all",
    "filter_one_step", "filter_all_step", "smooth_one_step", "smooth_all_step",
    "smooth_all_step_combined_ma_chunk", "compute_transition_posterior_prob",
    "get_statistics", "poisson_m_step_objective", "poisson_m_step_grad",
    "adam_init", "adam_update", "adam_run", "m_step", "fit_em", "decode_latent",
    "naive_bayes_chunk", "init_latent_posterior_from_uniform", "sample_latent",
    "sample_spikes", "jump_consensus", "downsampled_lml", "loglikelihood_gaussian_all",
    "gaussian_m_step_analytic", "fit_em_gaussian", "circular_shuffle_once", "compute_entropy",
]

NEG_MASK = -1e20          # decoder.py:46  masked latent log-likelihood
RATE_EPS = 1e-20          # decoder.py:39, fit_tuning_helper.py:78

_F = np.float64           # working precision of the restatement


@contextlib.contextmanager
def working_precision(dtype):
    """Run the restatement in `dtype` (np.float32 = reference-mimic)."""
    global _F
    old, _F = _F, dtype
    try:
        yield
    finally:
        _F = old


# ----------------------------------------------------------------------------
# kernels / basis  (gp_kernel.py, core.py:41-73)
# ----------------------------------------------------------------------------
def rbf_kernel_matrix(n, ls, var=1.0, dtype=np.float64):
    """gp_kernel.py:14-20 vmapped twice (core.py:51, gp_kernel.py:67):
    K[i,j] = exp(-(i-j)^2/ls^2)*var, logK[i,j] = -(i-j)^2/ls^2 + log(var)."""
    x = np.arange(n, dtype=dtype)
    d2 = (x[:, None] - x[None, :]) ** 2
    val = np.exp(-d2 / dtype(ls) ** 2) * dtype(var)
    logval = -d2 / dtype(ls) ** 2 + np.log(dtype(var))
    return val, logval


def generate_basis(lengthscale, n_latent_bin, explained_variance_threshold_basis=0.999,
                   include_bias=True, custom_kernel=None, dtype=np.float32):
    """core.py:41-73.  SVD of the RBF tuning kernel, keep the first n_basis
    columns scaled by S^(1/4), prepend a ones column.  The reference computes
    in float32 (no x64 anywhere), so the default dtype is float32 so that the
    n_basis count (cumsum threshold, core.py:54) matches; column signs follow
    LAPACK gesdd as in jax (inject the basis for strict parity)."""
    if custom_kernel is not None:
        kmat = np.asarray(custom_kernel, dtype=dtype)
    else:
        kmat, _ = rbf_kernel_matrix(n_latent_bin, lengthscale, 1.0, dtype=dtype)
    u, s, _ = np.linalg.svd(kmat)
    n_basis = int((np.cumsum(s / s.sum()) < explained_variance_threshold_basis).sum()) + 1
    sqrt_eig = np.sqrt(np.sqrt(s))
    basis = u[:, :n_basis] * sqrt_eig[:n_basis][None, :]
    if include_bias:
        basis = np.concatenate([np.ones((n_latent_bin, 1), dtype=basis.dtype), basis], axis=1)
    return basis


def _get_log(v):
    """gp_kernel.py:8-12: log, with +inf mapped to -10000 (never hit for
    probabilities; kept for fidelity)."""
    with np.errstate(divide="ignore"):
        lv = np.log(v)
    return np.where(lv == np.inf, -10000.0, lv)


def create_transition_prob_1d(n_latent, movement_variance=1.0, p_move_to_jump=0.01,
                              p_jump_to_move=0.01, custom_kernel=None):
    """gp_kernel.py:42-89.  Returns (K (D,L,L), logK (D,L,L), A (D,D), logA (D,D)).
    logK[d_next, i_prev, j_next]; rows normalised over j (gp_kernel.py:76-78).
    Dynamics 0 = continuous (RBF or custom), 1 = jump (uniform 1/L)."""
    L = n_latent
    if custom_kernel is None:
        k0, lk0 = rbf_kernel_matrix(L, movement_variance, 1.0)            # gp_kernel.py:63
    else:
        k0 = np.asarray(custom_kernel, dtype=np.float64)                   # gp_kernel.py:30-34
        lk0 = _get_log(k0)
    k1 = np.full((L, L), 1.0 / L)                                          # gp_kernel.py:36-40
    lk1 = np.full((L, L), float(_get_log(np.float64(1.0 / L))))
    ks, lks = [], []
    for k, lk in ((k0, lk0), (k1, lk1)):
        z = k.sum(axis=1, keepdims=True)                                   # gp_kernel.py:76
        ks.append(k / z)
        lks.append(lk - np.log(z))                                         # gp_kernel.py:78
    A = np.array([[1 - p_move_to_jump, p_move_to_jump],
                  [p_jump_to_move, 1 - p_jump_to_move]], dtype=np.float64)  # gp_kernel.py:85
    return np.array(ks), np.array(lks), A, _get_log(A)


def softplus(x):
    """jax.nn.softplus = logaddexp(x, 0)."""
    return np.logaddexp(x, 0.0)


def sigmoid(x):
    return 0.5 * (1.0 + np.tanh(0.5 * x))


def get_tuning_softplus(params, basis):
    """fit_tuning_helper.py:19-25: softplus(basis @ params) -> (L, N)."""
    return softplus(np.asarray(basis, _F) @ np.asarray(params, _F))


# ----------------------------------------------------------------------------
# emission  (decoder.py:30-71, 73-85)
# ----------------------------------------------------------------------------
def loglikelihood_poisson_all(y, tuning, ma_neuron=None, ma_latent=None, dt=1.0):
    """decoder.py:30-48 vmapped over time (decoder.py:60-71; :73-85 for a per-time dt).
    ll[t,l] = sum_n m[t,n] * (xlogy(y[t,n], lam[l,n]) - lam[l,n] - gammaln(y[t,n]+1)),
    lam = tuning*dt + 1e-20; ll[:, ~ma_latent] = -1e20."""
    y = np.asarray(y, _F)
    tuning = np.asarray(tuning, _F)
    T, N = y.shape
    L = tuning.shape[0]
    m = np.ones((T, N), _F) if ma_neuron is None else np.broadcast_to(np.asarray(ma_neuron, _F), (T, N))
    dt = np.broadcast_to(np.asarray(dt, _F), (T,))
    if np.all(dt == dt[0]):
        lam = tuning * dt[0] + RATE_EPS                                     # (L, N)
        loglam = np.log(lam)
        # sum_n m*y*log(lam) - sum_n m*lam - sum_n m*gammaln(y+1)
        ll = (m * y) @ loglam.T - m @ lam.T - (m * gammaln(y + 1.0)).sum(1, keepdims=True)
        # xlogy(0, lam) = 0 exactly; log(lam) is finite (lam >= 1e-20) so the
        # matrix form is identical.
    else:
        ll = np.empty((T, L), _F)
        g = gammaln(y + 1.0)
        for t in range(T):
            lam = tuning * dt[t] + RATE_EPS
            ll[t] = ((xlogy(y[t][None, :], lam) - lam - g[t][None, :]) * m[t][None, :]).sum(1)
    if ma_latent is not None:
        ml = np.asarray(ma_latent).astype(bool)
        ll = np.where(ml[None, :], ll, NEG_MASK)                            # decoder.py:46
    return ll


# ----------------------------------------------------------------------------
# forward filter  (decoder.py:151-198)
# ----------------------------------------------------------------------------
def filter_one_step(post_prev, logz_prev, ll_t, logK, logA, likelihood_scale=1.0):
    """decoder.py:151-172.  post_prev (D,L) log; returns new carry and
    (post, prior, log one-step predictive marginal)."""
    a = logsumexp(post_prev[:, None, :] + logA[:, :, None], axis=0)       # :160-161 (D_next, L_i)
    prior = logsumexp(a[:, :, None] + logK, axis=1)                        # :163-164 (D_next, L_j)
    u = prior + likelihood_scale * ll_t[None, :]                           # :166
    c = logsumexp(u)                                                       # :167
    post = u - c                                                           # :168
    return post, logz_prev + c, prior, c


def filter_all_step(ll, logK, logA, carry_init=None, likelihood_scale=1.0):
    """decoder.py:174-187.  Default carry = uniform log(1/(D*L)) posterior
    "at t=-1" and zero log marginal (decoder.py:181-183)."""
    D, L = logA.shape[0], logK.shape[1]
    if carry_init is None:
        carry_init = (np.log(np.ones((D, L), _F) / (D * L)), 0.0)
    post, logz = carry_init
    T = ll.shape[0]
    posts = np.empty((T, D, L), _F)
    priors = np.empty((T, D, L), _F)
    cs = np.empty(T, _F)
    for t in range(T):
        post, logz, prior, c = filter_one_step(post, logz, ll[t], logK, logA, likelihood_scale)
        posts[t], priors[t], cs[t] = post, prior, c
    return posts, logz, priors, cs


# ----------------------------------------------------------------------------
# backward smoother  (decoder.py:200-256)
# ----------------------------------------------------------------------------
def smooth_one_step(acausal_next, joint, post_curr, prior_next, logK, logA, with_joint=True):
    """decoder.py:200-226.  X[d,d',i,j] = logK[d',i,j] + logA[d,d'] +
    (acausal_next - prior_next)[d',j] + post_curr[d,i]; acausal = LSE over (d',j);
    joint = logaddexp(joint, X)."""
    diff = acausal_next - prior_next                                       # :212
    X = (logK[None, :, :, :] + logA[:, :, None, None]
         + diff[None, :, None, :] + post_curr[:, None, :, None])           # :215
    acausal = logsumexp(X, axis=(1, 3))                                    # :217
    if with_joint:
        joint = np.logaddexp(joint, X)                                     # :221
    return acausal, joint


def smooth_all_step(causal_post, causal_prior, logK, logA, carry_init=None, with_joint=True):
    """decoder.py:230-256.  Last chunk (carry_init None): seed with the last
    causal posterior, joint = -1e40 (which is -inf in the reference's float32,
    the 'overflow encountered in cast' of moser_data_decoding_model.ipynb:395),
    scan the rest and append the seed.  causal_prior[k] is the prior of the
    time step after causal_post[k]."""
    D, L = logA.shape[0], logK.shape[1]
    if carry_init is None:
        do_concat = True
        acausal = causal_post[-1]
        joint = np.full((D, D, L, L), -np.inf, _F)
        xs_post = causal_post[:-1]
    else:
        do_concat = False
        acausal, joint = carry_init
        xs_post = causal_post
    n = xs_post.shape[0]
    out = np.empty((n, D, L), _F)
    for k in range(n - 1, -1, -1):                                          # scan(reverse=True) :248
        acausal, joint = smooth_one_step(acausal, joint, xs_post[k], causal_prior[k], logK, logA, with_joint)
        out[k] = acausal
    if do_concat:
        out = np.concatenate([out, causal_post[-1][None]], axis=0)         # :253-254
    return out, joint


def loglikelihood_gaussian_all(y, tuning, noise_std, ma_neuron=None, ma_latent=None, dt=1.0):
    """decoder.py:50-57 vmapped over time: ll[t,l] = sum_n m[t,n] *
    norm.logpdf(y[t,n], tuning[l,n]*dt, noise_std); ll[:, ~ma_latent] = -1e20.
    dt may be a per-time-bin array (decoder.py:73-85, get_loglikelihood_ma_all_changing_dt)."""
    y = np.asarray(y, _F)
    tun = np.asarray(tuning, _F)
    T, N = y.shape
    dt_t = np.broadcast_to(np.asarray(dt, _F), (T,))[:, None]
    m = np.ones((T, N), _F) if ma_neuron is None else np.broadcast_to(np.asarray(ma_neuron, _F), (T, N))
    s = float(noise_std)
    c0 = -math.log(s) - 0.5 * math.log(2 * math.pi)
    # sum_n m*(c0 - (y - tuning dt_t)^2 / (2 s^2)), expanded into matrix products
    ll = (c0 * m.sum(1, keepdims=True) - 0.5 / s ** 2 * ((m * y * y).sum(1, keepdims=True)
                                                         - 2.0 * dt_t * ((m * y) @ tun.T)
                                                         + dt_t ** 2 * (m @ (tun * tun).T)))
    if ma_latent is not None:
        ml = np.asarray(ma_latent).astype(bool)
        ll = np.where(ml[None, :], ll, NEG_MASK)
    return ll


def smooth_all_step_combined_ma_chunk(y, tuning, logK, logA, ma_neuron=None, ma_latent=None,
                                      likelihood_scale=1.0, n_time_per_chunk=10000, with_joint=True,
                                      noise_std=None):
    """decoder.py:258-332: forward filter chunk by chunk with carry
    (post[-1], logZ) (:299), then backward smoother over chunks in reverse
    with carry (acausal[0], joint) (:322); the prior slice for chunk n is
    [start+1, stop+1) of the concatenated priors (:315).
    Returns (log_acausal (T,D,L), log_marginal_final, log_causal (T,D,L),
    log_one_step_predictive_marginals (T,), log_joint (D,D,L,L), ll (T,L))."""
    T = y.shape[0]
    n_chunks = int(math.ceil(T / n_time_per_chunk))
    L = tuning.shape[0]
    if ma_latent is None:
        ma_latent = np.ones(L)
    ma_neuron_arr = None if ma_neuron is None else np.asarray(ma_neuron, _F)
    carry = None
    posts, priors, cs, lls, slices = [], [], [], [], []
    for n in range(n_chunks):
        sl = slice(n * n_time_per_chunk, (n + 1) * n_time_per_chunk)
        slices.append(sl)
        if ma_neuron_arr is not None and ma_neuron_arr.ndim == 2:
            mn = ma_neuron_arr[sl]
        else:
            mn = ma_neuron_arr
        if noise_std is None:
            ll = loglikelihood_poisson_all(y[sl], tuning, mn, ma_latent)
        else:                                               # observation_model='gaussian'
            ll = loglikelihood_gaussian_all(y[sl], tuning, noise_std, mn, ma_latent)
        p, logz, pr, c = filter_all_step(ll, logK, logA, carry_init=carry, likelihood_scale=likelihood_scale)
        carry = (p[-1], logz)
        posts.append(p); priors.append(pr); cs.append(c); lls.append(ll)
    prior_all = np.concatenate(priors, 0)
    cs = np.concatenate(cs, 0)
    ll_all = np.concatenate(lls, 0)
    carry = None
    acausal_chunks = []
    joint = None
    for n in range(n_chunks - 1, -1, -1):
        sl = slices[n]
        start, stop = sl.start, min(sl.stop, T)
        pr = prior_all[start + 1:stop + 1]
        ac, joint = smooth_all_step(posts[n], pr, logK, logA, carry_init=carry, with_joint=with_joint)
        carry = (ac[0], joint)
        acausal_chunks.append(ac)
    acausal_chunks.reverse()
    return (np.concatenate(acausal_chunks, 0), logz, np.concatenate(posts, 0), cs, joint, ll_all)


def compute_transition_posterior_prob(log_joint):
    """decoder.py:334-375 (dict keys in jax's sorted pytree order)."""
    ljf = log_joint - logsumexp(log_joint)
    ljl = logsumexp(ljf, axis=(0, 1))
    ljd = logsumexp(ljf, axis=(2, 3))
    ltl = ljl - logsumexp(ljl, axis=1, keepdims=True)
    ltd = ljd - logsumexp(ljd, axis=1, keepdims=True)
    ltf = ljf - logsumexp(ljf, axis=(1, 3), keepdims=True)
    res = {'p_joint_full': np.exp(ljf), 'p_joint_latent': np.exp(ljl), 'p_joint_dynamics': np.exp(ljd),
           'p_transition_full': np.exp(ltf), 'p_transition_latent': np.exp(ltl),
           'p_transition_dynamics': np.exp(ltd),
           'log_joint_full': ljf, 'log_joint_latent': ljl, 'log_joint_dynamics': ljd,
           'log_transition_full': ltf, 'log_transition_latent': ltl, 'log_transition_dynamics': ltd}
    return {k: res[k] for k in sorted(res)}


# ----------------------------------------------------------------------------
# M-step  (fit_tuning_helper.py:28-42, 63-81, 124-205)
# ----------------------------------------------------------------------------
def get_statistics(log_posterior_probs, y):
    """fit_tuning_helper.py:28-42: P = exp(logpost); y_w = P^T y (L,N); t_w = sum_t P (L)."""
    P = np.exp(np.asarray(log_posterior_probs, _F))
    return P.T @ np.asarray(y, _F), P.sum(0)


def poisson_m_step_objective(W, param_prior_std, basis, yw, tw):
    """fit_tuning_helper.py:63-81: -sum[xlogy(yw, f+1e-20) - f*tw] - sum norm.logpdf(W; 0, sd)."""
    f = softplus(basis @ W)
    ll = np.sum(xlogy(yw, f + RATE_EPS) - f * tw[:, None])
    sd = float(param_prior_std)
    logprior = np.sum(-0.5 * (W / sd) ** 2 - math.log(sd) - 0.5 * math.log(2 * math.pi))
    return -ll - logprior


def poisson_m_step_grad(W, param_prior_std, basis, yw, tw):
    """Analytic gradient of poisson_m_step_objective (what jax.value_and_grad
    evaluates at fit_tuning_helper.py:140,168): jvp of xlogy wrt its 2nd arg is
    x/y, of softplus is sigmoid."""
    F = basis @ W
    f = softplus(F)
    G = (yw / (f + RATE_EPS) - tw[:, None]) * sigmoid(F)
    return -(basis.T @ G) + W / float(param_prior_std) ** 2


def adam_init(W):
    """optax.adam(lr).init: ScaleByAdamState(count=0, mu=0, nu=0)."""
    return {'count': 0, 'mu': np.zeros_like(W, dtype=_F), 'nu': np.zeros_like(W, dtype=_F)}


def adam_update(g, state, W, lr, b1=0.9, b2=0.999, eps=1e-8, eps_root=0.0):
    """optax 0.2.2 scale_by_adam + scale(-lr) + apply_updates."""
    mu = (1 - b1) * g + b1 * state['mu']
    nu = (1 - b2) * g ** 2 + b2 * state['nu']
    count = state['count'] + 1
    mu_hat = mu / (1 - b1 ** count)
    nu_hat = nu / (1 - b2 ** count)
    upd = -lr * (mu_hat / (np.sqrt(nu_hat + eps_root) + eps))
    return W + upd, {'count': count, 'mu': mu, 'nu': nu}


def adam_run(W, state, param_prior_std, basis, yw, tw, lr=0.01, maxiter=1000, tol=1e-6):
    """fit_tuning_helper.py:133-194: loss/grad at W0 recorded at history[0];
    while i < maxiter-1 and (i < 5 or |loss-loss_prev|/max(|loss|,1e-8) > tol):
    (loss, g) at current W; W <- adam(W, g); history[i+1] = loss; loss_prev <- old loss.
    Returns n_iter = i+1 and final_loss = last evaluated loss (before the last update)."""
    basis = np.asarray(basis, _F)
    W = np.asarray(W, _F)
    loss = poisson_m_step_objective(W, param_prior_std, basis, yw, tw)
    g = poisson_m_step_grad(W, param_prior_std, basis, yw, tw)
    err = float(np.sqrt(np.sum(g * g)))
    lh = np.zeros(maxiter); eh = np.zeros(maxiter)
    lh[0], eh[0] = loss, err
    i, loss_prev = 0, loss
    while (i < maxiter - 1) and (i < 5 or abs(loss - loss_prev) / max(abs(loss), 1e-8) > tol):
        new_loss = poisson_m_step_objective(W, param_prior_std, basis, yw, tw)
        g = poisson_m_step_grad(W, param_prior_std, basis, yw, tw)
        W, state = adam_update(g, state, W, lr)
        new_err = float(np.sqrt(np.sum(g * g)))
        i += 1
        lh[i], eh[i] = new_loss, new_err
        loss_prev, loss, err = loss, new_loss, new_err
    return {'params': W, 'opt_state': state, 'n_iter': i + 1, 'final_loss': loss,
            'final_error': err, 'loss_history': lh, 'error_history': eh}


def m_step(W, y, log_posterior_curr, basis, param_prior_std, opt_state, lr=0.01, maxiter=1000, tol=1e-6,
           stats_perturb=None):
    """core.py:802-827: suff-stats -> Adam -> trimmed histories.

    stats_perturb = (rng, eps) multiplies y_w and t_w by (1 + eps * N(0, 1)) elementwise
    before the Adam loop.  Not part of the reference: the golden generator uses it to run
    an ensemble of f64 fits whose statistics differ at the level of summation-order
    rounding (eps = 1e-15), which measures how far rounding alone moves a long M-step."""
    yw, tw = get_statistics(log_posterior_curr, y)
    if stats_perturb is not None:
        rng, eps = stats_perturb
        yw = yw * (1.0 + eps * rng.standard_normal(yw.shape))
        tw = tw * (1.0 + eps * rng.standard_normal(tw.shape))
    res = adam_run(W, opt_state, param_prior_std, basis, yw, tw, lr, maxiter, tol)
    n = res['n_iter']
    return {'params': res['params'], 'opt_state': res['opt_state'], 'n_iter': n,
            'final_loss': res['final_loss'], 'final_error': res['final_error'],
            'loss_history': res['loss_history'][:n], 'error_history': res['error_history'][:n]}


# ----------------------------------------------------------------------------
# EM driver / decode  (core.py:454-524, 592-713, 829-849)
# ----------------------------------------------------------------------------
def fit_em(y, params, basis, log_posterior_init, n_iter=20, movement_variance=1.0,
           p_move_to_jump=0.01, p_jump_to_move=0.01, param_prior_std=1.0, ma_neuron=None,
           ma_latent=None, n_time_per_chunk=10000, likelihood_scale=1.0, save_every=None,
           m_step_step_size=0.01, m_step_maxiter=1000, m_step_tol=1e-6, custom_kernel=None,
           stats_perturb=None):
    """core.py:829-849 + core.py:592-713 with injected params / basis /
    log_posterior_init (JAX PRNG is not reproducible without JAX).  stats_perturb: see
    m_step (ensemble runs of the golden generator only)."""
    y = np.asarray(y, _F)
    L = basis.shape[0]
    if save_every is None:
        save_every = n_iter
    _, logK, _, logA = create_transition_prob_1d(L, movement_variance, p_move_to_jump, p_jump_to_move, custom_kernel)
    logK, logA = logK.astype(_F), logA.astype(_F)
    opt_state = adam_init(params)                                          # core.py:847
    W = np.asarray(params, _F)
    basis = np.asarray(basis, _F)
    logpost = np.asarray(log_posterior_init, _F)
    log_marginal_l, saved = [], {'log_posterior_all_saved': [], 'params_saved': [],
                                 'tuning_saved': [], 'iter_saved': [], 'log_marginal_saved': []}
    m_step_res_l = {}
    for i in range(n_iter):
        m_res = m_step(W, y, logpost, basis, param_prior_std, opt_state, m_step_step_size,
                       m_step_maxiter, m_step_tol, stats_perturb)
        if i == 0:
            m_step_res_l = {k: [] for k in m_res.keys()}                   # core.py:655
        for k in m_res:
            if k not in ('params', 'opt_state'):
                m_step_res_l[k].append(m_res[k])
        W, opt_state = m_res['params'], m_res['opt_state']
        tuning = get_tuning_softplus(W, basis)                             # core.py:664
        out = smooth_all_step_combined_ma_chunk(y, tuning, logK, logA, ma_neuron, ma_latent,
                                                likelihood_scale, n_time_per_chunk, with_joint=False)
        log_post_all, logz = out[0], out[1]
        logpost = logsumexp(log_post_all, axis=1)                          # core.py:668
        log_marginal_l.append(logz)
        if i % save_every == 0:
            saved['log_posterior_all_saved'].append(log_post_all)
            saved['params_saved'].append(W)
            saved['tuning_saved'].append(tuning)
            saved['log_marginal_saved'].append(logz)
            saved['iter_saved'].append(i)
    posterior = np.exp(log_post_all)
    return {'log_posterior_all_saved': saved['log_posterior_all_saved'],
            'log_posterior_init': log_posterior_init, 'params_saved': saved['params_saved'],
            'tuning_saved': saved['tuning_saved'], 'iter_saved': saved['iter_saved'],
            'params': W, 'tuning': tuning, 'log_posterior_final': log_post_all,
            'log_marginal': logz, 'log_marginal_l': log_marginal_l,
            'log_marginal_saved': saved['log_marginal_saved'], 'posterior': posterior,
            'posterior_latent_marg': posterior.sum(1), 'posterior_dynamics_marg': posterior.sum(2),
            'm_step_res_l': m_step_res_l, 'opt_state': opt_state}


def gaussian_m_step_analytic(basis, yw, tw, noise_std, param_prior_std):
    """fit_tuning_helper.py:44-61: W = solve(B^T diag(tw) B / s^2 + I / p^2, B^T yw / s^2)."""
    B = np.asarray(basis, _F)
    G = np.einsum('qd,q,qb->db', B, np.asarray(tw, _F), B)
    H = G / noise_std ** 2 + np.eye(B.shape[1]) / param_prior_std ** 2
    return np.linalg.solve(H, B.T @ np.asarray(yw, _F) / noise_std ** 2)


def fit_em_gaussian(y, params, basis, log_posterior_init, n_iter=20, movement_variance=1.0,
                    p_move_to_jump=0.01, p_jump_to_move=0.01, noise_std=0.5, param_prior_std=1.0,
                    ma_neuron=None, ma_latent=None, likelihood_scale=1.0, stats_dtype=None):
    """GaussianGPLVMJump1D.fit_em (core.py:905-917) over AbstractGPLVMJump1D.fit_em
    (core.py:592-713): analytic M-step (core.py:898-904), linear tuning
    (fit_tuning_helper.py:12-17), Gaussian emission.  Returns params, tuning,
    posterior, log_marginal_l.  stats_dtype (e.g. np.float32) rounds y_w, t_w to that
    type before the solve: the tests use it to measure how far fp32 sufficient
    statistics alone move the fit (the noise floor of an fp32-stats implementation)."""
    y = np.asarray(y, _F)
    L = basis.shape[0]
    _, logK, _, logA = create_transition_prob_1d(L, movement_variance, p_move_to_jump, p_jump_to_move)
    W = np.asarray(params, _F)
    basis = np.asarray(basis, _F)
    logpost = np.asarray(log_posterior_init, _F)
    lml = []
    for i in range(n_iter):
        yw, tw = get_statistics(logpost, y)
        if stats_dtype is not None:
            yw, tw = yw.astype(stats_dtype).astype(_F), tw.astype(stats_dtype).astype(_F)
        W = gaussian_m_step_analytic(basis, yw, tw, noise_std, param_prior_std)
        tuning = basis @ W
        out = smooth_all_step_combined_ma_chunk(y, tuning, logK.astype(_F), logA.astype(_F), ma_neuron, ma_latent,
                                                likelihood_scale, with_joint=False, noise_std=noise_std)
        lpa, logz = out[0], out[1]
        logpost = logsumexp(lpa, axis=1)
        lml.append(logz)
    post = np.exp(lpa)
    return {'params': W, 'tuning': tuning, 'posterior': post, 'posterior_latent_marg': post.sum(1),
            'log_marginal_l': lml, 'log_marginal': lml[-1]}


def decode_latent(y, tuning, movement_variance=1.0, p_move_to_jump=0.01, p_jump_to_move=0.01,
                  ma_neuron=None, ma_latent=None, likelihood_scale=1.0, n_time_per_chunk=10000,
                  custom_kernel=None):
    """core.py:454-497 (+ decoder.compute_transition_posterior_prob)."""
    L = tuning.shape[0]
    _, logK, _, logA = create_transition_prob_1d(L, movement_variance, p_move_to_jump, p_jump_to_move, custom_kernel)
    logK, logA = logK.astype(_F), logA.astype(_F)
    lpa, logz, _, cs, joint, ll = smooth_all_step_combined_ma_chunk(
        np.asarray(y, _F), np.asarray(tuning, _F), logK, logA, ma_neuron, ma_latent,
        likelihood_scale, n_time_per_chunk, with_joint=True)
    post = np.exp(lpa)
    res = {'log_posterior_all': lpa, 'log_marginal_final': float(logz), 'posterior_all': post,
           'posterior_latent_marg': post.sum(1), 'posterior_dynamics_marg': post.sum(2),
           'log_one_step_predictive_marginals_all': cs, 'log_likelihood_all': ll}
    res.update(compute_transition_posterior_prob(joint))
    return res


def naive_bayes_chunk(y, tuning, ma_neuron=None, ma_latent=None, dt_l=1.0, n_time_per_chunk=10000):
    """decoder.py:88-149: per-time emission (dt per row), row-normalised."""
    y = np.asarray(y, _F)
    T = y.shape[0]
    dt_l = np.broadcast_to(np.asarray(dt_l, _F), (T,))
    ll = loglikelihood_poisson_all(y, tuning, ma_neuron, ma_latent, dt_l)
    lm = logsumexp(ll, axis=-1, keepdims=True)
    return ll - lm, lm[:, 0], float(lm.sum()), ll


# ----------------------------------------------------------------------------
# latent-only model (decoder_latentonly.py, core.py:76-375 / :919-1019)
# ----------------------------------------------------------------------------
def create_transition_prob_latent_1d(n_latent, movement_variance=1.0):
    """gp_kernel.py:92-118: row-normalised RBF over latent bins (the same kernel as
    the jump model's continuous dynamics, create_transition_prob_1d logK[0])."""
    K, logK, _, _ = create_transition_prob_1d(n_latent, movement_variance)
    return K[0], logK[0]


def smooth_latent_only(y, tuning, logK, ma_neuron=None, ma_latent=None, likelihood_scale=1.0, noise_std=None):
    """decoder_latentonly.py:34-226 in one chunk (the chunk carries are exact, so the
    result does not depend on n_time_per_chunk): filter from log(1/L)
    (:58-80), RTS smoother seeded with the last filter posterior and a -1e40 joint
    (:126-154).  Returns (acausal (T,L), logZ, causal (T,L), log c_t (T), joint (L,L),
    ll (T,L))."""
    if noise_std is None:
        ll = loglikelihood_poisson_all(y, tuning, ma_neuron, ma_latent)
    else:                                                   # observation_model='gaussian'
        ll = loglikelihood_gaussian_all(y, tuning, noise_std, ma_neuron, ma_latent)
    T, L = ll.shape
    post = np.log(np.ones(L, _F) / L)
    logz = 0.0
    causal = np.empty((T, L), _F)
    prior = np.empty((T, L), _F)
    cs = np.empty(T, _F)
    for t in range(T):
        pr = logsumexp(post[:, None] + logK, axis=0)                        # :45-48
        u = pr + likelihood_scale * ll[t]
        c = logsumexp(u)
        post = u - c
        logz += c
        causal[t], prior[t], cs[t] = post, pr, c
    acausal = np.empty((T, L), _F)
    acausal[T - 1] = causal[T - 1]
    joint = np.full((L, L), -1e40, _F)
    for t in range(T - 2, -1, -1):
        inside = logK + (acausal[t + 1] - prior[t + 1])[None, :] + causal[t][:, None]   # :109-112
        acausal[t] = logsumexp(inside, axis=1)
        joint = np.logaddexp(joint, inside)
    return acausal, float(logz), causal, cs, joint, ll


def compute_transition_posterior_prob_latent(log_joint):
    """decoder_latentonly.py:227-252."""
    lj = log_joint - logsumexp(log_joint)
    lt = lj - logsumexp(lj, axis=1, keepdims=True)
    return {'p_joint_latent': np.exp(lj), 'p_transition_latent': np.exp(lt),
            'log_joint_latent': lj, 'log_transition_latent': lt}


# ----------------------------------------------------------------------------
# synthetic data (numpy RNG; the reference's JAX PRNG cannot be reproduced)
# ----------------------------------------------------------------------------
def init_latent_posterior_from_uniform(u, random_scale=0.1):
    """core.py:571-583 given the uniform draws u (T,L): p = u*scale, row-normalise, log."""
    p = np.asarray(u, np.float64) * random_scale
    p = p / p.sum(1, keepdims=True)
    with np.errstate(divide='ignore'):
        lp = np.log(p)
    return np.where(lp == -np.inf, -1e40, lp)


def sample_latent(T, L, rng, movement_variance=1.0, p_move_to_jump=0.01, p_jump_to_move=0.01):
    """core.py:526-555 restated with a numpy Generator: dynamics first from
    A[prev], then latent from K[dyn_curr][latent_prev]."""
    K, _, A, _ = create_transition_prob_1d(L, movement_variance, p_move_to_jump, p_jump_to_move)
    d = int(rng.integers(2)); l = int(rng.integers(L))
    out = np.empty((T, 2), np.int64)
    cK = np.cumsum(K, axis=2)
    cA = np.cumsum(A, axis=1)
    u = rng.random((T, 2))
    for t in range(T):
        d = int(min(np.searchsorted(cA[d], u[t, 0] * cA[d, -1], side='right'), 1))
        l = int(min(np.searchsorted(cK[d, l], u[t, 1] * cK[d, l, -1], side='right'), L - 1))
        out[t] = (d, l)
    return out


def sample_spikes(tuning, latent, rng, dt=1.0):
    """core.py:795-800: y ~ Poisson(tuning[latent] * dt)."""
    return rng.poisson(np.asarray(tuning, np.float64)[latent] * dt)


def jump_consensus(jump_p, jump_p_all_chain, window_size=5, jump_p_thresh=0.4, consensus_thresh=0.8):
    """model_selection_helper.py:264-299, as scalar Python loops over chains and
    window rows (the window is jump_p_all_chain[jti-window_size : jti+window_size],
    numpy slice rules, negative start included)."""
    T, n_chain = np.asarray(jump_p_all_chain).shape
    ok_l, keep = [], []
    for jti in range(len(jump_p)):
        if not jump_p[jti] >= jump_p_thresh:
            continue
        rows = list(range(T))[jti - window_size:jti + window_size]
        n_hit = 0
        for c in range(n_chain):
            if any(jump_p_all_chain[r][c] > jump_p_thresh for r in rows):
                n_hit += 1
        ok = (n_hit / n_chain) >= consensus_thresh
        ok_l.append(ok)
        if ok:
            keep.append(jti)
    frac = float(np.mean(ok_l)) if ok_l else float('nan')
    filt = np.zeros(len(jump_p))
    filt[keep] = 1
    return frac, filt, np.array(ok_l, dtype=bool)


def downsampled_lml(y, tuning, masks, movement_variance=1.0, p_move_to_jump=0.01, p_jump_to_move=0.01,
                    ma_neuron=None, likelihood_scale=1.0):
    """model_selection_helper.py:243-260 with the latent masks given explicitly:
    log_marginal_final of one decode per mask, and their mean / std."""
    L = tuning.shape[0]
    _, logK, _, logA = create_transition_prob_1d(L, movement_variance, p_move_to_jump, p_jump_to_move)
    lml = []
    for m in masks:
        _, logz, *_ = smooth_all_step_combined_ma_chunk(np.asarray(y, _F), np.asarray(tuning, _F), logK.astype(_F),
                                                        logA.astype(_F), ma_neuron, np.asarray(m), likelihood_scale,
                                                        with_joint=False)
        lml.append(float(logz))
    lml = np.array(lml)
    return lml, lml.mean(), lml.std()


def circular_shuffle_once(y, rng_randint=np.random.randint):
    """test.py:19-24, one shuffle: column j rolled by randint(0, n_time), drawn per
    neuron in column order.  Returns (shuffled copy, shifts)."""
    y = np.asarray(y)
    n_time, n_neuron = y.shape
    out = y.copy()
    shifts = np.zeros(n_neuron, dtype=np.int64)
    for j in range(n_neuron):
        shifts[j] = rng_randint(0, n_time)
        out[:, j] = np.roll(y[:, j], shifts[j])
    return out, shifts


def compute_entropy(logp_l, axis=(-1, -2)):
    """test.py:70-79 with p = 0 states contributing 0."""
    p = np.exp(np.asarray(logp_l, np.float64))
    with np.errstate(invalid='ignore', divide='ignore'):
        return -np.sum(np.where(p > 0, p * np.log(np.where(p > 0, p, 1.0)), 0.0), axis=axis)
