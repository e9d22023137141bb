"""Oracle M-step: objective gradient, optax-0.2.2 Adam, the while-loop stop rule
(fit_tuning_helper.py:63-81, :124-196).  CPU only."""
import math
import os

import numpy as np

from oracle import gplvm_oracle as O


def _problem(seed=0, L=12, NB=5, N=4):
    rng = np.random.default_rng(seed)
    B = O.generate_basis(3.0, L).astype(np.float64)[:, :NB]
    W = rng.normal(size=(B.shape[1], N))
    yw = rng.gamma(2.0, 3.0, size=(L, N))
    yw[0, 0] = 0.0                              # xlogy(0, .) path
    tw = rng.gamma(2.0, 5.0, size=L)
    return B, W, yw, tw


def test_gradient_matches_finite_differences():
    B, W, yw, tw = _problem()
    g = O.poisson_m_step_grad(W, 1.3, B, yw, tw)
    eps = 1e-6
    num = np.zeros_like(W)
    for i in range(W.shape[0]):
        for j in range(W.shape[1]):
            Wp, Wm = W.copy(), W.copy()
            Wp[i, j] += eps
            Wm[i, j] -= eps
            num[i, j] = (O.poisson_m_step_objective(Wp, 1.3, B, yw, tw) -
                         O.poisson_m_step_objective(Wm, 1.3, B, yw, tw)) / (2 * eps)
    np.testing.assert_allclose(g, num, rtol=1e-6, atol=1e-6)


def test_objective_prior_term():
    B, W, yw, tw = _problem()
    sd = 0.7
    f = np.logaddexp(B @ W, 0)
    from scipy.special import xlogy
    ll = np.sum(xlogy(yw, f + 1e-20) - f * tw[:, None])
    lp = np.sum(-0.5 * (W / sd) ** 2 - math.log(sd) - 0.5 * math.log(2 * math.pi))
    assert abs(O.poisson_m_step_objective(W, sd, B, yw, tw) - (-ll - lp)) < 1e-9


def test_adam_update_hand_derived():
    """optax 0.2.2: mu/nu EMAs, bias correction with count+1, eps outside sqrt, -lr."""
    g = np.array([[0.5, -2.0]])
    W = np.array([[1.0, 1.0]])
    st = O.adam_init(W)
    W1, st1 = O.adam_update(g, st, W, 0.01)
    # first step: mu_hat = g, nu_hat = g^2 -> update = -lr * g/(|g| + 1e-8)
    np.testing.assert_allclose(W1, W - 0.01 * g / (np.abs(g) + 1e-8), rtol=1e-12)
    assert st1['count'] == 1
    g2 = np.array([[0.1, 0.3]])
    W2, st2 = O.adam_update(g2, st1, W1, 0.01)
    mu = 0.9 * (0.1 * g) + 0.1 * g2
    nu = 0.999 * (0.001 * g ** 2) + 0.001 * g2 ** 2
    upd = -0.01 * (mu / (1 - 0.9 ** 2)) / (np.sqrt(nu / (1 - 0.999 ** 2)) + 1e-8)
    np.testing.assert_allclose(W2, W1 + upd, rtol=1e-12)


def test_adam_loop_semantics():
    """History[0] and [1] are both the loss at W0; n_iter = bodies + 1; the loop runs
    at least 5 bodies; final_loss is the last evaluated loss (before the last update)."""
    B, W, yw, tw = _problem(1)
    r = O.adam_run(W, O.adam_init(W), 1.0, B, yw, tw, lr=0.01, maxiter=50, tol=1e-3)
    n = r['n_iter']
    assert 6 <= n <= 50
    lh = r['loss_history']
    assert lh[0] == lh[1]
    assert np.all(lh[n:] == 0)
    assert r['final_loss'] == lh[n - 1]
    # replay by hand
    Wc, st = W.copy(), O.adam_init(W)
    for _ in range(n - 1):
        Wc, st = O.adam_update(O.poisson_m_step_grad(Wc, 1.0, B, yw, tw), st, Wc, 0.01)
    np.testing.assert_allclose(r['params'], Wc, rtol=1e-12)
    # stop rule at n: relative change <= tol (or maxiter reached)
    rel = abs(lh[n - 1] - lh[n - 2]) / max(abs(lh[n - 1]), 1e-8)
    assert rel <= 1e-3 or n == 50


def test_adam_maxiter_one_is_evaluation_only():
    B, W, yw, tw = _problem(2)
    r = O.adam_run(W, O.adam_init(W), 1.0, B, yw, tw, maxiter=1)
    assert r['n_iter'] == 1
    np.testing.assert_array_equal(r['params'], W)


def test_fixed_iterations_with_tol_zero():
    B, W, yw, tw = _problem(3)
    r = O.adam_run(W, O.adam_init(W), 1.0, B, yw, tw, maxiter=17, tol=0.0)
    assert r['n_iter'] == 17


def test_working_precision_mimic_is_float32_and_restores():
    """oracle.working_precision(np.float32) = the reference's own fp32 arithmetic
    (used to size the reference's rounding noise in the EM goldens)."""
    f = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'decode_small.npz'))
    with O.working_precision(np.float32):
        r32 = O.decode_latent(f['y'], f['tuning'].astype(np.float32), movement_variance=float(f['mv']))
    assert r32['posterior_all'].dtype == np.float32
    assert O._F is np.float64
    r64 = O.decode_latent(f['y'].astype(np.float64), f['tuning'], movement_variance=float(f['mv']))
    d = np.abs(r32['posterior_all'] - r64['posterior_all']).max()
    assert 0 < d < 1e-2
