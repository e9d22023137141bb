"""Oracle (f64 numpy restatement of decoder.py) vs brute-force path enumeration.
CPU only."""
import numpy as np
import pytest

from oracle import gplvm_oracle as O
from oracle import brute


def run_oracle_on_ll(ll, logK, logA, s, chunk):
    """Drive the oracle's chunked filter/smoother (decoder.py:258-332) on a given ll."""
    T, L = ll.shape
    orig = O.loglikelihood_poisson_all
    try:
        O.loglikelihood_poisson_all = lambda yy, tt, mn, ml, dt=1.0: ll[yy[:, 0].astype(int)]
        yy = np.arange(T)[:, None] * np.ones((1, 2))
        return O.smooth_all_step_combined_ma_chunk(yy, np.zeros((L, 2)), logK, logA,
                                                   likelihood_scale=s, n_time_per_chunk=chunk)
    finally:
        O.loglikelihood_poisson_all = orig


@pytest.mark.parametrize("L,T,pmj,pjm,mv,s", [
    (2, 4, 0.01, 0.01, 1.0, 1.0),
    (3, 5, 0.1, 0.2, 1.0, 0.7),
    (4, 3, 0.3, 0.05, 0.5, 2.0),
    (3, 1, 0.01, 0.01, 1.0, 1.0),
    (3, 2, 0.0, 0.5, 1.0, 1.0),
])
@pytest.mark.parametrize("chunk", [1, 2, 10000])
def test_filter_smoother_joint_vs_enumeration(L, T, pmj, pjm, mv, s, chunk):
    rng = np.random.default_rng(L * 100 + T)
    K, logK, A, logA = O.create_transition_prob_1d(L, mv, pmj, pjm)
    ll = rng.normal(size=(T, L)) * 2.0
    post, joint, logZ, cs = brute.enumerate_posteriors(ll, K, A, s)
    lpa, lz, lca, c, lj, _ = run_oracle_on_ll(ll, logK, logA, s, chunk)
    np.testing.assert_allclose(np.exp(lpa), post, atol=1e-12)
    np.testing.assert_allclose(lz, logZ, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(c, cs, atol=1e-12)
    if T > 1:
        np.testing.assert_allclose(np.exp(lj), joint, atol=1e-12)
    else:
        assert np.all(np.isneginf(lj))   # the -1e40 initial joint (f32: -inf) is never updated


def test_masked_latents_vs_enumeration():
    L, T = 4, 4
    K, logK, A, logA = O.create_transition_prob_1d(L, 1.0, 0.05, 0.05)
    ll = np.random.default_rng(3).normal(size=(T, L))
    ll[:, 1] = O.NEG_MASK                       # decoder.py:46
    post, joint, logZ, _ = brute.enumerate_posteriors(ll, K, A, 1.0)
    lpa, lz, *_ = run_oracle_on_ll(ll, logK, logA, 1.0, 10000)
    np.testing.assert_allclose(np.exp(lpa), post, atol=1e-12)
    assert np.all(np.exp(lpa)[:, :, 1] < 1e-300)


def test_transition_kernel_orientation():
    """gp_kernel.py:42-89: logK[d_next, i_prev, j_next], rows normalised over j."""
    K, logK, A, logA = O.create_transition_prob_1d(7, 1.5, 0.02, 0.03)
    np.testing.assert_allclose(K.sum(axis=2), 1.0, atol=1e-14)
    np.testing.assert_allclose(np.exp(logK), K, rtol=1e-12)
    np.testing.assert_allclose(K[1], 1.0 / 7)
    np.testing.assert_allclose(A, [[0.98, 0.02], [0.03, 0.97]])
    x = np.arange(7.0)
    np.testing.assert_allclose(K[0][2], np.exp(-(x - 2) ** 2 / 1.5 ** 2) / np.exp(-(x - 2) ** 2 / 1.5 ** 2).sum())


def test_emission_formula():
    """decoder.py:30-48 on a hand case incl. xlogy(0, .) = 0, masks and -1e20."""
    y = np.array([[0., 2., 1.], [3., 0., 0.]])
    tun = np.array([[0.5, 1.0, 2.0], [1e-30, 3.0, 0.1]])
    ma = np.array([1., 0., 1.])
    ml = np.array([1, 0])
    ll = O.loglikelihood_poisson_all(y, tun, ma, ml)
    from scipy.special import gammaln, xlogy
    lam = tun + 1e-20
    exp0 = sum(ma[n] * (xlogy(y[0, n], lam[0, n]) - lam[0, n] - gammaln(y[0, n] + 1)) for n in range(3))
    exp1 = sum(ma[n] * (xlogy(y[1, n], lam[0, n]) - lam[0, n] - gammaln(y[1, n] + 1)) for n in range(3))
    np.testing.assert_allclose(ll[:, 0], [exp0, exp1], rtol=1e-14)
    assert np.all(ll[:, 1] == -1e20)


@pytest.mark.parametrize("L,T,mv,s", [(3, 4, 1.0, 1.0), (4, 3, 0.5, 0.6), (2, 1, 1.0, 1.0), (5, 3, 2.0, 1.3)])
def test_latent_only_vs_enumeration(L, T, mv, s):
    """decoder_latentonly restatement (D = 1) vs path enumeration."""
    rng = np.random.default_rng(L * 10 + T)
    K, logK = O.create_transition_prob_latent_1d(L, mv)
    ll = rng.normal(size=(T, L)) * 2.0
    post, joint, logZ, cs = brute.enumerate_posteriors(ll, K[None], np.ones((1, 1)), s)
    orig = O.loglikelihood_poisson_all
    try:
        O.loglikelihood_poisson_all = lambda yy, tt, mn, ml, dt=1.0: ll
        lpa, lz, lca, c, lj, _ = O.smooth_latent_only(np.zeros((T, 2)), np.zeros((L, 2)), logK, likelihood_scale=s)
    finally:
        O.loglikelihood_poisson_all = orig
    np.testing.assert_allclose(np.exp(lpa), post[:, 0], atol=1e-12)
    np.testing.assert_allclose(lz, logZ, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(c, cs, atol=1e-12)
    if T > 1:
        np.testing.assert_allclose(np.exp(lj), joint[0, 0], atol=1e-12)
