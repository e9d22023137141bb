"""Oracle checks for the Gaussian observation model (CPU): the emission against
scipy.stats.norm.logpdf element by element (decoder.py:50-57), and the analytic
M-step (fit_tuning_helper.py:44-61) as the stationary point of the expected
complete-data log posterior: B^T (y_w - diag(t_w) B W) / s^2 - W / p^2 = 0."""
import numpy as np
import pytest
from scipy.stats import norm

from oracle import gplvm_oracle as O


@pytest.mark.parametrize("masked", [False, True])
def test_gaussian_loglik_vs_scipy(masked):
    rng = np.random.default_rng(0)
    T, N, L = 40, 9, 13
    y = rng.normal(size=(T, N))
    tu = rng.normal(size=(L, N))
    ma = (rng.random((T, N)) > 0.3).astype(float) if masked else None
    ml = (rng.random(L) > 0.3).astype(float) if masked else None
    got = O.loglikelihood_gaussian_all(y, tu, 0.7, ma, ml, dt=1.5)
    m = np.ones((T, N)) if ma is None else ma
    ref = (norm.logpdf(y[:, None, :], 1.5 * tu[None], 0.7) * m[:, None, :]).sum(-1)
    if ml is not None:
        ref[:, ml == 0] = -1e20
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-9)


def test_gaussian_m_step_is_stationary():
    rng = np.random.default_rng(1)
    L, N = 60, 7
    B = O.generate_basis(5.0, L)
    P = rng.random((300, L))
    P /= P.sum(1, keepdims=True)
    y = rng.normal(size=(300, N))
    yw, tw = O.get_statistics(np.log(P), y)
    s, p = 0.4, 2.0
    W = O.gaussian_m_step_analytic(B, yw, tw, s, p)
    grad = B.T @ (yw - tw[:, None] * (B @ W)) / s ** 2 - W / p ** 2
    assert np.abs(grad).max() < 1e-8 * np.abs(B.T @ yw / s ** 2).max()
