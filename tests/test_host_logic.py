"""Host-side logic of the product package (no GPU): basis, banded transition,
reference API facts, constructor.  The oracle is used only as the checker."""
import json
import os

import numpy as np
import pytest

from oracle import gplvm_oracle as O
import poor_man_gplvm_amd as P
from poor_man_gplvm_amd.gp_kernel import banded_transition

HERE = os.path.dirname(os.path.abspath(__file__))
API = json.load(open(os.path.join(HERE, 'golden', 'reference_api.json')))


@pytest.mark.parametrize("L", [100, 256, 512])
def test_generate_basis_matches_oracle(L):
    b = P.generate_basis(10.0, L)
    o = O.generate_basis(10.0, L)
    assert b.shape == o.shape
    assert b.shape[1] == API['n_basis_ls10'][str(L)]      # 18 / 41 / 79
    np.testing.assert_allclose(np.abs(b), np.abs(o), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(b[:, 0], 1.0)


@pytest.mark.parametrize("L,mv", [(100, 1.0), (512, 1.0), (37, 0.5), (256, 2.0), (64, 3.5)])
def test_banded_transition_matches_dense(L, mv):
    tr = banded_transition(L, mv, 0.02, 0.03)
    K, logK, A, logA = P.create_transition_prob_1d(L, mv, 0.02, 0.03)
    Ko, _, Ao, _ = O.create_transition_prob_1d(L, mv, 0.02, 0.03)
    np.testing.assert_allclose(K, Ko, rtol=1e-12)
    np.testing.assert_allclose(tr.A, Ao)
    i, j = np.meshgrid(np.arange(L), np.arange(L), indexing='ij')
    d = np.abs(i - j)
    Kb = np.where(d <= tr.band, tr.g[np.minimum(d, tr.band)].astype(np.float64) * tr.invz[:, None], 0.0)
    np.testing.assert_allclose(Kb, np.where(d <= tr.band, K[0], 0.0), rtol=1e-6, atol=1e-37)
    assert np.max(np.where(d > tr.band, K[0], 0.0)) < 1e-29   # truncated mass is negligible


def test_band_limit_raises():
    with pytest.raises(NotImplementedError):
        banded_transition(512, 10.0)


def test_transition_selection():
    """Banded scans when the continuous kernel is a <= 32-bin RBF band, dense log-domain
    scans otherwise; kernels passed as logs are recovered in the same forms."""
    from poor_man_gplvm_amd.gp_kernel import (DenseTransition, BandedTransition, make_transition,
                                              transition_from_log_kernels, create_transition_prob_1d)
    assert isinstance(make_transition(100, 1.0), BandedTransition)
    assert isinstance(make_transition(100, 10.0), DenseTransition)
    L = 50
    Kc = np.exp(-np.abs(np.arange(L)[:, None] - np.arange(L)[None, :]) / 3.0)
    assert isinstance(make_transition(L, 1.0, custom_kernel=Kc), DenseTransition)
    _, lk, _, la = create_transition_prob_1d(L, 2.0, 0.05, 0.02)
    tr = transition_from_log_kernels(lk, la)
    ref = banded_transition(L, 2.0, 0.05, 0.02)
    assert isinstance(tr, BandedTransition) and tr.band <= ref.band
    np.testing.assert_allclose(tr.g, ref.g[:tr.band + 1], rtol=1e-6)
    assert np.all(ref.g[tr.band + 1:] < 1e-30)
    np.testing.assert_allclose(tr.invz, ref.invz, rtol=1e-6)
    np.testing.assert_allclose(tr.A, ref.A, rtol=1e-12)
    _, lk, _, la = create_transition_prob_1d(L, 1.0, custom_kernel=Kc)
    assert isinstance(transition_from_log_kernels(lk, la), DenseTransition)
    assert isinstance(transition_from_log_kernels(*create_transition_prob_1d(L, 1.0)[1::2], force_dense=True),
                      DenseTransition)
    lk_bad = lk.copy()
    lk_bad[1, 0, 0] += 1.0
    with pytest.raises(NotImplementedError):
        transition_from_log_kernels(lk_bad, la)


def test_log_joint_never_nan():
    """Underflowed joint counts (unvisited states) keep finite log values and normalise
    to the prior transition; masked latents keep the -1e20 sentinel sums."""
    from poor_man_gplvm_amd.core import log_joint_from_counts, compute_transition_posterior_prob
    L = 6
    _, logK, _, logA = P.create_transition_prob_1d(L, 1.0)
    S4 = np.random.default_rng(0).random((2, 2, L, L))
    S4[0, :, 2, :] = 0.0                  # state (d=0, i=2) never visited
    lj = log_joint_from_counts(S4, logK, logA)
    assert np.all(np.isfinite(lj))
    with np.errstate(invalid='raise', divide='raise'):
        r = compute_transition_posterior_prob(lj)
    for k, v in r.items():
        assert np.all(np.isfinite(v)), k
    row = r['p_transition_full'][0, :, 2, :].astype(np.float64)
    prior = np.exp(logA[0][:, None] + logK[:, 2, :])
    np.testing.assert_allclose(row, prior / prior.sum(), rtol=1e-5)


def test_constructor_and_api_without_gpu():
    m = P.PoissonGPLVMJump1D(30, n_latent_bin=100, tuning_lengthscale=10.)
    assert m.tuning_basis.shape == (100, 18)
    assert m.params.shape == (18, 30)
    lp, p = m.init_latent_posterior(50, 3)
    np.testing.assert_allclose(np.exp(lp).sum(1), 1.0, rtol=1e-5)
    lat = m.sample_latent(200, key=1)
    assert lat.shape == (200, 2) and lat[:, 0].max() <= 1 and lat[:, 1].max() < 100
    import inspect
    sig = inspect.signature(m.fit_em)
    for k in ['y', 'hyperparam', 'key', 'n_iter', 'log_posterior_init', 'ma_neuron', 'ma_latent',
              'n_time_per_chunk', 'dt', 'likelihood_scale', 'save_every', 'm_step_step_size',
              'm_step_maxiter', 'm_step_tol']:
        assert k in sig.parameters
    assert sig.parameters['n_iter'].default == 20 and sig.parameters['m_step_maxiter'].default == 1000
    sig = inspect.signature(m.decode_latent)
    assert list(sig.parameters)[:8] == ['y', 'tuning', 'hyperparam', 'ma_neuron', 'ma_latent',
                                        'likelihood_scale', 'n_time_per_chunk', 't_l']


def test_product_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    m = P.PoissonGPLVMJump1D(5, n_latent_bin=16, tuning_lengthscale=3.)
    with pytest.raises(Exception):
        m.fit_em(np.zeros((10, 5)), n_iter=1)


def test_run_em_rejects_zero_iterations():
    """n_iter = 0: the reference's loop leaves tuning / log_posterior_all unset and fails
    (core.py:650-681); run_em raises before any device work instead of returning an unset
    posterior."""
    with pytest.raises(ValueError, match="n_iter"):
        P.run_em(np.zeros((10, 5), np.float32), np.zeros((3, 5)), np.ones((16, 3), np.float32),
                 np.zeros((10, 16), np.float32), n_iter=0, transition=None)


def test_transition_posterior_key_order_matches_notebook():
    lj = np.log(np.random.default_rng(0).random((2, 2, 5, 5)))
    r = P.compute_transition_posterior_prob(lj)
    assert list(r) == API['decode_keys_recorded'][7:]
    ro = O.compute_transition_posterior_prob(lj)
    for k in r:
        np.testing.assert_allclose(r[k], ro[k], rtol=1e-5, atol=1e-7)


def test_product_does_not_import_oracle():
    import ast
    import glob
    pkg = os.path.join(os.path.dirname(HERE), 'poor_man_gplvm_amd')
    for f in glob.glob(os.path.join(pkg, '*.py')):
        tree = ast.parse(open(f).read())
        for node in ast.walk(tree):
            if isinstance(node, (ast.Import, ast.ImportFrom)):
                names = [a.name for a in node.names] + ([node.module] if getattr(node, 'module', None) else [])
                assert not any(n and n.split('.')[0] == 'oracle' for n in names), f


def test_masked_joint_sentinel_matches_fixture():
    """Linear-space joint counts S (exact zeros in masked rows/columns) assembled by
    log_joint_from_counts reproduce the reference's -1e20 sentinel arithmetic for the
    transition posteriors of masked latents (decode_masked.npz, oracle-made)."""
    from oracle import gplvm_oracle as O
    from poor_man_gplvm_amd.core import log_joint_from_counts, compute_transition_posterior_prob
    f = np.load(os.path.join(HERE, 'golden', 'decode_masked.npz'))
    ml = f['ma_latent'].astype(bool)
    L = ml.size
    _, logK, _, logA = O.create_transition_prob_1d(L, float(f['mv']))
    lpa, logz, _, cs, joint, ll = O.smooth_all_step_combined_ma_chunk(
        f['y'].astype(np.float64), f['tuning'].astype(np.float64), logK, logA, None, ml.astype(float),
        1.0, 10000, with_joint=True)
    with np.errstate(invalid='ignore'):
        S4 = np.exp(joint - logA[:, :, None, None] - logK[None])
    keep = (ml[:, None] & ml[None, :])[None, None] & np.isfinite(joint)
    S4 = np.where(keep, np.nan_to_num(S4), 0.0)
    r = compute_transition_posterior_prob(log_joint_from_counts(S4, logK, logA, ml))
    for k in ['p_transition_latent', 'p_transition_dynamics', 'p_joint_dynamics', 'p_joint_latent']:
        np.testing.assert_allclose(r[k], f[k], rtol=1e-6, atol=1e-9, err_msg=k)
    # the masked rows are the sentinel pattern: 1 at unmasked destinations in K's support
    assert np.all(r['p_transition_latent'][~ml][:, ~ml] == 0.0)
