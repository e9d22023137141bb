"""GPU parity of the shuffle tests (poor_man_gplvm_amd.test, reference test.py:10-79).

  * pmg_roll_columns equals np.roll per column (bit-exact, any shift incl. negative
    and >= n_time);
  * shuffle_and_decode (one resident spike buffer rolled on the device, one engine
    reused) returns exactly what decoding the reference's host-shuffled copies one by
    one returns (same seed -> same shifts; bit-identical arrays, every key), for the
    naive-Bayes and the dynamics decoder, on the jump, latent-only and Gaussian models;
  * one shuffle against the f64 oracle (the bars of test_gpu_parity's naive-Bayes and
    decode tests);
  * test_one_model's threshold is the 97.5 % quantile of the stacked shuffles.
"""
import numpy as np
import pytest
import torch

from oracle import gplvm_oracle as O
from tests.synth import make
from tests.test_gpu_parity import argmax_match, close_prob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _dev():
    torch.cuda.set_device(0)


@pytest.mark.parametrize("T,N", [(1000, 70), (333, 300), (5, 1)])
def test_roll_columns_kernel(T, N):
    from poor_man_gplvm_amd import _native as nat
    rng = np.random.default_rng(T + N)
    y = rng.integers(0, 9, size=(T, N)).astype(np.float32)
    s = rng.integers(-3 * T, 4 * T, size=N).astype(np.int64)
    s[0] = 0
    if N > 2:
        s[1], s[2] = T - 1, -1
    yt = torch.as_tensor(y, device='cuda')
    st = torch.as_tensor(s, device='cuda')
    out = torch.empty_like(yt)
    nat.check(nat.load().pmg_roll_columns(nat.ptr(yt), T, N, nat.ptr(st), nat.ptr(out), nat.stream_handle()),
              "pmg_roll_columns")
    want = np.stack([np.roll(y[:, j], s[j]) for j in range(N)], axis=1)
    np.testing.assert_array_equal(out.cpu().numpy(), want)


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert x.shape == y.shape, k
        np.testing.assert_array_equal(x, y, err_msg=k)


def _sequential(model, y, n_shuffle, seed, decoder_type, **kw):
    from poor_man_gplvm_amd import test as PT
    np.random.seed(seed)
    res = []
    for ys in PT.circular_shuffle_data(y, n_shuffle=n_shuffle):
        if decoder_type == 'naive_bayes':
            res.append(model.decode_latent_naive_bayes(ys, **kw))
        else:
            res.append(model.decode_latent(ys))
    return {k: np.array([d[k] for d in res]) for k in res[0]}


def _shuffled(model, y, n_shuffle, seed, decoder_type, **kw):
    from poor_man_gplvm_amd import test as PT
    np.random.seed(seed)
    return PT.shuffle_and_decode(model, y, n_shuffle=n_shuffle, decoder_type=decoder_type, **kw)


def test_shuffle_naive_bayes_matches_sequential_and_oracle():
    import poor_man_gplvm_amd as P
    N, L, T = 40, 100, 1500
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    m.tuning = d['tuning']
    got = _shuffled(m, d['y'], 5, 21, 'naive_bayes')
    _same(got, _sequential(m, d['y'], 5, 21, 'naive_bayes'))
    assert got['log_posterior_latent'].shape == (5, T, L) and got['log_marginal_total'].shape == (5,)
    np.random.seed(21)
    ys, _ = O.circular_shuffle_once(d['y'])
    lp, lml, lmt, ll = O.naive_bayes_chunk(ys, m.tuning.astype(np.float64))
    close_prob(got['posterior_latent'][0], np.exp(lp))
    np.testing.assert_allclose(got['log_marginal_l'][0], lml, rtol=1e-7, atol=1e-4)
    assert abs(got['log_marginal_total'][0] - lmt) <= 1e-9 * abs(lmt)
    # a shuffle destroys the population code: the true data decodes far better
    true = m.decode_latent_naive_bayes(d['y'])
    assert true['log_marginal_total'] > got['log_marginal_total'].max()


def test_shuffle_naive_bayes_per_bin_dt():
    import poor_man_gplvm_amd as P
    N, L, T = 24, 64, 800
    d = make(N, L, T)
    dt = np.random.default_rng(4).uniform(0.5, 1.5, size=T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    m.tuning = d['tuning']
    _same(_shuffled(m, d['y'], 3, 5, 'naive_bayes', dt_l=dt), _sequential(m, d['y'], 3, 5, 'naive_bayes', dt_l=dt))


def test_shuffle_dynamics_matches_sequential_and_oracle():
    import poor_man_gplvm_amd as P
    N, L, T = 30, 64, 2000
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    m.tuning = d['tuning']
    got = _shuffled(m, d['y'], 3, 8, 'dynamics')
    _same(got, _sequential(m, d['y'], 3, 8, 'dynamics'))
    assert got['posterior_all'].shape == (3, T, 2, L)
    np.random.seed(8)
    ys, _ = O.circular_shuffle_once(d['y'])
    ref = O.decode_latent(ys, m.tuning.astype(np.float64))
    close_prob(got['posterior_latent_marg'][0], ref['posterior_latent_marg'], rtol=2e-5)
    argmax_match(got['posterior_latent_marg'][0], ref['posterior_latent_marg'])
    assert abs(got['log_marginal_final'][0] - ref['log_marginal_final']) <= 1e-7 * abs(ref['log_marginal_final'])


def test_shuffle_latent_only_and_gaussian_models():
    import poor_man_gplvm_amd as P
    N, L, T = 20, 48, 900
    d = make(N, L, T)
    m1 = P.PoissonGPLVM1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    m1.tuning = d['tuning']
    g = _shuffled(m1, d['y'], 2, 1, 'dynamics')
    _same(g, _sequential(m1, d['y'], 2, 1, 'dynamics'))
    assert g['posterior_all'].shape == (2, T, L)
    mg = P.GaussianGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10., noise_std=0.5)
    mg.tuning = d['tuning']
    yg = (d['tuning'][d['latent'][:, 1]] + 0.5 * np.random.default_rng(3).normal(size=(T, N))).astype(np.float32)
    for dec in ('naive_bayes', 'dynamics'):
        _same(_shuffled(mg, yg, 2, 2, dec), _sequential(mg, yg, 2, 2, dec))


def test_test_one_model():
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import test as PT
    N, L, T = 30, 64, 1200
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    m.tuning = d['tuning']
    np.random.seed(0)
    r = PT.test_one_model(d['y'], m, n_shuffle=8)
    thr = np.quantile(r['decode_res_shuffle']['log_marginal_l'], 0.975, axis=0)
    np.testing.assert_array_equal(r['log_marg_thresh'], thr)
    sig = r['is_sig_tsd']['d'] if isinstance(r['is_sig_tsd'], dict) else np.asarray(r['is_sig_tsd'].d)
    np.testing.assert_array_equal(sig, r['decode_res_true']['log_marginal_l'] > thr)
    assert sig.mean() > 0.05      # the true tuning beats its shuffles well above the 2.5 % chance level
    np.random.seed(0)
    r2 = PT.test_one_model(d['y'], m, n_shuffle=4, decoder_type='dynamics')
    assert r2['log_marg_thresh'].shape == (T,)
