"""GPU parity of the dense log-domain scans (dense_scan.hip) and of the kernels passed to
_decode_latent, against the float64 oracle.

The dense scans run the reference's own log-space recursion (decoder.py:151-226) for
continuous kernels the banded linear-space scans cannot hold: custom_transition_kernel
(gp_kernel.py:30-34, 61-66), RBF kernels wider than 32 bins, and the latent-only model
(decoder_latentonly.py), whose far latent moves have weights (exp(-1000)) beyond the
fp32 / f64 range.  Bars: posteriors rel 1e-5 (atol 1e-12) for the jump model; for the
latent-only model max abs 1e-5 and < 10 % of the fp32 reference-mimic's deviation
(test_gpu_parity.latent_only_close); log marginal rel 1e-7; finite log outputs where
the reference's are finite.
"""
import warnings

import numpy as np
import pytest
import torch

from oracle import gplvm_oracle as O
from tests.synth import make
from tests.test_gpu_parity import argmax_match, close_prob, latent_only_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _dev():
    torch.cuda.set_device(0)


def _custom_kernel(L, seed=5):
    rng = np.random.default_rng(seed)
    i = np.arange(L)
    return np.exp(-np.abs(i[:, None] - i[None, :]) / 3.0) + 0.02 * rng.random((L, L))


@pytest.mark.parametrize("chunk", [None, 16])
def test_custom_transition_kernel_decode_vs_oracle(chunk):
    """Jump model with a dense custom continuous kernel (gp_kernel.py:61-66); chunk 16
    with no warm-up makes every boundary fail so the relaxation runs."""
    import poor_man_gplvm_amd as P
    N, L, T = 30, 80, 700
    d = make(N, L, T)
    Kc = _custom_kernel(L)
    sc = P.ScanConfig(chunk=chunk, warmup=0 if chunk else 48)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10., custom_transition_kernel=Kc,
                             scan_config=sc)
    r = m.decode_latent(d['y'], tuning=d['tuning'])
    ref = O.decode_latent(d['y'], d['tuning'], custom_kernel=Kc)
    close_prob(r['posterior_all'], ref['posterior_all'])
    argmax_match(r['posterior_latent_marg'], ref['posterior_latent_marg'])
    assert abs(r['log_marginal_final'] - ref['log_marginal_final']) <= 1e-7 * abs(ref['log_marginal_final'])
    np.testing.assert_allclose(r['log_one_step_predictive_marginals_all'],
                               ref['log_one_step_predictive_marginals_all'], rtol=1e-6, atol=1e-5)
    lp, lr = r['log_posterior_all'], ref['log_posterior_all']
    assert np.all(np.isfinite(lp))
    keep = lr > -60
    np.testing.assert_allclose(lp[keep], lr[keep], atol=2e-4)
    np.testing.assert_allclose(r['p_transition_full'], ref['p_transition_full'], rtol=1e-4, atol=1e-7)


def test_wide_movement_variance_vs_oracle():
    """movement_variance = 5 needs a 42-bin band (> 32): the dense scans take it."""
    import poor_man_gplvm_amd as P
    N, L, T = 40, 128, 800
    d = make(N, L, T, mv=5.0)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10., movement_variance=5.0)
    r = m.decode_latent(d['y'], tuning=d['tuning'])
    ref = O.decode_latent(d['y'], d['tuning'], movement_variance=5.0)
    close_prob(r['posterior_all'], ref['posterior_all'])
    assert abs(r['log_marginal_final'] - ref['log_marginal_final']) <= 1e-7 * abs(ref['log_marginal_final'])


@pytest.mark.parametrize("masked", [False, True])
def test_latent_only_far_moves_exact(masked):
    """Latent-only model on data sampled WITH jumps (moves of tens of bins): the log
    marginal includes transitions of weight exp(-1000) (tools/diag_lo_mask.py; round 1's
    banded scan gave -48336 against the reference's -47881 here)."""
    import poor_man_gplvm_amd as P
    N, L, T = 30, 100, 1500
    d = make(N, L, T)
    ml = None
    if masked:
        ml = np.zeros(L)
        ml[::3] = 1
        ml[np.random.default_rng(0).choice(L, 20, replace=False)] = 1
    _, logK = O.create_transition_prob_latent_1d(L, 1.0)
    lpa, lz, lca, cs, lj, ll = O.smooth_latent_only(d['y'], d['tuning'], logK, ma_latent=ml)
    m = P.PoissonGPLVM1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        res = m.decode_latent(d['y'], tuning=d['tuning'], ma_latent=ml)
    assert abs(res['log_marginal_final'] - lz) <= 1e-7 * abs(lz), (res['log_marginal_final'], lz)
    # the pairwise joint of a far move (rho ~ e^+1000 against K ~ e^-1000) is accumulated
    # in log space: finite, and equal to the reference's logaddexp accumulation
    keep = np.ones(L, bool) if ml is None else ml.astype(bool)
    for k in ('p_transition_latent', 'p_joint_latent', 'log_joint_latent'):
        assert not np.isnan(res[k]).any(), k
    ref = O.compute_transition_posterior_prob_latent(lj)
    np.testing.assert_allclose(res['p_transition_latent'][np.ix_(keep, keep)],
                               ref['p_transition_latent'][np.ix_(keep, keep)], rtol=1e-5, atol=1e-12)
    latent_only_close(res['posterior_all'], d['y'], d['tuning'], logK, ml)
    argmax_match(res['posterior_all'], np.exp(lpa))
    fwd = m.log_marginal_masked(d['y'], (np.ones(L) if ml is None else ml)[None], tuning=d['tuning'])[0]
    assert abs(fwd - lz) <= 1e-7 * abs(lz)


def test_latent_only_private_decode_signature():
    """PoissonGPLVM1D._decode_latent(y, tuning, hyperparam, log_latent_transition_kernel (L, L),
    ma_neuron, ...) -> the latent-only 6-tuple (core.py:943-953)."""
    import poor_man_gplvm_amd as P
    N, L, T = 20, 60, 400
    d = make(N, L, T)
    _, logK = O.create_transition_prob_latent_1d(L, 2.0)      # a kernel other than the model's
    m = P.PoissonGPLVM1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    la, lz, lc, cs, lj, ll = m._decode_latent(d['y'], d['tuning'], {}, logK, np.ones(N))
    rla, rlz, rlc, rcs, rlj, rll = O.smooth_latent_only(d['y'], d['tuning'], logK)
    assert la.shape == (T, L) and lj.shape == (L, L)
    latent_only_close(np.exp(la), d['y'], d['tuning'], logK)
    assert abs(lz - rlz) <= 1e-7 * abs(rlz)


@pytest.mark.parametrize("kind", ["banded_other_mv", "dense_custom"])
def test_decode_latent_uses_passed_kernels(kind):
    """_decode_latent scans with the kernels it is passed (core.py:777-786), not with the
    model's own hyper-parameters."""
    import poor_man_gplvm_amd as P
    N, L, T = 30, 64, 500
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10., movement_variance=1.0)
    if kind == "banded_other_mv":
        _, logK, _, logA = O.create_transition_prob_1d(L, 2.0, 0.05, 0.02)
    else:
        _, logK, _, logA = O.create_transition_prob_1d(L, 1.0, 0.01, 0.01, custom_kernel=_custom_kernel(L, 9))
    la, lz, lc, cs, lj, ll = m._decode_latent(d['y'], d['tuning'], {}, logK, logA, np.ones(N))
    rla, rlz, rlc, rcs, rlj, rll = O.smooth_all_step_combined_ma_chunk(d['y'], d['tuning'], logK, logA,
                                                                        with_joint=True)
    close_prob(np.exp(la), np.exp(rla))
    assert abs(lz - rlz) <= 1e-7 * abs(rlz)
    np.testing.assert_allclose(np.exp(lj - rlj.max()), np.exp(rlj - rlj.max()), rtol=1e-5, atol=1e-12)


def test_decode_latent_outputs_finite_with_unvisited_bins():
    """Strongly tuned neurons leave most latent bins unvisited (their f32 alpha
    underflows): every decode_latent output must stay finite, with no RuntimeWarning
    (round 1 returned NaN transition rows here)."""
    import poor_man_gplvm_amd as P
    N, L, T = 60, 100, 400
    d = make(N, L, T)
    tun = d['tuning'] * 8.0
    rng = np.random.default_rng(3)
    y = rng.poisson(tun[d['latent'][:, 1]]).astype(np.float32)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)
        r = m.decode_latent(y, tuning=tun)
    for k, v in r.items():
        if isinstance(v, np.ndarray):
            assert not np.isnan(v).any(), k
    for k in ('log_transition_full', 'log_transition_latent', 'log_joint_full', 'p_transition_full',
              'p_transition_latent'):
        assert np.all(np.isfinite(r[k])), k
    # every row, visited or not, is the reference's conditional (decode_exact: dense
    # log-domain scans with the full kernel, f64 joint)
    ref = O.decode_latent(y, tun)
    for k in ('p_transition_latent', 'p_transition_full', 'p_transition_dynamics', 'p_joint_latent'):
        np.testing.assert_allclose(r[k], ref[k], rtol=1e-5, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("L,T", [(1280, 200), (2600, 120)])
def test_large_latent_count_vs_oracle(L, T):
    """n_latent_bin > 1024 (the reference scans any L, decoder.py:151-172): the banded
    scans hold L <= 1024, so the model takes the dense log-domain scans with 8 (L <= 2048)
    or 16 (L <= 4096) latents per thread.  Decode (posterior, log marginal, one-step
    predictive) and one EM iteration (tuning, posterior) against the f64 oracle."""
    import poor_man_gplvm_amd as P
    N = 24
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    from poor_man_gplvm_amd.gp_kernel import DenseTransition, dense_transition
    assert isinstance(m._transition(1.0, 0.01, 0.01), DenseTransition)
    r = m.decode_latent(d['y'], tuning=d['tuning'])
    ref = O.decode_latent(d['y'], d['tuning'])
    close_prob(r['posterior_all'], ref['posterior_all'])
    argmax_match(r['posterior_latent_marg'], ref['posterior_latent_marg'])
    assert abs(r['log_marginal_final'] - ref['log_marginal_final']) <= 1e-7 * abs(ref['log_marginal_final'])
    np.testing.assert_allclose(r['log_one_step_predictive_marginals_all'],
                               ref['log_one_step_predictive_marginals_all'], rtol=1e-6, atol=1e-5)
    res, _ = P.run_em(d['y'].astype(np.float32), d['W0'], d['B'], d['lp0'], n_iter=1,
                      transition=dense_transition(L, 1.0), adam=P.AdamConfig(maxiter=40, tol=0.0))
    ref = O.fit_em(d['y'], d['W0'].astype(np.float64), d['B'].astype(np.float64), d['lp0'].astype(np.float64),
                   n_iter=1, m_step_maxiter=40, m_step_tol=0.0)
    np.testing.assert_allclose(res['tuning'], ref['tuning'], rtol=1e-5)
    close_prob(res['posterior_latent_marg'], ref['posterior_latent_marg'])


@pytest.mark.parametrize("T,L,spread,ws", [(300, 40, 5.0, False), (3000, 40, 40.0, True), (700, 72, 400.0, True),
                                           (2000, 33, 1500.0, True)])
def test_joint_log_accumulate_vs_logsumexp(T, L, spread, ws):
    """pmg_joint_log_accumulate(_ws): logS[x, x'] = LSE_t la_t[x] + lr_{t+1}[x'] against an
    f64 scipy logsumexp, rel 1e-12 on logS (every entry finite where the reference's is),
    for log inputs that drift by up to `spread` nats within a few steps (random walks, so
    row and column peaks sit at different times: spread 1500 forces the term-by-term
    fallback of blocks whose shifted sum leaves f64's range), with a fully masked row and
    column (-inf) and the time-split workspace path."""
    from scipy.special import logsumexp
    from poor_man_gplvm_amd import _native as nat
    rng = np.random.default_rng(int(T + L + spread))
    L2 = 2 * L
    la = np.cumsum(rng.standard_normal((T, L2)) * spread / 8, axis=0)
    lr = np.cumsum(rng.standard_normal((T, L2)) * spread / 8, axis=0)
    la[:, 3] = -np.inf
    lr[:, L2 - 5] = -np.inf
    lib = nat.load()
    a = torch.as_tensor(la, device='cuda')
    r = torch.as_tensor(lr, device='cuda')
    S = torch.empty((L2, L2), dtype=torch.float64, device='cuda')
    if ws:
        nws = int(lib.pmg_joint_log_workspace_size(T, L))
        assert nws > 0          # these shapes split in time: the combine path runs
        w = torch.empty(nws, dtype=torch.uint8, device='cuda')
        nat.check(lib.pmg_joint_log_accumulate_ws(nat.ptr(a), nat.ptr(r), T, L, nat.ptr(S), nat.ptr(w), w.numel(),
                                                  nat.stream_handle()), "joint")
    else:
        nat.check(lib.pmg_joint_log_accumulate(nat.ptr(a), nat.ptr(r), T, L, nat.ptr(S), nat.stream_handle()), "joint")
    got = S.cpu().numpy()
    with np.errstate(invalid='ignore'):
        ref = logsumexp(la[:-1, :, None] + lr[1:, None, :], axis=0)
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin)
    assert np.all(np.isneginf(got[~fin]))
    np.testing.assert_allclose(got[fin], ref[fin], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("T,L", [(200, 40), (4000, 16)])
def test_joint_log_block_fallback_deterministic(T, L):
    """The blocked joint's term-by-term fallback, forced: latent 1 of log
    alpha sits 900 nats below latent 0 at every step, so inside every 64 x 64 tile and
    64-step block its shifted terms underflow to 0 and the block sum of every entry of
    row 1 is 0; the right answer, -900 + lr + log(T - 1), is finite only if the fallback
    ran.  (4000, 16): a shape whose workspace size is nonzero, so the time splits and their
    combine run as well; (200, 40) runs unsplit."""
    from poor_man_gplvm_amd import _native as nat
    from scipy.special import logsumexp
    L2 = 2 * L
    la = np.zeros((T, L2))
    la[:, 1] = -900.0
    la[:, 5] = -1600.0
    rng = np.random.default_rng(T + L)
    lr = rng.standard_normal((T, L2)) * 0.1
    lr[:, 2] -= 850.0                      # a column 850 nats down: entry (1, 2) is ~1750 below the tile max
    lib = nat.load()
    nws = int(lib.pmg_joint_log_workspace_size(T, L))
    assert (nws > 0) == (T >= 2048)
    a = torch.as_tensor(la, device='cuda')
    r = torch.as_tensor(lr, device='cuda')
    S = torch.empty((L2, L2), dtype=torch.float64, device='cuda')
    w = torch.empty(nws, dtype=torch.uint8, device='cuda') if nws else None
    nat.check(lib.pmg_joint_log_accumulate_ws(nat.ptr(a), nat.ptr(r), T, L, nat.ptr(S), nat.ptr(w), nws,
                                              nat.stream_handle()), "joint")
    got = S.cpu().numpy()
    ref = logsumexp(la[:-1, :, None] + lr[1:, None, :], axis=0)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-9)
    assert got[1, 2] < -1700 and got[5, 2] < -2400
