"""Sticky device errors reach the caller on every path.

* Scan relaxation timeout: the relaxation kernels' grid barriers spin at most 2 s; a
  barrier that gives up sets a timeout word that stays set across later calls (their
  relaxations fail fast) until the host reads and clears it.  PMG_DEBUG_SPIN_TICKS=0
  makes the first barrier of a relaxation give up, so a call that has to repair
  boundaries must raise -- from the engine, a public decode, log_marginal_masked and the
  dense log-domain scans -- and the next call after the check must work again.
* Emission range flag (|log lam| >= 60 leaves the exact int8 digit range): raised from
  the naive-Bayes decode and log_marginal_masked, not only from fits.
"""
import os

import numpy as np
import pytest
import torch

from oracle import gplvm_oracle as O
from tests.synth import make
from tests.test_gpu_parity import _engine, close_prob

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _dev():
    torch.cuda.set_device(0)


@pytest.fixture
def spin0():
    os.environ["PMG_DEBUG_SPIN_TICKS"] = "0"
    try:
        yield
    finally:
        os.environ.pop("PMG_DEBUG_SPIN_TICKS", None)


def _flat(d, L, N, scale=1e-3, seed=11):
    rng = np.random.default_rng(seed)
    return (d['tuning'].mean(0, keepdims=True) * (1.0 + scale * rng.standard_normal((L, N)))).astype(np.float64)


def test_scan_timeout_raises_and_clears():
    from poor_man_gplvm_amd import _native as nat
    N, L, T = 24, 256, 3000
    d = make(N, L, T)
    tun = _flat(d, L, N)
    sp, eng = _engine(d, L, chunk=32, warmup=16)
    eng.set_tuning(tun)
    logz = torch.zeros(1, dtype=torch.float64, device='cuda')
    gamma = torch.empty((T, 2, L), dtype=torch.float32, device='cuda')
    os.environ["PMG_DEBUG_SPIN_TICKS"] = "0"
    try:
        eng.e_step(1.0, logz, gamma=gamma)
        eng.e_step(1.0, logz, gamma=gamma)      # a later call does not clear the word
    finally:
        os.environ.pop("PMG_DEBUG_SPIN_TICKS", None)
    with pytest.raises(nat.NativeError, match="timed out"):
        eng.scan_status()
    eng.scan_status()                           # cleared by the check
    eng.e_step(1.0, logz, gamma=gamma)          # normal spin bound: exact again
    f, b = eng.repairs()
    assert f > 0 and b > 0
    K, logK, A, logA = O.create_transition_prob_1d(L, 1.0)
    lpa, lz, *_ = O.smooth_all_step_combined_ma_chunk(d['y'], tun, logK, logA, with_joint=False)
    close_prob(gamma.cpu().numpy(), np.exp(lpa))


def test_decode_latent_raises_on_scan_timeout(spin0):
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import _native as nat
    N, L, T = 24, 128, 2000
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.,
                             scan_config=P.ScanConfig(chunk=16, warmup=2))
    with pytest.raises(nat.NativeError, match="timed out"):
        m.decode_latent(d['y'], tuning=_flat(d, L, N))


def test_log_marginal_masked_raises_on_scan_timeout(spin0):
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import _native as nat
    N, L, T = 24, 128, 2000
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.,
                             scan_config=P.ScanConfig(chunk=16, warmup=2))
    masks = np.ones((2, L))
    masks[1, :40] = 0
    with pytest.raises(nat.NativeError, match="timed out"):
        m.log_marginal_masked(d['y'], masks, tuning=_flat(d, L, N))


def test_dense_scan_timeout_raises(spin0):
    """A custom transition kernel runs the dense log-domain scans (dense_scan.hip)."""
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import _native as nat
    N, L, T = 24, 64, 3000
    d = make(N, L, T)
    ii = np.arange(L)
    kern = np.exp(-np.abs(ii[:, None] - ii[None, :]) / 3.0)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10., custom_transition_kernel=kern,
                             scan_config=P.ScanConfig(chunk=8, warmup=1))
    with pytest.raises(nat.NativeError, match="timed out"):
        m.decode_latent(d['y'], tuning=_flat(d, L, N))


@pytest.mark.parametrize("path", ["naive_bayes", "masked"])
def test_emission_range_flag_other_paths(path):
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import _native as nat
    N, L, T = 8, 32, 200
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    tun = np.array(d['tuning'], copy=True)
    tun[3, 2] = 1e30
    with pytest.raises(nat.NativeError, match="digit range"):
        if path == "naive_bayes":
            m.decode_latent_naive_bayes(d['y'], tuning=tun)
        else:
            m.log_marginal_masked(d['y'], np.ones((2, L)), tuning=tun)
    # in range: works (the flag of the failed call was cleared by its check)
    if path == "naive_bayes":
        m.decode_latent_naive_bayes(d['y'], tuning=d['tuning'])
    else:
        m.log_marginal_masked(d['y'], np.ones((2, L)), tuning=d['tuning'])


def test_adam_timeout_raises_and_clears():
    """The persistent Adam kernel's cross-workgroup waits (row-block B^T G exchange at
    L > 512, the lagged stop decision) are bounded by spin_ticks(): PMG_DEBUG_SPIN_TICKS=0
    makes the first wait give up.  The sticky word in the workspace survives later
    launches, adam_status() raises once and clears it, and a normal launch is exact again."""
    from oracle import gplvm_oracle as O
    from poor_man_gplvm_amd import _native as nat
    from poor_man_gplvm_amd.engine import AdamConfig
    N, L = 64, 1024
    d = make(N, L, 300)
    sp, eng = _engine(d, L)
    assert eng.lib.pmg_mstep_adam_supported(eng.L, eng.NB, N) == 1
    yw, tw = O.get_statistics(d['lp0'].astype(np.float64), d['y'])
    eng.yw.copy_(torch.as_tensor(yw, device='cuda'))
    eng.tw.copy_(torch.as_tensor(tw, device='cuda'))

    def run():
        W = torch.as_tensor(d['W0'].astype(np.float64), device='cuda').contiguous()
        mu, nu = torch.zeros_like(W), torch.zeros_like(W)
        cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
        stats = torch.zeros(4, dtype=torch.float64, device='cuda')
        lh = torch.zeros(200, dtype=torch.float64, device='cuda')
        eng.adam(W, mu, nu, cnt, AdamConfig(maxiter=200, tol=0.0), stats, lh, torch.zeros_like(lh))
        return W, stats
    os.environ["PMG_DEBUG_SPIN_TICKS"] = "0"
    try:
        run()
        torch.cuda.synchronize()
    finally:
        os.environ.pop("PMG_DEBUG_SPIN_TICKS", None)
    run()                                       # a later launch does not clear the word
    with pytest.raises(nat.NativeError, match="timed out"):
        eng.adam_status()
    eng.adam_status()                           # cleared by the check
    W, stats = run()
    eng.check_status()
    ref = O.adam_run(d['W0'].astype(np.float64), O.adam_init(d['W0']), 1.0, d['B'].astype(np.float64), yw, tw,
                     maxiter=200, tol=0.0)
    assert int(stats[0].item()) == ref['n_iter']
    B = d['B'].astype(np.float64)
    np.testing.assert_allclose(np.logaddexp(B @ W.cpu().numpy(), 0), np.logaddexp(B @ ref['params'], 0), rtol=1e-5)
