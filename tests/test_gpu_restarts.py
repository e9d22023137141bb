"""Batched restarts on one GPU (core.run_em_restarts / fit_em_restarts, engine.RestartBatchEM):
R restarts of one recording share one stacked-latent emission GEMM, one scan launch per
pass (blockIdx.y = restart) and one suff-stats GEMM; each restart keeps its own Adam
loop and stop rule.  Reference: the restart loop model_selection_helper.py:53-59 (one
fit_em per key, core.py:829-849).

Bars: with the same chunking and the same relaxation segment grid (#CUs / R segments
per restart, ScanConfig.relax_segments) a batched restart is the same computation as
the single-restart engine (identical int8 emission, rows of the same GEMMs, scans over
the same grid), so every output must be bit-identical; one restart is also checked
against the f64 oracle."""
import numpy as np
import pytest
import torch

from oracle import gplvm_oracle as O
from tests.synth import make
from tests.test_gpu_parity import RT, argmax_match

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _dev():
    torch.cuda.set_device(0)


def _inits(T, L, R, seed=11):
    return np.stack([O.init_latent_posterior_from_uniform(np.random.default_rng(seed + r).random((T, L)))
                     for r in range(R)]).astype(np.float32)


def _same(res, ref):
    assert res['m_step_res_l']['n_iter'] == ref['m_step_res_l']['n_iter']
    np.testing.assert_array_equal(res['tuning'], ref['tuning'])
    np.testing.assert_array_equal(res['posterior'], ref['posterior'])
    np.testing.assert_array_equal(res['log_marginal_l'], ref['log_marginal_l'])
    for a, b in zip(res['m_step_res_l']['loss_history'], ref['m_step_res_l']['loss_history']):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("R,L,mask", [(3, 64, False), (2, 128, True), (5, 32, False)])
def test_batched_restarts_match_single(R, L, mask):
    from poor_man_gplvm_amd import AdamConfig, ScanConfig, banded_transition, run_em, run_em_restarts
    N, T = 40, 1500
    d = make(N, L, T)
    lps = _inits(T, L, R)
    ml = None
    if mask:
        ml = np.ones(L)
        ml[[3, 17, 18, 90]] = 0
    sc = ScanConfig(chunk=40, chunk_bwd=80)
    kw = dict(n_iter=3, transition=banded_transition(L, 1.0), ma_latent=ml, adam=AdamConfig(maxiter=400),
              scan=sc)
    outs = run_em_restarts(d['y'], d['W0'], d['B'], lps, **kw)
    assert len(outs) == R
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    kw1 = dict(kw, scan=ScanConfig(chunk=40, chunk_bwd=80, relax_segments=max(1, cus // R)))
    for r in range(R):
        ref, _ = run_em(d['y'], d['W0'], d['B'], lps[r], **kw1)
        _same(outs[r][0], ref)
        assert outs[r][1]['batched_restarts'] == R
    # restarts really differ
    assert np.abs(outs[0][0]['tuning'] - outs[1][0]['tuning']).max() > 0


def test_batched_restart_vs_oracle():
    from poor_man_gplvm_amd import AdamConfig, banded_transition, run_em_restarts
    N, L, T, R = 30, 64, 800, 4
    d = make(N, L, T)
    lps = _inits(T, L, R, seed=5)
    outs = run_em_restarts(d['y'], d['W0'], d['B'], lps, n_iter=1, transition=banded_transition(L, 1.0),
                           adam=AdamConfig(maxiter=60, tol=0.0))
    for r in (0, 3):
        res = outs[r][0]
        ref = O.fit_em(d['y'], d['W0'].astype(np.float64), d['B'].astype(np.float64), lps[r].astype(np.float64),
                       n_iter=1, m_step_maxiter=60, m_step_tol=0.0)
        np.testing.assert_allclose(res['tuning'], ref['tuning'], rtol=RT)
        np.testing.assert_allclose(res['posterior_latent_marg'], ref['posterior_latent_marg'], rtol=RT, atol=1e-12)
        argmax_match(res['posterior_latent_marg'], ref['posterior_latent_marg'])
        np.testing.assert_allclose(res['log_marginal_l'], ref['log_marginal_l'], rtol=1e-7)


def test_fit_em_restarts_public_api():
    """fit_em_restarts leaves every model as its own fit_em would (same chunking at this T)."""
    import poor_man_gplvm_amd as P
    N, L, T, R = 24, 64, 1200, 3
    d = make(N, L, T)
    keys = [3, 17, 29]
    ms = [P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.) for _ in range(R)]
    ems = P.fit_em_restarts(ms, d['y'], keys, n_iter=2, m_step_maxiter=300)
    for m, em, k in zip(ms, ems, keys):
        one = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
        ref = one.fit_em(d['y'], key=k, n_iter=2, m_step_maxiter=300)
        _same(em, ref)
        np.testing.assert_allclose(m.params, one.params, rtol=1e-6)
        np.testing.assert_array_equal(em['log_posterior_init'], ref['log_posterior_init'])
        assert list(em) == list(ref)
        assert m.log_marginal_final == em['log_marginal']
    # Gaussian models are not batched: the helper falls back to one fit_em per key
    g = [P.GaussianGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.) for _ in range(2)]
    out = P.fit_em_restarts(g, d['y'], [1, 2], n_iter=1)
    assert len(out) == 2 and 'batched_restarts' not in g[0].fit_info


@pytest.mark.parametrize("L,NB_ls,N,R,maxiter,tol", [(256, 10., 256, 8, 1000, 1e-6), (64, 10., 40, 5, 300, 1e-6),
                                                     (128, 5., 300, 3, 50, 0.0)])
def test_batched_adam_bit_identical(L, NB_ls, N, R, maxiter, tol):
    """pmg_mstep_adam_batched (several restarts per persistent launch, up to 4 neurons per
    workgroup) == R pmg_mstep_adam calls: W / mu / nu and the step counts bit for bit (the
    per-element arithmetic does not depend on the neuron partition), iteration counts
    identical, loss histories to the last bits of their summation order."""
    import ctypes
    from poor_man_gplvm_amd import _native as nat
    from poor_man_gplvm_amd.engine import AdamConfig
    lib = nat.load()
    dev = torch.device('cuda', 0)
    B = O.generate_basis(NB_ls, L).astype(np.float32)
    NB = B.shape[1]
    rng = np.random.default_rng(4)
    W0 = torch.tensor(rng.normal(size=(R, NB, N)), dtype=torch.float64, device=dev)
    P = rng.random((R, 2000, L))
    P /= P.sum(-1, keepdims=True)
    y = rng.poisson(2.0, size=(2000, N)).astype(np.float64)
    yw = torch.tensor(np.concatenate([p.T @ y for p in P]), dtype=torch.float64, device=dev)     # (R L, N)
    tw = torch.tensor(np.concatenate([p.sum(0) for p in P]), dtype=torch.float64, device=dev)
    Bt = torch.tensor(B, device=dev)
    cfg = AdamConfig(maxiter=maxiter, tol=tol).to_c()
    mi = max(maxiter, 1)

    def run(batched):
        W, mu, nu = W0.clone(), torch.zeros_like(W0), torch.zeros_like(W0)
        cnt = torch.zeros(R, dtype=torch.int64, device=dev)
        st = torch.zeros((R, 4), dtype=torch.float64, device=dev)
        lh = torch.zeros((R, mi), dtype=torch.float64, device=dev)
        eh = torch.zeros_like(lh)
        for _ in range(2):    # two M-steps: the Adam state carries over
            if batched:
                assert lib.pmg_mstep_adam_batched_supported(L, NB, N, R)
                ws = torch.empty(int(lib.pmg_mstep_batched_workspace_size(L, NB, N, R, maxiter)), dtype=torch.uint8,
                                 device=dev)
                nat.check(lib.pmg_mstep_adam_batched(nat.ptr(W), nat.ptr(mu), nat.ptr(nu), nat.ptr(cnt), nat.ptr(Bt),
                                                     nat.ptr(yw), nat.ptr(tw), L, NB, N, R, ctypes.byref(cfg),
                                                     nat.ptr(st), nat.ptr(lh), nat.ptr(eh), nat.ptr(ws), ws.numel(),
                                                     nat.stream_handle()), "batched")
            else:
                ws = torch.empty(int(lib.pmg_mstep_workspace_size(N, maxiter)), dtype=torch.uint8, device=dev)
                for r in range(R):
                    nat.check(lib.pmg_mstep_adam(nat.ptr(W[r]), nat.ptr(mu[r]), nat.ptr(nu[r]), nat.ptr(cnt[r:r + 1]),
                                                 nat.ptr(Bt), nat.ptr(yw[r * L:(r + 1) * L]),
                                                 nat.ptr(tw[r * L:(r + 1) * L]), L, NB, N, ctypes.byref(cfg),
                                                 nat.ptr(st[r]), nat.ptr(lh[r]), nat.ptr(eh[r]), nat.ptr(ws),
                                                 ws.numel(), nat.stream_handle()), "single")
        torch.cuda.synchronize()
        return [t.cpu().numpy() for t in (W, mu, nu, cnt, st, lh)]
    a, b = run(True), run(False)
    for x, z in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, z)
    np.testing.assert_array_equal(a[4][:, 0], b[4][:, 0])          # n_iter per restart
    np.testing.assert_allclose(a[5], b[5], rtol=1e-12)             # loss histories
    assert len(set(a[4][:, 0].tolist())) >= 1 and np.all(a[4][:, 0] >= 1)
