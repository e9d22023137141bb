"""C3 (N=512, T=1e5, L=512) through size-independent properties: chunking invariance
of the time-parallel scan, normalisation, suff-stat consistency, a finite EM step."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3():
    import bench
    torch.cuda.set_device(0)
    y, B, W0, lp0 = bench.synth(512, 100000, 512)
    return y, B, W0, lp0


def _e_step(c3, chunk, warmup):
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, ScanConfig
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    y, B, W0, lp0 = c3
    sp = SpikeData(y)
    eng = DeviceEM(sp, 512, basis=B, scan=ScanConfig(chunk=chunk, warmup=warmup, adaptive=False))
    eng.set_transition(banded_transition(512, 1.0))
    W = torch.as_tensor(np.random.default_rng(0).normal(size=W0.shape), device='cuda')
    eng.compute_tuning(W)
    logz = torch.zeros(1, dtype=torch.float64, device='cuda')
    eng.e_step(1.0, logz)
    return eng, float(logz.item())


def test_chunking_invariance_and_normalisation(c3):
    e1, z1 = _e_step(c3, 49, 64)
    P1 = e1.P.cpu().numpy()
    r1 = e1.repairs()
    e2, z2 = _e_step(c3, 200, 32)
    P2 = e2.P.cpu().numpy()
    assert np.isfinite(z1) and abs(z1 - z2) <= 1e-9 * abs(z1)
    m = np.maximum(P1, P2) > 1e-12
    assert np.max(np.abs(P1[m] - P2[m]) / np.maximum(P1[m], P2[m])) < 2e-6
    np.testing.assert_allclose(P1.sum(1), 1.0, rtol=1e-5)
    assert r1[0] + r1[1] < 0.05 * (100000 // 49)


def test_suffstats_column_sums_and_em_step(c3):
    from poor_man_gplvm_amd.engine import AdamConfig
    eng, _ = _e_step(c3, None, 64)
    W = torch.as_tensor(c3[2].astype(np.float64), device='cuda').contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
    stats = torch.zeros(4, dtype=torch.float64, device='cuda')
    lh = torch.zeros(1000, dtype=torch.float64, device='cuda')
    eh = torch.zeros_like(lh)
    eng.m_step(W, mu, nu, cnt, AdamConfig(), stats, lh, eh)
    tw = eng.tw.cpu().numpy()
    np.testing.assert_allclose(tw, eng.P.double().sum(0).cpu().numpy(), rtol=1e-6)
    assert abs(tw.sum() - 100000) < 1e-2
    yw = eng.yw.cpu().numpy()
    np.testing.assert_allclose(yw.sum(0), c3[0].astype(np.float64).sum(0), rtol=1e-6)   # sum_l P = 1
    s = stats.cpu().numpy()
    assert 6 <= s[0] <= 1000 and np.isfinite(s[1]) and np.all(np.isfinite(W.cpu().numpy()))
