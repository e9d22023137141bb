"""Page-locked host buffers of the returned arrays (pmg_host_alloc / pmg_copy_d2h, the
_native.HostBuffer cache): contents after a device->host copy, reuse of a released block
of the same size, and release of the cache."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_host_array_copy_and_cache():
    from poor_man_gplvm_amd import _native as nat
    lib = nat.load()
    shape = (1000, 2, 96)
    g = torch.randn(shape, dtype=torch.float32, device='cuda')
    h = nat.host_array(shape, np.float32)
    assert h.shape == shape and h.dtype == np.float32 and h.flags.writeable
    nat.check(lib.pmg_copy_d2h(h.ctypes.data, g.data_ptr(), g.numel() * 4, nat.stream_handle()), "copy")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(h, g.cpu().numpy())
    p = h.ctypes.data
    del h                                   # back to the cache
    h2 = nat.host_array(shape, np.float32)  # same size: the cached block
    assert h2.ctypes.data == p
    v = h2.view()                           # a view keeps the block alive
    del h2
    h3 = nat.host_array(shape, np.float32)
    assert h3.ctypes.data != p
    del v, h3
    nat.release_host_cache()
    assert nat._host_cache_total == 0


def test_fit_and_decode_results_are_host_arrays():
    """fit_em / decode_latent hand back numpy arrays that stay valid after the model and
    the device tensors are gone (the pinned blocks are owned by the arrays)."""
    import gc
    import poor_man_gplvm_amd as P
    rng = np.random.default_rng(0)
    y = rng.poisson(0.5, size=(800, 20)).astype(np.float32)
    m = P.PoissonGPLVMJump1D(20, n_latent_bin=32, tuning_lengthscale=5.)
    res = m.fit_em(y, key=1, n_iter=2)
    dec = m.decode_latent(y)
    post, lp = res['posterior'].copy(), dec['log_posterior_all'].copy()
    plm = dec['posterior_latent_marg']
    del m
    gc.collect()
    torch.cuda.empty_cache()
    np.testing.assert_array_equal(res['posterior'], post)
    np.testing.assert_array_equal(dec['log_posterior_all'], lp)
    np.testing.assert_allclose(plm, dec['posterior_all'].sum(1), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(dec['posterior_dynamics_marg'], dec['posterior_all'].sum(2), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("T,L", [(1000, 96), (257, 300), (3, 1), (0, 16), (4100, 512)])
def test_posterior_outputs_one_pass(T, L):
    """pmg_posterior_outputs: log (bit-identical to pmg_log), latent marginal (the f32
    sum of the two dynamics rows, exact) and dynamics marginal (f64 sum rounded once) of
    a posterior with exact zeros (log -inf)."""
    from poor_man_gplvm_amd.engine import log_of, posterior_outputs
    rng = np.random.default_rng(T + L)
    g = rng.random((T, 2, L)).astype(np.float32)
    g[rng.random(g.shape) < 0.05] = 0.0
    gd = torch.as_tensor(g, device='cuda')
    lg, plm, pdm = posterior_outputs(gd)
    ref_log = log_of(gd)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(lg.cpu().numpy(), ref_log.cpu().numpy())
    np.testing.assert_array_equal(plm.cpu().numpy(), g[:, 0, :] + g[:, 1, :])
    np.testing.assert_allclose(pdm.cpu().numpy(), g.astype(np.float64).sum(2).astype(np.float32), rtol=1.2e-7)
    lg2, plm2, pdm2 = posterior_outputs(gd, log=False)
    assert lg2 is None
    np.testing.assert_array_equal(plm2.cpu().numpy(), plm.cpu().numpy())
    np.testing.assert_array_equal(pdm2.cpu().numpy(), pdm.cpu().numpy())
