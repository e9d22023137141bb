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
