"""pmg_tuning_softplus / pmg_tuning_softplus_batched (fit_tuning_helper.py:19-25:
softplus(basis @ W)) against an f64 numpy evaluation, including a basis wider than one
LDS pass (NB > 256) and partial row / neuron tiles; batched restarts must reproduce each
restart's single call bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _call(B, W, R=1):
    from poor_man_gplvm_amd import _native as nat
    lib = nat.load()
    L, NB = B.shape
    N = W.shape[-1]
    bt = torch.as_tensor(np.ascontiguousarray(B, np.float32), device='cuda')
    wt = torch.as_tensor(np.ascontiguousarray(W, np.float64), device='cuda')
    t64 = torch.empty((R * L, N), dtype=torch.float64, device='cuda')
    t32 = torch.empty((R * L, N), dtype=torch.float32, device='cuda')
    if R == 1:
        rc = lib.pmg_tuning_softplus(nat.ptr(bt), nat.ptr(wt), L, NB, N, nat.ptr(t64), nat.ptr(t32), nat.stream_handle())
    else:
        rc = lib.pmg_tuning_softplus_batched(nat.ptr(bt), nat.ptr(wt), L, NB, N, R, nat.ptr(t64), nat.ptr(t32),
                                             nat.stream_handle())
    nat.check(rc, "pmg_tuning_softplus")
    torch.cuda.synchronize()
    return t64.cpu().numpy(), t32.cpu().numpy()


@pytest.mark.parametrize("L,NB,N", [(512, 79, 512), (100, 101, 30), (1021, 300, 70), (7, 3, 65)])
def test_tuning_softplus_vs_numpy(L, NB, N):
    rng = np.random.default_rng(L + NB + N)
    B = rng.normal(size=(L, NB)).astype(np.float32)
    W = rng.normal(size=(NB, N)) * 0.3
    t64, t32 = _call(B, W)
    F = B.astype(np.float64) @ W
    ref = np.logaddexp(F, 0.0)
    np.testing.assert_allclose(t64, ref, rtol=1e-13, atol=1e-300)
    np.testing.assert_array_equal(t32, t64.astype(np.float32))


def test_tuning_softplus_batched_bit_identical():
    rng = np.random.default_rng(7)
    L, NB, N, R = 256, 41, 96, 3
    B = rng.normal(size=(L, NB)).astype(np.float32)
    Ws = rng.normal(size=(R, NB, N)) * 0.3
    t64, _ = _call(B, Ws, R)
    for r in range(R):
        one, _ = _call(B, Ws[r])
        np.testing.assert_array_equal(t64[r * L:(r + 1) * L], one)
