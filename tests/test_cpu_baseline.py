"""The fp32 torch-CPU restatement timed as bench.py's cpu_baseline computes the same
EM iteration as the float64 oracle (to float32 accuracy), so the baseline times the
reference's real work, not a shortcut."""
import numpy as np
import torch

from oracle import cpu_reference_fp32 as R
from oracle import gplvm_oracle as O
from tests.synth import make


def test_cpu_reference_matches_oracle():
    N, L, T = 12, 24, 60
    d = make(N, L, T)
    K, logK, A, logA = O.create_transition_prob_1d(L, 1.0)
    lpa, lz, lca, cs, lj, ll = O.smooth_all_step_combined_ma_chunk(d['y'], d['tuning'], logK, logA, with_joint=True)
    y = torch.as_tensor(d['y'], dtype=torch.float32)
    tun = torch.as_tensor(d['tuning'], dtype=torch.float32)
    lK, lA = R.transition_logs(L)
    np.testing.assert_allclose(lK.numpy(), logK, atol=2e-5)
    np.testing.assert_allclose(R.emission(y, tun).numpy(), ll, rtol=1e-5, atol=1e-3)
    posts, priors, logz = R.filter_all(R.emission(y, tun), lK, lA)
    assert abs(float(logz) - lz) <= 1e-5 * abs(lz)
    acausal, joint = R.smooth_all(posts, priors, lK, lA)
    np.testing.assert_allclose(np.exp(acausal.numpy()), np.exp(lpa), atol=1e-4)
    np.testing.assert_allclose(np.exp(joint.numpy()), np.exp(lj), atol=1e-3 * np.exp(lj).max())


def test_cpu_reference_adam_matches_oracle():
    N, L, T = 10, 20, 50
    d = make(N, L, T)
    B = d['B'].astype(np.float64)
    P = np.random.default_rng(1).dirichlet(np.ones(L), size=T)
    yw, tw = P.T @ d['y'], P.sum(0)
    W0 = np.random.default_rng(2).normal(size=(B.shape[1], N))
    ref = O.adam_run(W0, O.adam_init(W0), 1.0, B, yw, tw, maxiter=8, tol=0.0)
    W, _ = R.adam_steps(torch.as_tensor(W0, dtype=torch.float32), torch.as_tensor(B, dtype=torch.float32),
                        torch.as_tensor(yw, dtype=torch.float32), torch.as_tensor(tw, dtype=torch.float32), 7)
    np.testing.assert_allclose(W.numpy(), ref['params'], rtol=1e-4, atol=1e-5)
