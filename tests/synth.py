"""Seeded synthetic workloads: basis from generate_basis(ls, L),
W ~ N(0,1) seed 0, latent path seed 1, Poisson spikes seed 2, posterior init seed 3.
Test infrastructure: uses the oracle's samplers."""
import numpy as np

from oracle import gplvm_oracle as O


def make(N, L, T, ls=10.0, mv=1.0, seed=0, w_init_seed=7):
    B = O.generate_basis(ls, L).astype(np.float32)
    W = np.random.default_rng(seed).normal(size=(B.shape[1], N))
    tun = O.get_tuning_softplus(W, B)
    lat = O.sample_latent(T, L, np.random.default_rng(seed + 1), mv)
    y = O.sample_spikes(tun, lat[:, 1], np.random.default_rng(seed + 2)).astype(np.float32)
    lp0 = O.init_latent_posterior_from_uniform(np.random.default_rng(seed + 3).random((T, L))).astype(np.float32)
    W0 = np.random.default_rng(w_init_seed).normal(size=W.shape).astype(np.float32)
    return dict(y=y, B=B, W_true=W, tuning=tun, latent=lat, lp0=lp0, W0=W0)
