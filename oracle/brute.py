"""Brute-force path enumeration for tiny jump-GPLVM HMMs (TEST INFRASTRUCTURE ONLY).

Independent exact check of the oracle's filter/smoother: enumerate every
(dynamics, latent) path x_0..x_{T-1} of a D x L state space, weight it by

    p(x_0) * prod_t T(x_{t-1}, x_t) * prod_t exp(s * ll[t, l_t]),
    p(x_0) = sum_x 1/(D L) * T(x, x_0)      (decoder.py:181 -- the filter starts
                                              from a uniform state "at t = -1")
    T((d,i) -> (d',j)) = A[d,d'] * K[d',i,j]  (decoder.py:160-164)

and read off the smoothed marginals, the summed pairwise joint
(decoder.py:215-221), the one-step predictive marginals and the log marginal.
Cost is (D L)^T, so keep D*L <= 8 and T <= 6.
"""
from __future__ import annotations

import itertools

import numpy as np
from scipy.special import logsumexp


def enumerate_posteriors(ll, K, A, likelihood_scale=1.0):
    T, L = ll.shape
    D = A.shape[0]
    S = D * L
    trans = np.einsum('ab,bij->aibj', A, K).reshape(S, S)        # [(d,i),(d',j)]
    p0 = np.full(S, 1.0 / S) @ trans
    emis = np.exp(likelihood_scale * ll)                          # (T, L)
    states = [(d, l) for d in range(D) for l in range(L)]
    logw = []
    paths = list(itertools.product(range(S), repeat=T))
    for path in paths:
        w = np.log(p0[path[0]]) + likelihood_scale * ll[0, states[path[0]][1]]
        for t in range(1, T):
            w += np.log(trans[path[t - 1], path[t]]) + likelihood_scale * ll[t, states[path[t]][1]]
        logw.append(w)
    logw = np.array(logw)
    logZ = logsumexp(logw)
    pw = np.exp(logw - logZ)
    post = np.zeros((T, D, L))
    joint = np.zeros((D, D, L, L))
    for p, path in zip(pw, paths):
        for t in range(T):
            d, l = states[path[t]]
            post[t, d, l] += p
        for t in range(T - 1):
            d, i = states[path[t]]
            d2, j = states[path[t + 1]]
            joint[d, d2, i, j] += p
    # one-step predictive marginals: log p(o_t | o_<t) = logZ_{0..t} - logZ_{0..t-1}
    cs = np.empty(T)
    prev = 0.0
    for t in range(T):
        sub = ll[: t + 1]
        # marginal likelihood of the first t+1 observations by forward sums (exact, no enumeration
        # needed for this prefix quantity; checked against the full enumeration at t = T-1)
        alpha = p0 * np.tile(emis[0], D)
        for k in range(1, t + 1):
            alpha = (alpha @ trans) * np.tile(emis[k], D)
        cur = np.log(alpha.sum())
        cs[t] = cur - prev
        prev = cur
    del sub
    return post, joint, logZ, cs
