"""CPU baseline: the reference's EM iteration in float32 on all host cores (torch-CPU).

TEST / BENCH INFRASTRUCTURE ONLY.  Only ``bench.py``'s ``cpu_baseline`` leg imports this
module; the product package never does.

It restates the reference's own dataflow at its own precision (float32, no x64 anywhere
in the reference) so that the timed CPU work matches what JAX-CPU runs for one EM
iteration, vectorised per time step with torch's multi-threaded CPU kernels:
  * emission        decoder.py:30-48  ll = (m*y) @ log(lam)^T - m @ lam^T - sum gammaln(y+1)
  * forward filter  decoder.py:151-172 (dense logsumexp over the (D, L, L) kernel)
  * smoother        decoder.py:200-226 (dense (D, D, L, L) tensor per step, logsumexp
                    over (d', j), and the joint accumulated with logaddexp every step,
                    as smooth_all_step_combined_ma_chunk always does, decoder.py:221)
  * marginal        core.py:668
  * suff-stats      fit_tuning_helper.py:28-42
  * Adam loop       fit_tuning_helper.py:63-81 + :133-194 (value_and_grad + optax adam)
The numerics are checked against the float64 oracle in tests/test_cpu_baseline.py.
"""
from __future__ import annotations

import math

import torch

RATE_EPS = 1e-20


def transition_logs(L, movement_variance=1.0, p_move_to_jump=0.01, p_jump_to_move=0.01):
    """gp_kernel.py:42-89 in float32: logK (D, L, L) [d_next, i_prev, j_next], logA (D, D)."""
    x = torch.arange(L, dtype=torch.float32)
    lk0 = -(x[:, None] - x[None, :]) ** 2 / float(movement_variance) ** 2
    lk0 = lk0 - torch.logsumexp(lk0, dim=1, keepdim=True)
    lk1 = torch.full((L, L), -math.log(L), dtype=torch.float32)
    logK = torch.stack([lk0, lk1])
    A = torch.tensor([[1 - p_move_to_jump, p_move_to_jump], [p_jump_to_move, 1 - p_jump_to_move]],
                     dtype=torch.float32)
    return logK, torch.log(A)


def emission(y, tuning):
    """decoder.py:30-48 vmapped over time (decoder.py:60-71), no masks."""
    lam = tuning + RATE_EPS
    return y @ torch.log(lam).T - lam.sum(1)[None, :] - torch.lgamma(y + 1.0).sum(1, keepdim=True)


def filter_all(ll, logK, logA):
    """decoder.py:151-187: per step a = LSE_d(post + logA); prior = LSE_i(a + logK);
    post = prior + ll - c.  Returns (posts, priors, logZ)."""
    T, L = ll.shape
    D = logA.shape[0]
    post = torch.full((D, L), -math.log(D * L))
    posts = torch.empty((T, D, L))
    priors = torch.empty((T, D, L))
    logz = torch.zeros(())
    for t in range(T):
        a = torch.logsumexp(post[:, None, :] + logA[:, :, None], dim=0)
        prior = torch.logsumexp(a[:, :, None] + logK, dim=1)
        u = prior + ll[t][None, :]
        c = torch.logsumexp(u.reshape(-1), dim=0)
        post = u - c
        logz = logz + c
        posts[t], priors[t] = post, prior
    return posts, priors, logz


def smooth_all(posts, priors, logK, logA):
    """decoder.py:200-256 (single chunk): X[d,d',i,j] = logK + logA + (acausal_{t+1} -
    prior_{t+1}) + post_t; acausal_t = LSE_{d',j} X; joint = logaddexp(joint, X)."""
    T, D, L = posts.shape
    acausal = posts[-1]
    joint = torch.full((D, D, L, L), -math.inf)
    out = torch.empty((T, D, L))
    out[-1] = acausal
    base = logK[None, :, :, :] + logA[:, :, None, None]
    for t in range(T - 2, -1, -1):
        diff = acausal - priors[t + 1]
        X = base + diff[None, :, None, :] + posts[t][:, None, :, None]
        acausal = torch.logsumexp(X, dim=(1, 3))
        joint = torch.logaddexp(joint, X)
        out[t] = acausal
    return out, joint


def objective_and_grad(W, prior_std, basis, yw, tw):
    """fit_tuning_helper.py:63-81 and its gradient (value_and_grad)."""
    F = basis @ W
    f = torch.nn.functional.softplus(F)
    ll = torch.sum(torch.xlogy(yw, f + RATE_EPS) - f * tw[:, None])
    logprior = torch.sum(-0.5 * (W / prior_std) ** 2 - math.log(prior_std) - 0.5 * math.log(2 * math.pi))
    G = (yw / (f + RATE_EPS) - tw[:, None]) * torch.sigmoid(F)
    return -ll - logprior, -(basis.T @ G) + W / prior_std ** 2


def adam_steps(W, basis, yw, tw, n, lr=0.01, b1=0.9, b2=0.999, eps=1e-8, prior_std=1.0):
    """n bodies of the while loop of fit_tuning_helper.py:166-179 (optax 0.2.2 adam)."""
    mu = torch.zeros_like(W)
    nu = torch.zeros_like(W)
    loss = None
    for k in range(1, n + 1):
        loss, g = objective_and_grad(W, prior_std, basis, yw, tw)
        mu = (1 - b1) * g + b1 * mu
        nu = (1 - b2) * g * g + b2 * nu
        W = W - lr * (mu / (1 - b1 ** k)) / (torch.sqrt(nu / (1 - b2 ** k)) + eps)
        _ = float(torch.sqrt(torch.sum(g * g)))   # the error history the loop records
    return W, loss


def em_iteration_sample(y, tuning, basis, W, logK, logA, adam_bodies):
    """One EM iteration's work on a time sample: E-step (emission, filter, smoother with
    joint, dynamics marginal), sufficient statistics, `adam_bodies` Adam bodies."""
    ll = emission(y, tuning)
    posts, priors, logz = filter_all(ll, logK, logA)
    acausal, joint = smooth_all(posts, priors, logK, logA)
    logpost = torch.logsumexp(acausal, dim=1)                     # core.py:668
    P = torch.exp(logpost)
    yw, tw = P.T @ y, P.sum(0)                                    # fit_tuning_helper.py:38-41
    W, loss = adam_steps(W, basis, yw, tw, adam_bodies)
    return logz, joint, W
