"""Timings of the non-headline paths on one GPU (C3 shape: N=512, T=1e5, L=512):
  * Gaussian EM iteration (GaussianGPLVMJump1D): suff-stats, analytic M-step,
    linear tuning, Gaussian emission, fwd-bwd;
  * one masked forward-only decode of get_downsampled_lml (log_marginal_masked).
Per-kernel times from HIP events (KernelTimer); prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from bench import synth
from poor_man_gplvm_amd.engine import AdamConfig, DeviceEM, KernelTimer, ScanConfig, SpikeData
from poor_man_gplvm_amd.gp_kernel import banded_transition


def timed(fn, steps, warm):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    N, T, L = 512, 100000, 512
    y, B, W0, lp0 = synth(N, T, L)
    dev = torch.device("cuda", 0)
    out = {"config": f"N={N} T={T} L={L} nb={B.shape[1]}"}

    # Gaussian EM iteration (spikes reused as real-valued observations)
    yg = (y.astype(np.float32) + 0.25 * np.random.default_rng(5).normal(size=y.shape)).astype(np.float32)
    eng = DeviceEM(SpikeData(yg), L, basis=B, scan=ScanConfig())
    eng.noise_std, eng.gauss_prior_std = 0.5, 1.0
    eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    eng.set_log_posterior(lp0)
    W = torch.zeros((B.shape[1], N), dtype=torch.float64, device=dev)
    logz = torch.zeros(1, dtype=torch.float64, device=dev)

    def gauss_iter():
        eng.m_step(W, None, None, None, None, None, None, None)
        eng.compute_tuning(W)
        eng.e_step(1.0, logz)

    timed(gauss_iter, 1, 3)
    eng.timer = KernelTimer()
    s = timed(gauss_iter, 5, 0)
    eng.gaussian_status()
    out["gaussian_em_iter_ms"] = 1e3 * s
    out["gaussian_em_iters_per_s"] = 1.0 / s
    out["gaussian_kernels_ms"] = {k: round(v[1], 4) for k, v in eng.timer.summary().items()}
    em = out["gaussian_kernels_ms"].get("emission", 0.0)
    out["gaussian_emission_TFLOPs"] = 3.0 * T * L * N / (em * 1e-3) / 1e12 if em else None

    # masked forward-only decode (one downsampled-LML repeat)
    sp = SpikeData(y)
    e2 = DeviceEM(sp, L, scan=ScanConfig())
    e2.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    tun = np.log1p(np.exp(B.astype(np.float64) @ W0.astype(np.float64)))
    e2.set_tuning(tun)
    mask = np.zeros(L)
    mask[np.random.default_rng(0).choice(L, int(0.2 * L), replace=False)] = 1
    lz = torch.zeros(1, dtype=torch.float64, device=dev)

    def masked():
        e2.set_ma_latent(mask)
        e2.emission(1.0)
        e2.forward(1.0, lz)

    timed(masked, 1, 3)
    e2.timer = KernelTimer()
    s2 = timed(masked, 10, 0)
    out["masked_lml_ms_per_mask"] = 1e3 * s2
    out["masked_lml_kernels_ms"] = {k: round(v[1], 4) for k, v in e2.timer.summary().items()}

    # get_downsampled_lml's default n_repeat = 10 masks, batched (one emission contraction,
    # then per group: stacked masks, row references, one forward launch without alpha)
    R = 10
    rng = np.random.default_rng(1)
    masks = np.zeros((R, L), np.uint8)
    for r in range(R):
        masks[r, rng.choice(L, int(0.2 * L), replace=False)] = 1
    e2.set_ma_latent(None)
    e2.timer = None
    delta0, rblk0 = e2.emission_unmasked()
    mu8 = torch.as_tensor(masks, device=dev)
    lzR = torch.zeros(R, dtype=torch.float64, device=dev)
    Rg = e2.mask_batch_size(R)

    def masked_batch():
        for r0 in range(0, R, Rg):
            e2.masked_logz_batched(delta0, rblk0, mu8[r0:r0 + Rg], 1.0, lzR[r0:r0 + Rg])

    timed(masked_batch, 1, 2)
    e2.timer = KernelTimer()
    s3 = timed(masked_batch, 5, 0)
    out["masked_lml_batched_ms_per_mask"] = 1e3 * s3 / R
    out["masked_lml_batched_kernels_ms"] = {k: round(v[1], 4) for k, v in e2.timer.summary().items()}

    # naive-Bayes shuffles (test.shuffle_and_decode's default decoder), batched by stacking
    from poor_man_gplvm_amd import PoissonGPLVMJump1D
    from poor_man_gplvm_amd import test as PT
    m = PoissonGPLVMJump1D(N, n_latent_bin=L)
    m.tuning = tun
    dec = PT.ShuffleDecoder(m, y, 'naive_bayes')
    nsh = 8
    shifts = [np.random.default_rng(10 + i).integers(0, T, size=N) for i in range(nsh)]
    dec.decode_naive_bayes_batch(shifts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dec.decode_naive_bayes_batch(shifts)
    out["nb_shuffle_batched_ms_per_shuffle_incl_host_copies"] = 1e3 * (time.perf_counter() - t0) / nsh
    t0 = time.perf_counter()
    for s in shifts[:2]:
        dec.decode(s)
    out["nb_shuffle_sequential_ms_per_shuffle_incl_host_copies"] = 1e3 * (time.perf_counter() - t0) / 2
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
