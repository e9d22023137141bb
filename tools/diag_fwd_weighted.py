"""Diagnostic (not collected): how long must the forward warm-up be at steady state of a
C3 fit, under the unweighted Hilbert boundary metric (what k_verify checks) versus the
metric weighted by the exact smoothed posterior at the boundary (what the backward's
verification uses; an output-relevant criterion)?

Runs a C3 fit for n iterations, then, at the last one, the exact forward (verified +
repaired) and backward with gamma, and speculative forward main passes with warm-ups W:
for each, the fraction of chunk starts (s_in[c], the state at t_c - 1) further than tol
from the exact alpha[t_c - 1], unweighted and gamma-weighted."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hilbert_rows(x, y, w=None, lo_thr=1e-30, hi_thr=1e-20):
    import torch
    if w is not None:
        x, y = x * w, y * w
        lo_thr, hi_thr = 1e-14, 1e-12
    x = x / x.amax(1, keepdim=True)
    y = y / y.amax(1, keepdim=True)
    both = (x > lo_thr) & (y > lo_thr)
    bad = (~both) & (torch.maximum(x, y) > hi_thr)
    r = torch.where(both, torch.log(x.clamp_min(1e-38)) - torch.log(y.clamp_min(1e-38)), torch.zeros_like(x))
    hi = torch.where(both, r, torch.full_like(r, -1e30)).amax(1)
    lo = torch.where(both, r, torch.full_like(r, 1e30)).amin(1)
    d = (hi - lo).clamp_min(0)
    d[bad.any(1)] = float('inf')
    return d


def main():
    import torch
    from bench import synth, CONFIGS
    from poor_man_gplvm_amd import _native as nat
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    n_it = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    N, T, L = CONFIGS['c3']
    y, B, W0, lp0 = synth(N, T, L)
    dev = torch.device('cuda', 0)
    C = 49
    eng = DeviceEM(SpikeData(y), L, basis=B, scan=ScanConfig(chunk=C, chunk_bwd=98, warmup=48))
    eng.adaptive = True
    eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    eng.set_log_posterior(lp0)
    lib = eng.lib
    W = torch.as_tensor(W0.astype(np.float64), device=dev).contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    adam = AdamConfig()
    st = torch.zeros(4, dtype=torch.float64, device=dev)
    lh = torch.zeros(1000, dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    lz = torch.zeros(1, dtype=torch.float64, device=dev)
    gamma = torch.empty((T, 2, L), dtype=torch.float32, device=dev)
    for it in range(n_it):
        eng.m_step(W, mu, nu, cnt, adam, st, lh, eh)
        eng.compute_tuning(W)
        eng.e_step(1.0, lz, gamma=gamma if it == n_it - 1 else None, keep_alpha=it == n_it - 1)
    torch.cuda.synchronize()
    M = (T + C - 1) // C
    Lpad = int(lib.pmg_fwdbwd_lpad(L))
    p_in = lib.pmg_fwdbwd_state(nat.ptr(eng.ws_fb), T, L, C, nat.STATE_FWD_IN, 0)
    off = p_in - eng.ws_fb.data_ptr()
    s_in = eng.ws_fb[off:off + M * 2 * Lpad * 4].view(torch.float32).view(M, 2, Lpad)
    tc = torch.arange(1, M, device=dev) * C
    exact = eng.alpha[tc - 1].reshape(M - 1, 2 * L).clone()
    wgt = gamma[tc - 1].reshape(M - 1, 2 * L).clone()
    print(f"C3 after {n_it} EM iterations; {M - 1} forward boundaries, tol {eng.scan.tol:g}")
    alpha_save = eng.alpha.clone()
    for Wm in (2, 4, 8, 12, 16, 24, 32, 48):
        args = (nat.ptr(eng.delta), nat.ptr(eng.phi), nat.ptr(eng.mref), T, ctypes.byref(eng._tr_c), 1.0, C, Wm,
                float(eng.scan.tol), nat.ptr(eng.alpha), nat.ptr(eng.logc), nat.ptr(lz), nat.ptr(eng.ws_fb),
                eng.ws_fb.numel(), nat.stream_handle())
        nat.check(lib.pmg_forward_filter_phase(*args, 1), "fwd")
        torch.cuda.synchronize()
        spec = s_in[1:, :, :L].reshape(M - 1, 2 * L)
        du = hilbert_rows(spec, exact)
        dw = hilbert_rows(spec, exact, wgt)
        tol = eng.scan.tol
        print(f"W={Wm:3d}: unweighted fail {(du > tol).float().mean().item():.3f} (bitwise {(du == 0).float().mean().item():.3f})"
              f" | posterior-weighted fail {(dw > tol).float().mean().item():.3f} (bitwise {(dw == 0).float().mean().item():.3f})",
              flush=True)
    eng.alpha.copy_(alpha_save)


if __name__ == '__main__':
    main()
