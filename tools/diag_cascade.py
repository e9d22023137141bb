"""Diagnostic (not collected): how fast do chunk boundaries of the forward filter forget
their start in the first EM iterations of a C3 fit?

Per EM iteration it runs the exact (verified + repaired) forward, then speculative
passes with several warm-ups, and reports the Hilbert-metric distance between each
speculative chunk start (s_in[c], the state at t_c - 1 after the warm-up) and the
exact filtered state at the same time: quantiles and the fraction above tol.
It also reports how far the exact boundary states moved since the previous EM
iteration (the quality of a warm start from the last E-step)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hilbert_rows(x, y, lo_thr=1e-30, hi_thr=1e-20):
    import torch
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
    n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    SWEEP = [int(v) for v in sys.argv[3].split(',')] if len(sys.argv) > 3 and sys.argv[3] else []
    tol = float(sys.argv[4]) if len(sys.argv) > 4 else 3e-6
    N, T, L = CONFIGS[cfg]
    y, B, W0, lp0 = synth(N, T, L)
    dev = torch.device('cuda', 0)
    sp = SpikeData(y)
    C = 49 if cfg == 'c3' else max(32, -(-T // 2048))
    eng = DeviceEM(sp, L, basis=B, scan=ScanConfig(chunk=C, warmup=48, adaptive=False, tol=tol))
    eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    eng.set_log_posterior(lp0)
    lib = eng.lib
    W = torch.as_tensor(W0.astype(np.float64), device=dev).contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    adam = AdamConfig(lr=0.01, maxiter=1000, tol=1e-6)
    st = torch.zeros(4, dtype=torch.float64, device=dev)
    lh = torch.zeros(1000, dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    lz = torch.zeros(1, dtype=torch.float64, device=dev)
    M = (T + C - 1) // C
    Lpad = int(lib.pmg_fwdbwd_lpad(L))
    s_in_ptr = lib.pmg_fwdbwd_state(nat.ptr(eng.ws_fb), T, L, C, nat.STATE_FWD_IN, 0)
    base = eng.ws_fb.data_ptr()
    off = s_in_ptr - base
    s_in = eng.ws_fb[off:off + M * 2 * Lpad * 4].view(torch.float32).view(M, 2, Lpad)
    tc = torch.arange(1, M, device=dev) * C
    prev_exact = None
    for it in range(n_it):
        eng.m_step(W, mu, nu, cnt, adam, st, lh, eh)
        eng.compute_tuning(W)
        eng.emission(1.0)
        torch.cuda.synchronize()
        from poor_man_gplvm_amd.engine import KernelTimer
        timer = KernelTimer()
        eng.timer = timer
        t0 = time.perf_counter()
        eng.forward(1.0, lz)
        eng.backward(1.0)
        torch.cuda.synchronize()
        t_fb = time.perf_counter() - t0
        eng.timer = None
        sm = timer.summary()
        exact = eng.alpha[tc - 1].reshape(M - 1, 2 * L).clone()
        reps = eng.repairs()
        rr = eng.relax_rounds()
        line = [f"it{it} (tol {tol:g}): fwd {sm['forward_filter'][1]:.3f} + relax {sm['forward_repair'][1]:.3f} ms, "
                f"bwd {sm['backward_smoother'][1]:.3f} + relax {sm['backward_repair'][1]:.3f} ms "
                f"(wall {1e3 * t_fb:.1f} ms); recomputed chunks {reps}, rounds {rr}, adam_it {int(st[0].item())}, "
                f"logZ {lz.item():.6f}"]
        if prev_exact is not None:
            d = hilbert_rows(exact, prev_exact)
            line.append(f"  vs prev-iter exact: q50 {d.quantile(0.5).item():.3g} q90 {d.quantile(0.9).item():.3g} "
                        f"max {d.max().item():.3g} frac>1e-6 {(d > 1e-6).float().mean().item():.3f}")
        prev_exact = exact
        Bw = 0
        for Bw in SWEEP:
            args = (nat.ptr(eng.delta), nat.ptr(eng.phi), nat.ptr(eng.mref), T, __import__('ctypes').byref(eng._tr_c),
                    1.0, C, Bw, 1e-6, nat.ptr(eng.alpha), nat.ptr(eng.logc), nat.ptr(lz), nat.ptr(eng.ws_fb),
                    eng.ws_fb.numel(), nat.stream_handle())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nat.check(lib.pmg_forward_filter_phase(*args, 1), "fwd")
            torch.cuda.synchronize()
            t1 = time.perf_counter() - t0
            spec = s_in[1:, :, :L].reshape(M - 1, 2 * L)
            d = hilbert_rows(spec, exact)
            fin = d[torch.isfinite(d)]
            q = (lambda p: fin.quantile(p).item() if fin.numel() else float('nan'))
            line.append(f"  B={Bw:5d} ({1e3 * t1:6.1f} ms): frac>1e-6 {(d > 1e-6).float().mean().item():.3f} "
                        f"inf {(~torch.isfinite(d)).float().mean().item():.3f} q50 {q(0.5):.3g} q90 {q(0.9):.3g} "
                        f"q99 {q(0.99):.3g}")
        if SWEEP:  # restore the exact alpha for the backward / next M-step
            eng.forward(1.0, lz)
            eng.backward(1.0)
            torch.cuda.synchronize()
        print("\n".join(line), flush=True)


if __name__ == '__main__':
    main()
