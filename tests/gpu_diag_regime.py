"""Diagnostic (not collected): repairs and fwd/bwd time of the first EM iterations at
C3 for several (chunk, warm-up) settings (flat early tuning = slow forgetting)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import synth, CONFIGS
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig, KernelTimer
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    N, T, L = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'c3']
    y, B, W0, lp0 = synth(N, T, L)
    dev = torch.device('cuda', 0)
    sp = SpikeData(y)
    for C, Wu in [(49, 64), (196, 256), (784, 1024), (3136, 4096)]:
        eng = DeviceEM(sp, L, basis=B, scan=ScanConfig(chunk=C, warmup=Wu, adaptive=False))
        eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
        eng.set_log_posterior(lp0)
        W = torch.as_tensor(W0.astype(np.float64), device=dev).contiguous()
        mu, nu = torch.zeros_like(W), torch.zeros_like(W)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        adam = AdamConfig(lr=0.01, maxiter=1000, tol=1e-6)
        st = torch.zeros(4, dtype=torch.float64, device=dev)
        lh = torch.zeros(1000, dtype=torch.float64, device=dev)
        eh = torch.zeros_like(lh)
        lz = torch.zeros(1, dtype=torch.float64, device=dev)
        out = []
        for it in range(4):
            eng.m_step(W, mu, nu, cnt, adam, st, lh, eh)
            eng.compute_tuning(W)
            torch.cuda.synchronize()
            timer = KernelTimer()
            eng.timer = timer
            eng.e_step(1.0, lz)
            torch.cuda.synchronize()
            s = timer.summary()
            eng.timer = None
            out.append(f"it{it}: fwd {s['forward_filter'][1]:.2f} bwd {s['backward_smoother'][1]:.2f} ms rep {eng.repairs()} logZ {float(lz.item()):.6f}")
        print(f"C={C} W={Wu} M={(T + C - 1) // C}: " + " | ".join(out), flush=True)


if __name__ == '__main__':
    main()
