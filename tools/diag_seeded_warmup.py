"""Diagnostic (not collected): would seeding each forward chunk's warm-up from the PREVIOUS
EM iteration's filter state let the warm-up shrink?  

Runs a C3 fit for n iterations keeping the exact (verified + repaired) filter alpha of the
last two E-steps.  For every chunk boundary t_c (chunk 49) and warm-up W it runs W filter
steps of iteration n (its emission, the model's transition; dense f64 torch on the GPU)
from (a) iteration n-1's alpha at t_c - W - 1 (the seed) and (b) the uniform state (the
main pass today), and measures the Hilbert distance of the result to iteration n's exact
alpha at t_c - 1, unweighted (what k_verify checks) -- the fraction of boundaries above
tol is the fraction the relaxation would have to repair."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))


def main():
    import torch
    from bench import synth, CONFIGS
    from diag_fwd_weighted import hilbert_rows
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig
    from poor_man_gplvm_amd.gp_kernel import banded_transition, create_transition_prob_1d
    n_it = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    N, T, L = CONFIGS['c3']
    y, B, W0, lp0 = synth(N, T, L)
    dev = torch.device('cuda', 0)
    C = 49
    eng = DeviceEM(SpikeData(y), L, basis=B, scan=ScanConfig(chunk=C, chunk_bwd=98, warmup=48))
    eng.adaptive = True
    eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    eng.set_log_posterior(lp0)
    K, _, A, _ = create_transition_prob_1d(L, 1.0, 0.01, 0.01)
    Kt = torch.as_tensor(np.asarray(K, np.float64), device=dev)      # (2, L, L) [d', i, j]
    At = torch.as_tensor(np.asarray(A, np.float64), device=dev)      # (2, 2) [d, d']
    W = torch.as_tensor(W0.astype(np.float64), device=dev).contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.zeros(4, dtype=torch.float64, device=dev)
    lh = torch.zeros(1000, dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    lz = torch.zeros(1, dtype=torch.float64, device=dev)
    gam = torch.empty((T, 2, L), dtype=torch.float32, device=dev)
    prev = None
    for it in range(n_it):
        eng.m_step(W, mu, nu, cnt, AdamConfig(), st, lh, eh)
        eng.compute_tuning(W)
        keep = it >= n_it - 2
        eng.e_step(1.0, lz, gamma=gam if keep else None, keep_alpha=keep)
        if it == n_it - 2:
            prev = eng.alpha.double().clone()
    torch.cuda.synchronize()
    cur = eng.alpha.double()
    # iteration n's emission factor, per-row scaled: e = exp(delta + phi[block])
    blk = torch.arange(L, device=dev) // 32
    e = torch.exp(eng.delta.double() + eng.phi.double()[:, blk])
    M = (T + C - 1) // C
    tc = torch.arange(1, M, device=dev) * C
    exact = cur[tc - 1].reshape(M - 1, 2 * L)

    def run(state, t0, Wm):
        x = state / state.sum((1, 2), keepdim=True)
        for k in range(Wm):
            t = t0 + k
            # prior[d', j] = sum_d A[d, d'] sum_i x[d, i] K[d', i, j]
            mix = torch.einsum('mdi,de->mei', x, At)
            pr = torch.einsum('mei,eij->mej', mix, Kt)
            x = pr * e[t][:, None, :]
            x = x / x.sum((1, 2), keepdim=True)
        return x.reshape(x.shape[0], 2 * L)

    tol = eng.scan.tol
    print(f"C3 after {n_it} EM iterations; {M - 1} forward boundaries, tol {tol:g}", flush=True)
    for Wm in (2, 4, 8, 12, 16, 24, 32):
        t0 = tc - Wm
        seeded = run(prev[t0 - 1], t0, Wm)
        unif = run(torch.ones((M - 1, 2, L), dtype=torch.float64, device=dev), t0, Wm)
        ds = hilbert_rows(seeded, exact)
        du = hilbert_rows(unif, exact)
        print(f"W={Wm:3d}: seeded fail {(ds > tol).float().mean().item():.3f} (median {ds.median().item():.2e})"
              f" | uniform fail {(du > tol).float().mean().item():.3f} (median {du.median().item():.2e})", flush=True)
    d0 = hilbert_rows(prev[tc - 1].reshape(M - 1, 2 * L), exact)
    print(f"no warm-up, previous iteration's state at t_c - 1: fail {(d0 > tol).float().mean().item():.3f}"
          f" (median {d0.median().item():.2e})", flush=True)


if __name__ == '__main__':
    main()
