"""Diagnostic (not collected): persistent row-block Adam vs the tiled f64 kernel vs the f64
oracle on an L = 1024 shape (n_iter, max relative tuning deviation, loss histories)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gplvm_oracle as O  # noqa: E402
from tests.synth import make  # noqa: E402
from tests.test_gpu_parity import _engine  # noqa: E402


def run(N, L, maxiter, tol, tiled):
    from poor_man_gplvm_amd.engine import AdamConfig
    d = make(N, L, 500)
    sp, eng = _engine(d, L)
    if tiled:
        eng.PERSISTENT_MAX_L = 0
    yw, tw = O.get_statistics(d['lp0'].astype(np.float64), d['y'])
    eng.yw.copy_(torch.as_tensor(yw, device='cuda'))
    eng.tw.copy_(torch.as_tensor(tw, device='cuda'))
    W = torch.as_tensor(d['W0'].astype(np.float64), device='cuda').contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
    stats = torch.zeros(4, dtype=torch.float64, device='cuda')
    lh = torch.zeros(max(maxiter, 1), dtype=torch.float64, device='cuda')
    eh = torch.zeros_like(lh)
    eng.adam(W, mu, nu, cnt, AdamConfig(maxiter=maxiter, tol=tol), stats, lh, eh)
    ref = O.adam_run(d['W0'].astype(np.float64), O.adam_init(d['W0']), 1.0, d['B'].astype(np.float64), yw, tw,
                     maxiter=maxiter, tol=tol)
    B = d['B'].astype(np.float64)
    t_got = np.logaddexp(B @ W.cpu().numpy(), 0)
    t_ref = np.logaddexp(B @ ref['params'], 0)
    n = int(stats[0].item())
    rel = np.max(np.abs(t_got - t_ref) / np.abs(t_ref))
    lrel = np.max(np.abs(lh.cpu().numpy()[:n] - ref['loss_history'][:n]) / np.abs(ref['loss_history'][:n]))
    print(f"N={N} L={L} NB={B.shape[1]} maxiter={maxiter} tol={tol} {'tiled' if tiled else 'persistent'}: "
          f"n_iter {n} (oracle {ref['n_iter']}), tuning max rel {rel:.2e}, loss hist max rel {lrel:.2e}", flush=True)


if __name__ == '__main__':
    torch.cuda.set_device(0)
    for N, L, mi in [(128, 1024, 1000), (128, 1024, 200), (64, 1024, 1000), (30, 100, 1000), (128, 256, 1000)]:
        for tiled in (False, True):
            run(N, L, mi, 1e-6, tiled)
