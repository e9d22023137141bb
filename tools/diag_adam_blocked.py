"""Diagnostic (not collected): the Adam M-step at the C4 shape (N = L = 1024, NB = 154) as
the tiled f64 kernels, as neuron blocks of the persistent kernel (4 and 8 blocks), and
against the f64 oracle: max relative tuning differences after `maxiter` bodies."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gplvm_oracle as O  # noqa: E402
from tests.synth import make  # noqa: E402
from poor_man_gplvm_amd.engine import AdamConfig, DeviceEM, SpikeData  # noqa: E402
from poor_man_gplvm_amd.gp_kernel import banded_transition  # noqa: E402
from poor_man_gplvm_amd.timeshard import neuron_bounds  # noqa: E402

N = L = 1024
maxiter = int(sys.argv[1]) if len(sys.argv) > 1 else 150
d = make(N, L, 2000)
eng = DeviceEM(SpikeData(d['y']), L, basis=d['B'])
eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
yw, tw = O.get_statistics(d['lp0'].astype(np.float64), d['y'])
eng.yw.copy_(torch.as_tensor(yw, device='cuda'))
eng.tw.copy_(torch.as_tensor(tw, device='cuda'))
B = d['B'].astype(np.float64)


def run(mode):
    W = torch.as_tensor(d['W0'].astype(np.float64), device='cuda').contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
    st = torch.zeros(4, dtype=torch.float64, device='cuda')
    lh = torch.zeros(maxiter, dtype=torch.float64, device='cuda')
    cfg = AdamConfig(maxiter=maxiter, tol=0.0)
    if mode == 'tiled':
        eng.ADAM_BLOCKED = False
        eng.adam(W, mu, nu, cnt, cfg, st, lh, lh.clone())
        eng.ADAM_BLOCKED = True
    else:
        eng._adam_blocked(W, mu, nu, cnt, cfg, st, lh, lh.clone(), eng.yw, neuron_bounds(N, int(mode)))
    eng.adam_status()
    return W.cpu().numpy(), int(st[0].item())


ref = O.adam_run(d['W0'].astype(np.float64), O.adam_init(d['W0']), 1.0, B, yw, tw, maxiter=maxiter, tol=0.0)
tun_ref = np.logaddexp(B @ ref['params'], 0)
res = {m: run(m) for m in ('tiled', '8', '16')}
for m, (W, n) in res.items():
    t = np.logaddexp(B @ W, 0)
    print(m, 'n_iter', n, 'vs oracle tuning rel', np.abs(t / tun_ref - 1).max(), flush=True)
t4 = np.logaddexp(B @ res['16'][0], 0)
t8 = np.logaddexp(B @ res['8'][0], 0)
tt = np.logaddexp(B @ res['tiled'][0], 0)
print('16 vs 8 blocks', np.abs(t4 / t8 - 1).max(), 'W equal', np.array_equal(res['16'][0], res['8'][0]))
print('8 blocks vs tiled', np.abs(t8 / tt - 1).max())
