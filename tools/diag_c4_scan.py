"""C4 after one M-step from a random posterior: banded scan (chunk 64 / 200) vs the
dense log-domain scan (f64 state) on the same f64 tuning.  Which one is off, and where
(time bin mod chunk)?"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
import poor_man_gplvm_amd as P  # noqa: E402
from poor_man_gplvm_amd.engine import DeviceEM, ScanConfig, SpikeData  # noqa: E402
from poor_man_gplvm_amd.gp_kernel import transition_from_log_kernels, create_transition_prob_1d  # noqa: E402
from tests.synth import make  # noqa: E402

torch.cuda.set_device(0)
N, L, T = 1024, 1024, 100000
d = make(N, L, T)
sp = SpikeData(d['y'])
tr = P.banded_transition(L, 1.0)
eng = DeviceEM(sp, L, basis=d['B'], scan=ScanConfig(chunk=64, warmup=16, adaptive=False))
eng.set_transition(tr)
eng.set_log_posterior(d['lp0'])
W = torch.as_tensor(d['W0'].astype(np.float64), device='cuda').contiguous()
mu, nu = torch.zeros_like(W), torch.zeros_like(W)
cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
stats = torch.zeros(4, dtype=torch.float64, device='cuda')
lh = torch.zeros(40, dtype=torch.float64, device='cuda')
eng.m_step(W, mu, nu, cnt, P.AdamConfig(maxiter=40, tol=0.0), stats, lh, torch.zeros_like(lh))
eng.compute_tuning(W)
tun = eng.tuning64.cpu().numpy()
np.save('gpurun_out/c4_tuning.npy', tun.astype(np.float32))
del eng
torch.cuda.empty_cache()


def run(chunk, warmup, dense=False, tol=None):
    sc = ScanConfig(chunk=chunk, warmup=warmup, adaptive=False) if tol is None else \
        ScanConfig(chunk=chunk, warmup=warmup, adaptive=False, tol=tol)
    e = DeviceEM(sp, L, scan=sc)
    if dense:
        _, logK, _, logA = create_transition_prob_1d(L, 1.0)
        e.set_transition(transition_from_log_kernels(logK, logA, force_dense=True))
    else:
        e.set_transition(tr)
    e.set_tuning(tun)
    lz = torch.zeros(1, dtype=torch.float64, device='cuda')
    g = torch.empty((T, 2, L), dtype=torch.float32, device='cuda')
    lg = torch.empty((T, 2, L), dtype=torch.float32, device='cuda') if dense else None
    e.e_step(1.0, lz, gamma=g, log_gamma=lg)
    out = g.cpu().numpy().astype(np.float64)
    info = (lz.item(), e.repairs(), e.relax_rounds())
    del e, g
    torch.cuda.empty_cache()
    return out, info


res = {}
for name, args in [('b64', (64, 16)), ('b64w48', (64, 48)), ('b200', (200, 48)), ('b64tol', (64, 16, False, 1e-7)),
                   ('dense', (None, 48, True))]:
    res[name] = run(*args)
    print(name, 'logz %.6f' % res[name][1][0], 'repairs', res[name][1][1], 'rounds', res[name][1][2], flush=True)
ref = res['dense'][0]
for name in ('b64', 'b64w48', 'b200', 'b64tol'):
    a = res[name][0]
    m = np.maximum(a, ref) > 1e-12
    rel = np.zeros_like(a)
    rel[m] = np.abs(a[m] - ref[m]) / np.maximum(a[m], ref[m])
    bad = rel > 2e-5
    ts = np.unique(np.argwhere(bad)[:, 0])
    print(f'{name} vs dense: bad {int(bad.sum())} in {ts.size} bins, max rel {rel.max():.3e}, max abs '
          f'{np.abs(a - ref).max():.3e}', flush=True)
    if ts.size:
        print('   t mod 64 hist (first 16 residues):', np.bincount(ts % 64, minlength=64)[:16], flush=True)
        print('   t mod 64 hist (last 16 residues):', np.bincount(ts % 64, minlength=64)[48:], flush=True)
        print('   first ts', ts[:30], flush=True)
        worst = np.unravel_index(np.argmax(rel), rel.shape)
        print('   worst', worst, a[worst], ref[worst], flush=True)
