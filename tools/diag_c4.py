"""Diagnose single-GPU vs 8-shard differences at C4 (N=L=1024, T=1e5): where do
posterior elements > 1e-12 differ by more than rel 2e-5, and what are the filter
(alpha) values there -- are they in f32's denormal range?"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
import poor_man_gplvm_amd as P  # noqa: E402
from poor_man_gplvm_amd.engine import DeviceEM, ScanConfig, SpikeData  # noqa: E402
from poor_man_gplvm_amd.timeshard import LocalComm, TimeShardedEM, shard_layout  # noqa: E402
from tests.synth import make  # noqa: E402

torch.cuda.set_device(0)
N, L, T = 1024, 1024, 100000
d = make(N, L, T)
tr = P.banded_transition(L, 1.0)
sc = ScanConfig(chunk=64, warmup=16, adaptive=False)
eng = DeviceEM(SpikeData(d['y']), L, basis=d['B'], scan=sc)
eng.set_transition(tr)
eng.set_tuning(d['tuning'])
logz = torch.zeros(1, dtype=torch.float64, device='cuda')
gam = torch.empty((T, 2, L), dtype=torch.float32, device='cuda')
eng.e_step(1.0, logz, gamma=gam)
a1 = gam.cpu().numpy()
alpha = eng.alpha.cpu().numpy()
print('single logz', logz.item(), 'repairs', eng.repairs(), 'rounds', eng.relax_rounds(), flush=True)
del eng
torch.cuda.empty_cache()
lays = shard_layout(T, 8, chunk=64, halo=512)
te = TimeShardedEM(d['y'], d['B'], tr, LocalComm(8), lays, sc)
for s in te.shards:
    s.set_tuning(d['tuning'])
g = [torch.empty((s.T, 2, L), dtype=torch.float32, device='cuda') for s in te.shards]
lz2 = torch.zeros(1, dtype=torch.float64, device='cuda')
te.e_step(1.0, lz2, gamma=g)
a2 = np.concatenate([x[s.own].cpu().numpy() for s, x in zip(te.shards, g)], 0)
al2 = np.concatenate([s.alpha[s.own].cpu().numpy() for s in te.shards], 0)
print('sharded logz', lz2.item(), 'carry', te.carry_rounds, flush=True)
m = np.maximum(a1, a2) > 1e-12
rel = np.zeros_like(a1, dtype=np.float64)
rel[m] = np.abs(a1[m].astype(np.float64) - a2[m]) / np.maximum(a1[m], a2[m])
bad = rel > 2e-5
print('bad', int(bad.sum()), 'of', int(m.sum()), 'max rel', rel.max(), flush=True)
idx = np.argwhere(bad)
ts = np.unique(idx[:, 0])
print('bad time bins', ts.size, ts[:40], flush=True)
for (t, dd, l) in idx[:25]:
    print(f't={t} d={dd} l={l} g1={a1[t, dd, l]:.4e} g2={a2[t, dd, l]:.4e} alpha1={alpha[t, dd, l]:.4e} '
          f'alpha2={al2[t, dd, l]:.4e} row_max_alpha={alpha[t].max():.3e}', flush=True)
den = (np.abs(alpha) < 1.1754944e-38) & (alpha != 0)
print('denormal alpha fraction', den.mean(), 'at bad', den[bad].mean() if bad.any() else None, flush=True)
# abs error stats
ad = np.abs(a1.astype(np.float64) - a2)
print('max abs diff', ad.max(), 'max abs diff where >1e-9', ad[np.maximum(a1, a2) > 1e-9].max(), flush=True)
for thr in (1e-12, 1e-10, 1e-9, 1e-8, 1e-6):
    mm = np.maximum(a1, a2) > thr
    print(f'max rel where >{thr:g}:', (ad[mm] / np.maximum(a1, a2)[mm]).max(), flush=True)
