"""C4 one EM iteration, single vs 8 shards: which elements differ, and is it the
tuning (suff-stats re-associated over shards) or the scan?"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
import poor_man_gplvm_amd as P  # noqa: E402
from poor_man_gplvm_amd.engine import DeviceEM, ScanConfig, SpikeData  # noqa: E402
from poor_man_gplvm_amd.timeshard import LocalComm, TimeShardedEM, run_em_timesharded, shard_layout  # noqa: E402
from tests.synth import make  # noqa: E402

torch.cuda.set_device(0)
N, L, T = 1024, 1024, 100000
d = make(N, L, T)
tr = P.banded_transition(L, 1.0)
ad = P.AdamConfig(maxiter=40, tol=0.0)
sc = ScanConfig(chunk=64, warmup=16, adaptive=False)
ref, _ = P.run_em(d['y'], d['W0'], d['B'], d['lp0'], n_iter=1, transition=tr, adam=ad, scan=sc)
res, info = run_em_timesharded(d['y'], d['W0'], d['B'], d['lp0'], n_iter=1, transition=tr, world=8, adam=ad,
                               scan=sc, halo=512, chunk=64)
a, b = res['posterior'].astype(np.float64), ref['posterior'].astype(np.float64)
tu_rel = np.abs(res['tuning'].astype(np.float64) - ref['tuning']) / ref['tuning']
print('tuning max rel', tu_rel.max(), 'carry', info['carry_rounds'], 'logz', res['log_marginal_l'], ref['log_marginal_l'], flush=True)
m = np.maximum(a, b) > 1e-12
rel = np.zeros_like(a)
rel[m] = np.abs(a[m] - b[m]) / np.maximum(a[m], b[m])
idx = np.argwhere(rel > 2e-5)
print('bad', len(idx), 'max rel', rel.max(), flush=True)
print('bad t range', idx[:, 0].min() if len(idx) else None, idx[:, 0].max() if len(idx) else None,
      'unique t', np.unique(idx[:, 0]).size if len(idx) else 0, flush=True)
for thr in (1e-12, 1e-10, 1e-8, 1e-6, 1e-4):
    mm = np.maximum(a, b) > thr
    print(f'max rel where >{thr:g}:', (np.abs(a - b)[mm] / np.maximum(a, b)[mm]).max(), flush=True)
# same tuning for both: isolate the scan
tun = ref['tuning'].astype(np.float64)
eng = DeviceEM(SpikeData(d['y']), L, basis=d['B'], scan=sc)
eng.set_transition(tr)
eng.set_tuning(tun)
lz = torch.zeros(1, dtype=torch.float64, device='cuda')
g1 = torch.empty((T, 2, L), dtype=torch.float32, device='cuda')
eng.e_step(1.0, lz, gamma=g1)
al = eng.alpha.cpu().numpy()
g1 = g1.cpu().numpy().astype(np.float64)
print('single same-tuning vs run_em single: max abs', np.abs(g1 - b).max(), 'repairs', eng.repairs(), eng.relax_rounds(), flush=True)
del eng
torch.cuda.empty_cache()
te = TimeShardedEM(d['y'], d['B'], tr, LocalComm(8), shard_layout(T, 8, chunk=64, halo=512), sc)
for s in te.shards:
    s.set_tuning(tun)
gs = [torch.empty((s.T, 2, L), dtype=torch.float32, device='cuda') for s in te.shards]
lz2 = torch.zeros(1, dtype=torch.float64, device='cuda')
te.e_step(1.0, lz2, gamma=gs)
g2 = np.concatenate([x[s.own].cpu().numpy() for s, x in zip(te.shards, gs)], 0).astype(np.float64)
print('same tuning: sharded carry', te.carry_rounds, 'logz', lz.item(), lz2.item(), flush=True)
m = np.maximum(g1, g2) > 1e-12
rel2 = np.zeros_like(g1)
rel2[m] = np.abs(g1[m] - g2[m]) / np.maximum(g1[m], g2[m])
print('same tuning: bad', int((rel2 > 2e-5).sum()), 'max rel', rel2.max(), flush=True)
for (t, dd, l) in np.argwhere(rel > 2e-5)[:20]:
    print(f't={t} d={dd} l={l} sharded={a[t, dd, l]:.4e} single={b[t, dd, l]:.4e} alpha_single={al[t, dd, l]:.4e} '
          f'same-tuning sharded={g2[t, dd, l]:.4e} single={g1[t, dd, l]:.4e}', flush=True)
