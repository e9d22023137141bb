"""Per-phase ticks of the persistent Adam kernel body at a BASELINE shape
(PMG_ADAM_PROF stamps: rows | barrier 1 | element update | sums+barrier 2+publish | loop)
and its mean duration per body from HIP events.  usage: adam_prof.py [N T L] [maxiter]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from poor_man_gplvm_amd.engine import AdamConfig, DeviceEM, KernelTimer, SpikeData  # noqa: E402

N, T, L = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (512, 100000, 512)
maxiter = int(sys.argv[4]) if len(sys.argv) >= 5 else 300
torch.cuda.set_device(0)
y, B, W0, lp0 = bench.synth(N, T, L)
eng = DeviceEM(SpikeData(y), L, basis=B)
eng.set_log_posterior(lp0)
eng.timer = KernelTimer()
print(f'N={N} T={T} L={L} NB={B.shape[1]} maxiter={maxiter}', flush=True)
for rep in range(4):
    W = torch.as_tensor(W0.astype(np.float64), device='cuda').contiguous()
    z = torch.zeros_like(W)
    stats = torch.zeros(4, dtype=torch.float64, device='cuda')
    lh = torch.zeros(maxiter, dtype=torch.float64, device='cuda')
    if rep == 3:
        os.environ['PMG_ADAM_PROF'] = '1'
    eng.timer.reset()
    eng.m_step(W, z, z.clone(), torch.zeros(1, dtype=torch.int64, device='cuda'), AdamConfig(maxiter=maxiter, tol=0.0),
               stats, lh, lh.clone())
    s = eng.timer.summary()
    n = int(stats[0].item())
    ms = s['mstep_adam'][1]
    print(f'rep {rep}: n_iter {n}  adam {ms * 1e3:.1f} us  = {ms * 1e3 / max(n, 1):.2f} us/body  '
          f'suffstats {s["suffstats"][1] * 1e3:.1f} us', flush=True)
