"""Mean duration of pmg_tuning_softplus at C3 (L = N = 512, NB = 79) over 200 calls (HIP events)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poor_man_gplvm_amd import _native as nat  # noqa: E402
from poor_man_gplvm_amd.gp_kernel import generate_basis  # noqa: E402

L, N = 512, 512
B = generate_basis(10.0, L).astype(np.float32)
NB = B.shape[1]
W = np.random.default_rng(0).normal(size=(NB, N))
lib = nat.load()
bt = torch.as_tensor(B, device='cuda')
wt = torch.as_tensor(W, device='cuda')
t64 = torch.empty((L, N), dtype=torch.float64, device='cuda')
t32 = torch.empty((L, N), dtype=torch.float32, device='cuda')
call = lambda: lib.pmg_tuning_softplus(nat.ptr(bt), nat.ptr(wt), L, NB, N, nat.ptr(t64), nat.ptr(t32), nat.stream_handle())
for _ in range(20):
    call()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(200):
    call()
b.record()
b.synchronize()
import hashlib  # noqa: E402
print(os.environ.get('PMG_LIB_PATH', 'tree'), 'us per call', round(1e3 * a.elapsed_time(b) / 200, 2), 'sum', float(t64.sum()),
      'sha', hashlib.sha256(t64.cpu().numpy().tobytes() + t32.cpu().numpy().tobytes()).hexdigest()[:16])
