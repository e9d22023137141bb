"""Per-key relative errors of the transition / joint outputs (decode_latent goldens, the
scan joint of test_forward_backward_vs_oracle, the latent-only joint) -- the numbers
behind the tolerances documented in tests/test_gpu_parity.py."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gplvm_oracle as O  # noqa: E402
from tests.synth import make  # noqa: E402
import poor_man_gplvm_amd as P  # noqa: E402

torch.cuda.set_device(0)


def rel(a, b, floor):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    m = np.abs(b) > floor
    return float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m]))) if m.any() else 0.0


out = {}
for name in ('decode_small.npz', 'decode_masked.npz'):
    f = np.load(os.path.join(ROOT, 'tests', 'golden', name))
    L = f['tuning'].shape[0]
    m = P.PoissonGPLVMJump1D(f['y'].shape[1], n_latent_bin=L, tuning_lengthscale=5., movement_variance=float(f['mv']))
    r = m.decode_latent(f['y'].astype(np.float32), tuning=f['tuning'],
                        ma_latent=f['ma_latent'] if 'ma_latent' in f else None)
    for k in ['p_transition_latent', 'p_transition_dynamics', 'p_joint_dynamics', 'p_joint_latent']:
        for fl in (1e-7, 1e-4, 1e-2):
            out[f'{name}:{k}:rel>{fl:g}'] = rel(r[k], f[k], fl)
    out[f'{name}:posterior_all:rel>1e-7'] = rel(r['posterior_all'], f['posterior_all'], 1e-7)
print(json.dumps(out, indent=1))
