"""Diagnostic: latent-only masked log marginal, forward-only vs full decode vs oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import poor_man_gplvm_amd as P
from poor_man_gplvm_amd.engine import ScanConfig
from oracle import gplvm_oracle as O
from tests.synth import make

N, L, T = 30, 100, 1500
d = make(N, L, T)
m = np.zeros(L); m[::3] = 1; m[np.random.default_rng(0).choice(L, 20, replace=False)] = 1
_, logK = O.create_transition_prob_latent_1d(L, 1.0)
ref = O.smooth_latent_only(d['y'], d['tuning'], logK, ma_latent=m)[1]
ref_nm = O.smooth_latent_only(d['y'], d['tuning'], logK)[1]
for name, sc in [("default", None), ("seq", ScanConfig(chunk=4096)), ("warm512", ScanConfig(warmup=512, adaptive=False))]:
    for cls in (P.PoissonGPLVM1D, P.PoissonGPLVMJump1D):
        mod = cls(N, n_latent_bin=L, tuning_lengthscale=10., scan_config=sc)
        a = mod.log_marginal_masked(d['y'], m[None], tuning=d['tuning'])[0]
        b = mod.decode_latent(d['y'], tuning=d['tuning'], ma_latent=m)['log_marginal_final']
        c = mod.decode_latent(d['y'], tuning=d['tuning'])['log_marginal_final']
        print(name, cls.__name__, "fwd-only", a, "decode", b, "unmasked", c, flush=True)
print("oracle latent-only masked", ref, "unmasked", ref_nm)
print("oracle jump masked", O.downsampled_lml(d['y'], d['tuning'], [m])[0][0])
