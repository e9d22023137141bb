"""Diagnostic (not collected): where does the dense log-domain scan lose precision?
Latent-only decode vs the f64 oracle, one chunk (pure chain arithmetic) vs the default
chunking (boundaries + relaxation)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import poor_man_gplvm_amd as P  # noqa: E402
from oracle import gplvm_oracle as O  # noqa: E402
from tests.synth import make  # noqa: E402

N, L, T = 30, 100, 900
d = make(N, L, T)
_, logK = O.create_transition_prob_latent_1d(L, 1.0)
lpa, lz, lca, cs, lj, ll = O.smooth_latent_only(d['y'], d['tuning'], logK)
ref = np.exp(lpa)
refc = np.exp(lca)
for name, sc in [("one chunk", P.ScanConfig(chunk=T)), ("default", None), ("tol1e-7", P.ScanConfig(tol=1e-7))]:
    m = P.PoissonGPLVM1D(N, n_latent_bin=L, tuning_lengthscale=10., scan_config=sc)
    la, lzz, lc, c2, jj, l2 = m._decode_latent(d['y'], d['tuning'], {}, logK, np.ones(N))
    post, caus = np.exp(la), np.exp(lc)
    for what, a, b in (("posterior", post, ref), ("causal", caus, refc)):
        err = np.abs(a - b) / (np.abs(b) + 1e-12)
        bad = err > 1e-5
        tt, jj2 = np.nonzero(bad)
        print(f"{name:9s} {what:9s}: logZ err {lzz - lz:+.3e}  max rel {err.max():.2e} n>1e-5 {bad.sum()} "
              f"(values of bad: median {np.median(b[bad]) if bad.any() else 0:.2e}); bad t range "
              f"{(tt.min(), tt.max()) if bad.any() else ()}; max abs {np.abs(a - b).max():.2e}", flush=True)
    print("  rel err quantiles (b>1e-3):", np.quantile((np.abs(post - ref) / ref)[ref > 1e-3], [0.5, 0.9, 0.99, 1.0]))
