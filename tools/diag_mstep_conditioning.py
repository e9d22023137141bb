"""Conditioning of the Adam M-step at the C3 shape (N=512, L=512, 79 basis columns) on
the C3 golden fixture's first M-step: the f64 oracle's tuning after its full Adam loop
(maxiter 1000, tol 1e-6) when y_w / t_w are perturbed by eps relative noise, next to
the fp32 reference-mimic's deviation.  Shows why tuning cannot be compared at 1e-5 after
a full Adam loop at this shape (tests/test_gpu_configs.py::test_c3_one_em_iteration_vs_oracle).
Run: python tools/diag_mstep_conditioning.py > profiles/r03_mstep_conditioning.txt"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gplvm_oracle as O  # noqa: E402
from tests.synth import make  # noqa: E402


def main():
    f = np.load(os.path.join(ROOT, 'tests', 'golden', 'c3_sample.npz'))
    d = make(int(f['N']), int(f['L']), int(f['T']))
    W0, B = d['W0'].astype(np.float64), d['B'].astype(np.float64)
    P = np.exp(d['lp0'].astype(np.float64))
    y = d['y'].astype(np.float64)
    yw, tw = P.T @ y, P.sum(0)

    def run(yw_, tw_):
        r = O.adam_run(W0.copy(), O.adam_init(W0), 1.0, B, yw_, tw_, lr=0.01, maxiter=1000, tol=1e-6)
        return r['n_iter'], O.get_tuning_softplus(r['params'], B)

    n0, t0 = run(yw, tw)
    print(f"C3 first M-step (N=512, L=512, NB=79): f64 oracle n_iter {n0}; golden tuning max rel "
          f"{np.max(np.abs(t0 / f['em_tuning'] - 1)):.2e}")
    print(f"fp32 reference-mimic tuning max rel vs f64: "
          f"{np.max(np.abs(f['mimic32_tuning'].astype(np.float64) / t0 - 1)):.3e}")
    rng = np.random.default_rng(1)
    for eps in (1e-15, 1e-13, 1e-11, 1e-9, 1e-7):
        n, t = run(yw * (1 + eps * rng.standard_normal(yw.shape)), tw * (1 + eps * rng.standard_normal(tw.shape)))
        print(f"y_w, t_w perturbed by {eps:.0e} relative: n_iter {n}, tuning max rel {np.max(np.abs(t / t0 - 1)):.2e}")


if __name__ == '__main__':
    main()
