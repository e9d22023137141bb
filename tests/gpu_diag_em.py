"""Diagnostic (not collected): per-EM-iteration error budget of run_em vs the oracle on
the em_c1_fixed fixture inputs.  python tests/gpu_diag_em.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import gplvm_oracle as O  # noqa: E402


def rel(a, b, floor=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / (np.abs(b) + floor)


def main():
    import torch
    from poor_man_gplvm_amd import run_em, banded_transition, AdamConfig
    from poor_man_gplvm_amd.core import PoissonGPLVMJump1D
    f = np.load(os.path.join(HERE, 'golden', 'em_c1_fixed.npz'))
    y, B, W0, lp0 = f['y'].astype(np.float32), f['basis'], f['W0'], f['lp0']
    L = B.shape[0]
    for n_iter in (1, 2, 3):
        res, _ = run_em(y, W0, B, lp0, n_iter=n_iter, transition=banded_transition(L, float(f['mv'])),
                        adam=AdamConfig(maxiter=int(f['maxiter']), tol=float(f['tol'])))
        ref = O.fit_em(y.astype(np.float64), W0.astype(np.float64), B.astype(np.float64),
                       lp0.astype(np.float64), n_iter=n_iter, movement_variance=float(f['mv']),
                       m_step_maxiter=int(f['maxiter']), m_step_tol=float(f['tol']))
        rt = rel(res['tuning'], ref['tuning'])
        rw = np.abs(np.asarray(res['params'], np.float64) - ref['params'])
        pm, pr = res['posterior_latent_marg'], ref['posterior_latent_marg']
        rp = rel(pm, pr, 1e-12)
        big = pr > 1e-3
        print(f"n_iter={n_iter}: tuning rel max {rt.max():.2e} med {np.median(rt):.2e} | W abs max {rw.max():.2e}"
              f" | post rel max(P>1e-3) {rp[big].max():.2e} med {np.median(rp[big]):.2e} | "
              f"logZ rel {abs(res['log_marginal'] - ref['log_marginal']) / abs(ref['log_marginal']):.2e}")
        # E-step alone with the ORACLE's tuning (isolates E-step error)
        m = PoissonGPLVMJump1D(y.shape[1], n_latent_bin=L, movement_variance=float(f['mv']))
        dec = m.decode_latent(y, tuning=ref['tuning'])
        dref = O.decode_latent(y.astype(np.float64), ref['tuning'], movement_variance=float(f['mv']))
        pe = dec['posterior_latent_marg']
        pre = dref['posterior_latent_marg']
        rpe = rel(pe, pre, 1e-12)
        print(f"           E-step alone (oracle tuning): post rel max(P>1e-3) {rpe[pre > 1e-3].max():.2e} "
              f"abs max {np.abs(pe - pre).max():.2e}")
        # the same E-step in the oracle, with OUR tuning: how much does tuning error move it
        dref2 = O.decode_latent(y.astype(np.float64), np.asarray(res['tuning'], np.float64),
                                movement_variance=float(f['mv']))
        rpt = rel(dref2['posterior_latent_marg'], pre, 1e-12)
        print(f"           oracle E-step, our vs oracle tuning: post rel max(P>1e-3) {rpt[pre > 1e-3].max():.2e}")
    # M-step alone: Adam from the same exact (oracle) statistics
    yw, tw = O.get_statistics(lp0.astype(np.float64), y)
    r32 = O.m_step  # noqa


if __name__ == '__main__':
    main()
