"""Generate the committed golden fixtures (run from the repo root:
`python tests/golden/make_golden.py`).

The reference (JAX) cannot run in this image, so the fixtures are outputs of the
float64 oracle (oracle/gplvm_oracle.py, itself pinned by brute-force enumeration in
tests/test_oracle_brute.py) on explicit, seeded inputs -- they freeze the oracle's
behaviour and let the GPU tests check parity without re-running the slow oracle.
`reference_api.json` records API facts read from the reference's own files
(dict keys from core.py:484-495 / :696-712 and the key order printed in
ripple-type-GPLVM-tunings.ipynb cell 25)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import gplvm_oracle as O  # noqa: E402
from tests.synth import make  # noqa: E402


def em_case(name, N, L, T, n_iter, maxiter, tol, ls=10.0, mv=1.0, seed=0):
    d = make(N, L, T, ls=ls, mv=mv, seed=seed)
    r = O.fit_em(d['y'], d['W0'].astype(np.float64), d['B'].astype(np.float64), d['lp0'].astype(np.float64),
                 n_iter=n_iter, movement_variance=mv, m_step_maxiter=maxiter, m_step_tol=tol)
    # the same fit in the reference's own arithmetic (float32 reference-mimic): its
    # distance to the float64 answer is the reference's rounding noise floor
    with O.working_precision(np.float32):
        r32 = O.fit_em(d['y'], d['W0'], d['B'], d['lp0'], n_iter=n_iter, movement_variance=mv,
                       m_step_maxiter=maxiter, m_step_tol=tol)
    m = r['m_step_res_l']
    np.savez_compressed(os.path.join(HERE, name),
                        y=d['y'].astype(np.int16), basis=d['B'], W0=d['W0'], lp0=d['lp0'],
                        mv=mv, n_iter=n_iter, maxiter=maxiter, tol=tol,
                        params=r['params'].astype(np.float32), tuning=r['tuning'].astype(np.float32),
                        posterior=r['posterior'].astype(np.float32),
                        log_marginal_l=np.array(r['log_marginal_l']),
                        m_n_iter=np.array(m['n_iter']), m_final_loss=np.array(m['final_loss']),
                        m_final_error=np.array(m['final_error']),
                        m_loss_history_0=m['loss_history'][0],
                        mimic32_tuning=r32['tuning'].astype(np.float32),
                        mimic32_posterior_latent=r32['posterior_latent_marg'].astype(np.float32))


def decode_case(name, N, L, T, mv=1.0, seed=5, ma_latent=None):
    d = make(N, L, T, mv=mv, seed=seed)
    tun = d['tuning']
    r = O.decode_latent(d['y'], tun, movement_variance=mv, ma_latent=ma_latent)
    out = dict(y=d['y'].astype(np.int16), tuning=tun.astype(np.float64), mv=mv,
               log_marginal_final=r['log_marginal_final'],
               posterior_all=r['posterior_all'].astype(np.float32),
               log_one_step=r['log_one_step_predictive_marginals_all'],
               log_likelihood_all=r['log_likelihood_all'].astype(np.float32),
               p_transition_latent=r['p_transition_latent'], p_transition_dynamics=r['p_transition_dynamics'],
               p_joint_dynamics=r['p_joint_dynamics'], p_joint_latent=r['p_joint_latent'])
    if ma_latent is not None:
        out['ma_latent'] = np.asarray(ma_latent)
    np.savez_compressed(os.path.join(HERE, name), **out)


def main():
    em_case('em_c1_fixed.npz', N=30, L=100, T=400, n_iter=3, maxiter=40, tol=0.0)
    em_case('em_c1_one.npz', N=30, L=100, T=400, n_iter=1, maxiter=40, tol=0.0)
    em_case('em_small_stoprule.npz', N=20, L=64, T=300, n_iter=3, maxiter=1000, tol=1e-6)
    decode_case('decode_small.npz', N=24, L=48, T=200)
    ml = np.ones(48)
    ml[np.random.default_rng(9).choice(48, 20, replace=False)] = 0
    decode_case('decode_masked.npz', N=24, L=48, T=200, ma_latent=ml)
    api = {
        "fit_em_keys": ['log_posterior_all_saved', 'log_posterior_init', 'params_saved', 'tuning_saved',
                        'iter_saved', 'params', 'tuning', 'log_posterior_final', 'log_marginal',
                        'log_marginal_l', 'log_marginal_saved', 'posterior', 'posterior_latent_marg',
                        'posterior_dynamics_marg', 'm_step_res_l'],
        "m_step_res_keys": ['params', 'opt_state', 'n_iter', 'final_loss', 'final_error', 'loss_history',
                            'error_history'],
        "decode_keys_recorded": ['log_posterior_all', 'log_marginal_final', 'posterior_all',
                                 'posterior_latent_marg', 'posterior_dynamics_marg',
                                 'log_one_step_predictive_marginals_all', 'log_likelihood_all',
                                 'log_joint_dynamics', 'log_joint_full', 'log_joint_latent',
                                 'log_transition_dynamics', 'log_transition_full', 'log_transition_latent',
                                 'p_joint_dynamics', 'p_joint_full', 'p_joint_latent', 'p_transition_dynamics',
                                 'p_transition_full', 'p_transition_latent'],
        "sources": {"fit_em_keys": "core.py:696-712", "m_step_res_keys": "core.py:820-826",
                    "decode_keys_recorded": "ripple-type-GPLVM-tunings.ipynb cell 25 output"},
        "n_basis_ls10": {"100": None, "256": None, "512": None},
    }
    for L in (100, 256, 512):
        api["n_basis_ls10"][str(L)] = int(O.generate_basis(10.0, L).shape[1])
    with open(os.path.join(HERE, 'reference_api.json'), 'w') as f:
        json.dump(api, f, indent=1)
    for fn in sorted(os.listdir(HERE)):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == '__main__':
    main()
