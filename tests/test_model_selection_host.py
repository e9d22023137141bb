"""Model-selection host logic (reference model_selection_helper.py) on CPU.

The metrics are checked against the oracle's loop restatements; the evaluation /
selection drivers run on stand-in models whose decodes are the f64 oracle, so the
driver logic (metric names, best index, metric_overall, return layout) is
exercised without a GPU.  The GPU path of the same drivers is in
tests/test_gpu_model_selection.py.
"""
import numpy as np
import pytest

from oracle import gplvm_oracle as O
from poor_man_gplvm_amd import model_selection_helper as MS
from tests.synth import make


def test_generate_hyperparam_grid_order():
    grid, df = MS.generate_hyperparam_grid({'movement_variance': [1., 2.], 'tuning_lengthscale': [3., 5., 7.]})
    assert len(grid) == 6 and list(df.columns) == ['movement_variance', 'tuning_lengthscale']
    assert grid[0] == {'movement_variance': 1., 'tuning_lengthscale': 3.}
    assert grid[1] == {'movement_variance': 1., 'tuning_lengthscale': 5.}
    assert grid[5] == {'movement_variance': 2., 'tuning_lengthscale': 7.}
    assert df.iloc[4].to_dict() == grid[4]


@pytest.mark.parametrize("seed,window,pth,cth", [(0, 5, 0.4, 0.8), (1, 2, 0.3, 0.5), (2, 0, 0.4, 0.8),
                                                  (3, 20, 0.6, 1.0)])
def test_jump_consensus_vs_oracle(seed, window, pth, cth):
    rng = np.random.default_rng(seed)
    T, C = 300, 6
    chains = (rng.random((T, C)) ** 6)          # mostly small, some jumps
    chains[:8] = rng.random((8, C))             # jumps near t=0 exercise the negative slice start
    for c in range(C):
        jp = chains[:, c]
        a = MS.get_jump_consensus(jp, chains, window_size=window, jump_p_thresh=pth, consensus_thresh=cth)
        b = O.jump_consensus(jp, chains, window_size=window, jump_p_thresh=pth, consensus_thresh=cth)
        np.testing.assert_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[2], b[2])


def test_jump_consensus_no_jumps_is_nan():
    chains = np.zeros((50, 3))
    frac, filt, ok = MS.get_jump_consensus(chains[:, 0], chains)
    assert np.isnan(frac) and not filt.any() and ok.size == 0


@pytest.mark.parametrize("L,frac,R", [(100, 0.2, 10), (37, 0.6, 3), (512, 0.8, 4)])
def test_downsample_masks(L, frac, R):
    m = MS.downsample_latent_masks(L, frac, R, key=4)
    assert m.shape == (R, L)
    assert np.all(m.sum(1) == int(L * frac))
    assert set(np.unique(m)) <= {0., 1.}
    assert not np.array_equal(m[0], m[1]) or R == 1
    np.testing.assert_array_equal(m, MS.downsample_latent_masks(L, frac, R, key=4))


class _OracleModel:
    """Stand-in exposing the two methods the evaluation driver calls."""

    def __init__(self, tuning, mv):
        self.tuning, self.mv, self.n_latent_bin = tuning, mv, tuning.shape[0]

    def decode_latent(self, y, n_time_per_chunk=10000, **kw):
        return O.decode_latent(y, self.tuning, movement_variance=self.mv)

    def log_marginal_masked(self, y, masks, **kw):
        return O.downsampled_lml(y, self.tuning, masks, movement_variance=self.mv)[0]


def _eval_case(MS):
    """3 stand-in fits on a small recording (shared with the gloo sharding test)."""
    d = make(12, 30, 200)
    rng = np.random.default_rng(5)
    models = [_OracleModel(d['tuning'], 1.0),
              _OracleModel(d['tuning'] * np.exp(0.3 * rng.normal(size=d['tuning'].shape)), 1.0),
              _OracleModel(d['tuning'], 3.0)]
    return MS.evaluate_model_one_config(models, d['y'], key=1, latent_downsample_frac=[0.4, 0.8],
                                        downsample_n_repeat=3, jump_consensus_window_size=[3, 5])


def test_evaluate_model_one_config_with_oracle_models():
    d = make(12, 30, 200)
    rng = np.random.default_rng(5)
    models = [_OracleModel(d['tuning'], 1.0),
              _OracleModel(d['tuning'] * np.exp(0.3 * rng.normal(size=d['tuning'].shape)), 1.0),
              _OracleModel(d['tuning'], 3.0)]
    ev = MS.evaluate_model_one_config(models, d['y'], key=1, latent_downsample_frac=[0.4, 0.8],
                                      downsample_n_repeat=3, jump_consensus_window_size=[3, 5])
    assert list(ev) == ['log_marginal_test', 'log_one_step_predictive_marginal_test', 'downsampled_lml_0.4',
                        'downsampled_lml_0.8', 'jump_consensus_3', 'jump_consensus_5', 'metric_overall']
    lz = [O.decode_latent(d['y'], m.tuning, movement_variance=m.mv)['log_marginal_final'] for m in models]
    np.testing.assert_allclose(ev['log_marginal_test']['value_per_fit'], lz)
    masks = MS.downsample_latent_masks(30, 0.4, 3, key=1)
    ds = [O.downsampled_lml(d['y'], m.tuning, masks, movement_variance=m.mv)[1] for m in models]
    np.testing.assert_allclose(ev['downsampled_lml_0.4']['value_per_fit'], ds)
    overall = (ev['downsampled_lml_0.4']['value_per_fit'] + ev['downsampled_lml_0.8']['value_per_fit']) / 2
    np.testing.assert_allclose(ev['metric_overall']['value_per_fit'], overall)
    for v in ev.values():
        # nan (a chain without jumps) propagates through max / argmax as in the reference
        np.testing.assert_equal(v['best_index'], np.argmax(v['value_per_fit']))
        np.testing.assert_equal(v['best_value'], np.max(v['value_per_fit']))
    # the one-step predictive marginals sum to logZ (decoder.py:174-187)
    np.testing.assert_allclose(ev['log_one_step_predictive_marginal_test']['value_per_fit'], lz, rtol=1e-9)


def test_model_class_dict_matches_reference_names():
    """model_selection_helper.py:14: the four model_class_str values."""
    assert set(MS.model_class_dict) == {'poisson', 'gaussian', 'poisson_latentonly', 'gaussian_latentonly'}
    import poor_man_gplvm_amd as P
    assert MS.model_class_dict['gaussian_latentonly'] is P.GaussianGPLVM1D
    assert issubclass(P.GaussianGPLVM1D, P.PoissonGPLVM1D)      # latent-only engine


def test_restarts_batchable_rules():
    """core._restarts_batchable: which model lists fit_em_restarts runs as one batch."""
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd.core import _restarts_batchable
    mk = lambda cls=P.PoissonGPLVMJump1D, **kw: cls(12, **dict(dict(n_latent_bin=64, tuning_lengthscale=10.), **kw))
    assert _restarts_batchable([mk(), mk(), mk()], {})
    assert not _restarts_batchable([mk(n_latent_bin=100), mk(n_latent_bin=100)], {})      # L % 32
    assert not _restarts_batchable([mk(), mk(movement_variance=2.0)], {})                  # configs differ
    assert not _restarts_batchable([mk(), mk(rng_init_int=5)], {})                         # initial W differs
    assert not _restarts_batchable([mk(P.GaussianGPLVMJump1D), mk(P.GaussianGPLVMJump1D)], {})
    assert not _restarts_batchable([mk(), mk()], {'movement_variance': 9.0})               # dense transition
