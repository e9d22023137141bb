"""GPU parity of the model-selection path (reference model_selection_helper.py).

* log_marginal_masked (the inner loop of get_downsampled_lml, :243-260) vs the f64
  oracle's masked decode, mask by mask: log marginal rel 1e-7 (same bar as the
  decode goldens), and vs this package's own full decode_latent(ma_latent=m);
* get_downsampled_lml = mean / std of those;
* model_selection_one_split end to end on a tiny recording: result layout, best
  model / config consistent with the per-config table.
"""
import numpy as np
import pytest

from oracle import gplvm_oracle as O
from tests.synth import make

pytestmark = pytest.mark.gpu


def _smooth_data(N, L, T):
    """Spikes from a latent path without jumps (the latent-only model's own
    generative process, core.py:919-1019).  The device scan bands the continuous
    kernel at weights 1e-30 below its centre; a latent-only model decoding data
    with latent jumps wider than that band differs from the reference's dense
    log-domain kernel."""
    d = make(N, L, T)
    lat = O.sample_latent(T, L, np.random.default_rng(1), 1.0, 0.0, 1.0)
    d['y'] = O.sample_spikes(d['tuning'], lat[:, 1], np.random.default_rng(2)).astype(np.float32)
    return d


@pytest.mark.parametrize("model", ["jump", "latentonly"])
@pytest.mark.parametrize("N,L,T,frac", [(30, 100, 1500, 0.2), (24, 64, 700, 0.6), (40, 130, 2500, 0.8)])
def test_log_marginal_masked_vs_oracle(model, N, L, T, frac):
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import model_selection_helper as MS
    d = make(N, L, T) if model == "jump" else _smooth_data(N, L, T)
    cls = P.PoissonGPLVMJump1D if model == "jump" else P.PoissonGPLVM1D
    m = cls(N, n_latent_bin=L, tuning_lengthscale=10.)
    masks = MS.downsample_latent_masks(L, frac, 4, key=3)
    if model == "latentonly":
        # keep the kept bins within the continuous-kernel band of each other (the
        # device scan's limit for a model without a jump state; see the raise test)
        masks = np.zeros((4, L))
        for r in range(4):
            masks[r, ::3] = 1
            masks[r, np.random.default_rng(r).choice(L, int(L * frac), replace=False)] = 1
    got = m.log_marginal_masked(d['y'], masks, tuning=d['tuning'])
    if model == "jump":
        ref = O.downsampled_lml(d['y'], d['tuning'], masks)[0]
    else:
        _, logK = O.create_transition_prob_latent_1d(L, 1.0)
        ref = np.array([O.smooth_latent_only(d['y'], d['tuning'], logK, ma_latent=mk)[1] for mk in masks])
    np.testing.assert_allclose(got, ref, rtol=1e-7)
    full = [m.decode_latent(d['y'], tuning=d['tuning'], ma_latent=mk)['log_marginal_final'] for mk in masks]
    np.testing.assert_allclose(got, full, rtol=1e-9)
    if model == "jump":
        ds = MS.get_downsampled_lml(m, d['y'], downsample_frac=frac, n_repeat=4, key=3, tuning=d['tuning'])
        np.testing.assert_allclose(ds['value'], np.mean(ref), rtol=1e-7)
        np.testing.assert_allclose(ds['std'], np.std(ref), rtol=1e-4, atol=1e-6 * abs(np.mean(ref)))


def test_latent_only_mask_gap_wider_than_band():
    """Masks whose kept latent bins are further apart than any band: the latent-only
    model crosses the gap with its log-domain continuous kernel (decoder_latentonly.py),
    exactly as the reference."""
    import poor_man_gplvm_amd as P
    from oracle import gplvm_oracle as O
    d = make(10, 60, 100)
    m = P.PoissonGPLVM1D(10, n_latent_bin=60)
    ml = np.zeros(60)
    ml[[0, 5, 30, 31]] = 1                       # a gap of 25 bins
    _, logK = O.create_transition_prob_latent_1d(60, 1.0)
    lz = O.smooth_latent_only(d['y'], d['tuning'], logK, ma_latent=ml)[1]
    got = m.log_marginal_masked(d['y'], ml[None], tuning=d['tuning'])[0]
    assert abs(got - lz) <= 1e-7 * abs(lz)
    assert abs(m.decode_latent(d['y'], tuning=d['tuning'], ma_latent=ml)['log_marginal_final'] - lz) <= 1e-7 * abs(lz)


def test_log_marginal_masked_rejects_bad_masks():
    import poor_man_gplvm_amd as P
    d = make(10, 40, 100)
    m = P.PoissonGPLVMJump1D(10, n_latent_bin=40)
    with pytest.raises(ValueError):
        m.log_marginal_masked(d['y'], np.ones((2, 39)), tuning=d['tuning'])
    with pytest.raises(ValueError):
        m.log_marginal_masked(d['y'], np.zeros((1, 40)), tuning=d['tuning'])


def test_model_selection_one_split_end_to_end():
    from poor_man_gplvm_amd import model_selection_helper as MS
    d = make(20, 40, 1200)
    fit_kwargs = dict(MS.default_fit_kwargs, n_iter=3)
    res = MS.model_selection_one_split(d['y'], {'movement_variance': [1., 2.]}, key=0, fit_kwargs=fit_kwargs,
                                       n_repeat=2, latent_downsample_frac=[0.4, 0.8], downsample_n_repeat=3)
    tab = res['model_eval_result_all_configs']
    assert list(tab['movement_variance']) == [1., 2.]
    assert 'metric_overall_best_value' in tab and 'jump_consensus_best_value' in tab
    best_row = int(np.argmax(tab['metric_overall_best_value'].values))
    assert res['best_config'] == {'movement_variance': [1., 2.][best_row]}
    assert res['model_to_return_l'] == [res['best_model']]
    assert res['best_model'] in res['best_model_l'] and len(res['best_model_l']) == 2
    assert np.all(np.isfinite(tab['log_marginal_test_best_value'].values))
    # the recorded best test LML is the best model's own decode of the test split
    y_test = d['y'][int(1200 * 0.8):]
    lz = res['best_model_l'][int(tab['log_marginal_test_best_index'].values[best_row])].decode_latent(y_test)
    np.testing.assert_allclose(tab['log_marginal_test_best_value'].values[best_row], lz['log_marginal_final'],
                               rtol=1e-12)
