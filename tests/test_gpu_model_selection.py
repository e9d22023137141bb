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
    generative process, core.py:919-1019)."""
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
    # random downsampling leaves gaps of many bins between kept latents: the latent-only
    # model crosses them on the dense log-domain scans with the exact far-move weights
    masks = MS.downsample_latent_masks(L, frac, 4, key=3)
    got = m.log_marginal_masked(d['y'], masks, tuning=d['tuning'])
    if model == "jump":
        ref = O.downsampled_lml(d['y'], d['tuning'], masks)[0]
    else:
        _, logK = O.create_transition_prob_latent_1d(L, 1.0)
        ref = np.array([O.smooth_latent_only(d['y'], d['tuning'], logK, ma_latent=mk)[1] for mk in masks])
    np.testing.assert_allclose(got, ref, rtol=1e-7)
    # the batched path (one emission, per-mask pmg_emission_latent_mask, banded forward on
    # (delta, rblk)) vs one full masked decode per mask (the exact decode: dense scans on
    # the f64 ll): the same up to delta's f32 rounding (measured 3.3e-9 relative)
    full = [m.decode_latent(d['y'], tuning=d['tuning'], ma_latent=mk)['log_marginal_final'] for mk in masks]
    np.testing.assert_allclose(got, full, rtol=2e-8)
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
    # the recorded best test LML is the best model's own decode of the test split: bit for
    # bit the evaluation's decode_marginals (banded scans, no joint), and decode_latent's
    # (dense exact scans) within the scans' logZ bar
    y_test = d['y'][int(1200 * 0.8):]
    best = res['best_model_l'][int(tab['log_marginal_test_best_index'].values[best_row])]
    rec = tab['log_marginal_test_best_value'].values[best_row]
    assert rec == best.decode_marginals(y_test)['log_marginal_final']
    np.testing.assert_allclose(rec, best.decode_latent(y_test)['log_marginal_final'], rtol=1e-7)


@pytest.mark.parametrize("path", ["int8", "f64", "gaussian", "dt"])
def test_latent_mask_apply_matches_masked_emission(path):
    """pmg_emission_latent_mask on the unmasked emission == the emission run with the
    mask: masked bins -1e20, kept bins' ll to 2 f32 ulps of delta, unmasked blocks
    bit-identical; includes fully masked 32-bin blocks and a ragged last block."""
    import torch
    from poor_man_gplvm_amd import _native as nat
    from poor_man_gplvm_amd.engine import DeviceEM, SpikeData
    N, L, T = 37, 150, 900
    d = make(N, L, T)
    rng = np.random.default_rng(2)
    y = d['y'] if path != "gaussian" else (d['y'] + rng.normal(size=d['y'].shape)).astype(np.float32)
    ma = (rng.random(N) > 0.2).astype(np.float32) * (1.7 if path == "f64" else 1.0)
    ml = (rng.random(L) > 0.4).astype(np.uint8)
    ml[32:64] = 0                 # a fully masked block
    ml[96:128] = 1                # a block without masked bins
    ml[149] = 0                   # ragged last block (150 = 4 * 32 + 22)
    eng = DeviceEM(SpikeData(y, ma), L)
    if path == "gaussian":
        eng.noise_std = 0.5
    eng.set_tuning(d['tuning'])
    sh = nat.stream_handle()

    def emit(mask):
        eng.set_ma_latent(mask)
        if path == "dt":
            dtt = torch.as_tensor(rng.uniform(0.5, 1.5, T), device='cuda')
            nat.check(eng.lib.pmg_emission_poisson_dt(nat.ptr(eng.sp.y), nat.ptr(eng.sp.gconst),
                                                      nat.ptr(eng.tuning64), nat.ptr(eng.sp.ma), 0,
                                                      nat.ptr(eng.ma_latent), nat.ptr(dtt), T, L, N,
                                                      nat.ptr(eng.delta), nat.ptr(eng.rblk), sh), "dt")
        else:
            eng._emission_call(eng.sp, sh, 1.0)
        return eng.delta.clone(), eng.rblk.clone()

    rng_state = rng.bit_generator.state
    d0, r0 = emit(None)
    rng.bit_generator.state = rng_state      # the same per-bin dt for both calls
    dm, rm = emit(ml)
    mu8 = torch.as_tensor(ml, device='cuda')
    da, ra = torch.empty_like(d0), torch.empty_like(r0)
    nat.check(eng.lib.pmg_emission_latent_mask(nat.ptr(d0), nat.ptr(r0), T, L, nat.ptr(mu8), nat.ptr(da),
                                               nat.ptr(ra), sh), "pmg_emission_latent_mask")
    d0, dm, rm, da, ra = (x.cpu().numpy() for x in (d0, dm, rm, da, ra))
    blk = np.arange(L) // 32
    llm = dm.astype(np.float64) + rm[:, blk]
    lla = da.astype(np.float64) + ra[:, blk]
    keep = ml.astype(bool)
    assert np.all(lla[:, ~keep] <= -1e19) and np.all(llm[:, ~keep] <= -1e19)
    # kept bins: d0's own rounding (its block max may have been a masked bin) + delta's;
    # the f64 / Gaussian / per-bin-dt emissions keep an exact f64 block max, the mask
    # pass an f32-rounded one (as the int8 emission): a residual of ~2^-24 ulp_f32(ll)
    ulp = np.spacing(np.maximum(np.abs(d0[:, keep]), np.abs(dm[:, keep])).astype(np.float32)).astype(np.float64)
    err = np.abs(lla[:, keep] - llm[:, keep])
    assert np.all(err <= 1.5 * ulp + 1e-13 * np.abs(llm[:, keep])), (err / (ulp + 1e-300)).max()
    clean = np.array([ml[b * 32:(b + 1) * 32].all() for b in range(rm.shape[1])])
    np.testing.assert_array_equal(ra[:, clean], rm[:, clean])
    np.testing.assert_array_equal(da[:, np.repeat(clean, 32)[:L]], dm[:, np.repeat(clean, 32)[:L]])


@pytest.mark.parametrize("R,chunk", [(5, 40), (3, None)])
def test_masked_logz_batched_bit_identical(R, chunk):
    """DeviceEM.masked_logz_batched (R masks: one stacked mask launch, one row-reference
    launch, one forward launch, no alpha) == R single-mask forward filters on the same
    chunk grid and relaxation segments (pinned: ScanConfig(chunk=C, relax_segments=#CUs /
    MASK_BATCH_MAX)), bit for bit; a mask's logZ does not depend on how many masks share
    its batch (the first two masks alone give the same bits); and == the f64 oracle's
    masked log marginals at rel 1e-7."""
    import math
    import torch
    from poor_man_gplvm_amd import model_selection_helper as MS
    from poor_man_gplvm_amd.engine import DeviceEM, ScanConfig, SpikeData
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    N, L, T = 40, 128, 3000
    d = make(N, L, T)
    masks = MS.downsample_latent_masks(L, 0.3, R, key=5)
    C = chunk or max(32, int(math.ceil(DeviceEM.MASK_BATCH_MAX * T / 2048)))
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    tr = banded_transition(L, 1.0, 0.01, 0.01)

    def engine(sc):
        eng = DeviceEM(SpikeData(d['y']), L, scan=sc)
        eng.set_transition(tr)
        eng.set_tuning(d['tuning'])
        return eng
    eng = engine(ScanConfig(chunk=chunk))
    delta0, rblk0 = eng.emission_unmasked()
    mu8 = torch.as_tensor(np.asarray(masks, np.uint8), device='cuda')
    lz = torch.zeros(R, dtype=torch.float64, device='cuda')
    eng.masked_logz_batched(delta0, rblk0, mu8, 1.0, lz)
    got = lz.cpu().numpy()
    assert eng.masked_segments() == max(1, cus // DeviceEM.MASK_BATCH_MAX)
    lz2 = torch.zeros(2, dtype=torch.float64, device='cuda')
    eng.masked_logz_batched(delta0, rblk0, mu8[:2].contiguous(), 1.0, lz2)
    np.testing.assert_array_equal(lz2.cpu().numpy(), got[:2])
    one = engine(ScanConfig(chunk=C, relax_segments=max(1, cus // DeviceEM.MASK_BATCH_MAX)))
    d1, r1 = one.emission_unmasked()
    seq = np.empty(R)
    for r in range(R):
        z = torch.zeros(1, dtype=torch.float64, device='cuda')
        one.emission_from(d1, r1, mu8[r], 1.0)
        one.forward(1.0, z)
        seq[r] = z.item()
    one.check_status()
    np.testing.assert_array_equal(got, seq)
    ref = O.downsampled_lml(d['y'], d['tuning'], masks)[0]
    np.testing.assert_allclose(got, ref, rtol=1e-7)


def test_decode_marginals_match_decode_latent():
    """decode_marginals (banded scans, no pairwise joint: what evaluate_model_one_config
    reads) against decode_latent (dense exact scans + joint) and the f64 oracle: log
    marginal rel 1e-7, one-step marginals rel 1e-5 (atol 1e-5), dynamics marginal at the
    posterior bar (rel 1e-5, atol 1e-12)."""
    import poor_man_gplvm_amd as P
    from tests.test_gpu_parity import close_prob
    N, L, T = 40, 128, 2000
    d = make(N, L, T)
    m = P.PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.)
    a = m.decode_marginals(d['y'], tuning=d['tuning'])
    b = m.decode_latent(d['y'], tuning=d['tuning'])
    ref = O.decode_latent(d['y'], d['tuning'])
    for r in (a, b):
        np.testing.assert_allclose(r['log_marginal_final'], ref['log_marginal_final'], rtol=1e-7)
        np.testing.assert_allclose(r['log_one_step_predictive_marginals_all'],
                                   ref['log_one_step_predictive_marginals_all'], rtol=1e-5, atol=1e-5)
        close_prob(r['posterior_dynamics_marg'], ref['posterior_dynamics_marg'])
