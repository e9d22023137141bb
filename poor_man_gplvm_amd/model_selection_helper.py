"""Model selection (reference model_selection_helper.py): hyper-parameter grid,
independent EM restarts sharded over ranks, test-set evaluation and the
downsampled-LML / jump-consensus metrics.

`fit_model_one_config` keeps the reference's signature and return value
(lists of fitted models and fit_em dicts, in key order).  When torch.distributed
is initialised, restart k runs on rank k % world_size -- restarts are fully
independent, so there is no data-path collective -- and the per-rank results are
gathered with all_gather_object at the end so every rank returns the full lists.

`get_downsampled_lml` runs its n_repeat masked decodes through
`model.log_marginal_masked` (spikes uploaded once, emission + forward filter per
mask; the metric reads only log_marginal_final).  Latent masks are drawn with
numpy (PCG64 seeded from `key`) instead of jax threefry, so the chosen bins differ
from the reference's for the same key; the statistic is the same.
"""
from __future__ import annotations

import itertools

import numpy as np

from .core import GaussianGPLVM1D, GaussianGPLVMJump1D, PoissonGPLVM1D, PoissonGPLVMJump1D, fit_em_restarts

model_class_dict = {'poisson': PoissonGPLVMJump1D, 'gaussian': GaussianGPLVMJump1D,
                    'poisson_latentonly': PoissonGPLVM1D, 'gaussian_latentonly': GaussianGPLVM1D}

default_fit_kwargs = {'n_iter': 20, 'log_posterior_init': None, 'n_time_per_chunk': 10000, 'dt': 1.,
                      'likelihood_scale': 1., 'save_every': None,
                      'posterior_init_kwargs': {'random_scale': 0.1}}


def generate_hyperparam_grid(hyperparam_ranges):
    """model_selection_helper.py:17-33: dict of lists -> (list of dicts of every
    combination in itertools.product order, the same grid as a DataFrame)."""
    import pandas as pd
    keys = list(hyperparam_ranges.keys())
    grid = [dict(zip(keys, combo)) for combo in itertools.product(*[hyperparam_ranges[k] for k in keys])]
    return grid, pd.DataFrame(grid)


def split_keys(key, n):
    """Stand-in for jr.split(key, n): n independent integer seeds."""
    ss = np.random.SeedSequence(int(key) if np.isscalar(key) else abs(hash(np.asarray(key).tobytes())))
    return [int(c.generate_state(1)[0]) for c in ss.spawn(n)]


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except Exception:
        pass
    return None


_LOCAL_DEPTH = [0]     # > 0: inside a loop that is already sharded over ranks


class _local_only:
    """Inside an outer rank-sharded loop (e.g. evaluate_model_one_config's fits) the
    inner loops run locally: ranks process different items, so no collective of theirs
    may pair up."""

    def __enter__(self):
        _LOCAL_DEPTH[0] += 1

    def __exit__(self, *exc):
        _LOCAL_DEPTH[0] -= 1
        return False


def shard_map(n, fn):
    """Items 0..n-1 spread over the torch.distributed ranks (item k on rank k % world):
    fn(list of this rank's item indices) -> list of their results, in that order; the
    results of every rank are gathered (all_gather_object) and returned in item order
    on every rank.  Without an initialised process group: fn(range(n)).  The shard axis
    of the embarrassingly parallel loops of model selection and the shuffle tests
    (get_downsampled_lml's masks, shuffle_and_decode's shuffles)."""
    dist = _dist() if _LOCAL_DEPTH[0] == 0 else None
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    idx = list(range(rank, n, world))
    mine = list(zip(idx, fn(idx) if idx else []))
    if dist and world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        mine = [item for part in gathered for item in part]
    mine.sort(key=lambda r: r[0])
    return [r for _, r in mine]


def fit_model_one_config(config, y_train, key=0, fit_kwargs=default_fit_kwargs, model_class_str='poisson',
                         n_repeat=1, fit_fn=None):
    """model_selection_helper.py:35-60.  `fit_fn(model, y, key, fit_kwargs) -> em_res`
    replaces model.fit_em (used by the CPU gloo tests to exercise the sharding)."""
    if model_class_str not in model_class_dict:
        raise ValueError(f"Invalid model class: {model_class_str}")
    model_class = model_class_dict[model_class_str]
    key_l = list(key) if isinstance(key, list) else split_keys(key, n_repeat)
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    mine = []
    idx = list(range(rank, len(key_l), world))
    if fit_fn is None and len(idx) > 1:
        # this rank's restarts as ONE batched fit (core.fit_em_restarts: stacked-latent
        # emission / suff-stats GEMMs, one scan launch per pass for all of them; it runs
        # them one by one where the model cannot be batched)
        models = [model_class(n_neuron=np.asarray(y_train).shape[1], **config) for _ in idx]
        ems = fit_em_restarts(models, y_train, [key_l[k] for k in idx], hyperparam={}, **fit_kwargs)
        mine = list(zip(idx, models, ems))
    else:
        for k_idx in idx:
            model_fit = model_class(n_neuron=np.asarray(y_train).shape[1], **config)
            if fit_fn is None:
                em_res = model_fit.fit_em(y_train, hyperparam={}, key=key_l[k_idx], **fit_kwargs)
            else:
                em_res = fit_fn(model_fit, y_train, key_l[k_idx], fit_kwargs)
            mine.append((k_idx, model_fit, em_res))
    if dist and world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        mine = [item for part in gathered for item in part]
    mine.sort(key=lambda r: r[0])
    return [m for _, m, _ in mine], [e for _, _, e in mine]


def _seed_of(key):
    return int(key) if np.isscalar(key) else abs(hash(np.asarray(key).tobytes())) % (2 ** 63)


def downsample_latent_masks(n_latent_bin, downsample_frac, n_repeat, key):
    """The masks of get_downsampled_lml (model_selection_helper.py:249-256): n_repeat
    rows, each with int(n_latent_bin * downsample_frac) ones at distinct positions."""
    n_sel = int(n_latent_bin * downsample_frac)
    masks = np.zeros((n_repeat, n_latent_bin))
    for r, k in enumerate(split_keys(_seed_of(key), n_repeat)):
        masks[r, np.random.default_rng(k).choice(n_latent_bin, size=n_sel, replace=False)] = 1
    return masks


def get_downsampled_lml(model_fit, y_test, downsample_frac=0.2, n_repeat=10, key=4, **kwargs):
    """model_selection_helper.py:243-260: mean and std of log_marginal_final over
    n_repeat decodes, each restricted to a random subset of latent bins.
    kwargs are decode_latent's (tuning, hyperparam, ma_neuron, likelihood_scale)."""
    masks = downsample_latent_masks(model_fit.n_latent_bin, downsample_frac, n_repeat, key)
    kw = {k: v for k, v in kwargs.items() if k in ('tuning', 'hyperparam', 'ma_neuron', 'likelihood_scale')}
    # masks sharded over ranks when a process group is up (each rank: one batched pass)
    lml_l = np.asarray(shard_map(len(masks), lambda idx: list(model_fit.log_marginal_masked(y_test, masks[idx], **kw))),
                       np.float64)
    return {'value': np.mean(lml_l), 'std': np.std(lml_l)}


def get_jump_consensus(jump_p, jump_p_all_chain, window_size=5, jump_p_thresh=0.4, consensus_thresh=0.8):
    """model_selection_helper.py:264-299.  jump_p (T,), jump_p_all_chain (T, n_chain).
    For every t with jump_p[t] >= jump_p_thresh: the fraction of chains with some
    p > jump_p_thresh in rows [t - window_size, t + window_size) -- numpy slice
    semantics, so a negative start wraps as in the reference -- must reach
    consensus_thresh.  Returns (frac_consensus, is_jump_filtered (T,),
    whether_consensus_ma (n_jumps,)); frac_consensus is nan when there is no jump."""
    jump_p = np.asarray(jump_p)
    jump_p_all_chain = np.asarray(jump_p_all_chain)
    jti_l = np.nonzero(jump_p >= jump_p_thresh)[0]
    above = jump_p_all_chain > jump_p_thresh
    ok = np.array([above[j - window_size:j + window_size, :].any(axis=0).mean() >= consensus_thresh
                   for j in jti_l], dtype=bool)
    with np.errstate(invalid='ignore', divide='ignore'):
        frac = ok.mean() if len(ok) else np.float64(np.nan)
    is_jump_filtered = np.zeros(len(jump_p))
    is_jump_filtered[jti_l[ok]] = 1
    return frac, is_jump_filtered, ok


def _jump_consensus_values(jump_p_l, window_size, p_thresh, c_thresh):
    chains = np.array(jump_p_l).T  # (T, n_chain)
    return np.array([get_jump_consensus(jp, chains, window_size=window_size, jump_p_thresh=p_thresh,
                                        consensus_thresh=c_thresh)[0] for jp in chains.T])


def evaluate_model_one_config(model_fit_l, y_test, key=1, n_time_per_chunk=10000,
                              latent_downsample_frac=[0.2, 0.4, 0.6, 0.8], downsample_n_repeat=10,
                              metric_type_l=['log_marginal_test', 'log_one_step_predictive_marginal_test',
                                             'downsampled_lml', 'jump_consensus'],
                              jump_dynamics_index=1, jump_consensus_window_size=5,
                              jump_consensus_jump_p_thresh=0.4, jump_consensus_consensus_thresh=0.8):
    """model_selection_helper.py:62-147: per-fit metrics on the test data, each a dict
    {'value_per_fit', 'best_value', 'best_index'}; 'metric_overall' is the mean of
    the downsampled LMLs over latent_downsample_frac (so 'downsampled_lml' must be
    requested, as in the reference).

    Under torch.distributed the fits are sharded like the restarts: rank r decodes and
    scores fits k with k % world_size == r (one decode + the downsampled-LML masks per
    fit, all independent), then one all_gather_object of the per-fit scalars and jump
    probabilities; every rank assembles the same result."""
    want_ds = 'downsampled_lml' in metric_type_l
    want_jump = 'jump_consensus' in metric_type_l
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    mine = {}
    for k in range(rank, len(model_fit_l), world):
        with _local_only():          # the fits are the shard axis here
            m = model_fit_l[k]
            # only the log marginals and the dynamics marginal are read: no pairwise joint
            # (jump models; the latent-only models decode through decode_latent)
            dm = None if isinstance(m, PoissonGPLVM1D) else getattr(m, 'decode_marginals', None)
            dec = dm(y_test) if dm is not None else m.decode_latent(y_test, n_time_per_chunk=n_time_per_chunk)
            v = {'lml': dec['log_marginal_final'],
                 'os': np.asarray(dec['log_one_step_predictive_marginals_all']).sum()}
            if want_ds:
                v['ds'] = [get_downsampled_lml(m, y_test, downsample_frac=f, n_repeat=downsample_n_repeat, key=key)['value']
                           for f in latent_downsample_frac]
            if want_jump:
                v['jp'] = np.asarray(dec['posterior_dynamics_marg'])[:, jump_dynamics_index]
            mine[k] = v
    if dist and world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        mine = {k: v for part in parts for k, v in part.items()}
    per = [mine[k] for k in range(len(model_fit_l))]

    res = {}

    def put(name, vals):
        res[name] = {'value_per_fit': np.array(vals), 'best_value': None, 'best_index': None}

    if 'log_marginal_test' in metric_type_l:
        put('log_marginal_test', [v['lml'] for v in per])
    if 'log_one_step_predictive_marginal_test' in metric_type_l:
        put('log_one_step_predictive_marginal_test', [v['os'] for v in per])
    if want_ds:
        for i, frac in enumerate(latent_downsample_frac):
            put('downsampled_lml_' + str(frac), [v['ds'][i] for v in per])
    if want_jump:
        jp_l = [v['jp'] for v in per]
        thr = (jump_consensus_jump_p_thresh, jump_consensus_consensus_thresh)
        if isinstance(jump_consensus_window_size, int):
            put('jump_consensus', _jump_consensus_values(jp_l, jump_consensus_window_size, *thr))
        elif isinstance(jump_consensus_window_size, list):
            for w in jump_consensus_window_size:
                put('jump_consensus_' + str(w), _jump_consensus_values(jp_l, w, *thr))
        else:
            print(f"jump_consensus_window_size {jump_consensus_window_size} is not supported")

    overall = np.zeros(len(model_fit_l))
    for frac in latent_downsample_frac:
        overall += res['downsampled_lml_' + str(frac)]['value_per_fit']
    overall /= len(latent_downsample_frac)
    put('metric_overall', overall)
    for v in res.values():
        v['best_value'] = np.max(v['value_per_fit'])
        v['best_index'] = np.argmax(v['value_per_fit'])
    return res


def model_selection_one_split(y, hyperparam_dict, train_index=None, test_index=None, test_frac=0.2, key=0,
                              model_to_return_type='best_overall', fit_kwargs=default_fit_kwargs,
                              model_class_str='poisson', n_repeat=5, latent_downsample_frac=[0.2, 0.4, 0.6, 0.8],
                              downsample_n_repeat=10,
                              metric_type_l=['log_marginal_test', 'log_one_step_predictive_marginal_test',
                                             'downsampled_lml', 'jump_consensus'],
                              jump_dynamics_index=1, jump_consensus_window_size=5,
                              jump_consensus_jump_p_thresh=0.4, jump_consensus_consensus_thresh=0.8,
                              fit_fn=None):
    """model_selection_helper.py:149-241: fit n_repeat restarts per grid config on the
    train split, evaluate them on the test split, keep the best by metric_overall.
    Keys follow the reference; jr.split(key) is replaced by split_keys."""
    import pandas as pd
    T = np.asarray(y).shape[0]
    if 'latentonly' in model_class_str:
        metric_type_l = [m for m in metric_type_l if 'jump' not in m]
    if train_index is None:
        train_index = slice(0, int(T * (1 - test_frac)))
    if test_index is None:
        test_index = slice(int(T * (1 - test_frac)), T)
    y_train = np.asarray(y)[train_index]
    y_test = np.asarray(y)[test_index]
    grid_l, grid_df = generate_hyperparam_grid(hyperparam_dict)
    fit_kwargs = dict(fit_kwargs)
    if fit_kwargs.get('log_posterior_init') is not None:
        fit_kwargs['log_posterior_init'] = np.asarray(fit_kwargs['log_posterior_init'])[train_index]
    all_cfg = {}
    best_model, best_model_l, best_config = None, None, None
    model_to_return_l = []
    best_overall = -np.inf
    for ii, param_dict in enumerate(grid_l):
        print('== Config {} of {} =='.format(ii + 1, len(grid_l)))
        key = split_keys(_seed_of(key), 2)[0]
        key_fit, key_eval = split_keys(key, 2)
        model_fit_l, _ = fit_model_one_config(param_dict, y_train, key=key_fit, fit_kwargs=fit_kwargs,
                                              model_class_str=model_class_str, n_repeat=n_repeat, fit_fn=fit_fn)
        ev = evaluate_model_one_config(model_fit_l, y_test, key=key_eval,
                                       latent_downsample_frac=latent_downsample_frac,
                                       downsample_n_repeat=downsample_n_repeat, metric_type_l=metric_type_l,
                                       jump_dynamics_index=jump_dynamics_index,
                                       jump_consensus_window_size=jump_consensus_window_size,
                                       jump_consensus_jump_p_thresh=jump_consensus_jump_p_thresh,
                                       jump_consensus_consensus_thresh=jump_consensus_consensus_thresh)
        for k, v in ev.items():
            all_cfg.setdefault(k + '_best_value', []).append(v['best_value'])
            all_cfg.setdefault(k + '_best_index', []).append(v['best_index'])
        cur = ev['metric_overall']['best_value']
        if cur > best_overall:
            best_overall = cur
            best_model = model_fit_l[ev['metric_overall']['best_index']]
            best_model_l = model_fit_l
            best_config = param_dict
        if model_to_return_type == 'best_per_config':
            model_to_return_l.append(model_fit_l[ev['metric_overall']['best_index']])
        elif model_to_return_type == 'all':
            model_to_return_l.append(model_fit_l)
    if model_to_return_type == 'best_overall':
        model_to_return_l = [best_model]
    elif model_to_return_type == 'best_config':
        model_to_return_l = [best_model_l]
    return {'model_to_return_l': model_to_return_l, 'best_config': best_config, 'best_model': best_model,
            'best_model_l': best_model_l,
            'model_eval_result_all_configs': pd.DataFrame(all_cfg).join(grid_df),
            'hyperparam_grid_df': grid_df, 'hyperparam_tosweep_keys': grid_df.columns}
