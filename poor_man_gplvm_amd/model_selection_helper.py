"""Independent EM restarts (model_selection_helper.py:35-60), sharded over ranks.

`fit_model_one_config` keeps the reference's signature and return value
(lists of fitted models and fit_em dicts, in key order).  When torch.distributed
is initialised, restart k runs on rank k % world_size -- restarts are fully
independent, so there is no data-path collective -- and the per-rank results are
gathered with all_gather_object at the end so every rank returns the full lists.
"""
from __future__ import annotations

import numpy as np

from .core import PoissonGPLVMJump1D

model_class_dict = {'poisson': PoissonGPLVMJump1D}

default_fit_kwargs = {'n_iter': 20, 'log_posterior_init': None, 'n_time_per_chunk': 10000, 'dt': 1.,
                      'likelihood_scale': 1., 'save_every': None,
                      'posterior_init_kwargs': {'random_scale': 0.1}}


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


def fit_model_one_config(config, y_train, key=0, fit_kwargs=default_fit_kwargs, model_class_str='poisson',
                         n_repeat=1, fit_fn=None):
    """model_selection_helper.py:35-60.  `fit_fn(model, y, key, fit_kwargs) -> em_res`
    replaces model.fit_em (used by the CPU gloo tests to exercise the sharding)."""
    if model_class_str not in model_class_dict:
        raise ValueError(f"Invalid model class: {model_class_str} (only 'poisson' is implemented)")
    model_class = model_class_dict[model_class_str]
    key_l = list(key) if isinstance(key, list) else split_keys(key, n_repeat)
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    mine = []
    for k_idx in range(rank, len(key_l), world):
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
