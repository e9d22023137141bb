"""Restart sharding over torch.distributed ranks (model_selection_helper.py:35-60),
world_size 2 on the gloo backend (CPU).  The per-restart fit is the CPU oracle
(injected fit_fn) so the sharding/gather logic is exercised without a GPU."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from tests.synth import make


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fit(model, y, key, fit_kwargs):
    from oracle import gplvm_oracle as O
    lp0 = O.init_latent_posterior_from_uniform(np.random.default_rng(key).random((y.shape[0], model.n_latent_bin)))
    r = O.fit_em(y, model.params.astype(np.float64), model.tuning_basis.astype(np.float64), lp0,
                 n_iter=fit_kwargs['n_iter'], m_step_maxiter=10, m_step_tol=0.0)
    return {'log_marginal_l': r['log_marginal_l'], 'key': key}


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from poor_man_gplvm_amd import model_selection_helper as msh
    d = make(8, 16, 40)
    models, res = msh.fit_model_one_config({'n_latent_bin': 16, 'tuning_lengthscale': 3.0}, d['y'], key=11,
                                           fit_kwargs={'n_iter': 2}, n_repeat=5, fit_fn=_oracle_fit)
    out[rank] = [(r['key'], r['log_marginal_l']) for r in res]
    dist.destroy_process_group()


def test_restart_sharding_world2_matches_single_process():
    from poor_man_gplvm_amd import model_selection_helper as msh
    d = make(8, 16, 40)
    _, ref = msh.fit_model_one_config({'n_latent_bin': 16, 'tuning_lengthscale': 3.0}, d['y'], key=11,
                                      fit_kwargs={'n_iter': 2}, n_repeat=5, fit_fn=_oracle_fit)
    ref = [(r['key'], r['log_marginal_l']) for r in ref]
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    for rank in range(2):
        got = out[rank]
        assert [k for k, _ in got] == [k for k, _ in ref]
        for (_, a), (_, b) in zip(got, ref):
            np.testing.assert_allclose(a, b, rtol=0, atol=0)


def _eval_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from poor_man_gplvm_amd import model_selection_helper as msh
    from tests.test_model_selection_host import _eval_case
    out[rank] = _eval_case(msh)
    dist.destroy_process_group()


def test_evaluation_sharding_world2_matches_single_process():
    """evaluate_model_one_config with fits sharded over 2 gloo ranks equals the
    single-process result on every rank (stand-in models decode with the oracle)."""
    from poor_man_gplvm_amd import model_selection_helper as msh
    from tests.test_model_selection_host import _eval_case
    ref = _eval_case(msh)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_eval_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for rank in range(2):
        got = out[rank]
        assert list(got) == list(ref)
        for k in ref:
            np.testing.assert_array_equal(got[k]['value_per_fit'], ref[k]['value_per_fit'])
            np.testing.assert_equal(got[k]['best_index'], ref[k]['best_index'])


def _shard_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from poor_man_gplvm_amd import model_selection_helper as msh
    seen = []

    def fn(idx):
        seen.extend(idx)
        return [{'k': i, 'v': np.arange(3) * i} for i in idx]
    res = msh.shard_map(7, fn)
    out[rank] = ([r['k'] for r in res], [r['v'].tolist() for r in res], seen)
    dist.destroy_process_group()


def test_shard_map_world2():
    """shard_map (the rank axis of get_downsampled_lml's masks and shuffle_and_decode's
    shuffles): item k computed on rank k % 2 only, every rank gets all results in order."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_shard_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for rank in range(2):
        keys, vals, seen = out[rank]
        assert keys == list(range(7))
        assert vals == [(np.arange(3) * i).tolist() for i in range(7)]
        assert seen == list(range(rank, 7, 2))
