"""The RCCL path of the two shard axes: torch.distributed backend
"nccl" (= RCCL over xGMI on ROCm) with device tensors, one process per GPU.

* time shards of one recording (decoder.py:283-326 carries, fit_tuning_helper.py:28-42
  sums): timeshard.DistComm on RCCL runs run_em_timesharded on the README-shape golden
  (em_c1_one.npz) and must meet the golden's bars -- the exchange primitives
  (all_reduce of y_w / t_w and logZ, the carry shifts, the all_gather of the neuron-
  sharded Adam's W blocks) then run as RCCL collectives on device buffers;
* independent restarts (model_selection_helper.py:53-59): fit_model_one_config shards
  the restarts over the ranks and gathers them with all_gather_object over RCCL; each
  restart must equal the same restart fitted alone.

World 1 always runs (RCCL with one rank still initialises its communicator and launches
every collective); world 2 runs when two GPUs are visible (RCCL refuses two ranks on one
device), as on the driver's multi-GPU node.  The workers are spawned processes (the
test process has touched the GPU), each binds cuda:rank before any other GPU call and
talks to its peers over 127.0.0.1."""
import os
import socket

import numpy as np
import pytest
import torch

from tests.test_gpu_parity import HERE, RT, close_prob

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _nccl_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    import poor_man_gplvm_amd as P
    from poor_man_gplvm_amd import model_selection_helper as msh
    from poor_man_gplvm_amd.timeshard import DistComm, run_em_timesharded
    from tests.synth import make
    rec = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
    f = np.load(os.path.join(HERE, 'golden', 'em_c1_one.npz'))
    L = f['basis'].shape[0]
    for ns in (False, True):
        comm = DistComm()
        assert not comm.host            # device tensors, no host staging
        res, info = run_em_timesharded(f['y'].astype(np.float32), f['W0'], f['basis'], f['lp0'],
                                       n_iter=int(f['n_iter']), transition=P.banded_transition(L, float(f['mv'])),
                                       comm=comm, chunk=16, halo=32, neuron_sharded=ns,
                                       adam=P.AdamConfig(maxiter=int(f['maxiter']), tol=float(f['tol'])))
        rec[f'ts_{ns}'] = (info['params64'] if res is None else
                           (res['posterior_latent_marg'], res['tuning'], res['log_marginal_l'], info['params64'],
                            res['m_step_res_l']['n_iter']))
    d = make(24, 32, 1500)
    models, fits = msh.fit_model_one_config({'n_latent_bin': 32, 'tuning_lengthscale': 4.0}, d['y'], key=5,
                                            fit_kwargs={'n_iter': 3}, n_repeat=3)
    rec['restarts'] = [(np.asarray(r['log_marginal_l']), np.asarray(r['tuning'])) for r in fits]
    out[rank] = rec
    dist.barrier()
    dist.destroy_process_group()


def _run(world):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_nccl_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    return dict(out)


def _check(out, world):
    f = np.load(os.path.join(HERE, 'golden', 'em_c1_one.npz'))
    r0 = out[0]
    assert r0['backend'] == 'nccl' and r0['world'] == world
    for ns in (False, True):
        plm, tun, lz, W, n_iter = r0[f'ts_{ns}']
        np.testing.assert_allclose(tun, f['tuning'], rtol=RT)
        close_prob(plm, f['posterior'].astype(np.float64).sum(1))
        np.testing.assert_allclose(lz, f['log_marginal_l'], rtol=1e-7)
        assert n_iter == list(f['m_n_iter'])
        for r in range(1, world):       # every rank ends with the same W
            Wr = out[r][f'ts_{ns}']
            np.testing.assert_array_equal(Wr if isinstance(Wr, np.ndarray) else Wr[3], W)
    # the gathered restarts: identical lists on every rank, each equal to that restart alone
    import poor_man_gplvm_amd as P
    from tests.synth import make
    d = make(24, 32, 1500)
    for r in range(1, world):
        for (a_l, a_t), (b_l, b_t) in zip(out[r]['restarts'], r0['restarts']):
            np.testing.assert_array_equal(a_l, b_l)
            np.testing.assert_array_equal(a_t, b_t)
    from poor_man_gplvm_amd import model_selection_helper as msh
    keys = msh.split_keys(5, 3)
    for k, (lml, tun) in zip(keys, r0['restarts']):
        m = P.PoissonGPLVMJump1D(24, n_latent_bin=32, tuning_lengthscale=4.0)
        res = m.fit_em(d['y'], key=k, n_iter=3)
        # the same chunking; the relaxation segment grid differs (#CUs / R per restart in
        # the batch), so the test_gpu_restarts bars, not bit identity
        np.testing.assert_allclose(lml, res['log_marginal_l'], rtol=1e-7)
        np.testing.assert_allclose(tun, res['tuning'], rtol=RT)


def test_rccl_world1():
    _check(_run(1), 1)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs one GPU per rank; world 2 needs two GPUs")
def test_rccl_world2():
    _check(_run(2), 2)
