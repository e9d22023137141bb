"""Host logic of the time-sharded EM (poor_man_gplvm_amd/timeshard.py), CPU only:
the shard layout (own ranges partition [0, T), halos on whole chunks of the global
grid) and the exchange primitives, LocalComm vs DistComm over gloo at world size 2
(the same calls the GPU path makes, on host tensors)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from poor_man_gplvm_amd.timeshard import LocalComm, shard_layout


@pytest.mark.parametrize("T,world,chunk,halo", [(400, 1, None, 512), (400, 3, 16, 16), (1000, 8, 7, 30),
                                                (100000, 8, None, 512), (1_000_000, 8, None, 512),
                                                (97, 5, 8, 1), (64, 4, 16, 1000)])
def test_shard_layout(T, world, chunk, halo):
    lays = shard_layout(T, world, chunk=chunk, halo=halo)
    C = lays[0].chunk
    assert len(lays) == world and lays[0].start == 0 and lays[-1].stop == T
    for a, b in zip(lays, lays[1:]):
        assert a.stop == b.start
    for lay in lays:
        assert lay.T_own > 0 and lay.start % C == 0 and lay.ext_start % C == 0
        assert lay.ext_stop % C == 0 or lay.ext_stop == T
        assert lay.ext_start <= lay.start < lay.stop <= lay.ext_stop
        # the own range is whole local chunks; halos only where there is a neighbour
        assert lay.left % C == 0 and lay.c_first * C == lay.left
        assert (lay.c_last + 1) * C >= lay.left + lay.T_own > lay.c_last * C
        if lay.rank == 0:
            assert lay.left == 0
        else:
            assert lay.left >= min(halo, lay.start) and lay.c_first >= 1
        if lay.rank == world - 1:
            assert lay.right == 0
        else:
            assert lay.right >= min(halo, T - lay.stop) and lay.c_last + 1 < lay.n_chunks
    sizes = [lay.T_own for lay in lays[:-1]]
    assert not sizes or max(sizes) - min(sizes) <= C


def test_shard_layout_rejects_too_many_shards():
    with pytest.raises(ValueError):
        shard_layout(40, 8, chunk=16)


def _local_reference(world):
    comm = LocalComm(world)
    send = [torch.full((6,), float(r + 1)) for r in range(world)]
    right = [torch.zeros(6) for _ in range(world)]
    left = [torch.zeros(6) for _ in range(world)]
    comm.shift([s if r < world - 1 else None for r, s in enumerate(send)],
               [t if r > 0 else None for r, t in enumerate(right)], +1)
    comm.shift([s if r > 0 else None for r, s in enumerate(send)],
               [t if r < world - 1 else None for r, t in enumerate(left)], -1)
    sums = [[torch.arange(4, dtype=torch.float64) * (r + 1)] for r in range(world)]
    comm.allreduce_sum(sums)
    return right, left, sums, comm.allreduce_max_int([r % 2 for r in range(world)])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from poor_man_gplvm_amd.timeshard import DistComm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = DistComm()
    send = torch.full((6,), float(rank + 1))
    right, left = torch.zeros(6), torch.zeros(6)
    comm.shift([send if rank < world - 1 else None], [right if rank > 0 else None], +1)
    comm.shift([send if rank > 0 else None], [left if rank < world - 1 else None], -1)
    s = torch.arange(4, dtype=torch.float64) * (rank + 1)
    comm.allreduce_sum([[s]])
    mx = comm.allreduce_max_int([rank % 2])
    g = comm.gather_rank0([torch.arange(3 + rank, dtype=torch.float32) + 10 * rank])
    out[rank] = (right.numpy(), left.numpy(), s.numpy(), mx, [x.numpy() for x in g])
    dist.destroy_process_group()


def test_distcomm_gloo_matches_localcomm():
    world = 2
    right, left, sums, mx = _local_reference(world)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        rr, ll, ss, m, g = out[r]
        np.testing.assert_array_equal(rr, right[r].numpy())
        np.testing.assert_array_equal(ll, left[r].numpy())
        np.testing.assert_array_equal(ss, sums[r][0].numpy())
        assert m == mx
    g0 = out[0][4]
    assert len(g0) == 2 and out[1][4] == []
    np.testing.assert_array_equal(g0[1], np.arange(4, dtype=np.float32) + 10)


# ---------------------------------------------------------------- neuron-sharded Adam
def _kernel_mimic(W, mu, nu, count, kmax, tol, a, c, lr=0.01, b1=0.9, b2=0.999, eps=1e-8):
    """The persistent kernel's loop semantics on a separable objective
    f(W) = sum_n 0.5 a_n (w_n - c_n)^2 (stop rule of fit_tuning_helper.py:154-164;
    loss_hist[0] = loss_0, loss_hist[j+1] = loss_j; W after the stopping body)."""
    def loss_grad(w):
        return 0.5 * np.sum(a * (w - c) ** 2), a * (w - c)
    lh, eh = [], []
    if kmax <= 1:
        l0, g0 = loss_grad(W)
        return 1, np.array([l0]), np.array([np.sqrt(np.sum(g0 ** 2))])
    prev = None
    for j in range(10 ** 6):
        loss, g = loss_grad(W)
        lh.append(loss)
        eh.append(np.sqrt(np.sum(g ** 2)))
        count[0] += 1
        mu[:] = (1 - b1) * g + b1 * mu
        nu[:] = (1 - b2) * g * g + b2 * nu
        mh = mu / (1 - b1 ** count[0])
        nh = nu / (1 - b2 ** count[0])
        W[:] = W - lr * mh / (np.sqrt(nh) + eps)
        if j == 0:
            prev = loss
        rel = abs(loss - prev) / max(abs(loss), 1e-8)
        cont = (j + 1 < kmax - 1) and ((j + 1 < 5) or (rel > tol))
        prev = loss
        if not cont:
            return j + 2, np.array([lh[0]] + lh), np.array([eh[0]] + eh)


@pytest.mark.parametrize("max_batch", [None, 64])
@pytest.mark.parametrize("maxiter,tol,world", [(1000, 1e-6, 3), (40, 0.0, 2), (23, 0.0, 4), (1, 1e-6, 2),
                                               (7, 1e-6, 3), (150, 0.0, 2)])
def test_speculative_adam_matches_unsharded(maxiter, tol, world, max_batch):
    from poor_man_gplvm_amd.timeshard import neuron_bounds, speculative_adam
    rng = np.random.default_rng(0)
    N = 37
    a = rng.uniform(0.5, 2.0, N)
    c = rng.normal(size=N)
    W0 = rng.normal(size=N)
    # unsharded loop
    W, mu, nu, cnt = W0.copy(), np.zeros(N), np.zeros(N), [5]
    n_ref, lh_ref, eh_ref = _kernel_mimic(W, mu, nu, cnt, maxiter, tol, a, c)
    # neuron-sharded speculative loop (all ranks in this process: the reduce is the identity)
    bnd = neuron_bounds(N, world)
    sl = [dict(W=W0[x:y].copy(), mu=np.zeros(y - x), nu=np.zeros(y - x), cnt=[5], a=a[x:y], c=c[x:y])
          for x, y in bnd]

    def run(kmax):
        return [_kernel_mimic(d['W'], d['mu'], d['nu'], d['cnt'], kmax, -1.0, d['a'], d['c']) for d in sl]

    def snapshot():
        return [(d['W'].copy(), d['mu'].copy(), d['nu'].copy(), list(d['cnt'])) for d in sl]

    def restore(snap):
        for d, (w, m, v, k) in zip(sl, snap):
            d['W'][:], d['mu'][:], d['nu'][:], d['cnt'][:] = w, m, v, k

    res = speculative_adam(run, snapshot, restore, lambda x: x, maxiter, tol, max_batch=max_batch)
    assert res['n_iter'] == n_ref
    np.testing.assert_array_equal(np.concatenate([d['W'] for d in sl]), W)
    assert all(d['cnt'][0] == cnt[0] for d in sl)
    np.testing.assert_allclose(res['loss_history'], lh_ref, rtol=1e-13)
    np.testing.assert_allclose(res['error_history'], eh_ref, rtol=1e-13)
    assert res['final_loss'] == pytest.approx(lh_ref[-1], rel=1e-13)


def test_speculative_adam_rejects_desynchronised_slices():
    """Every local slice must run exactly `batch` bodies (tol < 0); a slice that stops
    early would desynchronise the ranks' loss all-reduce, so it raises instead."""
    from poor_man_gplvm_amd.timeshard import speculative_adam

    def run(kmax):
        return [(kmax, np.ones(kmax), np.ones(kmax)), (kmax - 3, np.ones(kmax - 3), np.ones(kmax - 3))]

    with pytest.raises(RuntimeError):
        speculative_adam(run, lambda: None, lambda s: None, lambda x: x, 1000, 1e-6)
