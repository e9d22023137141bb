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
