"""Multi-rank path on CPU (gloo, world size 2): head-hash sharding and the
epoch-boundary delta merge of kb2e_amd.distributed."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kb2e_amd import data
from kb2e_amd.distributed import merge_deltas, shard_heads


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shards_partition_the_triples():
    ds = data.synthetic("small", seed=0)
    parts = [shard_heads(ds.train, r, 4) for r in range(4)]
    assert sum(len(p) for p in parts) == len(ds.train)
    heads = [set(p[:, 0].tolist()) for p in parts]
    for a in range(4):
        for b in range(a + 1, 4):
            assert not heads[a] & heads[b]  # an entity's head triples live on one rank
    assert min(len(p) for p in parts) > 0.15 * len(ds.train)


def _worker(rank, world, port, out):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rows, ld = 6, 4
    base = [torch.arange(rows * ld, dtype=torch.float64) / 10.0, torch.ones(3 * ld, dtype=torch.float64)]
    tables = [b.clone() for b in base]
    # rank r updates entity row r and relation row 0 (shared)
    tables[0].view(rows, ld)[rank] += rank + 1
    tables[1].view(3, ld)[0] += 0.5
    masks = merge_deltas(tables, base, dist, [ld, ld])
    out[rank] = (tables[0].numpy().copy(), tables[1].numpy().copy(), masks[0].copy(), masks[1].copy())
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_merge_sums_rank_deltas_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    base_e = np.arange(24, dtype=np.float64).reshape(6, 4) / 10.0
    exp_e = base_e.copy()
    exp_e[0] += 1
    exp_e[1] += 2
    exp_r = np.ones((3, 4))
    exp_r[0] += 1.0  # both ranks' +0.5
    for r in range(world):
        e, rel, me, mr = out[r]
        assert np.allclose(e.reshape(6, 4), exp_e) and np.allclose(rel.reshape(3, 4), exp_r)
        assert me.tolist() == [1, 1, 0, 0, 0, 0] and mr.tolist() == [1, 0, 0]
