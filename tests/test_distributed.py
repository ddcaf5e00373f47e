"""Multi-rank path on CPU (gloo, world size 2, 3 and 4): head-hash sharding and the
epoch-boundary merge of kb2e_amd.distributed (reduce-scatter of entity deltas
to block owners + all-gather, all-reduce of relation/weight deltas, changed
rows renormalised) against numpy renorm(T0 + sum_r (T_r - T0))."""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kb2e_amd import data
from kb2e_amd.distributed import TableMerger, shard_heads


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


NE, NR, L = 11, 4, 3  # 11 entity rows: uneven blocks over 2 and 3 ranks


class CpuRows:
    """The engine's row constraint on CPU tensors: shrink rows longer than 1
    (TransE, common/utils.cpp:70-77) -- unit length for the weights (TransH w)."""

    def __init__(self, tables):
        self.tables = tables
        self.calls = []

    def synchronize(self):
        pass

    def renormalize(self, table, first, count, mask):
        t = self.tables[table].view(-1, L)[first:first + count]
        self.calls.append((table, first, count))
        for k in range(count):
            if mask is not None and not mask[k]:
                continue
            n = float(torch.sqrt((t[k] ** 2).sum()))
            if table == 2 or n > 1:
                t[k] /= n


def _initial():
    rng = np.random.default_rng(0)
    return [rng.uniform(-0.5, 0.5, (NE, L)), rng.uniform(-0.5, 0.5, (NR, L)), rng.uniform(-1, 1, (NR, L))]


def _rank_update(rank):
    """What rank `rank` trained: a few entity rows (some shared), a shared relation, a weight row."""
    rng = np.random.default_rng(100 + rank)
    d = [np.zeros((NE, L)), np.zeros((NR, L)), np.zeros((NR, L))]
    for e in {rank, rank + 3, 7, NE - 1}:
        d[0][e] = rng.normal(0, 0.8, L)
    d[1][1] = rng.normal(0, 0.8, L)
    d[2][rank % NR] = rng.normal(0, 0.3, L)
    return d


def _worker(rank, world, port, out):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    init = _initial()
    # rank 0's tables win the initial broadcast: others start from garbage
    tables = [torch.tensor(t if rank == 0 else t + 5.0).reshape(-1) for t in init]
    rows = CpuRows(tables)
    m = TableMerger(tables, [NE, NR, NR], [L, L, L], rows, dist)
    for t, d in zip(tables, _rank_update(rank)):
        t += torch.tensor(d).reshape(-1)
    m.merge()
    out[rank] = ([t.numpy().copy() for t in tables], rows.calls)
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_merge_matches_numpy_renorm_of_summed_deltas(world):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    init = _initial()
    exp = [t.copy() for t in init]
    changed = [np.zeros(len(t), bool) for t in init]
    for r in range(world):
        for k, d in enumerate(_rank_update(r)):
            exp[k] += d
            changed[k] |= (d != 0).any(1)
    for k, t in enumerate(exp):
        for i in np.nonzero(changed[k])[0]:
            n = np.linalg.norm(t[i])
            if k == 2 or n > 1:
                t[i] /= n
    block = (NE + world - 1) // world
    for r in range(world):
        tabs, calls = out[r]
        for k in range(3):
            assert np.allclose(tabs[k].reshape(-1, L), exp[k], atol=1e-12), (r, k)
        # each rank renormalised only its own entity block
        lo = min(NE, r * block)
        assert (0, lo, min(NE, lo + block) - lo) in calls


# ---- bench.py's rank launch (the driver runs `bench.py --gpus N`) ----

def _bench(args, env_extra):
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_bench_refuses_a_rank_count_that_disagrees_with_gpus():
    """--gpus 2 inside a 1-rank launch (and --gpus 1 inside a 2-rank one) exits
    non-zero before any work: a scaling line must never be a 1-GPU line."""
    out = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr, out.stderr[-500:]
    out = _bench(["--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr, out.stderr[-500:]


def test_bench_gpus_n_launches_n_ranks(monkeypatch):
    """`bench.py --gpus 4` without WORLD_SIZE runs torch.distributed.run with four
    ranks on 127.0.0.1 over this same command line, as a child process, and exits
    with the child's code."""
    import importlib
    import subprocess
    import sys

    import bench

    importlib.reload(bench)
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 2] == sys.executable and cmd[i - 1] == "-m"
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4" and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
