"""bench.py's multi-GPU path (head-hash shards, per-epoch delta all-reduce,
renormalisation) with two ranks on the one GPU of a test box: torchrun, gloo
over device tensors (RCCL will not put two ranks on one device).  Checks that
both ranks train, merge and report one JSON line with the N = 2 fields."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["transe_fb15k", "transr_fb15k"])
def test_bench_two_ranks_one_device(config):
    env = dict(os.environ, KB2E_DIST_ONE_DEVICE="1", KB2E_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29517" if config == "transe_fb15k" else "29518", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "120", "--warmup", "10", "--config", config, "--only", "--no-cpu-baseline", "--no-epoch", "--seed-epochs", "3"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and d["config"]["global_batch"] == 2 * (d["config"]["global_batch"] // 2)
    assert 0.3 < d["active_fraction"] < 1.0
    assert len(d["merge"]["ranks"]) == 2 and d["comm_nranks"] == 2 and len(d["pci_bus_ids"]) == 2


@pytest.mark.gpu
def test_bench_gpus_2_launches_its_own_ranks():
    """The driver's form, `python3 bench.py --gpus 2` with no launcher around it:
    bench.py starts torch.distributed.run itself (a child process, before any GPU
    call) and the line is a 2-rank line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(KB2E_DIST_ONE_DEVICE="1", KB2E_DIST_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "60", "--warmup", "5",
           "--config", "transe_fb15k", "--only", "--no-cpu-baseline", "--no-epoch"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert len(d["merge"]["ranks"]) == 2 and d["comm_nranks"] == 2
    assert sorted(r["rank"] for r in d["merge"]["ranks"]) == [0, 1]


def _merge_worker(rank, world, port, model, out):
    import numpy as np
    import torch
    import torch.distributed as dist

    from kb2e_amd import data
    from kb2e_amd.distributed import EpochMerger, shard_heads
    from kb2e_amd.engine import Engine

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ds = data.synthetic("small", seed=2)
    dim = 20
    eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=7 + rank,
                 schedule="parallel")
    eng.upload_triples(shard_heads(ds.train, rank, world))
    e0, r0, w0 = eng.init_params()
    if model == "R":
        eng.transr_seed(e0, r0)
    merger = EpochMerger(eng, dist)  # broadcasts rank 0's tables
    t0 = eng.download_params()
    eng.train_epoch()
    tr = eng.download_params()
    merger.merge()
    tm = eng.download_params()
    out[rank] = ([None if a is None else a.copy() for a in t0], [None if a is None else a.copy() for a in tr],
                 [None if a is None else a.copy() for a in tm])
    eng.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["E", "R"])
def test_epoch_merge_of_two_engines_matches_numpy(model):
    """Two real engines (two ranks on the test box's one GPU, gloo): after one
    epoch on their head shards, the merged tables on both ranks equal numpy
    renorm(T0 + sum_r (T_r - T0)) on the changed rows (TransE: rows shrink to
    length <= 1; TransR: entity, relation and matrix rows to unit length)."""
    import socket

    import numpy as np
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_merge_worker, args=(world, port, model, out), nprocs=world, join=True)
    t0 = out[0][0]
    for r in range(world):
        for k in range(3):
            if t0[k] is not None:
                assert np.array_equal(out[r][0][k], t0[k])  # both ranks started from rank 0's tables
    exp = []
    for k in range(3):
        if t0[k] is None:
            exp.append(None)
            continue
        base = t0[k].reshape(t0[k].shape[0], -1) if k < 2 else t0[k].reshape(-1, t0[k].shape[-1])
        tot = base.copy()
        unit_rows = np.zeros(len(base), bool)
        for r in range(world):
            d = out[r][1][k].reshape(base.shape) - base
            tot += d
            if k == 2 and model == "R":  # one mask row per relation, n matrix rows each
                ch = (d.reshape(t0[k].shape[0], -1) != 0).any(1)
                unit_rows |= np.repeat(ch, t0[k].shape[1])
            else:
                unit_rows |= (d != 0).any(1)
        for i in np.nonzero(unit_rows)[0]:
            n = np.linalg.norm(tot[i])
            if model == "R" or n > 1:
                tot[i] /= n
        exp.append(tot)
    for r in range(world):
        for k in range(3):
            if exp[k] is None:
                continue
            got = out[r][2][k].reshape(exp[k].shape)
            assert np.abs(got - exp[k]).max() < 1e-12, (r, k, np.abs(got - exp[k]).max())
