"""The multi-GPU epoch merge behind the C ABI (include/kb2e_engine.h
"Multi-GPU epoch merge", kb2e_amd/csrc/engine_merge.inc).

On the one-GPU test box:
* two engines on the same device in one process (kb2e_comm_init_group: the
  local kernel backend, since RCCL refuses two ranks on one GPU), each trained
  one epoch on its head-hash shard, merged with kb2e_merge_epoch_group, against
  numpy renorm(T0 + sum_r (T_r - T0)) on the changed rows;
* one engine on a one-rank RCCL communicator (kb2e_comm_unique_id +
  kb2e_comm_init_rank + kb2e_merge_epoch): the RCCL calls themselves;
* the drop-in CLI with --gpus 2 (both ranks on the one device): its epoch lines
  equal the Python group driver's losses on the same shards and seeds.
"""
import os
import subprocess

import numpy as np
import pytest

from kb2e_amd import data
from kb2e_amd.distributed import shard_heads
from kb2e_amd.engine import Engine, comm_init_group, merge_epoch_group

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _flat_rows(t, k, model):
    """The table as rows: entity / relation rows; TransH normals; TransR matrix rows."""
    return t.reshape(t.shape[0], -1) if k < 2 or model == "H" else t.reshape(-1, t.shape[-1])


def expected_merge(model, base, ranks):
    """numpy renorm(T0 + sum_r (T_r - T0)): TransE rows and TransH entity /
    relation rows shrink to length <= 1 (common/utils.cpp:70-77), TransH normals
    and every TransR row scale to unit length; only rows some rank changed."""
    exp = []
    for k in range(3):
        if base[k] is None:
            exp.append(None)
            continue
        b = _flat_rows(base[k], k, model)
        tot = b.copy()
        changed = np.zeros(len(b), bool)
        for tr in ranks:
            d = _flat_rows(tr[k], k, model) - b
            tot += d
            if k == 2 and model == "R":  # one mask entry per relation, n matrix rows each
                ch = (d.reshape(base[k].shape[0], -1) != 0).any(1)
                changed |= np.repeat(ch, base[k].shape[1])
            else:
                changed |= (d != 0).any(1)
        unit = model == "R" or (model == "H" and k == 2)
        for i in np.nonzero(changed)[0]:
            n = np.linalg.norm(tot[i])
            if unit or n > 1:
                tot[i] /= n
        exp.append(tot)
    return exp


def _engines(model, world, schedule="parallel", dim=20):
    ds = data.synthetic("small", seed=2)
    engs = []
    for r in range(world):
        eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=7 + r,
                     schedule=schedule)
        eng.upload_triples(shard_heads(ds.train, r, world))
        e0, r0, _ = eng.init_params()
        if model == "R":
            eng.transr_seed(e0, r0)
        engs.append(eng)
    return ds, engs


@pytest.mark.gpu
@pytest.mark.parametrize("model,schedule", [("E", "parallel"), ("H", "parallel"), ("R", "parallel"), ("R", "ordered")])
def test_group_merge_local_backend_matches_numpy(model, schedule):
    ds, engs = _engines(model, 2, schedule)
    try:
        comm_init_group(engs)  # rank 0's tables to both
        t0 = engs[0].download_params()
        t1 = engs[1].download_params()
        for k in range(3):
            if t0[k] is not None:
                assert np.array_equal(t0[k], t1[k])
        for e in engs:
            e.train_epoch()
        trained = [e.download_params() for e in engs]
        assert not np.array_equal(trained[0][0], trained[1][0])  # the shards differ
        merge_epoch_group(engs)
        exp = expected_merge(model, t0, trained)
        for e in engs:
            got = e.download_params()
            for k in range(3):
                if exp[k] is not None:
                    err = np.abs(_flat_rows(got[k], k, model) - exp[k]).max()
                    assert err < 1e-12, (model, k, err)
        # a second epoch + merge starts from the merged tables (the base moved)
        base = engs[0].download_params()
        for e in engs:
            e.train_epoch()
        trained = [e.download_params() for e in engs]
        merge_epoch_group(engs)
        exp = expected_merge(model, base, trained)
        got = engs[1].download_params()
        for k in range(3):
            if exp[k] is not None:
                assert np.abs(_flat_rows(got[k], k, model) - exp[k]).max() < 1e-12
    finally:
        for e in engs:
            e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["E", "R"])
def test_single_rank_rccl_merge(model):
    import torch  # noqa: F401  (torch's own RCCL in the process, as in bench.py)

    ds, engs = _engines(model, 1)
    eng = engs[0]
    try:
        eng.comm_init_rank(1, 0, Engine.comm_unique_id())
        assert eng.comm_info() == (1, 0, 0, ds.num_entities)
        t0 = eng.download_params()
        eng.train_epoch()
        tr = eng.download_params()
        eng.merge_epoch()
        exp = expected_merge(model, t0, [tr])
        got = eng.download_params()
        for k in range(3):
            if exp[k] is not None:
                assert np.abs(_flat_rows(got[k], k, model) - exp[k]).max() < 1e-12
        # training continues on the merged tables
        loss, act = eng.train_epoch()
        assert np.isfinite(loss) and act > 0
    finally:
        eng.close()


@pytest.mark.gpu
def test_merge_needs_a_communicator():
    ds, engs = _engines("E", 1)
    with pytest.raises(RuntimeError, match="comm_init"):
        engs[0].merge_epoch()
    engs[0].close()


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["E", "R"])
def test_cli_two_gpus_matches_python_group(tmp_path, model):
    """bin/trainTrans* --gpus 2 (one process driving two contexts) prints the
    epoch losses of the Python group driver on the same shards and seeds."""
    ds = data.synthetic("small", seed=2)
    d = str(tmp_path)
    data.write(ds, d)
    dim, epochs, seed = 20, 3, 11
    exe = os.path.join(ROOT, "bin", {"E": "trainTransE", "R": "trainTransR"}[model])
    cmd = [exe, "--datadir", d, "--outdir", d, "--size", str(dim), "--epochs", str(epochs), "--batches", "20",
           "--seed", str(seed), "--rate", "0.01", "--schedule", "1", "--gpus", "2"]
    if model == "R":  # TransE seed files from a one-GPU TransE run
        subprocess.run([os.path.join(ROOT, "bin", "trainTransE"), "--datadir", d, "--outdir", d, "--size", str(dim),
                        "--epochs", "2", "--method", "0", "--seed", "3"], check=True, capture_output=True, timeout=100)
        cmd += ["--seeddatadir", d, "--seedmethod", "0"]
    env = dict(os.environ, KB2E_CLI_ONE_DEVICE="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=100, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    cli = [float(ln.split("Loss: ")[1]) for ln in out.stdout.splitlines() if ln.startswith("Epoch: ")]
    assert len(cli) == epochs
    for f in ("entity2vec.bern", "relation2vec.bern") + (("weights.bern",) if model == "R" else ()):
        assert os.path.getsize(os.path.join(d, f)) > 0
    # the same run through the Python bindings
    engs = []
    for r in range(2):
        tr = shard_heads(ds.train, r, 2)
        eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=seed + r,
                     schedule="parallel")
        eng.upload_triples(tr)
        eng.init_params_device(fetch=False)
        if model == "R":
            eng.read_table(0, os.path.join(d, "entity2vec.unif"), 1)
            eng.read_table(1, os.path.join(d, "relation2vec.unif"), 0)
        engs.append(eng)
    try:
        comm_init_group(engs)
        py = []
        for _ in range(epochs):
            tot = 0.0
            for e in engs:
                e.train_batches(10)
            for e in engs:
                tot += e.take_stats()[0]
            merge_epoch_group(engs)
            py.append(tot)
    finally:
        for e in engs:
            e.close()
    for a, b in zip(cli, py):
        assert abs(a - b) <= 1e-6 * max(1.0, abs(b)) + 1e-6, (cli, py)
