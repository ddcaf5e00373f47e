"""GPU link-prediction evaluator vs the reference's eval binaries (golden) and
the oracle.  Energies are bit-identical FP64 restatements, so mean ranks and
hits@10 must match exactly (no ties in these tables)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_common import MANIFEST, tiny
from kb2e_amd import data
from kb2e_amd.engine import Engine
from oracle import orc

pytestmark = pytest.mark.gpu


def _load_run(name):
    run = MANIFEST["runs"][name]
    f = run["flags"]
    ds = tiny()
    d = os.path.join(GOLDEN, name)
    sfx = "bern" if f["method"] == 1 else "unif"
    n = f["size"]
    ent = data.read_table(os.path.join(d, f"entity2vec.{sfx}"), ds.num_entities, n)
    rel = data.read_table(os.path.join(d, f"relation2vec.{sfx}"), ds.num_relations, n)
    w = None
    if run["model"] == "H":
        w = data.read_table(os.path.join(d, f"weights.{sfx}"), ds.num_relations, n)
    if run["model"] == "R":
        w = data.read_table(os.path.join(d, f"weights.{sfx}"), ds.num_relations * n, n).reshape(-1, n, n)
    return run, ds, ent, rel, w


@pytest.mark.parametrize("name", ["transe_l1_bern", "transe_l2_unif", "transh_bern", "transe_seed_unif"])
def test_eval_matches_reference_binary(name):
    run, ds, ent, rel, w = _load_run(name)
    f = run["flags"]
    eng = Engine(run["model"], f["size"], ds.num_entities, ds.num_relations, distance=f["distance"],
                 method=f["method"])
    eng.upload_params(ent, rel, w)
    res = eng.evaluate(ds.test, np.concatenate([ds.test, ds.train, ds.valid]))
    ev = run["eval"]
    assert res["raw_rank"] == pytest.approx(ev["raw"]["rank"], abs=5e-7)
    assert res["filtered_rank"] == pytest.approx(ev["filtered"]["rank"], abs=5e-7)
    assert res["raw_hits10"] == pytest.approx(ev["raw"]["hits10"], abs=5e-7)
    assert res["filtered_hits10"] == pytest.approx(ev["filtered"]["hits10"], abs=5e-7)


def test_eval_transr_fixed_matches_oracle():
    run, ds, ent, rel, w = _load_run("transr_fixed")
    n = run["flags"]["size"]
    eng = Engine("R", n, ds.num_entities, ds.num_relations, transr_compat=False)
    eng.upload_params(ent, rel, w)
    filt = np.concatenate([ds.test, ds.train, ds.valid])
    res = eng.evaluate(ds.test, filt)
    m = orc.Model("R", n, ds.num_entities, ds.num_relations, transr_compat=False)
    m.set_tables(ent, rel, w)
    exp = m.evaluate(ds.test, filt)
    assert exp["ties"] == 0
    for k in ("raw_rank", "raw_hits10", "filtered_rank", "filtered_hits10"):
        assert res[k] == pytest.approx(exp[k], abs=1e-12), k


@pytest.mark.parametrize("model,dim", [("E", 50), ("H", 32)])
def test_eval_larger_set_matches_oracle(model, dim):
    ds = data.synthetic("small", seed=3)
    rng = np.random.default_rng(0)
    ent = rng.standard_normal((ds.num_entities, dim)) * 0.2
    rel = rng.standard_normal((ds.num_relations, dim)) * 0.2
    w = None
    if model == "H":
        w = rng.standard_normal((ds.num_relations, dim))
        w /= np.linalg.norm(w, axis=1, keepdims=True)
    eng = Engine(model, dim, ds.num_entities, ds.num_relations)
    eng.upload_params(ent, rel, w)
    filt = np.concatenate([ds.test, ds.train, ds.valid])
    res = eng.evaluate(ds.test, filt)
    m = orc.Model(model, dim, ds.num_entities, ds.num_relations)
    m.set_tables(ent, rel, w)
    exp = m.evaluate(ds.test, filt)
    assert exp["ties"] == 0
    for k in ("raw_rank", "raw_hits10", "filtered_rank", "filtered_hits10"):
        assert res[k] == pytest.approx(exp[k], abs=1e-12), k


# ---------------------------------------------------------------- TransR compat
# The reference's evalTransR never zeroes its energy work vectors
# (transr/transr.cpp:20-25, transr/evaluation.cpp:22-32): every energy depends on
# all energies computed before it in the cached relation-major loop
# (common/evaluation.cpp:107-121, 181-238).  The device replays that chain in
# the reference's operation order, so its energies are the oracle's bit for
# bit: ranks, hits, tie counts and the final work vectors must be EQUAL.


def _compat_vs_oracle(ds, n, ent, rel, w, *, distance=0, work=None, test=None):
    test = ds.test if test is None else test
    filt = np.concatenate([ds.test, ds.train, ds.valid])
    eng = Engine("R", n, ds.num_entities, ds.num_relations, distance=distance)
    eng.upload_params(ent, rel, w)
    res = eng.evaluate_transr_compat(test, filt, work)
    m = orc.Model("R", n, ds.num_entities, ds.num_relations, distance=distance, transr_compat=True)
    m.set_tables(ent, rel, w)
    w0 = np.zeros((2, n)) if work is None else np.asarray(work).reshape(2, n)
    m.set_transr_work(w0[0], w0[1])
    exp = m.evaluate(test, filt)
    for k in ("raw_rank", "raw_hits10", "filtered_rank", "filtered_hits10", "ties"):
        assert res[k] == exp[k], (k, res[k], exp[k])
    hw, tw = m.transr_work()
    assert np.array_equal(res["work"][0], hw) and np.array_equal(res["work"][1], tw)
    return res


def test_eval_transr_compat_matches_reference_binary():
    """Golden: the reference evalTransR's printed numbers on the transr_compat run
    (the oracle, and so the device, agree with them up to the exact ties)."""
    run, ds, ent, rel, w = _load_run("transr_compat")
    res = _compat_vs_oracle(ds, run["flags"]["size"], ent, rel, w)
    ev, n2 = run["eval"], 2 * len(ds.test)
    assert res["ties"] > 0
    assert abs(res["filtered_rank"] - ev["filtered"]["rank"]) * n2 <= res["ties"] + 1e-6
    assert abs(res["raw_rank"] - ev["raw"]["rank"]) * n2 <= res["ties"] + 1e-6
    assert abs(res["filtered_hits10"] - ev["filtered"]["hits10"]) * n2 <= res["ties"] + 1e-6
    assert abs(res["raw_hits10"] - ev["raw"]["hits10"]) * n2 <= res["ties"] + 1e-6


def _random_transr(ds, n, seed, scale=0.3):
    rng = np.random.default_rng(seed)
    ent = rng.standard_normal((ds.num_entities, n))
    ent /= np.linalg.norm(ent, axis=1, keepdims=True)
    rel = rng.standard_normal((ds.num_relations, n)) * scale
    w = np.eye(n)[None] + rng.standard_normal((ds.num_relations, n, n)) * (scale / np.sqrt(n))
    return ent, rel, w


@pytest.mark.parametrize("n,distance", [(20, 0), (50, 1), (100, 0), (128, 0)])
def test_eval_transr_compat_tiny_dims(n, distance):
    """n > 64: two and more elements per lane in the chain wave."""
    ds = tiny()
    ent, rel, w = _random_transr(ds, n, n)
    _compat_vs_oracle(ds, n, ent, rel, w, distance=distance)


@pytest.mark.parametrize("n,w_l2", [(200, "0"), (160, "0"), (50, "1")])
def test_eval_transr_compat_wide(n, w_l2, monkeypatch):
    """Above dim 140 W's n x n image no longer fits the LDS and the chain wave
    reads it from L2 (the reference's evalTransR takes any --size,
    transr/evaluation.cpp:22-32); KB2E_EVAL_W_L2=1 forces that form at n = 50.
    Still bit-identical to the oracle's energies."""
    monkeypatch.setenv("KB2E_EVAL_W_L2", w_l2)
    ds = tiny()
    ent, rel, w = _random_transr(ds, n, n)
    _compat_vs_oracle(ds, n, ent, rel, w, test=ds.test[:60])


def test_eval_transr_compat_small_set_with_state():
    """2,000 entities (the per-relation cache on), 1,000 test triples over 40
    relations, starting from non-zero work vectors (a process that already
    evaluated something)."""
    ds = data.synthetic("small", seed=5)
    n = 20
    ent, rel, w = _random_transr(ds, n, 1)
    work = np.random.default_rng(2).standard_normal((2, n))
    _compat_vs_oracle(ds, n, ent, rel, w, work=work)


def test_eval_transr_compat_without_cache():
    """|E| > 40,000 (common/evaluation.h:11): the reference evaluates with no cache,
    every corruption recomputed."""
    ds = data.synthetic("small", seed=6, counts=(40500, 3, 3000, 10, 12))
    n = 8
    ent, rel, w = _random_transr(ds, n, 3)
    _compat_vs_oracle(ds, n, ent, rel, w)


@pytest.mark.parametrize("model,dim,rows_l2", [("E", 200, "0"), ("H", 160, "0"), ("E", 512, "0"), ("E", 200, "1"),
                                               ("H", 512, "1")])
def test_eval_wide_rows_matches_oracle(model, dim, rows_l2, monkeypatch):
    """dim > 128 (the reference accepts any --size; a context takes <= 512);
    rows_l2: the rank tiles read the query rows from L2 instead of LDS (the
    form that lifts the ranking's dim limit past 600)."""
    monkeypatch.setenv("KB2E_EVAL_ROWS_L2", rows_l2)
    ds = tiny()
    rng = np.random.default_rng(dim)
    ent = rng.standard_normal((ds.num_entities, dim)) * 0.1
    rel = rng.standard_normal((ds.num_relations, dim)) * 0.1
    w = None
    if model == "H":
        w = rng.standard_normal((ds.num_relations, dim))
        w /= np.linalg.norm(w, axis=1, keepdims=True)
    eng = Engine(model, dim, ds.num_entities, ds.num_relations)
    eng.upload_params(ent, rel, w)
    filt = np.concatenate([ds.test, ds.train, ds.valid])
    res = eng.evaluate(ds.test, filt)
    m = orc.Model(model, dim, ds.num_entities, ds.num_relations)
    m.set_tables(ent, rel, w)
    exp = m.evaluate(ds.test, filt)
    for k in ("raw_rank", "raw_hits10", "filtered_rank", "filtered_hits10"):
        assert res[k] == pytest.approx(exp[k], abs=1e-12), k
