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
