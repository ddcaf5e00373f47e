"""TransH on the GPU (relation-owner dataflow) vs the reference and the oracle.

Parity bar: FP64 engine within 1e-11 absolute of the FP64 reference tables
(entities, relations, normals) after every epoch, identical hinge-active counts
and RNG consumption; the coupling loop (norm(a, b, rate) iterating,
common/utils.cpp:79-111) must actually fire in the oracle run being matched.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_common import F64_ATOL, F64_ATOL_COUPLED, golden_engine, max_abs, oracle_model
from kb2e_amd import data
from kb2e_amd.engine import Engine
from oracle import orc

pytestmark = pytest.mark.gpu


def test_golden_training_run_fp64():
    eng, run, ds, (ent, rel, w) = golden_engine("transh_bern")
    d = os.path.join(GOLDEN, "transh_bern")
    assert np.array_equal(w, np.load(os.path.join(d, "init_w.npy")))
    losses = np.load(os.path.join(d, "epoch_loss.npy"))
    actives = np.load(os.path.join(d, "epoch_active.npy"))
    for ep in range(run["flags"]["epochs"]):
        loss, act = eng.train_epoch()
        assert act == actives[ep]
        assert abs(loss - losses[ep]) <= 1e-9 * max(1.0, abs(losses[ep]))
        e, r, ww = eng.download_params()
        assert max_abs(e, np.load(os.path.join(d, f"epoch{ep}_ent.npy"))) < F64_ATOL
        assert max_abs(r, np.load(os.path.join(d, f"epoch{ep}_rel.npy"))) < F64_ATOL
        assert max_abs(ww, np.load(os.path.join(d, f"epoch{ep}_w.npy"))) < F64_ATOL
    after = np.load(os.path.join(d, "rand_after.npy"))
    assert [eng.rng_next() for _ in range(after.size)] == after.tolist()


# (33, 0.02) diverges from epoch 1 on by amplified rounding noise (see
# test_high_rate_divergence_is_rounding_noise), so it is matched for one epoch.
@pytest.mark.parametrize("dim,rate,epochs", [(50, 0.01, 3), (100, 0.01, 2), (33, 0.02, 1)])
def test_oracle_parity_with_coupling(dim, rate, epochs):
    ds = data.synthetic("small", seed=1)
    m = oracle_model("H", ds, dim, rate=rate, margin=1.0, method=1, batches=20)
    orc.srand(5)
    m.prep_train()
    eng = Engine("H", dim, ds.num_entities, ds.num_relations, rate=rate, margin=1.0, method=1, batches=20, seed=5)
    eng.upload_triples(ds.train)
    e0, r0, w0 = eng.init_params()
    oe, orl, ow = m.tables()
    assert np.array_equal(e0, oe) and np.array_equal(r0, orl) and np.array_equal(w0, ow)
    L = orc.lib()
    before = [L.orc_site_iterations(s) for s in range(3)]
    for ep in range(epochs):
        lo, ao = m.train_epoch()
        lg, ag = eng.train_epoch()
        ge, gr, gw = eng.download_params()
        oe, orl, ow = m.tables()
        err = max(max_abs(ge, oe), max_abs(gr, orl), max_abs(gw, ow))
        assert ag == ao, (ep, ag, ao)
        assert abs(lg - lo) <= 1e-9 * max(1.0, abs(lo)), (ep, lg, lo)
        assert err < F64_ATOL_COUPLED, (ep, err)
    fired = sum(L.orc_site_iterations(s) - before[s] for s in range(3))
    assert fired > 0, "the coupling loop never iterated: test does not exercise the dataflow"


def test_fp32_statistically_close():
    """FP32 hinge decisions flip against FP64 at the margin and every flip moves
    rows by O(lr) (SURVEY.md 0.8 saw the same for an all-float CPU build), so the
    FP32 bar is statistical: epoch loss and active count within 1%, median row
    difference below 1e-3."""
    ds = data.synthetic("small", seed=3)
    m = oracle_model("H", ds, 50, rate=0.01, batches=20)
    orc.srand(2)
    m.prep_train()
    eng = Engine("H", 50, ds.num_entities, ds.num_relations, rate=0.01, batches=20, seed=2, precision=32)
    eng.upload_triples(ds.train)
    eng.init_params()
    lo, ao = m.train_epoch()
    lg, ag = eng.train_epoch()
    assert abs(lg - lo) < 0.01 * lo and abs(ag - ao) < 0.01 * ao
    ge, gr, gw = eng.download_params()
    oe, orl, ow = m.tables()
    assert np.median(np.abs(ge - oe)) < 1e-3 and np.median(np.abs(gw - ow)) < 1e-3


def test_high_rate_divergence_is_rounding_noise():
    """At lr = 0.05 the orthogonality loop iterates ~900 times per batch and the
    dynamics amplify rounding differences (~4x per batch).  Parity is then
    checked where it is meaningful: ulp-level after the first batches (an
    ordering error would appear at once at the O(lr) scale), identical hinge
    decisions for the whole epoch, epoch loss within 1e-7."""
    ds = data.synthetic("small", seed=1)
    eng = Engine("H", 33, ds.num_entities, ds.num_relations, rate=0.05, batches=20, seed=5)
    eng.upload_triples(ds.train)
    eng.init_params()
    m = oracle_model("H", ds, 33, rate=0.05, batches=20)
    orc.srand(5)
    m.prep_train()
    tot_o = tot_g = 0.0
    for b in range(20):
        lo, ao = m.train_batches(1)
        eng.train_batches(1)
        lg, ag = eng.take_stats()
        assert ag == ao, (b, ag, ao)
        tot_o += lo
        tot_g += lg
        if b < 3:
            ge, gr, gw = eng.download_params()
            oe, orl, ow = m.tables()
            assert max(max_abs(ge, oe), max_abs(gr, orl), max_abs(gw, ow)) < 1e-13, b
    assert abs(tot_g - tot_o) < 1e-7 * tot_o
