"""TransR on the GPU (relation-owner dataflow, matrices in LDS) vs the reference.

Parity bar: FP64 engine within 1e-11 (golden runs: 2 epochs of the tiny set)
or 1e-9 (multi-epoch coupled oracle runs, see gpu_common.F64_ATOL_COUPLED) of
the FP64 reference tables -- entities, relations and every relation matrix --
with identical hinge-active counts.  Both the reference's accumulating energy
(compat, transr/transr.cpp:20-25) and the zeroed energy (fixed) are covered;
transRNorm (transr/trainer.cpp:35-64) must iterate in the runs being matched.
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


@pytest.mark.parametrize("name", ["transr_compat", "transr_fixed"])
def test_golden_training_run_fp64(name):
    eng, run, ds, _ = golden_engine(name)
    d = os.path.join(GOLDEN, name)
    e, r, w = eng.download_params()
    assert np.array_equal(w, np.load(os.path.join(d, "init_w.npy")))
    losses = np.load(os.path.join(d, "epoch_loss.npy"))
    actives = np.load(os.path.join(d, "epoch_active.npy"))
    for ep in range(run["flags"]["epochs"]):
        loss, act = eng.train_epoch()
        assert act == actives[ep], (ep, act, actives[ep])
        assert abs(loss - losses[ep]) <= 1e-9 * max(1.0, abs(losses[ep])), (loss, losses[ep])
        e, r, w = eng.download_params()
        err = max(max_abs(e, np.load(os.path.join(d, f"epoch{ep}_ent.npy"))),
                  max_abs(r, np.load(os.path.join(d, f"epoch{ep}_rel.npy"))),
                  max_abs(w, np.load(os.path.join(d, f"epoch{ep}_w.npy"))))
        assert err < F64_ATOL, (ep, err)
    if name == "transr_compat":
        hw, tw = eng.transr_work()
        assert max_abs(hw, np.load(os.path.join(d, "epoch1_hwork.npy"))) < 1e-6 * max(1, np.abs(hw).max())
    after = np.load(os.path.join(d, "rand_after.npy"))
    assert [eng.rng_next() for _ in range(after.size)] == after.tolist()


@pytest.mark.parametrize("compat,dim,shape", [(False, 32, "small"), (True, 20, "small"), (False, 50, "small"),
                                               (False, 65, "tiny"), (True, 96, "tiny"), (False, 100, "tiny"),
                                               (True, 100, "tiny"), (False, 128, "tiny"), (True, 160, "tiny"),
                                               (False, 260, "tiny")])
def test_oracle_parity_with_transrnorm(compat, dim, shape):
    """dim <= 64: Mr rows in registers (transr_owner_reg_kernel); above: the
    LDS-resident generic owner (engine_relowner.inc), K5's n = 100 included;
    above 137 the same owner on the matrix in L2 (the reference's --size has no
    limit, common/args.cpp:71-74), 260 with four element chunks a lane."""
    ds = data.synthetic(shape, seed=4)
    kw = dict(rate=0.005 if shape == "small" else 0.01, margin=1.0, method=1, batches=25 if shape == "small" else 10)
    m = oracle_model("R", ds, dim, transr_compat=compat, **kw)
    orc.srand(8)
    m.prep_train()
    eng = Engine("R", dim, ds.num_entities, ds.num_relations, seed=8, transr_compat=compat, **kw)
    eng.upload_triples(ds.train)
    e0, r0, w0 = eng.init_params()
    # seed with the init draws themselves (the oracle's transr_seed applies the same unit norm)
    m.transr_seed(e0, r0)
    eng.transr_seed(e0, r0)
    ge, gr, gw = eng.download_params()
    oe, orl, ow = m.tables()
    assert np.array_equal(ge, oe) and np.array_equal(gr, orl) and np.array_equal(gw, ow)
    L = orc.lib()
    before = [L.orc_site_iterations(s) for s in range(3)]
    for ep in range(2):
        lo, ao = m.train_epoch()
        lg, ag = eng.train_epoch()
        assert ag == ao, (ep, ag, ao)
        assert abs(lg - lo) <= 1e-8 * max(1.0, abs(lo)), (lg, lo)
        ge, gr, gw = eng.download_params()
        oe, orl, ow = m.tables()
        err = max(max_abs(ge, oe), max_abs(gr, orl), max_abs(gw, ow))
        assert err < F64_ATOL_COUPLED, (ep, err)
    assert sum(L.orc_site_iterations(s) - before[s] for s in range(3)) > 0


def test_fp32_statistically_close():
    """See test_gpu_transh.test_fp32_statistically_close for why FP32 is statistical."""
    ds = data.synthetic("small", seed=6)
    kw = dict(rate=0.005, batches=25, transr_compat=False)
    m = oracle_model("R", ds, 32, **kw)
    orc.srand(3)
    m.prep_train()
    eng = Engine("R", 32, ds.num_entities, ds.num_relations, seed=3, precision=32, **kw)
    eng.upload_triples(ds.train)
    e0, r0, _ = eng.init_params()
    m.transr_seed(e0, r0)
    eng.transr_seed(e0, r0)
    lo, ao = m.train_epoch()
    lg, ag = eng.train_epoch()
    assert abs(lg - lo) < 0.01 * lo and abs(ag - ao) < 0.01 * ao
    ge, gr, gw = eng.download_params()
    oe, orl, ow = m.tables()
    assert np.median(np.abs(ge - oe)) < 1e-3 and np.median(np.abs(gw - ow)) < 1e-3


def test_oracle_parity_dim512():
    """The widest context (dim 512, the engine's cap): the L2-resident owner with
    eight element chunks a lane, against the oracle over two epochs with
    transRNorm iterating (FP64 at 512 was untested)."""
    ds = data.synthetic("tiny", seed=4)
    kw = dict(rate=0.01, margin=1.0, method=1, batches=10)
    m = oracle_model("R", ds, 512, transr_compat=False, **kw)
    orc.srand(8)
    m.prep_train()
    eng = Engine("R", 512, ds.num_entities, ds.num_relations, seed=8, transr_compat=False, **kw)
    eng.upload_triples(ds.train)
    e0, r0, _ = eng.init_params()
    m.transr_seed(e0, r0)
    eng.transr_seed(e0, r0)
    L = orc.lib()
    before = [L.orc_site_iterations(s) for s in range(3)]
    for ep in range(2):
        lo, ao = m.train_epoch()
        lg, ag = eng.train_epoch()
        assert ag == ao, (ep, ag, ao)
        assert abs(lg - lo) <= 1e-8 * max(1.0, abs(lo)), (lg, lo)
        err = max(max_abs(x, y) for x, y in zip(eng.download_params(), m.tables()))
        assert err < F64_ATOL_COUPLED, (ep, err)
    assert sum(L.orc_site_iterations(s) - before[s] for s in range(3)) > 0


def _fp32_vs_oracle(shape, dim):
    """One FP32 ORDERED epoch against the FP64 oracle: (loss ratio - 1, active
    difference ratio, median |entity diff|, median |matrix diff|)."""
    ds = data.synthetic(shape, seed=6)
    kw = dict(rate=0.005 if shape == "small" else 0.01, batches=25 if shape == "small" else 10, transr_compat=False)
    m = oracle_model("R", ds, dim, **kw)
    orc.srand(3)
    m.prep_train()
    eng = Engine("R", dim, ds.num_entities, ds.num_relations, seed=3, precision=32, **kw)
    eng.upload_triples(ds.train)
    e0, r0, _ = eng.init_params()
    m.transr_seed(e0, r0)
    eng.transr_seed(e0, r0)
    lo, ao = m.train_epoch()
    lg, ag = eng.train_epoch()
    ge, gr, gw = eng.download_params()
    eng.close()
    oe, orl, ow = m.tables()
    return lg / lo - 1, (ag - ao) / ao, float(np.median(np.abs(ge - oe))), float(np.median(np.abs(gw - ow)))


def test_fp32_wide_statistically_close():
    """FP32 ORDERED on both sides of the owner's FP32 LDS limit (195): dim 190 keeps
    the matrix in LDS, 200 reads it from L2 (the float instantiation ADVICE r5
    found untested), and 512 is the widest context.  FP32 hinge decisions flip at
    the margin and transRNorm amplifies the flips, so the drift from the FP64
    oracle grows with the dim (diagnostic tools/diag/fp32_wide_probe.py: median
    entity drift 5.5e-3 at 120, 7.7e-3 at 190, 9.4e-3 at 200 after one epoch) and
    the bar is statistical: loss and active count within 1 %, and the L2 form's
    drift no larger than the LDS form's next to it (2x), not an absolute ulp bound."""
    d190 = _fp32_vs_oracle("small", 190)
    d200 = _fp32_vs_oracle("small", 200)
    d512 = _fp32_vs_oracle("tiny", 512)
    for d in (d190, d200, d512):
        assert abs(d[0]) < 0.01 and abs(d[1]) < 0.01, (d190, d200, d512)
    assert d200[2] < 2 * d190[2] and d200[3] < 2 * d190[3], (d190, d200)
    assert d512[2] < 1e-2 and d512[3] < 5e-3, d512
