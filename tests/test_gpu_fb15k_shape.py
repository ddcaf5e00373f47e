"""The GPU configs of BASELINE.json at their own shape (FB15k-shaped synthetic
set: 14,951 entities, 1,345 relations, 483,142 training triples, 100 batches
of 4,831 samples), trained for a few batches against the oracle.

* K2 TransE n=100 bern, K3 TransH n=100 bern, K4 TransR n=50 bern compat with
  the TransE-init (transr/trainer.cpp:88-113: TransE tables written and read
  back as the reference's %.6lf seed files).
* ORDERED (the reference's sample-by-sample order, common/trainer.cpp:69-107)
  against oracle/orc.c, the restatement pinned bit-exact to the compiled
  reference: identical hinge-active counts per batch, loss to 1e-9 relative,
  every table within F64_ATOL_COUPLED.
* PARALLEL (TransR: the default two sub-batches) against its CPU model
  (oracle/parallel.py) on the same glibc sample
  stream: identical active counts, loss 1e-9, tables 1e-9.

At this shape the paths that the 30k-triple sets do not reach switch on: hot
entity segments of hundreds of events (the long / four-wave folds), TransH's
normOrth relation pass behind its 64-flagged-sample gate
(kernels_transh_parallel.hpp kOrthRelMin; K3 starts from 50 trained epochs,
where most batches take it; the engine counts the batches whose relation pass
ran and the test asserts both branches ran),
and TransR's hottest relation with ~900 transRNorm pairs a batch (one
1,536-pair window of the chain kernel).
"""
import numpy as np
import pytest

from gpu_common import F64_ATOL_COUPLED, max_abs
from kb2e_amd import data
from kb2e_amd.engine import Engine
from kb2e_amd.linkpred import transe_seed
from oracle import orc

pytestmark = pytest.mark.gpu

SEED = 7
BATCHES = 100   # the reference's default --batches (common/args.cpp)
RATE = 0.001


@pytest.fixture(scope="module")
def fb():
    return data.synthetic("fb15k", seed=0)


@pytest.fixture(scope="module")
def transr_init(fb):
    """K4's TransE-init: 5 ORDERED TransE epochs at n = 50 unif, round-tripped
    through %.6lf (kb2e_amd.linkpred.transe_seed)."""
    return transe_seed(fb, 50, 5, seed=SEED)


@pytest.fixture(scope="module")
def transh_warm(fb):
    """K3 starts from tables after 50 PARALLEL epochs: from the init tables few
    samples a batch flag w.a > 0.1 (0-16 in the first 30 batches), later
    batches flag more than the gate's 64."""
    eng = Engine("H", 100, fb.num_entities, fb.num_relations, rate=RATE, method=1, batches=BATCHES, seed=SEED + 1,
                 schedule="parallel")
    try:
        eng.upload_triples(fb.train)
        eng.init_params()
        eng.train_batches(50 * BATCHES)
        eng.synchronize()
        return eng.download_params()
    finally:
        eng.close()


CONFIGS = {
    # name: (model, dim, method, compat, batches ORDERED, batches PARALLEL)
    "K2_transe": ("E", 100, 1, True, 20, 20),
    "K3_transh": ("H", 100, 1, True, 20, 30),
    "K4_transr": ("R", 50, 1, True, 12, 8),
}


def _pair(fb, name, schedule, transr_init, transh_warm):
    model, dim, method, compat, _, _ = CONFIGS[name]
    m = orc.Model(model, dim, fb.num_entities, fb.num_relations, rate=RATE, method=method, batches=BATCHES,
                  transr_compat=compat)
    m.set_triples(fb.train)
    orc.srand(SEED)
    m.prep_train()
    eng = Engine(model, dim, fb.num_entities, fb.num_relations, rate=RATE, method=method, batches=BATCHES,
                 seed=SEED, schedule=schedule, transr_compat=compat)
    eng.upload_triples(fb.train)
    e0, r0, w0 = eng.init_params()
    oe, orl, ow = m.tables()
    assert np.array_equal(e0, oe) and np.array_equal(r0, orl)
    if model == "R":
        m.transr_seed(*transr_init)
        eng.transr_seed(*transr_init)
    if model == "H":
        m.set_tables(*transh_warm)
        eng.upload_params(*transh_warm)
    assert m.batch_size() == len(fb.train) // BATCHES
    return m, eng


def _tables_err(eng, m):
    return max(max_abs(x, y) for x, y in zip(eng.download_params(), m.tables()) if x is not None)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fb15k_shape_ordered_vs_oracle(fb, transr_init, transh_warm, name):
    m, eng = _pair(fb, name, "ordered", transr_init, transh_warm)
    nb = CONFIGS[name][4]
    try:
        for b in range(nb):
            lo, ao = m.train_batches(1)
            eng.train_batches(1)
            lg, ag = eng.take_stats()
            assert ag == ao, (b, ag, ao)
            assert abs(lg - lo) <= 1e-9 * max(1.0, abs(lo)), (b, lg, lo)
            if b % 4 == 3 or b == nb - 1:
                err = _tables_err(eng, m)
                assert err < F64_ATOL_COUPLED, (b, err)
        if CONFIGS[name][0] == "R":
            ga, gb = eng.transr_work()
            oa, ob = m.transr_work()
            assert max(max_abs(ga, oa), max_abs(gb, ob)) < 1e-6 * max(1.0, np.abs(oa).max())
    finally:
        eng.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fb15k_shape_parallel_vs_model(fb, transr_init, transh_warm, name):
    from oracle.parallel import (ORTH_REL_MIN, transe_parallel_batches, transh_parallel_batches,
                                 transr_parallel_batches)
    model, dim, method, compat, _, nb = CONFIGS[name]
    m, eng = _pair(fb, name, "parallel", transr_init, transh_warm)
    try:
        pe, pr, pw = m.tables()
        B = m.batch_size()
        si, sj, side = m.sample_stream(B * nb)
        state = {"flag_hist": []}
        work = [np.zeros(dim), np.zeros(dim)]
        for b in range(nb):
            sl = slice(b * B, (b + 1) * B)
            args = (fb.train, si[sl], sj[sl], side[sl], B, 1)
            if model == "E":
                lo, ao = transe_parallel_batches(pe, pr, *args, rate=RATE)
            elif model == "H":
                lo, ao = transh_parallel_batches(pe, pr, pw, *args, rate=RATE, state=state, orth_rel_min=ORTH_REL_MIN)
            else:
                lo, ao = transr_parallel_batches(pe, pr, pw, *args, rate=RATE, l1=True, compat=compat, work=work,
                                                 St=8, cons="chunk1", sub=eng.cfg.sub_batches)  # (the default)
            eng.train_batches(1)
            lg, ag = eng.take_stats()
            assert ag == ao, (b, ag, ao)
            assert abs(lg - lo) <= 1e-9 * max(1.0, abs(lo)), (b, lg, lo)
            if b % 4 == 3 or b == nb - 1:
                got = eng.download_params()
                errs = [max_abs(x, y) for x, y in zip(got, (pe, pr, pw)) if y is not None]
                assert max(errs) < 1e-9, (b, errs)
        if model == "H":
            # the engine's gate on the previous batch's normOrth work took both passes:
            # batch 0 (no work before it) the one-wave pass alone, most later batches the
            # relation pass too -- counted on the device by the relation-pass kernel
            ran = eng.counter("transh_orth_rel_batches")
            assert nb // 3 <= ran <= nb - 1, (ran, nb)
    finally:
        eng.close()
