"""K5 (BASELINE configs[4]) at its real size on one GPU:
TransR n = 100, 1M entities, 10k relations, 16M training triples, 100 batches
of 160,000 samples, PARALLEL schedule, FP64.

The oracle cannot train at this size in test time (the reference's ORDERED
loop takes hours per epoch here), so the full-size run is pinned by properties
that do not depend on size (transr/trainer.cpp:144-188, common/trainer.cpp:
69-107, 129-147):

* the device sample stream equals the host glibc restatement (oracle/orc.c)
  for the first two batches;
* the hinge decisions and the batch loss equal a numpy evaluation of the
  reference's energy (transr/transr.cpp:13-38) on the tables the batch
  started from -- batch 0 on the uploaded tables, batch 1 on the tables batch 0
  left (the PARALLEL schedule takes every decision of a batch on its snapshot);
* every row stays finite; relation rows are unit (common::norm(.., false));
  entity rows and the rows of every Mr have norm <= 1 up to transRNorm's
  O(lr) moves (it moves both to shrink |W^T a|; the relation's pairs are taken
  one after another against the matrix the earlier ones left,
  kernels_transr_chainw.hpp -- the Jacobi sum of a hot relation's ~10^4
  corrections against one W' pushed Mr rows to norm 2.4 here);
* rows no active sample touches are bit-identical to what the batch started
  from (entities, relations and whole matrices).

Tables: numpy-drawn unit rows and identity Mr (bench.py --config transr_k5:
the reference's host randn init takes minutes at this size).
"""
import numpy as np
import pytest

from kb2e_amd import data
from kb2e_amd.engine import Engine
from oracle import orc

pytestmark = pytest.mark.gpu

N = 100
BATCHES = 100
SEED = 7
NORM_TOL = 1e-9
CONS_TOL = 1e-2  # transRNorm's moves: lr times a few rounds' gradients


@pytest.fixture(scope="module")
def k5():
    ds = data.synthetic("k5", seed=1)
    rng = np.random.default_rng(7)
    ent = rng.uniform(-1, 1, (ds.num_entities, N))
    ent /= np.linalg.norm(ent, axis=1, keepdims=True)
    rel = rng.uniform(-1, 1, (ds.num_relations, N))
    rel /= np.linalg.norm(rel, axis=1, keepdims=True)
    m = orc.Model("R", N, ds.num_entities, ds.num_relations, rate=0.001, method=1, distance=0, batches=BATCHES)
    m.set_triples(ds.train)
    orc.srand(SEED)
    B = m.batch_size()
    stream = m.sample_stream(2 * B)
    del m
    return ds, ent, rel, stream, B


def _batch_ids(ds, stream, b, B):
    si, sj, side = (x[b * B:(b + 1) * B] for x in stream)
    tr = ds.train[si]
    h, t, r = tr[:, 0], tr[:, 1], tr[:, 2]
    side = side.astype(bool)
    nh = np.where(side, h, sj)  # side 1: the tail is corrupted
    nt = np.where(side, sj, t)
    return h, t, r, nh, nt


def _project(ent_rows, w, r):
    """(e W_r)_i = sum_j W_r[j][i] e_j per sample, grouped by relation."""
    out = np.empty_like(ent_rows)
    order = np.argsort(r, kind="stable")
    rs = r[order]
    cuts = np.flatnonzero(np.diff(rs)) + 1
    for grp in np.split(order, cuts):
        out[grp] = ent_rows[grp] @ w[r[grp[0]]]
    return out


def _fixed_hinge(ent, rel, w, ids):
    h, t, r, nh, nt = ids
    if w is None:  # identity matrices
        ph, pt, pnh, pnt = ent[h], ent[t], ent[nh], ent[nt]
    else:
        ph, pt, pnh, pnt = (_project(ent[x], w, r) for x in (h, t, nh, nt))
    e1 = np.abs(pt - ph - rel[r]).sum(1)
    e2 = np.abs(pnt - pnh - rel[r]).sum(1)
    act = e1 + 1.0 > e2
    return act, float(np.sum((1.0 + e1 - e2)[act]))


def _check_rows(e0, r0, w0, e1, r1, w1, ids, act, ne, nr):
    h, t, r, nh, nt = ids
    assert np.isfinite(e1).all() and np.isfinite(r1).all() and np.isfinite(w1).all()
    assert np.abs(np.linalg.norm(r1, axis=1) - 1).max() < NORM_TOL
    assert np.linalg.norm(e1, axis=1).max() < 1 + CONS_TOL
    assert np.linalg.norm(w1, axis=2).max() < 1 + CONS_TOL
    touched_e = np.zeros(ne, bool)
    for x in (h, t, nh, nt):
        touched_e[x[act]] = True
    # transRNorm(entityVec_next_[relation], ...) (transr/trainer.cpp:187): the
    # reference constrains the ENTITY row whose id is the relation's id
    touched_e[r[act]] = True
    touched_r = np.zeros(nr, bool)
    touched_r[r[act]] = True
    assert np.array_equal(e1[~touched_e], e0[~touched_e])
    assert np.array_equal(r1[~touched_r], r0[~touched_r])
    assert np.array_equal(w1[~touched_r], w0[~touched_r])
    # the active samples' rows did move
    assert (np.abs(r1[touched_r] - r0[touched_r]).max(1) > 0).all()
    assert (np.abs(w1[touched_r] - w0[touched_r]).reshape(touched_r.sum(), -1).max(1) > 0).all()


def test_k5_full_size_fixed_energy(k5):
    """Two PARALLEL batches at full size, fixed energy: stream, hinge
    decisions, loss and row properties against numpy."""
    ds, ent, rel, stream, B = k5
    eng = Engine("R", N, ds.num_entities, ds.num_relations, rate=0.001, method=1, distance=0, batches=BATCHES,
                 seed=SEED, schedule="parallel", transr_compat=False)
    try:
        eng.upload_triples(ds.train)
        w = np.ascontiguousarray(np.broadcast_to(np.eye(N), (ds.num_relations, N, N)))
        eng.upload_params(ent, rel, w)
        prev = (ent, rel, w)
        for b in range(2):
            eng.train_batches(1)
            eng.synchronize()
            if b == 0:  # the device stream of the epoch in progress vs the host restatement
                gi, gj, gs = eng.sample_stream(2 * B)
                assert np.array_equal(gi, stream[0]) and np.array_equal(gj, stream[1])
                assert np.array_equal(gs, stream[2])
            loss, active = eng.take_stats()
            ids = _batch_ids(ds, stream, b, B)
            act, ref_loss = _fixed_hinge(prev[0], prev[1], None if b == 0 else prev[2], ids)
            assert active == int(act.sum()), (b, active, int(act.sum()))
            assert abs(loss - ref_loss) <= 1e-9 * abs(ref_loss), (b, loss, ref_loss)
            assert 0.05 * B < active < B
            cur = eng.download_params()
            _check_rows(*prev, *cur, ids, act, ds.num_entities, ds.num_relations)
            prev = cur
    finally:
        eng.close()


def test_k5_full_size_compat_energy(k5):
    """The bench's form (compat energy, the reference's accumulating work
    vectors): batch 0's hinge decisions against a numpy prefix sum of the
    projected rows over the batch's 2B energy calls (in call order: each
    sample's positive triple, then its corrupted one), and the row properties."""
    ds, ent, rel, stream, B = k5
    eng = Engine("R", N, ds.num_entities, ds.num_relations, rate=0.001, method=1, distance=0, batches=BATCHES,
                 seed=SEED, schedule="parallel", transr_compat=True)
    try:
        eng.upload_triples(ds.train)
        w = np.ascontiguousarray(np.broadcast_to(np.eye(N), (ds.num_relations, N, N)))
        eng.upload_params(ent, rel, w)
        hw0, tw0 = eng.transr_work()
        eng.train_batches(1)
        eng.synchronize()
        loss, active = eng.take_stats()
        ids = _batch_ids(ds, stream, 0, B)
        h, t, r, nh, nt = ids
        calls_h = np.empty((2 * B, N))
        calls_t = np.empty((2 * B, N))
        calls_h[0::2], calls_h[1::2] = ent[h], ent[nh]  # identity Mr: the projection is the row
        calls_t[0::2], calls_t[1::2] = ent[t], ent[nt]
        hv = np.cumsum(calls_h, axis=0) + hw0
        tv = np.cumsum(calls_t, axis=0) + tw0
        rr = np.repeat(rel[r], 2, axis=0)
        e = np.abs(tv - hv - rr).sum(1)
        e1, e2 = e[0::2], e[1::2]
        act = e1 + 1.0 > e2
        # the work vectors grow to |v| ~ 1e2 over the batch: the scan's summation
        # order moves energies by ~1e-11, so a decision may flip only at a near tie
        near = np.abs(e1 + 1.0 - e2) < 1e-8
        assert abs(active - int(act.sum())) <= int(near.sum()), (active, int(act.sum()), int(near.sum()))
        ref_loss = float(np.sum((1.0 + e1 - e2)[act]))
        assert abs(loss - ref_loss) <= 1e-8 * abs(ref_loss) + near.sum() * 1e-8, (loss, ref_loss)
        hw1, tw1 = eng.transr_work()
        assert np.abs(hw1 - hv[-1]).max() < 1e-8 * max(1.0, np.abs(hv[-1]).max())
        assert np.abs(tw1 - tv[-1]).max() < 1e-8 * max(1.0, np.abs(tv[-1]).max())
        cur = eng.download_params()
        _check_rows(ent, rel, w, *cur, ids, act, ds.num_entities, ds.num_relations)
    finally:
        eng.close()


@pytest.mark.parametrize("chain", ["lockstep"])
def test_k5_chain_kernels_agree(k5, chain, monkeypatch):
    """One full-size batch (compat energy) through each transRNorm chain kernel
    at n = 100 against the default one: the same pairs in the same order
    against the same matrices, so the tables agree to rounding (the kernels sum
    V = p K0 and the projections in different orders)."""
    ds, ent, rel, stream, B = k5
    w = np.ascontiguousarray(np.broadcast_to(np.eye(N), (ds.num_relations, N, N)))
    out = {}
    for name in ("default", chain):
        if name == "default":
            monkeypatch.delenv("KB2E_RPAR_CHAIN", raising=False)
        else:
            monkeypatch.setenv("KB2E_RPAR_CHAIN", name)
        eng = Engine("R", N, ds.num_entities, ds.num_relations, rate=0.001, method=1, distance=0,
                     batches=BATCHES, seed=SEED, schedule="parallel", transr_compat=True)
        try:
            eng.upload_triples(ds.train)
            eng.upload_params(ent, rel, w)
            eng.train_batches(1)
            eng.synchronize()
            out[name] = (eng.take_stats(), eng.download_params())
        finally:
            eng.close()
    (l0, a0), p0 = out["default"]
    (l1, a1), p1 = out[chain]
    assert a0 == a1 and l0 == l1  # the hinge pass comes before the chain
    for x0, x1 in zip(p0, p1):
        assert np.abs(x1 - x0).max() < 1e-11
    # the chain moved the hot relations' matrices (the comparison is not vacuous)
    assert np.abs(p0[2] - w).max() > 1e-6
