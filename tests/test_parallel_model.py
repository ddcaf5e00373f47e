"""The CPU model of the PARALLEL schedule (oracle/parallel.py) against the
reference restatement (oracle/orc.c), CPU only.

With every row kept strictly inside the unit ball, common::norm never rescales
(common/utils.cpp:70-77), so the reference's sequential updates and the summed
deltas of the PARALLEL schedule must agree up to the order of the additions:
this pins the model's energies, hinge decisions, directions and signs to the
reference's.  Bar: 1e-12 absolute, identical loss and active counts.
"""
import numpy as np
import pytest

from kb2e_amd import data
from oracle import orc
from oracle.parallel import transe_parallel_batches, transr_parallel_batches


@pytest.mark.parametrize("distance", [0, 1])
def test_transe_parallel_equals_reference_without_norms(distance):
    ds = data.synthetic("tiny", seed=3)
    dim, rate, batches = 20, 0.0005, 10
    m = orc.Model("E", dim, ds.num_entities, ds.num_relations, rate=rate, batches=batches, distance=distance)
    m.set_triples(ds.train)
    orc.srand(5)
    m.prep_train()
    e0, r0, _ = m.tables()
    # shrink every row to length <= 0.3: no norm can fire within 3 batches
    e0 = e0 * (0.3 / np.maximum(np.linalg.norm(e0, axis=1, keepdims=True), 1e-300))
    r0 = r0 * (0.3 / np.maximum(np.linalg.norm(r0, axis=1, keepdims=True), 1e-300))
    B = m.batch_size()
    si, sj, side = m.sample_stream(3 * B)
    m.set_tables(e0, r0)
    lo, ao = m.train_replay(si, sj, side)
    oe, orl, _ = m.tables()
    pe, pr = e0.copy(), r0.copy()
    lp, ap = transe_parallel_batches(pe, pr, ds.train, si, sj, side, B, 3, rate=rate, l1=distance == 0)
    assert ap == ao and ao > 0
    assert abs(lp - lo) <= 1e-9 * max(1.0, lo)
    assert np.abs(pe - oe).max() < 1e-12 and np.abs(pr - orl).max() < 1e-12
    # and the rows really moved
    assert np.abs(pe - e0).max() > 10 * rate


def _transr_sequential(E, R, W, triples, si, sj, side, rate, margin=1.0, l1=True, constraint=True):
    """One TransR batch exactly as the reference runs it (transr/trainer.cpp:
    35-64, 144-188; common/trainer.cpp:130-149), in numpy, with the fixed
    (zeroed) energy.  `constraint=False` drops transRNorm."""
    En, Rn, Wn = E.copy(), R.copy(), W.copy()
    n = E.shape[1]
    for k in range(len(si)):
        h, t, r = triples[si[k]]
        nh, nt = (h, sj[k]) if side[k] else (sj[k], t)

        def energy(a, b):
            d = W[r].T @ E[b] - W[r].T @ E[a] - R[r]
            return np.abs(d).sum() if l1 else (d * d).sum()

        if not energy(h, t) + margin > energy(nh, nt):
            continue
        for (a, b, beta) in ((h, t, -1.0), (nh, nt, 1.0)):
            for i in range(n):
                x = 2.0 * (W[r][:, i] @ E[b] - W[r][:, i] @ E[a] - R[r][i])
                if l1:
                    x = 1.0 if x > 0 else -1.0
                Wn[r][:, i] -= beta * rate * x * (E[a] - E[b])
                En[a] -= beta * rate * x * W[r][:, i]
                En[b] += beta * rate * x * W[r][:, i]
                Rn[r][i] -= beta * rate * x
            Rn[r] /= np.sqrt(Rn[r] @ Rn[r])
            En[a] /= np.sqrt(En[a] @ En[a])
            En[b] /= np.sqrt(En[b] @ En[b])
            Wn[r] /= np.sqrt((Wn[r] ** 2).sum(1, keepdims=True))
            if not constraint:
                continue
            for e in (a, b, r):
                while True:
                    p = Wn[r].T @ En[e]
                    if p @ p <= 1:
                        break
                    for i in range(n):
                        tmp = 2.0 * (Wn[r][:, i] @ En[e])
                        for j in range(n):
                            Wn[r][j, i] -= rate * tmp * En[e][j]
                            En[e][j] -= rate * tmp * Wn[r][j, i]
    return En, Rn, Wn


@pytest.mark.parametrize("distance", [0, 1])
def test_transr_parallel_first_order_equals_reference(distance):
    """One batch at a tiny learning rate.  (1) The numpy restatement of the
    reference batch equals the C oracle (which is pinned to the reference).
    (2) Without transRNorm, the PARALLEL schedule's change of every table equals
    the reference's to first order in lr (they differ only in where the norms
    fall, O(lr^2)), with identical hinge decisions and loss.  (transRNorm is a
    threshold loop whose fixes interact through W at the same order as the
    violations: its Jacobi form is a statistical relaxation, DESIGN.md.)"""
    ds = data.synthetic("tiny", seed=6)
    dim, rate, batches = 16, 1e-6, 30
    m = orc.Model("R", dim, ds.num_entities, ds.num_relations, rate=rate, batches=batches, distance=distance,
                  transr_compat=False)
    m.set_triples(ds.train)
    orc.srand(11)
    m.prep_train()
    e0, r0, w0 = m.tables()
    rng = np.random.default_rng(0)
    e0 = rng.standard_normal(e0.shape)
    r0 = rng.standard_normal(r0.shape)
    e0 /= np.linalg.norm(e0, axis=1, keepdims=True)
    r0 /= np.linalg.norm(r0, axis=1, keepdims=True)
    B = m.batch_size()
    si, sj, side = m.sample_stream(B)
    m.set_tables(e0, r0, w0)
    lo, ao = m.train_replay(si, sj, side)
    oe, orl, ow = m.tables()
    se, sr, sw = _transr_sequential(e0, r0, w0, ds.train, si, sj, side, rate, l1=distance == 0)
    assert np.abs(se - oe).max() < 1e-13 and np.abs(sr - orl).max() < 1e-13 and np.abs(sw - ow).max() < 1e-13
    qe, qr, qw = _transr_sequential(e0, r0, w0, ds.train, si, sj, side, rate, l1=distance == 0, constraint=False)
    pe, pr, pw = e0.copy(), r0.copy(), w0.copy()
    lp, ap = transr_parallel_batches(pe, pr, pw, ds.train, si, sj, side, B, 1, rate=rate, l1=distance == 0,
                                     constraint=False)
    assert ap == ao and ao > 0
    assert abs(lp - lo) <= 1e-9 * max(1.0, lo)
    for got, ref, start in ((pe, qe, e0), (pr, qr, r0), (pw, qw, w0)):
        d_ref = np.abs(ref - start).max()
        assert d_ref > 0
        assert np.abs((got - start) - (ref - start)).max() <= 1e-3 * d_ref


def test_transr_constraint_pairs_once_per_relation():
    """transRNorm pairs of the PARALLEL schedule: each (relation, entity) of the
    batch's active updates is constrained once, whatever the tiling (St), and
    (entity[r], r) is skipped when an update of r already holds entity r."""
    from oracle.parallel import transr_constraint

    rng = np.random.default_rng(4)
    n, rate = 4, 0.01
    ent0 = rng.standard_normal((5, n))
    ent0 *= 1.5 / np.linalg.norm(ent0, axis=1, keepdims=True)  # |W^T a| > 1 with W = I: every pair violates
    W0 = np.stack([np.eye(n), np.eye(n)])
    h, t = np.array([0, 0]), np.array([1, 2])
    nh, nt = np.array([0, 3]), np.array([4, 2])
    r, act = np.array([0, 0]), np.array([True, True])

    def single(a0, Wm):  # one pair, as transr_constraint's loop
        G, s0, p = np.zeros(n), a0 @ a0, Wm.T @ a0
        while p @ p > 1.0:
            G += 2.0 * p
            p = p - 2.0 * rate * (Wm.T @ (Wm @ p)) - 2.0 * rate * s0 * p
        return -rate * (Wm @ G), np.outer(-rate * a0, G)

    want_e, want_w = ent0.copy(), W0.copy()
    for e in (0, 1, 4, 2, 3):  # first occurrences in (sample, update, role) order; entity 0 = relation 0's pair
        da, dw = single(ent0[e], W0[0])
        want_e[e] += da
        want_w[0] += dw
    for St in (1, 2, 8):
        ent, W = ent0.copy(), W0.copy()
        transr_constraint(ent, W, h, t, nh, nt, r, act, rate, St)
        assert np.abs(ent - want_e).max() < 1e-15 and np.abs(W - want_w).max() < 1e-15


def test_transh_orth_order_two_passes():
    """PARALLEL TransH normOrth order (oracle/parallel.py transh_orth_order, the
    GPU's transh_orth_rel_kernel + transh_orth_fix_kernel): every flagged pair
    once; with one relation it is the reference's sample order; an entity row
    flagged under two relations waits for the second pass."""
    from oracle.parallel import transh_orth_order
    rng = np.random.default_rng(3)
    n_s = 200
    r = rng.integers(0, 5, n_s)
    h, t = rng.integers(0, 40, n_s), rng.integers(0, 40, n_s)
    nh, nt = rng.integers(0, 40, n_s), rng.integers(0, 40, n_s)
    ids = {k: (r[k], h[k], t[k], None, nh[k], nt[k]) for k in range(n_s)}
    flags = [[q for q in (0, 1, 2, 4, 5) if rng.random() < 0.3] for _ in range(n_s)]
    order = transh_orth_order(list(range(n_s)), flags, ids, r)
    want = [(k, q) for k in range(n_s) for q in flags[k]]
    assert sorted(order) == sorted(want) and len(order) == len(want)
    rels = {}
    for k in range(n_s):
        for q in flags[k]:
            if q:
                rels.setdefault(int(ids[k][q]), set()).add(int(r[k]))
    shared = [(k, q) for k, q in order if q and len(rels[int(ids[k][q])]) > 1]
    own = [(k, q) for k, q in order if not (q and len(rels[int(ids[k][q])]) > 1)]
    assert order == own + shared  # each pass in sample order, the shared rows last
    assert own == sorted(own) and shared == sorted(shared)
    r1 = np.zeros(n_s, dtype=int)  # one relation: nothing is shared, the reference's order
    assert transh_orth_order(list(range(n_s)), flags, ids, r1) == want
