"""Batch-by-batch comparison of the PARALLEL TransR engine with its numpy model
(tests/ infrastructure for debugging; GPU box).  ISO=1: apply the numpy
transRNorm step to the engine's own post-gradient state (an engine built with
KB2E_RPAR_NOC=1) and compare with the full engine -- isolates that kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402
from oracle import orc  # noqa: E402
from oracle.parallel import transr_constraint, transr_parallel_batches  # noqa: E402

St = int(os.environ.get("KB2E_RPAR_ST", "8"))
constraint = os.environ.get("NOC", "0") != "1"
iso = os.environ.get("ISO", "0") == "1"
ds = data.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "tiny"))
dim, rate, batches, seed = 20, 0.01, 10, 3


def make_engine(noc):
    os.environ["KB2E_RPAR_NOC"] = "1" if noc else "0"
    eng = Engine("R", dim, ds.num_entities, ds.num_relations, rate=rate, batches=batches, seed=seed,
                 schedule="parallel", transr_compat=False)
    eng.upload_triples(ds.train)
    e0, r0, _ = eng.init_params()
    eng.transr_seed(e0, r0)
    return eng


m = orc.Model("R", dim, ds.num_entities, ds.num_relations, rate=rate, batches=batches, transr_compat=False)
m.set_triples(ds.train)
orc.srand(seed)
m.prep_train()
pe, pr, pw = m.tables()
pe = pe / np.linalg.norm(pe, axis=1, keepdims=True)
B = m.batch_size()
si, sj, side = m.sample_stream(B * batches)
if iso:
    A = make_engine(True)
    A.train_batches(1)
    A.synchronize()
    ge0, gr0, gw0 = A.download_params()
    Bf = make_engine(False)
    Bf.train_batches(1)
    ge1, gr1, gw1 = Bf.download_params()
    print("post-gradient equal rel", np.abs(gr0 - gr1).max())
    h_all, t_all, r_all = ds.train[:, 0], ds.train[:, 1], ds.train[:, 2]
    i, j, sd = si[:B], sj[:B], side[:B].astype(bool)
    h, t, r = h_all[i], t_all[i], r_all[i]
    nh, nt = np.where(sd, h, j), np.where(sd, j, t)
    act = np.zeros(B, bool)
    qe, qr, qw = pe.copy(), pr.copy(), pw.copy()
    transr_parallel_batches(qe, qr, qw, ds.train, si[:B], sj[:B], side[:B], B, 1, rate=rate, St=St, constraint=False)
    print("numpy post-gradient vs engine: ent", np.abs(qe - ge0).max(), "W", np.abs(qw - gw0).max())
    # recover act from the model: recompute energies on the start tables
    Wr = pw[r]
    proj = lambda v: np.einsum("kji,kj->ki", Wr, pe[v])  # noqa: E731
    ph, pt, pnh, pnt = proj(h), proj(t), proj(nh), proj(nt)
    act = np.abs(pt - ph - pr[r]).sum(1) + 1.0 > np.abs(pnt - pnh - pr[r]).sum(1)
    for kw in ({"dedupe": False}, {"relpair": False}, {"max_iter": 1}, {"St": 1}, {"St": 64}):
        ce, cw = ge0.copy(), gw0.copy()
        kw2 = dict(kw)
        st2 = kw2.pop("St", St)
        transr_constraint(ce, cw, h, t, nh, nt, r, act, rate, st2, **kw2)
        print("variant", kw, "ent", np.abs(ce - ge1).max(), "W", np.abs(cw - gw1).max())
    ce, cw = ge0.copy(), gw0.copy()
    transr_constraint(ce, cw, h, t, nh, nt, r, act, rate, St)
    de, dw = np.abs(ce - ge1), np.abs(cw - gw1)
    print("constraint only: ent", de.max(), "W", dw.max(), "moved ent", np.abs(ge1 - ge0).max(), "np moved",
          np.abs(ce - ge0).max())
    ie = np.argsort(de.max(1))[-5:]
    print(" worst ent", ie, de.max(1)[ie], "gpu moved", np.abs(ge1 - ge0).max(1)[ie], "np moved",
          np.abs(ce - ge0).max(1)[ie])
    iw = np.argsort(dw.max((1, 2)))[-4:]
    print(" worst W", iw, dw.max((1, 2))[iw], "gpu moved", np.abs(gw1 - gw0).max((1, 2))[iw], "np moved",
          np.abs(cw - gw0).max((1, 2))[iw])
    sys.exit(0)

eng = make_engine(os.environ.get("KB2E_RPAR_NOC", "0") == "1")
for b in range(batches):
    sl = slice(b * B, (b + 1) * B)
    before = (pe.copy(), pr.copy(), pw.copy())
    lo, ao = transr_parallel_batches(pe, pr, pw, ds.train, si[sl], sj[sl], side[sl], B, 1, rate=rate, St=St,
                                     constraint=constraint)
    eng.train_batches(1)
    lg, ag = eng.take_stats()
    ge, gr, gw = eng.download_params()
    de, dr, dw = np.abs(ge - pe), np.abs(gr - pr), np.abs(gw - pw)
    print(f"batch {b}: active {ag} vs {ao}, loss {lg:.9f} vs {lo:.9f}, max|d| ent {de.max():.2e} rel {dr.max():.2e} "
          f"W {dw.max():.2e}")
    if max(de.max(), dr.max(), dw.max()) > 1e-9 or ag != ao:
        ie = np.argsort(de.max(1))[-5:]
        print(" worst ent rows", ie, de.max(1)[ie], "moved by", np.abs(pe - before[0]).max(1)[ie],
              "gpu moved", np.abs(ge - before[0]).max(1)[ie])
        iw = np.argsort(dw.max((1, 2)))[-3:]
        print(" worst W", iw, dw.max((1, 2))[iw])
        break
