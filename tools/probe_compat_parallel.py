#!/usr/bin/env python3
"""CPU probe: which PARALLEL-schedule term moves the TransR compat loss away
from the reference's (ORDERED) trajectory?

Trains the FB15k-shaped synthetic set with the reference restatement
(oracle/orc.c = ORDERED, the reference bit for bit) and with the CPU model of
the PARALLEL schedule (oracle/parallel.py) in its transRNorm variants (`cons`: jacobi, chunk<C>, seq), from the
same TransE-init tables and the same glibc sample stream, and prints per-epoch
losses plus table statistics (mean matrix-row length, mean |W_r^T e|).  Test
infrastructure only (it runs the oracle).

  python tools/probe_compat_parallel.py --epochs 4 --variants jacobi,chunk32
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from oracle import orc  # noqa: E402
from oracle.parallel import transr_parallel_batches  # noqa: E402


def table_stats(ent, rel, W, triples, rng):
    rows = np.sqrt((W ** 2).sum(2))
    k = rng.integers(0, len(triples), 4000)
    h, r = triples[k, 0], triples[k, 2]
    proj = np.einsum("kji,kj->ki", W[r], ent[h])
    return {"w_row_len": float(rows.mean()), "ent_len": float(np.sqrt((ent ** 2).sum(1)).mean()),
            "proj_len": float(np.sqrt((proj ** 2).sum(1)).mean()), "rel_len": float(np.sqrt((rel ** 2).sum(1)).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=4)
    ap.add_argument("--seed-epochs", type=int, default=20)
    ap.add_argument("--variants", default="jacobi,chunk32,seq")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--shape", default="fb15k")
    args = ap.parse_args()
    ds = data.synthetic(args.shape, seed=0)
    dim, NB = 50, 100
    t0 = time.time()
    te = orc.Model("E", dim, ds.num_entities, ds.num_relations, method=0, batches=NB)
    te.set_triples(ds.train)
    orc.srand(args.seed)
    te.prep_train()
    for _ in range(args.seed_epochs):
        te.train_epoch()
    se, sr, _ = te.tables()
    se, sr = np.round(se, 6), np.round(sr, 6)  # the %.6lf seed files
    print(f"seed tables {time.time() - t0:.1f} s", file=sys.stderr)

    def fresh():
        m = orc.Model("R", dim, ds.num_entities, ds.num_relations, method=1, batches=NB, transr_compat=True)
        m.set_triples(ds.train)
        orc.srand(args.seed)
        m.prep_train()
        m.transr_seed(se, sr)
        return m

    out = {"epochs": args.epochs, "seed": args.seed, "seed_epochs": args.seed_epochs}
    rng = np.random.default_rng(0)
    m = fresh()
    ent, rel, W = m.tables()
    B = m.batch_size()
    S = B * NB
    stream = m.sample_stream(S * args.epochs)
    t0 = time.time()
    ordered = fresh()
    ol = []
    for ep in range(args.epochs):
        loss, act = ordered.train_epoch()
        e2, r2, w2 = ordered.tables()
        ol.append({"loss": loss, "active": act, **table_stats(e2, r2, w2, ds.train, rng)})
        print(f"ordered epoch {ep}: {ol[-1]} ({time.time() - t0:.0f} s)", file=sys.stderr)
    out["ordered"] = ol
    for v in args.variants.split(","):
        # "<cons>/k<sub>": the form with phase B in `sub` ordered sub-batches
        cons, sub = (v.split("/k")[0], int(v.split("/k")[1])) if "/k" in v else (v, 1)
        pe, pr, pw = ent.copy(), rel.copy(), W.copy()
        work = [np.zeros(dim), np.zeros(dim)]
        pl = []
        t0 = time.time()
        for ep in range(args.epochs):
            sl = slice(ep * S, (ep + 1) * S)
            st = {}
            loss, act = transr_parallel_batches(pe, pr, pw, ds.train, stream[0][sl], stream[1][sl], stream[2][sl], B,
                                                NB, rate=0.001, compat=True, work=work, cons=cons, stats=st, sub=sub)
            pl.append({"loss": loss, "active": act, **st, **table_stats(pe, pr, pw, ds.train, rng)})
            print(f"parallel[{v}] epoch {ep}: {pl[-1]} ({time.time() - t0:.0f} s)", file=sys.stderr)
        out[f"parallel_{v}"] = pl
    print(json.dumps(out))


if __name__ == "__main__":
    main()
