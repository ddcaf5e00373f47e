#!/usr/bin/env python3
"""Link-prediction parity of the PARALLEL schedule against the ORDERED one
(= the reference: FP64 tables within 1e-11 of the reference's, tests/).

Trains the same synthetic FB15k-shaped set (kb2e_amd.data, planted TransE
structure) with both schedules on the GPU, from the same initial tables and the
same glibc sample stream, and scores both with the GPU evaluator
(kb2e_evaluate = EmbeddingEvaluation::run, common/evaluation.cpp:181-251) on
the same test subset with filter = train + valid + test.  Prints one JSON line.

  python tools/hits_parity.py --model E --epochs 1000 --test 5000
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
from kb2e_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="E", choices=["E", "H", "R"])
    ap.add_argument("--shape", default="fb15k")
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--test", type=int, default=5000, help="test triples scored (0 = all)")
    ap.add_argument("--rate", type=float, default=0.001)
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--schedules", default="ordered,parallel")
    ap.add_argument("--seed-epochs", type=int, default=0, help="TransR: TransE epochs for the seed tables")
    args = ap.parse_args()
    dim = args.dim or {"E": 100, "H": 100, "R": 50}[args.model]
    ds = data.synthetic(args.shape, seed=0)
    test = ds.test if args.test <= 0 else ds.test[: args.test]
    filt = np.concatenate([ds.train, ds.valid, ds.test])
    seed_tabs = None
    if args.model == "R" and args.seed_epochs > 0:
        # TransR starts from TransE embeddings (transr/trainer.cpp:88-113): unif TransE, ordered
        se = Engine("E", dim, ds.num_entities, ds.num_relations, rate=args.rate, method=0, seed=args.seed)
        se.upload_triples(ds.train)
        se.init_params()
        for _ in range(args.seed_epochs):
            se.train_epoch()
        seed_tabs = se.download_params()[:2]
        se.close()
    out = {"model": args.model, "shape": args.shape, "dim": dim, "epochs": args.epochs, "test": len(test),
           "rate": args.rate, "method": args.method}
    for sched in args.schedules.split(","):
        eng = Engine(args.model, dim, ds.num_entities, ds.num_relations, rate=args.rate, method=args.method,
                     seed=args.seed, schedule=sched)
        eng.upload_triples(ds.train)
        ent, rel, _ = eng.init_params()
        if args.model == "R":
            eng.transr_seed(*(seed_tabs if seed_tabs is not None else (ent, rel)))
        t0 = time.perf_counter()
        losses = []
        for ep in range(args.epochs):
            loss, act = eng.train_epoch()
            if ep % max(1, args.epochs // 10) == 0 or ep == args.epochs - 1:
                losses.append((ep, round(loss, 3), act))
                print(f"[{sched}] epoch {ep} loss {loss:.3f} active {act}", file=sys.stderr, flush=True)
        train_s = time.perf_counter() - t0
        res = eng.evaluate(test, filt)
        out[sched] = {"train_s": train_s, "samples_per_s": args.epochs * (len(ds.train) // 100) * 100 / train_s,
                      "losses": losses, **{k: float(v) for k, v in res.items()}}
        print(f"[{sched}] {json.dumps(out[sched])}", file=sys.stderr, flush=True)
        eng.close()
    s = args.schedules.split(",")
    if len(s) == 2:
        out["delta_filtered_hits10_pp"] = 100 * (out[s[1]]["filtered_hits10"] - out[s[0]]["filtered_hits10"])
        out["delta_raw_hits10_pp"] = 100 * (out[s[1]]["raw_hits10"] - out[s[0]]["raw_hits10"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
