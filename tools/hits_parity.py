#!/usr/bin/env python3
"""Link-prediction parity of the PARALLEL schedule against the ORDERED one
(= the reference: FP64 tables within 1e-11 of the reference's, tests/).

Trains a synthetic planted set (kb2e_amd.data) with both schedules on the GPU,
from the same initial tables and the same glibc sample stream, and scores both
with the GPU evaluator (kb2e_evaluate = EmbeddingEvaluation::run,
common/evaluation.cpp:181-251) on the same test triples with filter = train +
valid + test.  TransR is TransE-initialised (kb2e_amd.linkpred.transe_seed).
Prints one JSON line (kb2e_amd.linkpred.schedule_parity).

  python tools/hits_parity.py --model E --epochs 1000 --test 5000
  python tools/hits_parity.py --model R --epochs 100 --seed-epochs 200 --compat 1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kb2e_amd import data  # noqa: E402
from kb2e_amd.linkpred import schedule_parity  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="E", choices=["E", "H", "R"])
    ap.add_argument("--shape", default="fb15k")
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--test", type=int, default=5000, help="test triples scored (0 = all)")
    ap.add_argument("--rate", type=float, default=0.001)
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--batches", type=int, default=100)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--compat", type=int, default=1, help="TransR: 1 = the reference's accumulating energy")
    ap.add_argument("--seed-epochs", type=int, default=200, help="TransR: TransE epochs for the seed tables")
    args = ap.parse_args()
    dim = args.dim or {"E": 100, "H": 100, "R": 50}[args.model]
    ds = data.synthetic(args.shape, seed=0)
    test = ds.test if args.test <= 0 else ds.test[: args.test]
    out = schedule_parity(ds, args.model, dim, args.epochs, seed_epochs=args.seed_epochs, test=test,
                          rate=args.rate, method=args.method, batches=args.batches, seed=args.seed,
                          transr_compat=bool(args.compat), log=lambda m: print(m, file=sys.stderr, flush=True))
    out.update(shape=args.shape, rate=args.rate, method=args.method, batches=args.batches,
               transr_compat=bool(args.compat))
    for s in ("ordered", "parallel"):
        out[s]["losses"] = out[s]["losses"][:: max(1, args.epochs // 10)] + out[s]["losses"][-1:]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
