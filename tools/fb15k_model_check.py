#!/usr/bin/env python3
"""The PARALLEL TransR kernels against their CPU model (oracle/parallel.py) at
FB15k shape: same TransE-init seed tables, same glibc sample stream, `epochs`
epochs; prints per-epoch loss / active count of both and the largest table
differences.  The tests (tests/test_gpu_parallel.py) do this on the tiny set;
this checks that nothing specific to the FB15k-shaped batches (hot relations,
hub entities, many tiles a relation) separates the kernel from its model.
Test infrastructure (runs the oracle).

  python tools/fb15k_model_check.py --epochs 2 --seed-epochs 20
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
from kb2e_amd.linkpred import transe_seed  # noqa: E402
from oracle import orc  # noqa: E402
from oracle.parallel import transr_parallel_batches  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--seed-epochs", type=int, default=20)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cons", default="chunk1")  # the engine's per-pair sequential transRNorm
    args = ap.parse_args()
    ds = data.synthetic("fb15k", seed=0)
    dim, NB, rate = 50, 100, 0.001
    se, sr = transe_seed(ds, dim, args.seed_epochs, seed=args.seed)
    m = orc.Model("R", dim, ds.num_entities, ds.num_relations, method=1, batches=NB, transr_compat=True)
    m.set_triples(ds.train)
    orc.srand(args.seed)
    m.prep_train()
    m.transr_seed(se, sr)
    pe, pr, pw = m.tables()
    B = m.batch_size()
    eng = Engine("R", dim, ds.num_entities, ds.num_relations, rate=rate, method=1, batches=NB, seed=args.seed,
                 schedule="parallel", transr_compat=True)
    eng.upload_triples(ds.train)
    eng.init_params()
    eng.transr_seed(se, sr)
    ge, gr, gw = eng.download_params()
    out = {"init_diff": [float(np.abs(ge - pe).max()), float(np.abs(gr - pr).max()), float(np.abs(gw - pw).max())],
           "epochs": []}
    work = [np.zeros(dim), np.zeros(dim)]
    for ep in range(args.epochs):
        si, sj, side = m.sample_stream(B * NB)
        t0 = time.time()
        lo, ao = transr_parallel_batches(pe, pr, pw, ds.train, si, sj, side, B, NB, rate=rate, compat=True, work=work,
                                         cons=args.cons)
        tm = time.time() - t0
        lg, ag = eng.train_epoch()
        ge, gr, gw = eng.download_params()
        rec = {"epoch": ep, "model_loss": lo, "gpu_loss": lg, "model_active": ao, "gpu_active": ag,
               "max_diff": [float(np.abs(ge - pe).max()), float(np.abs(gr - pr).max()), float(np.abs(gw - pw).max())],
               "rows_over_1e-6": int((np.abs(ge - pe).max(1) > 1e-6).sum()), "model_s": tm}
        out["epochs"].append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
