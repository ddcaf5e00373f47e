#!/usr/bin/env python3
"""Batch-by-batch PARALLEL TransR (wide kernels, sub-batches) against oracle/parallel.py:
active counts and table errors after each batch (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402
from oracle import orc  # noqa: E402
from oracle.parallel import transr_parallel_batches  # noqa: E402

dim, sub, compat = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1"
os.environ.setdefault("KB2E_RPAR_ST", "4")
ds = data.load(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "tiny"))
rate, batches, seed = 0.01, 10, 3
m = orc.Model("R", dim, ds.num_entities, ds.num_relations, rate=rate, batches=batches, transr_compat=compat)
m.set_triples(ds.train)
orc.srand(seed)
m.prep_train()
pe, pr, pw = m.tables()
eng = Engine("R", dim, ds.num_entities, ds.num_relations, rate=rate, batches=batches, seed=seed, schedule="parallel",
             transr_compat=compat, sub_batches=sub)
eng.upload_triples(ds.train)
e0, r0, w0 = eng.init_params()
eng.transr_seed(e0, r0)
pe = pe / np.linalg.norm(pe, axis=1, keepdims=True)
work = [np.zeros(dim), np.zeros(dim)]
B = m.batch_size()
si, sj, side = m.sample_stream(B * batches)
for b in range(batches):
    sl = slice(b * B, (b + 1) * B)
    lo, ao = transr_parallel_batches(pe, pr, pw, ds.train, si[sl], sj[sl], side[sl], B, 1, rate=rate, compat=compat,
                                     work=work, St=4, cons="chunk1", sub=sub)
    eng.train_batches(1)
    lg, ag = eng.take_stats()
    ge, gr, gw = eng.download_params()
    we = np.abs(gw - pw).reshape(ds.num_relations, -1).max(1)
    ee = np.abs(ge - pe).max(1)
    rb = sorted(set(ds.train[si[sl], 2].tolist()))
    print(b, "active", ag, ao, "loss %.6f %.6f" % (lg, lo), "err ent %.2e rel %.2e w %.2e" % (ee.max(),
          np.abs(gr - pr).max(), we.max()), "bad W rels", np.nonzero(we > 1e-9)[0].tolist(), "batch rels", rb,
          "bad ents", int((ee > 1e-9).sum()), flush=True)
