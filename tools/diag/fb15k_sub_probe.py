#!/usr/bin/env python3
"""FB15k-shaped PARALLEL TransR (n = 50 compat, TransE-init, as test_gpu_fb15k_shape
K4) against oracle/parallel.py batch by batch with a chosen sub-batch count:
active counts and per-table errors after each batch, the relations whose W rows
differ with their sample counts in each sub-batch (diagnostic).

    python tools/diag/fb15k_sub_probe.py <sub> [batches]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402
from kb2e_amd.linkpred import transe_seed  # noqa: E402
from oracle import orc  # noqa: E402
from oracle.parallel import sub_batch_bounds, transr_parallel_batches  # noqa: E402

sub = int(sys.argv[1])
nbat = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dim, rate, batches, seed = 50, 0.001, 100, 7
fb = data.synthetic("fb15k", seed=0)
ent0, rel0 = transe_seed(fb, dim, 5, seed=seed)
m = orc.Model("R", dim, fb.num_entities, fb.num_relations, rate=rate, method=1, batches=batches, transr_compat=True)
m.set_triples(fb.train)
orc.srand(seed)
m.prep_train()
eng = Engine("R", dim, fb.num_entities, fb.num_relations, rate=rate, method=1, batches=batches, seed=seed,
             schedule="parallel", transr_compat=True, sub_batches=sub)
eng.upload_triples(fb.train)
eng.init_params()
m.transr_seed(ent0, rel0)
eng.transr_seed(ent0, rel0)
pe, pr, pw = m.tables()
B = m.batch_size()
si, sj, side = m.sample_stream(B * nbat)
work = [np.zeros(dim), np.zeros(dim)]
for b in range(nbat):
    sl = slice(b * B, (b + 1) * B)
    lo, ao = transr_parallel_batches(pe, pr, pw, fb.train, si[sl], sj[sl], side[sl], B, 1, rate=rate, l1=True,
                                     compat=True, work=work, St=8, cons="chunk1", sub=sub)
    eng.train_batches(1)
    lg, ag = eng.take_stats()
    ge, gr, gw = eng.download_params()
    we = np.abs(gw - pw).reshape(fb.num_relations, -1).max(1)
    ee = np.abs(ge - pe).max(1)
    re_ = np.abs(gr - pr).max(1)
    rels = fb.train[si[sl], 2]
    bad = np.nonzero(we > 1e-9)[0]
    per_sub = []
    for lo_, hi_ in sub_batch_bounds(B, sub):
        per_sub.append(np.bincount(rels[lo_:hi_], minlength=fb.num_relations))
    print(b, "active", ag, ao, "loss %.6f %.6f" % (lg, lo),
          "err ent %.2e (%d rows) rel %.2e (%d) w %.2e (%d rels)" % (ee.max(), int((ee > 1e-9).sum()), re_.max(),
                                                                     int((re_ > 1e-9).sum()), we.max(), len(bad)),
          flush=True)
    cnt = np.bincount(rels, minlength=fb.num_relations)
    for r in bad[:12]:
        print("   rel", int(r), "W err %.2e" % we[r], "samples per sub-batch", [int(c[r]) for c in per_sub],
              "rank", int((cnt > cnt[r]).sum()), flush=True)
    pe, pr, pw = ge.copy(), gr.copy(), gw.copy()  # (continue from the device tables: one batch's error at a time)
