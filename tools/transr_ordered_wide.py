#!/usr/bin/env python3
"""Time ORDERED TransR batches at a wide dim on the FB15k-shaped set (ADVICE r5:
the L2-resident relation owner at dim 512 and how far its batch time sits from the
bounded ticket waits' timeout).  One JSON line: ms per batch, the busiest
owner's update count, and the timeout floor (2^26 spins of s_sleep 1 = 64
cycles each at 2.4 GHz, i.e. before the spin loop's own load latency)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dim", type=int, default=512)
ap.add_argument("--batches", type=int, default=3)
ap.add_argument("--precision", type=int, default=64)
args = ap.parse_args()
ds = data.synthetic("fb15k", seed=0)
eng = Engine("R", args.dim, ds.num_entities, ds.num_relations, rate=0.001, method=1, batches=100, seed=7,
             precision=args.precision, schedule="ordered", transr_compat=True)
eng.upload_triples(ds.train)
e0, r0, _ = eng.init_params()
eng.transr_seed(e0, r0)
eng.train_batches(1)  # (the epoch's sample stream and index)
eng.synchronize()
times = []
for _ in range(args.batches):
    t0 = time.perf_counter()
    eng.train_batches(1)
    eng.synchronize()
    times.append(time.perf_counter() - t0)
loss, act = eng.take_stats()  # raises if a ticket wait timed out
rel = np.bincount(ds.train[:, 2], minlength=ds.num_relations)
floor_s = (1 << 26) * 64 / 2.4e9
print(json.dumps({"dim": args.dim, "precision": args.precision, "ms_per_batch": [t * 1e3 for t in times],
                  "batch_samples": len(ds.train) // 100, "hottest_relation_share": float(rel.max() / rel.sum()),
                  "active": act, "timeout_floor_s": floor_s,
                  "margin": floor_s / max(times)}))
