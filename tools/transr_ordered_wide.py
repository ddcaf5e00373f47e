#!/usr/bin/env python3
"""Time ORDERED TransR batches at a wide dim on the FB15k-shaped set (ADVICE r5:
the L2-resident relation owner at dim 512 and how its batch time compares with
the ticket waits' bound).  One JSON line: ms per batch (batch 0, which also
builds the epoch's sample stream and index, left out), the batch size, and the
ticket waits' wall-clock bound (KB2E_TICKET_WAIT_S, 600 s)."""
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
ap.add_argument("--nbatches", type=int, default=100, help="the reference's --batches (smaller batches: shorter chains)")
args = ap.parse_args()
ds = data.synthetic("fb15k", seed=0)
eng = Engine("R", args.dim, ds.num_entities, ds.num_relations, rate=0.001, method=1, batches=args.nbatches, seed=7,
             precision=args.precision, schedule="ordered", transr_compat=True)
eng.upload_triples(ds.train)
t0 = time.perf_counter()
e0, r0, _, _ = eng.init_params_device()  # (the reference's randn draws, made on the device)
eng.transr_seed(e0, r0)
print(f"init {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
times = []
for q in range(args.batches + 1):  # (batch 0 carries the epoch's sample stream and index)
    t0 = time.perf_counter()
    eng.train_batches(1)
    eng.synchronize()
    dt = time.perf_counter() - t0
    print(f"batch {q}: {dt * 1e3:.1f} ms", file=sys.stderr, flush=True)
    if q:
        times.append(dt)
loss, act = eng.take_stats()  # raises if a ticket wait timed out
rel = np.bincount(ds.train[:, 2], minlength=ds.num_relations)
floor_s = float(os.environ.get("KB2E_TICKET_WAIT_S", 600))  # the ticket waits' wall-clock bound
print(json.dumps({"dim": args.dim, "precision": args.precision, "ms_per_batch": [t * 1e3 for t in times],
                  "batch_samples": len(ds.train) // args.nbatches, "hottest_relation_share": float(rel.max() / rel.sum()),
                  "active": act, "timeout_floor_s": floor_s,
                  "margin": floor_s / max(times)}))
