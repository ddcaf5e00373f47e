#!/usr/bin/env python3
"""Sweep schedule-parity settings on a small planted set (picks the GPU test's
configuration); one JSON line per setting on stdout.  Besides ORDERED vs
PARALLEL (same seed), ORDERED with another glibc seed measures how far two
equally valid runs of the reference's own algorithm land apart."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kb2e_amd import data  # noqa: E402
from kb2e_amd.linkpred import train_and_evaluate, transe_seed  # noqa: E402

log = lambda m: print(m, file=sys.stderr, flush=True)  # noqa: E731
ds = data.synthetic("small", seed=0, counts=(2000, 40, 30000, 1000, 8000))
runs = [
    ("E", 50, 300, dict(rate=0.001)),
    ("H", 50, 300, dict(rate=0.001)),
    ("R", 32, 50, dict(rate=0.001, transr_compat=False)),
    ("R", 32, 150, dict(rate=0.001, transr_compat=True)),
]
for model, dim, epochs, kw in runs:
    st = transe_seed(ds, dim, 300) if model == "R" else None
    out = {"model": model, "dim": dim, "epochs": epochs, "kw": kw, "random": 10 / ds.num_entities}
    for name, sched, seed in (("ordered", "ordered", 7), ("parallel", "parallel", 7), ("ordered_s8", "ordered", 8),
                              ("parallel_s8", "parallel", 8)):
        r = train_and_evaluate(ds, model, dim, sched, epochs, seed=seed, seed_tables=st, **kw)
        r["losses"] = r["losses"][-1:]
        out[name] = r
    if model == "R":
        out["seed_only"] = train_and_evaluate(ds, "R", dim, "ordered", 0, seed_tables=st, transr_compat=False)
    print(json.dumps(out), flush=True)
