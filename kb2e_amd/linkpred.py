"""Train-then-evaluate driver for link-prediction comparisons (host side).

Runs the reference's train binary sequence (``transe/bin/trainTransE.cpp:9-20``:
prepTrain, bfgs epochs) on the GPU engine and scores the result with the GPU
evaluator (``kb2e_evaluate`` = ``EmbeddingEvaluation::run``,
``common/evaluation.cpp:181-251``; filter = train + valid + test as the
reference's eval binaries pass it, ``common/evaluation.cpp:41-62``).

TransR starts from TransE tables ("TransE-init", ``transr/trainer.cpp:88-113``):
``transe_seed`` trains TransE with the ORDERED schedule (the reference's exact
semantics) and round-trips the tables through the reference's ``%.6lf`` text
format, exactly what ``trainTransR --seeddatadir`` reads.

Used by tools/hits_parity.py (FB15k-shaped runs) and the schedule-parity GPU
test (tests/test_gpu_hits_parity.py).
"""
from __future__ import annotations

import os
import tempfile
import time

import numpy as np

from . import data
from .engine import Engine


def transe_seed(ds, dim, epochs, *, rate=0.001, seed=7, batches=100, device=0):
    """TransE n=dim unif (the reference's historical seed method) -> (entity, relation)
    tables as trainTransR reads them back from entity2vec.unif / relation2vec.unif."""
    eng = Engine("E", dim, ds.num_entities, ds.num_relations, rate=rate, method=0, seed=seed, batches=batches,
                 device=device, schedule="ordered")
    try:
        eng.upload_triples(ds.train)
        eng.init_params()
        if epochs:
            eng.train_batches(epochs * batches)
        eng.synchronize()
        ent, rel, _ = eng.download_params()
    finally:
        eng.close()
    with tempfile.TemporaryDirectory() as d:
        data.write_table(os.path.join(d, "entity2vec.unif"), ent)
        data.write_table(os.path.join(d, "relation2vec.unif"), rel)
        return (data.read_table(os.path.join(d, "entity2vec.unif"), ds.num_entities, dim),
                data.read_table(os.path.join(d, "relation2vec.unif"), ds.num_relations, dim))


def train_and_evaluate(ds, model, dim, schedule, epochs, *, test=None, rate=0.001, method=1, distance=0,
                       batches=100, seed=7, transr_compat=True, seed_tables=None, device=0, log=None,
                       sub_batches=None):
    """Train `epochs` epochs with one schedule and evaluate; returns a dict with
    the four EmbeddingEvaluation::run numbers, losses and timing."""
    test = ds.test if test is None else test
    filt = np.concatenate([ds.train, ds.valid, ds.test])
    eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                 batches=batches, seed=seed, transr_compat=transr_compat, device=device, schedule=schedule,
                 sub_batches=sub_batches)
    try:
        eng.upload_triples(ds.train)
        ent, rel, _ = eng.init_params()
        if model in ("R", "transr", 2):
            eng.transr_seed(*(seed_tables if seed_tables is not None else (ent, rel)))
        losses = []
        t0 = time.perf_counter()
        for ep in range(epochs):
            loss, act = eng.train_epoch()
            losses.append((ep, float(loss), int(act)))
            if log is not None and (ep % max(1, epochs // 10) == 0 or ep == epochs - 1):
                log(f"[{model}/{schedule}] epoch {ep} loss {loss:.3f} active {act}")
        train_s = time.perf_counter() - t0
        res = eng.evaluate(test, filt)
    finally:
        eng.close()
    S = (len(ds.train) // batches) * batches
    return {"train_s": train_s, "samples_per_s": epochs * S / max(train_s, 1e-9), "losses": losses,
            **{k: float(v) for k, v in res.items()}}


def schedule_parity(ds, model, dim, epochs, *, seed_epochs=0, test=None, schedules=("ordered", "parallel"),
                    **kw):
    """Both schedules from the same initial tables and the same glibc sample
    stream; returns {schedule: result, "delta_filtered_hits10_pp": ...}."""
    seed_tables = None
    if model == "R":
        seed_tables = transe_seed(ds, dim, seed_epochs, rate=kw.get("rate", 0.001), seed=kw.get("seed", 7),
                                  batches=kw.get("batches", 100), device=kw.get("device", 0))
    out = {"model": model, "dim": dim, "epochs": epochs, "seed_epochs": seed_epochs,
           "test": int(len(ds.test if test is None else test)), "entities": ds.num_entities,
           "random_hits10": 10.0 / ds.num_entities}
    for s in schedules:
        out[s] = train_and_evaluate(ds, model, dim, s, epochs, test=test, seed_tables=seed_tables, **kw)
    if len(schedules) == 2:
        a, b = schedules
        for k in ("filtered_hits10", "raw_hits10"):
            out[f"delta_{k}_pp"] = 100.0 * (out[b][k] - out[a][k])
        out["delta_filtered_rank"] = out[b]["filtered_rank"] - out[a]["filtered_rank"]
    return out
