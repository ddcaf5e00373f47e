"""Shared helpers for the GPU parity tests (tests/ only)."""
import json
import os

import numpy as np

from conftest import GOLDEN
from kb2e_amd import data
from kb2e_amd.engine import SAMPLER_GLIBC, SAMPLER_REPLAY, Engine
from oracle import orc

MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))

# FP64 engine vs the FP64 reference: same operations in the same order per
# element; only the order of the 64-lane sums (energies, vector lengths)
# differs, which moves results by a few ulps per update.
F64_ATOL = 1e-11
# Multi-epoch runs with the coupling loops (TransH orthogonality, TransR
# transRNorm) iterating: those loops divide by running sums and amplify the
# ulp-level differences of the 64-lane sums.  An ordering error would show up
# at the learning-rate scale (1e-3..1e-2), eight orders above this.
F64_ATOL_COUPLED = 1e-9
# FP32 engine vs FP64 reference over one epoch of the tiny set.
F32_ATOL = 2e-4


def tiny():
    return data.load(os.path.join(GOLDEN, "tiny"))


def golden_engine(name, precision=64, sampler=SAMPLER_GLIBC, schedule="ordered"):
    run = MANIFEST["runs"][name]
    f = run["flags"]
    ds = tiny()
    eng = Engine(run["model"], f["size"], ds.num_entities, ds.num_relations, rate=f["rate"], margin=f["margin"],
                 method=f["method"], distance=f["distance"], batches=f["batches"], seed=f["seed"],
                 precision=precision, sampler=sampler, transr_compat=not run["transr_fixed"], schedule=schedule)
    eng.upload_triples(ds.train)
    init = eng.init_params()
    if run["model"] == "R":
        sd = os.path.join(GOLDEN, "transe_seed_unif")
        ent = data.read_table(os.path.join(sd, "entity2vec.unif"), ds.num_entities, f["size"])
        rel = data.read_table(os.path.join(sd, "relation2vec.unif"), ds.num_relations, f["size"])
        eng.transr_seed(ent, rel)
    return eng, run, ds, init


def oracle_model(kind, ds, dim, **kw):
    m = orc.Model(kind, dim, ds.num_entities, ds.num_relations, **kw)
    m.set_triples(ds.train)
    return m


def max_abs(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)))) if np.size(a) else 0.0
