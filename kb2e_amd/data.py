"""Datasets in the reference's on-disk formats, plus synthetic generators.

File formats (reference ``common/loader.cpp:15-62``, ``common/constants.h:23-30``):

* ``entity2id.txt`` / ``relation2id.txt``: ``"<name>\\t<id>"`` per line, ids dense
  from 0 (``README.md:4``).
* ``train.txt`` / ``valid.txt`` / ``test.txt``: ``"<head>\\t<tail>\\t<relation>"``
  names per line; lines naming an unknown id are skipped with a message.

The synthetic generator follows SURVEY.md section 8(d): Zipf entity popularity
and relation frequency, and triples planted by a hidden translation model
(tail = the nearest of 8 Zipf-drawn candidates to ``E_h + R_r`` in 20-d) so
link prediction is learnable.  numpy PCG64, fixed seeds.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

ENTITY_ID_FILE = "entity2id.txt"
RELATION_ID_FILE = "relation2id.txt"
TRAIN_FILE = "train.txt"
VALID_FILE = "valid.txt"
TEST_FILE = "test.txt"


@dataclass
class Dataset:
    """Dense-id triples.  Arrays are int32 (head, tail, relation) in file order."""

    num_entities: int
    num_relations: int
    train: np.ndarray  # [N, 3] (h, t, r)
    valid: np.ndarray
    test: np.ndarray

    def split(self, name: str) -> np.ndarray:
        return {"train": self.train, "valid": self.valid, "test": self.test}[name]


# (entities, relations, train, valid, test) of the shapes BASELINE.json names.
SHAPES = {
    "tiny": (200, 10, 3000, 200, 200),
    "small": (2000, 40, 30000, 1000, 1000),
    "wn18": (40943, 18, 141442, 5000, 5000),
    "fb15k": (14951, 1345, 483142, 50000, 59071),
    "k5": (1000000, 10000, 16000000, 0, 0),
}


def _zipf_probs(n: int, a: float) -> np.ndarray:
    p = 1.0 / np.arange(1, n + 1, dtype=np.float64) ** a
    return p / p.sum()


def synthetic(shape: str = "fb15k", seed: int = 0, *, planted: bool | None = None,
              entity_zipf: float | None = None, relation_zipf: float | None = None,
              counts: tuple | None = None) -> Dataset:
    """Generate a dataset of the named shape (see ``SHAPES``)."""
    ne, nr, ntr, nva, nte = counts if counts is not None else SHAPES[shape]
    if planted is None:
        planted = shape != "k5"
    ea = entity_zipf if entity_zipf is not None else (0.6 if shape == "k5" else 0.8)
    ra = relation_zipf if relation_zipf is not None else (0.9 if shape == "k5" else 1.0)
    rng = np.random.Generator(np.random.PCG64(seed))
    # Popularity ranks are shuffled over ids so hot rows are not all low ids.
    eperm = rng.permutation(ne).astype(np.int64)
    rperm = rng.permutation(nr).astype(np.int64)
    pe = _zipf_probs(ne, ea)
    pr = _zipf_probs(nr, ra)
    total = ntr + nva + nte
    want = int(total * 1.35) + 64
    keys = np.empty(0, dtype=np.int64)
    out_h = []
    out_t = []
    out_r = []
    if planted:
        dim = 20
        E = rng.standard_normal((ne, dim)).astype(np.float32)
        R = rng.standard_normal((nr, dim)).astype(np.float32) * 0.5
    seen = 0
    while seen < total:
        h = eperm[rng.choice(ne, size=want, p=pe)]
        r = rperm[rng.choice(nr, size=want, p=pr)]
        if planted:
            cand = eperm[rng.choice(ne, size=(want, 8), p=pe)]
            target = E[h] + R[r]
            d = ((E[cand] - target[:, None, :]) ** 2).sum(-1)
            t = cand[np.arange(want), d.argmin(1)]
        else:
            t = eperm[rng.choice(ne, size=want, p=pe)]
        ok = h != t
        h, t, r = h[ok], t[ok], r[ok]
        k = (h * nr + r) * ne + t
        k_all = np.concatenate([keys, k])
        _, first = np.unique(k_all, return_index=True)
        first = np.sort(first)
        new = first[first >= keys.size] - keys.size
        keys = np.concatenate([keys, k[new]])
        out_h.append(h[new])
        out_t.append(t[new])
        out_r.append(r[new])
        seen = keys.size
    H = np.concatenate(out_h)[:total]
    T = np.concatenate(out_t)[:total]
    Rr = np.concatenate(out_r)[:total]
    order = rng.permutation(total)
    trip = np.stack([H, T, Rr], axis=1)[order].astype(np.int32)
    return Dataset(ne, nr, trip[:ntr], trip[ntr:ntr + nva], trip[ntr + nva:])


def write(ds: Dataset, datadir: str) -> None:
    """Write the reference's text files (names ``/m/e<id>`` and ``/r/r<id>``)."""
    os.makedirs(datadir, exist_ok=True)
    with open(os.path.join(datadir, ENTITY_ID_FILE), "w") as f:
        f.write("".join(f"/m/e{i}\t{i}\n" for i in range(ds.num_entities)))
    with open(os.path.join(datadir, RELATION_ID_FILE), "w") as f:
        f.write("".join(f"/r/r{i}\t{i}\n" for i in range(ds.num_relations)))
    for name, arr in ((TRAIN_FILE, ds.train), (VALID_FILE, ds.valid), (TEST_FILE, ds.test)):
        with open(os.path.join(datadir, name), "w") as f:
            f.write("".join(f"/m/e{h}\t/m/e{t}\t/r/r{r}\n" for h, t, r in arr.tolist()))


def _load_ids(path: str) -> dict:
    ids = {}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 2:
                ids[parts[0]] = int(parts[1])
    return ids


def _load_triples(path: str, ent: dict, rel: dict) -> np.ndarray:
    rows = []
    if not os.path.exists(path):
        return np.zeros((0, 3), dtype=np.int32)
    with open(path) as f:
        for line in f:
            parts = line.split()
            if len(parts) < 3:
                continue
            h, t, r = parts[0], parts[1], parts[2]
            if h not in ent or t not in ent or r not in rel:
                # common/loader.cpp:40-57: report and skip
                continue
            rows.append((ent[h], ent[t], rel[r]))
    return np.asarray(rows, dtype=np.int32).reshape(-1, 3)


def load(datadir: str) -> Dataset:
    """Read a dataset directory in the reference's format."""
    ent = _load_ids(os.path.join(datadir, ENTITY_ID_FILE))
    rel = _load_ids(os.path.join(datadir, RELATION_ID_FILE))
    return Dataset(len(ent), len(rel),
                   _load_triples(os.path.join(datadir, TRAIN_FILE), ent, rel),
                   _load_triples(os.path.join(datadir, VALID_FILE), ent, rel),
                   _load_triples(os.path.join(datadir, TEST_FILE), ent, rel))


def write_table(path: str, table: np.ndarray) -> None:
    """``"%.6lf\\t"`` per value, one row per line (common/trainer.cpp:109-127)."""
    t = np.asarray(table, dtype=np.float64)
    t = t.reshape(-1, t.shape[-1])
    with open(path, "w") as f:
        for row in t:
            f.write("".join("%.6f\t" % v for v in row.tolist()) + "\n")


def read_table(path: str, rows: int, dim: int) -> np.ndarray:
    with open(path) as f:
        vals = np.array(f.read().split(), dtype=np.float64)
    if vals.size < rows * dim:
        raise ValueError(f"short embedding file {path}: {vals.size} < {rows * dim}")
    return vals[: rows * dim].reshape(rows, dim)
