"""Multi-GPU data parallelism: one process per GPU, triples sharded by head.

SURVEY.md 8(e): every rank trains the triples whose head entity hashes to it
(sampling only from its shard, with the reference's per-batch semantics on a
full replica of the tables).  At each epoch boundary the ranks exchange their
table deltas with one all-reduce (sum) over RCCL and re-apply the reference's
norm constraints (kb2e_renormalize):

    T <- renorm(T0 + sum_r (T_r - T0))

Rows touched by one rank get exactly that rank's update; shared rows (popular
relations) get every rank's contribution, like a sequential pass over the
shards.  This is a documented relaxation of the single-GPU semantics (local
SGD per epoch); single-GPU runs are exact.
"""
from __future__ import annotations

import ctypes as C

import numpy as np


class _DeviceArray:
    """__cuda_array_interface__ view of engine-owned device memory."""

    def __init__(self, ptr, count, typestr):
        self.__cuda_array_interface__ = {"shape": (int(count),), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 3, "strides": None}


def engine_tables(eng):
    """torch tensors aliasing the engine's tables (entity, relation[, weights])."""
    import torch

    from .engine import lib

    e, r, w = C.c_void_p(), C.c_void_p(), C.c_void_p()
    ne, nr, nw = C.c_int64(), C.c_int64(), C.c_int64()
    st = lib().kb2e_device_tables(eng.h, C.byref(e), C.byref(r), C.byref(w), C.byref(ne), C.byref(nr),
                                  C.byref(nw))
    if st != 0:
        raise RuntimeError("kb2e_device_tables failed")
    typestr = "<f8" if eng.cfg.precision == 64 else "<f4"
    out = []
    for p, n in ((e, ne), (r, nr), (w, nw)):
        if p.value and n.value:
            out.append(torch.as_tensor(_DeviceArray(p.value, n.value, typestr), device="cuda"))
    return out


def merge_deltas(tables, base, dist, row_len):
    """In place: tables <- base + all_reduce_sum(tables - base).  Returns, per
    table, a uint8 mask of the rows any rank changed (numpy, for renormalize)."""
    masks = []
    for t, b, rl in zip(tables, base, row_len):
        t.sub_(b)
        dist.all_reduce(t)
        masks.append((t.view(-1, rl) != 0).any(dim=1).to("cpu").numpy().astype(np.uint8))
        t.add_(b)
    while len(masks) < 3:
        masks.append(None)
    return masks


class EpochMerger:
    """Epoch-boundary exchange for one engine (rank)."""

    def __init__(self, eng, dist):
        self.eng = eng
        self.dist = dist
        self.tables = engine_tables(eng)
        # all ranks start from rank 0's tables
        eng.synchronize()
        for t in self.tables:
            dist.broadcast(t, 0)
        self.base = [t.clone() for t in self.tables]

    def merge(self):
        import torch

        self.eng.synchronize()
        masks = merge_deltas(self.tables, self.base, self.dist, self.row_lengths())
        torch.cuda.synchronize()
        self.eng.renormalize(*masks)
        self.eng.synchronize()
        for t, b in zip(self.tables, self.base):
            b.copy_(t)

    def row_lengths(self):
        """Elements per mask row of each table (weights: one mask row per relation)."""
        ld = self.tables[0].numel() // self.eng.ne
        out = [ld, ld]
        if len(self.tables) > 2:
            out.append(self.tables[2].numel() // self.eng.nr)
        return out


def shard_heads(triples: np.ndarray, rank: int, world: int) -> np.ndarray:
    """The training triples rank `rank` owns: head entity hash mod world."""
    h = triples[:, 0].astype(np.uint64)
    owner = ((h * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)) % np.uint64(world)
    return triples[owner == rank]
