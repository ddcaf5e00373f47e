"""Multi-GPU data parallelism: one process per GPU, triples sharded by head.

SURVEY.md 8(e): every rank trains the triples whose head entity hashes to it
(sampling only from its shard, with the reference's per-batch semantics on a
full replica of the tables).  At each epoch boundary the ranks merge their
table deltas and re-apply the reference's norm constraints:

    T <- renorm(T0 + sum_r (T_r - T0))

* relations and the relation weights (TransH normals, TransR matrices): one
  all-reduce (sum) of the deltas over RCCL, then every rank renormalises the
  rows any rank changed (the same rows on every rank: the summed delta is the
  same everywhere);
* entities: a reduce-scatter of the deltas to the owner of each contiguous
  block of rows, the owner adds them, renormalises its changed rows, and an
  all-gather hands every rank the merged table -- the all-reduce's bytes, but
  each rank renormalises only 1/N of the rows.

Two implementations of the same merge:

* `NativeMerger` (the product path, RCCL): the merge runs inside the engine
  (kb2e_comm_init_rank / kb2e_merge_epoch, engine_merge.inc) on the engine's
  own stream over the engine's own RCCL communicator; torch.distributed only
  hands rank 0's communicator id to the other ranks.
* `EpochMerger` / `TableMerger` (gloo: the CPU tests and the one-GPU
  rehearsal, where RCCL refuses two ranks on one device): the same phases
  over torch tensors that alias the engine's tables, with the changed-row
  masks on the device (kb2e_renormalize_rows takes a device mask).  Rows touched by one rank get exactly that rank's
update; shared rows (popular relations) get every rank's contribution, like a
sequential pass over the shards.  This is a documented relaxation of the
single-GPU semantics (local SGD per epoch); single-GPU runs are exact.
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


class _EngineRows:
    """The norm constraint of a live engine on a row range (device mask)."""

    def __init__(self, eng):
        self.eng = eng

    def synchronize(self):
        self.eng.synchronize()

    def renormalize(self, table, first, count, mask):
        import torch

        if mask is not None and mask.is_cuda:
            torch.cuda.synchronize()  # torch's stream wrote the rows; the engine's stream renormalises them
        self.eng.renormalize_rows(table, first, count, mask.data_ptr() if mask is not None else None)


def _host_staged(dist, t):
    """gloo over device tensors (the one-GPU rehearsal, tests/test_gpu_distributed.py)
    runs these collectives through host copies."""
    return t.is_cuda and dist.get_backend() == "gloo"


def _reduce_scatter(dist, out, inp):
    if _host_staged(dist, inp):
        o = out.cpu()
        dist.reduce_scatter_tensor(o, inp.cpu())
        out.copy_(o)
    else:
        dist.reduce_scatter_tensor(out, inp)


def _all_gather(dist, out, inp):
    if _host_staged(dist, inp):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu())
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp)


def _changed(delta, row_len):
    """uint8 mask of the rows with a non-zero delta (on the tensor's device)."""
    import torch

    return (delta.view(-1, row_len) != 0).any(dim=1).to(torch.uint8)


class TableMerger:
    """The epoch-boundary exchange over tables given as flat tensors.

    tables: [entity, relation(, weights)] flat tensors (views of the engine's
    memory on a GPU; plain tensors in the CPU tests); units: rows per table
    (entities, relations, relations); unit_len: elements per unit;
    rows: an object with renormalize(table, first, count, mask) and
    synchronize()."""

    def __init__(self, tables, units, unit_len, rows, dist):
        import torch

        self.tables, self.units, self.unit_len, self.rows, self.dist = tables, units, unit_len, rows, dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        rows.synchronize()
        for t in tables:  # every rank starts from rank 0's tables
            dist.broadcast(t, 0)
        self.base = [t.clone() for t in tables]
        self._torch_sync(tables[0])  # the engine's stream must not run before torch's copies land
        ne, L = units[0], unit_len[0]
        self.block = (ne + self.world - 1) // self.world  # entity rows per owner
        self.lo = min(ne, self.rank * self.block)
        self.hi = min(ne, self.lo + self.block)
        dev, dt = tables[0].device, tables[0].dtype
        self.send = torch.zeros(self.block * self.world * L, dtype=dt, device=dev)
        self.recv = torch.zeros(self.block * L, dtype=dt, device=dev)

    def merge(self):
        import torch

        self.rows.synchronize()
        ne, L = self.units[0], self.unit_len[0]
        ent, base = self.tables[0], self.base[0]
        # entities: reduce-scatter the deltas to the block owners
        torch.sub(ent, base, out=self.send[: ne * L])
        _reduce_scatter(self.dist, self.recv, self.send)
        n_own = self.hi - self.lo
        own = ent[self.lo * L: self.hi * L]
        torch.add(base[self.lo * L: self.hi * L], self.recv[: n_own * L], out=own)
        if n_own:
            mask = _changed(self.recv[: n_own * L], L)
            self.rows.renormalize(0, self.lo, n_own, mask)
        self.recv[: n_own * L].copy_(own)
        _all_gather(self.dist, self.send, self.recv)
        ent.copy_(self.send[: ne * L])
        # relations and weights: all-reduce the deltas, every rank renormalises
        for k in range(1, len(self.tables)):
            t, b = self.tables[k], self.base[k]
            t.sub_(b)
            self.dist.all_reduce(t)
            mask = _changed(t, self.unit_len[k])
            t.add_(b)
            self.rows.renormalize(k, 0, self.units[k], mask)
        self.rows.synchronize()
        for t, b in zip(self.tables, self.base):
            b.copy_(t)
        self._torch_sync(self.tables[0])  # the next batches (engine stream) write the tables

    @staticmethod
    def _torch_sync(t):
        if t.is_cuda:
            import torch

            torch.cuda.synchronize()


class EpochMerger(TableMerger):
    """TableMerger over a live engine's device tables (one engine per rank)."""

    def __init__(self, eng, dist):
        tables = engine_tables(eng)
        ld = tables[0].numel() // eng.ne
        units = [eng.ne, eng.nr] + ([eng.nr] if len(tables) > 2 else [])
        unit_len = [ld, ld] + ([tables[2].numel() // eng.nr] if len(tables) > 2 else [])
        super().__init__(tables, units, unit_len, _EngineRows(eng), dist)


class NativeMerger:
    """The epoch merge inside the engine over its own RCCL communicator
    (kb2e_comm_init_rank + kb2e_merge_epoch): rank 0 makes the RCCL id, the
    torch process group broadcasts it, every rank joins (rank 0's tables are
    broadcast by the engine)."""

    def __init__(self, eng, dist):
        import torch

        from .engine import COMM_ID_BYTES, Engine

        rank, world = dist.get_rank(), dist.get_world_size()
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        buf = torch.zeros(COMM_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            buf.copy_(torch.tensor(list(Engine.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(buf, 0)
        eng.comm_init_rank(world, rank, bytes(buf.cpu().tolist()))
        self.eng = eng

    def merge(self):
        self.eng.merge_epoch()


def make_merger(eng, dist):
    """NativeMerger over RCCL; the torch-side TableMerger when the group is gloo."""
    if dist.get_backend() == "nccl":
        return NativeMerger(eng, dist)
    return EpochMerger(eng, dist)


def shard_heads(triples: np.ndarray, rank: int, world: int) -> np.ndarray:
    """The training triples rank `rank` owns: head entity hash mod world."""
    h = triples[:, 0].astype(np.uint64)
    owner = ((h * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)) % np.uint64(world)
    return triples[owner == rank]
