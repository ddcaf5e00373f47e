"""ctypes wrapper of oracle/liborc.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module -- as the checker or the CPU baseline, never as the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

MODELS = {"E": 0, "H": 1, "R": 2, "transe": 0, "transh": 1, "transr": 2}


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liborc.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library missing: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int)
        u8p = C.POINTER(C.c_uint8)
        vp = C.c_void_p
        ll = C.c_longlong
        sig = {
            "orc_srand": (None, [C.c_uint]),
            "orc_rand": (C.c_int, []),
            "orc_randmax": (C.c_int, [C.c_int]),
            "orc_randn": (C.c_double, [C.c_double] * 4),
            "orc_norm": (None, [dp, C.c_int, C.c_int]),
            "orc_norm_orth": (None, [dp, dp, C.c_int, C.c_double]),
            "orc_norm_orth_iterations": (ll, []),
            "orc_transr_norm": (None, [dp, dp, C.c_int, C.c_double]),
            "orc_transr_norm_iterations": (ll, []),
            "orc_site_iterations": (ll, [C.c_int]),
            "orc_create": (vp, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                C.c_int, C.c_int, C.c_int, C.c_int]),
            "orc_destroy": (None, [vp]),
            "orc_set_triples": (C.c_int, [vp, ip, ip, ip, C.c_int]),
            "orc_prep_train": (None, [vp]),
            "orc_transr_seed": (None, [vp, dp, dp]),
            "orc_get_tables": (None, [vp, dp, dp, dp]),
            "orc_set_tables": (None, [vp, dp, dp, dp]),
            "orc_get_transr_work": (None, [vp, dp, dp]),
            "orc_set_transr_work": (None, [vp, dp, dp]),
            "orc_train_epoch": (C.c_double, [vp, C.POINTER(ll)]),
            "orc_train_batches": (C.c_double, [vp, C.c_int, C.POINTER(ll)]),
            "orc_train_replay": (C.c_double, [vp, ip, ip, u8p, ll, C.POINTER(ll)]),
            "orc_sample_stream": (None, [vp, ll, ip, ip, u8p]),
            "orc_batch_size": (C.c_int, [vp]),
            "orc_triple_energy": (C.c_double, [vp, C.c_int, C.c_int, C.c_int]),
            "orc_begin_batch": (None, [vp]),
            "orc_gradient_update": (None, [vp, C.c_int, C.c_int, C.c_int, C.c_int]),
            "orc_end_batch": (None, [vp]),
            "orc_evaluate": (None, [vp, ip, ip, ip, C.c_int, ip, ip, ip, C.c_int, dp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def srand(seed: int) -> None:
    lib().orc_srand(seed)


def rand() -> int:
    return lib().orc_rand()


def randmax(x: int) -> int:
    return lib().orc_randmax(x)


def randn(miu, sigma, lo, hi) -> float:
    return lib().orc_randn(miu, sigma, lo, hi)


def norm(a: np.ndarray, ignore_short: bool = True) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64).copy()
    lib().orc_norm(_dp(a), a.size, int(ignore_short))
    return a


def norm_orth(a, b, rate):
    a = np.ascontiguousarray(a, dtype=np.float64).copy()
    b = np.ascontiguousarray(b, dtype=np.float64).copy()
    lib().orc_norm_orth(_dp(a), _dp(b), a.size, rate)
    return a, b


def transr_norm(a, b, rate):
    a = np.ascontiguousarray(a, dtype=np.float64).copy()
    b = np.ascontiguousarray(b, dtype=np.float64).copy()
    lib().orc_transr_norm(_dp(a), _dp(b), a.size, rate)
    return a, b


class Model:
    """One reference trainer (common::Trainer + model subclass) on the CPU."""

    def __init__(self, model, dim, num_entities, num_relations, *, rate=0.001, margin=1.0,
                 method=1, distance=0, batches=100, transr_compat=True):
        self.kind = MODELS[model] if isinstance(model, str) else int(model)
        self.n, self.ne, self.nr = dim, num_entities, num_relations
        self.h = lib().orc_create(self.kind, dim, num_entities, num_relations, rate, margin,
                                  method, distance, batches, int(transr_compat))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)
            self.h = None

    def set_triples(self, triples: np.ndarray) -> None:
        t = np.ascontiguousarray(triples, dtype=np.int32)
        h, tl, r = (np.ascontiguousarray(t[:, k]) for k in range(3))
        self._keep = (h, tl, r)
        lib().orc_set_triples(self.h, _ip(h), _ip(tl), _ip(r), len(t))

    def prep_train(self) -> None:
        lib().orc_prep_train(self.h)

    def transr_seed(self, ent, rel) -> None:
        ent = np.ascontiguousarray(ent, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        lib().orc_transr_seed(self.h, _dp(ent), _dp(rel))

    def wshape(self):
        if self.kind == 1:
            return (self.nr, self.n)
        if self.kind == 2:
            return (self.nr, self.n, self.n)
        return None

    def tables(self):
        ent = np.zeros((self.ne, self.n))
        rel = np.zeros((self.nr, self.n))
        w = np.zeros(self.wshape()) if self.wshape() else None
        lib().orc_get_tables(self.h, _dp(ent), _dp(rel), _dp(w))
        return ent, rel, w

    def set_tables(self, ent, rel, w=None):
        ent = np.ascontiguousarray(ent, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
        lib().orc_set_tables(self.h, _dp(ent), _dp(rel), _dp(w))

    def transr_work(self):
        a = np.zeros(self.n)
        b = np.zeros(self.n)
        lib().orc_get_transr_work(self.h, _dp(a), _dp(b))
        return a, b

    def set_transr_work(self, a, b):
        a = np.ascontiguousarray(a, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
        lib().orc_set_transr_work(self.h, _dp(a), _dp(b))

    def train_epoch(self):
        act = C.c_longlong(0)
        loss = lib().orc_train_epoch(self.h, C.byref(act))
        return loss, act.value

    def train_batches(self, nb):
        act = C.c_longlong(0)
        loss = lib().orc_train_batches(self.h, nb, C.byref(act))
        return loss, act.value

    def train_replay(self, si, sj, side):
        si = np.ascontiguousarray(si, dtype=np.int32)
        sj = np.ascontiguousarray(sj, dtype=np.int32)
        side = np.ascontiguousarray(side, dtype=np.uint8)
        act = C.c_longlong(0)
        loss = lib().orc_train_replay(self.h, _ip(si), _ip(sj), side.ctypes.data_as(C.POINTER(C.c_uint8)),
                                      len(si), C.byref(act))
        return loss, act.value

    def sample_stream(self, count):
        si = np.zeros(count, np.int32)
        sj = np.zeros(count, np.int32)
        side = np.zeros(count, np.uint8)
        lib().orc_sample_stream(self.h, count, _ip(si), _ip(sj), side.ctypes.data_as(C.POINTER(C.c_uint8)))
        return si, sj, side

    def batch_size(self):
        return lib().orc_batch_size(self.h)

    def energy(self, h, t, r):
        return lib().orc_triple_energy(self.h, h, t, r)

    def begin_batch(self):
        lib().orc_begin_batch(self.h)

    def gradient_update(self, h, t, r, corrupted):
        lib().orc_gradient_update(self.h, h, t, r, int(corrupted))

    def end_batch(self):
        lib().orc_end_batch(self.h)

    def evaluate(self, test, filt):
        test = np.ascontiguousarray(test, dtype=np.int32)
        filt = np.ascontiguousarray(filt, dtype=np.int32)
        cols = [np.ascontiguousarray(test[:, k]) for k in range(3)]
        fcols = [np.ascontiguousarray(filt[:, k]) for k in range(3)]
        out = np.zeros(5)
        lib().orc_evaluate(self.h, _ip(cols[0]), _ip(cols[1]), _ip(cols[2]), len(test),
                           _ip(fcols[0]), _ip(fcols[1]), _ip(fcols[2]), len(filt), _dp(out))
        return {"raw_rank": out[0], "raw_hits10": out[1], "filtered_rank": out[2], "filtered_hits10": out[3], "ties": int(out[4])}
