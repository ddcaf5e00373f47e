"""ctypes binding of libkb2e.so (include/kb2e_engine.h).

This is the product path for Python callers (bench.py, tests): every call goes
through the C ABI into the HIP engine.  There is no CPU fallback -- if the
library or a GPU is missing, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KB2E_LIB") or os.path.join(HERE, "libkb2e.so")

MODELS = {"transe": 0, "transh": 1, "transr": 2, "E": 0, "H": 1, "R": 2}
STATUS = {0: "OK", 1: "EINVAL", 2: "EDEVICE", 3: "ESTATE", 4: "ENOMEM", 5: "EUNSUPPORTED", 6: "ESAMPLER"}
SAMPLER_GLIBC, SAMPLER_REPLAY = 0, 1
SCHEDULES = {"ordered": 0, "parallel": 1}

# Every symbol include/kb2e_engine.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "kb2e_default_config", "kb2e_create", "kb2e_destroy", "kb2e_last_error", "kb2e_upload_triples",
    "kb2e_init_params", "kb2e_transr_seed", "kb2e_upload_params", "kb2e_download_params", "kb2e_get_transr_work",
    "kb2e_set_transr_work", "kb2e_set_sample_stream", "kb2e_get_sample_stream", "kb2e_train_epoch", "kb2e_train_batches",
    "kb2e_synchronize", "kb2e_take_stats", "kb2e_rng_next", "kb2e_profile_enable", "kb2e_profile_query", "kb2e_counter",
    "kb2e_device_bytes", "kb2e_device_tables", "kb2e_renormalize", "kb2e_evaluate", "kb2e_evaluate_transr_compat",
    "kb2e_renormalize_rows", "kb2e_init_params_device", "kb2e_write_table", "kb2e_format_table",
    "kb2e_read_table", "kb2e_comm_unique_id", "kb2e_comm_init_rank", "kb2e_comm_init_group", "kb2e_merge_epoch",
    "kb2e_merge_epoch_group", "kb2e_comm_info", "kb2e_get_config",
]
COMM_ID_BYTES = 128
READ_VERBATIM, READ_UNIT, READ_SHRINK = 0, 1, 2


class Config(C.Structure):
    _fields_ = [
        ("model", C.c_int32), ("dim", C.c_int32), ("num_entities", C.c_int32), ("num_relations", C.c_int32),
        ("learning_rate", C.c_double), ("margin", C.c_double), ("method", C.c_int32), ("distance", C.c_int32),
        ("num_batches", C.c_int32), ("seed", C.c_uint32), ("precision", C.c_int32), ("sampler", C.c_int32),
        ("transr_compat", C.c_int32), ("device", C.c_int32), ("schedule", C.c_int32), ("sub_batches", C.c_int32),
    ]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"kb2e HIP engine not built: {LIB_PATH} missing (run `make`)")
        L = C.CDLL(LIB_PATH)
        vp, i32, i64, dp = C.c_void_p, C.c_int32, C.c_int64, C.POINTER(C.c_double)
        i32p, u8p = C.POINTER(C.c_int32), C.POINTER(C.c_uint8)
        sig = {
            "kb2e_default_config": (None, [C.POINTER(Config)]),
            "kb2e_create": (i32, [C.POINTER(Config), C.POINTER(vp)]),
            "kb2e_get_config": (i32, [vp, C.POINTER(Config)]),
            "kb2e_destroy": (None, [vp]),
            "kb2e_last_error": (C.c_char_p, [vp]),
            "kb2e_upload_triples": (i32, [vp, i32p, i32p, i32p, i64]),
            "kb2e_init_params": (i32, [vp, dp, dp, dp]),
            "kb2e_init_params_device": (i32, [vp, dp, dp, dp, C.POINTER(i64)]),
            "kb2e_write_table": (i32, [vp, i32, C.c_char_p]),
            "kb2e_format_table": (i32, [vp, i32, C.c_char_p, i64, C.POINTER(i64)]),
            "kb2e_read_table": (i32, [vp, i32, C.c_char_p, i32]),
            "kb2e_upload_params": (i32, [vp, dp, dp, dp]),
            "kb2e_transr_seed": (i32, [vp, dp, dp]),
            "kb2e_download_params": (i32, [vp, dp, dp, dp]),
            "kb2e_get_transr_work": (i32, [vp, dp, dp]),
            "kb2e_set_transr_work": (i32, [vp, dp, dp]),
            "kb2e_set_sample_stream": (i32, [vp, i32p, i32p, u8p, i64]),
            "kb2e_get_sample_stream": (i32, [vp, i32p, i32p, u8p, i64]),
            "kb2e_train_epoch": (i32, [vp, dp, C.POINTER(i64)]),
            "kb2e_train_batches": (i32, [vp, i32]),
            "kb2e_synchronize": (i32, [vp]),
            "kb2e_take_stats": (i32, [vp, dp, C.POINTER(i64)]),
            "kb2e_rng_next": (i32, [vp]),
            "kb2e_profile_enable": (i32, [vp, i32]),
            "kb2e_profile_query": (i32, [vp, C.c_char_p, dp, C.POINTER(i64)]),
            "kb2e_device_bytes": (i64, [vp]),
            "kb2e_counter": (i32, [vp, C.c_char_p, C.POINTER(i64)]),
            "kb2e_device_tables": (i32, [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(i64),
                                         C.POINTER(i64), C.POINTER(i64)]),
            "kb2e_renormalize": (i32, [vp, u8p, u8p, u8p]),
            "kb2e_renormalize_rows": (i32, [vp, i32, i64, i64, vp]),
            "kb2e_evaluate": (i32, [vp, i32p, i32p, i32p, i64, i32p, i32p, i32p, i64, dp]),
            "kb2e_evaluate_transr_compat": (i32, [vp, i32p, i32p, i32p, i64, i32p, i32p, i32p, i64, dp, dp, vp,
                                                  vp]),
            "kb2e_comm_unique_id": (i32, [u8p]),
            "kb2e_comm_init_rank": (i32, [vp, i32, i32, u8p]),
            "kb2e_comm_init_group": (i32, [C.POINTER(vp), i32]),
            "kb2e_merge_epoch": (i32, [vp]),
            "kb2e_merge_epoch_group": (i32, [C.POINTER(vp), i32]),
            "kb2e_comm_info": (i32, [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i64), C.POINTER(i64)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


class EngineError(RuntimeError):
    pass


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


class Engine:
    """One training context on one GPU (the drop-in for Trainer::bfgs)."""

    def __init__(self, model, dim, num_entities, num_relations, *, rate=0.001, margin=1.0, method=1,
                 distance=0, batches=100, seed=0, precision=64, sampler=SAMPLER_GLIBC, transr_compat=True,
                 device=0, schedule="ordered", sub_batches=None):
        self.kind = MODELS[model] if isinstance(model, str) else int(model)
        self.n, self.ne, self.nr = dim, num_entities, num_relations
        cfg = Config()
        lib().kb2e_default_config(C.byref(cfg))
        cfg.model, cfg.dim, cfg.num_entities, cfg.num_relations = self.kind, dim, num_entities, num_relations
        cfg.learning_rate, cfg.margin, cfg.method, cfg.distance = rate, margin, method, distance
        cfg.num_batches, cfg.seed, cfg.precision, cfg.sampler = batches, seed, precision, sampler
        cfg.transr_compat, cfg.device = int(transr_compat), device
        cfg.schedule = SCHEDULES[schedule] if isinstance(schedule, str) else int(schedule)
        if sub_batches is not None:  # (None: the engine's default by width, kb2e_default_config)
            cfg.sub_batches = int(sub_batches)
        h = C.c_void_p()
        st = lib().kb2e_create(C.byref(cfg), C.byref(h))
        if st != 0:
            raise EngineError(f"kb2e_create failed: {STATUS.get(st, st)}")
        self.h = h
        self.cfg = Config()  # the context's own, defaults resolved (kb2e_get_config)
        self._check(lib().kb2e_get_config(self.h, C.byref(self.cfg)), "kb2e_get_config")

    def _check(self, st, what):
        if st != 0:
            msg = lib().kb2e_last_error(self.h)
            raise EngineError(f"{what}: {STATUS.get(st, st)}: {msg.decode() if msg else ''}")

    def close(self):
        if getattr(self, "h", None):
            lib().kb2e_destroy(self.h)
            self.h = None

    __del__ = close

    def wshape(self):
        return {0: None, 1: (self.nr, self.n), 2: (self.nr, self.n, self.n)}[self.kind]

    def upload_triples(self, triples):
        t = np.ascontiguousarray(triples, dtype=np.int32)
        cols = [np.ascontiguousarray(t[:, k]) for k in range(3)]
        self._check(lib().kb2e_upload_triples(self.h, _ip(cols[0]), _ip(cols[1]), _ip(cols[2]), len(t)),
                    "upload_triples")

    def init_params(self):
        ent = np.zeros((self.ne, self.n))
        rel = np.zeros((self.nr, self.n))
        w = np.zeros(self.wshape()) if self.wshape() else None
        self._check(lib().kb2e_init_params(self.h, _dp(ent), _dp(rel), _dp(w)), "init_params")
        return ent, rel, w

    def init_params_device(self, fetch=True):
        """Trainer::prepTrain's draws made on the device (same values, same rng
        position); returns (ent, rel, w, near_ties), the tables None if not fetched."""
        ties = C.c_int64(0)
        if not fetch:
            self._check(lib().kb2e_init_params_device(self.h, None, None, None, C.byref(ties)), "init_params_device")
            return None, None, None, ties.value
        ent = np.zeros((self.ne, self.n))
        rel = np.zeros((self.nr, self.n))
        w = np.zeros(self.wshape()) if self.wshape() else None
        self._check(lib().kb2e_init_params_device(self.h, _dp(ent), _dp(rel), _dp(w), C.byref(ties)),
                    "init_params_device")
        return ent, rel, w, ties.value

    def write_table(self, table, path):
        """The device table (0 entities, 1 relations, 2 weights) as the reference's "%.6lf\\t" text file."""
        self._check(lib().kb2e_write_table(self.h, int(table), os.fsencode(path)), "write_table")

    def format_table(self, table):
        need = C.c_int64(0)
        lib().kb2e_format_table(self.h, int(table), None, 0, C.byref(need))
        buf = C.create_string_buffer(max(1, need.value))
        self._check(lib().kb2e_format_table(self.h, int(table), buf, need.value, C.byref(need)), "format_table")
        return buf.raw[:need.value]

    def read_table(self, table, path, mode=READ_VERBATIM):
        """Load a device table from "%lf" text (parsed on the device); mode: READ_VERBATIM / READ_UNIT / READ_SHRINK."""
        self._check(lib().kb2e_read_table(self.h, int(table), os.fsencode(path), int(mode)), "read_table")

    def transr_seed(self, ent, rel):
        ent = np.ascontiguousarray(ent, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        self._check(lib().kb2e_transr_seed(self.h, _dp(ent), _dp(rel)), "transr_seed")

    def upload_params(self, ent, rel, w=None):
        ent = np.ascontiguousarray(ent, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
        self._check(lib().kb2e_upload_params(self.h, _dp(ent), _dp(rel), _dp(w)), "upload_params")

    def download_params(self):
        ent = np.zeros((self.ne, self.n))
        rel = np.zeros((self.nr, self.n))
        w = np.zeros(self.wshape()) if self.wshape() else None
        self._check(lib().kb2e_download_params(self.h, _dp(ent), _dp(rel), _dp(w)), "download_params")
        return ent, rel, w

    def transr_work(self):
        a, b = np.zeros(self.n), np.zeros(self.n)
        self._check(lib().kb2e_get_transr_work(self.h, _dp(a), _dp(b)), "get_transr_work")
        return a, b

    def set_transr_work(self, a, b):
        a = np.ascontiguousarray(a, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
        self._check(lib().kb2e_set_transr_work(self.h, _dp(a), _dp(b)), "set_transr_work")

    def set_sample_stream(self, si, sj, side):
        si = np.ascontiguousarray(si, dtype=np.int32)
        sj = np.ascontiguousarray(sj, dtype=np.int32)
        side = np.ascontiguousarray(side, dtype=np.uint8)
        self._keep = (si, sj, side)
        self._check(lib().kb2e_set_sample_stream(self.h, _ip(si), _ip(sj),
                                                 side.ctypes.data_as(C.POINTER(C.c_uint8)), len(si)),
                    "set_sample_stream")

    def sample_stream(self, count):
        si = np.zeros(count, np.int32)
        sj = np.zeros(count, np.int32)
        side = np.zeros(count, np.uint8)
        self._check(lib().kb2e_get_sample_stream(self.h, _ip(si), _ip(sj), side.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                 count), "get_sample_stream")
        return si, sj, side

    # ------------------------------------------------ multi-GPU epoch merge
    @staticmethod
    def comm_unique_id():
        """A fresh RCCL id (bytes) for kb2e_comm_init_rank; made on one rank, handed to all."""
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        st = lib().kb2e_comm_unique_id(buf)
        if st != 0:
            raise EngineError(f"kb2e_comm_unique_id failed: {STATUS.get(st, st)}")
        return bytes(buf)

    def comm_init_rank(self, nranks, rank, comm_id):
        """Join the RCCL communicator (collective); rank 0's tables are broadcast."""
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(bytes(comm_id))
        self._check(lib().kb2e_comm_init_rank(self.h, int(nranks), int(rank), buf), "comm_init_rank")

    def merge_epoch(self):
        """T <- renorm(T0 + sum_r (T_r - T0)) over the communicator (collective)."""
        self._check(lib().kb2e_merge_epoch(self.h), "merge_epoch")

    def comm_info(self):
        n, r = C.c_int32(), C.c_int32()
        lo, cnt = C.c_int64(), C.c_int64()
        self._check(lib().kb2e_comm_info(self.h, C.byref(n), C.byref(r), C.byref(lo), C.byref(cnt)), "comm_info")
        return n.value, r.value, lo.value, cnt.value

    def train_epoch(self):
        loss = C.c_double(0)
        act = C.c_int64(0)
        self._check(lib().kb2e_train_epoch(self.h, C.byref(loss), C.byref(act)), "train_epoch")
        return loss.value, act.value

    def train_batches(self, nb):
        self._check(lib().kb2e_train_batches(self.h, int(nb)), "train_batches")

    def synchronize(self):
        self._check(lib().kb2e_synchronize(self.h), "synchronize")

    def take_stats(self):
        loss = C.c_double(0)
        act = C.c_int64(0)
        self._check(lib().kb2e_take_stats(self.h, C.byref(loss), C.byref(act)), "take_stats")
        return loss.value, act.value

    def rng_next(self):
        return lib().kb2e_rng_next(self.h)

    def profile(self, on=True):
        """on: False/0 off, True/1 every batch, P > 1 every P-th batch."""
        self._check(lib().kb2e_profile_enable(self.h, int(on)), "profile_enable")

    def profile_query(self, name):
        ms = C.c_double(0)
        n = C.c_int64(0)
        self._check(lib().kb2e_profile_query(self.h, name.encode(), C.byref(ms), C.byref(n)), "profile_query")
        return ms.value, n.value

    def counter(self, name):
        """A device-side schedule counter (include/kb2e_engine.h kb2e_counter)."""
        v = C.c_int64(0)
        self._check(lib().kb2e_counter(self.h, name.encode(), C.byref(v)), "counter")
        return v.value

    def renormalize(self, ent_rows=None, rel_rows=None, w_rows=None):
        keep = [None if m is None else np.ascontiguousarray(m, dtype=np.uint8) for m in (ent_rows, rel_rows, w_rows)]
        ptrs = [None if m is None else m.ctypes.data_as(C.POINTER(C.c_uint8)) for m in keep]
        self._check(lib().kb2e_renormalize(self.h, *ptrs), "renormalize")

    def renormalize_rows(self, table, first, count, device_mask_ptr=None):
        """Norm constraint on rows [first, first + count) of table 0/1/2, mask in device memory."""
        self._check(lib().kb2e_renormalize_rows(self.h, int(table), int(first), int(count), device_mask_ptr),
                    "renormalize_rows")

    def evaluate(self, test, filt):
        """Link prediction (raw/filtered mean rank and hits@10) on the device tables."""
        test = np.ascontiguousarray(test, dtype=np.int32)
        filt = np.ascontiguousarray(filt, dtype=np.int32)
        tc = [np.ascontiguousarray(test[:, k]) for k in range(3)]
        fc = [np.ascontiguousarray(filt[:, k]) for k in range(3)]
        out = np.zeros(4)
        self._check(lib().kb2e_evaluate(self.h, _ip(tc[0]), _ip(tc[1]), _ip(tc[2]), len(test), _ip(fc[0]),
                                        _ip(fc[1]), _ip(fc[2]), len(filt), _dp(out)), "evaluate")
        return {"raw_rank": out[0], "raw_hits10": out[1], "filtered_rank": out[2], "filtered_hits10": out[3]}

    def evaluate_transr_compat(self, test, filt, work=None):
        """TransR link prediction with the reference evalTransR's accumulating
        energy work vectors; returns the ranks plus "ties" and the final "work"."""
        test = np.ascontiguousarray(test, dtype=np.int32)
        filt = np.ascontiguousarray(filt, dtype=np.int32)
        tc = [np.ascontiguousarray(test[:, k]) for k in range(3)]
        fc = [np.ascontiguousarray(filt[:, k]) for k in range(3)]
        w = np.zeros(2 * self.n) if work is None else np.ascontiguousarray(work, dtype=np.float64).reshape(-1).copy()
        out = np.zeros(5)
        self._check(lib().kb2e_evaluate_transr_compat(self.h, _ip(tc[0]), _ip(tc[1]), _ip(tc[2]), len(test),
                                                      _ip(fc[0]), _ip(fc[1]), _ip(fc[2]), len(filt), _dp(w),
                                                      _dp(out), None, None), "evaluate_transr_compat")
        return {"raw_rank": out[0], "raw_hits10": out[1], "filtered_rank": out[2], "filtered_hits10": out[3],
                "ties": int(out[4]), "work": w.reshape(2, self.n)}

    def device_bytes(self):
        return lib().kb2e_device_bytes(self.h)


def _handles(engines):
    arr = (C.c_void_p * len(engines))(*[e.h for e in engines])
    return arr


def comm_init_group(engines):
    """One host thread driving every engine (kb2e_comm_init_group): RCCL over the
    engines' devices, or the local kernel backend when they share a device."""
    st = lib().kb2e_comm_init_group(_handles(engines), len(engines))
    if st != 0:
        raise EngineError(f"comm_init_group: {STATUS.get(st, st)}: {lib().kb2e_last_error(engines[0].h).decode()}")


def merge_epoch_group(engines):
    st = lib().kb2e_merge_epoch_group(_handles(engines), len(engines))
    if st != 0:
        raise EngineError(f"merge_epoch_group: {STATUS.get(st, st)}: {lib().kb2e_last_error(engines[0].h).decode()}")
