"""Device init and text tables on the GPU.

* kb2e_init_params_device (Trainer::prepTrain, common/trainer.cpp:34-58, its
  randn rejection sampler common/utils.cpp:26-38) must produce the reference's
  initial tables bit for bit and leave the glibc stream at the same position:
  checked against the reference's own init fixtures, against the host init
  (itself pinned to those fixtures) at FB15k shape, and through the training
  epoch that follows (identical loss and active count).
* kb2e_format_table / kb2e_write_table must produce exactly the bytes of
  glibc's "%.6lf\\t" (common/trainer.cpp:109-127); Python's "%.6f" rounds the
  same way (exact binary value, ties to even).
* kb2e_read_table must give strtod's value for every token (Python float() is
  correctly rounded too) and fail like the reference on a short file.
"""
import math
import os
import time

import numpy as np
import pytest

from conftest import GOLDEN
from gpu_common import MANIFEST, tiny
from kb2e_amd import data
from kb2e_amd.engine import READ_SHRINK, READ_UNIT, READ_VERBATIM, Engine, EngineError

pytestmark = pytest.mark.gpu


def _engine(name, ds=None):
    run = MANIFEST["runs"][name]
    f = run["flags"]
    ds = ds or tiny()
    eng = Engine(run["model"], f["size"], ds.num_entities, ds.num_relations, rate=f["rate"], margin=f["margin"],
                 method=f["method"], distance=f["distance"], batches=f["batches"], seed=f["seed"],
                 transr_compat=not run["transr_fixed"])
    eng.upload_triples(ds.train)
    return eng, run, ds


@pytest.mark.parametrize("name", ["transe_l1_bern", "transe_l2_unif", "transh_bern", "transr_compat"])
def test_device_init_matches_reference(name):
    eng, run, ds = _engine(name)
    ent, rel, w, ties = eng.init_params_device()
    assert ties == 0
    d = os.path.join(GOLDEN, name)
    if run["model"] != "R":  # reference fixtures of the drawn tables (TransR's are overwritten by the seed)
        assert np.array_equal(ent, np.load(os.path.join(d, "init_ent.npy")))
        assert np.array_equal(rel, np.load(os.path.join(d, "init_rel.npy")))
    if run["model"] in ("H", "R"):
        assert np.array_equal(w, np.load(os.path.join(d, "init_w.npy")))
    host, _, _ = _engine(name)
    he, hr, hw = host.init_params()
    assert np.array_equal(ent, he) and np.array_equal(rel, hr)
    if hw is not None:
        assert np.array_equal(w, hw)
    # the stream continues at the same word
    assert [eng.rng_next() for _ in range(5)] == [host.rng_next() for _ in range(5)]


@pytest.mark.parametrize("name", ["transe_l1_bern", "transh_bern"])
def test_device_init_then_training_is_unchanged(name):
    eng, run, ds = _engine(name)
    eng.init_params_device(fetch=False)
    host, _, _ = _engine(name)
    host.init_params()
    for _ in range(2):
        assert eng.train_epoch() == host.train_epoch()
    a, b = eng.download_params(), host.download_params()
    for x, y in zip(a, b):
        if x is not None:
            assert np.array_equal(x, y)


@pytest.mark.parametrize("model,dim", [("E", 100), ("H", 100), ("R", 50)])
def test_device_init_fb15k_shape(model, dim):
    """~1.6M randn values (~160M glibc words at TransE's 2% acceptance) across
    several device chunks: bit-exact against the host init, same stream position."""
    ds = data.synthetic("fb15k", seed=0)
    engs = []
    for _ in range(2):
        e = Engine(model, dim, ds.num_entities, ds.num_relations, seed=7, batches=100)
        e.upload_triples(ds.train)
        engs.append(e)
    t0 = time.perf_counter()
    ent, rel, w, ties = engs[0].init_params_device()
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    he, hr, hw = engs[1].init_params()
    t_host = time.perf_counter() - t0
    print(f"init {model} n={dim}: device {t_dev:.3f} s, host {t_host:.3f} s, near ties {ties}")
    assert ties == 0
    assert np.array_equal(ent, he) and np.array_equal(rel, hr)
    if hw is not None:
        assert np.array_equal(w, hw)
    assert engs[0].rng_next() == engs[1].rng_next()


def _tricky_tables(rng, ne, nr, n):
    ent = rng.standard_normal((ne, n)) * 0.3
    rel = rng.standard_normal((nr, n))
    specials = np.array([0.0, -0.0, 0.0078125, -0.0234375, 5e-7, -5e-7, 4.9999999999999998e-7, 1e-9, -1e-9,
                         0.9999995, 123456.7890125, 2.0 ** 60, -(2.0 ** 70) + 3.0, 1e300, 5e-324, math.inf,
                         -math.inf, math.nan, 0.5e-6, 1.5e-6, 2.5e-6, 3.5e-6])
    flat = ent.reshape(-1)
    flat[: specials.size] = specials
    # exact ties at the sixth digit: (2k + 1) / 2^7, k odd and even
    rel.reshape(-1)[: 200] = (2.0 * np.arange(200) + 1) / 128.0 * np.where(np.arange(200) % 2, 1, -1)
    return ent, rel


def _printf(table):
    t = table.reshape(-1, table.shape[-1])
    return "".join("".join("%.6f\t" % v for v in row) + "\n" for row in t).encode()


def test_format_table_is_printf(tmp_path):
    ds = tiny()
    n = 20
    eng = Engine("H", n, ds.num_entities, ds.num_relations, seed=7, batches=10)
    rng = np.random.default_rng(3)
    ent, rel = _tricky_tables(rng, ds.num_entities, ds.num_relations, n)
    w = rng.standard_normal((ds.num_relations, n)) * 1e-3
    eng.upload_params(ent, rel, w)
    for table, arr in ((0, ent), (1, rel), (2, w)):
        want = _printf(arr)
        assert eng.format_table(table) == want
        path = tmp_path / f"t{table}.txt"
        eng.write_table(table, str(path))
        assert path.read_bytes() == want


def test_format_table_transr_weights_and_fp32(tmp_path):
    ds = tiny()
    n = 20
    eng = Engine("R", n, ds.num_entities, ds.num_relations, seed=7, batches=10, precision=32)
    eng.upload_triples(ds.train)
    eng.init_params_device(fetch=False)
    ent, rel, w = eng.download_params()  # FP32 tables widened to double, as the writer does
    assert eng.format_table(2) == _printf(w.reshape(-1, n))
    assert eng.format_table(0) == _printf(ent)


def test_read_table_is_strtod(tmp_path):
    ds = tiny()
    n = 20
    eng = Engine("E", n, ds.num_entities, ds.num_relations, seed=7, batches=10)
    rng = np.random.default_rng(5)
    toks = ["%.6f" % v for v in rng.standard_normal(ds.num_entities * n)]
    odd = ["1e-5", "+.5", "5.", "-0.000000", "12345678901234567890", "0.1234567890123456789012", "1e-400",
           "2.5E+3", "inf", "-inf", "1e400", "00012.5000", "9007199254740993", "0.30000000000000004441"]
    toks[: len(odd)] = odd
    text = ""
    for k, t in enumerate(toks):  # mixed separators, as fscanf accepts
        text += t + ("\n" if k % n == n - 1 else ("\t" if k % 3 else "  "))
    path = tmp_path / "ent.txt"
    path.write_text(text + "0.5 0.25\n")  # extra numbers after the table are ignored
    eng.read_table(0, str(path), READ_VERBATIM)
    got = eng.download_params()[0].reshape(-1)
    want = np.array([float(t) for t in toks])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))

    # a short file fails with the reference's message (transr/trainer.cpp:94-96)
    short = tmp_path / "short.txt"
    short.write_text(" ".join(toks[:-1]))
    with pytest.raises(EngineError, match="Failed to read embedding values from seed file"):
        eng.read_table(0, str(short), READ_VERBATIM)
    bad = tmp_path / "bad.txt"
    bad.write_text(" ".join(toks[:5] + ["abc"] + toks[6:]))
    with pytest.raises(EngineError):
        eng.read_table(0, str(bad), READ_VERBATIM)


def test_read_table_norm_modes_match_host_seed(tmp_path):
    """READ_UNIT is the TransR seed step's common::norm(row, false) (transr/
    trainer.cpp:99), READ_SHRINK the default common::norm (len > 1 only)."""
    ds = tiny()
    n = 20
    sd = os.path.join(GOLDEN, "transe_seed_unif")
    ent = data.read_table(os.path.join(sd, "entity2vec.unif"), ds.num_entities, n)
    rel = data.read_table(os.path.join(sd, "relation2vec.unif"), ds.num_relations, n)
    a = Engine("R", n, ds.num_entities, ds.num_relations, seed=7, batches=10)
    a.upload_triples(ds.train)
    a.init_params()
    a.transr_seed(ent, rel)  # host form
    b = Engine("R", n, ds.num_entities, ds.num_relations, seed=7, batches=10)
    b.upload_triples(ds.train)
    b.init_params_device(fetch=False)
    b.read_table(0, os.path.join(sd, "entity2vec.unif"), READ_UNIT)
    b.read_table(1, os.path.join(sd, "relation2vec.unif"), READ_VERBATIM)
    for x, y in zip(a.download_params(), b.download_params()):
        assert np.array_equal(x, y)
    big = tmp_path / "big.txt"
    data.write_table(str(big), ent * 3.0)
    b.read_table(0, str(big), READ_SHRINK)
    e3 = np.array(open(big).read().split(), dtype=np.float64).reshape(-1, n)
    lens = np.sqrt(np.array([sum(v * v for v in row) for row in e3]))  # sequential sum, as the reference
    want = np.where((lens > 1)[:, None], e3 / lens[:, None], e3)
    assert np.array_equal(b.download_params()[0], want)
