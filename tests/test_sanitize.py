"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer,
no GPU: the drop-in CLI's argument parser and file loader
(kb2e_amd/csrc/host/kb2e_cli.cpp: common/args.cpp:53-122, common/loader.cpp:
15-62), the host triple store and sample stream (host_data.hpp:
common/trainer.cpp:79-98, pinned to the oracle's stream), the "%.6lf" / "%lf"
text code (textio.hpp) and the Bloom prefilter.  Each is built here with
g++ -fsanitize=address,undefined -fno-sanitize-recover=all, so any finding
fails the run.  (`make sanitize` builds the same, plus the engine library with
its host code instrumented for the GPU box: tools/gpu_sanitize.sh.)"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from kb2e_amd import data

SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
       "-std=c++17"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
TINY = os.path.join(GOLDEN, "tiny")


def _build(tmp, name, src, extra):
    exe = str(tmp / name)
    subprocess.run(["g++", *SAN, *extra, "-o", exe, os.path.join(ROOT, "tests", "native", src)], check=True,
                   capture_output=True)
    return exe


def _run(args, timeout=120):
    out = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr[-3000:]
    return out


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    lib = os.path.join(ROOT, "kb2e_amd")
    if not os.path.exists(os.path.join(lib, "libkb2e.so")):
        pytest.fail("build first (make): host_check links libkb2e.so for the CLI's engine calls")
    return _build(tmp_path_factory.mktemp("san"), "host_check", "host_check.cpp",
                  ["-I" + os.path.join(ROOT, "include"), "-L" + lib, "-lkb2e", "-Wl,-rpath," + lib])


def test_cli_arguments(host_check):
    out = _run([host_check, "args"])
    assert out.returncode == 0
    line = out.stdout.strip()
    # the reference's defaults (common/constants.h:28-40) and its Options line (common/args.cpp:33-50)
    assert line.startswith("Options: [datadir: '../data', outdir: '.', size: 100, rate: 0.001000, margin: 1.000000, "
                           "method: bern, batches: 100, epochs: 1000, distance: 0, seeddatadir: '.', seedmethod: unif")
    assert line.endswith("precision 64 device 0 transrcompat 1 schedule 0 gpus 1")
    out = _run([host_check, "args", "--size", "50", "-rate", "0.01", "--method", "0", "--seed", "7", "--epochs", "3",
                "--seeddatadir", "x" * 700, "--schedule", "5", "--gpus", "0", "--transrcompat", "0"])
    assert out.returncode == 0
    assert "size: 50, rate: 0.010000" in out.stdout and "method: unif" in out.stdout and "seed: 7]" in out.stdout
    assert "seeddatadir: '" + "x" * 700 + "'" in out.stdout
    assert out.stdout.strip().endswith("transrcompat 0 schedule 1 gpus 1")
    out = _run([host_check, "args", "--size"])  # every flag needs a value (common/utils.cpp:55-68)
    assert out.returncode == 1 and "Argument missing for size" in out.stdout
    out = _run([host_check, "args", "--help"])
    assert out.returncode == 0 and out.stdout.startswith("USAGE: ")


def test_loader_matches_python(host_check, tmp_path):
    out = _run([host_check, "load", TINY])
    assert out.returncode == 0
    ne, nr, nt, _ = out.stdout.split()
    ds = data.load(TINY)
    assert (int(ne), int(nr), int(nt)) == (ds.num_entities, ds.num_relations, len(ds.train))
    # unknown names are reported and skipped (common/loader.cpp:40-57); an over-long
    # token must not overflow the loader's buffers
    d = tmp_path / "bad"
    d.mkdir()
    (d / "entity2id.txt").write_text("a\t0\nb\t1\n" + "c" * 900 + "\t2\n")
    (d / "relation2id.txt").write_text("r\t0\n")
    (d / "train.txt").write_text("a\tb\tr\na\tzz\tr\n" + "q" * 2000 + "\ta\tr\nb\ta\tr\n")
    out = _run([host_check, "load", str(d)])
    assert out.returncode == 0, out.stdout + out.stderr
    assert "not found in the identity file: zz" in out.stdout


@pytest.mark.parametrize("method", [1, 0])
def test_host_stream_matches_oracle(host_check, method):
    """The host sampler (the CLI's KB2E_HOST_SAMPLER path) draws the reference's
    glibc stream: same (i, j, side) as the oracle (oracle/orc.c, pinned to the
    reference by tests/test_oracle_golden.py)."""
    from oracle import orc
    ds = data.load(TINY)
    count = 3000
    out = _run([host_check, "stream", TINY, "7", str(count), str(method)])
    assert out.returncode == 0
    got = np.array(out.stdout.split(), dtype=np.int64).reshape(count, 3)
    m = orc.Model("E", 10, ds.num_entities, ds.num_relations, rate=0.01, method=method, batches=1)
    m.set_triples(ds.train)
    orc.srand(7)
    si, sj, side = m.sample_stream(count)
    assert np.array_equal(got[:, 0], si) and np.array_equal(got[:, 1], sj) and np.array_equal(got[:, 2], side)


def test_textio_and_bloom_under_sanitizers(tmp_path):
    exe = _build(tmp_path, "textio_check", "textio_check.cpp", ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"])
    out = _run([exe, "30000", "3"])
    assert out.returncode == 0 and out.stdout.startswith("ok "), out.stdout
    exe = _build(tmp_path, "bloom_check", "bloom_check.cpp", ["-I" + os.path.join(ROOT, "kb2e_amd", "csrc")])
    out = _run([exe, "20000"])
    assert out.returncode == 0, out.stdout
