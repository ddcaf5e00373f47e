"""The reference-side binding (integration/gpu_trainer.h): the reference's own
trainer classes, compiled from /root/reference's headers and objects
(oracle/_ref/common.a), with bfgs() running on the engine through the C ABI.
Epoch lines must equal the reference binaries' and the %.6lf files must be the
reference's text (common/trainer.cpp:109-127, transh/trainer.cpp:94-105,
transr/trainer.cpp:128-142; up to <= 2 values on a 1e-6 rounding boundary)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from gpu_common import MANIFEST

BIN = os.path.join(ROOT, "bin", "binding")


def _run(tmp_path, prog, name, extra=(), env=None, check=True):
    exe = os.path.join(BIN, prog)
    if not os.path.exists(exe):
        pytest.skip("binding not built (make binding needs /root/reference)")
    run = MANIFEST["runs"][name]
    out = tmp_path / "out"
    out.mkdir(exist_ok=True)
    args = [exe, "--datadir", os.path.join(GOLDEN, "tiny"), "--outdir", str(out)]
    for k, v in run["flags"].items():
        args += ["--" + k, str(v)]
    args += list(extra)
    res = subprocess.run(args, capture_output=True, text=True, timeout=300, check=check,
                         env=dict(os.environ, **(env or {})))
    return res, out


def _epoch_lines(text):
    return [ln for ln in text.splitlines() if ln.startswith("Epoch:")]


def _compare_files(out, name, files):
    for f in files:
        mine = np.array(open(out / f).read().split(), dtype=np.float64)
        ref = np.array(open(os.path.join(GOLDEN, name, f)).read().split(), dtype=np.float64)
        assert mine.shape == ref.shape
        assert np.abs(mine - ref).max() <= 1.000001e-6
        assert (mine != ref).sum() <= 2


CASES = [("trainTransE", "transe_l1_bern", [], ["entity2vec.bern", "relation2vec.bern"]),
         ("trainTransE", "transe_l2_unif", [], ["entity2vec.unif", "relation2vec.unif"]),
         ("trainTransH", "transh_bern", [], ["entity2vec.bern", "relation2vec.bern", "weights.bern"]),
         ("trainTransR", "transr_compat", ["--seeddatadir", os.path.join(GOLDEN, "transe_seed_unif")],
          ["entity2vec.bern", "relation2vec.bern", "weights.bern"])]


@pytest.mark.gpu
@pytest.mark.parametrize("prog,name,extra,files", CASES)
def test_binding_matches_reference_run(tmp_path, prog, name, extra, files):
    res, out = _run(tmp_path, prog, name, extra)
    ref = open(os.path.join(GOLDEN, name, "stdout.txt")).read()
    assert _epoch_lines(res.stdout) == _epoch_lines(ref)
    assert "Options: [" in res.stdout
    _compare_files(out, name, files)


@pytest.mark.gpu
def test_binding_transr_fixed(tmp_path):
    res, out = _run(tmp_path, "trainTransR", "transr_fixed",
                    ["--seeddatadir", os.path.join(GOLDEN, "transe_seed_unif")], env={"KB2E_TRANSR_FIXED": "1"})
    ref = open(os.path.join(GOLDEN, "transr_fixed", "stdout.txt")).read()
    assert _epoch_lines(res.stdout) == _epoch_lines(ref)
    _compare_files(out, "transr_fixed", ["entity2vec.bern", "relation2vec.bern", "weights.bern"])


def test_binding_fails_loudly_without_engine(tmp_path):
    """CPU box: the reference's parse/load/init run, then kb2e_create reports
    the missing GPU the reference's way (message + exit(1))."""
    if os.path.exists("/dev/kfd"):  # a GPU box: the engine would start
        pytest.skip("GPU present")
    res, out = _run(tmp_path, "trainTransE", "transe_l1_bern", check=False)
    assert res.returncode == 1, res.stdout
    assert "kb2e_create failed" in res.stdout and "Number of Entities: 200" in res.stdout
