"""Drop-in check: the trainTransE/H/R binaries (C++ host over the C ABI) run
with the reference's flags on the reference's file formats and reproduce the
reference binaries' stdout epoch lines and %.6lf embedding files."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from gpu_common import MANIFEST, golden_engine

pytestmark = pytest.mark.gpu


def _run(tmp_path, prog, name, extra=()):
    run = MANIFEST["runs"][name]
    exe = tmp_path / prog
    if not exe.exists():
        exe.symlink_to(os.path.join(ROOT, "bin", "kb2e"))
    out = tmp_path / "out"
    out.mkdir(exist_ok=True)
    args = [str(exe), "--datadir", os.path.join(GOLDEN, "tiny"), "--outdir", str(out)]
    for k, v in run["flags"].items():
        args += ["--" + k, str(v)]
    args += list(extra)
    res = subprocess.run(args, capture_output=True, text=True, timeout=300, check=True)
    return res.stdout, out, run


def _epoch_lines(text):
    return [l for l in text.splitlines() if l.startswith("Epoch:")]


def _compare_files(out, name, files):
    for f in files:
        mine = np.array(open(out / f).read().split(), dtype=np.float64)
        ref = np.array(open(os.path.join(GOLDEN, name, f)).read().split(), dtype=np.float64)
        assert mine.shape == ref.shape
        # identical text except where an ulp difference crosses a 1e-6 rounding boundary
        assert np.abs(mine - ref).max() <= 1.000001e-6
        assert (mine != ref).sum() <= 2


def test_train_transe_cli(tmp_path):
    stdout, out, run = _run(tmp_path, "trainTransE", "transe_l1_bern")
    ref = open(os.path.join(GOLDEN, "transe_l1_bern", "stdout.txt")).read()
    assert _epoch_lines(stdout) == _epoch_lines(ref)
    assert "Number of Entities: 200" in stdout and "Options: [datadir:" in stdout
    _compare_files(out, "transe_l1_bern", ["entity2vec.bern", "relation2vec.bern"])


def test_train_transh_cli(tmp_path):
    stdout, out, run = _run(tmp_path, "trainTransH", "transh_bern")
    ref = open(os.path.join(GOLDEN, "transh_bern", "stdout.txt")).read()
    assert _epoch_lines(stdout) == _epoch_lines(ref)
    _compare_files(out, "transh_bern", ["entity2vec.bern", "relation2vec.bern", "weights.bern"])


def test_train_transr_cli(tmp_path):
    stdout, out, run = _run(tmp_path, "trainTransR", "transr_compat",
                            ["--seeddatadir", os.path.join(GOLDEN, "transe_seed_unif")])
    ref = open(os.path.join(GOLDEN, "transr_compat", "stdout.txt")).read()
    assert _epoch_lines(stdout) == _epoch_lines(ref)
    _compare_files(out, "transr_compat", ["entity2vec.bern", "relation2vec.bern", "weights.bern"])


def test_missing_seed_file_fails_like_reference(tmp_path):
    with pytest.raises(subprocess.CalledProcessError) as e:
        _run(tmp_path, "trainTransR", "transr_compat", ["--seeddatadir", str(tmp_path / "nowhere")])
    assert e.value.returncode == 1 and "Failed to read embedding values from seed file" in e.value.stdout


def test_eval_cli_matches_reference_eval(tmp_path):
    stdout, out, run = _run(tmp_path, "trainTransE", "transe_l1_bern")
    exe = tmp_path / "evalTransE"
    exe.symlink_to(os.path.join(ROOT, "bin", "kb2e"))
    f = run["flags"]
    res = subprocess.run([str(exe), "--datadir", os.path.join(GOLDEN, "tiny"), "--outdir",
                          os.path.join(GOLDEN, "transe_l1_bern"), "--size", str(f["size"]), "--method",
                          str(f["method"]), "--distance", str(f["distance"])],
                         capture_output=True, text=True, timeout=300, check=True)
    lines = {l.split("--")[0].strip(): l for l in res.stdout.splitlines() if "Hits@10" in l}
    ev = run["eval"]
    assert lines["Raw"] == "Raw      -- Rank: %f, Hits@10: %f" % (ev["raw"]["rank"], ev["raw"]["hits10"])
    assert lines["Filtered"] == "Filtered -- Rank: %f, Hits@10: %f" % (ev["filtered"]["rank"], ev["filtered"]["hits10"])


@pytest.mark.parametrize("prog,name", [("trainTransE", "transe_l1_bern"), ("trainTransH", "transh_bern")])
def test_train_cli_parallel_schedule(tmp_path, prog, name):
    """--schedule 1: the PARALLEL schedule behind the same CLI and file formats.
    The CLI's epoch lines and %.6lf files are the library's PARALLEL run of the
    same flags (tests/test_gpu_parallel.py ties that run to oracle/parallel.py,
    test_gpu_hits_parity.py to the reference's Hits@10); the losses stay close
    to the reference's (the schedule differs from it at O(lr^2) per row with
    several updates a batch)."""
    stdout, out, run = _run(tmp_path, prog, name, ["--schedule", "1"])
    ref = open(os.path.join(GOLDEN, name, "stdout.txt")).read()
    mine, theirs = _epoch_lines(stdout), _epoch_lines(ref)
    assert len(mine) == len(theirs) == run["flags"]["epochs"]
    lm = np.array([float(l.split("Loss:")[1]) for l in mine])
    lr = np.array([float(l.split("Loss:")[1]) for l in theirs])
    assert np.all(np.abs(lm - lr) <= 0.05 * np.abs(lr) + 1.0)
    eng, run, ds, _ = golden_engine(name, schedule="parallel")
    for ep in range(run["flags"]["epochs"]):
        loss, _ = eng.train_epoch()
        assert abs(loss - lm[ep]) <= 1e-6 * max(1.0, abs(loss)) + 5e-7, (ep, loss, mine[ep])
    tabs = dict(zip(["entity2vec.bern", "relation2vec.bern", "weights.bern"], eng.download_params()))
    for f, t in tabs.items():
        if t is None:
            continue
        a = np.array(open(out / f).read().split(), dtype=np.float64)
        b = np.array(open(os.path.join(GOLDEN, name, f)).read().split(), dtype=np.float64)
        assert a.shape == b.shape == (t.size,) and np.isfinite(a).all()
        # the library's tables as printed with %.6lf (summation order of the
        # parallel row sums may move an entry by an ulp across a rounding edge)
        assert np.abs(a - t.reshape(-1)).max() <= 1.000001e-6, f
        # (closeness to the reference's own tables is the loss check above: on
        # this tiny set each relation takes ~40 updates a batch, the relaxation's
        # worst case, and its Hits@10 parity is test_gpu_hits_parity.py's)


def test_eval_transr_cli_compat(tmp_path):
    """bin/evalTransR on the reference's transr_compat output files: the stateful
    compat energy (the reference evalTransR's), printed as the reference prints
    it; equal to the reference's lines up to the exact ties of that run."""
    from gpu_common import tiny
    from kb2e_amd import data
    from kb2e_amd.engine import Engine

    run = MANIFEST["runs"]["transr_compat"]
    f = run["flags"]
    d = os.path.join(GOLDEN, "transr_compat")
    exe = tmp_path / "evalTransR"
    exe.symlink_to(os.path.join(ROOT, "bin", "kb2e"))
    res = subprocess.run([str(exe), "--datadir", os.path.join(GOLDEN, "tiny"), "--outdir", d, "--size",
                          str(f["size"]), "--method", str(f["method"]), "--distance", str(f["distance"])],
                         capture_output=True, text=True, timeout=300, check=True)
    lines = {l.split("--")[0].strip().split("\r")[-1]: l for l in res.stdout.splitlines() if "Hits@10" in l}
    got = {k: [float(x.split(":")[1]) for x in v.split("--")[1].split(",")] for k, v in lines.items()}
    ds = tiny()
    n = f["size"]
    eng = Engine("R", n, ds.num_entities, ds.num_relations)
    eng.upload_params(data.read_table(os.path.join(d, "entity2vec.bern"), ds.num_entities, n),
                      data.read_table(os.path.join(d, "relation2vec.bern"), ds.num_relations, n),
                      data.read_table(os.path.join(d, "weights.bern"), ds.num_relations * n, n).reshape(-1, n, n))
    mine = eng.evaluate_transr_compat(ds.test, np.concatenate([ds.test, ds.train, ds.valid]))
    assert got["Raw"] == pytest.approx([mine["raw_rank"], mine["raw_hits10"]], abs=5e-7)
    assert got["Filtered"] == pytest.approx([mine["filtered_rank"], mine["filtered_hits10"]], abs=5e-7)
    ev, n2 = run["eval"], 2 * len(ds.test)
    assert abs(got["Filtered"][0] - ev["filtered"]["rank"]) * n2 <= mine["ties"] + 1e-3
    assert abs(got["Raw"][0] - ev["raw"]["rank"]) * n2 <= mine["ties"] + 1e-3
    assert "Processed 100.00%" in res.stdout
