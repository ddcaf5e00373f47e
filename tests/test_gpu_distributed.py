"""bench.py's multi-GPU path (head-hash shards, per-epoch delta all-reduce,
renormalisation) with two ranks on the one GPU of a test box: torchrun, gloo
over device tensors (RCCL will not put two ranks on one device).  Checks that
both ranks train, merge and report one JSON line with the N = 2 fields."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["transe_fb15k", "transr_fb15k"])
def test_bench_two_ranks_one_device(config):
    env = dict(os.environ, KB2E_DIST_ONE_DEVICE="1", KB2E_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29517" if config == "transe_fb15k" else "29518", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "120", "--warmup", "10", "--config", config, "--only", "--no-cpu-baseline", "--no-epoch", "--seed-epochs", "3"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and d["config"]["global_batch"] == 2 * (d["config"]["global_batch"] // 2)
    assert 0.3 < d["active_fraction"] < 1.0
