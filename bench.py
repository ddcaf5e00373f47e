#!/usr/bin/env python3
"""Throughput benchmark of the kb2e_amd training hot path (driver contract).

A "step" is one batch of Trainer::bfgs (common/trainer.cpp:75-100): floor(|train|
/ batches) samples, each = 1 training triple + 1 Bernoulli-corrupted triple,
scored, hinge-tested and applied with the reference's ordered norm updates.
Workload = BASELINE.json configs[1]: TransE n=100 bern on FB15k (synthetic
FB15k-shaped data, 14,951 entities / 1,345 relations / 483,142 triples), FP64
like the reference.  `value` = training triples (samples) per second over the
whole job, inputs resident in HBM; epochs' sampling + index build included.

N>1 (torchrun): weak scaling -- each rank owns the triples whose head hashes to
it and trains its shard; at every epoch boundary the ranks
average the tables over RCCL (kb2e_amd.distributed).
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.distributed import shard_heads  # noqa: E402

CONFIGS = {
    # name: (model, shape, dim, method, distance, rate)
    "transe_fb15k": ("E", "fb15k", 100, 1, 0, 0.001),
    "transh_fb15k": ("H", "fb15k", 100, 1, 0, 0.001),
    "transr_fb15k": ("R", "fb15k", 50, 1, 0, 0.001),
    "transe_wn18": ("E", "wn18", 50, 0, 0, 0.001),
}
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec


def algorithmic_bytes_per_sample(model, n, s, active_frac):
    """ids 12 B + filter probe 8 B, gathers of the rows read by
    the energies, read-modify-write of the rows an active update touches."""
    if model == "E":
        return 20 + 4 * n * s + active_frac * 8 * n * s, 20 + 4 * n * s, active_frac * 8 * n * s
    if model == "H":
        return 20 + 5 * n * s + active_frac * 10 * n * s, 20 + 5 * n * s, active_frac * 10 * n * s
    full = 20 + (n * n + 5 * n) * s + active_frac * (2 * n * n + 10 * n) * s
    return full, 20 + (n * n + 5 * n) * s, active_frac * (2 * n * n + 10 * n) * s


def _epoch_stamps(cmd, limit_s):
    """Run the reference on one core under a pseudo-terminal (so its stdout is
    line-buffered, as in a shell) and time-stamp each `Epoch:` line."""
    import pty
    import select

    master, slave = pty.openpty()
    try:
        os.sched_setaffinity(0, {min(os.sched_getaffinity(0))})
        pin = True
    except (AttributeError, OSError):
        pin = False
    p = subprocess.Popen(cmd, stdout=slave, stderr=subprocess.DEVNULL, close_fds=True)
    os.close(slave)
    stamps, buf, t0 = [], b"", time.time()
    try:
        while len(stamps) < 4 and time.time() - t0 < limit_s:
            r, _, _ = select.select([master], [], [], 1.0)
            if not r:
                if p.poll() is not None:
                    break
                continue
            try:
                chunk = os.read(master, 4096)
            except OSError:
                break
            if not chunk:
                break
            buf += chunk
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                if line.startswith(b"Epoch:"):
                    stamps.append(time.time())
    finally:
        p.kill()
        p.wait()
        os.close(master)
        if pin:
            os.sched_setaffinity(0, set(range(os.cpu_count() or 1)))
    return stamps


def cpu_baseline(cfg_name, ds, budget_s=25.0):
    """The reference itself (oracle/_ref, compiled from the reference sources)
    on this host, single-threaded, on the same synthetic dataset; falls back to
    the C restatement (oracle/liborc.so) when the binary is absent."""
    model, shape, dim, method, distance, rate = CONFIGS[cfg_name]
    binary = os.path.join(ROOT, "oracle", "_ref", {"E": "trainTransE", "H": "trainTransH", "R": "trainTransR"}[model])
    S = (len(ds.train) // 100) * 100
    if os.path.exists(binary) and model == "E":
        with tempfile.TemporaryDirectory() as d:
            data.write(ds, d)
            cmd = [binary, "--datadir", d, "--outdir", d, "--size", str(dim), "--epochs", "4", "--method",
                   str(method), "--distance", str(distance), "--rate", str(rate), "--seed", "7"]
            stamps = _epoch_stamps(cmd, budget_s * 2)
        if len(stamps) >= 2:
            per_epoch = (stamps[-1] - stamps[0]) / (len(stamps) - 1)  # epoch 0 (init) excluded
            return {"value": S / per_epoch, "unit": "triples/s", "cores": 1, "kind": "reference",
                    "sample": f"{len(stamps) - 1} steady epochs ({S} samples each) of {os.path.basename(binary)} "
                              f"on the same synthetic {shape}-shaped data, 1 thread (pinned to one core)"}
    from oracle import orc  # CPU restatement (port) fallback
    m = orc.Model(model, dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                  batches=100)
    m.set_triples(ds.train)
    orc.srand(7)
    m.prep_train()
    if model == "R":
        e, r, _ = m.tables()
        m.transr_seed(e, r)
    B = m.batch_size()
    t0 = time.time()
    nb = 0
    while time.time() - t0 < budget_s and nb < 100:
        m.train_batches(1)
        nb += 1
    dt = time.time() - t0
    return {"value": nb * B / dt, "unit": "triples/s", "cores": 1, "kind": "port",
            "sample": f"{nb} batches ({B} samples each) of the C restatement, 1 thread"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="transe_fb15k", choices=sorted(CONFIGS))
    ap.add_argument("--precision", type=int, default=64, choices=[32, 64])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        import torch

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from kb2e_amd.engine import Engine

    model, shape, dim, method, distance, rate = CONFIGS[args.config]
    ds = data.synthetic(shape, seed=0)
    train = shard_heads(ds.train, rank, world) if world > 1 else ds.train
    batches = 100
    eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                 batches=batches, seed=7 + rank, precision=args.precision, device=local if world > 1 else 0)
    eng.upload_triples(train)
    ent, rel, w = eng.init_params()
    if model == "R":
        eng.transr_seed(ent, rel)  # seed = the init draws (no TransE run in the bench)
    B = len(train) // batches
    merger = None
    if world > 1:
        from kb2e_amd.distributed import EpochMerger
        merger = EpochMerger(eng, dist)

    def run(steps):
        done = 0
        while done < steps:
            k = min(steps - done, batches - (run.pos % batches))
            eng.train_batches(k)
            done += k
            run.pos += k
            if merger is not None and run.pos % batches == 0:
                merger.merge()
    run.pos = 0

    run(args.warmup)
    eng.synchronize()
    eng.take_stats()
    eng.profile(True)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    run(args.steps)
    eng.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    loss, active = eng.take_stats()
    fold_ms, fold_n = eng.profile_query("fold" if model == "E" else "relowner")
    score_ms, score_n = eng.profile_query("score")
    samples = args.steps * B
    if dist is not None:
        import torch

        t = torch.tensor([elapsed, float(samples), float(active)], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        samples = float(t[1])
        active = float(t[2])
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    a = active / max(1.0, samples)
    s = 8 if args.precision == 64 else 4
    per_sample, score_bytes, fold_bytes = algorithmic_bytes_per_sample(model, dim, s, a)
    dominant = ("fold" if model == "E" else "relowner") if fold_ms >= score_ms else "score"
    if dominant == "score":
        avg_ms, bytes_per_launch = score_ms / max(1, score_n), score_bytes * B
    else:
        avg_ms, bytes_per_launch = fold_ms / max(1, fold_n), fold_bytes * B
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.config}_f{args.precision}.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(dominant, {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    out = {
        "metric": "training triples/sec (1/2/4/8 MI355X) + FB15k Hits@10(Filter)",
        "value": samples / elapsed,
        "unit": "triples/s (1 triple = 1 positive + 1 corrupted)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if args.precision == 64 else "f32",
        "data": f"synthetic {shape}-shaped (kb2e_amd.data.synthetic, seed 0), reference glibc sample stream seed 7",
        "config": {"workload": f"{args.config}: {'TransE' if model == 'E' else 'TransH' if model == 'H' else 'TransR'} "
                               f"n={dim} {'bern' if method else 'unif'} L{distance + 1}, {batches} batches of {B}",
                   "global_batch": B * world, "parallelism": f"dp{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "kernel": dominant,
                     "kernel_avg_us": avg_ms * 1e3, "algorithmic_bytes_per_launch": bytes_per_launch,
                     "step_achieved_GBs": per_sample * samples / elapsed / 1e9},
        "active_fraction": a,
    }
    if not args.no_cpu_baseline and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, ds)
        except Exception as e:  # the baseline is reported, never the target
            out["cpu_baseline"] = {"value": None, "error": str(e)}
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
