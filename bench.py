#!/usr/bin/env python3
"""Throughput benchmark of the kb2e_amd training hot path (driver contract).

A "step" is one batch of Trainer::bfgs (common/trainer.cpp:75-100): floor(|train|
/ batches) samples, each = 1 training triple + 1 Bernoulli-corrupted triple,
scored, hinge-tested and applied.  Workload (default) = BASELINE.json's north-star
target, configs[3]: TransR n=50 bern L1 on FB15k (synthetic FB15k-shaped data,
14,951 entities / 1,345 relations / 483,142 triples), TransE-init: the seed
tables come from a TransE n=50 unif run (ORDERED schedule = the reference's
exact semantics) written and read back as the reference's `%.6lf` seed files
(transr/trainer.cpp:88-113); the CPU baseline reads the very same files.  FP64
like the reference.  `value` = training triples (samples) per second over the
whole job, inputs resident in HBM.

Timing: warmup runs W batches and then on to the next epoch boundary, so the
K timed batches always start an epoch: the epoch's sampling commit, its event
index (keys, radix sort, segments) and the prefetch of the next epoch's sample
stream are inside the timed region (for K < batches this over-weights the
per-epoch work; `epoch` in each schedule's record is one whole epoch timed the
same way).

Schedules (include/kb2e_engine.h kb2e_schedule): `value` is the PARALLEL
schedule (the data-parallel form: the reference's sample stream, snapshot
energies, hinge decisions and directions; summed row deltas and one norm per
batch; link-prediction parity in DESIGN.md), and the same line carries the
ORDERED schedule (bit-faithful to the reference) measured on the same
workload under "schedules".

N>1 (torchrun): each rank owns the triples whose head hashes to it
 and runs batches of the single-GPU size over its shard
(100 / N batches per epoch), so per-GPU work per step is fixed (weak scaling);
at every epoch boundary the ranks sum their table deltas over RCCL and
re-apply the norm constraints inside the engine (kb2e_merge_epoch, its own
RCCL communicator; kb2e_amd.distributed.NativeMerger).
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
    # BASELINE configs[4]: 1M entities, 10k relations, 16M triples;
    # tables drawn by numpy (the reference's host randn init takes minutes at this size)
    "transr_k5": ("R", "k5", 100, 1, 0, 0.001),
}
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
SEED_EPOCHS = 100  # TransE epochs behind the TransR seed tables ("TransE-init")
LATE_EPOCH = 50  # the steady-state epoch timed beside the K batches (bench.py --late-epoch)


def host_cpu():
    """lscpu model name and the host's CPU count."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}


def transe_seed(ds, dim, seed_dir, epochs=SEED_EPOCHS, device=0):
    """TransR's TransE-init (transr/trainer.cpp:88-113): TransE n=dim, unif, on the
    GPU with the ORDERED schedule (the reference's exact semantics), written as the
    reference writes it (entity2vec.unif / relation2vec.unif, "%.6lf\t",
    common/trainer.cpp:109-127) and read back, so GPU and CPU runs start from
    the same quantised tables."""
    from kb2e_amd.engine import Engine

    eng = Engine("E", dim, ds.num_entities, ds.num_relations, rate=0.001, method=0, seed=7, device=device,
                 schedule="ordered")
    eng.upload_triples(ds.train)
    eng.init_params()
    for _ in range(epochs):
        eng.train_batches(100)
    eng.synchronize()
    ent, rel, _ = eng.download_params()
    eng.close()
    os.makedirs(seed_dir, exist_ok=True)
    data.write_table(os.path.join(seed_dir, "entity2vec.unif"), ent)
    data.write_table(os.path.join(seed_dir, "relation2vec.unif"), rel)
    return (data.read_table(os.path.join(seed_dir, "entity2vec.unif"), ds.num_entities, dim),
            data.read_table(os.path.join(seed_dir, "relation2vec.unif"), ds.num_relations, dim))


def algorithmic_bytes_per_sample(model, n, s, active_frac):
    """ids 12 B + filter probe 8 B, gathers of the rows read by
    the energies, read-modify-write of the rows an active update touches."""
    if model == "E":
        return 20 + 4 * n * s + active_frac * 8 * n * s, 20 + 4 * n * s, active_frac * 8 * n * s
    if model == "H":
        return 20 + 5 * n * s + active_frac * 10 * n * s, 20 + 5 * n * s, active_frac * 10 * n * s
    full = 20 + (n * n + 5 * n) * s + active_frac * (2 * n * n + 10 * n) * s
    return full, 20 + (n * n + 5 * n) * s, active_frac * (2 * n * n + 10 * n) * s


def _ref_epoch_seconds(cmd, epochs, limit_s):
    """Seconds per epoch of the reference binary on one core, from the
    timestamps of its `Epoch: %d, Loss: %f` lines (common/trainer.cpp:105),
    read through a pseudo-terminal so its stdout is line-buffered: the mean
    over epochs 1..epochs-1 (epoch 0 and the data loading / init before it are
    excluded)."""
    import pty
    import select

    cpu = min(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None

    def pin():
        if cpu is not None:
            os.sched_setaffinity(0, {cpu})

    master, slave = pty.openpty()
    p = subprocess.Popen(cmd + ["--epochs", str(epochs)], stdout=slave, stderr=subprocess.DEVNULL,
                         stdin=subprocess.DEVNULL, preexec_fn=pin, close_fds=True)
    os.close(slave)
    stamps, buf, t_end = {}, b"", time.perf_counter() + limit_s
    try:
        while time.perf_counter() < t_end:
            r, _, _ = select.select([master], [], [], 1.0)
            if not r:
                if p.poll() is not None:
                    break
                continue
            try:
                chunk = os.read(master, 4096)
            except OSError:  # EIO: the child closed the terminal
                break
            if not chunk:
                break
            now = time.perf_counter()
            buf += chunk
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                if line.startswith(b"Epoch: "):
                    stamps[int(line.split(b",")[0][7:])] = now
    finally:
        if p.poll() is None:
            p.kill()
        p.wait()
        os.close(master)
    last = max(stamps) if stamps else -1
    if last < 1 or 0 not in stamps:
        raise RuntimeError(f"reference printed epochs {sorted(stamps)} within {limit_s} s")
    return (stamps[last] - stamps[0]) / last, last


def _ref_epoch_seconds_diff(cmd, epochs):
    """Seconds per epoch of the reference binary on one core without a
    terminal: wall time of an `epochs`-epoch run minus that of a 1-epoch run,
    over epochs - 1 (data loading, init and epoch 0 cancel)."""
    cpu = min(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None

    def pin():
        if cpu is not None:
            os.sched_setaffinity(0, {cpu})

    walls = []
    for e in (1, epochs):
        t0 = time.perf_counter()
        subprocess.run(cmd + ["--epochs", str(e)], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       stdin=subprocess.DEVNULL, preexec_fn=pin, check=True)
        walls.append(time.perf_counter() - t0)
    return (walls[1] - walls[0]) / (epochs - 1), epochs - 1


def cpu_baseline(cfg_name, ds, seed_dir=None, budget_s=25.0):
    """The reference itself (oracle/_ref, compiled from the reference sources)
    on this host, single-threaded, on the same synthetic dataset; falls back to
    the C restatement (oracle/liborc.so) when the binary is absent."""
    model, shape, dim, method, distance, rate = CONFIGS[cfg_name]
    binary = os.path.join(ROOT, "oracle", "_ref", {"E": "trainTransE", "H": "trainTransH", "R": "trainTransR"}[model])
    S = (len(ds.train) // 100) * 100
    if os.path.exists(binary):
        # epochs 1..E-1 timed (>= 3): ~10-40 s of training
        epochs = {"E": 9, "H": 6, "R": 4}[model]
        with tempfile.TemporaryDirectory() as d:
            data.write(ds, d)
            cmd = [binary, "--datadir", d, "--outdir", d, "--size", str(dim), "--method", str(method),
                   "--distance", str(distance), "--rate", str(rate), "--seed", "7"]
            seed_note = ""
            if model == "R":
                # the same TransE seed files the GPU run read (transr/trainer.cpp:88-113)
                cmd += ["--seeddatadir", seed_dir, "--seedmethod", "0"]
                seed_note = f", seeded from the GPU run's TransE-init files ({SEED_EPOCHS} TransE epochs)"
            try:
                per_epoch, timed = _ref_epoch_seconds(cmd, epochs, budget_s * 8)
                how = (f"mean time of epochs 1..{timed} from the timestamps of its Epoch lines (epoch 0 and init "
                       f"excluded)")
            except OSError:  # no pseudo-terminal on this host: two whole runs, differenced
                per_epoch, timed = _ref_epoch_seconds_diff(cmd, epochs)
                how = (f"(wall of a {epochs}-epoch run - wall of a 1-epoch run) / {timed} (init and epoch 0 "
                       f"cancel)")
        return {"value": S / per_epoch, "unit": "triples/s", "cores": 1, "kind": "reference", **host_cpu(),
                "sample": f"{os.path.basename(binary)} (compiled from the reference sources) on the same synthetic "
                          f"{shape}-shaped data{seed_note}, 1 thread pinned to one core; {how}, {S} samples per "
                          f"epoch"}
    from oracle import orc  # CPU restatement (port) fallback
    m = orc.Model(model, dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                  batches=100)
    m.set_triples(ds.train)
    orc.srand(7)
    m.prep_train()
    if model == "R":
        m.transr_seed(data.read_table(os.path.join(seed_dir, "entity2vec.unif"), ds.num_entities, dim),
                      data.read_table(os.path.join(seed_dir, "relation2vec.unif"), ds.num_relations, dim))
    B = m.batch_size()
    t0 = time.time()
    nb = 0
    while time.time() - t0 < budget_s and nb < 100:
        m.train_batches(1)
        nb += 1
    dt = time.time() - t0
    return {"value": nb * B / dt, "unit": "triples/s", "cores": 1, "kind": "port", **host_cpu(),
            "sample": f"{nb} batches ({B} samples each) of the C restatement, 1 thread"}


def phase_bytes(model, n, s, a):
    """(phase A bytes, phase B bytes) per sample."""
    _, score_b, fold_b = algorithmic_bytes_per_sample(model, n, s, a)
    return score_b, fold_b


def measure(args, schedule, ds, train, rank, world, local, dist, steps, warmup, seed_tabs=None, late=0):
    """Train `warmup` then time `steps` batches of one schedule; returns a dict."""
    from kb2e_amd.engine import Engine

    model, shape, dim, method, distance, rate = CONFIGS[args.config]
    batches = max(1, 100 // world)
    eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                 batches=batches, seed=7 + rank, precision=args.precision, device=local if world > 1 else 0,
                 schedule=schedule, sub_batches=args.sub_batches)
    eng.upload_triples(train)
    if shape == "k5":
        import numpy as np

        rng = np.random.default_rng(7)
        ent = rng.uniform(-1, 1, (ds.num_entities, dim))
        ent /= np.linalg.norm(ent, axis=1, keepdims=True)
        rel = rng.uniform(-1, 1, (ds.num_relations, dim))
        rel /= np.linalg.norm(rel, axis=1, keepdims=True)
        w = np.broadcast_to(np.eye(dim), (ds.num_relations, dim, dim)).reshape(eng.wshape())  # identity Mr
        eng.upload_params(ent, rel, np.ascontiguousarray(w))
    else:
        eng.init_params()  # consumes the reference's init draws (also for TransR, transr/trainer.cpp:70-86)
        if model == "R":
            eng.transr_seed(*seed_tabs)
    B = len(train) // batches
    merger = None
    if world > 1:
        from kb2e_amd.distributed import make_merger
        merger = make_merger(eng, dist)  # RCCL inside the engine (kb2e_merge_epoch); gloo: torch-side

    def run(k_steps):
        done = 0
        while done < k_steps:
            k = min(k_steps - done, batches - (run.pos % batches))
            eng.train_batches(k)
            done += k
            run.pos += k
            if merger is not None and run.pos % batches == 0:
                t0 = time.perf_counter()  # (the merge returns once the merged tables are in place)
                merger.merge()
                run.merge_s += time.perf_counter() - t0
                run.merges += 1
    run.pos = 0
    run.merge_s = 0.0
    run.merges = 0

    def to_epoch_start():
        if run.pos % batches:
            run(batches - run.pos % batches)

    def timed(k):
        eng.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        run(k)
        eng.synchronize()
        if dist is not None:
            dist.barrier()
        return time.perf_counter() - t0

    run(warmup)
    to_epoch_start()  # the timed batches start an epoch (its sampling commit + index build inside)
    eng.synchronize()
    eng.take_stats()
    run.merge_s, run.merges = 0.0, 0  # merges inside the timed batches only
    # HIP-event timing of the batch kernels on every 10th batch (events cost
    # device time; sampling keeps the timed run unperturbed); per-epoch kernels always
    eng.profile(10)
    elapsed = timed(steps)
    merge_s, merges = run.merge_s, run.merges
    loss, active = eng.take_stats()
    device_bytes = eng.device_bytes()
    # phase B span: TransE/TransH "fold_phase" (ordered: per-row folds; parallel:
    # the apply kernels), TransR "apply" (parallel) or the relation owners (ordered)
    if model == "R":
        fold_name = "apply" if schedule == "parallel" else "relowner"
    elif model == "H":
        fold_name = "fold_phase" if schedule == "parallel" else "relowner"
    else:
        fold_name = "apply" if schedule == "parallel" else "fold_phase"
    fold_ms, fold_n = eng.profile_query(fold_name)
    score_ms, score_n = eng.profile_query("score")
    kernels_us = {}
    for k in ("score", "fold", "fold_long", "apply", "tickets", "desc", "relowner", "fold_phase", "index", "sample"):
        ms, n = eng.profile_query(k)
        if n:
            kernels_us[k] = ms / n * 1e3
    epoch_s = None
    if not args.no_epoch:
        eng.profile(0)
        to_epoch_start()
        epoch_s = timed(batches)
    late_s = None
    if late and not args.no_epoch:
        # steady state: train on to `late` epochs, then time the next whole epoch
        # (hinge-active samples fall and TransH's orthogonality list grows with training)
        to_epoch_start()
        if run.pos < late * batches:
            run(late * batches - run.pos)
        eng.synchronize()
        late_s = timed(batches)
    comm = None
    if merger is not None:
        # what the communicator saw, per rank (kb2e_comm_info for the in-engine RCCL
        # merge; torch.distributed's view for the gloo merger) and the rank's device
        import torch

        if type(merger).__name__ == "NativeMerger":
            nr, rk, first, cnt = eng.comm_info()
        else:
            nr, rk, first, cnt = dist.get_world_size(), dist.get_rank(), -1, -1
        dev = torch.cuda.current_device()
        bus = getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", -1)
        row = torch.zeros((world, 6), dtype=torch.float64, device="cuda")
        row[rank] = torch.tensor([nr, rk, first, cnt, dev, bus], dtype=torch.float64)
        dist.all_reduce(row, op=dist.ReduceOp.SUM)
        comm = [{"rank": int(x[1]), "comm_nranks": int(x[0]), "entity_block": [int(x[2]), int(x[3])],
                 "device": int(x[4]), "pci_bus_id": int(x[5])} for x in row.tolist()]
    # PARALLEL TransR runs each batch as `sub_batches` phase-A / phase-B launch pairs,
    # each over B / sub_batches samples (the roofline's units per launch below)
    sub_batches = eng.cfg.sub_batches if model == "R" and schedule == "parallel" else 1
    eng.close()
    samples = steps * B
    if dist is not None:
        import torch

        t = torch.tensor([elapsed, float(samples), float(active), merge_s, float(merges), float(device_bytes)],
                         dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed = float(mx[0])
        samples = float(t[1])
        active = float(t[2])
        merge_s, merges, device_bytes = float(mx[3]), int(mx[4]), int(mx[5])
    a = active / max(1.0, samples)
    s = 8 if args.precision == 64 else 4
    score_b, fold_b = phase_bytes(model, dim, s, a)
    per_sample = score_b + fold_b
    units = B / sub_batches  # samples one launch (span) processes
    if fold_ms >= score_ms:
        dominant, avg_ms, bytes_per_launch = fold_name, fold_ms / max(1, fold_n), fold_b * units
    else:
        dominant, avg_ms, bytes_per_launch = "score", score_ms / max(1, score_n), score_b * units
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    # HBM bytes per launch from the PMC counters (FETCH_SIZE + WRITE_SIZE): counter
    # passes cannot share this timed run (separate rocprofv3 --pmc runs,
    # tools/gpu_profile.sh), so the value is read from the committed profile of the
    # same command, named in traffic_source
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.config}_{schedule}_f{args.precision}.json")
    if os.path.exists(pmc) and args.dim is None:  # (the committed counters are the config's own width)
        try:
            fams = json.load(open(pmc))
            v = fams.get(dominant, {}).get("hbm_bytes_per_launch")
            traffic = float(v) if v else None
            traffic_src = os.path.relpath(pmc, ROOT) if traffic else None
        except (OSError, ValueError):
            traffic = None
    epoch_rec = None
    if epoch_s is not None:
        if dist is not None:
            import torch

            t = torch.tensor([epoch_s], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            epoch_s = float(t[0])
        epoch_rec = {"value": batches * B * world / epoch_s, "ms": epoch_s * 1e3, "batches": batches}
    late_rec = None
    if late_s is not None:
        if dist is not None:
            import torch

            t = torch.tensor([late_s], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            late_s = float(t[0])
        late_rec = {"value": batches * B * world / late_s, "ms": late_s * 1e3, "batches": batches,
                    "epoch_index": late}
    merge_rec = None
    if merger is not None:  # the epoch merge's share of the timed region (max over ranks)
        merge_rec = {"merges": merges, "ms_per_merge": merge_s / merges * 1e3 if merges else None,
                     "share_of_timed": merge_s / elapsed, "kind": type(merger).__name__, "ranks": comm}
    return {
        "value": samples / elapsed, "ms_per_step": elapsed / steps * 1e3, "B": B, "batches": batches,
        "sub_batches": sub_batches,
        "merge": merge_rec, "device_bytes_per_gpu": device_bytes,
        "epoch": epoch_rec,
        "late_epoch": late_rec,
        "active_fraction": a,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     # the PMC bytes over the same live launch time: the physical HBM rate
                     "traffic_GBs": traffic / (avg_ms * 1e-3) / 1e9 if traffic and avg_ms > 0 else None,
                     "traffic_frac": traffic / (avg_ms * 1e-3) / 1e9 / PEAK_HBM_GBS if traffic and avg_ms > 0 else None,
                     "kernel": dominant,
                     "kernel_avg_us": avg_ms * 1e3, "algorithmic_bytes_per_launch": bytes_per_launch,
                     "samples_per_launch": units,
                     "kernels_avg_us": kernels_us, "step_achieved_GBs": per_sample * samples / elapsed / 1e9},
    }


def launch_ranks(n):
    """Run this same command as `torch.distributed.run --nproc-per-node n` in a
    child process (one rank per GPU, rendezvous on 127.0.0.1) and return its exit
    code; rank 0's JSON line goes straight to this process's stdout."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.stdout.flush()
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="transr_fb15k", choices=sorted(CONFIGS))
    ap.add_argument("--precision", type=int, default=64, choices=[32, 64])
    ap.add_argument("--schedule", default="parallel", choices=["ordered", "parallel"],
                    help="schedule of the headline value; the other one is reported beside it")
    ap.add_argument("--only", action="store_true", help="measure the --schedule only")
    ap.add_argument("--sub-batches", type=int, default=None,
                    help="PARALLEL TransR sub-batches (kb2e_config.sub_batches; default: the engine's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-epoch", action="store_true", help="skip the whole-epoch timing")
    ap.add_argument("--seed-epochs", type=int, default=SEED_EPOCHS)
    ap.add_argument("--late-epoch", type=int, default=LATE_EPOCH,
                    help="also time the whole epoch with this index (steady state); 0: skip")
    ap.add_argument("--dim", type=int, default=None,
                    help="another embedding width on the config's data (A/B lines, e.g. the n > 128 wide path)")
    args = ap.parse_args()
    if args.dim is not None:  # (the config's model and data at another width; named in config.dim)
        m_, sh_, _, me_, di_, ra_ = CONFIGS[args.config]
        CONFIGS[args.config] = (m_, sh_, args.dim, me_, di_, ra_)
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus {args.gpus}: need at least one GPU")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` on its own: one rank per GPU, launched here as a child
        # (nothing in this process has touched the GPU yet: numpy and kb2e_amd.data only)
        sys.exit(launch_ranks(args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the rank count must match the GPU count")
    dist = None
    if world > 1:
        import torch.distributed as dist
        import torch

        # test knobs (tests/test_gpu_distributed.py): every rank on device 0, gloo
        if os.environ.get("KB2E_DIST_ONE_DEVICE"):
            local = 0
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("KB2E_DIST_BACKEND", "nccl"))

    model, shape, dim, method, distance, rate = CONFIGS[args.config]
    ds = data.synthetic(shape, seed=1 if shape == "k5" else 0)
    train = shard_heads(ds.train, rank, world) if world > 1 else ds.train
    seed_tmp = tempfile.TemporaryDirectory()
    seed_tabs = None
    if model == "R" and shape != "k5":
        # every rank draws the same seed (fixed glibc seed), no broadcast needed
        seed_tabs = transe_seed(ds, dim, seed_tmp.name, epochs=args.seed_epochs, device=local if world > 1 else 0)
    main_run = measure(args, args.schedule, ds, train, rank, world, local, dist, args.steps, args.warmup, seed_tabs,
                       late=args.late_epoch if shape != "k5" else 0)
    other = "ordered" if args.schedule == "parallel" else "parallel"
    other_run = None
    if not args.only:
        other_run = measure(args, other, ds, train, rank, world, local, dist, args.steps, args.warmup, seed_tabs)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    B, batches = main_run["B"], main_run["batches"]
    out = {
        "metric": "training triples/sec (1/2/4/8 MI355X) + FB15k Hits@10(Filter)",
        "value": main_run["value"],
        "unit": "triples/s (1 triple = 1 positive + 1 corrupted)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_run["ms_per_step"],
        "higher_is_better": True,
        # every rank runs batches of the single-GPU size over its head-hash shard
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64" if args.precision == 64 else "f32",
        "data": f"synthetic {shape}-shaped (kb2e_amd.data.synthetic, seed {1 if shape == 'k5' else 0}), reference "
                f"glibc sample stream seed 7" + (", numpy-drawn unit-row tables, identity Mr" if shape == "k5" else "")
                + (f", TransE-init: {args.seed_epochs} TransE n={dim} unif epochs (ORDERED), %.6lf seed files"
                   if seed_tabs is not None else ""),
        "config": {"workload": f"{args.config}: {'TransE' if model == 'E' else 'TransH' if model == 'H' else 'TransR'} "
                               f"n={dim} {'bern' if method else 'unif'} L{distance + 1}, {batches} batches of {B} "
                               f"per GPU, {args.schedule} schedule"
                               + (", compat energy, TransE-init" if model == "R" and shape != "k5" else ""),
                   "global_batch": B * world, "parallelism": f"dp{world}" if world > 1 else "single",
                   "schedule": args.schedule, "sub_batches": main_run["sub_batches"]},
        "roofline": main_run["roofline"],
        "active_fraction": main_run["active_fraction"],
        "timing": "K batches from an epoch boundary (epoch sampling commit + index build inside"
                  + (", the epoch merges falling inside them" if world > 1 else "") + ")",
        "device_bytes_per_gpu": main_run["device_bytes_per_gpu"],
    }
    if main_run["merge"] is not None:
        out["merge"] = main_run["merge"]
        ranks = main_run["merge"]["ranks"] or []
        # the communicator's rank count as every rank saw it (min over ranks) and the
        # device each rank drove: N distinct PCI buses = N GPUs
        out["comm_nranks"] = min(r["comm_nranks"] for r in ranks) if ranks else None
        out["pci_bus_ids"] = [r["pci_bus_id"] for r in ranks]
    out["schedules"] = {args.schedule: {"value": main_run["value"], "ms_per_step": main_run["ms_per_step"],
                                        "epoch": main_run["epoch"], "late_epoch": main_run["late_epoch"]}}
    if other_run is not None:
        out["schedules"][other] = {"value": other_run["value"], "ms_per_step": other_run["ms_per_step"],
                                   "epoch": other_run["epoch"], "active_fraction": other_run["active_fraction"],
                                   "roofline": other_run["roofline"]}
    if not args.no_cpu_baseline and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, ds, seed_tmp.name)
        except Exception as e:  # the baseline is reported, never the target
            out["cpu_baseline"] = {"value": None, "error": str(e)}
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
