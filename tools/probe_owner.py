"""Per-phase cycle breakdown of the relation-owner kernels (diagnostic build).

    make prof && python tools/probe_owner.py [--model R] [--batches 20]

Loads kb2e_amd/libkb2e_prof.so (compiled with -DKB2E_OWNER_PROF): every owner
workgroup accumulates clock64() deltas per phase and the engine prints the
sums to stderr on take_stats().  Cycles are summed over owners, so the
per-update figures are an average over all updates of the run."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["decode/switch", "wait tickets", "load rows", "rank-1 W | H: deltas", "deltas+r | H: norms",
          "(unused)",
          "transRNorm check | H: orth(r)", "transRNorm iterate | H: orth(h,t)", "store+release"]


def child(args):
    os.environ["KB2E_LIB"] = os.path.join(ROOT, "kb2e_amd", "libkb2e_prof.so")
    import time
    from kb2e_amd import data
    from kb2e_amd.engine import Engine
    ds = data.synthetic("fb15k", seed=0, relation_zipf=args.zipf)
    eng = Engine(args.model, args.dim, ds.num_entities, ds.num_relations, rate=0.001, method=1, distance=0,
                 batches=100, seed=7, precision=args.precision)
    eng.upload_triples(ds.train)
    ent, rel, w = eng.init_params()
    if args.model == "R":
        eng.transr_seed(ent, rel)
    eng.train_batches(2)
    eng.synchronize()
    eng.take_stats()
    t0 = time.perf_counter()
    eng.train_batches(args.batches)
    eng.synchronize()
    dt = time.perf_counter() - t0
    loss, active = eng.take_stats()
    print(f"batches {args.batches} wall {dt * 1e3:.1f} ms active {active}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="R")
    ap.add_argument("--dim", type=int, default=50)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--zipf", type=float, default=None, help="relation Zipf exponent of the synthetic data")
    args = ap.parse_args()
    if args.child:
        return child(args)
    cmd = [sys.executable, __file__, "--child", "--model", args.model, "--dim", str(args.dim), "--batches",
           str(args.batches), "--precision", str(args.precision)]
    if args.zipf is not None:
        cmd += ["--zipf", str(args.zipf)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    print(res.stdout)
    if args.model == "E":
        FOLD = ["first chunk", "LDS + p_m", "chain", "materialise", "next chunk decode"]
        for line in res.stderr.splitlines():
            if line.startswith("fold_prof"):
                f = [int(x) for x in line.split()[1:]]
                g, v = f[0], f[1:]
                ev, steps, chunks = max(1, v[10]), max(1, v[11]), max(1, v[12])
                print(f"{'segments >= 512 events' if g == 0 else 'shorter segments'}: events {v[10]} "
                      f"steps {v[11]} chunks {v[12]}")
                for k, name in enumerate(FOLD):
                    print(f"  {name:20s} {v[k] / ev:8.0f} cycles/event  {v[k] / chunks:9.0f} cycles/chunk")
                print(f"  chain per step {v[2] / steps:8.0f} cycles")
            if line.startswith("long_prof"):
                v = [int(x) for x in line.split()[1:]]
                ev, phases = max(1, v[10]), max(1, v[12])
                print(f"4-wave long fold: events {v[10]}, wave-phases {v[12]} ({v[12] / 4:.0f} chunk phases)")
                for wv, name in enumerate(["chain", "materialise+P0", "decode+t", "cross t+table"]):
                    print(f"  wave {wv} {name:16s} work {v[wv] / (phases / 4):8.0f} cycles/phase  "
                          f"barrier wait {v[4 + wv] / (phases / 4):8.0f}")
                print(f"  chain per event {v[0] / ev:8.0f} cycles")
        return
    rows = {}
    for line in res.stderr.splitlines():
        if line.startswith("owner_prof"):
            f = line.split()
            rows[int(f[1])] = [int(x) for x in f[2:]]
    if res.returncode or not rows:
        print(res.stderr[-3000:])
        sys.exit(1)
    total = [sum(v[k] for v in rows.values()) for k in range(16)]
    hot = max(rows, key=lambda o: rows[o][11])
    for title, v in (("all owners", total), (f"busiest owner {hot}", rows[hot])):
        updates = max(1, v[11])
        cyc = sum(v[:9])
        print(f"{title}: updates {updates}  transRNorm iterations {v[10]} ({v[10] / updates:.2f}/update)")
        for k, name in enumerate(PHASES):
            print(f"  {name:24s} {v[k] / updates:9.0f} cycles/update  {100 * v[k] / max(1, cyc):5.1f}%")
        print(f"  {'total':24s} {cyc / updates:9.0f} cycles/update")

if __name__ == "__main__":
    main()
