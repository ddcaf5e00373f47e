#!/usr/bin/env python3
"""Seed envelope of link-prediction quality and the loss trajectory, per schedule.

For each glibc seed (the reference's only seed, `srand(args.seed)`,
transe/bin/trainTransE.cpp:13) trains the FB15k-shaped synthetic set with the
ORDERED schedule (= the reference bit for bit) and the PARALLEL schedule from the
same initial tables and sample stream, and scores both with the GPU evaluator
(common/evaluation.cpp:181-251, filter = train + valid + test).  TransR is
TransE-initialised per seed (transr/trainer.cpp:88-113).  One JSON line per
seed is appended to --out as it finishes; the last line is the summary
(min / max / mean per schedule, and where PARALLEL's values sit in ORDERED's
envelope).

  python tools/seed_envelope.py --model R --compat 1 --seeds 7,8,9,10,11 --out env.jsonl
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.linkpred import train_and_evaluate, transe_seed  # noqa: E402

METRICS = ("filtered_rank", "filtered_hits10", "raw_rank", "raw_hits10", "final_loss", "mean_loss_last10")


# two-sided 95 % Student t quantiles by degrees of freedom
T975 = {1: 12.706, 2: 4.303, 3: 3.182, 4: 2.776, 5: 2.571, 6: 2.447, 7: 2.365, 8: 2.306, 9: 2.262, 10: 2.228}


def paired_interval(d):
    """Mean of the paired deltas, its standard error and 95 % t interval."""
    d = np.asarray(d, dtype=np.float64)
    k = len(d)
    mean = float(d.mean())
    if k < 2:
        return {"n": k, "mean": mean}
    se = float(d.std(ddof=1) / np.sqrt(k))
    t = T975.get(k - 1, 1.96)
    lo, hi = mean - t * se, mean + t * se
    return {"n": k, "mean": mean, "se": se, "ci95": [lo, hi], "covers_zero": bool(lo <= 0.0 <= hi),
            "same_sign": int(max((d > 0).sum(), (d < 0).sum()))}


def summarize(rows, schedules):
    out = {"seeds": [r["seed"] for r in rows]}
    for s in schedules:
        st = {}
        for m in METRICS:
            v = np.array([r[s][m] for r in rows], dtype=np.float64)
            st[m] = {"min": float(v.min()), "max": float(v.max()), "mean": float(v.mean()),
                     "std": float(v.std(ddof=1)) if len(v) > 1 else 0.0}
        # per-epoch loss envelope
        L = np.array([[x[1] for x in r[s]["losses"]] for r in rows], dtype=np.float64)
        st["loss_envelope"] = {"min": L.min(0).tolist(), "max": L.max(0).tolist(), "mean": L.mean(0).tolist()}
        out[s] = st
    if "ordered" in schedules and "parallel" in schedules:
        o, p = out["ordered"], out["parallel"]
        cmp = {}
        for m in METRICS:
            cmp[m] = {"parallel_mean": p[m]["mean"], "ordered_mean": o[m]["mean"],
                      "rel_delta_of_means": (p[m]["mean"] - o[m]["mean"]) / abs(o[m]["mean"]),
                      "ordered_rel_spread": (o[m]["max"] - o[m]["min"]) / abs(o[m]["mean"]),
                      "parallel_mean_inside_ordered_envelope": o[m]["min"] <= p[m]["mean"] <= o[m]["max"]}
        # paired per-seed deltas (same stream, same init) with a 95 % t interval of
        # their mean: a systematic term shows as an interval that excludes 0 even
        # when the schedules' means sit inside each other's cross-seed spread
        for m in METRICS:
            d = np.array([(r["parallel"][m] - r["ordered"][m]) / abs(r["ordered"][m]) for r in rows])
            cmp[m]["paired_rel_delta"] = d.tolist()
            cmp[m]["paired"] = paired_interval(d)
        Lo = np.array(o["loss_envelope"]["min"]), np.array(o["loss_envelope"]["max"])
        Lp = np.array(p["loss_envelope"]["mean"])
        cmp["parallel_mean_loss_epochs_inside_ordered_envelope"] = int(((Lp >= Lo[0]) & (Lp <= Lo[1])).sum())
        cmp["epochs"] = int(len(Lp))
        out["compare"] = cmp
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="R", choices=["E", "H", "R"])
    ap.add_argument("--shape", default="fb15k")
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--seed-epochs", type=int, default=500)
    ap.add_argument("--test", type=int, default=0, help="test triples scored (0 = all)")
    ap.add_argument("--compat", type=int, default=1)
    ap.add_argument("--batches", type=int, default=100, help="batches an epoch (the reference's --batches)")
    ap.add_argument("--seeds", default="7,8,9")
    ap.add_argument("--schedules", default="ordered,parallel")
    ap.add_argument("--sub", type=int, default=None, help="PARALLEL TransR sub-batches (kb2e_config.sub_batches)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--summarize", nargs="*", default=None,
                    help="only write the summary of the per-seed rows in these JSONL files (runs split over calls)")
    args = ap.parse_args()
    if args.summarize is not None:
        by_seed = {}  # rows of one seed from several files (e.g. ORDERED and PARALLEL runs) merged
        for fn in args.summarize:
            for line in open(fn):
                r = json.loads(line)
                if "seed" in r and "summary" not in r:
                    by_seed.setdefault(r["seed"], {}).update(r)
        rows = [by_seed[k] for k in sorted(by_seed)]
        schedules = tuple(s for s in ("ordered", "parallel") if all(s in r for r in rows))
        r0 = rows[0]
        ds = data.synthetic(args.shape, seed=0)
        summ = {"summary": summarize(rows, schedules), "model": r0["model"], "dim": r0["dim"],
                "transr_compat": r0["transr_compat"], "epochs": r0["epochs"], "shape": args.shape,
                "random_hits10": 10.0 / ds.num_entities, "files": args.summarize}
        with open(args.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
            f.write(json.dumps(summ) + "\n")
        print(json.dumps(summ["summary"].get("compare", {})))
        return
    dim = args.dim or {"E": 100, "H": 100, "R": 50}[args.model]
    schedules = tuple(args.schedules.split(","))
    ds = data.synthetic(args.shape, seed=0)
    test = ds.test if args.test <= 0 else ds.test[: args.test]
    rows = []
    log = lambda m: print(m, file=sys.stderr, flush=True)  # noqa: E731
    for seed in [int(s) for s in args.seeds.split(",")]:
        seed_tables = None
        if args.model == "R":
            seed_tables = transe_seed(ds, dim, args.seed_epochs, seed=seed)
        row = {"seed": seed, "model": args.model, "dim": dim, "epochs": args.epochs, "batches": args.batches,
               "seed_epochs": args.seed_epochs, "transr_compat": bool(args.compat), "test": int(len(test))}
        for s in schedules:
            r = train_and_evaluate(ds, args.model, dim, s, args.epochs, test=test, seed=seed, batches=args.batches,
                                   transr_compat=bool(args.compat), seed_tables=seed_tables, log=log,
                                   sub_batches=args.sub if s == "parallel" else None)
            if s == "parallel" and args.sub is not None:
                r["sub_batches"] = args.sub
            ls = [x[1] for x in r["losses"]]
            r["final_loss"] = ls[-1]
            r["mean_loss_last10"] = float(np.mean(ls[-10:]))
            row[s] = r
            log(f"seed {seed} {s}: MR {r['filtered_rank']:.1f} H10 {100 * r['filtered_hits10']:.3f}% "
                f"loss {ls[-1]:.0f} ({r['train_s']:.1f} s)")
        rows.append(row)
        with open(args.out, "a") as f:
            f.write(json.dumps(row) + "\n")
    summ = {"summary": summarize(rows, schedules), "model": args.model, "dim": dim,
            "transr_compat": bool(args.compat), "epochs": args.epochs, "shape": args.shape,
            "random_hits10": 10.0 / ds.num_entities}
    with open(args.out, "a") as f:
        f.write(json.dumps(summ) + "\n")
    print(json.dumps(summ["summary"].get("compare", {})))


if __name__ == "__main__":
    main()
