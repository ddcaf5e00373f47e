"""Train the same configuration with two engine builds and report whether the
tables are bit-identical (e.g. after a reduction rewrite that should not
change any result).

    python tools/compare_libs.py kb2e_amd/libkb2e.so kb2e_amd/libkb2e_other.so --model H --dim 33
"""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path.insert(0, ROOT)
    from kb2e_amd import data
    from kb2e_amd.engine import Engine
    ds = data.synthetic(args.shape, seed=4)
    eng = Engine(args.model, args.dim, ds.num_entities, ds.num_relations, rate=args.rate, method=1,
                 distance=args.distance, batches=25, seed=8, precision=args.precision)
    eng.upload_triples(ds.train)
    ent, rel, w = eng.init_params()
    if args.model == "R":
        eng.transr_seed(ent, rel)
    losses = []
    for _ in range(args.epochs):
        losses.append(eng.train_epoch()[0])
    e, r, w = eng.download_params()
    np.savez(args.out, e=e, r=r, w=w if w is not None else np.zeros(1), loss=np.array(losses))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--model", default="H")
    ap.add_argument("--dim", type=int, default=33)
    ap.add_argument("--rate", type=float, default=0.02)
    ap.add_argument("--distance", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--shape", default="small")
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--out")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    outs = []
    with tempfile.TemporaryDirectory() as d:
        for k, lib in enumerate(args.libs):
            out = os.path.join(d, f"{k}.npz")
            env = dict(os.environ, KB2E_LIB=os.path.abspath(lib))
            cmd = [sys.executable, __file__, "--child", "--out", out, "--model", args.model, "--dim", str(args.dim),
                   "--rate", str(args.rate), "--distance", str(args.distance), "--epochs", str(args.epochs),
                   "--shape", args.shape, "--precision", str(args.precision)]
            subprocess.run(cmd, env=env, check=True)
            outs.append(dict(np.load(out)))
    a = outs[0]
    for lib, b in zip(args.libs[1:], outs[1:]):
        diffs = {k: float(np.abs(a[k] - b[k]).max()) for k in a}
        same = all(np.array_equal(a[k], b[k]) for k in a)
        print(f"{args.libs[0]} vs {lib}: {'bit-identical' if same else 'DIFFERENT'} {diffs}")


if __name__ == "__main__":
    main()
