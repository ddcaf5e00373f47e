"""A/B of the transRNorm kernels (register-resident vs LDS-round) on the tiny
set: max table differences after each of a few batches, FP64 and FP32."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402

ds = data.synthetic("tiny", seed=0)
dim = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for prec in (64, 32):
    runs = {}
    for mode in ("wave", "tile"):
        os.environ["KB2E_RPAR_CONS"] = mode
        eng = Engine("R", dim, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=3, precision=prec,
                     schedule="parallel", transr_compat=False)
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        out = []
        for b in range(12):
            eng.train_batches(1)
            eng.synchronize()
            out.append((eng.download_params(), eng.take_stats()))
        runs[mode] = out
        eng.close()
    for b in range(12):
        (ta, sa), (tb, sb) = runs["wave"][b], runs["tile"][b]
        d = [float(np.nanmax(np.abs(x - y))) for x, y in zip(ta, tb)]
        nan = [bool(np.isnan(x).any()) for x in ta]
        print(f"prec {prec} batch {b}: stats wave {sa} tile {sb} maxdiff {d} nan {nan}", flush=True)
