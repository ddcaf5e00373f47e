"""Dev tool: TransE fold time vs relation skew (is the hottest row's chain the
bound?).  Optional argv: values of KB2E_FOLD_LONG to compare (default: engine's)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402

for lm in (sys.argv[1:] or [None]):
    if lm is not None:
        os.environ["KB2E_FOLD_LONG"] = lm
    for rz in (1.0, 0.5, 0.0):
        ds = data.synthetic("fb15k", seed=0, relation_zipf=rz)
        cnt = np.bincount(ds.train[:, 2], minlength=ds.num_relations)
        eng = Engine("E", 100, ds.num_entities, ds.num_relations, rate=0.001, batches=100, seed=7)
        eng.upload_triples(ds.train)
        eng.init_params()
        eng.train_epoch()
        eng.profile(True)
        t = time.time()
        eng.train_epoch()
        dt = time.time() - t
        out = []
        for k in ("score", "fold", "fold_long"):
            ms, n = eng.profile_query(k)
            if n:
                out.append(f"{k} {ms / n * 1e3:.1f} us")
        print(f"long_min {lm}: relation zipf {rz}: top share {cnt.max() / cnt.sum():.3f}  epoch {dt * 1e3:.1f} ms  "
              + "  ".join(out), flush=True)
