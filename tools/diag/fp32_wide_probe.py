#!/usr/bin/env python3
"""FP32 ORDERED TransR against the FP64 oracle across the owner's LDS / L2 switch
(FP32: LDS up to dim 195, L2 above): median element differences after one epoch
(diagnostic for tests/test_gpu_transr.py::test_fp32_wide_statistically_close)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402
from oracle import orc  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "small"
dims = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "120,190,196,200").split(",")]
ds = data.synthetic(shape, seed=6)
kw = dict(rate=0.005 if shape == "small" else 0.01, batches=25 if shape == "small" else 10, transr_compat=False)
for dim in dims:
    m = orc.Model("R", dim, ds.num_entities, ds.num_relations, **kw)
    m.set_triples(ds.train)
    orc.srand(3)
    m.prep_train()
    row = [dim]
    for prec in (64, 32):
        eng = Engine("R", dim, ds.num_entities, ds.num_relations, seed=3, precision=prec, **kw)
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        if prec == 64:
            m.transr_seed(e0, r0)
            lo, ao = m.train_epoch()
            oe, orl, ow = m.tables()
        lg, ag = eng.train_epoch()
        ge, gr, gw = eng.download_params()
        eng.close()
        row += [prec, f"loss {lg / lo - 1:+.2e}", f"act {ag - ao:+d}", f"ent {np.median(np.abs(ge - oe)):.2e}",
                f"w {np.median(np.abs(gw - ow)):.2e}", f"maxent {np.abs(ge - oe).max():.2e}"]
    print(*row, flush=True)
