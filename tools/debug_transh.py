import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kb2e_amd import data
from kb2e_amd.engine import Engine
from oracle import orc
dim, rate, model = int(sys.argv[1]), float(sys.argv[2]), sys.argv[3]
ds = data.synthetic("small", seed=1)
eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=rate, margin=1.0, method=1, batches=20, seed=5)
eng.upload_triples(ds.train); eng.init_params()
m = orc.Model(model, dim, ds.num_entities, ds.num_relations, rate=rate, margin=1.0, method=1, batches=20)
m.set_triples(ds.train); orc.srand(5); m.prep_train()
L = orc.lib()
for b in range(20):
    before = [L.orc_site_iterations(s) for s in range(3)]
    lo, ao = m.train_batches(1)
    eng.train_batches(1); lg, ag = eng.take_stats()
    ge, gr, gw = eng.download_params(); oe, orl, ow = m.tables()
    de, dr = np.abs(ge-oe).max(1), np.abs(gr-orl).max(1)
    dw = np.abs(gw-ow).max(1) if gw is not None else np.zeros(1)
    it = [L.orc_site_iterations(s)-before[s] for s in range(3)]
    print(f"batch {b}: act {ag} vs {ao} dloss {lg-lo:.2e} ent {de.max():.2e} rel {dr.max():.2e} w {dw.max():.2e} iters {it}", flush=True)
    if max(de.max(), dr.max(), dw.max()) > 1e-9:
        for name, d in (("ent", de), ("rel", dr), ("w", dw)):
            bad = np.argsort(-d)[:4]; print(f"  worst {name}", bad.tolist(), d[bad].tolist())
        break
