"""Dev tool: fold time vs relation skew (is the hottest row's chain the bound?)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kb2e_amd import data
from kb2e_amd.engine import Engine
for rz in (1.0, 0.5, 0.0):
    ds = data.synthetic("fb15k", seed=0, relation_zipf=rz)
    cnt = np.bincount(ds.train[:, 2], minlength=ds.num_relations)
    eng = Engine("E", 100, ds.num_entities, ds.num_relations, rate=0.001, batches=100, seed=7)
    eng.upload_triples(ds.train); eng.init_params(); eng.train_epoch()
    eng.profile(True)
    t = time.time(); eng.train_epoch(); dt = time.time() - t
    ms, n = eng.profile_query("fold")
    print(f"relation zipf {rz}: top relation share {cnt.max()/cnt.sum():.3f}  epoch {dt*1e3:.1f} ms  fold avg {ms/n*1e3:.1f} us", flush=True)
