"""Quick throughput probe (dev tool): FB15k-shaped TransE/TransH/TransR epochs."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kb2e_amd import data
from kb2e_amd.engine import Engine

model = sys.argv[1] if len(sys.argv) > 1 else "E"
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 100
prec = int(sys.argv[3]) if len(sys.argv) > 3 else 64
epochs = int(sys.argv[4]) if len(sys.argv) > 4 else 2
t = time.time()
ds = data.synthetic("fb15k", seed=0)
print(f"gen {time.time()-t:.1f}s", flush=True)
eng = Engine(model, dim, ds.num_entities, ds.num_relations, rate=0.001, batches=100, seed=7, precision=prec)
eng.upload_triples(ds.train)
eng.init_params()
eng.profile(True)
for ep in range(epochs):
    t = time.time()
    loss, act = eng.train_epoch()
    dt = time.time() - t
    S = (len(ds.train) // 100) * 100
    print(f"{model} n={dim} f{prec} epoch {ep}: {dt*1e3:.1f} ms  {S/dt/1e6:.2f} M samples/s  loss {loss:.1f} active {act}", flush=True)
for k in ("index", "score", "fold", "relowner", "tickets", "sync"):
    ms, n = eng.profile_query(k)
    if n: print(f"  {k:10s} {ms:9.2f} ms over {n} launches ({ms/n*1e3:.1f} us avg)")
