"""Time a schedule with and without the engine's per-kernel HIP-event timing
(host launch cost vs device time)."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "E"
sched = sys.argv[2] if len(sys.argv) > 2 else "parallel"
dim = {"E": 100, "H": 100, "R": 50}[model]
ds = data.synthetic("fb15k", seed=0)
eng = Engine(model, dim, ds.num_entities, ds.num_relations, batches=100, seed=7, schedule=sched)
eng.upload_triples(ds.train)
e, r, _ = eng.init_params()
if model == "R":
    eng.transr_seed(e, r)
eng.train_batches(100)
eng.synchronize()
for prof in (False, True, False):
    eng.profile(prof)
    t0 = time.perf_counter()
    eng.train_batches(300)
    t1 = time.perf_counter()
    eng.synchronize()
    t2 = time.perf_counter()
    print(f"profile={prof}: host queue {1e6 * (t1 - t0) / 300:.1f} us/batch, total {1e6 * (t2 - t0) / 300:.1f} us/batch")
