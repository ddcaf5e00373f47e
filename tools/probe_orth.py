"""TransH PARALLEL orthogonality-fix statistics (libkb2e_prof.so, KB2E_OWNER_PROF):
tasks, w switches and per-phase cycles of transh_orth_fix_kernel on the bench's
FB15k-shaped TransH workload, 100 batches at a time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("KB2E_LIB", os.path.join(ROOT, "kb2e_amd", "libkb2e_prof.so"))
from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402

ds = data.synthetic("fb15k", seed=0)
eng = Engine("H", 100, ds.num_entities, ds.num_relations, rate=0.001, method=1, batches=100, seed=7,
             schedule="parallel")
eng.upload_triples(ds.train)
eng.init_params()
for ep in range(4):
    eng.train_batches(100)
    print(f"epoch {ep}", eng.take_stats(), file=sys.stderr, flush=True)
