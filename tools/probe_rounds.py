"""transRNorm rounds / cycles per tile of the PARALLEL TransR schedule
(KB2E_RPAR_STATS), on the bench's K4 workload (TransE-init seed)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["KB2E_RPAR_STATS"] = "1"
from kb2e_amd import data  # noqa: E402
from kb2e_amd.engine import Engine  # noqa: E402
from kb2e_amd.linkpred import transe_seed  # noqa: E402

compat = sys.argv[1] == "compat" if len(sys.argv) > 1 else True
seed_epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 100
ds = data.synthetic("fb15k", seed=0)
st = transe_seed(ds, 50, seed_epochs)
eng = Engine("R", 50, ds.num_entities, ds.num_relations, batches=100, seed=7, schedule="parallel",
             transr_compat=compat)
eng.upload_triples(ds.train)
eng.init_params()
eng.transr_seed(*st)
for ep in range(3):
    for k in range(4):
        eng.train_batches(25)
        print(f"epoch {ep} part {k}", eng.take_stats(), file=sys.stderr, flush=True)
