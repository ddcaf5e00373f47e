"""Link-prediction parity of the PARALLEL schedule (the bench headline) with
the ORDERED schedule, which is the reference bit for bit (FP64 tables within
1e-11 of the compiled reference's, test_gpu_transe/transh/transr.py).

Both schedules train the same planted synthetic set from the same initial
tables and the same glibc sample stream; the GPU evaluator (kb2e_evaluate =
EmbeddingEvaluation::run, common/evaluation.cpp:181-251, bit-identical energies
and ranks to the reference eval binaries, test_gpu_eval.py) scores both on
8,000 test triples (16,000 rankings), filter = train + valid + test.
TransR is TransE-initialised (transr/trainer.cpp:88-113): 300 ORDERED TransE
epochs written and read back as the reference's %.6lf seed files.

Bars (BASELINE.json north_star: "matching Hits@10(Filter) +-0.5"):
  * |PARALLEL - ORDERED| <= 0.5 pp in filtered and raw Hits@10, filtered mean
    rank within 2 %;
  * the ORDERED run learns: filtered Hits@10 >= 10x random (10 / |E|) for
    TransE, TransH and TransR with the zeroed (fixed) energy.
For scale: two ORDERED runs that differ only in the glibc seed land
0.17-0.28 pp apart on this set (tools/hits_sweep.py, profiles/hits_sweep_r10_small.jsonl).

TransR compat (the reference's accumulating work-vector energy,
transr/transr.cpp:20-25) does not learn under the reference's own algorithm:
its ORDERED run ends *below* the seed tables' Hits@10 (1.1 % after 150 epochs
against 2.5 % for the seed alone on this set), so only the schedule delta is
asserted for it.

TransR runs at the north-star width n = 50 and at K5's n = 100 (fixed energy,
the form that learns), and the loss trajectory is bounded too: the mean loss of
the last 10 epochs within LOSS_TOL_REL of ORDERED's.  On the FB15k-shaped set
the ORDERED seed envelope (5 glibc seeds) spans +-3.6 % around its mean and
PARALLEL compat sits 2.6 % below it at n = 50
(profiles/seed_envelope_r17_fb15k_R_compat.jsonl, .._r18_.._parallel_seq.jsonl);
with fixed energy at n = 100 the paired gap is +0.16 % [-0.04, +0.36]
(profiles/seed_envelope_r22_fb15k_R100_fixed.jsonl), so fixed energy is held
to LOSS_TOL_FIXED.
"""
import pytest

from kb2e_amd import data
from kb2e_amd.linkpred import schedule_parity

pytestmark = pytest.mark.gpu

HITS_TOL_PP = 0.5
RANK_TOL_REL = 0.02
LOSS_TOL_REL = 0.05
LOSS_TOL_FIXED = 0.02


@pytest.fixture(scope="module")
def ds():
    return data.synthetic("small", seed=0, counts=(2000, 40, 30000, 1000, 8000))


@pytest.mark.parametrize("model,dim,epochs,compat,learns", [
    ("E", 50, 300, True, True),
    ("H", 50, 300, True, True),
    ("R", 50, 50, False, True),   # fixed energy
    ("R", 50, 50, True, False),   # compat energy (the reference default)
    ("R", 100, 50, False, True),  # K5's width: the pipelined wide chain (kernels_transr_chainwp.hpp), fixed energy
])
def test_parallel_schedule_matches_reference_hits10(ds, model, dim, epochs, compat, learns):
    out = schedule_parity(ds, model, dim, epochs, seed_epochs=300, rate=0.001, method=1, batches=100, seed=7,
                          transr_compat=compat)
    o, p = out["ordered"], out["parallel"]
    print({k: (o[k], p[k]) for k in ("filtered_hits10", "raw_hits10", "filtered_rank", "raw_rank")})
    if learns:
        assert o["filtered_hits10"] >= 10 * out["random_hits10"], o
    assert abs(out["delta_filtered_hits10_pp"]) <= HITS_TOL_PP, out
    assert abs(out["delta_raw_hits10_pp"]) <= HITS_TOL_PP, out
    assert abs(p["filtered_rank"] - o["filtered_rank"]) <= RANK_TOL_REL * o["filtered_rank"], out
    # same sample stream: the final epoch's hinge-active counts stay close
    assert abs(p["losses"][-1][2] - o["losses"][-1][2]) <= 0.05 * o["losses"][-1][2]
    # and the loss trajectory: the last 10 epochs' mean loss
    lo = sum(x[1] for x in o["losses"][-10:]) / 10
    lp = sum(x[1] for x in p["losses"][-10:]) / 10
    print("last-10 loss", lp, lo, (lp - lo) / lo)
    assert abs(lp - lo) <= (LOSS_TOL_REL if compat or model != "R" else LOSS_TOL_FIXED) * lo, (lp, lo)
