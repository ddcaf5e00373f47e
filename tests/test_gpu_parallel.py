"""PARALLEL schedule on the GPU vs its CPU model (oracle/parallel.py).

The schedule keeps the reference's sample stream, snapshot energies, hinge
decisions and update directions and applies each touched row's summed delta
plus one norm per batch (include/kb2e_engine.h KB2E_SCHEDULE_PARALLEL).  The
CPU model follows the same arithmetic (L1 deltas as integer sign counts), so
the bar is the ulp-level difference of the 64-lane sums in the norms:
1e-11 absolute per epoch, identical active counts, loss to 1e-9 relative.
"""
import os

import numpy as np
import pytest

from gpu_common import max_abs, tiny
from kb2e_amd import data
from kb2e_amd.engine import Engine
from oracle import orc
from oracle.parallel import transe_parallel_batches

pytestmark = pytest.mark.gpu

P_ATOL = 1e-11


def _transe_vs_model(ds, dim, epochs, *, distance=0, method=1, batches=20, rate=0.01, seed=3, apply_long=None,
                     monkeypatch=None):
    if apply_long is not None:
        monkeypatch.setenv("KB2E_APPLY_LONG", str(apply_long))
    m = orc.Model("E", dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                  batches=batches)
    m.set_triples(ds.train)
    orc.srand(seed)
    m.prep_train()
    pe, pr, _ = m.tables()
    eng = Engine("E", dim, ds.num_entities, ds.num_relations, rate=rate, method=method, distance=distance,
                 batches=batches, seed=seed, schedule="parallel")
    eng.upload_triples(ds.train)
    e0, r0, _ = eng.init_params()
    assert np.array_equal(e0, pe) and np.array_equal(r0, pr)
    B = m.batch_size()
    for ep in range(epochs):
        si, sj, side = m.sample_stream(B * batches)
        lo, ao = transe_parallel_batches(pe, pr, ds.train, si, sj, side, B, batches, rate=rate, l1=distance == 0)
        lg, ag = eng.train_epoch()
        assert ag == ao, (ep, ag, ao)
        assert abs(lg - lo) <= 1e-9 * max(1.0, abs(lo))
        ge, gr, _ = eng.download_params()
        assert max_abs(ge, pe) < P_ATOL and max_abs(gr, pr) < P_ATOL, (ep, max_abs(ge, pe), max_abs(gr, pr))
    return eng


@pytest.mark.parametrize("dim,distance", [(50, 0), (100, 0), (100, 1), (17, 0), (200, 0), (130, 1)])
def test_transe_parallel_small(dim, distance):
    """Ragged and multi-chunk row widths on a 30k-triple set, 2 epochs."""
    _transe_vs_model(data.synthetic("small", seed=1), dim, 2, distance=distance)


@pytest.mark.parametrize("apply_long", [0, 1, 64])
def test_transe_parallel_long_segments(apply_long, monkeypatch):
    """Every segment through the 16-wave long path (1), none (0), the default split."""
    _transe_vs_model(data.synthetic("small", seed=2), 64, 2, batches=5, apply_long=apply_long,
                     monkeypatch=monkeypatch)


def test_transe_parallel_single_batch_self_loops():
    ds = data.synthetic("tiny", seed=5)
    extra = np.array([[3, 3, 1], [7, 7, 2]] + ds.train[:50].tolist(), dtype=np.int32)
    ds.train = np.concatenate([ds.train, extra])
    _transe_vs_model(ds, 20, 3, batches=1, method=0)


def test_transe_parallel_deterministic():
    ds = data.synthetic("small", seed=4)
    outs = []
    for _ in range(2):
        eng = Engine("E", 100, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=8, schedule="parallel")
        eng.upload_triples(ds.train)
        eng.init_params()
        eng.train_epoch()
        outs.append(eng.download_params()[:2])
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def _cons_form(dim, mfma):
    """The transRNorm form the engine runs (engine_transr_parallel.inc): the
    per-relation sequential chain (every pair against the matrix the earlier
    ones left) in FP64 up to n = 112 -- kernels_transr_pipe.hpp on
    the n <= 64 matrix-core path, kernels_transr_chainwp.hpp at 64 < n <= 100,
    kernels_transr_chainw.hpp elsewhere -- unless
    KB2E_RPAR_CONS picks the Jacobi tile / wave kernels; Jacobi above 112."""
    ck = os.environ.get("KB2E_RPAR_CONS", "")
    if ck in ("tile", "jacobi") and dim <= 128:
        return "jacobi"
    assert dim <= 512, "PARALLEL TransR trains n <= 512"
    return "chunk1"


def _transr_vs_model(ds, dim, epochs, monkeypatch, *, St=8, compat=False, distance=0, batches=10, rate=0.01,
                     seed=3, atol=1e-9, mfma=True, sub=1):
    from oracle.parallel import transr_parallel_batches
    monkeypatch.setenv("KB2E_RPAR_ST", str(St))
    monkeypatch.setenv("KB2E_RPAR_MFMA", "1" if mfma else "0")
    cons = _cons_form(dim, mfma)
    m = orc.Model("R", dim, ds.num_entities, ds.num_relations, rate=rate, distance=distance, batches=batches,
                  transr_compat=compat)
    m.set_triples(ds.train)
    orc.srand(seed)
    m.prep_train()
    pe, pr, pw = m.tables()
    eng = Engine("R", dim, ds.num_entities, ds.num_relations, rate=rate, distance=distance, batches=batches,
                 seed=seed, schedule="parallel", transr_compat=compat, sub_batches=sub)
    eng.upload_triples(ds.train)
    e0, r0, w0 = eng.init_params()
    assert np.array_equal(e0, pe) and np.array_equal(r0, pr) and np.array_equal(w0, pw)
    eng.transr_seed(e0, r0)  # TransR seed step with the init tables (transr/trainer.cpp:88-113)
    pe = pe / np.linalg.norm(pe, axis=1, keepdims=True)
    work = [np.zeros(dim), np.zeros(dim)]
    B = m.batch_size()
    for ep in range(epochs):
        si, sj, side = m.sample_stream(B * batches)
        lo, ao = transr_parallel_batches(pe, pr, pw, ds.train, si, sj, side, B, batches, rate=rate,
                                         l1=distance == 0, compat=compat, work=work, St=St, cons=cons, sub=sub)
        lg, ag = eng.train_epoch()
        assert ag == ao, (ep, ag, ao)
        assert abs(lg - lo) <= 1e-9 * max(1.0, abs(lo))
        ge, gr, gw = eng.download_params()
        errs = (max_abs(ge, pe), max_abs(gr, pr), max_abs(gw, pw))
        assert max(errs) < atol, (ep, errs)


@pytest.mark.parametrize("mfma", [True, False])
@pytest.mark.parametrize("dim,distance,St", [(20, 0, 8), (20, 1, 4), (50, 0, 8), (33, 0, 2), (40, 0, 8), (64, 0, 1),
                                             (65, 0, 2), (96, 0, 8), (100, 0, 8), (100, 1, 4), (112, 0, 2),
                                             (128, 0, 1)])
def test_transr_parallel_fixed(dim, distance, St, mfma, monkeypatch):
    """Fixed (zeroed) energy; tiles of St samples (several per hot relation); the
    matrix-core kernels and the VALU ones.  St must not exceed the engine's own
    LDS-bounded choice (KB2E_RPAR_ST only lowers it)."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, distance=distance, mfma=mfma)


@pytest.mark.parametrize("dim,distance,St,compat", [(20, 0, 8, False), (50, 0, 8, True), (33, 1, 4, False)])
def test_transr_parallel_cons_tile_kernel(dim, distance, St, compat, monkeypatch):
    """The LDS-round transRNorm kernel (transr_cons_tile_kernel), which n <= 64
    replaces by the register-resident one (kernels_transr_cons.hpp) by default."""
    monkeypatch.setenv("KB2E_RPAR_CONS", "tile")
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, distance=distance, compat=compat)


@pytest.mark.parametrize("dim,St,compat", [(20, 8, False), (50, 4, True), (64, 2, True), (17, 8, False), (18, 8, False),
                                            (49, 8, False), (33, 4, True)])
def test_transr_parallel_chain_widths(dim, St, compat, monkeypatch):
    """The per-relation sequential transRNorm kernel (kernels_transr_pipe.hpp) at
    one to four column slices (n = 17 .. 64): relations of the tiny set hold ~90
    pairs a batch, so several 32-pair chunks and several violators a chunk, each
    pair against the matrix the earlier ones left."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=compat)


@pytest.mark.parametrize("dim,compat,env,St", [(50, True, "KB2E_RPAR_CHAIN_LIST=64", 8),
                                               (33, False, "KB2E_RPAR_CHAIN_LIST=64", 8),
                                               (50, True, "KB2E_RPAR_CHAIN_TILES=2", 1),
                                               (20, False, "KB2E_RPAR_CHAIN_TILES=3", 1)])
def test_transr_parallel_chain_windows(dim, compat, env, St, monkeypatch):
    """The chain kernels over several windows of a relation's pairs
    (KB2E_RPAR_CHAIN_LIST=64 against ~90 pairs a relation a batch on the tiny
    set; FB15k's hottest relation fits one 1,536-pair window): W_c, K0 and the
    tail bookkeeping carry across windows, the result is the same model's.
    KB2E_RPAR_CHAIN_TILES caps the tiles a window (one sample a tile), so the
    window holding the relation's last active sample usually ends before the
    relation's trailing inactive tiles: the tail (the last update's pairs after
    W_c's rows are renormalised) must still be isolated there."""
    name, val = env.split("=")
    monkeypatch.setenv(name, val)
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=compat)


@pytest.mark.parametrize("chain", ["default", "lockstep"])
@pytest.mark.parametrize("dim,compat,mfma", [(100, True, False), (100, False, False), (72, True, True),
                                             (20, True, False), (88, False, True)])
def test_transr_parallel_wide_chain_windows(dim, compat, mfma, chain, monkeypatch):
    """The wide chain kernels over several windows of a relation (256 samples
    for the pipelined kernel, kernels_transr_chainwp.hpp, the default at
    64 < n <= 100; 512 for the lockstep one, kernels_transr_chainw.hpp,
    KB2E_RPAR_CHAIN=lockstep): the small set's hottest relation holds ~700
    samples a batch (B = 3,000), so W_c, K0, the pipeline's pending W update and
    the held-back tail (the relation's last update) carry across windows; n = 20
    on the VALU path runs the lockstep kernel at one column tile either way."""
    if chain != "default":
        monkeypatch.setenv("KB2E_RPAR_CHAIN", chain)
    _transr_vs_model(data.synthetic("small", seed=1), dim, 1, monkeypatch, St=2 if mfma else 8, compat=compat,
                     mfma=mfma, rate=0.001)


@pytest.mark.parametrize("dim,St", [(20, 8), (50, 8)])
def test_transr_parallel_jacobi_wave_kernel(dim, St, monkeypatch):
    """KB2E_RPAR_CONS=jacobi: the register-resident tile kernel (every pair of
    the batch against the same matrix, corrections summed)."""
    monkeypatch.setenv("KB2E_RPAR_CONS", "jacobi")
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=True)


@pytest.mark.parametrize("mfma", [True, False])
@pytest.mark.parametrize("dim,St", [(20, 8), (50, 8), (65, 2), (100, 8)])
def test_transr_parallel_compat(dim, St, mfma, monkeypatch):
    """The reference's accumulating work-vector energy (transr/transr.cpp:20-25).
    n = 65: matrix-core images at St = 2; n = 100 (K5): the VALU tile kernels
    (the f64 matrix-core transRNorm image does not fit the LDS there)."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=True, mfma=mfma)


@pytest.mark.parametrize("dim,mfma", [(50, True), (100, True), (100, False)])
def test_transr_parallel_compat_chunk_prefix(dim, mfma, monkeypatch):
    """The compat scan's chunk prefix made once by rpar_scan_prefix_kernel (the
    path of batches with more than kScanDirectMax chunks, K5), forced on the
    tiny set: the same model within rounding."""
    monkeypatch.setenv("KB2E_RPAR_SCAN_PREFIX", "1")
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=2 if dim > 64 else 8, compat=True, mfma=mfma)


def test_transr_parallel_compat_prefix_paths_agree(monkeypatch):
    """Batches of more than kScanDirectMax chunks of the compat work-vector scan
    (K5) take the chunk prefix from rpar_scan_prefix_kernel, which sums in another
    order than every chunk block summing its own prefix.  On batches that large
    (the small set in 2 batches: ~470 chunks each) both paths must give the same
    hinge decisions up to margin ties and the same loss to rounding."""
    ds = data.synthetic("small", seed=1)
    out = {}
    for pre in ("0", "1"):
        monkeypatch.setenv("KB2E_RPAR_SCAN_PREFIX", pre)
        eng = Engine("R", 50, ds.num_entities, ds.num_relations, rate=0.001, batches=2, seed=3, schedule="parallel")
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        out[pre] = [eng.train_epoch() for _ in range(2)]
        eng.close()
    for (l0, a0), (l1, a1) in zip(out["0"], out["1"]):
        assert abs(a0 - a1) <= 2, (a0, a1)
        assert abs(l0 - l1) <= 1e-9 * l0 + 2.0 * abs(a0 - a1), (l0, l1)


@pytest.mark.parametrize("dim", [100, 128])
def test_transr_parallel_rows8(dim, monkeypatch):
    """KB2E_RPAR_ROWS8=1: the relation-row passes four rows a wave, eight elements a
    lane (n <= 128; a different norm reduction order): the same model."""
    monkeypatch.setenv("KB2E_RPAR_ROWS8", "1")
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=2, mfma=False)


def _hub_dataset(ne=300, nr=6, count=4000, seed=5):
    """Entity 0 heads ~half the triples: its event segments run to hundreds of
    events a batch (pair_prev_long_kernel's LDS table path)."""
    rng = np.random.default_rng(seed)
    h = np.where(rng.random(count) < 0.5, 0, rng.integers(1, ne, count))
    t = rng.integers(1, ne, count)
    r = rng.integers(0, nr, count)
    tr = np.unique(np.stack([h, t, r], 1).astype(np.int32), axis=0)
    tr = tr[rng.permutation(len(tr))]
    return data.Dataset(ne, nr, tr, tr[:0], tr[:0])


@pytest.mark.parametrize("St", [8, 1])
def test_transr_parallel_hub_entity(St, monkeypatch):
    """Per-relation pair dedupe through long entity segments (hub entity)."""
    _transr_vs_model(_hub_dataset(), 20, 2, monkeypatch, St=St, batches=5)


def test_transr_parallel_independent_of_tile_size(monkeypatch):
    """transRNorm pairs are deduplicated per relation per batch, so cutting the
    relations into tiles of 1, 2 or 8 samples changes only the order of the
    floating-point sums (the tile partials)."""
    ds = tiny()
    outs = []
    for St in (1, 2, 8):
        monkeypatch.setenv("KB2E_RPAR_ST", str(St))
        eng = Engine("R", 20, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=3,
                     schedule="parallel")
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        stats = [eng.train_epoch() for _ in range(2)]
        outs.append((stats, eng.download_params()))
    for stats, tabs in outs[1:]:
        assert [a for _, a in stats] == [a for _, a in outs[0][0]]
        for x, y in zip(tabs, outs[0][1]):
            assert max_abs(x, y) < 1e-12


@pytest.mark.parametrize("dim,St,compat", [(120, 2, False), (128, 1, True), (113, 2, False)])
def test_transr_parallel_generic_chain_wide(dim, St, compat, monkeypatch):
    """112 < n <= 128: the pair-by-pair chain in double arithmetic without the matrix
    cores (kernels_transr_chaing.hpp), the same CPU model as every other width."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=compat)


@pytest.mark.parametrize("dim,St,compat,mfma", [(20, 8, False, True), (50, 8, True, True), (33, 4, True, False),
                                                (100, 8, False, False)])
def test_transr_parallel_generic_chain_forced(dim, St, compat, mfma, monkeypatch):
    """KB2E_RPAR_CHAIN=gen: the generic chain where the matrix-core chains would run
    (their model, so the same bar), on both phase-A paths."""
    monkeypatch.setenv("KB2E_RPAR_CHAIN", "gen")
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=compat, mfma=mfma)


def test_transr_parallel_generic_chain_windows(monkeypatch):
    """The generic chain over several 128-sample windows of a relation (the small
    set's hottest relation holds ~700 samples a batch): W_c and the held-back tail
    carry across windows."""
    monkeypatch.setenv("KB2E_RPAR_CHAIN", "gen")
    _transr_vs_model(data.synthetic("small", seed=1), 50, 1, monkeypatch, St=8, compat=True, rate=0.001)


@pytest.mark.parametrize("dim,compat,St_cap", [(160, False, 8), (160, True, 8), (260, False, 8), (260, True, 2),
                                               (384, False, 8), (512, True, 8)])
def test_transr_parallel_wide(dim, compat, St_cap, monkeypatch):
    """128 < n <= 512 (kernels_transr_widep.hpp: every matrix from global memory,
    up to four element pairs a lane): the same model as the narrower kernels --
    summed gradient step, then transRNorm pair by pair per relation (cons =
    "chunk1") -- against oracle/parallel.py, both energies, two epochs of the tiny
    set (several chunks and violators a relation); St_cap caps the tile size below
    the LDS-bounded choice (several tiles a relation)."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St_cap, compat=compat, mfma=False)


@pytest.mark.parametrize("sub,prefix", [(1, "0"), (1, "1"), (3, "0"), (3, "1")])
def test_transr_parallel_wide_compat_scan(sub, prefix, monkeypatch):
    """The wide kernels' compat scan in both forms (KB2E_RPAR_SCAN_PREFIX: the chunks'
    prefix made once, or summed by every chunk block), whole batches and sub-batches
    (phase A on the start-of-batch copies), n = 200."""
    monkeypatch.setenv("KB2E_RPAR_SCAN_PREFIX", prefix)
    _transr_vs_model(tiny(), 200, 2, monkeypatch, St=4, compat=True, mfma=False, sub=sub)


def test_transr_parallel_wide_fp32_close():
    """FP32 tables at n = 200 on the wide kernels: loss and active counts within 1 %
    of the FP64 run over two epochs (FP32 hinge decisions flip at the margin)."""
    ds = data.synthetic("small", seed=1)
    out = {}
    for prec in (64, 32):
        eng = Engine("R", 200, ds.num_entities, ds.num_relations, rate=0.001, batches=10, seed=3, precision=prec,
                     schedule="parallel", transr_compat=False)
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        out[prec] = [eng.train_epoch() for _ in range(2)]
        eng.close()
    for (l64, a64), (l32, a32) in zip(out[64], out[32]):
        assert abs(a64 - a32) <= 0.01 * a64 and abs(l64 - l32) <= 0.01 * l64


def test_transr_parallel_refuses_above_512():
    """Every --size up to the engine's cap trains PARALLEL; wider contexts are refused
    at creation (KB2E_EINVAL, as for every model)."""
    from kb2e_amd.engine import EngineError
    ds = tiny()
    with pytest.raises(EngineError, match="EINVAL"):
        Engine("R", 513, ds.num_entities, ds.num_relations, schedule="parallel")


def test_transr_parallel_fp32_chain_close(monkeypatch):
    """FP32 tables take the same pair-by-pair chain (double arithmetic, FP32
    storage): epoch loss and active counts within 1 % of the FP64 run, the tables
    within FP32 rounding drift (median 1e-3)."""
    ds = data.synthetic("small", seed=1)
    out, tabs = {}, {}
    for prec in (64, 32):
        eng = Engine("R", 50, ds.num_entities, ds.num_relations, rate=0.001, batches=10, seed=3, precision=prec,
                     schedule="parallel", transr_compat=False)
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        out[prec] = [eng.train_epoch() for _ in range(2)]
        tabs[prec] = eng.download_params()
        eng.close()
    for (l64, a64), (l32, a32) in zip(out[64], out[32]):
        assert abs(a64 - a32) <= 0.01 * a64 and abs(l64 - l32) <= 0.01 * l64
    for x, y in zip(tabs[64], tabs[32]):
        assert np.median(np.abs(x - y)) < 1e-3


def test_transr_parallel_fp32_close(monkeypatch):
    """FP32 tables: hinge decisions flip at the margin, so statistics, not elements.
    (Both on the Jacobi transRNorm, which KB2E_RPAR_CONS=jacobi asks for by name; by
    default FP32 takes the generic pair-by-pair chain: test_transr_parallel_fp32_chain_close.)"""
    monkeypatch.setenv("KB2E_RPAR_CONS", "jacobi")
    ds = tiny()
    out = {}
    for prec in (64, 32):
        eng = Engine("R", 20, ds.num_entities, ds.num_relations, rate=0.01, batches=10, seed=3, precision=prec,
                     schedule="parallel", transr_compat=False)
        eng.upload_triples(ds.train)
        e0, r0, _ = eng.init_params()
        eng.transr_seed(e0, r0)
        out[prec] = [eng.train_epoch() for _ in range(2)]
    for (l64, a64), (l32, a32) in zip(out[64], out[32]):
        assert abs(a64 - a32) <= 0.01 * a64 and abs(l64 - l32) <= 0.01 * l64


def _transh_vs_model(ds, dim, epochs, *, batches=10, rate=0.01, seed=3, method=1, atol=1e-9, orth_min=None):
    from oracle.parallel import ORTH_REL_MIN, transh_parallel_batches
    m = orc.Model("H", dim, ds.num_entities, ds.num_relations, rate=rate, method=method, batches=batches)
    m.set_triples(ds.train)
    orc.srand(seed)
    m.prep_train()
    pe, pr, pw = m.tables()
    eng = Engine("H", dim, ds.num_entities, ds.num_relations, rate=rate, method=method, batches=batches, seed=seed,
                 schedule="parallel")
    eng.upload_triples(ds.train)
    e0, r0, w0 = eng.init_params()
    assert np.array_equal(e0, pe) and np.array_equal(r0, pr) and np.array_equal(w0, pw)
    B = m.batch_size()
    state = {}  # the previous batch's flagged samples, across epochs as in the engine
    for ep in range(epochs):
        si, sj, side = m.sample_stream(B * batches)
        lo, ao = transh_parallel_batches(pe, pr, pw, ds.train, si, sj, side, B, batches, rate=rate, state=state,
                                         orth_rel_min=ORTH_REL_MIN if orth_min is None else orth_min)
        lg, ag = eng.train_epoch()
        assert ag == ao, (ep, ag, ao)
        assert abs(lg - lo) <= 1e-9 * max(1.0, abs(lo))
        ge, gr, gw = eng.download_params()
        errs = (max_abs(ge, pe), max_abs(gr, pr), max_abs(gw, pw))
        assert max(errs) < atol, (ep, errs)


@pytest.mark.parametrize("dim", [20, 100, 17, 130])
def test_transh_parallel(dim):
    """Tiny set, lr 0.01: the orthogonality loop fires; ragged and multi-chunk widths."""
    _transh_vs_model(tiny(), dim, 2)


@pytest.mark.parametrize("orth_min", [0, 1 << 30, 8])
def test_transh_parallel_orth_gate(orth_min, monkeypatch):
    """normOrth's relation pass runs only when the previous batch's normOrth work
    was at least KB2E_HPAR_ORTH_MIN loop iterations (0: always; huge: never, the
    one-wave pass takes the relations' own pairs in its first sweep; 8: batches
    of both kinds on the tiny set).  The result does not depend on it: one CPU
    model for all three."""
    monkeypatch.setenv("KB2E_HPAR_ORTH_MIN", str(orth_min))
    _transh_vs_model(tiny(), 20, 2, orth_min=orth_min)


@pytest.mark.parametrize("orth_min", [0, 1 << 30])
def test_transh_parallel_orth_requeue(orth_min, monkeypatch):
    """KB2E_HPAR_ORTH_Q=0: the one-wave pass's second sweep (the entity rows several
    relations flagged) lists the flags again instead of running from its LDS queue
    (the form past 512 queued samples); the same CPU model."""
    monkeypatch.setenv("KB2E_HPAR_ORTH_Q", "0")
    monkeypatch.setenv("KB2E_HPAR_ORTH_MIN", str(orth_min))
    _transh_vs_model(tiny(), 20, 2, orth_min=orth_min)


@pytest.mark.parametrize("waves", [16, 4])
def test_transh_parallel_unfused(waves, monkeypatch):
    """KB2E_HPAR_FUSE=0: the relation normals and the row sums as two launches, the
    normals' workgroups of 16 or 4 waves (as many relation segments each: the small
    ones a wave's, the larger ones the whole workgroup's)."""
    monkeypatch.setenv("KB2E_HPAR_FUSE", "0")
    monkeypatch.setenv("KB2E_WAPPLY_WAVES", str(waves))
    _transh_vs_model(data.synthetic("small", seed=1), 64, 1, batches=20, rate=0.001)


def test_transh_parallel_small():
    _transh_vs_model(data.synthetic("small", seed=1), 64, 2, batches=20, rate=0.001)



def test_transr_chain_wait_timeout_fails_loudly(monkeypatch):
    """A bounded in-workgroup wait of the pipelined chain that times out (forced:
    KB2E_CONS_DBG bit 32 keeps one helper wave from arriving) leaves invalid
    tables; kb2e_synchronize and kb2e_download_params report it, not only
    kb2e_take_stats (engine_relowner.inc check_dataflow)."""
    monkeypatch.setenv("KB2E_CONS_DBG", "32")
    ds = tiny()
    eng = Engine("R", 20, ds.num_entities, ds.num_relations, rate=0.01, batches=20, seed=7, schedule="parallel")
    eng.upload_triples(ds.train)
    e0, r0, _ = eng.init_params()
    eng.transr_seed(e0, r0)
    eng.train_batches(1)
    with pytest.raises(RuntimeError, match="timed out"):
        eng.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        eng.download_params()
    eng.close()


@pytest.mark.parametrize("sub", [2, 3, 4])
@pytest.mark.parametrize("dim,compat,mfma,St", [(50, True, True, 8), (20, False, True, 8), (33, True, False, 4),
                                                 (100, True, False, 8), (100, False, True, 2)])
def test_transr_parallel_sub_batches(dim, compat, mfma, St, sub, monkeypatch):
    """kb2e_config.sub_batches: phase B of every batch in `sub` ordered
    sub-batches of ceil(B / sub) samples (3 leaves a shorter last one), phase A on
    the start-of-batch tables, against oracle/parallel.py with the same `sub`:
    the pipelined chain (n = 50, 20), the lockstep / VALU paths (33), K5's width
    on both phase-A paths (100)."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=compat, mfma=mfma, sub=sub)


@pytest.mark.parametrize("dim,compat,mfma,St,sub,batches", [(50, True, True, 8, 2, 9), (50, True, True, 8, 3, 7),
                                                             (20, True, True, 4, 4, 9), (33, True, False, 4, 2, 9),
                                                             (100, True, False, 8, 2, 9), (100, True, True, 8, 4, 9),
                                                             (160, True, True, 8, 2, 9), (50, False, True, 8, 2, 9)])
def test_transr_parallel_sub_batches_ragged(dim, compat, mfma, St, sub, batches, monkeypatch):
    """Batches that `sub` does not divide (333 samples at 9 batches, 428 at 7: the
    last sub-batch shorter, as on the FB15k-shaped set's 4,831): the compat scan
    of a sub-batch covers its own calls only, so the carried work vectors the
    next batch starts from are the reference's."""
    _transr_vs_model(tiny(), dim, 2, monkeypatch, St=St, compat=compat, mfma=mfma, sub=sub, batches=batches)


def test_transr_parallel_sub_batches_small_set(monkeypatch):
    """Sub-batches on the 30k-triple set (a hot relation of ~700 samples a batch:
    several chunks and windows a sub-batch), compat energy, n = 50."""
    _transr_vs_model(data.synthetic("small", seed=1), 50, 1, monkeypatch, St=8, compat=True, rate=0.001, sub=4)


@pytest.mark.parametrize("model,dim,schedule,sub,want", [("R", 50, "parallel", None, 2), ("R", 64, "parallel", None, 2),
                                                          ("R", 65, "parallel", None, 3), ("R", 100, "parallel", None, 3),
                                                          ("R", 300, "parallel", None, 3), ("R", 50, "ordered", None, 1),
                                                          ("E", 50, "parallel", None, 1), ("R", 50, "parallel", 1, 1),
                                                          ("R", 100, "parallel", 4, 4)])
def test_sub_batch_default_by_width(model, dim, schedule, sub, want):
    """kb2e_config.sub_batches = 0 (kb2e_default_config) resolves by width at
    kb2e_create -- 2 for PARALLEL TransR at n <= 64, 3 above, 1 elsewhere -- and
    kb2e_get_config reports the count the context runs; an explicit count stays."""
    ds = tiny()
    eng = Engine(model, dim, ds.num_entities, ds.num_relations, batches=10, schedule=schedule, sub_batches=sub)
    try:
        assert eng.cfg.sub_batches == want
    finally:
        eng.close()
