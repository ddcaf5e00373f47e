"""CPU model of the engine's PARALLEL schedule (TEST INFRASTRUCTURE ONLY).

The PARALLEL schedule (include/kb2e_engine.h KB2E_SCHEDULE_PARALLEL,
kb2e_amd/csrc/kernels_parallel.hpp) is not the reference's algorithm: it keeps
the reference's sample stream, snapshot energies, hinge decisions and update
directions (common/trainer.cpp:130-149, transe/trainer.cpp:24-46) and replaces
the per-update renormalisation sequence with one summed delta + one
common::norm per touched row and batch.  This module restates that relaxation
in numpy on top of the C oracle's sample stream, so tests can check the GPU
kernels element by element.  Only tests/ import it.
"""
from __future__ import annotations

import numpy as np


def _norm_rows(tab: np.ndarray, rows: np.ndarray, ignore_short: bool = True) -> None:
    """common::norm (common/utils.cpp:70-77) on the listed rows."""
    if rows.size == 0:
        return
    v = tab[rows]
    ln = np.sqrt((v * v).sum(axis=1))
    scale = (ln > 1.0) if ignore_short else np.ones_like(ln, dtype=bool)
    v[scale] = v[scale] / ln[scale, None]
    tab[rows] = v


def transe_parallel_batches(ent, rel, triples, si, sj, side, B, nbatches, *, rate, margin=1.0, l1=True):
    """Train `nbatches` TransE batches of the PARALLEL schedule in place.

    Returns (loss, active).  Per batch: energies and directions from the
    start-of-batch tables (transe/transe.cpp:10-28, transe/trainer.cpp:27-35);
    deltas summed per row (L1: integer sign counts, as the kernel); then
    row <- norm(row + rate * sum) for every row an active update touched.
    """
    loss = 0.0
    active = 0
    h_all, t_all, r_all = triples[:, 0], triples[:, 1], triples[:, 2]
    for b in range(nbatches):
        sl = slice(b * B, (b + 1) * B)
        i, j, sd = si[sl], sj[sl], side[sl].astype(bool)
        h, t, r = h_all[i], t_all[i], r_all[i]
        nh = np.where(sd, h, j)
        nt = np.where(sd, j, t)
        dp = ent[t] - ent[h] - rel[r]
        dn = ent[nt] - ent[nh] - rel[r]
        ep = np.abs(dp).sum(1) if l1 else (dp * dp).sum(1)
        en = np.abs(dn).sum(1) if l1 else (dn * dn).sum(1)
        act = ep + margin > en
        loss += float((margin + ep - en)[act].sum())
        active += int(act.sum())
        if l1:
            xp = np.where(dp > 0, 1, -1).astype(np.int64)
            xn = np.where(dn > 0, 1, -1).astype(np.int64)
            acc_e = np.zeros(ent.shape, np.int64)
            acc_r = np.zeros(rel.shape, np.int64)
        else:
            xp, xn = 2.0 * dp, 2.0 * dn
            acc_e = np.zeros(ent.shape)
            acc_r = np.zeros(rel.shape)
        a = np.nonzero(act)[0]
        # modifier: -1 for the training triple, +1 for the corrupted one
        # (transe/trainer.cpp:25, 38-40): rel -= m lr x, head -= m lr x, tail += m lr x
        for (hh, tt, xx, m) in ((h[a], t[a], xp[a], -1), (nh[a], nt[a], xn[a], 1)):
            np.add.at(acc_r, r[a], -m * xx)
            np.add.at(acc_e, hh, -m * xx)
            np.add.at(acc_e, tt, m * xx)
        er = np.unique(np.concatenate([h[a], t[a], nh[a], nt[a]]))
        rr = np.unique(r[a])
        ent[er] = ent[er] + rate * acc_e[er]
        rel[rr] = rel[rr] + rate * acc_r[rr]
        _norm_rows(ent, er)
        _norm_rows(rel, rr)
    return loss, active


def sub_batch_bounds(B, sub):
    """The sample ranges of a batch's `sub` sub-batches: ceil(B / sub) samples
    each, the last one the rest (kb2e_config.sub_batches)."""
    bs = -(-B // sub)
    return [(j * bs, min(B, (j + 1) * bs)) for j in range(sub) if j * bs < B]


def transr_parallel_batches(ent, rel, W, triples, si, sj, side, B, nbatches, *, rate, margin=1.0, l1=True,
                            compat=False, work=None, St=32, constraint=True, cons="jacobi", stats=None, sub=1):
    """Train `nbatches` TransR batches of the PARALLEL schedule in place
    (kb2e_amd/csrc/kernels_transr_parallel.hpp).  Returns (loss, active).

    Per batch, from the start-of-batch tables (transr/trainer.cpp:144-188):
    projections, energies (compat: the reference's accumulating work vectors,
    transr/transr.cpp:20-25, carried in `work` = [head, tail]), hinge, x, d =
    h - t, y = W x; summed dW, dr per relation, summed entity deltas; unit
    norms; then transRNorm (transr/trainer.cpp:35-64) on every (h', r), (t', r)
    pair of an active update and (entity'[r], r) once per relation, iterated
    while |W^T a|^2 > 1 (transr_constraint: `cons` picks the kernel's form).

    sub > 1: the batch's phase B in `sub` ordered sub-batches (sub_batch_bounds):
    the energies, hinge decisions and update directions (x, d = h - t, y = W x)
    all come from the start-of-batch tables as before (the reference's snapshot,
    common/trainer.cpp:132-133), and each sub-batch in turn sums its own deltas,
    renormalises and runs its transRNorm pairs (first occurrences per relation per
    sub-batch) -- nearer the reference's renormalisation after every update
    (transr/trainer.cpp:174-187) by a factor `sub` in the samples summed per norm.
    """
    loss = 0.0
    active = 0
    h_all, t_all, r_all = triples[:, 0], triples[:, 1], triples[:, 2]
    for b in range(nbatches):
        sl = slice(b * B, (b + 1) * B)
        i, j, sd = si[sl], sj[sl], side[sl].astype(bool)
        h, t, r = h_all[i], t_all[i], r_all[i]
        nh = np.where(sd, h, j)
        nt = np.where(sd, j, t)
        Wr = W[r]                                   # [B][j][i]
        proj = lambda v: np.einsum("kji,kj->ki", Wr, ent[v])
        ph, pt, pnh, pnt = proj(h), proj(t), proj(nh), proj(nt)
        R = rel[r]
        if compat:
            calls_h = np.stack([ph, pnh], 1).reshape(-1, ph.shape[1])
            calls_t = np.stack([pt, pnt], 1).reshape(-1, pt.shape[1])
            hw = work[0] + np.cumsum(calls_h, axis=0)
            tw = work[1] + np.cumsum(calls_t, axis=0)
            work[0], work[1] = hw[-1].copy(), tw[-1].copy()
            dpe = (tw[0::2] - hw[0::2]) - R
            dne = (tw[1::2] - hw[1::2]) - R
        else:
            dpe, dne = (pt - ph) - R, (pnt - pnh) - R
        ep = np.abs(dpe).sum(1) if l1 else (dpe * dpe).sum(1)
        en = np.abs(dne).sum(1) if l1 else (dne * dne).sum(1)
        act = ep + margin > en
        loss += float((margin + ep - en)[act].sum())
        active += int(act.sum())
        dp, dn = (pt - ph) - R, (pnt - pnh) - R    # fresh projections (transr/trainer.cpp:147-157)
        xp = np.where(dp > 0, 1.0, -1.0) if l1 else 2.0 * dp
        xn = np.where(dn > 0, 1.0, -1.0) if l1 else 2.0 * dn
        Wsnap = W.copy()
        d_pos, d_neg = ent[h] - ent[t], ent[nh] - ent[nt]  # the snapshot's h - t (phase A)
        for (s0, s1) in sub_batch_bounds(B, sub):
            in_sub = np.zeros(B, bool)
            in_sub[s0:s1] = True
            act_j = act & in_sub
            a = np.nonzero(act_j)[0]
            ups = [(h[a], t[a], xp[a], d_pos[a], rate), (nh[a], nt[a], xn[a], d_neg[a], -rate)]  # c = -lr beta
            dW = np.zeros_like(W)
            dr = np.zeros_like(rel)
            acc = np.zeros_like(ent)
            for (hh, tt, xx, d, c) in ups:
                np.add.at(dW, r[a], c * np.einsum("kj,ki->kji", d, xx))
                np.add.at(dr, r[a], c * xx)
                y = np.einsum("kji,ki->kj", Wsnap[r[a]], xx)
                np.add.at(acc, hh, c * y)
                np.add.at(acc, tt, -c * y)
            ra = np.unique(r[a])
            W[ra] += dW[ra]
            rel[ra] += dr[ra]
            rel[ra] /= np.sqrt((rel[ra] ** 2).sum(1, keepdims=True))
            W[ra] /= np.sqrt((W[ra] ** 2).sum(2, keepdims=True))
            ea = np.unique(np.concatenate([h[a], t[a], nh[a], nt[a]]))
            ent[ea] += acc[ea]
            ent[ea] /= np.sqrt((ent[ea] ** 2).sum(1, keepdims=True))
            if constraint:
                transr_constraint(ent, W, h, t, nh, nt, r, act_j, rate, St, cons=cons, stats=stats)
    return loss, active


def _relation_pairs(r, rr, act, h, t, nh, nt, relpair, ne):
    """The transRNorm pairs of relation rr in the batch: the (h', r), (t', r)
    entities of its active updates in (sample, update, role) order, then
    (entity'[r], r) (transr/trainer.cpp:185-187); first occurrences only."""
    slots = []
    for kk in np.nonzero((r == rr) & act)[0]:
        slots += [h[kk], t[kk], nh[kk], nt[kk]]
    if relpair and rr < ne:
        slots.append(rr)
    seen, uniq = set(), []
    for e in slots:
        if e not in seen:
            seen.add(e)
            uniq.append(int(e))
    return uniq


def _relation_items(r, rr, act, h, t, nh, nt, relpair, ne):
    """_relation_pairs with each pair's update: (entity, (sample, update)), the
    (entity'[r], r) pair last as (r, None)."""
    items, seen = [], set()
    for kk in np.nonzero((r == rr) & act)[0]:
        for u, (hh, tt) in enumerate(((h[kk], t[kk]), (nh[kk], nt[kk]))):
            for e in (int(hh), int(tt)):
                if e not in seen:
                    seen.add(e)
                    items.append((e, (int(kk), u)))
    if relpair and rr < ne and int(rr) not in seen:
        items.append((int(rr), None))
    return items


def transr_norm_rounds(p, a0, K0, Q0, eps, max_iter=256):
    """transRNorm's loop (transr/trainer.cpp:35-64) on the projection p = W^T a:
    p_{t+1} = p_t - eps (K0 + |a|^2) p_t, G = sum of 2 p_t over the rounds t < m
    while |p_t|^2 > 1.  With v = (K0 + |a|^2) p = kappa p + w (w orthogonal to
    p) and rho = 1 - eps kappa: p_t = rho^t p - eps t rho^(t-1) w to first order
    in eps along w (exact for m <= 2, geometric for long runs), so
    |p_t|^2 = rho^2t Q0 + eps^2 t^2 rho^(2t-2) |w|^2 and
    G = 2 (S0 p - eps S1 w), S0 = sum rho^t, S1 = sum t rho^(t-1).  Returns (G, m)."""
    s0 = a0 @ a0
    V = K0 @ p
    pp, pV, VV = p @ p, p @ V, V @ V
    v = V + s0 * p
    pv, vv = pV + s0 * pp, VV + 2.0 * s0 * pV + s0 * s0 * pp   # p.v, |v|^2 (as the kernel sums them)
    kappa = pv / pp
    w = v - kappa * p
    w2 = max(vv - kappa * pv, 0.0)
    rho = 1.0 - eps * kappa

    e2w = eps * eps * w2
    m, S0, S1, rt, rtm1 = 0, 0.0, 0.0, 1.0, 0.0  # rt = rho^t, rtm1 = rho^(t-1) (0 at t = 0)
    while m < max_iter and rt * rt * pp + e2w * m * m * rtm1 * rtm1 > 1.0:
        S0 += rt
        S1 += m * rtm1
        m += 1
        rtm1 = rt
        rt *= rho
    return 2.0 * (S0 + eps * S1 * kappa) * p - 2.0 * eps * S1 * v, m


def transr_constraint(ent, W, h, t, nh, nt, r, act, rate, St=None, dedupe=True, relpair=True, max_iter=256,
                      cons="jacobi", stats=None):
    """transRNorm step of the PARALLEL TransR schedule, in place.

    cons = "jacobi" (kernels_transr_mfma.hpp / kernels_transr_parallel.hpp tile
    kernels): per relation of the batch, pairs (h', r), (t', r) of the active
    updates in (sample, update, role) order, then (entity'[r], r)
    (transr/trainer.cpp:187); first occurrences per relation only (the GPU's
    per-batch (relation, entity) table, kernels_transr_parallel.hpp
    transr_pair_dup: independent of how the relation is cut into tiles, so St is
    unused); every pair against the same W' (Jacobi), the loop iterated on the
    projection p = W^T a: p <- p - 2 lr W^T W p - 2 lr |a0|^2 p, G += 2 p while
    |p|^2 > 1, then da = -lr W G, dW = -lr a0 G^T, all summed.

    cons = "chunk<C>" (kernels_transr_seq.hpp, the default for n <= 64): the
    same pairs of a relation walked in order, C at a time; inside a chunk every
    pair against the chunk's W_c (Jacobi), and W_c takes the chunk's
    corrections before the next chunk (Gauss-Seidel across chunks, as the
    reference's successive calls see each other's shrinks).  The pairs of the
    relation's last update (the corrupted triple of its last active sample) and
    (entity'[r], r) form the final chunk, after W_c's rows are renormalised
    (the reference renormalises W' at every update, so only the last update's
    shrinks outlive the batch); likewise an entity's corrections from pairs
    before its own last update are followed by a unit norm, those of its last
    update (or of (entity'[r], r) when no update touches the row) are not.
    Per violator the rounds in closed form (transr_norm_rounds, K0 = W'^T W');
    W_c -= lr a G^T, and da = -lr W G with the relation's final matrix.

    cons = "seq" (probe only, tools/probe_compat_parallel.py): the reference's
    own loop (oracle/orc.c transr_norm) on each pair in order, on the evolving
    matrix.
    """
    ra = np.unique(r[act])
    ne = ent.shape[0]
    if cons == "seq":
        from oracle import orc
        for rr in ra:
            Wm = W[rr].copy()
            nf = 0
            pairs = _relation_pairs(r, rr, act, h, t, nh, nt, relpair, ne)
            for e in pairs:
                if stats is not None:
                    pp = Wm.T @ ent[e]
                    nf += int(pp @ pp > 1.0)
                ent[e], Wm = orc.transr_norm(ent[e], Wm, rate)
            W[rr] = Wm
            if stats is not None:
                stats["pairs"] = stats.get("pairs", 0) + len(pairs)
                stats["fired"] = stats.get("fired", 0) + nf
        return
    W0 = W.copy()
    E1 = ent.copy()
    if cons.startswith("chunk"):
        flags = cons[5:].lstrip("0123456789")  # probe only: "r" renormalise the rows at every chunk
        C = int(cons[5:len(cons) - len(flags)])
        eps = 2.0 * rate
        # the last active update touching every entity (its unit norm in the
        # reference comes after every transRNorm shrink of earlier updates)
        last_upd = {}
        for kk in np.nonzero(act)[0]:
            for u, (hh, tt) in enumerate(((h[kk], t[kk]), (nh[kk], nt[kk]))):
                last_upd[int(hh)] = (int(kk), u)
                last_upd[int(tt)] = (int(kk), u)
        dE_pre = np.zeros_like(ent)
        dE_post = np.zeros_like(ent)
        for rr in ra:
            items = _relation_items(r, rr, act, h, t, nh, nt, relpair, ne)
            kl = int(np.nonzero((r == rr) & act)[0][-1])
            head = [it for it in items if it[1] != (kl, 1) and it[1] is not None]
            tail = [it for it in items if it[1] == (kl, 1) or it[1] is None]
            Wc = W0[rr].copy()
            K0 = Wc.T @ Wc
            changed = False
            recs = []  # (entity, post, G): da = -lr W G with the relation's final matrix
            chunks = [head[c0:c0 + C] for c0 in range(0, len(head), C)]
            first_tail = len(chunks)  # the last update's pairs: chunks of their own (C = 1: one by one)
            chunks += [tail[c0:c0 + C] for c0 in range(0, len(tail), C)]
            for ci, chunk in enumerate(chunks):
                if changed and (ci == first_tail or "r" in flags):
                    # the relation's last update renormalises the rows (transr/trainer.cpp:178-180):
                    # only its own shrinks outlive the batch
                    Wc = Wc / np.sqrt((Wc ** 2).sum(1, keepdims=True))
                A = E1[[e for e, _ in chunk]]
                P = A @ Wc                      # rows p_k = W_c^T a_k
                Q0 = (P * P).sum(1)
                dW = np.zeros_like(Wc)
                for k in np.nonzero(Q0 > 1.0)[0]:
                    e, key = chunk[k]
                    G, m = transr_norm_rounds(P[k], A[k], K0, Q0[k], eps, max_iter)
                    post = (e not in last_upd) if key is None else last_upd.get(e) == key
                    recs.append((e, post, G))
                    dW -= rate * np.outer(A[k], G)
                    changed = True
                    if stats is not None:
                        stats["fired"] = stats.get("fired", 0) + 1
                        stats["rounds"] = stats.get("rounds", 0) + m
                if stats is not None:
                    stats["pairs"] = stats.get("pairs", 0) + len(chunk)
                Wc = Wc + dW
            W[rr] = Wc
            for e, post, G in recs:
                (dE_post if post else dE_pre)[e] += -rate * (Wc @ G)
        pre = np.nonzero(np.any(dE_pre != 0, axis=1))[0]
        ent[pre] += dE_pre[pre]
        ent[pre] /= np.sqrt((ent[pre] ** 2).sum(1, keepdims=True))
        ent += dE_post
        return
    assert cons == "jacobi", cons
    dWc = np.zeros_like(W)
    for rr in ra:
        for e in _relation_pairs(r, rr, act, h, t, nh, nt, relpair, ne):
            a0 = E1[e]
            Wm = W0[rr]
            G = np.zeros_like(a0)
            s0 = a0 @ a0
            p = Wm.T @ a0
            it = 0
            for _ in range(max_iter):
                if not (p @ p > 1.0):
                    break
                G += 2.0 * p
                p = p - 2.0 * rate * (Wm.T @ (Wm @ p)) - 2.0 * rate * s0 * p
                it += 1
            if stats is not None:
                stats["pairs"] = stats.get("pairs", 0) + 1
                stats["fired"] = stats.get("fired", 0) + (it > 0)
            ent[e] += -rate * (Wm @ G)
            dWc[rr] += np.outer(-rate * a0, G)
    W[ra] += dWc[ra]


def transh_orth_order(samples, flags, ids, r):
    """The order of the PARALLEL TransH normOrth replays (kernels_transh_parallel.hpp
    transh_orth_rel_kernel, then transh_orth_fix_kernel): first the (sample, row)
    pairs whose row only their own relation touches this batch -- the relation
    row (q = 0) and the entity rows flagged under that relation alone -- samples
    in order (the relations' passes touch disjoint rows and normals, so this is
    one valid order of the per-relation passes); then, samples in order, the
    entity rows flagged under several relations.  flags[i]: the flagged row
    slots q of samples[i] (0 relation, 1 h, 2 t, 4 h', 5 t'); ids[kk][q]: the
    row id.  Returns [(sample, q)]."""
    ent_rels = {}
    for kk, fl in zip(samples, flags):
        for q in fl:
            if q != 0:
                ent_rels.setdefault(int(ids[kk][q]), set()).add(int(r[kk]))
    out = []
    for phase in (0, 1):
        for kk, fl in zip(samples, flags):
            for q in fl:
                shared = q != 0 and len(ent_rels[int(ids[kk][q])]) > 1
                if shared == (phase == 1):
                    out.append((kk, q))
    return out


ORTH_REL_MIN = 64  # kernels_transh_parallel.hpp kOrthRelMin (normOrth iterations; a schedule choice only)


def transh_parallel_batches(ent, rel, W, triples, si, sj, side, B, nbatches, *, rate, margin=1.0, state=None,
                            orth_rel_min=ORTH_REL_MIN):
    """Train `nbatches` TransH batches of the PARALLEL schedule in place
    (kb2e_amd/csrc/kernels_transh_parallel.hpp).  Returns (loss, active).

    From the start-of-batch tables (transh/transh.cpp:10-29,
    transh/trainer.cpp:11-46): energies (always L1), x, sum_x; the h/t/r rows
    take the TransE summed sign counts and one norm; w gets the summed
    beta lr ((hs - ts) x + sum_x (h - t)) and one unit norm; then every
    (r', w'), (h', w'), (t', w') pair of an active update with w'.a > 0.1 (the
    relation row once per sample) runs the reference's normOrth
    (common/utils.cpp:79-111): first the pairs whose row only their relation
    touches (per relation, samples in order), then the entity rows flagged
    under several relations (samples in order).  The GPU runs the first pass as a
    wave per relation when the previous batch's normOrth work (loop iterations)
    was at least `orth_rel_min` and on its one wave otherwise, with the same
    result (the relations' own pairs touch disjoint rows and normals), so the
    gate does not enter the model; `state` records the flagged-sample counts for
    the tests.
    """
    from oracle import orc

    state = {} if state is None else state
    loss = 0.0
    active = 0
    h_all, t_all, r_all = triples[:, 0], triples[:, 1], triples[:, 2]
    for b in range(nbatches):
        sl = slice(b * B, (b + 1) * B)
        i, j, sd = si[sl], sj[sl], side[sl].astype(bool)
        h, t, r = h_all[i], t_all[i], r_all[i]
        nh = np.where(sd, h, j)
        nt = np.where(sd, j, t)
        w = W[r]
        R = rel[r]

        def proj_diff(hh, tt):
            hs = (w * ent[hh]).sum(1)
            ts = (w * ent[tt]).sum(1)
            d = ent[tt] - ts[:, None] * w - (ent[hh] - hs[:, None] * w) - R
            return hs, ts, d

        hsp, tsp, dp = proj_diff(h, t)
        hsn, tsn, dn = proj_diff(nh, nt)
        ep, en = np.abs(dp).sum(1), np.abs(dn).sum(1)
        act = ep + margin > en
        loss += float((margin + ep - en)[act].sum())
        active += int(act.sum())
        a = np.nonzero(act)[0]
        acc_e = np.zeros(ent.shape, np.int64)
        acc_r = np.zeros(rel.shape, np.int64)
        acc_w = np.zeros_like(W)
        for (hh, tt, d, hs, ts, m) in ((h, t, dp, hsp, tsp, -1), (nh, nt, dn, hsn, tsn, 1)):
            x = np.where(d[a] > 0, 1, -1).astype(np.int64)
            np.add.at(acc_r, r[a], -m * x)
            np.add.at(acc_e, hh[a], -m * x)
            np.add.at(acc_e, tt[a], m * x)
            sx = (x * w[a]).sum(1)
            dw = (m * rate) * ((hs[a] - ts[a])[:, None] * x + sx[:, None] * (ent[hh[a]] - ent[tt[a]]))
            np.add.at(acc_w, r[a], dw)
        er = np.unique(np.concatenate([h[a], t[a], nh[a], nt[a]]))
        rr = np.unique(r[a])
        ent[er] = ent[er] + rate * acc_e[er]
        rel[rr] = rel[rr] + rate * acc_r[rr]
        W[rr] = W[rr] + acc_w[rr]
        _norm_rows(ent, er)
        _norm_rows(rel, rr)
        _norm_rows(W, rr, ignore_short=False)
        flags = []
        for kk in a:
            rows = [(rel, r[kk]), (ent, h[kk]), (ent, t[kk]), None, (ent, nh[kk]), (ent, nt[kk])]
            flags.append([q for q in range(6) if rows[q] is not None and W[r[kk]] @ rows[q][0][rows[q][1]] > 0.1])
        ids = {kk: (r[kk], h[kk], t[kk], None, nh[kk], nt[kk]) for kk in a}
        # the two-pass order whichever kernel runs it: the gate on the previous batch's
        # normOrth work (orth_rel_min) picks the relation pass or the one-wave pass's
        # first sweep, which give the same result (kernels_transh_parallel.hpp
        # transh_orth_fix_kernel); not applied here
        order = transh_orth_order(list(a), flags, ids, r)
        state["orth_flagged"] = sum(1 for fl in flags if fl)
        if "flag_hist" in state:  # tests: the per-batch counts the gate saw
            state["flag_hist"].append(state["orth_flagged"])
        for kk, q in order:
            rows = [(rel, r[kk]), (ent, h[kk]), (ent, t[kk]), None, (ent, nh[kk]), (ent, nt[kk])]
            tab, row = rows[q]
            va, vb = orc.norm_orth(tab[row], W[r[kk]], rate)
            tab[row] = va
            W[r[kk]] = vb
    return loss, active
