"""LogProgress (MatchFinder.cpp:55-56, 137-164, 296-309) on CPU: the oracle's text, printed by its
literal SearchRange at every buffer refill, against the event model the GPU seed stage uses
(mums_capi.hip progress_log): every genome's 10 000-mer buffers exhausted at the masked key of
their last mer, events in key order, the genomes of one seed group in the merge's head order
(restart_plan.h head_order, restated below), the reference's percent / newline rule."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle


def head_order(masked, genomes, K, S):
    """The order the merge holds the heads of `genomes` when it reaches masked key K: partition
    refinement over the distinct keys below K down to the start points S (restart_plan.h:156-230)."""
    cls = [(frozenset(genomes), 0)]
    p, active = {}, set()
    for g in genomes:
        a = int(np.searchsorted(masked[g], K, "left"))
        if a > S[g]:
            p[g] = a - 1
            active.add(g)
    while any(len(c) > 1 and c & active for c, _ in cls):
        X = max(int(masked[g][p[g]]) for g in active)
        pres = {g for g in active if int(masked[g][p[g]]) == X}
        nc = []
        for c, cnt in cls:
            A, B = c & pres, c - pres
            if not A:
                nc.append((c, cnt))
            elif not B:
                nc.append((c, cnt + 1))
            elif (cnt + 1) & 1:
                nc += [(A, cnt + 1), (B, cnt)]
            else:
                nc += [(B, cnt), (A, cnt + 1)]
        cls = nc
        for g in pres:
            st = int(np.searchsorted(masked[g], X, "left"))
            if st > S[g]:
                p[g] = st - 1
            else:
                active.discard(g)
    return [g for c, cnt in cls for g in sorted(c, reverse=bool(cnt & 1))]


def model_text(seqs, seed, start_points=None) -> str:
    G = len(seqs)
    sp = list(start_points) if start_points is not None else [0] * G
    ev = []
    total = 0
    masked = []
    for g, s in enumerate(seqs):
        keys = oracle.seed_keys(s, seed)
        sml = oracle.build_sml(s, seed)
        masked.append(keys[sml] >> np.uint64(1) if len(sml) else keys)
        m = len(sml)
        total += len(s)   # Length() = sequence length (MatchFinder.cpp:146, SortedMerList.cpp:814)
        for a in range(sp[g], m, 10_000):
            e = min(a + 10_000, m)
            ev.append((int(masked[g][e - 1]), g, e - a))
    ev.sort(key=lambda x: (x[0], x[1]))
    i = 0
    while i < len(ev):
        j = i + 1
        while j < len(ev) and ev[j][0] == ev[i][0]:
            j += 1
        gs = {e[1] for e in ev[i:j]}
        if len(gs) > 1 and len({e[2] for e in ev[i:j]}) > 1:
            rank = {g: r for r, g in enumerate(head_order(masked, gs, ev[i][0], sp))}
            ev[i:j] = sorted(ev[i:j], key=lambda e: rank[e[1]])
        i = j
    out, processed, prog = [], sum(sp), -1.0
    for _, _, size in ev:
        processed += size
        old = prog
        prog = (processed / total) * 100.0
        if int(old) != int(prog):
            out.append(f"{int((prog / 100.0) * 100)}%..")
        if int(int(old) / 10) != int(int(prog) / 10):   # C++ integer division truncates
            out.append("\n")
    return "".join(out)


@pytest.mark.parametrize("G,n,p,w", [(3, 600_000, 0.01, 15), (2, 400_000, 1.0, 13), (4, 250_000, 0.02, 11),
                                     (2, 9_999, 0.01, 11), (5, 123_457, 0.05, 15)])
def test_progress_event_model_matches_oracle(G, n, p, w):
    seqs = oracle.generate(G, n, p, 40 + G)
    seed = oracle.get_seed(w)
    _, _, ref = oracle.find_matches(seqs, seed)
    assert ref["restarts"] == 0
    assert model_text(seqs, seed) == ref["progress"]


@pytest.mark.parametrize("sp", [[1000, 25_000, 7], [150_000, 0, 190_000], [9_990, 19_990, 29_990]])
def test_progress_event_model_with_start_points(sp):
    """unequal last buffers end in one seed group here: the head order decides the text"""
    seqs = oracle.generate(3, 200_000, 0.02, 777)
    seed = oracle.get_seed(15)
    _, _, ref = oracle.find_matches(seqs, seed, start_points=sp)
    assert model_text(seqs, seed, sp) == ref["progress"]


def test_progress_text_shape():
    seqs = oracle.generate(3, 2_000_000, 0.01, 5)
    _, _, ref = oracle.find_matches(seqs, oracle.get_seed(15))
    t = ref["progress"]
    vals = [int(x) for x in t.replace("\n", "").split("%..") if x]
    # total = sequence lengths (MatchFinder.cpp:146): a linear genome's last L-1 positions
    # hold no mer, so the text stops at 99%
    assert vals == sorted(vals) and vals[0] == 0 and vals[-1] == 99
    assert t.count("\n") == 9 and t.endswith("90%..\n" + "".join(f"{v}%.." for v in range(91, 100)))


def test_progress_total_is_sequence_length():
    """MatchFinder.cpp:146 sums SortedMerList::Length() = header.length = seq_len
    (SortedMerList.cpp:814), not SMLLength = n - L + 1: on linear sequences the
    processed / total ratio ends below 1, so the text never prints a final 100%."""
    seqs = oracle.generate(2, 30_000, 0.01, 7)
    seed = oracle.get_seed(15)
    _, _, ref = oracle.find_matches(seqs, seed)
    assert ref["restarts"] == 0
    assert "100%" not in ref["progress"] and "99%.." in ref["progress"]
    assert model_text(seqs, seed) == ref["progress"]
