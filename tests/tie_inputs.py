"""Inputs on which the order of equal seed mers in a SortedMerList can matter (test data only).

MemorySML::Create sorts {position, mer} with std::sort and bmer_lessthan (MemorySML.cpp:54,
SortedMerList.h:311-314): equal mers keep libstdc++ introsort's order, not position order.
That order is observable where a start point lands inside a run of equal full keys or where
the first copy of a repeated seed is chosen:
  * MER_REPEAT_LIMIT restarts: GetBreakpoint puts the other genomes' starts one past the
    FindMer hit (MatchFinder.cpp:113-121), inside the run of the break mer; the break mer is
    the key after a dropped group, e.g. "A...AC" at the right end of every N gap, so genomes
    with several gaps hold several equal full keys there;
  * ParallelMemHash chunk starts (ParallelMemHash.cpp:75-83, the same GetBreakpoint);
  * FindMatchesFromPosition start points (SML indices, MemHash.cpp:117-127);
  * repeat tolerance > 0 (the first copy per genome is hashed, MemHash.cpp:139-162) and
    enumeration tolerance > 1 (the odometer over the copies, MatchFinder.cpp:342-393).
CASES maps a name to (seqs, options); options are find_matches keyword arguments (w = seed
weight, cls = MemHash / MaskedMemHash / PairwiseMatchFinder / ParallelMemHash).
"""
from __future__ import annotations

import numpy as np

from tests import repeat_inputs

_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def multi_gap(G=3, n=120_000, ngaps=6, gap=(900, 3200), p=0.01, seed=1, rc=True):
    """Related genomes with several N runs each (own positions per genome): the key right
    after the all-A group ("A...AC" boundary seeds) occurs once per gap and genome."""
    rng = np.random.default_rng(seed)
    base = _ACGT[rng.integers(0, 4, n)]
    out = []
    for g in range(G):
        s = base.copy()
        hit = rng.random(n) < p
        s[hit] = _ACGT[rng.integers(0, 4, int(hit.sum()))]
        for a in np.sort(rng.integers(0, n - gap[1], ngaps)):
            ln = int(rng.integers(gap[0], gap[1]))
            s[a:a + ln] = ord("N")
        if rc and g == 2:
            comp = np.zeros(256, dtype=np.uint8)
            for x, y in zip(b"ACGTN", b"TGCAN"):
                comp[x] = y
            s = comp[s[::-1]]
        out.append(s.tobytes())
    return out


def tandem_blocks(G=3, n=60_000, unit=37, copies=300, blocks=4, p=0.01, seed=3):
    """Related genomes with several tandem arrays of one short unit (runs of equal full keys
    of every length up to `copies`) -- for repeat / enumeration tolerance and chunk starts."""
    rng = np.random.default_rng(seed)
    elem = _ACGT[rng.integers(0, 4, unit)]
    base = _ACGT[rng.integers(0, 4, n)]
    pieces, prev = [], 0
    for c in np.sort(rng.integers(0, n, blocks)):
        pieces.append(base[prev:c])
        pieces.append(np.tile(elem, int(rng.integers(copies // 2, copies))))
        prev = c
    pieces.append(base[prev:])
    b = np.concatenate(pieces)
    out = []
    for g in range(G):
        s = b.copy()
        hit = rng.random(len(s)) < p
        s[hit] = _ACGT[rng.integers(0, 4, int(hit.sum()))]
        out.append(s.tobytes())
    return out


def dup_block(G=3, n=40_000, frac=0.5, p=0.01, seed=5, tail=3000):
    """Related genomes where genome 1 carries a second, slightly mutated copy of a block of
    frac * n bases: those seed mers occur twice in genome 1 and once elsewhere, so a start
    point or chunk start inside such a run of two decides which copy a group keeps.
    Genome 0 gets a random tail so that it is the longest (ParallelMemHash chunks it)."""
    rng = np.random.default_rng(seed)
    base = _ACGT[rng.integers(0, 4, n)]
    out = []
    for g in range(G):
        s = base.copy()
        hit = rng.random(n) < p
        s[hit] = _ACGT[rng.integers(0, 4, int(hit.sum()))]
        if g == 1:
            a = int(rng.integers(0, n - int(frac * n)))
            blk = s[a:a + int(frac * n)].copy()
            hb = rng.random(len(blk)) < 0.002
            blk[hb] = _ACGT[rng.integers(0, 4, int(hb.sum()))]
            c = int(rng.integers(0, n))
            s = np.concatenate([s[:c], blk, s[c:]])
        if g == 0:
            s = np.concatenate([s, _ACGT[rng.integers(0, 4, int(frac * n) + tail)]])
        out.append(s.tobytes())
    return out


def _cases():
    c = {}
    for sd in range(6):
        c[f"multi_gap_{sd}"] = (lambda sd=sd: multi_gap(seed=sd), dict(w=15))
    c["multi_gap_G5"] = (lambda: multi_gap(G=5, n=80_000, ngaps=4, seed=11), dict(w=15))
    c["multi_gap_w19"] = (lambda: multi_gap(G=4, n=100_000, ngaps=5, seed=12), dict(w=19))
    c["multi_gap_w23"] = (lambda: multi_gap(G=3, n=100_000, ngaps=5, seed=13), dict(w=23))
    c["multi_gap_masked"] = (lambda: multi_gap(G=4, n=80_000, ngaps=5, seed=14), dict(w=15, cls="MaskedMemHash",
                                                                                       seq_mask=11))
    c["multi_gap_startpts"] = (lambda: multi_gap(G=3, n=90_000, ngaps=5, seed=15),
                               dict(w=15, start_points=[1200, 30_000, 7]))
    c["n_gapped_3000"] = (lambda: repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)),
                                                         shift=500, seed=1), dict(w=15))
    c["n_gapped_buffers"] = (lambda: repeat_inputs.n_gapped(G=4, n=90_000, gaps=((2_000, 25_000), (60_000, 10_022)),
                                                            shift=1_300, seed=13), dict(w=15))
    for t in (False, True):
        c[f"high_copy_{'tandem' if t else 'spread'}"] = (
            lambda t=t: repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=t, seed=2), dict(w=15))
    c["high_copy_rtol2"] = (lambda: repeat_inputs.high_copy(G=3, n=40_000, copies=1500, seed=17),
                            dict(w=15, repeat_tol=2))
    c["ngap_rtol1_etol2"] = (lambda: repeat_inputs.n_gapped(G=3, n=60_000, gaps=((20_000, 3000),), seed=23),
                             dict(w=15, repeat_tol=1, enum_tol=2))
    for sd in range(3):
        c[f"tandem_rtol1_{sd}"] = (lambda sd=sd: tandem_blocks(seed=20 + sd), dict(w=15, repeat_tol=1))
        c[f"tandem_rtol2_etol3_{sd}"] = (lambda sd=sd: tandem_blocks(seed=30 + sd, copies=120),
                                        dict(w=13, repeat_tol=2, enum_tol=3))
        c[f"tandem_compat_{sd}"] = (lambda sd=sd: tandem_blocks(G=3, n=50_000, copies=200, seed=40 + sd),
                                    dict(w=13, cls="ParallelMemHash", chunk_size=3000))
    # ParallelMemHash chunks holding a seed group above MER_REPEAT_LIMIT: the chunk's SearchRange
    # returns false at the group and ParallelMemHash.cpp:97 ignores it (the chunk is cut there)
    for sd, chunk in enumerate((20_000, 25_000, 40_000)):
        c[f"multi_gap_compat_{sd}"] = (lambda sd=sd: multi_gap(G=3, n=100_000, ngaps=5, seed=200 + sd),
                                       dict(w=15, cls="ParallelMemHash", chunk_size=chunk))
    c["multi_gap_compat_G5"] = (lambda: multi_gap(G=5, n=80_000, ngaps=4, seed=210),
                                dict(w=13, cls="ParallelMemHash", chunk_size=15_000))
    c["n_gapped_compat_buffers"] = (lambda: repeat_inputs.n_gapped(G=4, n=90_000, gaps=((2_000, 25_000), (60_000, 10_022)),
                                                                   shift=1_300, seed=13),
                                    dict(w=15, cls="ParallelMemHash", chunk_size=45_000))
    c["high_copy_compat"] = (lambda: repeat_inputs.high_copy(G=3, n=60_000, copies=2000, seed=2),
                             dict(w=15, cls="ParallelMemHash", chunk_size=5000))
    c["high_copy_tandem_compat"] = (lambda: repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=True, seed=2),
                                    dict(w=15, cls="ParallelMemHash", chunk_size=20_000))
    c["multi_gap_pairwise"] = (lambda: multi_gap(G=3, n=60_000, ngaps=4, seed=16), dict(w=15, cls="PairwiseMatchFinder"))
    for sd in range(4):
        rng = np.random.default_rng(100 + sd)
        sp = [int(rng.integers(0, 30_000)), int(rng.integers(0, 50_000)), int(rng.integers(0, 30_000))]
        c[f"dup_block_startpts_{sd}"] = (lambda sd=sd: dup_block(seed=50 + sd), dict(w=15, start_points=sp))
        for k in range(2):   # genome 1 only: its start point often splits a run of two copies
            sp1 = [0, int(rng.integers(1, 50_000)), 0]
            c[f"dup_block_startpt1_{sd}_{k}"] = (lambda sd=sd: dup_block(seed=80 + sd), dict(w=15, start_points=sp1))
        c[f"dup_block_compat_{sd}"] = (lambda sd=sd: dup_block(seed=60 + sd),
                                       dict(w=15, cls="ParallelMemHash", chunk_size=[2000, 3500, 5000, 7000][sd]))
    c["dup_block_rtol1"] = (lambda: dup_block(seed=70), dict(w=15, repeat_tol=1))
    c["dup_block_etol2"] = (lambda: dup_block(seed=71), dict(w=15, repeat_tol=1, enum_tol=2))
    c["dup_block_masked_rtol1"] = (lambda: dup_block(G=4, seed=72), dict(w=15, cls="MaskedMemHash", seq_mask=13,
                                                                         repeat_tol=1))
    for sd in list(range(0, 24)) + [26, 95, 98, 99, 106]:
        c[f"mixed_{sd}"] = (lambda sd=sd: repeat_inputs.mixed_repeats(sd), dict(w=15))
    return c


CASES = _cases()


def oracle_kwargs(opts):
    """find_matches keyword arguments of the oracle for a case's options."""
    cls = opts.get("cls", "MemHash")
    return dict(repeat_tol=opts.get("repeat_tol", 0), enum_tol=opts.get("enum_tol", 1),
                masked=cls == "MaskedMemHash", seq_mask=opts.get("seq_mask", 0),
                pairwise=cls == "PairwiseMatchFinder", parallel_compat=cls == "ParallelMemHash",
                chunk_size=opts.get("chunk_size", 0), start_points=opts.get("start_points"))
