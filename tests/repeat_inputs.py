"""Repeat-rich synthetic genomes for the MER_REPEAT_LIMIT restart tests (test data only).

N-gapped assemblies: N encodes as A (SortedMerList.cpp:29-47), so a run of N gives
one all-A seed key per window -- a key group of thousands of records.  High-copy
inserts: every seed window of an inserted element occurs once per copy.
"""
from __future__ import annotations

import numpy as np

_ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for a, b in zip(b"ACGTN", b"TGCAN"):
    _COMP[a] = b


def _rand(rng, n):
    return _ACGT[rng.integers(0, 4, n)]


def _mutate(rng, s, p):
    s = s.copy()
    hit = rng.random(len(s)) < p
    s[hit] = _ACGT[rng.integers(0, 4, int(hit.sum()))]
    return s


def _relatives(rng, base, G, p):
    out = [base.copy()]
    for g in range(1, G):
        d = _mutate(rng, base, p)
        if g == 2:
            d = _COMP[d[::-1]]
        out.append(d)
    return out


def n_gapped(G=3, n=60_000, gaps=((20_000, 3000),), p=0.01, seed=7, shift=0):
    """Related genomes, each with N runs at (start + g * shift, length) (after relatives are made)."""
    rng = np.random.default_rng(seed)
    gs = _relatives(rng, _rand(rng, n), G, p)
    for g, s in enumerate(gs):
        for (a, ln) in gaps:
            a2 = min(max(0, a + g * shift), len(s) - ln)
            s[a2:a2 + ln] = ord("N")
    return [s.tobytes() for s in gs]


def high_copy(G=3, n=40_000, copies=2000, unit=120, copy_p=0.004, p=0.01, seed=11, tandem=False,
              only_genome=None):
    """A base genome with `copies` (slightly mutated) copies of one element inserted,
    then related genomes (p substitutions, genome 2 reverse-complemented).  only_genome:
    insert into that genome alone, after the relatives are made."""
    rng = np.random.default_rng(seed)
    elem = _rand(rng, unit)

    def insert(base):
        pieces = []
        cuts = np.sort(rng.integers(0, len(base), copies)) if not tandem else np.full(copies, len(base) // 2)
        prev = 0
        for c in cuts:
            pieces.append(base[prev:c])
            pieces.append(_mutate(rng, elem, copy_p))
            prev = c
        pieces.append(base[prev:])
        return np.concatenate(pieces)

    base = _rand(rng, n)
    if only_genome is None:
        gs = _relatives(rng, insert(base), G, p)
    else:
        gs = _relatives(rng, base, G, p)
        gs[only_genome] = insert(gs[only_genome])
    return [s.tobytes() for s in gs]


def mixed_repeats(seed):
    """Fuzz generator: 2-5 related genomes, each with its own number of copies (0, 1, 2 or
    100-1100) of one shared element and sometimes an N run -- key groups just above
    MER_REPEAT_LIMIT whose restart depends on the list order of the genomes' heads."""
    rng = np.random.default_rng(seed)
    G = int(rng.integers(2, 6))
    n = int(rng.integers(5000, 30000))
    unit = int(rng.integers(40, 150))
    elem = _rand(rng, unit)
    base = _rand(rng, n)
    gs = []
    for g in range(G):
        s = _mutate(rng, base, 0.01)
        k = int(rng.choice([0, 1, 2, int(rng.integers(100, 1100))]))
        pieces, prev = [], 0
        for c in np.sort(rng.integers(0, len(s), k)):
            pieces.append(s[prev:c])
            pieces.append(_mutate(rng, elem, float(rng.choice([0, 0.003]))))
            prev = c
        pieces.append(s[prev:])
        s = np.concatenate(pieces)
        if rng.random() < 0.3:
            a = int(rng.integers(0, len(s) - 1))
            ln = int(rng.integers(100, 3000))
            s[a:a + ln] = ord("N")
        gs.append(s.tobytes())
    return gs
