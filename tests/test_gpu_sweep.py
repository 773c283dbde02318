"""Randomised parity sweep of the whole FindMatches (seeded, reproducible): genome counts
2-48, lengths, divergence, seed weights 9-21 (ranks 0-1), table sizes down to 1,
MemHash / MaskedMemHash with random presence masks, repeat tolerance, and the sliced
FindMatches forced at random slice sizes -- every MatchList, MemCount and collision
count equal to the oracle's."""
import random

import pytest

pytestmark = pytest.mark.gpu


def cases(n=120, seed=20261016):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        G = rng.choice([2, 2, 3, 4, 5, 8, 13, 33, 48])
        length = rng.choice([5_000, 20_000, 60_000, 150_000]) if G <= 8 else rng.choice([5_000, 15_000])
        p = rng.choice([0.001, 0.01, 0.03, 0.1, 0.3, 1.0])
        w = rng.choice([9, 11, 13, 15, 17, 19, 21])
        rank = rng.choice([0, 0, 1]) if w in (11, 13, 15) else 0
        table = rng.choice([None, None, 1, 7, 97, 1009])
        masked = rng.random() < 0.25
        mask = rng.getrandbits(G) | 1 if masked and rng.random() < 0.5 else ((1 << G) - 1 if masked else 0)
        rep = rng.choice([0, 0, 0, 1])
        chunk = rng.choice([None, None, 64, 1000, 20_000])
        out.append((i, G, length, p, w, rank, table, masked, mask, rep, chunk))
    return out


@pytest.mark.parametrize("i,G,n,p,w,rank,table,masked,mask,rep,chunk", cases(), ids=lambda v: str(v))
def test_findmatches_sweep(gpu_lib, oracle_mod, monkeypatch, i, G, n, p, w, rank, table, masked, mask, rep, chunk):
    seqs = oracle_mod.generate(G, n, p, 1000 + i)
    seed = oracle_mod.get_seed(w, rank)
    kw = dict(repeat_tol=rep)
    if table:
        kw["table_size"] = table
    if masked:
        kw.update(masked=True, seq_mask=mask)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, **kw)
    if chunk:
        monkeypatch.setenv("MUMS_DEV_FIND_CHUNK", str(chunk))
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        if masked:
            mh.SetMask(mask)
        if table:
            mh.SetTableSize(table)
        if rep:
            mh.SetRepeatTolerance(rep)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["mem_count"] == ost["mem_count"] and st["collision_count"] == ost["collision_count"]
