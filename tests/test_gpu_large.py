"""BASELINE configs 3 and 5 at full size on the GPU.

C3 (8 x 100 Mbp, w19): the whole FindMatches against the oracle's known answer recorded in
this container (tests/golden/large_cases.json, tests/golden/make_large_golden.py): match
count, md5 of the MatchList text, MemCount, collisions, AddHashEntry calls.
C5 (2 x 3 Gbp, w19, chunked mode, > 2^32 seed-mers): the seed stage at full size, checked
by size-independent properties (seed-mer count, probe / group counts invariant under 16 vs
32 key chunks and the streaming layout, sampled keys = oracle keys), and a scaled 2 x 50 Mbp
C5 FindMatches through the chunked mode against the oracle's recorded answer."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

_LARGE_PATH = os.path.join(GOLDEN, "large_cases.json")
LARGE = json.load(open(_LARGE_PATH)) if os.path.exists(_LARGE_PATH) else {}


def case(name):
    if name not in LARGE:
        pytest.skip(f"{name} known answer not recorded (tests/golden/make_large_golden.py)")
    return LARGE[name]


def md5_text(ml):
    return hashlib.md5(ml.text().encode()).hexdigest()


@pytest.mark.parametrize("variant", [None, ("MUMS_DEV_SORT3", "3"), ("MUMS_DEV_OS_XCD", "1")],
                         ids=["four_pass", "three_pass", "xcd_queues"])
def test_c3_findmatches_known_answer(gpu_lib, oracle_mod, monkeypatch, variant):
    """variant: the three 10-bit passes with the parity bit unsorted (radix_wide.hip), or the
    XCD-grouped claim queues of the four-pass sort."""
    import torch
    if variant:
        monkeypatch.setenv(*variant)
    c = case("c3")
    seqs = oracle_mod.generate(c["G"], c["n"], c["p"], c["gen_seed"])
    dev = [torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda() for s in seqs]
    del seqs
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(c["seed"])
        ml = mh.FindMatches(dev)
        st = mh.stats()
    assert st["seedmers"] == c["seedmers"]
    assert st["probes"] == c["probes"]
    assert len(ml) == c["matches"] and st["mem_count"] == c["mem_count"]
    assert st["collision_count"] == c["collisions"]
    assert st["restarts"] == c["restarts"]
    assert md5_text(ml) == c["md5"]


@pytest.mark.parametrize("find_chunk", [None, 5_000_000], ids=["one_pass", "sliced"])
def test_c5_scaled_findmatches_chunked(gpu_lib, oracle_mod, monkeypatch, find_chunk):
    """Chunked seed stage; FindMatches in one pass, then in 9 slices of 5e6 probes (the
    path the full 2 x 3 Gbp run takes with 2^28-probe slices)."""
    c = case("c5s")
    seqs = oracle_mod.generate(c["G"], c["n"], c["p"], c["gen_seed"])
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(16_000_000))   # 2 x 50 Mbp in >= 8 key chunks
    if find_chunk:
        monkeypatch.setenv("MUMS_DEV_FIND_CHUNK", str(find_chunk))
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(c["seed"])
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert st["chunks"] >= 8
    assert st["probes"] == c["probes"]
    assert len(ml) == c["matches"] and st["collision_count"] == c["collisions"]
    assert md5_text(ml) == c["md5"]


def synth_pair(n, p, seed, dev):
    import torch
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    step = 1 << 28
    for o in range(0, n, step):
        k = min(step, n - o)
        x = lut[torch.randint(0, 4, (k,), generator=gen, device=dev, dtype=torch.uint8).long()]
        a[o:o + k] = x
        mut = torch.rand(k, generator=gen, device=dev) < p
        sub = lut[torch.randint(0, 4, (k,), generator=gen, device=dev, dtype=torch.uint8).long()]
        b[o:o + k] = torch.where(mut, sub, x)
    torch.cuda.synchronize()
    return a, b


def test_c5_full_seed_stage(gpu_lib, oracle_mod):
    import torch
    n = 3_000_000_000
    dev = torch.device("cuda", 0)
    a, b = synth_pair(n, 0.01, 2024, dev)
    seed = oracle_mod.get_seed(19)
    L = 27
    m = n - L + 1
    counts = {}
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.AddSequence(a)
        mh.AddSequence(b)
        for cap in (None, 200_000_000):   # default chunks, then twice as many (or more)
            if cap:
                os.environ["MUMS_DEV_CHUNK_RECORDS"] = str(cap)
            try:
                mh.FindStage(gpu_lib.STAGE_SEEDS)
            finally:
                os.environ.pop("MUMS_DEV_CHUNK_RECORDS", None)
            st = mh.stats()
            counts[cap] = (st["chunks"], st["probes"], st["groups"], st["seedmers"])
        # sampled windows: GPU keys == oracle keys of the same bases
        rng = random.Random(5)
        for g, t in ((0, a), (1, b)):
            for _ in range(3):
                s0 = rng.randrange(0, m - 4000)
                ref = oracle_mod.seed_keys(bytes(t[s0:s0 + 4000 + L - 1].cpu().numpy()), seed)
                got = mh.SeedKeysRange(g, s0, 4000)
                assert np.array_equal(got, ref)
        # the last window of each genome
        for g, t in ((0, a), (1, b)):
            ref = oracle_mod.seed_keys(bytes(t[m - 100:].cpu().numpy()), seed)
            assert np.array_equal(mh.SeedKeysRange(g, m - 100, 100), ref)
    c0, c1 = counts[None], counts[200_000_000]
    assert c0[3] == c1[3] == 2 * m
    assert c1[0] > c0[0] >= 8
    assert c0[1:3] == c1[1:3]
    # related genomes (p = 0.01): a position is a shared unique seed when its 19 care bases
    # are unmutated, 0.99^19 = 0.83 of the positions
    assert c0[1] > 0.8 * m


def test_c5_full_findmatches(gpu_lib, oracle_mod):
    """BASELINE config 5 end to end on one GPU: 2 x 3 Gbp related (p = 0.01), w19, chunked
    seed stage (> 2^32 seed-mers) and FindMatches in 2^28-probe slices (2.5e9 AddHashEntry
    calls).  Size-independent checks: every call either inserted an entry or collided
    (probes = MemCount + collisions); the MatchList is unchanged with half-size slices;
    sampled matches begin and end with a seed hit (care positions equal in both genomes)."""
    import torch
    n = 3_000_000_000
    dev = torch.device("cuda", 0)
    a, b = synth_pair(n, 0.01, 2024, dev)
    seed = oracle_mod.get_seed(19)
    res = {}
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.AddSequence(a)
        mh.AddSequence(b)
        for chunk in (None, 1 << 27):
            if chunk:
                os.environ["MUMS_DEV_FIND_CHUNK"] = str(chunk)
            try:
                mh.CreateMatches()
            finally:
                os.environ.pop("MUMS_DEV_FIND_CHUNK", None)
            ml = mh.GetMatchList()
            res[chunk] = (ml, mh.stats())
    ml, st = res[None]
    ml2, st2 = res[1 << 27]
    assert st["seedmers"] == 2 * (n - 26)
    assert st["probes"] > (1 << 31)                   # beyond the former 2^30 limit
    assert st["probes"] == st["mem_count"] + st["collision_count"]
    assert len(ml) > 0 and np.array_equal(ml.lengths, ml2.lengths) and np.array_equal(ml.starts, ml2.starts)
    assert st["chains"] == st2["chains"]
    # sampled forward and reverse entries are maximal seed chains: hits at the
    # first and last column, none within L columns before the first or after the last
    L = 27
    care = [k for k in range(L) if (seed >> (L - 1 - k)) & 1]
    a_h, b_h = a.cpu().numpy(), b.cpu().numpy()
    fwd = np.nonzero((ml.starts > 0).all(axis=1))[0]
    rev = np.nonzero((ml.starts[:, 0] > 0) & (ml.starts[:, 1] < 0))[0]
    assert len(fwd) > 0 and len(rev) > 0
    rng = random.Random(9)
    picks = rng.sample(list(fwd), min(200, len(fwd))) + rng.sample(list(rev), min(100, len(rev)))
    for i in picks:
        s0, s1, ln = int(ml.starts[i, 0]), int(ml.starts[i, 1]), int(ml.lengths[i])
        assert is_maximal_chain((a_h, b_h), (s0, s1), ln, L, care), (i, s0, s1, ln)
    # the check itself rejects a truncated entry
    i = picks[0]
    s0, s1, ln = int(ml.starts[i, 0]), int(ml.starts[i, 1]), int(ml.lengths[i])
    assert not is_maximal_chain((a_h, b_h), (s0, s1 if s1 > 0 else s1 - 1), ln - 1, L, care)


_COMP = np.zeros(256, dtype=np.uint8)
for _x, _y in zip(b"ACGTacgt", b"TGCAtgca"):
    _COMP[_x] = _y


def column_chars(seq, s, ln, c0, c1, pad):
    """Characters of alignment columns c0..c1 of a component: start s > 0 reads
    base s - 1 + c, s < 0 the complement of base |s| - 1 + ln - 1 - c; outside -> pad."""
    cols = np.arange(c0, c1 + 1)
    pos = (s - 1 + cols) if s > 0 else (-s - 1 + ln - 1 - cols)
    ok = (pos >= 0) & (pos < len(seq))
    out = np.full(len(cols), pad, dtype=np.int16)
    v = seq[pos[ok]]
    out[ok] = v if s > 0 else _COMP[v]
    return out


def is_maximal_chain(seqs, starts, ln, L, care):
    """hit(0) and hit(ln - L), and no hit column in [-L, -1] or [ln - L + 1, ln] (a hit within
    L of the chain's ends would have extended it, MatchFinder.h:218-374)."""
    c0, c1 = -L, ln
    x = [column_chars(sq, st, ln, c0, c1 + L - 1, pad=-1 - g) for g, (sq, st) in enumerate(zip(seqs, starts))]

    def hit(c):
        return all(x[0][c - c0 + k] == x[1][c - c0 + k] for k in care)

    if not (hit(0) and hit(ln - L)):
        return False
    return not any(hit(c) for c in list(range(-L, 0)) + list(range(ln - L + 1, ln + 1)))
