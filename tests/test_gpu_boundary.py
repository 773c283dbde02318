"""Boundary members of MemHash beyond FindMatches, through the C ABI against the oracle:
MemTableCount (MemHash.h:100), PrintDistribution (MemHash.cpp:253-264), WriteFile
(MemHash.cpp:301-324), GetDnaSeedMer ranges."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def oracle_buckets(lengths, starts, T):
    """hash bucket of every stored entry: CalculateOffset (MatchHashEntry.cpp:141-160) with
    the entry's own length (invariant under ExtendMatch), MemHash.cpp:213."""
    out = np.zeros(len(lengths), dtype=np.int64)
    for i, (ln, row) in enumerate(zip(lengths.tolist(), starts.tolist())):
        ref = next(g for g, s in enumerate(row) if s != 0)
        off = 0
        for s in row[ref + 1:]:
            if s != 0:
                off += s - row[ref] - (ln if s < 0 else 0)
        out[i] = ((off % T) + T) % T
    return out


@pytest.mark.parametrize("T", [40000, 7, 1001])
def test_mem_table_count_and_distribution(gpu_lib, oracle_mod, T):
    seqs = oracle_mod.generate(3, 300_000, 0.02, 71)
    seed = oracle_mod.get_seed(15)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, table_size=T)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.SetTableSize(T)
        ml = mh.FindMatches(seqs)
        counts = mh.MemTableCount()
        dist = mh.PrintDistribution(ml)
        wf = mh.WriteFile(ml, names=["a.fa", "", "c.fa"], lengths=[len(s) for s in seqs])
        mc = mh.MemCount()
    b = oracle_buckets(lengths, starts, T)
    assert np.array_equal(counts, np.bincount(b, minlength=T).astype(np.uint32))
    assert np.all(np.diff(b) >= 0)   # bucket-major output
    lines = dist.splitlines()
    assert len(lines) == T
    bases = np.bincount(b, weights=lengths.astype(np.float64), minlength=T)
    for i in (0, int(b[0]), int(b[-1]), T - 1):
        k, c, s = lines[i].split("\t")
        assert int(k) == i and int(c) == counts[i] and int(s) == int(bases[i])
    head = wf.split("\n", 9)
    assert head[0] == "FormatVersion\t1" and head[1] == "SequenceCount\t3"
    assert head[2] == "Sequence0File\ta.fa" and head[4] == "Sequence1File\tnull"
    assert head[3] == "Sequence0Length\t300000" and head[8] == f"MatchCount\t{mc}"
    assert wf.endswith(oracle_mod.match_text(lengths, starts))


def test_seed_keys_range(gpu_lib, oracle_mod):
    seqs = oracle_mod.generate(2, 100_000, 0.02, 3)
    seed = oracle_mod.get_seed(19)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        m = 100_000 - 27 + 1
        full = mh.SeedKeys(1, m)
        for a, c in ((0, 10), (1, 17), (15, 1), (16, 5000), (12345, 777), (m - 33, 33), (m, 0)):
            assert np.array_equal(mh.SeedKeysRange(1, a, c), full[a:a + c])
        with pytest.raises(gpu_lib.MumsError):
            mh.SeedKeysRange(1, m - 3, 4)
