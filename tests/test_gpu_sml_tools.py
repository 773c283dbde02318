"""GPU SeedOccurrenceList (SeedOccurrenceList.h:22-87), per-genome SortedMerList and the
MatchList filters (MatchList.h:636-664) against the oracle, bit for bit (float32 bits
for the frequencies)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(lm, seqs, seed, stage=None):
    mh = lm.MemHash(0)
    mh.SetSeed(seed)
    for s in seqs:
        mh.AddSequence(s)
    if stage is None:
        mh.CreateMatches()
    else:
        mh.FindStage(stage)
    return mh


@pytest.mark.parametrize("G,n,p,w,gseed", [(3, 200000, 0.02, 15, 1), (2, 50000, 1.0, 7, 2), (2, 300000, 0.01, 19, 3),
                                          (2, 100000, 1.0, 5, 4)])
def test_seed_occurrence_vs_oracle(gpu_lib, oracle_mod, G, n, p, w, gseed):
    seqs = oracle_mod.generate(G, n, p, gseed)
    seqs[1] = seqs[1][: n // 2] + seqs[0][:5000] * 3          # repeats -> frequencies > 1
    seed = oracle_mod.get_seed(w)
    with _run(gpu_lib, seqs, seed, gpu_lib.STAGE_SEEDS) as mh:
        for g, s in enumerate(seqs):
            ref = oracle_mod.seed_occurrence(s, seed)
            got = mh.SeedOccurrence(g, len(s))
            assert (got.view(np.uint32) == ref.view(np.uint32)).all()
            sml = mh.SortedMerList(g, max(len(s) - oracle_mod.lib().oracle_seed_length(seed) + 1, 0))
            assert (sml == oracle_mod.build_sml(s, seed)).all()


def test_seed_occurrence_short_and_tiny(gpu_lib, oracle_mod):
    seed = oracle_mod.get_seed(15)
    seqs = [b"ACGTACGTAC", b"A", b"ACGTTGCA" * 3 + b"ACG", oracle_mod.generate(1, 5000, 1.0, 9)[0]]
    with _run(gpu_lib, seqs, seed, gpu_lib.STAGE_SEEDS) as mh:
        for g, s in enumerate(seqs):
            ref = oracle_mod.seed_occurrence(s, seed)
            assert (mh.SeedOccurrence(g, len(s)).view(np.uint32) == ref.view(np.uint32)).all()


def test_match_filters(gpu_lib, oracle_mod):
    seqs = oracle_mod.generate(4, 300000, 0.03, 11)
    seed = oracle_mod.get_seed(15)
    lengths, starts, _ = oracle_mod.find_matches(seqs, seed)
    mult = (starts != 0).sum(axis=1)
    with _run(gpu_lib, seqs, seed) as mh:
        ml = mh.GetMatchList()
        assert (ml.lengths == lengths).all()
        mh.MultiplicityFilter(3)
        f = mh.GetMatchList()
        keep = mult == 3
        assert 0 < len(f) < len(ml)
        assert (f.lengths == lengths[keep]).all() and (f.starts == starts[keep]).all()
        mh.LengthFilter(40)
        f2 = mh.GetMatchList()
        keep2 = keep & (lengths >= 40)
        assert (f2.lengths == lengths[keep2]).all() and (f2.starts == starts[keep2]).all()
        mh.LengthFilter(10 ** 9)
        assert len(mh.GetMatchList()) == 0


def _parse_sml_file(path):
    """DNAFileSML v5 (SortedMerList.h:48-63 raw struct, 2352 B on x86-64; FileSML.cpp:336-345)."""
    import struct
    raw = open(path, "rb").read()
    (version, abits, seed, slen, sw, length, uniq, wsize, le, sid, circ) = struct.unpack_from("<IIQIIQIIBxhB", raw, 0)
    table = raw[45:300]
    desc = raw[300:2348].split(b"\0", 1)[0]
    nw = (2 * length) // 32 + (1 if (2 * length) % 32 else 0) + 2
    words = np.frombuffer(raw, dtype=np.uint32, count=nw, offset=2352)
    pos = np.frombuffer(raw, dtype=np.uint32, offset=2352 + 4 * nw)
    return dict(version=version, alphabet_bits=abits, seed=seed, seed_length=slen, seed_weight=sw, length=length,
                unique_mers=uniq, word_size=wsize, little_endian=le, id=sid, circular=circ, table=table,
                description=desc, words=words, positions=pos)


def test_dnafilesml_write_and_load(gpu_lib, oracle_mod, tmp_path):
    """DNAFileSML v5 files from the GPU SMLs: header as dmSML's InitSML writes it, the
    translate32 words, the SML positions; loading them back (FileSML::LoadFile) gives the
    same FindMatches result as the original sequences."""
    seqs = oracle_mod.generate(3, 120001, 0.02, 21)
    seed = oracle_mod.get_seed(15)
    L = oracle_mod.lib().oracle_seed_length(seed)
    paths = [str(tmp_path / f"g{g}.sml") for g in range(3)]
    with _run(gpu_lib, seqs, seed, gpu_lib.STAGE_SEEDS) as mh:
        for g in range(3):
            mh.WriteSML(g, paths[g], f"genome {g}")
    table = bytearray(255)
    for c in b"cCbByY":
        table[c] = 1
    for c in b"gGsSkK":
        table[c] = 2
    table[ord("t")] = table[ord("T")] = 3
    for g, s in enumerate(seqs):
        h = _parse_sml_file(paths[g])
        assert (h["version"], h["alphabet_bits"], h["seed"], h["seed_length"], h["length"]) == (5, 2, seed, L, len(s))
        assert (h["seed_weight"], h["unique_mers"], h["word_size"], h["little_endian"], h["id"], h["circular"]) == \
            (15, 0xFFFFFFFF, 32, 1, 0, 0)
        assert h["table"] == bytes(table) and h["description"] == f"genome {g}".encode()
        ref_words = oracle_mod.pack(s)
        full = (2 * len(s)) // 32
        assert (h["words"][:full] == ref_words[:full]).all()
        rem = (2 * len(s)) % 32
        if rem:
            mask = np.uint32(((1 << rem) - 1) << (32 - rem))
            assert (h["words"][full] & mask) == (ref_words[full] & mask)
        assert (h["positions"] == oracle_mod.build_sml(s, seed)).all()
    lengths, starts, _ = oracle_mod.find_matches(seqs, seed)
    with gpu_lib.MemHash(0) as mh2:
        for p in paths:
            assert mh2.AddSequenceFromSML(p) == seed
        mh2.SetSeed(seed)
        mh2.CreateMatches()
        ml = mh2.GetMatchList()
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
