"""GPU ParallelMemHash chunk-compat mode (compat.hip)
against the reference's known answer and the pinned oracle restatement, bit for bit."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

PCOMPAT = json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["parallel_compat"]


def gpu_parallel(lm, seqs, seed, chunk, masked=False, mask=0):
    with lm.ParallelMemHash(0, chunk) as mh:
        mh.SetSeed(seed)
        if masked:
            mh._check(mh._lib.mums_set_mask(mh._ctx, 1, mask))
        ml = mh.FindMatches(seqs)
        return ml, mh.stats()


@pytest.mark.parametrize("case", PCOMPAT, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}")
def test_parallel_known_answer(gpu_lib, oracle_mod, case):
    """4 x 10 Mbp related: the patched OpenMP reference's 15 893 matches, md5 of the text."""
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    ml, st = gpu_parallel(gpu_lib, seqs, oracle_mod.get_seed(case["w"]), case["chunk_size"])
    txt = ml.text()
    assert st["chunks"] == case["chunks"]
    assert len(ml) == case["matches"]
    assert hashlib.md5(txt.encode()).hexdigest() == case["md5"]
    assert st["mem_count"] == case["matches"]


COMPAT_SMALL = [(2, 200000, 0.01, 15, 5000, 1), (3, 300000, 0.03, 15, 3000, 2), (4, 200000, 0.01, 15, 2000, 3),
                (3, 500000, 0.05, 15, 7000, 4), (3, 200000, 1.0, 11, 1003, 6), (3, 200000, 0.01, 12, 999, 8),
                (2, 1000000, 0.01, 15, 200000, 12345), (5, 300000, 0.02, 17, 4000, 9)]


@pytest.mark.parametrize("G,n,p,w,chunk,gseed", COMPAT_SMALL)
def test_parallel_vs_oracle(gpu_lib, oracle_mod, G, n, p, w, chunk, gseed):
    seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    ml, st = gpu_parallel(gpu_lib, seqs, seed, chunk)
    assert st["chunks"] == ost["chunks"]
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()


def test_parallel_masked_and_ragged(gpu_lib, oracle_mod):
    """MaskedMemHash semantics inside the chunked search, genomes of different lengths
    (the longest SML defines the chunks, ParallelMemHash.cpp:64-73)."""
    seqs = oracle_mod.generate(3, 400000, 0.02, 77)
    seqs = [seqs[0], seqs[1][:250000], seqs[2][50000:]]
    seed = oracle_mod.get_seed(15)
    for masked, mask in ((False, 0), (True, 7), (True, 6)):
        lengths, starts, _ = oracle_mod.find_matches(seqs, seed, masked=masked, seq_mask=mask, parallel_compat=True,
                                                     chunk_size=3000)
        ml, _ = gpu_parallel(gpu_lib, seqs, seed, 3000, masked=masked, mask=mask)
        assert (ml.lengths == lengths).all() and (ml.starts == starts).all()


def test_parallel_single_chunk_equals_serial(gpu_lib, oracle_mod):
    """One chunk (every SML shorter than CHUNK_SIZE): ParallelMemHash = MemHash minus the
    duplicates MergeTable collapses."""
    seqs = oracle_mod.generate(3, 150000, 0.03, 5)
    seed = oracle_mod.get_seed(15)
    ml, st = gpu_parallel(gpu_lib, seqs, seed, 200000)
    lengths, starts, _ = oracle_mod.find_matches(seqs, seed)
    assert st["chunks"] == 1
    serial = oracle_mod.match_text(lengths, starts).splitlines()
    dedup = [l for i, l in enumerate(serial) if i == 0 or serial[i - 1] != l]
    assert ml.text().splitlines() == dedup


LARGE = json.load(open(os.path.join(GOLDEN, "large_cases.json")))


def test_parallel_ngaps_known_answer(gpu_lib, oracle_mod):
    """BASELINE config 2's shape (4 x 10 Mbp related, w15) with 20 N runs per genome under
    ParallelMemHash (chunk 200 000): the chunk holding the all-A seed group (> 1000 records)
    is cut there (SearchRange returns false, ParallelMemHash.cpp:97 ignores it) -- the
    oracle's recorded answer (tests/golden/make_large_golden.py pc_ngaps)."""
    from tests import tie_inputs
    c = LARGE["pc_ngaps"]
    seqs = tie_inputs.multi_gap(G=c["G"], n=c["n"], ngaps=c["ngaps"], gap=(900, 3200), p=c["p"], seed=c["gen_seed"])
    ml, st = gpu_parallel(gpu_lib, seqs, c["seed"], c["chunk_size"])
    assert st["chunks"] == c["chunks"] and st["restarts"] == c["restarts"]
    assert len(ml) == c["matches"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == c["md5"]


@pytest.mark.parametrize("copies,tandem,chunk,w", [(1500, False, 7000, 15), (2500, False, 20_000, 13),
                                                   (2000, True, 50_000, 15), (1200, False, 3000, 11)])
def test_parallel_repeat_limit_cuts_vs_oracle(gpu_lib, oracle_mod, copies, tandem, chunk, w):
    """High-copy repeats: seed groups above MER_REPEAT_LIMIT inside many chunks, each chunk cut
    at its first firing group (buffers of 10 000 from the chunk start, head order)."""
    from tests import repeat_inputs
    seqs = repeat_inputs.high_copy(G=4, n=300_000, copies=copies, tandem=tandem, seed=copies + chunk)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    assert ost["restarts"] > 0
    ml, st = gpu_parallel(gpu_lib, seqs, seed, chunk)
    assert st["chunks"] == ost["chunks"] and st["restarts"] == ost["restarts"]
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()


@pytest.mark.parametrize("case", ["known"] + [f"small{i}" for i in (0, 1, 4, 7)])
def test_parallel_merge_exact_pass_everywhere(gpu_lib, oracle_mod, monkeypatch, case):
    """MergeTable's two passes (compat.hip): the speculative append check, then the exact
    batched merge from a bucket's first entry that does not append.  The test hook runs every
    bucket through the exact pass from its first entry; both must give the oracle's list."""
    if case == "known":
        c = PCOMPAT[0]
        seqs = oracle_mod.generate(c["G"], c["n"], c["p"], 12345)
        w, chunk = c["w"], c["chunk_size"]
    else:
        G, n, p, w, chunk, gseed = COMPAT_SMALL[int(case[5:])]
        seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    if case != "known":
        lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    for exact in (False, True):
        with monkeypatch.context() as m:
            if exact:
                m.setenv("MUMS_DEV_COMPAT_MERGE_EXACT", "1")
            ml, st = gpu_parallel(gpu_lib, seqs, seed, chunk)
        if case == "known":   # the patched reference's 15 893 entries, md5 of the text
            assert len(ml) == c["matches"], exact
            assert hashlib.md5(ml.text().encode()).hexdigest() == c["md5"], exact
            continue
        assert len(ml) == len(lengths), exact
        assert (ml.lengths == lengths).all() and (ml.starts == starts).all(), exact


@pytest.mark.parametrize("idx", [0, 3, 4, 7])
def test_parallel_sml_builds_agree(gpu_lib, oracle_mod, monkeypatch, idx):
    """The compat SMLs from the MemHash path's packed onesweep stream (default for 2w+1 <= 39)
    and from the 64-bit (genome, ckey) radix sort (MUMS_DEV_COMPAT_RADIX, wider seeds) give
    the oracle's list, progress text and match log."""
    G, n, p, w, chunk, gseed = COMPAT_SMALL[idx]
    seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    for radix in (False, True):
        with monkeypatch.context() as m:
            if radix:
                m.setenv("MUMS_DEV_COMPAT_RADIX", "1")
            with gpu_lib.ParallelMemHash(0, chunk) as mh:
                mh.SetSeed(seed)
                mh.LogProgress(True)
                ml = mh.FindMatches(seqs)
                text = mh.ProgressLog()
                st = mh.stats()
        assert st["chunks"] == ost["chunks"], radix
        assert len(ml) == len(lengths) and (ml.lengths == lengths).all() and (ml.starts == starts).all(), radix
        assert text == ost["progress"], radix


@pytest.mark.parametrize("n,chunk", [(300_000, 150), (320_000, 140)])
def test_parallel_many_chunks(gpu_lib, oracle_mod, n, chunk):
    """2000 chunks (the chunk partition's LDS counters hold up to 2048) and 2286 (past them:
    the (chunk, ckey) radix sort) give the oracle's list."""
    seqs = oracle_mod.generate(3, n, 0.02, 41)
    seed = oracle_mod.get_seed(15)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    ml, st = gpu_parallel(gpu_lib, seqs, seed, chunk)
    assert st["chunks"] == ost["chunks"] > 1500
    assert len(ml) == len(lengths) and (ml.lengths == lengths).all() and (ml.starts == starts).all()


@pytest.mark.parametrize("env", [{"MUMS_DEV_COMPAT_PAIRS": "1"}, {"MUMS_DEV_COMPAT_GID_SCAN": "1"}])
def test_parallel_probe_views_agree(gpu_lib, oracle_mod, monkeypatch, env):
    """The chunk-major stream as packed records (default; group keys = the masked key's low
    bits, or numbered by a scan) and as (key2, index) pairs give the oracle's list."""
    for idx in (1, 4, 7):
        G, n, p, w, chunk, gseed = COMPAT_SMALL[idx]
        seqs = oracle_mod.generate(G, n, p, gseed)
        seed = oracle_mod.get_seed(w)
        lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            ml, st = gpu_parallel(gpu_lib, seqs, seed, chunk)
        assert len(ml) == len(lengths) and (ml.lengths == lengths).all() and (ml.starts == starts).all(), env


def test_parallel_c3shape_known_answer(gpu_lib, oracle_mod):
    """ParallelMemHash at BASELINE config 3's shape -- G = 8, the default w19 seed (0x7b974ef),
    related p = 0.01 with genome 2 reverse-complemented -- at 8 x 10 Mbp: the oracle's literal
    one-thread schedule (a MergeTable after each of the 50 chunks, ParallelMemHash.cpp:42-121)
    recorded in tests/golden/large_cases.json (make_large_golden.py pc_c3shape)."""
    c = LARGE["pc_c3shape"]
    seqs = oracle_mod.generate(c["G"], c["n"], c["p"], c["gen_seed"])
    assert oracle_mod.get_seed(c["w"]) == c["seed"]
    ml, st = gpu_parallel(gpu_lib, seqs, c["seed"], c["chunk_size"])
    assert st["chunks"] == c["chunks"]
    assert len(ml) == c["matches"] and st["mem_count"] == c["mem_count"]
    assert ml.text().split("\n", 1)[0] == c["first_line"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == c["md5"]


@pytest.mark.parametrize("idx", [0, 1, 2, 3, 4, 5, 7, "ragged", "many"])
def test_parallel_direct_records_agree(gpu_lib, oracle_mod, monkeypatch, capfd, idx):
    """The chunk-major records straight from the sorted stream (chunked.hip cd_*: every block
    boundary closed, single-chunk blocks in stream order, blocks holding a chunk start
    partitioned inside), with the chunk starts from the stream too (compat_fast_chunks) or from
    the genome-major SMLs (MUMS_DEV_COMPAT_SML), and the partition + compat_recs path
    (MUMS_DEV_COMPAT_PART) give the
    oracle's list, genomes of different lengths and 2000 chunks included; the direct form is
    taken on all of them but the one whose runs the tie replay reorders."""
    if idx == "ragged":
        seqs = oracle_mod.generate(3, 400000, 0.02, 77)
        seqs, w, chunk = [seqs[0], seqs[1][:250000], seqs[2][50000:]], 15, 3000
    elif idx == "many":
        seqs, w, chunk = oracle_mod.generate(3, 300_000, 0.02, 41), 15, 150
    else:
        G, n, p, w, chunk, gseed = COMPAT_SMALL[idx]
        seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    flags = []
    for env in (None, "MUMS_DEV_COMPAT_PART", "MUMS_DEV_COMPAT_SML"):
        with monkeypatch.context() as m:
            m.setenv("MUMS_DEV_COMPAT_DEBUG", "1")
            if env:
                m.setenv(env, "1")
            ml, st = gpu_parallel(gpu_lib, seqs, seed, chunk)
        err = capfd.readouterr().err.splitlines()
        flags.append([l for l in err if l.startswith("compat direct:")])
        if env is None:
            fast = [l for l in err if l.startswith("compat fast chunks:")]
            print(idx, fast)
        assert st["chunks"] == ost["chunks"], env
        assert len(ml) == len(lengths) and (ml.lengths == lengths).all() and (ml.starts == starts).all(), env
    assert flags[1] == []   # the partition path never tries the direct form
    if idx == 5:   # (w12 over 999-mer chunks: chunk starts inside equal-key runs, the tie replay
        return     # reorders them and the partition path runs)
    assert len(flags[0]) == 1 and flags[0][0].startswith("compat direct: flags 0,"), flags[0]
