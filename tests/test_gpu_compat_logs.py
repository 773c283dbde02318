"""ParallelMemHash observability (SURVEY.md B.3 patched build, one OpenMP thread):
LogProgress -- every chunk's SearchRange text in chunk order, mers_processed set once for the
whole loop (ParallelMemHash.cpp:56-61, 86-101; MatchFinder.cpp:296-309) -- and SetMatchLog --
per chunk the thread-table inserts in AddHashEntry call order, then MergeTable's inserts
(ParallelMemHash.cpp:105-121; MemHash.cpp:238-241) -- against the oracle's literal restatement,
byte for byte / entry for entry, on plain chunked inputs and on chunks cut by MER_REPEAT_LIMIT."""
import numpy as np
import pytest

from tests import tie_inputs

pytestmark = pytest.mark.gpu

PLAIN = [(2, 200_000, 0.01, 15, 5000, 1), (3, 300_000, 0.03, 15, 3000, 2), (4, 200_000, 0.01, 15, 2000, 3),
         (3, 200_000, 1.0, 11, 1003, 6), (5, 300_000, 0.02, 17, 4000, 9), (2, 1_000_000, 0.01, 15, 200_000, 12345),
         (3, 150_000, 0.02, 13, 1_000_000, 5)]

CUT = sorted(n for n, (_, o) in tie_inputs.CASES.items() if o.get("cls") == "ParallelMemHash")


def run_gpu(lm, seqs, seed, chunk):
    with lm.ParallelMemHash(0, chunk) as mh:
        mh.SetSeed(seed)
        mh.LogProgress(True)
        mh.SetMatchLog(True)
        ml = mh.FindMatches(seqs)
        return ml, mh.ProgressLog(), mh.MatchLog(), mh.stats()


def check(lm, oracle_mod, seqs, w, chunk):
    seed = oracle_mod.get_seed(w)
    with oracle_mod.sml_tie_rule("std"):
        lengths, starts, ref = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    ml, text, log, st = run_gpu(lm, seqs, seed, chunk)
    assert st["chunks"] == ref["chunks"] and st["restarts"] == ref["restarts"]
    assert len(ml) == len(lengths) and (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert text == ref["progress"]
    ref_len, ref_s = ref["match_log"]
    assert len(log) == len(ref_len)
    assert np.array_equal(log.lengths, ref_len) and np.array_equal(log.starts, ref_s)
    return ref


@pytest.mark.parametrize("G,n,p,w,chunk,gseed", PLAIN)
def test_compat_progress_and_match_log(gpu_lib, oracle_mod, G, n, p, w, chunk, gseed):
    ref = check(gpu_lib, oracle_mod, oracle_mod.generate(G, n, p, gseed), w, chunk)
    assert ref["progress"]


@pytest.mark.parametrize("name", CUT)
def test_compat_logs_cut_chunks(gpu_lib, oracle_mod, name):
    gen, opts = tie_inputs.CASES[name]
    check(gpu_lib, oracle_mod, gen(), opts.get("w", 15), opts["chunk_size"])
