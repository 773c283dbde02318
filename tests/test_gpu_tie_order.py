"""GPU parity of the SortedMerList tie order (MemorySML::Create's std::sort with bmer_lessthan,
MemorySML.cpp:54, SortedMerList.h:311-314): smlsort.hip replays libstdc++'s introsort for the
runs of equal seed mers that matter, and the HIP path must equal the oracle built in that
order (oracle/std_sort.h, pinned to the real std::sort by tests/test_sml_tie_order_cpu.py).

* every input of tests/tie_inputs.py (restarts at "A...AC" gap keys, start points inside
  runs of duplicated seeds, ParallelMemHash chunk starts, repeat / enumeration tolerance,
  PairwiseMatchFinder): MatchList, collisions, restarts and the offset log (the CPU test
  tests/test_sml_tie_order_cpu.py shows these inputs change under position order);
* mums_build_sml (the SML itself) on inputs with long runs of equal keys: poly-A, tandem
  repeats, N gaps, every weight."""
import numpy as np
import pytest

from tests import repeat_inputs, tie_inputs

pytestmark = pytest.mark.gpu


def run_case(lm, seqs, opts):
    cls = opts.get("cls", "MemHash")
    seed_w = opts.get("w", 15)
    if cls == "ParallelMemHash":
        mh = lm.ParallelMemHash(0, chunk_size=opts["chunk_size"])
    else:
        mh = getattr(lm, cls)(0)
    with mh:
        from oracle import oracle
        mh.SetSeed(oracle.get_seed(seed_w))
        mh.SetRepeatTolerance(opts.get("repeat_tol", 0))
        mh.SetEnumerationTolerance(opts.get("enum_tol", 1))
        if cls == "MaskedMemHash":
            mh.SetMask(opts.get("seq_mask", 0))
        if opts.get("start_points") is not None:
            ml = mh.FindMatchesFromPosition(seqs, opts["start_points"])
        else:
            ml = mh.FindMatches(seqs)
        return ml, mh.stats(), mh.OffsetLog()


@pytest.mark.parametrize("name", sorted(tie_inputs.CASES))
def test_tie_inputs_vs_std_sort_oracle(gpu_lib, oracle_mod, name):
    gen, opts = tie_inputs.CASES[name]
    seqs = gen()
    compat = opts.get("cls") == "ParallelMemHash"
    with oracle_mod.sml_tie_rule("std"):
        ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, oracle_mod.get_seed(opts.get("w", 15)),
                                                           **tie_inputs.oracle_kwargs(opts))
    ml, st, offlog = run_case(gpu_lib, seqs, opts)
    assert len(ml) == len(ref_len), (len(ml), len(ref_len))
    assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all()
    if compat:
        # a group above MER_REPEAT_LIMIT ends its ParallelMemHash chunk (SearchRange's ignored
        # return, ParallelMemHash.cpp:97): one cut chunk per oracle restart
        assert st["restarts"] == ref["restarts"]
        assert st["chunks"] == ref["chunks"]
    else:   # (the compat mode's collision count is not the thread tables' sum)
        assert st["collision_count"] == ref["collision_count"]
        assert st["restarts"] == ref["restarts"]
        assert np.array_equal(offlog, ref["offset_log"])


def _sml_inputs():
    rng = np.random.default_rng(7)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    unit = acgt[rng.integers(0, 4, 23)]
    tandem = np.concatenate([acgt[rng.integers(0, 4, 5000)], np.tile(unit, 900), acgt[rng.integers(0, 4, 7000)]])
    return {
        "polyA": [b"A" * 50_000],
        "polyAC": [b"AC" * 30_000],
        "tandem": [tandem.tobytes()],
        "n_gapped": repeat_inputs.n_gapped(G=2, n=60_000, gaps=((5_000, 4000), (30_000, 900)), seed=3),
        "dup_block": tie_inputs.dup_block(seed=5),
        "iid_small": [acgt[rng.integers(0, 4, 40_000)].tobytes()],
    }


@pytest.mark.parametrize("w", [5, 9, 15, 19, 23])
@pytest.mark.parametrize("name", sorted(_sml_inputs()))
def test_sorted_mer_list_std_sort_order(gpu_lib, oracle_mod, name, w):
    seqs = _sml_inputs()[name]
    seed = oracle_mod.get_seed(w)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        for g, s in enumerate(seqs):
            with oracle_mod.sml_tie_rule("std"):
                ref = oracle_mod.build_sml(s, seed)
            got = mh.SortedMerList(g, len(ref))
            assert np.array_equal(got, ref)

