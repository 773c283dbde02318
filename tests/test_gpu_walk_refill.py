"""Chain walks with refilled lanes (chain_walk_refill_kernel, MUMS_DEV_WALK_REFILL=1) against the
one-shot short-walk kernel and the oracle.  Inputs span short walks (2 % substitutions), long
walks that overrun the per-lane budget and go on to the lane-group kernel (0.05 %), a
reverse-complemented genome and a non-palindromic seed (generic hit words).  The switch is read
per call, so both kernels run in one process on the same MemHash."""
import pytest

pytestmark = pytest.mark.gpu


def _revcomp(s: bytes) -> bytes:
    return s[::-1].translate(bytes.maketrans(b"ACGT", b"TGCA"))


CASES = [
    # (G, n, p, seed weight, reverse-complement genome 1, seed rank: 0 palindromic)
    (4, 200_000, 0.02, 15, False, 0),
    (3, 300_000, 0.0005, 15, False, 0),
    (5, 120_000, 0.005, 13, True, 0),
    (2, 250_000, 0.001, 11, True, 0),
    (3, 150_000, 0.002, 15, True, 1),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c[0]}_n{c[1]}_p{c[2]}_w{c[3]}{'_rc' if c[4] else ''}_r{c[5]}")
def test_walk_refill_matches_oracle(gpu_lib, oracle_mod, monkeypatch, case):
    G, n, p, w, rc, rank = case
    seqs = oracle_mod.generate(G, n, p, 700 + G)
    if rc:
        seqs[1] = _revcomp(seqs[1])
    seed = oracle_mod.get_seed(w, rank)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed)
    assert len(lengths) > 0
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        for var in ({}, {"MUMS_DEV_WALK_REFILL": "1"}, {"MUMS_DEV_WALK_REFILL": "1", "MUMS_DEV_FIND_CHUNK": "30000"},
                    {"MUMS_DEV_WALK_SORT": "1"}, {"MUMS_DEV_WALK_SORT": "2"},
                    {"MUMS_DEV_WALK_SORT": "2", "MUMS_DEV_FIND_CHUNK": "30000"}):
            with monkeypatch.context() as m:
                for k, v in var.items():
                    m.setenv(k, v)
                mh.CreateMatches()
                st = mh.stats()
                ml = mh.GetMatchList()
            assert len(ml) == len(lengths), var
            assert (ml.lengths == lengths).all() and (ml.starts == starts).all(), var
            assert st["collision_count"] == ost["collision_count"], var
