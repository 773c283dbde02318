"""The onesweep sort's optional segment fix-up (MUMS_DEV_SEGFIX, radix_seg.hip): the lowest
key digit finished inside the segments of the higher digits instead of by a fourth pass,
with the parity bit left out under the default tolerances and restored before the
MER_REPEAT_LIMIT restart.  Every mode must give the same MatchList, MemCount and collision
count as the oracle: 1 = tile kernel + big-segment kernel, 2 = dirty segments forced
through the big-segment kernel as well."""
import pytest

from tests import repeat_inputs
from tests.test_gpu_restart import check as restart_check

pytestmark = pytest.mark.gpu

SHAPES = [
    # (G, n, p, w, repeat_tol, table)
    (4, 200_000, 0.01, 19, 0, None),
    (8, 100_000, 0.01, 19, 0, None),
    (3, 150_000, 0.05, 15, 0, None),
    (48, 20_000, 0.01, 11, 0, 97),     # short keys: long segments (the big list)
    (5, 60_000, 0.1, 17, 1, 7),        # repeat tolerance: exact order kept
    (2, 300_000, 1.0, 21, 0, None),
]


def _gpu(gpu_lib, seqs, seed, rep=0, table=None):
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        if table:
            mh.SetTableSize(table)
        if rep:
            mh.SetRepeatTolerance(rep)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    return ml, st


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("G,n,p,w,rep,table", SHAPES, ids=lambda v: str(v))
def test_segfix_matches_oracle(gpu_lib, oracle_mod, monkeypatch, mode, G, n, p, w, rep, table):
    seqs = oracle_mod.generate(G, n, p, 4242 + G + w)
    seed = oracle_mod.get_seed(w, 0)
    kw = dict(repeat_tol=rep)
    if table:
        kw["table_size"] = table
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, **kw)
    monkeypatch.setenv("MUMS_DEV_SEGFIX", mode)
    ml, st = _gpu(gpu_lib, seqs, seed, rep, table)
    assert st["sort_passes"] >= 1
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["mem_count"] == ost["mem_count"] and st["collision_count"] == ost["collision_count"]


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("kind", ["n_gapped", "high_copy"])
def test_segfix_restart_inputs(gpu_lib, oracle_mod, monkeypatch, mode, kind):
    """MER_REPEAT_LIMIT restart after a parity-masked sort: seg_parity_fix restores the
    exact SML order before the restart replays SearchRange (restarts, offset log, MatchList)."""
    if kind == "n_gapped":
        seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    else:
        seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, seed=2)
    monkeypatch.setenv("MUMS_DEV_SEGFIX", mode)
    restart_check(gpu_lib, oracle_mod, seqs)
