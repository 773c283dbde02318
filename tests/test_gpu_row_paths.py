"""The probe-row width fallbacks and the development switches, toggled per call inside one
process (they are read per call, not cached): int32 rows (materialize_dispatch) vs 64-bit rows,
the int32 rows flagged bad and rebuilt wide (the retry the genome-length guard makes
unreachable on real inputs), the line-order rows of the sliced path (gather_line_rows, retry
in chains.hip), the bucket sort's per-key atomics and the line sort without key runs.  Every
variant must give the oracle's MatchList and collision count."""
import pytest

pytestmark = pytest.mark.gpu

VARIANTS = [
    {},
    {"MUMS_DEV_WIDE_ROWS": "1"},
    {"MUMS_DEV_WIDE_ROWS": "retry"},
    {"MUMS_DEV_FIND_CHUNK": "40000"},
    {"MUMS_DEV_FIND_CHUNK": "40000", "MUMS_DEV_WIDE_LINE_ROWS": "1"},
    {"MUMS_DEV_FIND_CHUNK": "40000", "MUMS_DEV_WIDE_LINE_ROWS": "retry"},
    {"MUMS_DEV_RS_NOAGG": "1"},
    {"MUMS_DEV_LINE_NORUNS": "1"},
    {"MUMS_DEV_LINE_GATHER": "1"},
    {"MUMS_DEV_LINE_GATHER": "1", "MUMS_DEV_FIND_CHUNK": "40000"},
]


@pytest.mark.parametrize("masked", [0, 7])
def test_row_paths_one_process(gpu_lib, oracle_mod, monkeypatch, masked):
    seqs = oracle_mod.generate(3 if masked else 4, 150_000, 0.02, 901 + masked)
    seed = oracle_mod.get_seed(15)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, masked=bool(masked), seq_mask=masked)
    assert len(lengths) > 10
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        if masked:
            mh.SetMask(masked)
        for s in seqs:
            mh.AddSequence(s)
        for var in VARIANTS:
            with monkeypatch.context() as m:
                for k, v in var.items():
                    m.setenv(k, v)
                mh.CreateMatches()
                st = mh.stats()
                ml = mh.GetMatchList()
            assert len(ml) == len(lengths), var
            assert (ml.lengths == lengths).all() and (ml.starts == starts).all(), var
            assert st["collision_count"] == ost["collision_count"], var
            if "MUMS_DEV_FIND_CHUNK" in var:
                assert st["probes"] > 40000
