"""GPU chunked mode for more than 2^32 seed-mers per context (BASELINE config 5; chunked.hip):
33-bit record indices, MSD-digit chunks of < 2^30 records processed one after the other.
Forced on small inputs (MUMS_DEV_CHUNK_RECORDS caps the records per chunk, so 2-256 chunks
run) and checked bit for bit against the oracle; the 2 x 3 Gbp run itself is in bench_c5."""
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_chunks():
    def _set(cap, stream=False):
        os.environ["MUMS_DEV_CHUNK_RECORDS"] = str(cap)
        if stream:   # one scatter per chunk into a chunk-sized buffer (HBM-constrained layout)
            os.environ["MUMS_DEV_CHUNK_STREAM"] = "1"
    yield _set
    os.environ.pop("MUMS_DEV_CHUNK_RECORDS", None)
    os.environ.pop("MUMS_DEV_CHUNK_STREAM", None)


@pytest.mark.parametrize("G,n,p,w,cap,masked,stream", [(3, 300000, 0.02, 19, 100000, 0, 0),
                                                       (4, 200000, 0.03, 17, 120000, 0, 0),
                                                       (2, 1000000, 0.01, 19, 300000, 0, 0),
                                                       (5, 100000, 0.05, 18, 20000, 0, 0),
                                                       (3, 400000, 0.01, 16, 600000, 0, 0),
                                                       (3, 300000, 0.02, 19, 60000, 7, 0),
                                                       (3, 200000, 1.0, 17, 80000, 0, 0),
                                                       (3, 300000, 0.02, 19, 100000, 0, 1),
                                                       (4, 200000, 0.03, 17, 120000, 7, 1),
                                                       # w20-21 (msd_split of every chunk): 12 / 10 implicit bits
                                                       (3, 300000, 0.02, 21, 100000, 0, 0),
                                                       (2, 1000000, 0.01, 21, 300000, 0, 0),
                                                       (4, 200000, 0.03, 20, 120000, 7, 0),
                                                       (3, 200000, 1.0, 21, 50000, 0, 0)])
def test_chunked_vs_oracle(gpu_lib, oracle_mod, force_chunks, G, n, p, w, cap, masked, stream):
    seqs = oracle_mod.generate(G, n, p, 99 + G)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, masked=bool(masked), seq_mask=masked)
    force_chunks(cap, stream)
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        if masked:
            mh.SetMask(masked)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert st["chunks"] >= 2
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["probes"] == ost["probes"] and st["mem_count"] == ost["mem_count"]
    assert st["collision_count"] == ost["collision_count"]


def test_chunked_seed_stage_counts(gpu_lib, oracle_mod, force_chunks):
    """Seed stage only: the chunked probe count equals the unchunked one."""
    seqs = oracle_mod.generate(4, 500000, 0.01, 5)
    seed = oracle_mod.get_seed(19)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        ref = mh.stats()
        force_chunks(150000)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        got = mh.stats()
    assert got["chunks"] >= 8
    assert (got["probes"], got["groups"], got["seedmers"]) == (ref["probes"], ref["groups"], ref["seedmers"])


def test_chunked_w21_streaming_layout_refused(gpu_lib, oracle_mod, force_chunks):
    """w20-21 keep side bytes next to the resident records: the streaming layout refuses them."""
    seqs = oracle_mod.generate(2, 200000, 0.02, 5)
    force_chunks(100000, stream=True)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(21))
        with pytest.raises(gpu_lib.MumsError, match="resident"):
            mh.FindMatches(seqs)
