"""Multi-GPU MemHash through the C ABI (mums_shard_run, shard_comm.hip): the whole sharded
pipeline (keys, count all-gather, key ranges, record all-to-allv, merge, bucket ranges, row
all-to-allv, packed all-gather, chains + replay) with ranks as threads of one process.
On the one-GPU test box the ranks share device 0: the host-staged in-process communicator
covers 1-4 ranks, RCCL (ncclCommInitAll) covers one rank.  Results = the oracle's
MemHash::FindMatches bit for bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(gpu_lib, oracle_mod, G, n, w, p, world, comm, table_size=40000, layout="blocks"):
    seqs = oracle_mod.generate(G, n, p, 500 + G * 11 + world)
    seed = oracle_mod.get_seed(w)
    lengths, starts, st = oracle_mod.find_matches(seqs, seed, table_size=table_size)
    with gpu_lib.ShardedMemHash([0] * world, comm=comm, table_size=table_size, layout=layout) as sh:
        sh.SetSeed(seed)
        ml = sh.FindMatches(seqs)
        coll = sum(s["collision_count"] for s in sh.stats_per_rank)
    assert len(ml) == len(lengths)
    assert np.array_equal(ml.lengths, lengths) and np.array_equal(ml.starts, starts)
    assert coll == st["collision_count"]


@pytest.mark.parametrize("world", [1, 2, 3, 4])
@pytest.mark.parametrize("G,n,w,p", [(4, 300_000, 15, 0.02), (5, 200_000, 13, 0.05), (3, 500_000, 17, 1.0)])
def test_shard_run_local_comm(gpu_lib, oracle_mod, world, G, n, w, p):
    run(gpu_lib, oracle_mod, G, n, w, p, world, "local")


def test_shard_run_local_comm_small_table(gpu_lib, oracle_mod):
    run(gpu_lib, oracle_mod, 4, 200_000, 15, 0.03, 3, "local", table_size=7)


def test_shard_run_more_ranks_than_genomes(gpu_lib, oracle_mod):
    run(gpu_lib, oracle_mod, 2, 300_000, 15, 0.02, 3, "local")


@pytest.mark.parametrize("G,n,w,p", [(4, 300_000, 15, 0.02), (8, 200_000, 19, 0.01)])
def test_shard_run_rccl_one_rank(gpu_lib, oracle_mod, G, n, w, p):
    run(gpu_lib, oracle_mod, G, n, w, p, 1, "rccl")


@pytest.mark.parametrize("G,n,w,p,world,table_size", [(2, 300_000, 19, 0.02, 2, 40000), (2, 250_000, 15, 0.03, 4, 40000),
                                                      (3, 200_000, 17, 0.02, 3, 7), (2, 100_003, 13, 0.05, 6, 40000)])
def test_shard_run_position_slices(gpu_lib, oracle_mod, G, n, w, p, world, table_size):
    """BASELINE config 5 layout through the ABI: every genome cut into world / G position
    slices; FindMatches all-gathers the packed slices into the whole genomes."""
    run(gpu_lib, oracle_mod, G, n, w, p, world, "local", table_size=table_size, layout="slices")


@pytest.mark.parametrize("world", [2, 3])
def test_shard_run_failure_is_collective(gpu_lib, oracle_mod, world, monkeypatch):
    """A rank whose local step fails (here: mums_shard_merge refusing a key chunk, forced
    small, that one MSD bucket overfills -- on the rank owning the repeat group's bucket only)
    must not leave the other ranks blocked in the next collective: every rank returns the
    same status."""
    from tests import repeat_inputs
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=False, seed=2)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", "3000")
    with gpu_lib.ShardedMemHash([0] * world, comm="local") as sh:
        sh.SetSeed(oracle_mod.get_seed(15))
        with pytest.raises(gpu_lib.MumsError):
            sh.FindMatches(seqs)
        assert sh.rank_status == [gpu_lib.MUMS_E_UNSUPPORTED] * world, sh.rank_status


@pytest.mark.parametrize("G,n,w,p,world,layout", [(2, 300_000, 21, 0.02, 2, "slices"), (2, 250_000, 21, 0.03, 4, "slices"),
                                                  (2, 200_000, 21, 0.02, 8, "slices"), (3, 200_000, 21, 0.02, 3, "blocks"),
                                                  (4, 150_000, 20, 0.02, 2, "blocks"), (2, 200_000, 20, 0.05, 4, "slices")])
def test_shard_run_ib33_wide_seeds(gpu_lib, oracle_mod, G, n, w, p, world, layout, monkeypatch):
    """Above 2^32 seed-mers (forced small: MUMS_DEV_SHARD_IB33) the records carry 33-bit indices
    and 31 key bits, so the default seed of 3 Gbp genomes (w21, getDefaultSeedWeight,
    SeedMasks.h:389-401) has 12 MSD bits: 8 scattered, 4 as side bytes split before the
    exchange (msdsplit.hip).  FindMatches over 2-8 ranks = the oracle's MatchList."""
    monkeypatch.setenv("MUMS_DEV_SHARD_IB33", "1")
    run(gpu_lib, oracle_mod, G, n, w, p, world, "local", layout=layout)


@pytest.mark.parametrize("G,n,w,p,world,layout,ib33", [(4, 200_000, 15, 0.03, 2, "blocks", False),
                                                       (5, 120_000, 17, 0.02, 3, "blocks", False),
                                                       (2, 200_000, 19, 0.02, 4, "slices", False),
                                                       (3, 150_000, 21, 0.02, 3, "slices", True),
                                                       (4, 100_000, 20, 0.03, 2, "blocks", True)])
def test_shard_run_pairwise(gpu_lib, oracle_mod, G, n, w, p, world, layout, ib33, monkeypatch):
    """PairwiseMatchFinder over ranks (PairwiseMatchFinder.cpp:37-73): every rank writes the pair
    rows of its key range's groups (mums_capi.hip shard_enum_rows), the owners replay them as for
    MemHash.  33-bit records forced small with MUMS_DEV_SHARD_IB33.  MatchList and collisions =
    the oracle's PairwiseMatchFinder."""
    if ib33:
        monkeypatch.setenv("MUMS_DEV_SHARD_IB33", "1")
    seqs = oracle_mod.generate(G, n, p, 700 + G * 13 + world)
    seed = oracle_mod.get_seed(w)
    lengths, starts, st = oracle_mod.find_matches(seqs, seed, pairwise=True)
    with gpu_lib.ShardedMemHash([0] * world, comm="local", layout=layout, pairwise=True) as sh:
        sh.SetSeed(seed)
        ml = sh.FindMatches(seqs)
        coll = sum(s["collision_count"] for s in sh.stats_per_rank)
    assert len(ml) == len(lengths)
    assert np.array_equal(ml.lengths, lengths) and np.array_equal(ml.starts, starts)
    assert coll == st["collision_count"]


def test_shard_run_pairwise_repeats(gpu_lib, oracle_mod):
    from tests import repeat_inputs
    seqs = repeat_inputs.high_copy(G=4, n=50_000, copies=30, tandem=False, seed=7)
    seed = oracle_mod.get_seed(15)
    lengths, starts, st = oracle_mod.find_matches(seqs, seed, pairwise=True)
    with gpu_lib.ShardedMemHash([0] * 3, comm="local", pairwise=True) as sh:
        sh.SetSeed(seed)
        ml = sh.FindMatches(seqs)
        coll = sum(s["collision_count"] for s in sh.stats_per_rank)
    assert np.array_equal(ml.lengths, lengths) and np.array_equal(ml.starts, starts)
    assert coll == st["collision_count"]


def test_shard_chains_labelled_where_the_probes_are(gpu_lib, oracle_mod):
    """BASELINE config-3 shape at 8 x 10 Mbp (related, w15) over 4 in-process ranks: every
    rank labels the chains of its own probes (mums_shard_chain_label), the bucket owners merge
    the entries and replay.  MatchList = the oracle's; the chain stage divides like the seed
    stage: the largest rank labels <= 1.5 x the mean probe count (by bucket owner one rank
    would label ~95 %: the related genomes' main diagonal is one hash bucket).  Only the probes
    the owners' replay needs travel (mums_shard_kept_export: chain-first and suspicious calls),
    so the owner of the main diagonal's bucket receives <= 10 % of all probes; the others are
    counted as collisions, and every owner still accounts for all AddHashEntry calls of its
    buckets."""
    G, n, w, p, world = 8, 10_000_000, 15, 0.01, 4
    seqs = oracle_mod.generate(G, n, p, 12345)
    seed = oracle_mod.get_seed(w)
    lengths, starts, st = oracle_mod.find_matches(seqs, seed, omp_threads=16)
    with gpu_lib.ShardedMemHash([0] * world, comm="local") as sh:
        sh.SetSeed(seed)
        ml = sh.FindMatches(seqs)
        coll = sum(s["collision_count"] for s in sh.stats_per_rank)
        info = sh.chain_info
        owned = [s["probes"] for s in sh.stats_per_rank]   # rows each bucket owner replayed
    assert len(ml) == len(lengths)
    assert np.array_equal(ml.lengths, lengths) and np.array_equal(ml.starts, starts)
    assert coll == st["collision_count"]
    lab = [i["probes"] for i in info]
    assert sum(lab) == sum(owned)
    mean = sum(lab) / world
    assert max(lab) <= 1.5 * mean, lab
    assert max(owned) > 1.5 * mean, owned   # (the bucket owners' AddHashEntry calls stay skewed ...)
    rows = [i["owned_rows"] for i in info]   # (... but not the rows they receive)
    assert max(rows) <= max(1.5 * sum(rows) / world, 0.10 * sum(lab)), (rows, sum(lab))
    xi = sh.exchange_info
    assert sum(x["recv_rows"] for x in xi) == sum(rows) == sum(x["sent_rows"] for x in xi)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_shard_kept_rows_equal_all_rows(gpu_lib, oracle_mod, monkeypatch, world):
    """The kept-probe export and the every-row export (MUMS_DEV_SHARD_ALL_ROWS) give the oracle's
    MatchList and collision count; the kept export sends fewer rows."""
    G, n, w, p = 5, 400_000, 15, 0.02
    seqs = oracle_mod.generate(G, n, p, 77 + world)
    seed = oracle_mod.get_seed(w)
    lengths, starts, st = oracle_mod.find_matches(seqs, seed)
    sent = {}
    for all_rows in (False, True):
        with monkeypatch.context() as m:
            if all_rows:
                m.setenv("MUMS_DEV_SHARD_ALL_ROWS", "1")
            with gpu_lib.ShardedMemHash([0] * world, comm="local", table_size=7 if world == 3 else 40000) as sh:
                sh.SetSeed(seed)
                ml = sh.FindMatches(seqs)
                coll = sum(s["collision_count"] for s in sh.stats_per_rank)
                sent[all_rows] = sum(x["sent_rows"] for x in sh.exchange_info)
        if world != 3:
            assert len(ml) == len(lengths), all_rows
            assert np.array_equal(ml.lengths, lengths) and np.array_equal(ml.starts, starts), all_rows
            assert coll == st["collision_count"], all_rows
        else:   # 7 hash buckets: the oracle with the same table size
            l7, s7, st7 = oracle_mod.find_matches(seqs, seed, table_size=7)
            assert np.array_equal(ml.lengths, l7) and np.array_equal(ml.starts, s7), all_rows
            assert coll == st7["collision_count"], all_rows
    assert sent[False] < sent[True], sent


@pytest.mark.parametrize("world", [2, 3])
def test_shard_bucket_owner_chains_switch(gpu_lib, oracle_mod, monkeypatch, world):
    """MUMS_DEV_SHARD_BUCKET_CHAINS: the previous layout (rows only, chains labelled by the
    bucket owner) still gives the oracle's MatchList."""
    monkeypatch.setenv("MUMS_DEV_SHARD_BUCKET_CHAINS", "1")
    run(gpu_lib, oracle_mod, 4, 300_000, 15, 0.02, world, "local")


@pytest.mark.parametrize("world", [2, 4])
def test_shard_chains_sliced_labels(gpu_lib, oracle_mod, monkeypatch, world):
    """Ranks with more probes than one labelling slice (MUMS_DEV_FIND_CHUNK, config 5 on 8
    ranks: 3e8 probes per rank > 2^28): the slices' entries merge on the rank, then again on
    the bucket owner."""
    monkeypatch.setenv("MUMS_DEV_FIND_CHUNK", "20000")
    run(gpu_lib, oracle_mod, 4, 300_000, 15, 0.02, world, "local")
