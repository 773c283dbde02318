"""The C++ host path (include/mums_memhash.hpp, the reference's host language) through the
C ABI on the GPU: tools/mums_find output must equal the reference's known answers."""
import hashlib
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
CASES = [c for c in json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["cases"] if not c.get("large")]


@pytest.fixture(scope="module")
def tool():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)
    return os.path.join(ROOT, "tools", "mums_find")


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_cpp_host_known_answers(tool, case):
    args = [tool, "gen", str(case["G"]), str(case["n"]), str(case["w"]), str(case["p"])]
    if case["mode"] == "MaskedMemHash":
        args.append(str(case["mask"]))
    out = subprocess.run(args, check=True, capture_output=True, timeout=300).stdout
    assert out.count(b"\n") == case["matches"]
    assert hashlib.md5(out).hexdigest() == case["md5"]


@pytest.mark.parametrize("ranks", ["--gpus 1", "--local 2", "--local 3", "--local 2 --slices", "--local 4 --slices"])
@pytest.mark.parametrize("case", [c for c in CASES if c["mode"] == "MemHash" and c["n"] <= 10_000_000],
                         ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}")
def test_cpp_sharded_known_answers(tool, case, ranks):
    """mums::ShardedMemHash (one thread per rank, mums_shard_run; --gpus: RCCL communicators
    from ncclCommInitAll, --local: ranks sharing device 0; --slices: position slices per
    rank, the BASELINE config 5 layout) = the reference's known answers."""
    if "--slices" in ranks and int(ranks.split()[1]) % case["G"]:
        pytest.skip("position slices need a rank count that is a multiple of G")
    args = [tool] + ranks.split() + ["gen", str(case["G"]), str(case["n"]), str(case["w"]), str(case["p"])]
    out = subprocess.run(args, check=True, capture_output=True, timeout=300).stdout
    assert out.count(b"\n") == case["matches"]
    assert hashlib.md5(out).hexdigest() == case["md5"]


@pytest.mark.parametrize("ranks", ["", "--gpus 1", "--local 2", "--local 4"])
def test_cpp_parallel_compat_known_answer(tool, ranks):
    """ParallelMemHash through the C++ host (mums_set_parallel_compat; sharded:
    ShardedMemHash::SetParallelCompat, the chunk-range ranks of DESIGN.md §6b) = the patched
    OpenMP reference's MatchList of SURVEY.md Appendix C (md5 of the text)."""
    case = json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["parallel_compat"][0]
    args = [tool] + ranks.split() + ["--compat", str(case["chunk_size"]), "gen", str(case["G"]), str(case["n"]),
                                     str(case["w"]), str(case["p"])]
    out = subprocess.run(args, check=True, capture_output=True, timeout=300).stdout
    assert out.count(b"\n") == case["matches"]
    assert hashlib.md5(out).hexdigest() == case["md5"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_cpp_deferred_sml_known_answers(tool, case):
    """The drop-in SML path (Aligner.cpp:1181-1184, CreateMemorySMLs MatchList.h:409-435):
    HipSML::Create per genome records the sequence and seed only, MemHash::FindMatches takes
    the genomes and the seed pattern from ml.sml_table -- the reference's known answers, and
    no SML was materialised (no key or sort work outside the one device pipeline)."""
    args = [tool, "sml", str(case["G"]), str(case["n"]), str(case["w"]), str(case["p"])]
    if case["mode"] == "MaskedMemHash":
        args.append(str(case["mask"]))
    r = subprocess.run(args, check=True, capture_output=True, timeout=300)
    assert r.stdout.count(b"\n") == case["matches"]
    assert hashlib.md5(r.stdout).hexdigest() == case["md5"]
    assert b"materialized 0" in r.stderr, r.stderr


@pytest.mark.parametrize("g,w", [(0, 15), (2, 15), (1, 11)])
def test_cpp_deferred_sml_readback(tool, oracle_mod, g, w):
    """A deferred SML read through operator[] equals the oracle's MemorySML::Create
    (positions in std::sort order, mer = GetDnaSeedMer at the position); FindMer returns
    SortedMerList::bsearch's index (restated below); Read past the end returns false."""
    import numpy as np
    G, n, p, stride = 3, 200_000, 0.02, 997
    out = subprocess.run([tool, "smldump", str(G), str(n), str(w), str(p), str(g), str(stride)], check=True,
                         capture_output=True, timeout=300)
    assert b"materialized 1" in out.stderr, out.stderr
    lines = out.stdout.decode().splitlines()
    seq = oracle_mod.generate(G, n, p, 12345)[g]
    seed = oracle_mod.get_seed(w)
    pos = oracle_mod.build_sml(seq, seed)
    keys = oracle_mod.seed_keys(seq, seed)
    m = len(pos)
    got = np.array([[int(x) for x in l.split("\t")] for l in lines[:m]], dtype=np.uint64)
    assert np.array_equal(got[:, 0], pos.astype(np.uint64))
    assert np.array_equal(got[:, 1], keys[pos])
    mers = keys[pos]

    def bsearch(q, start, end):   # SortedMerList.cpp:380-394
        while True:
            mid = (start + end) // 2
            if mers[mid] == q:
                return mid
            if mers[mid] < q and mid < end:
                start = mid + 1
            elif mers[mid] > q and start < mid:
                end = mid - 1
            else:
                return mid

    finds = [l.split("\t") for l in lines[m:] if l.startswith("find")]
    assert len(finds) == (m + stride - 1) // stride
    for _, i, f, r in finds:
        q = mers[int(i)]
        assert int(f) == 1 and int(r) == bsearch(q, 0, len(seq) - oracle_mod.lib().oracle_seed_length(seed))
    assert lines[-1] == "read\t0\t5"
