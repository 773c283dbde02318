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
