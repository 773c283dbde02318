"""Development: the sharded restart's two paths (the local plan and the gathered plan) on one
input, per rank: restart info, probe counts and the first differing probes."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libmems_amd as lm  # noqa: E402
from oracle import oracle  # noqa: E402
from tests import repeat_inputs  # noqa: E402


def run(seqs, world, mode):
    if mode == "gather":
        os.environ["MUMS_DEV_SHARD_RESTART"] = "gather"
    else:
        os.environ.pop("MUMS_DEV_SHARD_RESTART", None)
    with lm.ShardedMemHash([0] * world, comm="local") as sh:
        sh.SetSeed(oracle.get_seed(15))
        sh.FindMatches(seqs, stage=lm.STAGE_SEEDS)
        out = []
        for mh in sh.ranks:
            n = np.zeros(1, dtype=np.uint64)
            mh._check(mh._lib.mums_probe_count(mh._ctx, n.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_uint64))))
            P = int(n[0])
            b = np.zeros(P, dtype=np.uint32)
            r = np.zeros(P, dtype=np.uint64)
            mh._check(mh._lib.mums_probe_copy(mh._ctx, b.ctypes.data, r.ctypes.data, P))
            out.append((b, r))
        return out, sh.restart_info, sh.OffsetLog()


seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=False, seed=2)
a, ia, la = run(seqs, 2, "local")
b, ib, lb = run(seqs, 2, "gather")
print("info local", ia)
print("info gather", ib)
print("offset logs equal", np.array_equal(la, lb))
for r in range(2):
    print("rank", r, "probes", len(a[r][0]), len(b[r][0]))
    n = min(len(a[r][1]), len(b[r][1]))
    d = np.nonzero(a[r][1][:n] != b[r][1][:n])[0]
    if len(d):
        i = d[0]
        print("  first diff at", i, "local", a[r][1][i:i + 5], "gather", b[r][1][i:i + 5])
    sa, sb = set(a[r][1].tolist()), set(b[r][1].tolist())
    print("  only local", sorted(sa - sb)[:10], "only gather", sorted(sb - sa)[:10])


def find(seqs, world, mode):
    if mode == "gather":
        os.environ["MUMS_DEV_SHARD_RESTART"] = "gather"
    else:
        os.environ.pop("MUMS_DEV_SHARD_RESTART", None)
    with lm.ShardedMemHash([0] * world, comm="local") as sh:
        sh.SetSeed(oracle.get_seed(15))
        return sh.FindMatches(seqs)


ref_len, ref_starts, ref = oracle.find_matches(seqs, oracle.get_seed(15))
for mode in ("local", "gather"):
    ml = find(seqs, 2, mode)
    print(mode, "matches", len(ml), "oracle", len(ref_len))
with lm.MemHash(0) as mh:
    mh.SetSeed(oracle.get_seed(15))
    print("single context", len(mh.FindMatches(seqs)))
