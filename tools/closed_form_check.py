"""Development check: the closed-form big-bucket path (bigq_*) runs and equals the oracle
(MUMS_DEV_BIG_BUCKET / MUMS_DEV_GRID_SLOW force it onto small buckets; stats on stderr)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MUMS_DEV_BIG_BUCKET", "8")
os.environ.setdefault("MUMS_DEV_GRID_SLOW", "0")
os.environ.setdefault("MUMS_DEV_REPLAY_STATS", "1")
import libmems_amd as lm  # noqa: E402
from oracle import oracle  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(float(sys.argv[2]) * 1e6) if len(sys.argv) > 2 else 10_000_000
w, p = 15, 0.01
seqs = oracle.generate(G, n, p, 12345)
seed = oracle.get_seed(w)
ln, st_, ref = oracle.find_matches(seqs, seed)
with lm.MemHash(0) as mh:
    mh.SetSeed(seed)
    ml = mh.FindMatches(seqs)
    st = mh.stats()
ok = len(ml) == len(ln) and (ml.lengths == ln).all() and (ml.starts == st_).all()
print(f"matches {len(ml)} vs {len(ln)}, collisions {st['collision_count']} vs {ref['collision_count']}, equal={ok}")
