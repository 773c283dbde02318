"""Ad-hoc GPU-vs-oracle parity sweep (development tool; the judged tests live in tests/)."""
import sys, time, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import libmems_amd
from oracle import oracle

CFGS = [(2, 100_000, 15, 0.01, 0, 0), (3, 200_000, 15, 0.03, 0, 0), (2, 1_000_000, 15, 0.01, 0, 0),
        (2, 1_000_000, 15, 1.0, 0, 0), (3, 1_000_000, 15, 0.05, 0, 0), (3, 1_000_000, 15, 0.01, 1, 7),
        (4, 300_000, 19, 0.01, 0, 0), (5, 200_000, 11, 0.02, 0, 0)]
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    CFGS = CFGS[:2]
bad = 0
for G, n, w, p, masked, mask in CFGS:
    seqs = oracle.generate(G, n, p, 12345)
    seed = oracle.get_seed(w)
    t0 = time.time(); rl, rs, rst = oracle.find_matches(seqs, seed, masked=bool(masked), seq_mask=mask); t1 = time.time()
    cls = libmems_amd.MaskedMemHash if masked else libmems_amd.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        if masked: mh.SetMask(mask)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    ok = len(ml) == len(rl) and (ml.lengths == rl).all() and (ml.starts == rs).all()
    ok2 = st["collision_count"] == rst["collision_count"] and st["mem_count"] == rst["mem_count"]
    print(f"G={G} n={n} w={w} p={p} masked={masked}: gpu {len(ml)} oracle {len(rl)} match={ok} counters={ok2} "
          f"(gpu coll {st['collision_count']} oracle {rst['collision_count']}) oracle {t1-t0:.2f}s gpu {st['ms_total']:.2f}ms "
          f"[keys {st['ms_keys']:.2f} sort {st['ms_sort']:.2f} groups {st['ms_groups']:.2f} buckets {st['ms_buckets']:.2f} replay {st['ms_replay']:.2f}]", flush=True)
    if not ok:
        bad += 1
        n_show = 0
        for i in range(min(len(ml), len(rl))):
            if ml.lengths[i] != rl[i] or (ml.starts[i] != rs[i]).any():
                print("  first diff at", i, "gpu", ml.lengths[i], ml.starts[i].tolist(), "oracle", rl[i], rs[i].tolist())
                n_show += 1
                if n_show > 4: break
sys.exit(1 if bad else 0)
