"""Development probe: does RCCL accept two ranks on one GPU in one process
(ncclCommInitAll with devices [0, 0])?  Prints the outcome; never part of the tests."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libmems_amd as lm  # noqa: E402
from oracle import oracle  # noqa: E402

try:
    with lm.ShardedMemHash([0, 0], comm="rccl") as sh:
        seqs = oracle.generate(4, 200_000, 0.02, 5)
        sh.SetSeed(oracle.get_seed(15))
        ml = sh.FindMatches(seqs)
        ref = oracle.find_matches(seqs, oracle.get_seed(15))
        print("rccl [0,0]:", len(ml), "matches; oracle", len(ref[0]), "equal", bool((ml.starts == ref[1]).all()))
except Exception as e:  # noqa: BLE001
    print("rccl [0,0] refused:", e)
