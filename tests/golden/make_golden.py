"""Regenerate the small MatchList text fixtures in tests/golden/ with the C oracle and
verify each against the reference md5 recorded in appendix_c.json.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

SMALL = {  # fixture name -> (G, n, w, p)
    "c1_related.txt": (2, 1000000, 15, 0.01),
    "c1_iid.txt": (2, 1000000, 15, 1.0),
    "g3_200k_p003.txt": (3, 200000, 15, 0.03),
}


def main():
    cases = json.load(open(os.path.join(HERE, "appendix_c.json")))["cases"]
    for name, (G, n, w, p) in SMALL.items():
        case = next(c for c in cases if (c["G"], c["n"], c["w"], c["p"]) == (G, n, w, p) and c["mode"] == "MemHash")
        seqs = oracle.generate(G, n, p, 12345)
        lengths, starts, _ = oracle.find_matches(seqs, oracle.get_seed(w))
        txt = oracle.match_text(lengths, starts)
        md5 = hashlib.md5(txt.encode()).hexdigest()
        assert md5 == case["md5"], (name, md5, case["md5"])
        with open(os.path.join(HERE, name), "w") as f:
            f.write(txt)
        print(name, len(lengths), md5)


if __name__ == "__main__":
    main()
