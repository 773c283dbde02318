"""Large-input known answers of the CPU oracle, recorded once in this container (the GPU
box checks the HIP path against them without re-running the oracle for minutes):

  c3: BASELINE config 3, 8 x 100 Mbp related (p = 0.01, genome 2 reverse-complemented,
      SURVEY.md Appendix C generator, seed 12345), default seed weight 19 (0x7b974ef),
      MemHash::FindMatches -> match count, md5 of the MatchList text, MemCount,
      collisions, AddHashEntry calls (probes), largest seed group, restarts.
  c5s: BASELINE config 5 scaled to 2 x 50 Mbp (w19), same record.
  pc_ngaps: ParallelMemHash (chunk 200 000) on BASELINE config 2's shape, 4 x 10 Mbp related,
      w15, with 20 N runs of 900-3200 bases per genome (tests/tie_inputs.multi_gap, seed
      4246): every chunk holding an N run meets the all-A seed group above MER_REPEAT_LIMIT
      and is cut there (ParallelMemHash.cpp:97) -> matches, md5, chunks, cut chunks.
  pc_c3shape: ParallelMemHash (chunk 200 000) at BASELINE config 3's shape scaled to
      8 x 10 Mbp (w19, G = 8), the one-thread schedule with a MergeTable after every chunk.

    python tests/golden/make_large_golden.py [c3] [c5s]   (c3: about 15 minutes, ~25 GB RAM)
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

CASES = {
    "c3": dict(G=8, n=100_000_000, p=0.01, gen_seed=12345, w=19),
    # BASELINE config 5 scaled to 2 x 50 Mbp: the GPU runs it in the chunked mode (forced)
    "c5s": dict(G=2, n=50_000_000, p=0.01, gen_seed=12345, w=19),
    "pc_ngaps": dict(G=4, n=10_000_000, p=0.01, gen_seed=4246, w=15, ngaps=20, chunk_size=200_000),
    # ParallelMemHash at BASELINE config 3's shape (G = 8, w19 0x7b974ef, related p = 0.01 with
    # genome 2 reverse-complemented) at 10 Mbp per genome: 50 chunks of the literal per-chunk
    # MergeTable restatement (ParallelMemHash.cpp:42-121)
    "pc_c3shape": dict(G=8, n=10_000_000, p=0.01, gen_seed=12345, w=19, chunk_size=200_000),
}
OUT = os.path.join(HERE, "large_cases.json")


def inputs(name):
    c = CASES[name]
    if "ngaps" in c:
        from tests import tie_inputs
        return tie_inputs.multi_gap(G=c["G"], n=c["n"], ngaps=c["ngaps"], gap=(900, 3200), p=c["p"], seed=c["gen_seed"])
    return oracle.generate(c["G"], c["n"], c["p"], c["gen_seed"])


def run(name):
    c = CASES[name]
    t0 = time.time()
    seqs = inputs(name)
    seed = oracle.get_seed(c["w"])
    kw = dict(parallel_compat=True, chunk_size=c["chunk_size"]) if "chunk_size" in c else {}
    lengths, starts, st = oracle.find_matches(seqs, seed, **kw)
    del seqs
    txt = oracle.match_text(lengths, starts)
    rec = dict(c, seed=seed, matches=int(len(lengths)), md5=hashlib.md5(txt.encode()).hexdigest(),
               mem_count=int(st["mem_count"]), collisions=int(st["collision_count"]), probes=int(st["probes"]),
               max_group=int(st["max_group"]), restarts=int(st["restarts"]), seedmers=int(st["seedmers"]),
               first_line=txt.split("\n", 1)[0], oracle_seconds=round(time.time() - t0, 1))
    if "chunk_size" in c:
        rec["chunks"] = int(st["chunks"])
    return rec


def main():
    names = sys.argv[1:] or list(CASES)
    have = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        rec = run(name)
        have[name] = rec
        print(name, json.dumps(rec))
        with open(OUT, "w") as f:
            json.dump(have, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
