"""CPU checks of the oracle's SeedOccurrenceList restatement (SeedOccurrenceList.h:22-87)
against a pure-Python transcription of the same loops over the oracle's SML.  No
reference fixture covers SeedOccurrenceList: parity for this row is unpinned beyond the
shared SML construction (the oracle's SML is pinned through the Appendix C md5s)."""
import numpy as np
import pytest


def py_seed_occurrence(oracle, seq, seed):
    L = oracle.lib().oracle_seed_length(seed)
    n = len(seq)
    keys = oracle.seed_keys(seq, seed)
    sml = oracle.build_sml(seq, seed)
    m = len(sml)
    w = oracle.lib().oracle_seed_weight(seed)
    mask = ((1 << (2 * w)) - 1) << (64 - 2 * w)
    count = np.zeros(n, dtype=np.float32)
    seed_start, cur, seedI = 0, 1, 1
    for seedI in range(1, m):
        if (int(keys[sml[seedI]]) & mask) == (int(keys[sml[seedI - 1]]) & mask):
            cur += 1
            continue
        for i in range(seed_start, seedI):
            count[sml[i]] = cur
        seed_start, cur = seedI, 1
    else:
        seedI = max(m, 1)
    for i in range(seed_start, min(seedI, m)):
        count[sml[i]] = cur
    for i in range(seedI, n):
        count[i] = 1
    if n:
        s = float(L - 1) + float(count[0])
        buf = [np.float32(1.0)] * L
        buf[0] = count[0]
        for i in range(1, n):
            count[i - 1] = np.float32(s / L)
            s += float(count[i])
            s -= float(buf[i % L])
            buf[i % L] = count[i]
    count[count == 0] = 1
    return count


@pytest.mark.parametrize("n,p,w,gseed", [(3000, 1.0, 11, 1), (5000, 1.0, 7, 2), (20, 1.0, 15, 3), (5, 1.0, 15, 4),
                                        (1, 1.0, 15, 5), (4000, 1.0, 5, 6)])
def test_oracle_seed_occurrence_matches_transcription(oracle_mod, n, p, w, gseed):
    seq = oracle_mod.generate(1, n, p, gseed)[0]
    seed = oracle_mod.get_seed(w)
    a = oracle_mod.seed_occurrence(seq, seed)
    b = py_seed_occurrence(oracle_mod, seq, seed)
    assert a.dtype == np.float32 and len(a) == n
    assert (a.view(np.uint32) == b.view(np.uint32)).all()
    assert (a > 0).all()
