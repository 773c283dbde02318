"""Rows A1-A5 on the CPU: seed-pattern table, 2-bit packing and canonical spaced-seed
keys of the oracle, checked against an independent pure-Python restatement of
SortedMerList.cpp (small inputs only)."""
import random

import numpy as np
import pytest

CODE = {c: 1 for c in "cCbByY"} | {c: 2 for c in "gGsSkK"} | {c: 3 for c in "tT"}


def py_pack(seq: bytes):
    """translate32 (SortedMerList.cpp:425-460): base i -> bits 31-2(i%16) of word i/16."""
    nw = (2 * len(seq)) // 32 + (1 if (2 * len(seq)) % 32 else 0) + 2
    w = [0] * nw
    for i, ch in enumerate(seq):
        w[i // 16] |= CODE.get(chr(ch), 0) << (30 - 2 * (i % 16))
    return w


def py_key(words, pos, seed):
    """GetMer (:321-342) + GetSeedMer (:726-762) + RevCompMer (:597-614) + GetDnaSeedMer (:764-769)."""
    L = seed.bit_length() - ((seed & -seed).bit_length() - 1)
    w = bin(seed).count("1")
    wi, bit = (pos * 2) // 32, (pos * 2) % 32
    mer = (words[wi] << 32) | words[wi + 1]
    if bit:
        mer = ((mer << bit) & (2**64 - 1)) | (words[wi + 2] >> (32 - bit))
    mer &= ((2**64 - 1) << (64 - 2 * L)) & (2**64 - 1)
    sm = 0
    for k in range(L):
        if seed & (1 << (L - 1 - k)):
            sm = (sm << 2) | ((mer >> (62 - 2 * k)) & 3)
    f = (sm << (64 - 2 * w)) & (2**64 - 1)
    rc = 0
    for k in range(w):  # complement of the w chars, reversed
        rc = (rc << 2) | (3 - ((sm >> (2 * k)) & 3))
    r = ((rc << (64 - 2 * w)) & (2**64 - 1)) | 1
    return min(f, r)


def test_seed_table_defaults(oracle_mod):
    assert oracle_mod.get_seed(15) == 0x7AC9AF
    assert oracle_mod.get_seed(19) == 0x7B974EF
    assert oracle_mod.get_seed(11) == 0x7954F          # table quirk: a weight-12 pattern
    L = oracle_mod.lib()
    for w in range(5, 32):
        s = oracle_mod.get_seed(w)
        sl, sw = L.oracle_seed_length(s), L.oracle_seed_weight(s)
        assert 1 <= sl <= 32
        if w != 11:
            assert sw == w
        # rank-0 patterns are palindromic for weights 5..31
        bits = format(s, f"0{sl}b")
        assert bits == bits[::-1]
    assert oracle_mod.get_seed(22) == (1 << 22) - 1       # solid seeds from weight 22
    assert oracle_mod.get_seed(40) == (1 << 32) - 1       # weight > 31 -> solid 32
    assert oracle_mod.get_seed(15, 2147483647) == (1 << 15) - 1   # SOLID_SEED


@pytest.mark.parametrize("n,expect", [(10**6, 15), (10**7, 17), (10**8, 19), (5 * 10**6, 15), (3 * 10**9, 21),
                                      (1000, 7), (10, 0), (0, 0)])
def test_default_seed_weight(oracle_mod, n, expect):
    assert oracle_mod.lib().oracle_default_seed_weight(n) == expect


def test_pack_matches_python(oracle_mod):
    rng = random.Random(7)
    seq = bytes(rng.choice(b"ACGTNacgtRYKMSWBDHVn") for _ in range(1001))
    assert oracle_mod.pack(seq).tolist() == py_pack(seq)
    with pytest.raises(ValueError):
        oracle_mod.pack(b"ACGT-ACGT")


@pytest.mark.parametrize("weight,rank", [(15, 0), (19, 0), (11, 0), (9, 1), (19, 2), (21, 1), (5, 0), (25, 0)])
def test_seed_keys_match_python(oracle_mod, weight, rank):
    rng = random.Random(weight * 31 + rank)
    seq = bytes(rng.choice(b"ACGTACGTNacgt") for _ in range(700))
    seed = oracle_mod.get_seed(weight, rank)
    keys = oracle_mod.seed_keys(seq, seed)
    words = py_pack(seq)
    assert len(keys) == len(seq) - (seed.bit_length() - ((seed & -seed).bit_length() - 1)) + 1
    for p in range(len(keys)):
        assert int(keys[p]) == py_key(words, p, seed), p


def test_sml_is_sorted_permutation(oracle_mod):
    seqs = oracle_mod.generate(1, 5000, 1.0, 99)
    seed = oracle_mod.get_seed(15)
    keys = oracle_mod.seed_keys(seqs[0], seed)
    sml = oracle_mod.build_sml(seqs[0], seed)
    assert sorted(sml.tolist()) == list(range(len(keys)))
    k = keys[sml]
    assert (np.diff(k.astype(np.float64)) >= 0).all() or all(int(k[i]) <= int(k[i + 1]) for i in range(len(k) - 1))


def test_short_and_empty_sequences(oracle_mod):
    seed = oracle_mod.get_seed(15)
    assert len(oracle_mod.seed_keys(b"ACGT", seed)) == 0          # SMLLength 0 when n < L
    l, s, st = oracle_mod.find_matches([b"ACGT" * 3, b""], seed)
    assert len(l) == 0 and st["seedmers"] == 0


@pytest.mark.parametrize("w", [16, 17, 19, 21, 24])
def test_top_digit_identity(w):
    """seeds.hip builds the keys pass's MSD histogram with ckey_top_static (seed_device.h):
    the top K = 2w+1-32 bits of the canonical key (min(v, rc) << 1 | parity) equal
    min(top_K(v), top_K(rc)), and top_K(rc) needs only v's low ceil(K/2) bases
    (complemented, base order reversed).  Checked on random and low-entropy seed values."""
    K = 2 * w + 1 - 32
    B = (K + 1) // 2
    rnd = random.Random(w)
    for i in range(20000):
        v = rnd.getrandbits(2 * w)
        if i % 5 == 0:   # long runs of one base / near-palindromes
            v = rnd.choice([0, (1 << 2 * w) - 1, int("01" * w, 2), int("10" * w, 2)]) ^ (rnd.getrandbits(4) << rnd.randrange(2 * w - 4))
        rc = 0
        for k in range(w):
            rc = (rc << 2) | (3 - ((v >> (2 * k)) & 3))
        par = 1 if rc < v else 0
        ckey = ((rc if par else v) << 1) | par
        want = ckey >> (2 * w + 1 - K)
        ft = v >> (2 * w - K)
        lowc = ~v & ((1 << 2 * B) - 1)
        rr = 0
        for k in range(B):   # base k of the low bases lands at base position k from the top
            rr = (rr << 2) | ((lowc >> (2 * k)) & 3)
        rt = rr >> (2 * B - K)
        assert want == min(ft, rt), (w, hex(v))
