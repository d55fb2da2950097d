"""Host restatement of the character-bag lower bound that k_bag_rows / k_compact_lev (spk_ctx.hip,
spk_gamma.hip) use to decide free-text Levenshtein cells before the exact pass: 60 buckets ('a'-'z', 'A'-'Z',
digits mod 8) in 4-bit saturating counts, the count of other units and the length (255: no bag), the bound
max(la, lb) - (Σ min over buckets + min(other_a, other_b)), skipped when a bucket saturates on both sides.
Property checked against the oracle's Levenshtein (the reference's levenshtein over code points): the bound
never exceeds the distance, so a cell it decides (bound > cut) really is past the cut."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as orc  # noqa: E402


def bag_row(s):
    if s is None:
        return None
    units = s.encode("utf-16-le")
    n16 = len(units) // 2
    if n16 > 128 or n16 != len(s):  # past 128 units, or a surrogate pair
        return None
    cnt = np.zeros(60, dtype=np.int64)
    other = 0
    for ch in s:
        u = ord(ch)
        if 97 <= u <= 122:
            b = u - 97
        elif 65 <= u <= 90:
            b = 26 + u - 65
        elif 48 <= u <= 57:
            b = 52 + ((u - 48) & 7)
        else:
            other += 1
            continue
        cnt[b] = min(cnt[b] + 1, 15)
    return cnt, other, n16


def bag_bound(a, b):
    ra, rb = bag_row(a), bag_row(b)
    if ra is None or rb is None:
        return None
    (ca, oa, la), (cb, ob, lb) = ra, rb
    if ((ca == 15) & (cb == 15)).any():
        return None
    inter = min(int(np.minimum(ca, cb).sum()) + min(oa, ob), min(la, lb))
    return max(la, lb) - inter


def _strings(rng, n):
    alpha = list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789 ,.-") + ["é", "ß", "ü", "\U0001F600"]
    out = []
    for _ in range(n):
        k = int(rng.integers(0, 90))
        out.append("".join(alpha[int(i)] for i in rng.integers(0, len(alpha), k)))
    return out


def test_bag_bound_never_exceeds_levenshtein():
    rng = np.random.Generator(np.random.PCG64(5))
    a_s, b_s = _strings(rng, 600), _strings(rng, 600)
    decided = 0
    for a, b in zip(a_s, b_s):
        bnd = bag_bound(a, b)
        if bnd is None:
            continue
        d = orc.levenshtein(a, b)
        assert bnd <= d, (a, b, bnd, d)
        cut = int(np.floor(0.4 * (len(a) + len(b)) / 2.0)) + 1
        decided += bnd > cut
    assert decided > 100  # unrelated random strings: most are decided


@pytest.mark.parametrize("a,b", [("", "abc"), ("aaaaaaaaaaaaaaaaaaaa", "aaaaaaaaaaaaaaaaaaab"), ("Ab1 ,", "bA1, "),
                                 ("x" * 128, "y" * 128), ("x" * 129, "y"), ("\U0001F600", "a"), ("99999999", "11111111")])
def test_bag_bound_edges(a, b):
    bnd = bag_bound(a, b)
    if bnd is not None:
        assert bnd <= orc.levenshtein(a, b)
    if len(a) > 128 or "\U0001F600" in a:
        assert bnd is None  # no bag: the exact pass decides
    if a.startswith("aaaa"):
        assert bnd is None  # 'a' saturated on both sides


# ---- bigram-count rows (k_bigram_rows, k_compact_lev<true>): short-string Levenshtein columns ----------------------
def bigram_bucket(c1, c2):
    """spk_ctx.hip bigram_bucket: 120 buckets of a hashed code-point pair."""
    x = ((c1 * 0x9E3779B1) ^ (c2 * 0x85EBCA77)) & 0xFFFFFFFF
    x = ((x ^ (x >> 15)) * 0x2C1B3C6D) & 0xFFFFFFFF
    return (x >> 16) % 120


def bigram_row(s):
    if s is None:
        return None
    n16 = len(s.encode("utf-16-le")) // 2
    if n16 > 254 or n16 != len(s):  # past 254 units, or a surrogate pair
        return None
    cnt = np.zeros(120, dtype=np.int64)
    for c1, c2 in zip(s, s[1:]):
        b = bigram_bucket(ord(c1), ord(c2))
        cnt[b] = min(cnt[b] + 1, 3)
    return cnt, n16


def bigram_decides(a, b, cut):
    """k_compact_lev<true>'s decision: the cell's distance is at least `cut` (q-gram lemma, q = 2)."""
    ra, rb = bigram_row(a), bigram_row(b)
    if ra is None or rb is None or cut < 1:
        return False
    (ca, la), (cb, lb) = ra, rb
    if ((ca == 3) & (cb == 3)).any():
        return False
    return int(np.minimum(ca, cb).sum()) < max(la, lb) - 1 - 2 * (cut - 1)


def _email_like(rng, n):
    """Short strings with a shared structure (name.name99@domain), the shape whose unrelated pairs the bigram bound
    decides, plus near-duplicates (a few edits) that it must never decide."""
    syl = ["ar", "bel", "cor", "dan", "el", "fin", "gor", "hal", "is", "jor", "kel", "lo", "mar", "nel", "or", "pet"]
    dom = ["@mail.com", "@inbox.org", "@uni.ac.uk", "@corp.example"]
    out = []
    for _ in range(n):
        w1 = "".join(syl[int(i)] for i in rng.integers(0, len(syl), int(rng.integers(1, 4))))
        w2 = "".join(syl[int(i)] for i in rng.integers(0, len(syl), int(rng.integers(1, 4))))
        out.append(f"{w1}.{w2}{int(rng.integers(0, 100)):02d}{dom[int(rng.integers(0, 4))]}")
    return out


def _edit(rng, s, k):
    s = list(s)
    for _ in range(k):
        op, i = int(rng.integers(3)), int(rng.integers(len(s) + 1))
        if op == 0:
            s.insert(i, chr(97 + int(rng.integers(26))))
        elif op == 1 and s:
            del s[min(i, len(s) - 1)]
        elif s:
            s[min(i, len(s) - 1)] = chr(97 + int(rng.integers(26)))
    return "".join(s)


def test_bigram_bound_never_decides_a_cell_within_the_cut():
    rng = np.random.Generator(np.random.PCG64(6))
    a_s = _email_like(rng, 1500)
    b_s = _email_like(rng, 1000) + [_edit(rng, a, int(rng.integers(0, 8))) for a in a_s[1000:]]
    decided = 0
    for t in (0.3, 0.2, 0.5):
        for a, b in zip(a_s, b_s):
            cut = int(np.floor(t * (len(a) + len(b)) / 2.0)) + 1
            if bigram_decides(a, b, cut):
                assert orc.levenshtein(a, b) >= cut, (a, b, cut)
                decided += 1
    assert decided > 500  # unrelated pairs at ratio 0.3 / 0.2: most are decided


@pytest.mark.parametrize("a,b,cut", [("", "abcdef", 2), ("ab", "ba", 1), ("abababababab", "babababababa", 2),
                                     ("x" * 60, "y" * 60, 5), ("\U0001F600abc", "abcd", 1), ("é" * 10, "e" * 10, 3),
                                     ("a" * 300, "b" * 300, 10)])
def test_bigram_bound_edges(a, b, cut):
    if bigram_decides(a, b, cut):
        assert orc.levenshtein(a, b) >= cut
    if "\U0001F600" in a or len(a) > 254:
        assert not bigram_decides(a, b, cut)  # no row: the exact pass decides
