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
