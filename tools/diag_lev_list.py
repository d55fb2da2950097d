"""Diagnostic: which email cells does the filter hand to the Levenshtein exact pass at cfg2 size, and
which bound would have decided them (bag / length / bigram presence sets, emulated on the host)."""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as orc  # noqa: E402
from splink_amd.engine import Job  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

COLS = ["first_name", "surname", "dob", "city", "email"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
df = make_records(n, surname_vocab=15000, arrow=True)[["unique_id"] + COLS]
st = Params(cfg_settings(2), AmdSession(0)).settings
job = Job("dedupe_only", [df], "unique_id", 0)
job.block(st["blocking_rules"])
mode = int(os.environ.get("DIAG_MODE", "1"))
job.ctx.gammas_set_simple(mode)
job.gammas(st)
cnt = job.ctx.gammas_exact_counts(5)
print("exact counts", cnt, "pairs", job.n_pairs, flush=True)
lst = job.ctx.gammas_exact_list(4, cnt[4])
l, r = job.pair_rows()
em = job.tables[0]["email"].to_numpy(object)
rng = np.random.default_rng(0)
sample = lst[rng.choice(len(lst), min(20000, len(lst)), replace=False)]


def bucket(ch):
    u = ord(ch)
    if u < 128:
        if "a" <= ch <= "z":
            return u - 97
        if "A" <= ch <= "Z":
            return u - 65
        if "0" <= ch <= "9":
            return 26 + (u - 48) % 3
        return 29 + u % 3
    return (((u * 2654435761) & 0xFFFFFFFF) >> 16) & 31


def bag_lb(a, b):
    ca = collections.Counter(bucket(c) for c in a)
    cb = collections.Counter(bucket(c) for c in b)
    sa = {k: min(v, 3) for k, v in ca.items()}
    sb = {k: min(v, 3) for k, v in cb.items()}
    both = [k for k in sa if sa[k] == 3 and sb.get(k, 0) == 3]
    inter = sum(min(sa[k], sb.get(k, 0)) for k in sa if k not in both)
    ra = len(a) - sum(v for k, v in sa.items() if k not in both)
    rb = len(b) - sum(v for k, v in sb.items() if k not in both)
    if both:
        inter += min(ra, rb)
    return max(len(a), len(b)) - min(inter, min(len(a), len(b)))


def pres_lb(a, b):
    def S(s):
        return {((((ord(s[i]) << 16) | ord(s[i + 1])) * 0x9E3779B1) & 0xFFFFFFFF) >> 24 for i in range(len(s) - 1)}
    A, B = S(a), S(b)
    na, nb = len(a) - 1, len(b) - 1
    common = min(na - len(A - B), nb - len(B - A))
    return (max(na, nb) - common + 1) // 2


stats = collections.Counter()
ex = []
for p in sample:
    a, b = em[l[p]], em[r[p]]
    if a is None or b is None:
        stats["null"] += 1
        continue
    if a == b:
        stats["equal"] += 1
        continue
    th = 0.3 * (len(a) + len(b)) / 2
    lo = max(abs(len(a) - len(b)), bag_lb(a, b))
    hi = max(len(a), len(b))
    d = orc.levenshtein(a, b)
    stats["d<=th" if d <= th else "d>th"] += 1
    if lo > th:
        stats["bag_decides_F"] += 1
        if len(ex) < 8:
            ex.append((a, b, lo, th))
    elif hi <= th:
        stats["hi_decides_T"] += 1
    elif pres_lb(a, b) > th:
        stats["bigram_decides_F"] += 1
    else:
        stats["open"] += 1
print(dict(stats))
for e in ex:
    print(e)

# shape of the exact pass's work: pattern / text lengths after the common prefix / suffix strip,
# and the longest text of each wave of 64 consecutive list entries (what a wave's scan runs)
first = lst[: min(len(lst), 64 * 4000)]
ms, ns = [], []
for p in first:
    a, b = em[l[p]], em[r[p]]
    if a is None or b is None or a == b:
        ms.append(0)
        ns.append(0)
        continue
    pre = 0
    while pre < min(len(a), len(b)) and a[pre] == b[pre]:
        pre += 1
    suf = 0
    while suf < min(len(a), len(b)) - pre and a[-1 - suf] == b[-1 - suf]:
        suf += 1
    ra, rb = len(a) - pre - suf, len(b) - pre - suf
    ms.append(max(ra, rb))
    ns.append(min(ra, rb))
ms, ns = np.array(ms), np.array(ns)
wn = ns[: len(ns) // 64 * 64].reshape(-1, 64)
print("stripped pattern m: mean %.1f p50 %d p90 %d max %d; text n: mean %.1f p50 %d p90 %d" % (
    ms.mean(), np.median(ms), np.percentile(ms, 90), ms.max(), ns.mean(), np.median(ns), np.percentile(ns, 90)))
print("wave max n: mean %.1f; sum n / sum wave-max n = %.2f; m > 32: %.3f" % (
    wn.max(axis=1).mean(), wn.sum() / (wn.max(axis=1).sum() * 64), (ms > 32).mean()))
lens = np.array([len(em[l[p]]) for p in first if em[l[p]] is not None])
print("email length mean %.1f" % lens.mean())
