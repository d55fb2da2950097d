"""Seeded synthetic person records for the benchmark configs.

The reference's own demo dataset (`splink_demos` fake_1000, README.md:34) is not
available offline, so every config is generated here from numpy PCG64 with a
fixed seed.  Schema: unique_id, first_name, surname, dob, city, email
(+ address for config 5) and the ground-truth `cluster` id.

Duplicates: 20 % of entities get 1 + Geometric(0.5) extra copies.  Each copy
corrupts each field with p = 0.2 (one insert / delete / substitute /
transpose).  Every field of every record is nulled with p = 0.05.  About 1 %
of names carry a Latin-1 accent and 0.1 % a supplementary-plane character, so
the UTF-16 semantics of Jaro-Winkler are exercised.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

SEED = 20261015

_ONSETS = ["b", "br", "c", "ch", "d", "dr", "f", "g", "gr", "h", "j", "k", "l", "m",
           "n", "p", "r", "s", "sh", "st", "t", "th", "v", "w", "y", "z", "", ""]
_VOWELS = ["a", "e", "i", "o", "u", "ai", "ea", "ie", "ou", "y"]
_CODAS = ["", "", "n", "r", "s", "l", "m", "th", "ck", "ll", "nd", "rt", "x"]
_STREET_TYPES = ["Street", "Road", "Lane", "Avenue", "Close", "Drive", "Way", "Crescent"]
_DOMAINS = ["example.com", "mail.co.uk", "post.net", "inbox.org", "webmail.com",
            "fastmail.io", "letters.uk", "corp.example", "home.net", "uni.ac.uk"]
_BUILDINGS = ["House", "Court", "Mansions", "Lodge", "Tower", "Heights", "Place", "Gardens"]
_NOTES = ["leave parcels with the neighbour at number 12", "ring the bell twice and wait",
          "side entrance via the garden gate", "deliveries to the rear door after 6pm",
          "third floor, lift out of order", "use the intercom, code at reception",
          "opposite the old post office", "next to the primary school car park"]
_ACCENTS = "éèêëáàâäíìîïóòôöúùûüçñ"
_SUPPLEMENTARY = ["\U0001D400", "\U0001F600", "\U00020BB7", "\U0001D49C"]


def _word(rng: np.random.Generator, lo: int, hi: int) -> str:
    while True:
        n_syl = int(rng.integers(1, 4))
        w = "".join(_ONSETS[rng.integers(len(_ONSETS))] + _VOWELS[rng.integers(len(_VOWELS))]
                    + _CODAS[rng.integers(len(_CODAS))] for _ in range(n_syl))
        if lo <= len(w) <= hi:
            return w


def _vocab(rng: np.random.Generator, size: int, lo: int, hi: int) -> np.ndarray:
    out: dict = {}
    while len(out) < size:
        w = _word(rng, lo, hi)
        if w not in out:
            out[w] = None
    return np.array([w.capitalize() for w in out], dtype=object)


def _zipf_p(size: int, s: float) -> np.ndarray:
    p = 1.0 / np.arange(1, size + 1, dtype=np.float64) ** s
    return p / p.sum()


def _corrupt(rng: np.random.Generator, s: str) -> str:
    if not s:
        return s
    op = int(rng.integers(4))
    i = int(rng.integers(len(s)))
    letters = "abcdefghijklmnopqrstuvwxyz"
    c = letters[rng.integers(26)]
    if op == 0:
        return s[:i] + c + s[i:]
    if op == 1 and len(s) > 1:
        return s[:i] + s[i + 1:]
    if op == 3 and i + 1 < len(s):
        return s[:i] + s[i + 1] + s[i] + s[i + 2:]
    return s[:i] + c + s[i + 1:]


def _sprinkle(rng: np.random.Generator, s: str, alphabet) -> str:
    if not s:
        return s
    i = int(rng.integers(len(s)))
    return s[:i] + alphabet[rng.integers(len(alphabet))] + s[i + 1:]


def make_records(n: int, seed: int = SEED, surname_vocab: int = 15000, surname_s: float = 0.3,
                 first_vocab: int = 5000, city_vocab: int = 2000, with_address: bool = False,
                 arrow: bool = False) -> pd.DataFrame:
    """Return `n` synthetic person records as a pandas DataFrame (deterministic in `seed`).

    arrow=True gives Arrow-backed string columns (pd.ArrowDtype(large_string)), the columnar form a
    Spark / Arrow source hands over; the values are identical."""
    rng = np.random.Generator(np.random.PCG64(seed))
    vocabs = _vocabs(rng, surname_vocab, first_vocab, city_vocab)
    return _records(rng, n, vocabs, surname_s, with_address, arrow)


def _vocabs(rng: np.random.Generator, surname_vocab: int, first_vocab: int, city_vocab: int):
    firsts = _vocab(rng, first_vocab, 3, 12)
    surnames = _vocab(rng, surname_vocab, 3, 14)
    cities = _vocab(rng, city_vocab, 4, 12)
    streets = _vocab(rng, 500, 4, 10)
    return firsts, surnames, cities, streets


def _records(rng: np.random.Generator, n: int, vocabs, surname_s: float, with_address: bool,
             arrow: bool) -> pd.DataFrame:
    firsts, surnames, cities, streets = vocabs
    # entities -> cluster sizes
    n_ent = n
    dup = rng.random(n_ent) < 0.2
    sizes = np.ones(n_ent, dtype=np.int64)
    sizes[dup] += rng.geometric(0.5, size=int(dup.sum()))
    cum = np.cumsum(sizes)
    n_ent = int(np.searchsorted(cum, n) + 1)
    sizes = sizes[:n_ent]
    sizes[-1] -= int(cum[n_ent - 1] - n)
    cluster = np.repeat(np.arange(n_ent), sizes)
    copy_no = np.arange(n) - np.repeat(np.cumsum(sizes) - sizes, sizes)

    e_first = rng.choice(len(firsts), size=n_ent, p=_zipf_p(len(firsts), 1.1))
    e_sur = rng.choice(len(surnames), size=n_ent, p=_zipf_p(len(surnames), surname_s))
    e_city = rng.choice(len(cities), size=n_ent, p=_zipf_p(len(cities), 1.1))
    e_dob = rng.integers(0, 29220, size=n_ent)  # days since 1930-01-01, up to 2009-12-31
    e_num = rng.integers(1, 100, size=n_ent)
    e_dom = rng.integers(0, len(_DOMAINS), size=n_ent)

    first = firsts[e_first[cluster]].copy()
    sur = surnames[e_sur[cluster]].copy()
    city = cities[e_city[cluster]].copy()
    dob_days = e_dob[cluster]
    base = np.datetime64("1930-01-01")
    dob = np.datetime_as_string(base + dob_days.astype("timedelta64[D]"), unit="D").astype(object)
    email = np.array([f"{f.lower()}.{s.lower()}{k:02d}@{_DOMAINS[d]}" for f, s, k, d in
                      zip(first, sur, e_num[cluster], e_dom[cluster])], dtype=object)
    cols = {"first_name": first, "surname": sur, "dob": dob, "city": city, "email": email}
    if with_address:
        # free-text addresses of 30-128 characters (cfg5): flat / building, house and street, an
        # optional district, city, postcode and an optional delivery note, per entity
        e_house = rng.integers(1, 400, size=n_ent)
        e_street = rng.integers(0, len(streets), size=n_ent)
        e_type = rng.integers(0, len(_STREET_TYPES), size=n_ent)
        e_flat = rng.integers(0, 60, size=n_ent)
        e_bldg = rng.integers(0, len(streets), size=n_ent)
        e_dist = rng.integers(0, len(cities), size=n_ent)
        e_note = rng.integers(0, 2 * len(_NOTES), size=n_ent)
        e_parts = rng.random((n_ent, 3))
        addr = []
        for i in range(n):
            e = cluster[i]
            head = ""
            if e_flat[e] < 20:
                head = f"Flat {e_flat[e]}, "
                if e_parts[e, 0] < 0.5:
                    head += f"{streets[e_bldg[e]]} {_BUILDINGS[e_bldg[e] % len(_BUILDINGS)]}, "
            dist = f"{cities[e_dist[e]]} District, " if e_parts[e, 1] < 0.5 else ""
            a = (f"{head}{e_house[e]} {streets[e_street[e]]} {_STREET_TYPES[e_type[e]]}, {dist}"
                 f"{cities[e_city[e]]}, AB{e % 90 + 10} {e % 9}XY")
            if e_note[e] < len(_NOTES) and e_parts[e, 2] < 0.7:
                a += f" ({_NOTES[e_note[e]]})"
            addr.append(a[:127])  # <= 128 characters after the one-edit corruption below
        cols["address"] = np.array(addr, dtype=object)

    # non-ASCII sprinkles on names
    for name in ("first_name", "surname"):
        arr = cols[name]
        acc = np.nonzero(rng.random(n) < 0.01)[0]
        for i in acc:
            arr[i] = _sprinkle(rng, arr[i], _ACCENTS)
        sup = np.nonzero(rng.random(n) < 0.001)[0]
        for i in sup:
            arr[i] = _sprinkle(rng, arr[i], _SUPPLEMENTARY)

    # typo corruption on duplicate copies, then nulls everywhere
    is_copy = copy_no > 0
    for name, arr in cols.items():
        hit = np.nonzero(is_copy & (rng.random(n) < 0.2))[0]
        for i in hit:
            arr[i] = _corrupt(rng, arr[i])
        nulls = rng.random(n) < 0.05
        arr[nulls] = None

    perm = rng.permutation(n)
    df = pd.DataFrame({"unique_id": np.arange(n, dtype=np.int64)})
    for name, arr in cols.items():
        df[name] = arr[perm]
    df["cluster"] = cluster[perm]
    if arrow:
        import pyarrow as pa
        for name in cols:
            df[name] = pd.Series(pa.array(df[name].tolist(), type=pa.large_string()),
                                 dtype=pd.ArrowDtype(pa.large_string()))
    return df


_FORK_VOCABS = None  # the parent's vocabularies, inherited by forked workers


def _chunk(args):
    seed, i, n_i, vocab_args, surname_s, with_address = args
    vocabs = _FORK_VOCABS if _FORK_VOCABS is not None else \
        _vocabs(np.random.Generator(np.random.PCG64(seed)), *vocab_args)
    df = _records(np.random.Generator(np.random.PCG64([seed, i + 1])), n_i, vocabs, surname_s, with_address, True)
    return {c: (df[c].array._pa_array.combine_chunks() if c not in ("unique_id", "cluster") else df[c].to_numpy())
            for c in df.columns}


def make_records_parallel(n: int, chunks: int, workers: int, seed: int = SEED, surname_vocab: int = 15000,
                          surname_s: float = 0.3, first_vocab: int = 5000, city_vocab: int = 2000,
                          with_address: bool = False) -> pd.DataFrame:
    """`n` records generated as `chunks` independent populations over ONE shared vocabulary (the same
    name / city / street lists as make_records(seed)), each from its own PCG64 stream [seed, i + 1], in
    `workers` processes; Arrow-backed string columns.  For the 100M-record rows, where the serial
    generator would take ~7 minutes.  Deterministic in (n, chunks, seed), but not equal to
    make_records(n): duplicates stay inside a chunk, unique_id and cluster are offset per chunk."""
    import multiprocessing as mp

    import pyarrow as pa
    sizes = [n // chunks + (1 if i < n % chunks else 0) for i in range(chunks)]
    jobs = [(seed, i, sizes[i], (surname_vocab, first_vocab, city_vocab), surname_s, with_address)
            for i in range(chunks)]
    global _FORK_VOCABS
    _FORK_VOCABS = _vocabs(np.random.Generator(np.random.PCG64(seed)), surname_vocab, first_vocab, city_vocab)
    try:
        with mp.get_context("fork").Pool(workers) as pool:
            parts = pool.map(_chunk, jobs, chunksize=1)
    finally:
        _FORK_VOCABS = None
    df = pd.DataFrame({"unique_id": np.arange(n, dtype=np.int64)})
    for c in parts[0]:
        if c == "unique_id":
            continue
        if c == "cluster":
            off = np.cumsum([0] + [int(p["cluster"].max()) + 1 for p in parts[:-1]])
            df[c] = np.concatenate([p[c] + o for p, o in zip(parts, off)])
        else:
            arr = pa.chunked_array([p[c] for p in parts]).combine_chunks()
            df[c] = pd.Series(arr, dtype=pd.ArrowDtype(pa.large_string()))
        for p in parts:
            p[c] = None
    return df


# Named benchmark / parity configs (BASELINE.json "configs").
CONFIGS = {
    1: dict(n=1000, surname_vocab=100, first_vocab=300, city_vocab=80),
    2: dict(n=1_000_000, surname_vocab=15000),
    4: dict(n=20_000_000, surname_vocab=300000),
    5: dict(n=100_000_000, surname_vocab=600000, with_address=True),
}


def cfg_settings(cfg: int = 2, max_iterations: int = 10) -> dict:
    """Settings dict for configs 1/2/4: first/surname JW-3, dob/city exact-2, email Lev-3;
    config 5 adds the free-text address column as Levenshtein-4 (case_statements.py:128-141)."""
    st = {
        "link_type": "dedupe_only",
        "proportion_of_matches": 0.01,
        "max_iterations": max_iterations,
        "em_convergence": 1e-12,
        "retain_matching_columns": False,
        "retain_intermediate_calculation_columns": False,
        "blocking_rules": ["l.surname = r.surname", "l.dob = r.dob"],
        "comparison_columns": [
            {"col_name": "first_name", "num_levels": 3,
             "case_expression": _jw3("first_name")},
            {"col_name": "surname", "num_levels": 3,
             "case_expression": _jw3("surname")},
            {"col_name": "dob", "num_levels": 2,
             "case_expression": _eq2("dob")},
            {"col_name": "city", "num_levels": 2,
             "case_expression": _eq2("city")},
            {"col_name": "email", "num_levels": 3,
             "case_expression": _lev3("email")},
        ],
    }
    if cfg == 5:
        st["comparison_columns"].append({"col_name": "address", "num_levels": 4, "case_expression": _lev4("address")})
    return st


def _jw3(c):
    return (f"case when {c}_l is null or {c}_r is null then -1 "
            f"when jaro_winkler_sim({c}_l, {c}_r) > 0.94 then 2 "
            f"when jaro_winkler_sim({c}_l, {c}_r) > 0.88 then 1 else 0 end")


def _eq2(c):
    return (f"case when {c}_l is null or {c}_r is null then -1 "
            f"when {c}_l = {c}_r then 1 else 0 end")


def _lev3(c):
    return (f"case when {c}_l is null or {c}_r is null then -1 "
            f"when {c}_l = {c}_r then 2 "
            f"when levenshtein({c}_l, {c}_r)/((length({c}_l) + length({c}_r))/2) <= 0.3 then 1 "
            f"else 0 end")


def _lev4(c):
    ratio = f"levenshtein({c}_l, {c}_r)/((length({c}_l) + length({c}_r))/2)"
    return (f"case when {c}_l is null or {c}_r is null then -1 "
            f"when {c}_l = {c}_r then 3 "
            f"when {ratio} <= 0.2 then 2 "
            f"when {ratio} <= 0.4 then 1 "
            f"else 0 end")
