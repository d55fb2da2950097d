"""The CPU oracle under AddressSanitizer + UBSan (the parity arbiter gets a sanitizer build).

`make -C oracle asan` compiles splink_oracle.c into oracle/_asan/oracle_selftest with every sanitizer
finding fatal.  The driver runs the oracle's entry points on
  * the reference-generated string fixtures (tests/golden/string_values.json: JW and Levenshtein of
    the reference's own test strings) -- bit-exact against the fixture values;
  * empty, one-unit, 255-257-unit (the oracle's stack / heap switch) and 1000-unit strings with
    surrogate pairs and non-BMP code points;
  * the template-gamma program (dedupe and link branches, NULL rows) and the E / M statistics,
    log-likelihood, scores and Bayes combine of a small EM problem,
and every value must equal the -O2 OpenMP library's (the statistics, summed in a different
partition of threads, to 1e-12 relative).  CPU only."""
import shutil
import subprocess

import numpy as np
import pytest

import oracle as orc
from conftest import load_golden

HERE = orc.HERE
EXE = f"{HERE}/_asan/oracle_selftest"


@pytest.fixture(scope="module")
def selftest():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    r = subprocess.run(["make", "-s", "-C", HERE, "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("no sanitizer runtime for gcc here: " + r.stderr[-300:])

    def run(text):
        p = subprocess.run([EXE], input=text, capture_output=True, text=True, timeout=300,
                           env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1",
                                "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
        assert p.returncode == 0, p.stderr[-3000:]
        assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
        return p.stdout.split("\n")
    return run


def _units(s):
    u16 = np.frombuffer(s.encode("utf-16-le", "surrogatepass"), dtype=np.uint16)
    u32 = [ord(c) for c in s]
    return u16.tolist(), u32


def _pair_line(a, b):
    a16, a32 = _units(a)
    b16, b32 = _units(b)
    return " ".join(str(v) for v in [len(a16), *a16, len(b16), *b16, len(a32), *a32, len(b32), *b32])


def test_strings_golden_and_edges(selftest):
    g = load_golden("string_values")
    pairs = [tuple(p) for p in g["pairs"]]
    rng = np.random.Generator(np.random.PCG64(5))
    alpha = list("abcdefgh") + ["é", "\U0001F600", "\U0001D400", "￿"]
    extra = [("", ""), ("", "a"), ("a", ""), ("a", "a"), ("ab", "ba")]
    for n in (1, 2, 127, 128, 129, 255, 256, 257, 258, 600, 1000):
        for _ in range(3):
            a = "".join(rng.choice(alpha, size=n))
            b = "".join(rng.choice(alpha, size=max(0, n + int(rng.integers(-3, 4)))))
            extra.append((a, b))
    text = "S %d\n%s\n" % (len(pairs) + len(extra), "\n".join(_pair_line(a, b) for a, b in pairs + extra))
    out = selftest(text)
    for i, (a, b) in enumerate(pairs + extra):
        jw_s, lev_s = out[i].split()
        jw, lev = float.fromhex(jw_s), int(lev_s)
        assert jw == orc.jaro_winkler(a, b), (a, b)
        assert lev == orc.levenshtein(a, b), (a, b)
        if i < len(pairs):  # the reference's own values
            assert jw == g["jw"][i], (a, b, jw, g["jw"][i])
            assert lev == g["lev"][i], (a, b)


def test_template_gammas(selftest):
    rng = np.random.Generator(np.random.PCG64(9))
    alpha = list("abcde") + ["é", "\U0001F600"]
    R = 60
    cols = []
    for k in range(3):
        vals = ["".join(rng.choice(alpha, size=int(rng.integers(0, 14)))) for _ in range(R)]
        for r in rng.choice(R, size=6, replace=False):
            vals[r] = None
        cols.append(vals)
    specs = [("eq", 2, []), ("jw", 3, [0.94, 0.88]), ("lev", 4, [0.2, 0.4])]
    pl = rng.integers(0, R, size=400).astype(np.int32)
    pr = rng.integers(0, R, size=400).astype(np.int32)
    sc = [orc.StrCol(c) for c in cols]
    want = orc.template_gammas(specs, sc, sc, pl, pr)
    for link in (0, 1):
        lines = ["G 3 %d %d %d" % (R, len(pl), link)]
        kinds = {"eq": 0, "jw": 1, "lev": 2}
        for kind, nlev, thr in specs:
            t = list(thr) + [0.0] * (3 - len(thr))
            lines.append(" ".join([str(kinds[kind]), str(nlev)] + [float(x).hex() for x in t]))
        for vals in cols:
            for v in vals:
                a16, a32 = _units(v or "")
                lines.append(" ".join(str(x) for x in [0 if v is None else 1, len(a16), *a16, len(a32), *a32]))
        lines += ["%d %d" % (a, b) for a, b in zip(pl, pr)]
        out = selftest("\n".join(lines) + "\n")
        got = np.array([[int(x) for x in out[i].split()] for i in range(len(pl))], dtype=np.int8)
        assert np.array_equal(got, want), link


def test_em_statistics(selftest):
    rng = np.random.Generator(np.random.PCG64(13))
    nlev = np.array([2, 3, 4], dtype=np.int32)
    P = 3000
    gam = np.stack([rng.integers(-1, L, size=P) for L in nlev], axis=1).astype(np.int8)
    m = [list(rng.dirichlet(np.ones(L))) for L in nlev]
    u = [list(rng.dirichlet(np.ones(L))) for L in nlev]
    lam = 0.0123
    mq = [orc.quantise(x) for row in m for x in row]
    uq = [orc.quantise(x) for row in u for x in row]
    text = "E 3 %d %s %s\n%s\n%s\n%s\n%s\n" % (
        P, float(repr(lam)).hex(), float(repr(1 - lam)).hex(), " ".join(map(str, nlev)),
        " ".join(x.hex() for x in mq), " ".join(x.hex() for x in uq), " ".join(map(str, gam.reshape(-1))))
    out = selftest(text)
    stats = np.array([float.fromhex(x) for x in out[0].split()])
    want = orc.em_stats(gam, nlev, lam, m, u)
    assert np.allclose(stats, want, rtol=1e-12, atol=0)
    ll = [float.fromhex(x) for x in out[1].split()]
    want_ll = orc.log_likelihood(gam, nlev, lam, m, u)
    assert ll[1] == P and abs(ll[0] - want_ll) <= 1e-12 * abs(want_ll)
    mp = np.array([float.fromhex(x) for x in out[2].split()])
    want_mp = orc.score(gam, nlev, lam, m, u)
    assert np.array_equal(mp, want_mp, equal_nan=True)
    assert float.fromhex(out[3]) == orc._bayes(list(mp[:4]))
