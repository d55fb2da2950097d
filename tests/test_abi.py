"""The C-ABI library loads without a GPU and exports every symbol include/splink_hip.h declares."""
import os
import re

from conftest import ROOT

from splink_amd import _native as N


def declared_functions():
    text = open(os.path.join(ROOT, "include", "splink_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(spk_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("spk_ctx_create", "spk_block", "spk_gammas", "spk_em_histogram", "spk_em_finalize",
                     "spk_score", "spk_tf_apply", "spk_jaro_winkler_sim"):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = N.load_library()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(N.EXPORTS) == set(declared_functions())


def test_struct_layouts_match_header():
    assert N.OPERAND_DTYPE.itemsize == 40
    assert N.INSTR_DTYPE.itemsize == 32
    assert N.PROGRAM_DTYPE.itemsize == 16


def test_no_device_means_loud_failure():
    if N.device_count() > 0:
        return
    import pytest
    with pytest.raises(N.NativeUnavailable):
        N.Context(0)


def test_tf_limbs_to_sum_exact():
    """spk_tf_limbs_to_sum (host only): fixed-point accumulators of mp values (term_frequencies.py:49-65's
    per-value Σmp) relative to each value's scale (ilogb of its largest term + 1) convert back within
    1e-15 of the exact sum, carries included, down to subnormal match probabilities."""
    import math
    import struct
    import numpy as np
    from splink_amd import _native as N
    L, B = N.TF_LIMBS, 20

    def exponent(x):  # ilogb(x) + 1, subnormals included (spk_tf.hip tf_exponent)
        return math.frexp(x)[1]

    def limbs(x, E):  # restatement of spk_tf.hip tf_limbs: y = x 2^-E, truncated below 2^-260
        out = [0] * L
        if not x > 0.0:
            return out
        bits = struct.unpack("<Q", struct.pack("<d", x))[0]
        ex = (bits >> 52) & 0x7FF
        m = (bits & ((1 << 52) - 1)) | ((1 << 52) if ex else 0)
        s = (ex if ex else 1) - 1075 - E + B * (L - 1)
        for j in range(L):
            sh = B * (L - 1 - j) - s
            v = (m >> sh if sh < 64 else 0) if sh >= 0 else ((m << -sh) & ((1 << 64) - 1) if -sh < 64 else 0)
            out[j] = v & ((1 << B) - 1)
        return out
    rng = np.random.Generator(np.random.PCG64(3))
    values = [[1.0, 0.5], [1e-30, 3e-31, 0.7], list(rng.random(40) ** 8), [0.0], list(rng.random(5) * 1e-50),
              [1e-300, 3e-305, 2e-301], [5e-324, 1e-320, 2.5e-310], list(rng.random(7) * 1e-200)]
    acc = np.zeros((len(values), L), dtype=np.int64)
    scale = np.full(len(values), N.TF_NO_SCALE, dtype=np.int32)
    exact = []
    for v, xs in enumerate(values):
        pos = [x for x in xs if x > 0]
        if pos:
            scale[v] = max(exponent(float(x)) for x in pos)
        counts = rng.integers(1, 5000, len(xs))
        for x, c in zip(xs, counts):
            acc[v] += int(c) * np.array(limbs(float(x), int(scale[v])), dtype=np.int64)
        exact.append(math.fsum(float(c) * float(x) for x, c in zip(xs, counts)))
    got = N.tf_limbs_to_sum(acc, scale)
    for g, e in zip(got, exact):
        assert (g == e == 0.0) or abs(g - e) <= 1e-15 * abs(e), (g, e)
