"""bench.string_rates on a stub job (host logic only, no GPU): DP cells of the cells in each Levenshtein
column's exact list (nominal len_l·len_r, and the word-steps x word width the scans update) over that
launch's time, comparisons per second over the γ-pass time."""
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class _StubCtx:
    def gammas_exact_counts(self, n):
        return [0, 2][:n]

    def gammas_exact_ms(self, n):
        return [-1.0, 0.5][:n]

    def enable_timing(self, on=True, exact=False):
        self.exact_timing = on and exact

    def gammas_set_streams(self, streams, min_pairs=1 << 22):
        self.streams = streams

    def gammas_exact_list(self, k, n):
        assert k == 1 and n == 2
        return np.array([1, 3], dtype=np.int32)  # pair ordinals the Levenshtein exact pass evaluated


class _StubJob:
    def __init__(self, table, l, r):
        self.tables = [table]
        self._lr = (np.asarray(l, dtype=np.int32), np.asarray(r, dtype=np.int32))
        self.ctx = _StubCtx()

    def pair_rows(self):
        return self._lr

    def gammas(self, st):  # bench.exact_pass_ms: one pass on one stream with per-launch events
        assert self.ctx.exact_timing and self.ctx.streams == 1


def test_string_rates_counts_dp_cells_and_rates():
    t = pd.DataFrame({"name": ["ab", "abc", None, "é"], "email": ["a@b", None, "xyzw", "ü@x"]})
    st = {"comparison_columns": [
        {"col_name": "name", "case_expression": "case when jaro_winkler_sim(name_l, name_r) > 0.9 then 1 else 0 end"},
        {"col_name": "email", "case_expression": "case when levenshtein(email_l, email_r) <= 1 then 1 else 0 end"},
    ]}
    l, r = [0, 0, 1, 2], [1, 3, 3, 3]
    out = bench.string_rates(_StubJob(t, l, r), st, len(l), g_ms=2.0)
    lev = out["levenshtein_exact_pass"]["email"]
    # listed pairs 1 (rows 0, 3: 3 x 3 code points) and 3 (rows 2, 3: 4 x 3)
    assert lev["dp_cells_nominal"] == 21 and lev["exact_cells"] == 2
    assert np.isclose(lev["gcups_nominal"], 21 / 0.5e-3 / 1e9)
    # the scans: no common prefix / suffix, 3 text units each (shorter side), 32-bit words, no early exit
    assert lev["dp_cells_scanned_est"] == 2 * 3 * 32
    assert np.isclose(lev["gcups_scanned"], 192 / 0.5e-3 / 1e9)
    assert np.isclose(lev["exact_cells_per_s"], 2 / 0.5e-3)
    assert np.isclose(out["comparisons_per_s"], 4 * 2 / 2e-3)
    assert np.isclose(out["jw_comparisons_per_s"], 4 / 2e-3)
    assert np.isclose(out["lev_comparisons_per_s"], 4 / 2e-3)


def test_lev_scan_cells_early_exit_and_strip():
    # equal strings and a side that strips to nothing: no scan
    assert bench.lev_scan_cells("abc", "abc", 2) == 0
    assert bench.lev_scan_cells("abc", "abcd", 2) == 0
    # common prefix and suffix stripped: "x" vs "yz" -> one text unit, 32 rows
    assert bench.lev_scan_cells("abxcd", "abyzcd", 2) == 32
    # dissimilar 40 vs 40 units at cut 3: the bound passes cut at the first tested unit (j = 3) -> 4 steps, the
    # wide pattern (40 > 32 rows) still in its 32-bit phase (J0 = 31 - 3 = 28)
    assert bench.lev_scan_cells("a" * 40, "b" * 40, 3) == 4 * 32
