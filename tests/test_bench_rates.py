"""bench.string_rates on a stub job (host logic only, no GPU): Σ len_l·len_r over the pairs of each
Levenshtein column, comparisons per second over the γ-pass time."""
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class _StubJob:
    def __init__(self, table, l, r):
        self.tables = [table]
        self._lr = (np.asarray(l, dtype=np.int32), np.asarray(r, dtype=np.int32))

    def pair_rows(self):
        return self._lr


def test_string_rates_counts_dp_cells_and_rates():
    t = pd.DataFrame({"name": ["ab", "abc", None, "é"], "email": ["a@b", None, "xyzw", "ü@x"]})
    st = {"comparison_columns": [
        {"col_name": "name", "case_expression": "case when jaro_winkler_sim(name_l, name_r) > 0.9 then 1 else 0 end"},
        {"col_name": "email", "case_expression": "case when levenshtein(email_l, email_r) <= 1 then 1 else 0 end"},
    ]}
    l, r = [0, 0, 1, 2], [1, 3, 3, 3]
    out = bench.string_rates(_StubJob(t, l, r), st, len(l), g_ms=2.0)
    # email code points: 3, null (0), 4, 3 -> 3*0 + 3*3 + 0*3 + 4*3
    assert out["lev_dp_cells_per_pass"] == 21
    assert np.isclose(out["lev_effective_gcups"], 21 / 2e-3 / 1e9)
    assert np.isclose(out["comparisons_per_s"], 4 * 2 / 2e-3)
    assert np.isclose(out["jw_comparisons_per_s"], 4 / 2e-3)
    assert np.isclose(out["lev_comparisons_per_s"], 4 / 2e-3)
