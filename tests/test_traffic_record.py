"""The committed HBM-traffic record behind bench.py's roofline.traffic (CPU).

tools/traffic.py groups rocprofv3 counter rows by kernel name.  Round 3's record left the filter kernel
out of the γ group after a rename; these tests pin the group to the kernels the sources launch and the
record's γ figure to its own per-kernel rows."""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import traffic  # noqa: E402

LAUNCH = re.compile(r"\b(k_[a-z0-9_]+)(?:<[^<>]*>)?<<<")


def _launched(*files):
    names = set()
    for f in files:
        with open(os.path.join(ROOT, "splink_amd", "csrc", f)) as fh:
            names |= set(LAUNCH.findall(fh.read()))
    return names


def test_gamma_group_covers_every_gamma_launch():
    launched = _launched("spk_gamma.hip", "spk_filter.hip")
    assert "k_filter" in launched
    unknown = launched - set(traffic.GAMMA_KERNELS) - set(traffic.NOT_GAMMA_KERNELS)
    assert not unknown, f"kernels launched by the γ sources but in neither traffic.py list: {unknown}"
    for k in launched & set(traffic.GAMMA_KERNELS):
        assert traffic.GAMMA.search(f"void spk::{k}<3, 5, false>(spk::FiltArgs)"), k
    for k in traffic.NOT_GAMMA_KERNELS:
        assert not traffic.GAMMA.search(f"spk::{k}(x)"), k
    # kernels of other entry points never count as γ traffic
    for k in ("k_em_iter<unsigned short, 64, true>", "k_score<unsigned short, true>", "k_hist_lanes", "k_enum<true>"):
        assert not traffic.GAMMA.search(f"void spk::{k}(a)"), k


def _bench_traffic_file():
    import bench
    return bench.TRAFFIC_FILE


def test_bench_traffic_record_matches_its_kernel_rows():
    path = _bench_traffic_file()
    if not os.path.exists(path):
        pytest.skip(f"{path} not recorded yet")
    with open(path) as f:
        rec = json.load(f)
    g = rec["gamma"]
    rows = rec["per_kernel_avg_kib"]
    assert any("k_filter" in k for k in g["kernels"]), "the filter kernel must be in the γ group"
    want = 0.0
    for k, x in rows.items():
        if traffic.GAMMA.search(k) and not traffic.GAMMA_ONCE.search(k):
            want += (x["fetch_kib"] + x["write_kib"]) * x["dispatches"] * 1024.0 / g["calls"]
    assert g["traffic_bytes_per_call"] == pytest.approx(want, rel=1e-12)
    assert g["traffic_bytes_per_call"] == pytest.approx(g["fetch_bytes_per_call"] + g["write_bytes_per_call"],
                                                        rel=1e-12)
