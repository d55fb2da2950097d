"""HBM traffic per launch from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE in separate runs).

    python tools/traffic.py --fetch DIR --write DIR [--calib DIR] [--head-em N] [--out profiles/rN_traffic.json]

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters (KiB per dispatch, from the L2's memory-side
request counters).  Corrections, per access shape:
  * streams (16-byte lanes, coalesced): FETCH_SIZE reports half the bytes on gfx950
    (MI355X_MICROARCH.md "HBM [CDNA4]"), confirmed by tools/calib_fetch's k_stream16 (ratio 0.500);
  * scattered loads (one load per 128-byte line, 4 / 8 / 16 bytes): FETCH_SIZE reports 64 bytes per
    line (tools/calib_fetch k_gather*, 66.0 B per gather with the index stream), and their kernel time
    (16M lines in 354 us vs 2 GiB streamed in 403 us) matches 64-byte sectors, not 128-byte lines,
    so the counter is taken as is (factor 1).
The comparison pass (gamma group) is gather-bound: its traffic is FETCH_SIZE x 1 (+ WRITE_SIZE), with
the x 2 stream reading as an upper bound; the E/M kernels stream: x 2.

Kernel groups, per call of the C-ABI entry point (one "launch" of bench.py's roofline):
  gamma : every kernel spk_gammas launches (GAMMA_KERNELS: the filter k_filter, the exact / slow passes,
          list compaction), per call (calls = k_prefix dispatches), from the per-kernel averages
          (gamma_traffic); the one-time image builds are reported apart
  em    : k_em_iter (histogram + E-step + M-step sums, one launch) per E+M iteration; the first --head-em calls
          (bench.py's warmup + timed steps at the headline size), the rest reported as em_at_scale
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

# Every kernel spk_gammas launches (spk_gamma.hip, spk_filter.hip); tests/test_traffic_record.py checks
# the list against the sources' launch sites, so a renamed or new kernel cannot drop out of the group.
GAMMA_KERNELS = ("k_build_image", "k_view_image", "k_filter", "k_gamma_filter", "k_gamma_exact",
                 "k_gamma_exact_simple", "k_lev_refill", "k_gamma_slow", "k_gamma_slow_lev", "k_gamma_rest", "k_gamma_huge",
                 "k_compact", "k_compact_lev", "k_prefix")
# launched from the same sources by other entry points (spk_gammas_load / _copy, the bulk UDFs)
NOT_GAMMA_KERNELS = ("k_codes_from_gammas", "k_gammas_from_codes", "k_udf", "k_udf_huge")
GAMMA = re.compile(r"\b(?:spk::)?(" + "|".join(GAMMA_KERNELS) + r")\b")
EM = re.compile(r"k_hist|k_em_iter|k_em_finalize")
# built once per table / pair-set change, not per call: reported beside the per-call traffic
GAMMA_ONCE = re.compile(r"\b(?:spk::)?(k_build_image|k_view_image)\b")


def gamma_traffic(per_kernel_avg_kib, calls):
    """Per-call HBM bytes of the γ pass from the per-kernel averages (KiB per dispatch): every GAMMA
    kernel but the one-time image builds, FETCH_SIZE x 1 + WRITE_SIZE, x dispatches / calls."""
    f = w = once = 0.0
    for k, x in per_kernel_avg_kib.items():
        if not GAMMA.search(k):
            continue
        fb, wb = x["fetch_kib"] * x["dispatches"] * 1024.0, x["write_kib"] * x["dispatches"] * 1024.0
        if GAMMA_ONCE.search(k):
            once += fb + wb
        else:
            f += fb / calls
            w += wb / calls
    return {"fetch_bytes_per_call": f, "write_bytes_per_call": w, "traffic_bytes_per_call": f + w,
            "fetch_bytes_per_call_x2": 2 * f, "traffic_bytes_per_call_upper": 2 * f + w,
            "image_build_bytes_once": once}


def read_counter(d, name):
    """[(dispatch id, kernel name, value)] in dispatch order."""
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    return sorted(out)


def calls_of(rows, pat):
    return [i for i, (d, k, v) in enumerate(rows) if re.search(pat, k)]


def split_em(rows, head):
    """EM dispatches grouped per E+M iteration: k_em_iter (one launch), or k_hist + k_em_finalize."""
    calls, cur = [], []
    for d, k, v in rows:
        if not EM.search(k):
            continue
        cur.append(v)
        if "k_em_iter" in k or "k_em_finalize" in k:
            calls.append(sum(cur))
            cur = []
    return calls[:head], calls[head:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib")
    ap.add_argument("--head-em", type=int, default=3)
    ap.add_argument("--out")
    ap.add_argument("--recompute", help="rewrite the gamma group of an existing record from its per-kernel rows")
    a = ap.parse_args()
    if a.recompute:
        with open(a.recompute) as f:
            res = json.load(f)
        calls = res["gamma"]["calls"]
        res["gamma"] = {"calls": calls, **gamma_traffic(res["per_kernel_avg_kib"], calls),
                        "kernels": [k for k in res["per_kernel_avg_kib"] if GAMMA.search(k)],
                        "correction": "recomputed by tools/traffic.py --recompute from per_kernel_avg_kib"}
        print(json.dumps(res["gamma"], indent=1))
        with open(a.out or a.recompute, "w") as f:
            json.dump(res, f, indent=1)
        return
    fetch, write = read_counter(a.fetch, "FETCH_SIZE"), read_counter(a.write, "WRITE_SIZE")
    res = {"source": {"fetch_pass": a.fetch, "write_pass": a.write}}
    n_calls = max(1, len(calls_of(fetch, r"k_prefix")))
    fh, ft = split_em(fetch, a.head_em)
    wh, wt = split_em(write, a.head_em)
    for name, fs, ws in (("em", fh, wh), ("em_at_scale", ft, wt)):
        if fs:
            fb = 2.0 * 1024.0 * sum(fs) / len(fs)
            wb = 1024.0 * sum(ws) / max(1, len(ws))
            res[name] = {"calls": len(fs), "fetch_bytes_per_call": fb, "write_bytes_per_call": wb,
                         "traffic_bytes_per_call": fb + wb, "correction": "2 x FETCH_SIZE (streams) + WRITE_SIZE"}
    per_kernel = collections.defaultdict(lambda: {"dispatches": 0, "fetch_kib": 0.0, "write_kib": 0.0})
    for d, k, v in fetch:
        s = re.sub(r"\(.*", "", k)[:80]
        per_kernel[s]["dispatches"] += 1
        per_kernel[s]["fetch_kib"] += v
    for d, k, v in write:
        per_kernel[re.sub(r"\(.*", "", k)[:80]]["write_kib"] += v
    res["per_kernel_avg_kib"] = {k: {"dispatches": x["dispatches"], "fetch_kib": x["fetch_kib"] / max(1, x["dispatches"]),
                                     "write_kib": x["write_kib"] / max(1, x["dispatches"])}
                                 for k, x in per_kernel.items()}
    res["gamma"] = {"calls": n_calls, **gamma_traffic(res["per_kernel_avg_kib"], n_calls),
                    "kernels": [k for k in res["per_kernel_avg_kib"] if GAMMA.search(k)],
                    "correction": "FETCH_SIZE x 1 (scattered line gathers, calibrated) + WRITE_SIZE; x 2 = stream "
                                  "upper bound; image builds (once per table change) excluded from the per-call figure"}
    if a.calib:
        cal = collections.defaultdict(list)
        for d, k, v in read_counter(a.calib, "FETCH_SIZE"):
            cal[re.sub(r"\(.*", "", k)[:40]].append(v)
        res["calibration"] = {k: {"fetch_kib_avg": sum(v) / len(v), "dispatches": len(v)} for k, v in cal.items()}
        res["calibration"]["note"] = ("tools/calib_fetch: k_stream16 reads 2 GiB (2097152 KiB); k_gather* read one "
                                      "4/8/16-byte word from each of 16M distinct 128-byte lines")
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
