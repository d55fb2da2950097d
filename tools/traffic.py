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
  gamma : every kernel spk_gammas launches (k_build_image, k_view_image, k_gamma_*), per call
          (calls = k_prefix dispatches)
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

GAMMA = re.compile(r"k_build_image|k_view_image|k_gamma_|k_compact|k_prefix")
EM = re.compile(r"k_hist|k_em_iter|k_em_finalize")


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
    a = ap.parse_args()
    fetch, write = read_counter(a.fetch, "FETCH_SIZE"), read_counter(a.write, "WRITE_SIZE")
    res = {"source": {"fetch_pass": a.fetch, "write_pass": a.write}}
    n_calls = max(1, len(calls_of(fetch, r"k_prefix")))
    fg = sum(v for d, k, v in fetch if GAMMA.search(k)) * 1024.0 / n_calls
    wg = sum(v for d, k, v in write if GAMMA.search(k)) * 1024.0 / n_calls
    res["gamma"] = {"calls": n_calls, "fetch_bytes_per_call": fg, "fetch_bytes_per_call_x2": 2 * fg,
                    "write_bytes_per_call": wg, "traffic_bytes_per_call": fg + wg,
                    "traffic_bytes_per_call_upper": 2 * fg + wg,
                    "correction": "FETCH_SIZE x 1 (scattered line gathers, calibrated); x 2 = stream upper bound"}
    fh, ft = split_em(fetch, a.head_em)
    wh, wt = split_em(write, a.head_em)
    for name, fs, ws in (("em", fh, wh), ("em_at_scale", ft, wt)):
        if fs:
            fb = 2.0 * 1024.0 * sum(fs) / len(fs)
            wb = 1024.0 * sum(ws) / max(1, len(ws))
            res[name] = {"calls": len(fs), "fetch_bytes_per_call": fb, "write_bytes_per_call": wb,
                         "traffic_bytes_per_call": fb + wb, "correction": "2 x FETCH_SIZE (streams) + WRITE_SIZE"}
    if a.calib:
        cal = collections.defaultdict(list)
        for d, k, v in read_counter(a.calib, "FETCH_SIZE"):
            cal[re.sub(r"\(.*", "", k)[:40]].append(v)
        res["calibration"] = {k: {"fetch_kib_avg": sum(v) / len(v), "dispatches": len(v)} for k, v in cal.items()}
        res["calibration"]["note"] = ("tools/calib_fetch: k_stream16 reads 2 GiB (2097152 KiB); k_gather* read one "
                                      "4/8/16-byte word from each of 16M distinct 128-byte lines")
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
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
