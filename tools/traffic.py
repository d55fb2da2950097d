"""HBM traffic per launch from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE in separate runs).

    python tools/traffic.py --fetch DIR --write DIR [--em-bytes B] [--out profiles/rN_traffic.json]

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters (KiB per dispatch, from the L2's
memory-side request counters).  The correction follows MI355X_MICROARCH.md "HBM [CDNA4]": on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so fetched bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is taken as is.  The calibration kernel is k_hist_lanes:
it streams exactly P x 2 bytes of comparison codes with 16-byte loads, so its corrected
fetch / algorithmic ratio (--em-bytes) is reported next to the figures.

Kernel groups, per call of the C-ABI entry point (one "launch" of bench.py's roofline):
  gamma : every kernel spk_gammas launches (k_build_image, k_gamma_*), summed per call
  em    : k_hist_lanes / k_hist + k_hist_reduce, per spk_em_histogram call
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

GROUPS = {"gamma": re.compile(r"k_build_image|k_gamma_"), "em": re.compile(r"k_hist")}


def read_counter(d, name):
    """{kernel name: [value per dispatch]}"""
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def group_total(per_kernel, pat):
    tot, n = 0.0, 0
    for k, vs in per_kernel.items():
        if pat.search(k):
            tot += sum(vs)
            n += len(vs)
    return tot, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--em-bytes", type=float, default=None, help="algorithmic bytes of one k_hist launch")
    ap.add_argument("--out")
    a = ap.parse_args()
    fetch = read_counter(a.fetch, "FETCH_SIZE")
    write = read_counter(a.write, "WRITE_SIZE")
    # calls = dispatches of the kernel each entry point launches exactly once per call
    calls = {"gamma": len([v for k, vs in fetch.items() if re.search(r"k_gamma_simple|k_gamma_rows", k) for v in vs]),
             "em": len([v for k, vs in fetch.items() if re.search(r"k_hist_lanes|k_hist<", k) for v in vs])}
    res = {"source": {"fetch_pass": a.fetch, "write_pass": a.write, "calls": calls},
           "correction": "bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md HBM [CDNA4])"}
    for g, pat in GROUPS.items():
        f, nf = group_total(fetch, pat)
        w, nw = group_total(write, pat)
        fb = 2.0 * f * 1024.0 / max(1, calls[g])
        wb = w * 1024.0 / max(1, calls[g])
        res[g] = {"fetch_bytes_per_call": fb, "write_bytes_per_call": wb, "traffic_bytes_per_call": fb + wb,
                  "dispatches": [nf, nw]}
    if a.em_bytes:
        res["em"]["calibration_fetch_over_algorithmic"] = res["em"]["fetch_bytes_per_call"] / a.em_bytes
    per_kernel = {}
    for k in sorted(set(fetch) | set(write)):
        short = re.sub(r"\(.*", "", k)[:80]
        fs, ws = fetch.get(k, []), write.get(k, [])
        per_kernel[short] = {"dispatches": max(len(fs), len(ws)),
                             "fetch_bytes_avg": 2048.0 * sum(fs) / max(1, len(fs)),
                             "write_bytes_avg": 1024.0 * sum(ws) / max(1, len(ws))}
    res["per_kernel"] = per_kernel
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
