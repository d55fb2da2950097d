"""Summarise rocprofv3 --pmc counter CSVs per kernel (per dispatch averages).

    python tools/pmc_summary.py gpurun_out/pmc1_TAG gpurun_out/pmc2_TAG ... [--match REGEX] [--json OUT]
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    args = sys.argv[1:]
    match, out = None, None
    if "--match" in args:
        i = args.index("--match"); match = args[i + 1]; del args[i:i + 2]
    if "--json" in args:
        i = args.index("--json"); out = args[i + 1]; del args[i:i + 2]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in args:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if match and not re.search(match, k):
                    continue
                vals[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    summary = {}
    for k, cs in vals.items():
        summary[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        summary[k]["dispatches"] = max(len(v) for v in cs.values())
    for k, cs in summary.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {v:14.4g}")
    if out:
        with open(out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
