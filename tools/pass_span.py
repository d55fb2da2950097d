"""Span of each comparison pass in a rocprofv3 kernel trace: from the first k_filter start to the last end of a
comparison-pass kernel (filter, compaction, exact / slow passes) before the next k_em_iter.  Under the two-stream
split both windows' kernels overlap inside one span, so rocprof's per-launch averages are per window and the span is
what the bench line's HIP-event γ time brackets.

    python tools/pass_span.py gpurun_out/prof_r6f/run_kernel_trace.csv [--last 20]
"""
import argparse
import csv

PASS = ("k_filter", "k_gamma_filter", "k_prefix", "k_compact", "k_gamma_exact", "k_lev_refill", "k_gamma_slow",
        "k_gamma_rest", "k_gamma_huge", "k_bag_rows")


def spans(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out, lo, hi = [], None, None
    for r in rows:
        name = r["Kernel_Name"].replace("spk::", "")
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "k_em_iter" in name:
            if lo is not None:
                out.append((hi - lo) / 1e3)
            lo = hi = None
        elif any(k in name for k in PASS):
            if lo is None and "filter" in name:
                lo = t0
            if lo is not None:
                hi = max(hi or t1, t1)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=20)
    a = ap.parse_args()
    s = spans(a.trace)
    srt = sorted(s)
    med = srt[len(srt) // 2] if srt else float("nan")
    tail = s[-a.last:]
    print(f"passes {len(s)} median span us {med:.1f} mean of the last {len(tail)} {sum(tail) / max(len(tail), 1):.1f}")
