"""One complete linkage job on one GPU, timed end to end, with parity checks (a separately labelled row,
never bench.py's headline).

    python tools/full_job.py --records 20000000 --shard 0/8 [--iters 10] [--sample 2000000] [--out FILE]
    python tools/full_job.py --config 3 --records 10000000 --shard 0/8 ...   (link_only 2 x 10M + tf)

The job is BASELINE configs[3]'s per-GPU share: a 20M-record synthetic dedupe (blocking surname | dob,
the five cfg2 comparison columns) whose candidate-pair ordinals are split over 8 GPUs; this process is
rank `shard` and generates only its slice of the ordinal space (spk_block shard / n_shards), exactly as
each rank of an 8-GPU run does.  Without a process group the EM statistics are this shard's (the RCCL
all-reduce of the 8-rank job is a 4.6 KB histogram per iteration).

Timed stages (wall clock, inputs in host memory as Arrow-backed columns, generation excluded):
blocking (raw column upload + device keys + clustering + pair generation), the comparison-vector
pass (first call: column upload + device decode), 10 EM iterations (histogram + finalize + the host
M-step), the final scoring pass.  Parity: every comparison vector of a strided sample of pairs against
oracle.template_gammas, and the 10 EM iterations of λ / m / u plus the final match probabilities of
all of this shard's pairs against oracle.em_iterate (1e-9).

--config 5 adds cfg5's free-text address column (30-128 characters, Levenshtein-4) to the five cfg2
columns; with --records 20000000 --shard 0/5 one GPU holds ~1.2B pairs, cfg5's per-GPU pair count
(100M records, ~10B pairs over 8 GPUs).

--config 3 is BASELINE configs[2]'s per-GPU share: link_only between two synthetic tables of
`--records` rows each (one 2 x records population split in halves, so duplicates straddle them),
rules surname | dob | email, the five cfg2 columns, and the term-frequency
adjustment on surname after EM (device dictionary ids as tf value ids; timed as `tf_adjust`).  Its
parity adds every pair's tf_adjusted_match_prob against a numpy restatement of
term_frequencies.py:49-117 over host-factorised values (1e-9).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

COLS = ["first_name", "surname", "dob", "city", "email"]
SPECS = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3])]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=20_000_000)
    ap.add_argument("--surname-vocab", type=int, default=300_000)
    ap.add_argument("--shard", default="0/8")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--sample", type=int, default=2_000_000, help="pairs in the strided gamma parity sample")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--config", type=int, default=4, choices=[3, 4, 5])
    ap.add_argument("--rules", default=None,
                    help="blocking rules separated by '|' (default: the config's; e.g. "
                         "'l.surname = r.surname|l.dob = r.dob and l.city = r.city')")
    ap.add_argument("--chunks", type=int, default=0,
                    help="generate the records as this many independent chunks over one vocabulary, in parallel "
                         "(synthetic.make_records_parallel; 0 = the serial make_records)")
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--tf-mode", type=int, default=0, help="spk_tf_set_mode: 0 histogram when it fits, 1 / 2 the sort")
    ap.add_argument("--no-prefetch", dest="prefetch", action="store_false",
                    help="upload the comparison-only columns in the first comparison call (no background prefetch)")
    a = ap.parse_args()
    global COLS, SPECS
    if a.config == 5:  # + the free-text address column, Levenshtein-4 (cfg5's columns)
        COLS = COLS + ["address"]
        SPECS = SPECS + [("lev", 4, [0.2, 0.4])]
    shard, n_shards = (int(x) for x in a.shard.split("/"))

    import torch
    torch.cuda.set_device(0)
    from splink_amd.engine import Job, m_step_rows
    from splink_amd.params import Params
    from splink_amd.session import AmdSession
    from splink_amd.synthetic import cfg_settings, make_records, make_records_parallel

    t0 = time.time()
    link = a.config == 3
    n_gen = a.records * (2 if link else 1)
    if a.chunks:
        df = make_records_parallel(n_gen, a.chunks, a.workers, surname_vocab=a.surname_vocab,
                                   with_address=a.config == 5)[["unique_id"] + COLS]
    else:
        df = make_records(n_gen, surname_vocab=a.surname_vocab, arrow=True,
                          with_address=a.config == 5)[["unique_id"] + COLS]
    inputs = [df.iloc[:a.records].reset_index(drop=True), df.iloc[a.records:].reset_index(drop=True)] if link else [df]
    del df
    gen_s = time.time() - t0
    log(f"generated {a.records} records x {len(inputs)} in {gen_s:.1f}s")
    settings = cfg_settings(5 if a.config == 5 else 4, max_iterations=a.iters)
    if link:
        settings["link_type"] = "link_only"
        settings["blocking_rules"] = ["l.surname = r.surname", "l.dob = r.dob", "l.email = r.email"]
        for c in settings["comparison_columns"]:
            if c["col_name"] == "surname":
                c["term_frequency_adjustments"] = True
    if a.rules:
        settings["blocking_rules"] = [r.strip() for r in a.rules.split("|")]
    params = Params(settings, AmdSession(0))
    st = params.settings

    # device memory in use (hipMemGetInfo: every allocation on the device, the library's included)
    free0, total_mem = torch.cuda.mem_get_info(0)
    mem = {"device_total_bytes": int(total_mem), "in_use_before_job_bytes": int(total_mem - free0)}

    def mem_mark(stage):
        free, _ = torch.cuda.mem_get_info(0)
        mem[f"after_{stage}_bytes"] = int(total_mem - free)
        if "job" in locals_ref:  # what the library itself holds, by part (spk_ctx_memory)
            mem[f"after_{stage}_library_by_part"] = locals_ref["job"].ctx.memory()
            mem["peak_reserved_by_torch_bytes"] = int(torch.cuda.max_memory_reserved(0))

    locals_ref = {}

    wall = {}
    t_job = time.perf_counter()
    t = time.perf_counter()
    from splink_amd.blocking import _comparison_only_columns
    # the comparison-only columns upload in the background while the uid ranks and blocking run
    pre = _comparison_only_columns(st, st["blocking_rules"], inputs) if a.prefetch else None
    job = Job(st["link_type"], inputs, "unique_id", 0, shard=(shard, n_shards), prefetch=pre)
    locals_ref["job"] = job
    job.ctx.enable_timing(True)
    wall["job_setup_incl_uid_rank"] = time.perf_counter() - t
    t = time.perf_counter()
    job.block(st["blocking_rules"])
    wall["block"] = time.perf_counter() - t
    wall["block_keys_and_cluster"] = job.timings["block_keys_s"]
    block_dev = job.ctx.kernel_ms()["block"]
    mem_mark("block")
    log(f"shard {shard}/{n_shards}: {job.n_pairs} pairs of {job.n_candidates} candidates, block {wall['block']:.2f}s")
    t = time.perf_counter()
    job.gammas(st)
    wall["gammas_first_call_incl_column_decode"] = time.perf_counter() - t
    gamma_dev = job.ctx.kernel_ms()["gamma"]
    mem_mark("gammas")
    names, nlev = job.code_meta
    exact_cells = dict(zip(names, job.ctx.gammas_exact_counts(len(names))))
    job.gammas(st)  # a second pass (row images built, lists sized): the per-pass device time
    gamma_warm = job.ctx.kernel_ms()["gamma"]
    windows = job.ctx.gammas_windows()
    lam0, lp0 = params.params["λ"], params._level_probabilities()
    t = time.perf_counter()
    em_dev = []
    for _ in range(a.iters):
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        ms = job.ctx.kernel_ms()
        em_dev.append(ms["em_hist"] + max(ms["em_final"], 0.0))  # em_final = -1: one launch
        lam, rows = m_step_rows(stats, names, nlev)
        params._update_params(lam, rows)
    wall["em_iterations"] = time.perf_counter() - t
    # how concentrated the comparison patterns are (what bounds the lane-private E+M histogram)
    hist_t = job._device_hist()
    job.ctx.em_histogram(hist_t.data_ptr())
    hist_h = np.sort(hist_t.cpu().numpy())[::-1]
    patterns = {"n_patterns": int(len(hist_h)), "occupied": int((hist_h > 0).sum()),
                "top_share": [round(float(x) / max(int(hist_h.sum()), 1), 5) for x in hist_h[:16]]}
    t = time.perf_counter()
    mp = job.score(params.params["λ"], params._level_probabilities(), want_host=False)
    torch.cuda.synchronize()
    wall["score"] = time.perf_counter() - t
    score_dev = job.ctx.kernel_ms()["score"]
    mem_mark("score")
    if link:  # term-frequency adjustment on surname (term_frequencies.py:122-168), device value ids
        from splink_amd.term_frequencies import _bayes_pair
        t = time.perf_counter()
        col = job._col_index[("surname", "str")]
        job.ctx.tf_set_mode(a.tf_mode)
        n_values = job.ctx.tf_column_values(col)
        tf_values = int(n_values)
        sums, counts = job.ctx.tf_accumulate_column(col, n_values)
        wall["tf_sums"] = time.perf_counter() - t
        with np.errstate(invalid="ignore", divide="ignore"):
            adj_lambda = np.where(counts > 0, sums / np.maximum(counts, 1), np.nan)
        table = _bayes_pair(adj_lambda, float(1 - params.params["λ"]))
        # tf_adjusted_match_prob stays on the device, as the scores do (want_host=False above); the parity pass
        # reads it back (spk_tf_copy)
        job.ctx.tf_apply_columns([col], [table], 0, job.n_pairs, want_adj=False, want_host=False)
        wall["tf_adjust"] = time.perf_counter() - t
        mem_mark("tf")
    total = time.perf_counter() - t_job
    # outside the job's wall: the same pass on one stream (spk_gammas_set_streams), against the default split
    job.ctx.gammas_set_streams(1)
    job.gammas(st)
    gamma_one_stream = job.ctx.kernel_ms()["gamma"]
    job.ctx.gammas_set_streams(2)
    P = job.n_pairs
    row = {
        "row": "full job, one GPU (separately labelled; never the headline)",
        "workload": (f"cfg3 per-GPU share: link_only {a.records} x {a.records} records, blocking surname|dob|email, "
                     f"5 columns, tf on surname, pair-ordinal shard {shard}/{n_shards}") if link else
                    (f"cfg{a.config} columns at {a.records} records: blocking "
                     f"{' | '.join('(' + r + ')' for r in st['blocking_rules'])}, {len(COLS)} columns, "
                     f"pair-ordinal shard {shard}/{n_shards}"),
        "records": a.records, "candidates_total": int(job.n_candidates), "pairs_this_gpu": int(P),
        "iterations": a.iters, "wall_s": wall, "job_wall_s": total, "job_timings_s": dict(job.timings),
        "device_ms": {"block": block_dev, "gamma_pass_first": gamma_dev, "gamma_pass": gamma_warm, "gamma_pass_one_stream": gamma_one_stream,
                      "gamma_windows": windows,
                      "em_per_iter_mean": float(np.mean(em_dev)), "score": score_dev,
                      "em_per_iter": [round(x, 4) for x in em_dev]},
        "exact_cells_per_column": exact_cells,
        "pattern_concentration": patterns,
        "pairs_per_s_job": P / total,
        "pairs_per_s_gamma_plus_em_iter": P / ((gamma_warm + float(np.mean(em_dev))) / 1e3),
        "generation_s_excluded": gen_s,
        "generation": (f"make_records_parallel: {a.chunks} chunks over one vocabulary, {a.workers} processes"
                       if a.chunks else "make_records (serial)"),
        "surname_vocab": a.surname_vocab,
        "blocking_rules": st["blocking_rules"],
        "device_memory": {**mem, "peak_in_use_bytes": max(v for k, v in mem.items()
                                                             if k.startswith("after_") and k.endswith("_bytes"))},
        "lambda_final": params.params["λ"],
    }
    if link:
        row["tf_n_values"] = tf_values  # distinct surnames: n_values x patterns decides histogram vs sort
        row["tf_mode"] = a.tf_mode
    if not a.no_parity:
        import oracle as orc
        t = time.perf_counter()
        l, r = job.pair_rows()
        step = max(1, P // a.sample)
        idx = np.arange(0, P, step)
        sl, sr = l[idx], r[idx]
        rows_used, inv = np.unique(np.concatenate([sl, sr]), return_inverse=True)
        if link:  # rows index the two tables separately
            tl, tr = job.tables[0], job.r_table()
            ul, il = np.unique(sl, return_inverse=True)
            ur, ir = np.unique(sr, return_inverse=True)
            ocl = [orc.StrCol(tl.take(ul)[c].tolist()) for c in COLS]
            ocr = [orc.StrCol(tr.take(ur)[c].tolist()) for c in COLS]
            ref = orc.template_gammas(SPECS, ocl, ocr, il.astype(np.int32), ir.astype(np.int32))
        else:
            table = job.tables[0]
            sub = table.take(rows_used)
            ocols = [orc.StrCol(sub[c].tolist()) for c in COLS]
            ref = orc.template_gammas(SPECS, ocols, ocols, inv[:len(sl)].astype(np.int32),
                                      inv[len(sl):].astype(np.int32))
        gam = job.gammas_host()
        bad = int((gam[idx] != ref).any(axis=1).sum())
        row["parity_gamma"] = {"sampled_pairs": int(len(idx)), "stride": int(step), "mismatches": bad}
        hist_o, mp_o = orc.em_iterate(gam, nlev, lam0, [m for m, _ in lp0], [u for _, u in lp0], a.iters, 1e-300)
        lam_o, m_o, u_o = hist_o[-1]
        rel = lambda x, y: abs(x - y) <= 1e-9 * max(abs(x), abs(y), 1e-300)  # noqa: E731
        ok = rel(params.params["λ"], lam_o) and all(
            rel(x, y) for k, (m, u) in enumerate(params._level_probabilities())
            for x, y in zip(list(m) + list(u), list(m_o[k]) + list(u_o[k])))
        mp_dev = job.score(params.params["λ"], params._level_probabilities())
        mp_ok = bool(np.allclose(mp_dev, mp_o, rtol=1e-9, atol=0, equal_nan=True))
        row["parity_em"] = {"iterations": len(hist_o), "lambda_m_u_1e-9": bool(ok), "match_probability_1e-9": mp_ok,
                            "pairs": int(P)}
        if link:
            tf_mp = job.ctx.tf_copy(0, job.n_pairs)
            row["parity_tf"] = tf_parity(job, l, r, mp_dev, params.params["λ"], tf_mp)
        row["parity_check_s"] = time.perf_counter() - t
    out = json.dumps(row)
    print(out, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out + "\n")


def tf_parity(job, l, r, mp, lam, tf_mp):
    """term_frequencies.py:49-117 restated with numpy over host-factorised surname values (not the
    device's dictionary ids): per value v, adj_lambda = mean mp over pairs with surname_l = surname_r
    = v (NULL mp excluded from sum and count), adj = bayes(adj_lambda, 1 - λ), 0.5 without a lookup,
    tf_adjusted_match_prob = bayes(mp, adj)."""
    import pandas as pd
    vl = job.tables[0]["surname"]
    vr = job.r_table()["surname"]
    codes, uniq = pd.factorize(pd.concat([vl, vr], ignore_index=True), use_na_sentinel=True)
    cl, cr = codes[:len(vl)], codes[len(vl):]
    a, b = cl[l], cr[r]
    ok = (a >= 0) & (a == b)
    good = ok & ~np.isnan(mp)
    n_v = len(uniq)
    s = np.bincount(a[good], weights=mp[good], minlength=n_v)
    c = np.bincount(a[good], minlength=n_v)
    one_minus = float(repr(1 - lam))
    with np.errstate(invalid="ignore", divide="ignore"):
        adj_lambda = np.where(c > 0, s / np.maximum(c, 1), np.nan)
        tnum = adj_lambda * one_minus
        tden = tnum + (1 - adj_lambda) * (1 - one_minus)
        tab = np.where(tden == 0, np.nan, tnum / tden)
        adj = np.full(len(mp), 0.5)
        look = tab[np.where(ok, a, 0)]
        sel = ok & ~np.isnan(look)
        adj[sel] = look[sel]
        num = mp * adj
        den = num + (1 - mp) * (1 - adj)
        want = np.where(den == 0, np.nan, num / den)
    same = np.isclose(tf_mp, want, rtol=1e-9, atol=0, equal_nan=True)
    return {"pairs": int(len(mp)), "pairs_with_equal_surname": int(ok.sum()), "tf_adjusted_match_prob_1e-9": bool(same.all()),
            "mismatches": int((~same).sum())}


if __name__ == "__main__":
    main()
