"""Benchmark: candidate pairs scored per second (comparison vectors + E + M per EM iteration).

Workload (BASELINE.json configs[1]): synthetic person records, dedupe, blocking
`l.surname = r.surname` OR `l.dob = r.dob`, five comparison columns (first_name / surname
Jaro-Winkler-3, dob / city exact-2, email Levenshtein-3).  At N GPUs the job is one global
dedupe of 1M x sqrt(N) records (~46M x N candidate pairs), pairs sharded by ordinal across
ranks (weak scaling: ~46M pairs per GPU), one RCCL all-reduce of the comparison-pattern
histogram per EM iteration.

One timed step = the comparison-vector pass over every pair resident in HBM (spk_gammas) +
one E+M iteration (one GPU: spk_em_iteration_start / _wait, a single launch; N GPUs:
spk_em_histogram -> RCCL all-reduce -> spk_em_finalize) + the host M-step (Params update).  On one
GPU the loop is software-pipelined: pass i is queued before the host M-step of iteration i - 1.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--records R] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
warnings.filterwarnings("ignore")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md "Chip-level parameters")
# HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this same command
# (scripts_gpu_round.sh -> tools/traffic.py); the counters cannot be read inside a timed run.
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r6_traffic.json")
# per-kernel issue counters of the same command (rocprofv3 --pmc passes, tools/pmc_summary.py)
PMC_FILE = os.path.join(ROOT, "profiles", "r6_pmc_kernels.json")
PMC_FILE_CFG5 = os.path.join(ROOT, "profiles", "r6_cfg5_lev_pmc.json")  # tools/gpu/pmc_cfg5_lev.sh
COLS = ["first_name", "surname", "dob", "city", "email"]
WORKLOADS = {2: "cfg2: synthetic person-record dedupe, 1M x sqrt(N) records, blocking surname|dob, "
                "5 comparison columns (JW-3 x2, exact-2 x2, Levenshtein-3)",
             4: "cfg4: synthetic person-record dedupe of 20M records (fixed: strong scaling), blocking surname|dob "
                "(~6.2e9 candidate pairs, BASELINE.md cfg4 note), 5 comparison columns (JW-3 x2, exact-2 x2, "
                "Levenshtein-3), pair ordinals sharded over the ranks",
             5: "cfg5 columns at cfg2 size: synthetic person-record dedupe, 1M x sqrt(N) records, blocking "
                "surname|dob, 6 comparison columns (JW-3 x2, exact-2 x2, Levenshtein-3, free-text address "
                "30-128 chars Levenshtein-4)"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_LINE_FD = 1


def emit(line: dict):
    """The one JSON line of the run, on the process's original stdout."""
    sys.stdout.flush()
    os.write(_LINE_FD, (json.dumps(line) + "\n").encode())


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` without a launcher's WORLD_SIZE: start N fresh rank processes of this script, one
    per GPU (RANK = LOCAL_RANK = g, WORLD_SIZE = N, rendezvous on 127.0.0.1), and return the first non-zero
    exit code, else 0.  This process never imports torch or touches a GPU (the ranks are children, not an
    exec of it); rank 0 writes the JSON line to the inherited stdout.  A rank that fails ends the others
    (they would wait in a collective for it)."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for g in range(n):
        env = dict(os.environ, RANK=str(g), LOCAL_RANK=str(g), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      start_new_session=True))
    code = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    log(f"bench.py: rank {procs.index(p)} exited with {rc}; ending the other ranks")
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    return code


GAMMA_STREAMS = 2  # --gamma-streams
GAMMA_GRAPH = False  # --gamma-graph


def timed_run(config, records, shard, world, rank, local, steps, warmup):
    """Build one workload's job (records, blocking, first comparison pass) and time `steps` steps after
    `warmup` untimed ones, bracketed by a barrier + device synchronisation; the wall time is the maximum
    over ranks.  Returns the job and what the line reports about it."""
    import torch
    from splink_amd import distributed as D
    from splink_amd.engine import Job, m_step_rows
    from splink_amd.params import Params
    from splink_amd.session import AmdSession
    from splink_amd.synthetic import cfg_settings, make_records
    t0 = time.time()
    cols = COLS + (["address"] if config == 5 else [])
    if config == 4:
        # the job's size does not grow with N: its ordinal space is split over the ranks (strong scaling)
        from splink_amd.synthetic import make_records_parallel
        n_records = 20_000_000
        df = make_records_parallel(n_records, 16, 16, surname_vocab=300_000)[["unique_id"] + cols]
    else:
        n_records = int(round(records * math.sqrt(world)))
        # Arrow-backed string columns: the columnar form a Spark / Arrow source hands over (values identical
        # to the object-column records; spk_raw_utf8 takes their buffers without a per-row pass)
        df = make_records(n_records, surname_vocab=15000, with_address=config == 5, arrow=True)[["unique_id"] + cols]
    log(f"[rank {rank}] generated {n_records} records in {time.time() - t0:.1f}s")

    settings = cfg_settings(config, max_iterations=10)
    params = Params(settings, AmdSession(local))
    st = params.settings

    job = Job("dedupe_only", [df], "unique_id", local, shard=shard)
    job.ctx.enable_timing(True)
    job.ctx.gammas_set_streams(GAMMA_STREAMS)
    job.ctx.gammas_set_graph(GAMMA_GRAPH)
    t0 = time.time()
    job.block(st["blocking_rules"])
    block_s = time.time() - t0
    block_kernel_ms = job.ctx.kernel_ms()["block"]
    log(f"[rank {rank}] blocking: {job.n_pairs} local pairs of {job.n_candidates} candidates "
        f"({block_s:.2f}s wall incl. host key prep, {block_kernel_ms:.1f} ms device)")
    t0 = time.time()
    job.gammas(st)  # uploads columns (device decode through the clustering permutation), first launch
    first_gammas_s = time.time() - t0
    names, nlev = job.code_meta

    host = {"gammas_call": [], "em_wait": [], "m_step_host": [], "em_start": []}
    dev = {"gamma": [], "em_hist": [], "em_final": []}
    pending = [False]

    def finish_m_step():
        """Statistics of the enqueued E+M iteration, then the host M-step (Params update)."""
        t0 = time.perf_counter()
        stats = job.em_wait()
        t1 = time.perf_counter()
        lam, rows = m_step_rows(stats, names, nlev)
        params._update_params(lam, rows)
        t2 = time.perf_counter()
        host["em_wait"].append((t1 - t0) * 1e3)
        host["m_step_host"].append((t2 - t1) * 1e3)
        pending[0] = False
        ms = job.ctx.kernel_ms_done()  # the newest completed launches (the next comparison pass may be running)
        for k in dev:
            dev[k].append(ms[k])

    def step():
        """Comparison pass i, then E+M iteration i.  Software-pipelined: pass i is queued before the host
        finishes the M-step of iteration i - 1 (pass i does not depend on it; E+M i does), so the device
        never waits for the host.  The order of device work and its results are those of the plain loop."""
        t0 = time.perf_counter()
        job.gammas(st)
        t1 = time.perf_counter()
        if pending[0]:
            finish_m_step()
        t2 = time.perf_counter()
        job.em_start(params.params["λ"], params._level_probabilities())
        pending[0] = True
        t3 = time.perf_counter()
        host["gammas_call"].append((t1 - t0) * 1e3)
        host["em_start"].append((t3 - t2) * 1e3)

    def barrier():
        torch.cuda.synchronize()
        D.barrier()
        torch.cuda.synchronize()

    for _ in range(warmup):
        step()
    if pending[0]:
        finish_m_step()
    for v in list(host.values()) + list(dev.values()):
        v.clear()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    finish_m_step()  # the last iteration's M-step is part of the timed work
    barrier()
    elapsed = time.perf_counter() - t0
    # per-launch device times of the timed steps (HIP events on the context stream, read as each
    # launch completed)
    gamma_ms = dev["gamma"]
    hist_ms = dev["em_hist"]
    fin_ms = [max(x, 0.0) for x in dev["em_final"]]  # one GPU: the E-step runs inside the histogram launch
    local_pairs = job.n_pairs
    elapsed = D.max_over_ranks(elapsed)
    total_pairs = D.sum_over_ranks(local_pairs)
    ms_per_step = elapsed * 1000.0 / steps

    return argparse.Namespace(job=job, df=df, params=params, st=st, cols=cols, names=names, nlev=nlev,
                              n_records=n_records, gamma_ms=gamma_ms, hist_ms=hist_ms, fin_ms=fin_ms, host=host,
                              local_pairs=local_pairs, total_pairs=total_pairs, ms_per_step=ms_per_step,
                              block_s=block_s, block_kernel_ms=block_kernel_ms, first_gammas_s=first_gammas_s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment this script starts them itself")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend: nccl (= RCCL) for the benchmark; gloo rehearses N ranks on the CPU "
                         "(--dry-run) or on fewer GPUs (ranks share devices round-robin, exchange host-staged)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rendezvous only: every rank joins the group and the all-reduce that counts "
                         "them, rank 0 prints the line without running the workload (no GPU needed with gloo)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--records", type=int, default=1_000_000, help="records at N=1 (scaled by sqrt(N))")
    ap.add_argument("--config", type=int, default=2, choices=[2, 4, 5],
                    help="2: the headline workload; 4: BASELINE configs[3], a 20M-record dedupe sharded over the "
                         "ranks (strong scaling); 5: + free-text address Levenshtein-4 (cfg5's columns at cfg2's size)")
    ap.add_argument("--share", type=str, default=None,
                    help="k/n: run rank k's share of an n-rank job on this one GPU (e.g. --config 4 --share 0/8)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cfg5-steps", type=int, default=10,
                    help="the cfg5_columns sub-record of a one-GPU cfg2 run: steps timed (0 = off)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--gamma-graph", action="store_true",
                    help="replay unchanged comparison passes from a captured HIP graph (measured slower; A/B only)")
    ap.add_argument("--gamma-streams", type=int, default=2, choices=[1, 2],
                    help="comparison pass as two concurrent half windows on two streams (2, default) or one (1)")
    ap.add_argument("--em-scale", type=int, default=8,
                    help="separate E/M streaming row: the run's comparison vectors tiled this many times (0 = off)")
    args = ap.parse_args()
    global GAMMA_STREAMS
    GAMMA_STREAMS = args.gamma_streams
    global GAMMA_GRAPH
    GAMMA_GRAPH = args.gamma_graph

    if "WORLD_SIZE" not in os.environ:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            log(f"bench.py: --gpus {n}: need at least one rank")
            sys.exit(2)
        if n > 1:
            sys.exit(launch_ranks(n, sys.argv[1:]))  # this process only waits for its ranks
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            log(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # stdout carries only rank 0's JSON line: whatever the libraries print there (gloo's connection notes,
    # RCCL / HIP diagnostics) goes to stderr
    global _LINE_FD
    _LINE_FD = os.dup(1)
    os.dup2(2, 1)
    import torch
    n_dev = torch.cuda.device_count()
    if args.backend == "nccl" and n_dev < world:
        # RCCL runs one rank per GPU; refuse instead of benching fewer GPUs under a larger label
        log(f"bench.py: --gpus {world} needs {world} visible GPUs, {n_dev} visible")
        sys.exit(3)
    if n_dev == 0 and not args.dry_run:
        log("bench.py: no GPU visible (the workload runs on the GPU; --dry-run --backend gloo rehearses the launch)")
        sys.exit(3)
    dev = local % n_dev if n_dev else -1  # gloo rehearsal: ranks share the visible devices round-robin
    if dev >= 0:
        torch.cuda.set_device(dev)
    ranks_seen = 1
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
            one = torch.ones(1, dtype=torch.int64, device=f"cuda:{dev}")
        else:
            dist.init_process_group("gloo")
            one = torch.ones(1, dtype=torch.int64)
        dist.all_reduce(one)
        ranks_seen = int(one.item())
        assert ranks_seen == dist.get_world_size() == world, (ranks_seen, world)
    if args.dry_run:
        if rank == 0:
            emit({"metric": "candidate pairs scored/sec (gammas+E+M per iter)", "value": None,
                  "unit": "pairs/s", "n_gpus": world, "ranks_seen": ranks_seen, "backend": args.backend,
                  "devices_visible": n_dev, "dry_run": True})
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    local = dev

    shard = (rank, world)
    if args.share:
        k, n = (int(x) for x in args.share.split("/"))
        assert world == 1 and 0 <= k < n, "--share runs one rank's share on one GPU"
        shard = (k, n)
    R = timed_run(args.config, args.records, shard, world, rank, local, args.steps, args.warmup)
    job, df, params, st, cols, names, nlev = R.job, R.df, R.params, R.st, R.cols, R.names, R.nlev
    n_records, gamma_ms, hist_ms, fin_ms, host = R.n_records, R.gamma_ms, R.hist_ms, R.fin_ms, R.host
    local_pairs, total_pairs, ms_per_step = R.local_pairs, R.total_pairs, R.ms_per_step
    block_s, block_kernel_ms, first_gammas_s = R.block_s, R.block_kernel_ms, R.first_gammas_s

    # ---- full job (blocking excluded from the metric): score pass for the record
    t0 = time.perf_counter()
    job.score(params.params["λ"], params._level_probabilities(), want_host=False)
    torch.cuda.synchronize()
    score_ms = job.ctx.kernel_ms()["score"]

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- roofline of the dominant kernel (comparison-vector pass) -------------------------
    # SURVEY §8(d) algorithmic bytes: 8 + K bytes per pair (read the int32 pair, write the γ vector)
    # plus every record's field bytes once (UTF-8).  The pass writes a packed 2-byte code instead of
    # K bytes of γ; both figures are reported.
    from splink_amd.table import arrow_utf8
    K = len(cols)
    code_bytes = 2 if job.ctx.n_patterns() <= 65536 else 4
    g_ms = float(np.mean(gamma_ms))
    h_ms = float(np.mean(hist_ms))
    f_ms = float(np.mean(fin_ms))
    rec_bytes = int(sum(arrow_utf8(df[c])[0][-1] for c in cols))
    gamma_bytes = local_pairs * (8 + K) + rec_bytes
    gamma_bytes_packed = local_pairs * (8 + code_bytes) + rec_bytes
    roofline = {"bound": "hbm", "kernel": "spk_gammas pass (k_filter + list compaction + the exact passes of the undecided cells)",
                "achieved": gamma_bytes / (g_ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gamma_bytes / (g_ms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                "algorithmic_bytes_per_launch": gamma_bytes,
                "algorithmic_bytes_note": f"SURVEY 8(d): pairs x (8 + K={K}) + UTF-8 field bytes {rec_bytes}",
                "bytes_per_launch_packed_codes": gamma_bytes_packed, "avg_launch_ms": g_ms,
                "note": "comparison pass is VALU / gather-latency bound (string work), not HBM-bound; its HBM fraction is shown per the contract"}
    # E/M: the kernel streams each pair's packed code once per iteration (code_bytes per pair, an exact
    # re-encoding of the K-byte γ vector SURVEY 8(d) counts); frac is on those streamed bytes over the
    # whole E+M iteration's device time (one launch on one GPU: histogram + E-step + M-step sums).
    em_ms = h_ms + f_ms
    em_bytes = local_pairs * code_bytes
    em_roofline = {"bound": "hbm", "kernel": "k_em_iter (histogram + E-step + M-step sums, one launch)",
                   "avg_launch_ms": em_ms, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "algorithmic_bytes_per_launch": em_bytes, "bytes_per_pair": code_bytes,
                   "achieved": em_bytes / (em_ms / 1e3) / 1e9, "frac": em_bytes / (em_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                   "code_compression": {"contract_bytes_per_pair": K, "streamed_bytes_per_pair": code_bytes,
                                        "factor": K / code_bytes},
                   "note": "frac on the bytes the kernel streams (the packed code); the code packs SURVEY 8(d)'s "
                           "K bytes of gamma per pair into code_bytes (code_compression)"}
    # SURVEY 8(d)'s whole-EM figure (10 iterations + the final scoring pass) on streamed bytes
    t_em = 10 * em_ms / 1e3 + score_ms / 1e3
    headline = {"formula": "(P*cb*iters + P*(cb+8)) / t_EM / 8e12, cb = code bytes streamed, iters=10, "
                           "t_EM = 10*E+M iteration + k_score",
                "value": (local_pairs * code_bytes * 10 + local_pairs * (code_bytes + 8)) / t_em / 8e12,
                "t_em_ms": t_em * 1e3}

    traffic = None
    if os.path.exists(TRAFFIC_FILE):
        with open(TRAFFIC_FILE) as f:
            traffic = json.load(f)
        roofline["traffic"] = traffic["gamma"]["traffic_bytes_per_call"]
        em_roofline["traffic"] = traffic["em"]["traffic_bytes_per_call"]
        roofline["traffic_source"] = em_roofline["traffic_source"] = (
            os.path.relpath(TRAFFIC_FILE, ROOT) + ": rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this command")

    issue = issue_counters(args.config)

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(job, df, st, args.cpu_seconds, cols)

    # (cfg4: billions of pairs per GPU -- already the scale of the E/M row, and too many to copy to the host)
    rates = string_rates(job, st, local_pairs, g_ms) if (world == 1 and args.config != 4) else None

    em_scale = None
    if world == 1 and args.em_scale > 0 and args.config != 4:
        em_scale = em_streaming(job, names, nlev, params, args.em_scale)

    out = {
        "metric": "candidate pairs scored/sec (gammas+E+M per iter)",
        "value": total_pairs / (ms_per_step / 1e3),
        "unit": "pairs/s",
        "n_gpus": world,
        "ranks_seen": ranks_seen,
        "backend": args.backend if world > 1 else None,
        "devices_used": min(world, n_dev),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.config == 4 else "weak",
        "vs_baseline": None,
        "dtype": "fp64",
        "data": "synthetic",
        "config": {"workload": WORKLOADS[args.config],
                   "records": n_records, "candidate_pairs": total_pairs, "comparison_columns": len(cols),
                   "candidate_ordinals_total": job.n_candidates, "shard": list(shard),
                   "comparison_windows": job.ctx.gammas_windows(),
                   "parallelism": f"pair-ordinal shards x{world}, " + (
                       "RCCL all-reduce of pattern histogram" if args.backend == "nccl" or world == 1 else
                       "gloo all-reduce of pattern histogram (host-staged rehearsal, ranks sharing GPUs)")},
        "roofline": roofline,
        "roofline_em": em_roofline,
        "issue_gamma_kernels": issue,
        "hbm_headline_contract": headline,
        "breakdown_ms": {"gamma": g_ms, "em_hist": h_ms, "em_final": f_ms, "score": score_ms,
                         "block_device": block_kernel_ms, "block_wall": block_s * 1e3,
                         "block_keys_wall": job.timings.get("block_keys_s", 0.0) * 1e3,
                         "first_gammas_call_incl_column_decode": first_gammas_s * 1e3,
                         **{f"host_wall_{k}": float(np.mean(v)) for k, v in host.items()}},
        "device_lds_per_block": job.ctx.lds_per_block(),
        "input": "Arrow-backed string columns (pd.ArrowDtype(large_string)); keys, ids, ranks, clustering on the device",
        "deferred_pairs": job.ctx.gammas_deferred(),
        "exact_cells_per_column": dict(zip(names, job.ctx.gammas_exact_counts(len(names)))),
        # pairs whose level the blocking key implies (the filter reads nothing for that column there)
        "implied_pairs_per_column": dict(zip(names, job.ctx.gammas_implied_pairs(len(names)))),
        "cpu_baseline": cpu,
        "string_rates": rates,
        "em_at_scale": em_scale,
    }
    if world == 1 and args.config == 2 and args.cfg5_steps > 0 and not args.share:
        # cfg5's columns in the same run, after the headline (never the headline): the free-text address
        # column's Levenshtein passes are the other workload the comparison kernels are tuned on
        del job, R
        out["cfg5_columns"] = cfg5_record(args, local)
    emit(out)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def issue_counters(config):
    """The γ kernels are issue-bound, not HBM-bound: their VALU / SALU issue against the SIMD peaks and the
    share of wave time stalled, from the committed counter passes of this config's bench command."""
    pmc_file = PMC_FILE_CFG5 if config == 5 else PMC_FILE
    if not os.path.exists(pmc_file):
        return None
    with open(pmc_file) as f:
        pmc = json.load(f)
    issue = {"source": os.path.relpath(pmc_file, ROOT) + ": rocprofv3 --pmc SQ_* passes of this config's "
             "comparison pass", "peak_note": "valu_util = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x kernel cycles "
             "at 2.4 GHz); kernels that ran under 10 us per launch (near-empty lists) are left out"}
    for name, key in (("filter", "k_filter"), ("levenshtein_exact", "k_gamma_exact_simple<1,"),
                      ("levenshtein_refill", "k_lev_refill"), ("levenshtein_slow", "k_gamma_slow_lev"),
                      ("bag_compaction", "k_compact_lev"), ("jw_exact", "k_gamma_exact_simple<2,")):
        for k, v in pmc.items():
            if key in k and float(v.get("_dur_ns", 0.0)) >= 10000.0:
                issue[name] = {x: round(float(v[x]), 4) for x in ("valu_util", "salu_util", "wait_frac", "l2_hit",
                                                                   "_dur_ns") if x in v}
                break
    return issue


def exact_pass_ms(job, st, names):
    """Each column's exact-pass launch time from one extra, untimed comparison pass on one stream with per-launch
    events (kept out of the timed loop: the events cost host time per launch, and under the two-stream split a
    column's two launches overlap)."""
    job.ctx.enable_timing(True, exact=True)
    job.ctx.gammas_set_streams(1)
    try:
        job.gammas(st)
        return job.ctx.gammas_exact_ms(len(names))
    finally:
        job.ctx.gammas_set_streams(GAMMA_STREAMS)
        job.ctx.enable_timing(True)


def cfg5_record(args, local):
    """`bench.py --config 5` at one GPU, timed in the default run after the cfg2 headline: step time, the γ
    pass and its per-column exact passes, E+M, and the committed counters of its Levenshtein kernels."""
    R = timed_run(5, args.records, (0, 1), 1, 0, local, args.cfg5_steps, min(args.warmup, 3))
    job, names = R.job, R.names
    g_ms = float(np.mean(R.gamma_ms))
    em_ms = float(np.mean(R.hist_ms)) + float(np.mean(R.fin_ms))
    xms = exact_pass_ms(job, R.st, names)
    return {"workload": WORKLOADS[5], "records": R.n_records, "candidate_pairs": R.total_pairs,
            "steps": args.cfg5_steps, "warmup": min(args.warmup, 3), "ms_per_step": R.ms_per_step,
            "value": R.total_pairs / (R.ms_per_step / 1e3), "unit": "pairs/s",
            "breakdown_ms": {"gamma": g_ms, "em": em_ms,
                             "exact_pass_per_column": {n: float(x) for n, x in zip(names, xms) if x > 0}},
            "exact_cells_per_column": dict(zip(names, [int(x) for x in job.ctx.gammas_exact_counts(len(names))])),
            "issue_gamma_kernels": issue_counters(5)}


def em_streaming(job, names, nlev, params, reps, iters=10):
    """Separate labelled row (never the headline): the E/M kernels at a per-GPU pair count where
    launch ramp and fixed costs no longer dominate -- the run's own comparison vectors tiled `reps`
    times (cfg4 puts ~125-250M pairs on each GPU, cfg5 ~1.25B).  Reports k_hist (2 B/pair) and the
    final scoring pass k_score (2 + 8 B/pair) against HBM peak, the per-iteration re-streaming EM
    rate, and the O(#patterns) finalize alone (the iteration-invariant 'pattern-count' EM cost)."""
    g = job.gammas_host()
    big = np.tile(g, (reps, 1))
    del g
    job.load_gammas(names, nlev, big)
    P = big.shape[0]
    del big
    cb = 2 if job.ctx.n_patterns() <= 65536 else 4
    lam, lp = params.params["λ"], params._level_probabilities()
    for _ in range(2):
        job.em_stats(lam, lp)
    hist, fin = [], []
    for _ in range(iters):
        job.em_stats(lam, lp)
        ms = job.ctx.kernel_ms()
        hist.append(ms["em_hist"])
        fin.append(max(ms["em_final"], 0.0))
    sc = []
    for _ in range(3):
        job.score(lam, lp, want_host=False)
        sc.append(job.ctx.kernel_ms()["score"])
    h, f, s = float(np.median(hist)), float(np.median(fin)), float(np.median(sc[1:]))
    h = h + f  # the whole E+M iteration (one launch on one GPU)
    hb, sb = P * cb, P * (cb + 8)
    return {"pairs": P, "source": f"the run's comparison vectors tiled x{reps}",
            "em_iteration": {"bound": "hbm", "kernel": "k_em_iter", "avg_launch_ms": h, "algorithmic_bytes_per_launch": hb,
                             "achieved": hb / (h / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": hb / (h / 1e3) / 1e9 / HBM_PEAK_GBS},
            "k_score": {"bound": "hbm", "avg_launch_ms": s, "algorithmic_bytes_per_launch": sb,
                        "achieved": sb / (s / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": sb / (s / 1e3) / 1e9 / HBM_PEAK_GBS},
            "em_restream_pairs_per_s": P / (h / 1e3)}


def lev_scan_cells(a: str, b: str, cut: int) -> int:
    """DP cells the exact pass's bit-parallel scan updates for one listed cell of rows <= 64 units (a host
    restatement of spk_strsim.h lev_rows_planes_np / myers_plane_text[_lazy]): common prefix and suffix
    stripped, the longer remainder is the pattern (m rows) and the scan runs over the shorter one (n text
    units), one word-step per text unit of 32 rows (m <= 32; the lazy scan also up to its switch unit
    J0 = 31 - cut, taken per cell here, per wave in the kernel) or 64 rows, stopping after the first
    fourth unit j whose bound D[m][j + 1] - (n - 1 - j) exceeds cut.  Equal strings (decided before any
    scan) and a side that strips to empty count 0."""
    la, lb = len(a), len(b)
    mn = min(la, lb)
    pre = 0
    while pre < mn and a[pre] == b[pre]:
        pre += 1
    suf = 0
    while suf < mn - pre and a[la - 1 - suf] == b[lb - 1 - suf]:
        suf += 1
    ra, rb = a[pre:la - suf], b[pre:lb - suf]
    if not ra or not rb:
        return 0
    pat, txt = (ra, rb) if len(ra) >= len(rb) else (rb, ra)
    m, n = len(pat), len(txt)
    wide = m > 32
    j0 = (31 - cut if cut < 31 else 0) if wide else n
    col = list(range(m + 1))  # D[i][0]
    cells = 0
    for j in range(n):
        cells += 64 if (wide and j >= j0) else 32
        prev, col[0] = col[0], j + 1
        for i in range(1, m + 1):
            cur = min(col[i] + 1, col[i - 1] + 1, prev + (pat[i - 1] != txt[j]))
            prev, col[i] = col[i], cur
        if (j & 3) == 3 and col[m] - (n - 1 - j) > cut:
            break
    return cells


def string_rates(job, st, pairs, g_ms):
    """Rates of the string work in the last γ pass (Levenshtein GCUPS, JW comparisons/s).

    Levenshtein GCUPS counts DP cells of the cells the exact pass evaluated, over that launch's own
    HIP-event time: Σ over the column's exact list of len_l · len_r (code points, before the common
    prefix / suffix strip and the early exit, so the cells a full DP of those strings would update)
    ÷ k_gamma_exact_simple<true>'s time.  Pairs the filter settled from bounds are not counted as
    cells; they appear in `comparisons_per_s` (all pairs x columns over the whole γ pass)."""
    l, r = job.pair_rows()
    t = job.tables[0]
    sec = g_ms / 1e3
    names = [c["col_name"] for c in st["comparison_columns"]]
    exact = job.ctx.gammas_exact_counts(len(names))
    xms = exact_pass_ms(job, st, names)
    lev, n_jw, n_lev = {}, 0, 0
    rng = np.random.Generator(np.random.PCG64(7))
    for k, c in enumerate(st["comparison_columns"]):
        expr = (c.get("case_expression") or "").lower()
        if "levenshtein" in expr:
            n_lev += 1
            vals = t[c["col_name"]]
            ln = vals.str.len().fillna(0).to_numpy(np.int64)
            items = job.ctx.gammas_exact_list(k, int(exact[k]))
            # -1 slots (k_compact_lev): decided by their character-bag distance, or sent straight to the slow pass
            n_bag = int((items < 0).sum())
            items = items[items >= 0]
            nominal = int(np.dot(ln[l[items]], ln[r[items]]))
            # cells the scans actually update, from a host restatement of the scan over a random sample of
            # the listed cells (rows <= 64 units: the exact pass's own; longer rows go to the 128-bit pass)
            thr = [float(x) for x in re.findall(r"<=\s*([0-9.]+)", expr)] or [0.0]
            sample = rng.choice(len(items), size=min(2000, len(items)), replace=False) if len(items) else []
            tot = cnt = 0
            for i in sample:
                a, b = vals.iat[int(l[items[i]])], vals.iat[int(r[items[i]])]
                if not isinstance(a, str) or not isinstance(b, str) or max(len(a), len(b)) > 64:
                    continue
                # simple_lev_cut: one unit over the largest passing distance (ratio tests: t x mean length)
                ratio = "length(" in expr
                cut = max(int(np.floor(x * (len(a) + len(b)) / 2.0 if ratio else x)) + 1 for x in thr)
                tot += lev_scan_cells(a, b, cut)
                cnt += 1
            scanned = tot / cnt * len(items) if cnt else None
            sec_x = xms[k] / 1e3 if xms[k] > 0 else None
            lev[c["col_name"]] = {"exact_cells": int(exact[k]), "cells_compacted_out": n_bag, "exact_pass_ms": xms[k],
                                  "dp_cells_nominal": nominal,
                                  "gcups_nominal": nominal / sec_x / 1e9 if sec_x else None,
                                  "dp_cells_scanned_est": scanned,
                                  "gcups_scanned": scanned / sec_x / 1e9 if (sec_x and scanned) else None,
                                  "scan_sample": {"cells": int(cnt), "rows_le_64_units_of": int(len(sample))},
                                  "exact_cells_per_s": exact[k] / sec_x if sec_x else None}
        elif "jaro_winkler" in expr:
            n_jw += 1
    K = len(st["comparison_columns"])
    return {"comparisons_per_s": pairs * K / sec, "jw_comparisons_per_s": pairs * n_jw / sec,
            "lev_comparisons_per_s": pairs * n_lev / sec, "levenshtein_exact_pass": lev,
            "note": "comparisons/s: all pairs x columns over the whole γ pass; levenshtein_exact_pass: "
                    "gcups_scanned = DP cells the bit-parallel scans update (word-steps x word width after the "
                    "prefix / suffix strip and the early exit, bench.lev_scan_cells over a 2000-cell sample, "
                    "extrapolated to the list) over that launch's HIP-event time; gcups_nominal = len_l x len_r "
                    "of the same cells (the work a full DP would do)"}


def cpu_baseline(job, df, st, seconds, col_names):
    """The CPU oracle (C/OpenMP restatement) on a bounded sample of the same pairs: γ + E + M."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    n_max = min(job.n_pairs, 50_000_000)
    l, r = job.ctx.pairs_copy(0, n_max)  # a prefix of the pairs is all the sample needs
    t = job.tables[0]  # pair rows index the job's (blocking-key clustered) table
    cols = [orc.StrCol(t[c].tolist()) for c in col_names]
    specs = [("jw", 3, [0.94, 0.88]), ("jw", 3, [0.94, 0.88]), ("eq", 2, []), ("eq", 2, []), ("lev", 3, [0.3]),
             ("lev", 4, [0.2, 0.4])][:len(col_names)]
    lp = [(c["m_probabilities"], c["u_probabilities"]) for c in st["comparison_columns"]]
    nlev = [c["num_levels"] for c in st["comparison_columns"]]
    n = min(len(l), 200_000)
    while True:
        t0 = time.perf_counter()
        g = orc.template_gammas(specs, cols, cols, l[:n], r[:n])
        orc.em_stats(g, nlev, 0.01, [m for m, _ in lp], [u for _, u in lp])
        dt = time.perf_counter() - t0
        if dt >= seconds / 3 or n >= len(l):
            break
        n = min(len(l), int(n * max(2.0, seconds / 2 / max(dt, 1e-3))))
    return {"value": n / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"first {n} of the same candidate pairs, gammas ({len(col_names)} template columns) + one E+M pass, "
                      f"oracle/splink_oracle.c OpenMP ({dt:.1f}s)"}


if __name__ == "__main__":
    main()
