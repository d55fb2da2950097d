"""One rank of tests/test_gpu_parity.py::test_sharded_ranks_match_single_process (run as a child process).

Every rank uses cuda:0 with the gloo backend, so the sharded device path -- spk_block with
shard=(rank, world), per-rank comparison vectors, the histogram all-reduce between
spk_em_histogram and spk_em_finalize -- runs on a one-GPU box exactly as bench.py runs it per GPU.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from splink_amd.engine import Job, m_step_rows  # noqa: E402
from splink_amd.params import Params  # noqa: E402
from splink_amd.session import AmdSession  # noqa: E402
from splink_amd.synthetic import cfg_settings, make_records  # noqa: E402

COLS = ["first_name", "surname", "dob", "city", "email"]
ITERS = 5


def records():
    # Arrow-backed string columns: a sharded rank uploads its slice of each and all-gathers the rest
    return make_records(20000, seed=23, surname_vocab=500, first_vocab=300, city_vocab=80,
                        arrow=True)[["unique_id"] + COLS]


def run(shard, want_job=False):
    df = records()
    params = Params(cfg_settings(2, max_iterations=ITERS), AmdSession(0))
    st = params.settings
    job = Job("dedupe_only", [df], "unique_id", 0, shard=shard)
    job.block(st["blocking_rules"])
    job.gammas(st)
    names, nlev = job.code_meta
    initial = (params.params["λ"], params._level_probabilities())
    for _ in range(ITERS):
        stats = job.em_stats(params.params["λ"], params._level_probabilities())
        lam, rows = m_step_rows(stats, names, nlev)
        params._update_params(lam, rows)
    out = {"n_pairs": int(job.n_pairs), "lambda": params.params["λ"],
           "pi": [[list(m), list(u)] for m, u in params._level_probabilities()],
           "replicated_ingest": bool(job.replicate_ingest), "table_digest": int(job.ctx.table_digest(0))}
    if want_job:
        return out, job, initial, nlev
    return out


def run_link_tf():
    """The link_tf golden (link_only, 3 OR'd rules, tf on surname) through the public API on this
    rank's shard of the pairs: EM histogram and tf (Σmp, count) tables all-reduced over the ranks."""
    import copy
    import pandas as pd
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conftest import load_golden
    from splink_amd import Splink
    g = load_golden("link_tf")
    linker = Splink(copy.deepcopy(g["settings_in"]), AmdSession(0), df_l=pd.DataFrame(g["df_l"]),
                    df_r=pd.DataFrame(g["df_r"]))
    df_e = linker.get_scored_comparisons()
    tf = linker.make_term_frequency_adjustments(df_e)
    conv = lambda d: {c: [None if (isinstance(v, float) and v != v) else (v.item() if hasattr(v, "item") else v)  # noqa: E731
                          for v in d[c].tolist()] for c in d.columns}
    return {"df_e": conv(df_e.toPandas()), "df_e_columns": list(df_e.toPandas().columns),
            "df_tf": conv(tf.toPandas()), "df_tf_columns": list(tf.toPandas().columns),
            "lambda": linker.params.params["λ"], "n_pairs": df_e.count()}


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    out = run_link_tf() if len(sys.argv) > 2 and sys.argv[2] == "link_tf" else run((rank, world))
    with open(f"{sys.argv[1]}.{rank}", "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
