"""bench.py's rank launcher on the CPU (no GPU): `python bench.py --gpus N` without a launcher's WORLD_SIZE
starts N rank processes itself (bench.launch_ranks), each joins the process group and rank 0 prints the
line.  --dry-run --backend gloo stops after the rendezvous and the all-reduce that counts the ranks, so the
launch path the driver's 1/2/4/8-GPU runs take is exercised here without the workload."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [x for x in out.splitlines() if x.strip()]
    assert len(lines) == 1, out  # stdout is the JSON line alone (gloo's own notes go to stderr)
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_gloo_ranks(n):
    r = _run(["--gpus", str(n), "--backend", "gloo", "--dry-run"])
    assert r.returncode == 0, r.stderr
    line = _line(r.stdout)
    assert line["n_gpus"] == n and line["ranks_seen"] == n and line["backend"] == "gloo" and line["dry_run"]


def test_one_rank_needs_no_launcher():
    r = _run(["--gpus", "1", "--backend", "gloo", "--dry-run"])
    assert r.returncode == 0, r.stderr
    line = _line(r.stdout)
    assert line["n_gpus"] == 1 and line["ranks_seen"] == 1


def test_nccl_refuses_more_ranks_than_gpus():
    # this container has no GPU: RCCL ranks cannot start, and the launcher exits non-zero naming the count
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode != 0
    assert "needs 2 visible GPUs, 0 visible" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--backend", "gloo", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
