"""CPU: ``bench.py --gpus N`` launches N ranks itself (torch.distributed.run as a child process) when it
is not already one rank of a distributed launch, and rank 0 reports the world it ran in.  The
--selftest workload runs the same launcher, rank environment, flat bucketed all-reduce and
max-over-ranks timing over gloo on a small CPU model (no GPU here)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--selftest", "--steps", "2", "--warmup", "1",
                        "--batch", "8", *extra], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE line
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    res = _run("--gpus", "2")
    assert res["n_gpus"] == 2
    assert res["config"]["parallelism"] == "dp2"
    assert res["config"]["buckets"] >= 2
    assert res["grads_identical_across_ranks"]


def test_bench_default_is_one_rank():
    res = _run()
    assert res["n_gpus"] == 1
