"""bench.py --gpus N starts N ranks itself when no launcher set WORLD_SIZE (the driver's 8-GPU
SCALE run must measure N GPUs, never one process on GPU 0). CPU: the measurement protocol's
dry run over gloo (barrier, timed region, max over ranks, one JSON line from rank 0)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--dist-dry-run", "--steps", "3", "--warmup", "1", "--batch", "8"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    # and nothing else on stdout (the process-group libraries' own lines go to stderr)
    assert r.stdout.strip().splitlines() == lines, r.stdout
    return json.loads(lines[0])


def test_bench_gpus_2_launches_two_ranks():
    line = _run(2)
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 16


def test_bench_gpus_3_launches_three_ranks():
    line = _run(3)
    assert line["n_gpus"] == 3 and line["config"]["parallelism"] == "dp3"
