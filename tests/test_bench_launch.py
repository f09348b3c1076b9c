"""bench.py's rank launch on the CPU: `--gpus N` without a launcher starts N ranks itself (a
child torch.distributed.run) and the record reports the world the ranks saw; a launcher world
that disagrees with --gpus is an error.  `--launch-check` stops before any GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


def test_gpus_2_without_launcher_runs_two_ranks():
    p = _run(["--gpus", "2", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_seen"] == 2 and rec["ranks_reported"] == 2 and rec["rank_sum"] == 1


def test_world_size_mismatch_is_an_error():
    p = _run(["--gpus", "2", "--launch-check"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr
