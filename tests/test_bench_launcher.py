"""bench.py's multi-rank plumbing on CPU: `--gpus N` starts N rank processes itself (gloo process
group here), the timed region is the max over ranks, rank 0 prints one JSON line with n_gpus = N;
a world size that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, env=e, timeout=300)


def test_launcher_two_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--launcher-check"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dist"]["world_size"] == 2 and d["dist"]["launcher"] == "bench.py --gpus"
    assert d["ms_per_step"] >= 20.0  # the max over ranks (rank 1 sleeps 20 ms)


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--launcher-check"], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
