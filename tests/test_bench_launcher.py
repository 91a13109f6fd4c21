"""bench.py --gpus N without a launcher spawns N ranks itself (torch.distributed.run, rendezvous on
127.0.0.1), each checks WORLD_SIZE == --gpus, and timings are reduced max-over-ranks: exercised on
the CPU with gloo at world 2 (the GPU work of each rank is not run here)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launcher-selftest", *extra],
                          capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)


def test_gpus_2_spawns_two_ranks():
    p = _run("--gpus", "2")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["max_over_ranks"] == 1.0


def test_world_size_mismatch_is_refused():
    p = _run("--gpus", "2", env={"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr
