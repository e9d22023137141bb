"""bench.py --gpus N outside a launcher starts N ranks itself (torch.distributed.run on
127.0.0.1) and reports the world size the process group saw; checked on the CPU with
the gloo self-test mode (no GPU is touched)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=180, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout       # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_launcher_two_ranks():
    r = _run("--gpus", "2", "--launcher-selftest", "--steps", "3")
    assert r["n_gpus"] == 2 and r["steps"] == 3 and r["value"] > 0


def test_launcher_one_rank_in_process():
    r = _run("--gpus", "1", "--launcher-selftest", "--steps", "2")
    assert r["n_gpus"] == 1
