"""bench.py's launch contract on the CPU: `--gpus N` without a launcher must
run N rank processes (or fail) -- never report N GPUs from one process."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus2_without_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--spawn-probe"])
    assert r.returncode == 0, r.stderr
    ranks = sorted((json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")), key=lambda d: d["rank"])
    assert [(d["rank"], d["local_rank"], d["world"]) for d in ranks] == [(0, 0, 2), (1, 1, 2)]


def test_launcher_world_size_wins():
    r = _run(["--gpus", "8", "--spawn-probe"], {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1"})
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines == [{"rank": 0, "local_rank": 0, "world": 1}]  # one process runs, one rank is reported
    assert "running 1 rank" in r.stderr


def test_failing_rank_fails_the_job():
    # rank processes that cannot start (a bogus backend on a CPU box) must surface a non-zero status
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--channels", "1", "--ir", "64", "--backend", "nonexistent",
              "--no-cpu-baseline", "--pmc", "off"])
    assert r.returncode != 0
    assert not any(l.startswith("{") for l in r.stdout.splitlines())
