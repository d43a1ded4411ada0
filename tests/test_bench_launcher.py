"""bench.py --gpus N launches N ranks by itself (VERDICT r2 "Next round" item 2).

Without WORLD_SIZE in the environment, `bench.py --gpus N` starts N fresh child
processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set)
before torch or libmz is imported, and rank 0 prints the one JSON line.  The
`--launcher-selftest` mode makes the ranks join a gloo group and all-reduce
their rank ids on the CPU (no GPU call), so the launcher runs here."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_gpus2_self_launch_gloo():
    r = _run(["--gpus", "2", "--launcher-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                   # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["rank_sum"] == 3.0   # ranks 0 and 1 joined one group
    assert d["pid"] != os.getpid()


def test_gpus1_runs_in_process():
    r = _run(["--gpus", "1", "--launcher-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--launcher-selftest"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
