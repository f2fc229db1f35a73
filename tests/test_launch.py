"""`python bench.py --gpus N` as its own launcher (benchlib/launch.py), rehearsed on the CPU
with gloo and bench's stub step (`--workload launch_probe`): N ranks, each with its own
RANK / LOCAL_RANK and the right world size, one result line from rank 0, a failing rank
fails the job, and a launcher's WORLD_SIZE that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

import pytest

from benchlib.launch import WorldMismatch, needs_spawn, resolve_world

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run_bench(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], env=env, capture_output=True, text=True,
                          timeout=timeout, cwd="/tmp")


@pytest.mark.parametrize("n", [2, 8])
def test_gpus_flag_spawns_ranks(n):
    r = run_bench(["--workload", "launch_probe", "--gpus", str(n), "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints, the parent prints nothing
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n
    ranks = rec["ranks"]
    assert [x["rank"] for x in ranks] == list(range(n))
    assert [x["local_rank"] for x in ranks] == list(range(n))
    assert all(x["env_world_size"] == n and x["group_world_size"] == n for x in ranks)
    assert len({x["pid"] for x in ranks}) == n  # one process per rank
    # bench's timed_loop: every rank reports the same MAX over ranks
    assert len({x["elapsed_s"] for x in ranks}) == 1
    assert rec["elapsed_s"] >= 3 * 0.002 * n


def test_failing_rank_fails_the_job():
    r = run_bench(["--workload", "launch_probe", "--gpus", "3", "--steps", "2", "--warmup", "0",
                   "--probe-fail-rank", "1"], env_extra={"SAS_LAUNCH_GRACE_S": "1"}, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip() == ""  # rank 0 never got past the rendezvous: no line


def test_world_size_mismatch_refused():
    r = run_bench(["--workload", "launch_probe", "--gpus", "4"],
                  env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE is 2" in r.stderr


def test_resolve_world():
    assert resolve_world(None, {}) == (1, 0, 0)
    assert resolve_world(4, {}) == (4, 0, 0)
    assert needs_spawn(4, {}) and not needs_spawn(1, {}) and not needs_spawn(None, {})
    env = {"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}
    assert not needs_spawn(8, env)
    assert resolve_world(8, env) == (8, 5, 5)
    assert resolve_world(None, env) == (8, 5, 5)  # no --gpus: the launcher's world
    with pytest.raises(WorldMismatch):
        resolve_world(2, env)
    with pytest.raises(WorldMismatch):
        resolve_world(None, {"WORLD_SIZE": "2", "RANK": "2"})
