"""bench.py's own multi-rank launch: `bench.py --gpus N`
without a launcher must start N ranks itself, before any GPU call, and rank 0
must print ONE aggregated line with n_gpus = N. Checked on the CPU with the
--selftest stand-in step under gloo (the GPU step is covered by the driver's
SCALE run); the default (N = 1) command is unchanged."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=240, cwd=ROOT)


def test_gpus_2_spawns_two_ranks_and_one_line():
    r = _run("--gpus", "2", "--selftest", "--steps", "3", "--warmup", "1", "--batch", "256")
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout                  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_size_seen"] == 2
    assert res["config"]["global_batch"] == 512 and res["config"]["parallelism"] == "dp2"
    assert res["steps"] == 3
    assert res["checks"] == {"partition": True, "allreduce": True, "status_or": True}, res["checks"]


def test_c4_partition_world_8():
    """C4 (BASELINE configs[3]: 8 ranks x 256 crops) rehearsed on the CPU: the
    launcher starts 8 gloo ranks, each draws its 256 crops from seed 1234 +
    rank, the GradBuckets exchange over the LSTM 512/512 ParamStore layout
    leaves every rank the sum of all 8 gradients (Adam's scale 1/8), the status
    word is OR-reduced, and rank 0 prints one line with the max-over-ranks time."""
    r = _run("--gpus", "8", "--selftest", "--steps", "2", "--warmup", "1", "--batch", "256")
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 8 and res["world_size_seen"] == 8
    assert res["config"]["global_batch"] == 2048 and res["config"]["parallelism"] == "dp8"
    assert res["checks"] == {"partition": True, "allreduce": True, "status_or": True}, res["checks"]
    assert res["grad_values"] > 10_000_000                  # the whole LSTM 512/512 flat gradient


def test_single_rank_default_is_unchanged():
    r = _run("--selftest", "--steps", "2", "--warmup", "0")
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout.strip())
    assert res["n_gpus"] == 1 and res["world_size_seen"] == 1


def test_failing_rank_fails_the_job():
    """A rank that dies makes the launcher stop the others and exit non-zero
    (a bad flag makes every child's argparse exit 2)."""
    r = _run("--gpus", "2", "--selftest", "--steps", "notanint")
    assert r.returncode != 0
