"""bench.py's own multi-rank launcher: `bench.py --gpus N` without torch.distributed.run starts N
rank processes itself, before any HIP call, and prints rank 0's one JSON line with n_gpus = N; a failing rank makes
the whole run fail (and ends its siblings); a --gpus value that disagrees with an outer launcher's WORLD_SIZE is
refused. Checked on the CPU with the launcher's gloo-only stub ranks (the same Dist set-up, barriers and
max-over-ranks as a real run, no GPU call)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=timeout)


def test_gpus2_self_launch_prints_one_line_with_two_ranks():
    r = _run(["--gpus", "2", "--stub"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["max_rank"] == 1.0


def test_failing_rank_fails_the_run():
    r = _run(["--gpus", "2", "--stub", "--stub-fail-rank", "1"])
    assert r.returncode != 0
    assert "rank(s) failed" in r.stderr


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "3", "--stub"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_ranks_sharing_one_gpu_are_refused():
    """two ranks that see the same physical GPU (a one-GPU box) are refused, not labelled as two
    GPUs."""
    r = _run(["--gpus", "2", "--stub", "--stub-devices", "0000:05:00.0"])
    assert r.returncode != 0
    assert "distinct GPU" in r.stderr and "--allow-shared" in r.stderr


def test_ranks_sharing_one_gpu_labelled_with_allow_shared():
    r = _run(["--gpus", "2", "--stub", "--stub-devices", "0000:05:00.0", "--allow-shared"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert d["n_gpus"] == 1 and d["n_ranks"] == 2 and d["shared_gpu"] is True


def test_distinct_gpus_count_as_gpus():
    r = _run(["--gpus", "2", "--stub", "--stub-devices", "0000:05:00.0,0000:15:00.0"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert d["n_gpus"] == 2 and d["shared_gpu"] is False
