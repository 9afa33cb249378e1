"""bench.py --gpus N starts N ranks by construction (CPU, no GPU needed).

The driver runs `python bench.py --gpus N` for its scaling curve; round 5's bench.py parsed --gpus and ignored it, so
such a run measured one process on GPU 0.  These tests run the real bench.py with its --launcher-selftest hook: every
rank reports the rank variables torch.distributed.run gave it and exits before any GPU call, and the parent reports
whether it initialised HIP (it must not: the children own the GPUs).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env_without_ranks():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def _json_lines(text):
    out = []
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            out.append(json.loads(line))
    return out


def test_bench_gpus_n_launches_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launcher-selftest"], capture_output=True, text=True,
                       timeout=300, env=_env_without_ranks(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    ranks = sorted((d for d in recs if "rank" in d), key=lambda d: d["rank"])
    assert [d["rank"] for d in ranks] == [0, 1, 2]
    assert [d["local_rank"] for d in ranks] == [0, 1, 2]
    assert all(d["world_size"] == 3 for d in ranks)
    assert not any(d["hip_initialized"] for d in ranks)
    parent = [d["launcher"] for d in recs if "launcher" in d]
    assert parent == [{"gpus": 3, "rc": 0, "parent_hip_initialized": False}]


def test_bench_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--launcher-selftest"], capture_output=True, text=True, timeout=120,
                       env=_env_without_ranks(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _json_lines(r.stdout)
    assert recs == [{"rank": 0, "local_rank": 0, "world_size": 1, "hip_initialized": False}]


def test_bench_rejects_a_world_that_is_not_gpus():
    env = _env_without_ranks()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launcher-selftest"], capture_output=True, text=True,
                       timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr
