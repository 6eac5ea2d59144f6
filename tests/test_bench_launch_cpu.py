"""bench.py's N-GPU launch and shard plan, on the CPU over gloo.

`python bench.py --gpus N` starts N ranks itself (fastfourierconvolution_amd/launch.py) when no
launcher set WORLD_SIZE; `--dry-run` runs the launch and the batch plan without a GPU.  These
tests check that N ranks really start, that strong scaling splits the BASELINE global batches
(256 / 512 / 1024) and weak scaling (the default) keeps the configuration's batch per GPU, and that
a GPU count that cannot be honoured is an error rather than a silent one-GPU line.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _bench(*argv, env=None, timeout=180):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    e.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run([sys.executable, BENCH, *argv], capture_output=True, text=True, env=e, timeout=timeout,
                          cwd=ROOT)


def _line(res):
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout       # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("workload,n,per", [("gen64", 2, [128, 128]), ("fgan128", 2, [256, 256]),
                                            ("fgan128sn", 4, [256] * 4), ("gen64", 3, [86, 85, 85])])
def test_strong_scaling_plan(workload, n, per):
    line = _line(_bench("--gpus", str(n), "--dry-run", "--workload", workload, "--scaling", "strong"))
    assert line["n_gpus"] == n and line["scaling"] == "strong"
    assert line["global_batch"] == {"gen64": 256, "fgan128": 512, "fgan128sn": 1024}[workload]
    assert line["per_gpu_batch"] == per and line["tiles_global_batch"]
    assert line["parallelism"] == f"dp{n}+syncbn"


def test_weak_scaling_plan():
    line = _line(_bench("--gpus", "2", "--dry-run", "--scaling", "weak", "--workload", "fgan128", "--batch", "64"))
    assert line["global_batch"] == 128 and line["per_gpu_batch"] == [64, 64]


@pytest.mark.parametrize("workload,gb", [("gen64", 256), ("fgan128", 512), ("fgan128sn", 1024)])
def test_strong_scaling_is_default(workload, gb):
    """the default N-GPU line splits the configuration's batch over the GPUs (BASELINE configs[3]/[4]:
    "batch 512 / 1024 sharded across 8xMI355X")"""
    line = _line(_bench("--gpus", "2", "--dry-run", "--workload", workload))
    assert line["scaling"] == "strong" and line["per_gpu_batch"] == [gb // 2, gb // 2] and line["global_batch"] == gb
    assert line["tiles_global_batch"]


def test_single_rank_plan():
    line = _line(_bench("--dry-run"))
    assert line["n_gpus"] == 1 and line["global_batch"] == 256 and line["parallelism"] == "dp1"


def test_more_gpus_than_visible_fails():
    res = _bench("--gpus", "2", env={"ROCR_VISIBLE_DEVICES": ""})
    if res.returncode == 0:
        pytest.fail("bench.py --gpus 2 with no visible GPU must not succeed")
    assert res.returncode == 3 and "visible" in res.stderr


def test_launcher_world_mismatch_fails():
    res = _bench("--gpus", "4", "--dry-run", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert res.returncode == 3 and "WORLD_SIZE=2" in res.stderr


def test_spawn_ranks_env_and_failure(tmp_path):
    """every rank sees its own RANK / LOCAL_RANK and the shared WORLD_SIZE / MASTER_*; one failing
    rank fails the job and the others are stopped"""
    sys.path.insert(0, ROOT)
    from fastfourierconvolution_amd.launch import spawn_ranks
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        out = sys.argv[1]
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        open(os.path.join(out, "r" + os.environ["RANK"]), "w").write(" ".join(os.environ[k] for k in keys))
        if len(sys.argv) > 2 and os.environ["RANK"] == sys.argv[2]:
            sys.exit(7)
        if len(sys.argv) > 2:
            time.sleep(60)      # a healthy rank stuck waiting: the launcher must stop it
    """))
    assert spawn_ranks(str(script), [str(tmp_path)], 3) == 0
    rows = sorted((tmp_path / f"r{r}").read_text().split() for r in range(3))
    assert [r[:4] for r in rows] == [[str(r), str(r), "3", "3"] for r in range(3)]
    assert {r[4] for r in rows} == {"127.0.0.1"} and len({r[5] for r in rows}) == 1
    import time
    t0 = time.time()
    assert spawn_ranks(str(script), [str(tmp_path), "1"], 3) == 7
    assert time.time() - t0 < 30
