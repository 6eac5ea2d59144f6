"""The N > 1 launch path's two host-side rules, on the CPU (no GPU, no HIP call).

* ``launch.visible_gpus`` counts GPUs from the KFD topology in sysfs and the *_VISIBLE_DEVICES
  filters, so ``bench.py --gpus N``'s parent never initialises HIP before it spawns the ranks
  (on the GPU box tests/test_gpu_launch.py checks /dev/kfd stays closed).
* ``graphs.capture_step`` agrees on graph vs eager across ranks BEFORE any replay: one rank
  failing its capture makes every rank fall back to eager (bench.py capture), over a
  world-size-2 gloo group with the failure forced on rank 1.
"""
from __future__ import annotations

import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from fastfourierconvolution_amd import launch  # noqa: E402


def _fake_topology(root, gpus, cpus=1):
    """sysfs KFD nodes: `cpus` CPU agents (gpu_id 0) then GPU agents with render minors that do
    not exist in /dev/dri here (minor 0 = not checked)"""
    i = 0
    for _ in range(cpus):
        d = root / str(i)
        d.mkdir()
        (d / "gpu_id").write_text("0\n")
        (d / "properties").write_text("cpu_cores_count 8\nsimd_count 0\ndrm_render_minor 0\n")
        i += 1
    for g in range(gpus):
        d = root / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{1000 + g}\n")
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\ndrm_render_minor 0\n")
        i += 1
    return str(root)


@pytest.mark.parametrize("env,want", [({}, 8), ({"HIP_VISIBLE_DEVICES": "0,1"}, 2),
                                      # HIP reads CUDA_VISIBLE_DEVICES only when HIP_VISIBLE_DEVICES is
                                      # unset or empty; the two lists are never combined
                                      ({"HIP_VISIBLE_DEVICES": ""}, 8),
                                      ({"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7", "CUDA_VISIBLE_DEVICES": "0"}, 8),
                                      ({"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "0,1"}, 2),
                                      ({"ROCR_VISIBLE_DEVICES": ""}, 0),
                                      ({"ROCR_VISIBLE_DEVICES": "3"}, 1),
                                      ({"ROCR_VISIBLE_DEVICES": "0,1,2", "HIP_VISIBLE_DEVICES": "1,2"}, 2),
                                      ({"CUDA_VISIBLE_DEVICES": "0,9"}, 1),
                                      ({"ROCR_VISIBLE_DEVICES": "GPU-0123456789abcdef,1"}, 2)])
def test_visible_gpus_from_sysfs(tmp_path, monkeypatch, env, want):
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    nodes = _fake_topology(tmp_path, 8, cpus=2)
    assert launch.kfd_gpus(nodes) == 8
    assert launch.visible_gpus(nodes) == want


def test_visible_gpus_skips_unopenable_render_node(tmp_path, monkeypatch):
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    nodes = _fake_topology(tmp_path, 2)
    (tmp_path / "1" / "properties").write_text("simd_count 1024\ndrm_render_minor 250\n")   # no /dev/dri here
    assert launch.visible_gpus(nodes) == 1


def test_visible_gpus_no_kfd(tmp_path):
    assert launch.visible_gpus(str(tmp_path / "absent")) == 0


def test_visible_gpus_does_not_import_hip_modules():
    """the count never reaches torch.cuda (whose device_count may call hipGetDeviceCount)"""
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); import torch; torch.cuda.device_count = None; "
            "from fastfourierconvolution_amd.launch import visible_gpus; print(visible_gpus())" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert int(r.stdout.strip()) >= 0


# --------------------------------------------------------------------------- capture agreement
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _w_capture(rank, port, fail_rank, out_dir):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    os.environ["RANK"] = str(rank)
    if fail_rank is not None:
        os.environ["FFC_FAIL_CAPTURE_RANK"] = str(fail_rank)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    from fastfourierconvolution_amd.graphs import capture_step
    replays = []

    class FakeGraph:
        def replay(self):
            replays.append(1)

    calls = []
    g = capture_step(lambda: calls.append(1), capture=lambda step: FakeGraph())
    # after the vote, the ranks run the same number of "collectives": one all-reduce per step
    run = g.replay if g is not None else (lambda: calls.append(1))
    x = torch.ones(1)
    for _ in range(3):
        run()
        dist.all_reduce(x)
    with open(os.path.join(out_dir, f"r{rank}"), "w") as f:
        f.write(f"{int(g is not None)} {len(replays)} {float(x)}")
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [None, 1, 0])
def test_capture_agreement_before_replay(tmp_path, fail_rank):
    mp.spawn(_w_capture, args=(_free_port(), fail_rank, str(tmp_path)), nprocs=2, join=True)
    got = [(tmp_path / f"r{r}").read_text().split() for r in range(2)]
    want_graph = "1" if fail_rank is None else "0"
    for graph, nrep, x in got:
        assert graph == want_graph                    # every rank made the same choice
        assert nrep == ("3" if fail_rank is None else "0")   # nobody replayed a graph another rank lacks
        assert float(x) == 8.0                        # 3 matched all-reduces: 1 -> 2 -> 4 -> 8
