"""One process per GPU: the rank launcher behind ``bench.py --gpus N``.

The reference's only multi-GPU path is ``nn.DataParallel`` (train_cond.py:66-68, one thread per
GPU in one process).  Here every GPU gets its own process, as ``torch.distributed.run`` would
start them: the parent never touches the GPU (``visible_gpus`` reads the KFD topology from
sysfs, no HIP call; tests/test_gpu_launch.py checks /dev/kfd stays closed), starts N fresh children with RANK / LOCAL_RANK / WORLD_SIZE /
LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, waits for all of them and exits with the first
failing child's status (the others are terminated by PID).  No exec of the parent, so nothing
replaces a process that has initialised the GPU.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

__all__ = ["free_port", "kfd_gpus", "rank_env", "spawn_ranks", "visible_gpus"]


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _visible_filter(n: int, var: str) -> int:
    """Apply one ``*_VISIBLE_DEVICES`` list to ``n`` enumerated devices: unset keeps all, an
    empty string hides all, otherwise the entries that name a device (an index < n, or a
    ``GPU-<uuid>`` ROCr accepts) up to the first invalid one, as the runtimes parse it."""
    v = os.environ.get(var)
    if v is None:
        return n
    k = 0
    for tok in (t.strip() for t in v.split(",")):
        if tok.startswith("GPU-") and var == "ROCR_VISIBLE_DEVICES":
            k += 1
        elif tok.isdigit() and int(tok) < n:
            k += 1
        else:
            break
    return min(k, n)


def kfd_gpus(nodes_dir: str = KFD_NODES) -> int:
    """GPU agents in the KFD topology (nodes with a non-zero ``gpu_id``) whose render node this
    process may open -- what ROCr will enumerate -- read from sysfs only."""
    try:
        names = os.listdir(nodes_dir)
    except OSError:
        return 0
    n = 0
    for name in names:
        d = os.path.join(nodes_dir, name)
        try:
            with open(os.path.join(d, "gpu_id")) as f:
                if int(f.read().strip() or "0") == 0:
                    continue                     # CPU node
            minor = None
            with open(os.path.join(d, "properties")) as f:
                for line in f:
                    key, _, val = line.partition(" ")
                    if key == "drm_render_minor":
                        minor = int(val)
        except (OSError, ValueError):
            continue
        if minor is not None and minor > 0 and not os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
            continue                             # present on the host, not granted to this process
        n += 1
    return n


def visible_gpus(nodes_dir: str = KFD_NODES) -> int:
    """GPUs this process could use, counted WITHOUT any HIP / HSA call (so a parent that spawns
    the ranks never opens /dev/kfd: ``torch.cuda.device_count()`` falls back to hipGetDeviceCount
    when amdsmi discovery fails).  KFD topology, then ROCR_VISIBLE_DEVICES (ROCr), then ONE of the
    HIP runtime's lists: HIP_VISIBLE_DEVICES when it is non-empty, else CUDA_VISIBLE_DEVICES when
    that is non-empty (HIP reads the second only in place of the first, an empty value counting
    as unset), as the ROCm stack applies them."""
    n = _visible_filter(kfd_gpus(nodes_dir), "ROCR_VISIBLE_DEVICES")
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if os.environ.get(var):
            return _visible_filter(n, var)
    return n


def rank_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    # dmabuf IPC only on this pool's driver (RCCL / tensor sharing across processes)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(script: str, argv: list[str], nproc: int, port: int | None = None,
                poll_s: float = 0.05) -> int:
    """Run ``python script *argv`` as ranks 0..nproc-1 of one job; return the job's exit status
    (0 when every rank exited 0, else the first non-zero status seen)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = free_port() if port is None else port
    procs = [subprocess.Popen([sys.executable, script, *argv], env=rank_env(r, nproc, port))
             for r in range(nproc)]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:          # one rank failed: the others would block in a collective
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc if rc >= 0 else 128 - rc      # killed by signal s -> 128 + s, as a shell reports it
