"""One process per GPU: the rank launcher behind ``bench.py --gpus N``.

The reference's only multi-GPU path is ``nn.DataParallel`` (train_cond.py:66-68, one thread per
GPU in one process).  Here every GPU gets its own process, as ``torch.distributed.run`` would
start them: the parent never touches the GPU (``torch.cuda.device_count()`` does not initialise
HIP on this image), starts N fresh children with RANK / LOCAL_RANK / WORLD_SIZE /
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

__all__ = ["free_port", "rank_env", "spawn_ranks", "visible_gpus"]


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    """GPUs this process could use, counted without initialising HIP."""
    import torch
    return torch.cuda.device_count()


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
