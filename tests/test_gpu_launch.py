"""bench.py --gpus N's parent process on a real GPU box: it counts GPUs without any HIP call and
refuses a GPU count it cannot honour.

The parent spawns the rank processes as fresh children; it must not have opened /dev/kfd (a HIP /
HSA initialisation) before it does.  ``launch.visible_gpus`` reads the KFD topology in sysfs;
this test runs it in a subprocess that has also imported torch and bench.py, and looks at that
process's open file descriptors.  The count must equal what HIP itself reports (a separate
process calls torch.cuda.device_count()).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import os, sys
sys.path.insert(0, %r)
import torch
import bench                                   # what the launching parent imports
from fastfourierconvolution_amd.launch import visible_gpus
n = visible_gpus()
fds = []
for fd in os.listdir('/proc/self/fd'):
    try:
        fds.append(os.readlink('/proc/self/fd/' + fd))
    except OSError:
        pass
print(n, int(any(f.startswith('/dev/kfd') for f in fds)), int(any(f.startswith('/dev/dri') for f in fds)))
"""


def test_visible_gpus_is_hip_free_and_matches_hip():
    r = subprocess.run([sys.executable, "-c", PROBE % ROOT], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    n, kfd, dri = (int(v) for v in r.stdout.split()[-3:])
    assert kfd == 0 and dri == 0, "counting GPUs opened the GPU driver"
    h = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=300)
    assert h.returncode == 0, h.stderr[-2000:]
    assert n == int(h.stdout.split()[-1]) >= 1


def test_bench_refuses_more_gpus_than_visible():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    h = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=300)
    n = int(h.stdout.split()[-1]) + 1
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 3 and "visible" in r.stderr, (r.returncode, r.stderr[-2000:])
