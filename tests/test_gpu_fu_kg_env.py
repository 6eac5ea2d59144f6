"""The fused FU's bin-group pass 0 (FFC_FU_KGROUPS=2, off by default: DESIGN.md §4f) run in a child
process with the switch on: tests/test_gpu_bn_fold.py's bin-group cases (against one workgroup per
sample, and bitwise repeats) and the gen64 timed shapes against the fp64 oracle."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bin_groups_in_subprocess():
    env = dict(os.environ, FFC_FU_KGROUPS="2")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_bn_fold.py"),
                        os.path.join(ROOT, "tests", "test_gpu_timed_shapes.py"),
                        "-k", "bin_group or gen64_strong or gen64_train"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "skipped" not in r.stdout.splitlines()[-1] or " passed" in r.stdout.splitlines()[-1], tail
