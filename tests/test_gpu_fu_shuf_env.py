"""The fused FU's cross-lane column DFTs (FFC_FU_SHUF=1, fft_common.h lane_fft_dif / lane_ifft_dit;
off by default: DESIGN.md §4f) run in a child process with the switch on: the golden FU / generator
cases, the gen64 timed shapes against the fp64 oracle, and the FU repeat / fold tests."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lane_column_dfts_in_subprocess():
    env = dict(os.environ, FFC_FU_SHUF="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py"),
                        os.path.join(ROOT, "tests", "test_gpu_timed_shapes.py"),
                        os.path.join(ROOT, "tests", "test_gpu_bn_fold.py"),
                        "-k", "golden or gen64 or fu_repeat or fold_and_spill"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout.splitlines()[-1], tail
