"""Host-side sanitizer runs of the C ABI (race detection / sanitizers).

GPU AddressSanitizer is not available on this pool, so the sanitizers cover the host code:
every csrc/ source is compiled host-only (hipcc --offload-new-driver --cuda-host-only: no device code, fast) with
  * AddressSanitizer + UndefinedBehaviorSanitizer, and
  * ThreadSanitizer,
linked with tests/native/abi_sanitize.cpp, and run.  The driver hits every entry point's argument
validation, sweeps the shape queries over extreme sizes, and fails calls from 8 threads at once
to check that ffc_last_error() is thread-local.  Any sanitizer report fails the test
(halt_on_error / exitcode).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fastfourierconvolution_amd", "csrc")
DRIVER = os.path.join(ROOT, "tests", "native", "abi_sanitize.cpp")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
SAN = {
    "asan": ["-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}
ENV = {
    "asan": {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1:abort_on_error=0:exitcode=86",
             "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=87"},
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1:exitcode=88"},
}


def _host_flags(kind):
    out = []
    for f in SAN[kind]:
        out += ["-Xarch_host", f]
    return out


def _build(kind, out_dir):
    # the new offload driver lets a host-only object (no device image) link on its own
    common = ["-O1", "-g", "-std=c++17", "--offload-arch=gfx950", "--offload-new-driver", "--cuda-host-only",
              "-fno-gpu-sanitize",
              "-fno-omit-frame-pointer", *_host_flags(kind)]
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))

    def comp(src):
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        r = subprocess.run([HIPCC, *common, "-x", "hip", "-c", src, "-o", obj], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        return obj
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(comp, srcs))
    drv = os.path.join(out_dir, "driver.o")
    r = subprocess.run([HIPCC, "-O1", "-g", "-std=c++17", *SAN[kind], "-c", DRIVER, "-o", drv],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    exe = os.path.join(out_dir, "abi_sanitize")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "--offload-new-driver", "--hip-link", "-fno-gpu-sanitize",
                        *SAN[kind], "-pthread", drv, *objs, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_abi_under_sanitizer(kind, tmp_path):
    exe = _build(kind, str(tmp_path))
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    env.update(ENV[kind])
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "checks ok" in r.stdout
