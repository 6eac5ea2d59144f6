#!/bin/bash
# r03 session a: HIP capture-mode probe, launcher + RCCL capture tests, gen64 bench baseline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
o=gpurun_out/r03a
timeout -k 10 60 ./tools/capture_mode_probe > $o/capture_mode_probe.json 2>&1; echo "probe rc=$?"; cat $o/capture_mode_probe.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_launch.py tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread > $o/tests_launch_rccl.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests_launch_rccl.log; exit 1; }
tail -3 $o/tests_launch_rccl.log
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --cpu-seconds 5 > $o/bench_gen64.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_gen64.log; exit 1; }
grep '^{' $o/bench_gen64.log | cut -c1-600
