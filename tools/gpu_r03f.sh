#!/bin/bash
# r03 session f: persistent convq — parity, per-layer probe (persist on / off), gen64 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03f; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_convq.py tests/test_gpu_timed_shapes.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for p in 1 0; do
  FFC_CONVQ_PERSIST=$p timeout -k 10 200 python tools/convq_probe.py 256 gen64 > $o/probe_p$p.log 2>&1 || { echo "probe rc=$?"; tail $o/probe_p$p.log; exit 1; }
  echo "== persist $p"; grep -v amdgpu.ids $o/probe_p$p.log | sed -e 's/\[[^]]*\]//g'
  FFC_CONVQ_PERSIST=$p timeout -k 10 200 python tools/convq_probe.py 32 gen64 > $o/probe32_p$p.log 2>&1 || { echo "probe rc=$?"; tail $o/probe32_p$p.log; exit 1; }
  grep -v amdgpu.ids $o/probe32_p$p.log | sed -e 's/\[[^]]*\]//g'
  FFC_CONVQ_PERSIST=$p timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $o/bench_p$p.log 2>&1 || { echo "bench rc=$?"; tail $o/bench_p$p.log; exit 1; }
  grep '^{' $o/bench_p$p.log | cut -c150-330
done
