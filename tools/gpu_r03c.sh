#!/bin/bash
# r03 session c: convq staging slots A/B (2 = default lib, 3, 4): parity, per-layer probe, gen64 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03c; mkdir -p $o
export TMPDIR=/tmp
for v in q3 q4; do
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_convq.py -x -q --timeout 120 --timeout-method thread > $o/tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -30 $o/tests_$v.log; exit 1; }
  tail -1 $o/tests_$v.log
done
for v in "" _q3 _q4; do
  lib=$PWD/fastfourierconvolution_amd/libffc_amd$v.so
  FFC_LIB_PATH=$lib timeout -k 10 300 python tools/convq_probe.py 256 gen64 > $o/probe_gen64$v.log 2>&1 || { echo "probe rc=$?"; tail $o/probe_gen64$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $o/probe_gen64$v.log
  FFC_LIB_PATH=$lib timeout -k 10 300 python tools/convq_probe.py 512 fgan128 > $o/probe_fgan128$v.log 2>&1 || { echo "probe rc=$?"; tail $o/probe_fgan128$v.log; exit 1; }
  grep -v amdgpu.ids $o/probe_fgan128$v.log
  FFC_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $o/bench_gen64$v.log 2>&1 || { echo "bench rc=$?"; tail $o/bench_gen64$v.log; exit 1; }
  grep '^{' $o/bench_gen64$v.log | cut -c150-330
done
