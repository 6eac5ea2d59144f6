#!/bin/bash
# r03 session k: convq staging without issue-time waits: parity (Q=2 default, Q=3 variant), probes, trace, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03k; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_convq.py tests/test_gpu_timed_shapes.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd_q3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_convq.py -x -q --timeout 120 --timeout-method thread > $o/tests_q3.log 2>&1 || { echo "tests q3 rc=$?"; tail -30 $o/tests_q3.log; exit 1; }
tail -1 $o/tests_q3.log
for v in "" _q3; do
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd$v.so timeout -k 10 200 python tools/convq_probe.py 256 gen64 > $o/probe$v.log 2>&1 || { echo "probe rc=$?"; tail $o/probe$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $o/probe$v.log | sed -e 's/\[[^]]*\]//g'
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd$v.so timeout -k 10 200 python tools/convq_probe.py 512 fgan128 > $o/probe_f$v.log 2>&1 || { echo "probe rc=$?"; tail $o/probe_f$v.log; exit 1; }
  grep -v amdgpu.ids $o/probe_f$v.log | sed -e 's/\[[^]]*\]//g' | cut -c1-60
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $o/bench$v.log 2>&1 || { echo "bench rc=$?"; tail $o/bench$v.log; exit 1; }
  grep '^{' $o/bench$v.log | cut -c150-330
done
cd tools
export FFC_LIB_PATH=$PWD/../fastfourierconvolution_amd/libffc_amd_traceq.so
for a in "0 256 2 gen64" "1 256 0 gen64" "2 256 0 gen64"; do
  timeout -k 10 120 python trace_convq.py $a >> ../$o/trace.log 2>&1 || { echo "trace $a rc=$?"; tail ../$o/trace.log; exit 1; }
done
grep -v amdgpu.ids ../$o/trace.log
