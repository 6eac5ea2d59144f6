#!/bin/bash
# r03 session j: per-section cycle trace of persistent convq (diagnostic build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03j; mkdir -p $o
export FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd_traceq.so
cd tools
for a in "0 256 2 gen64" "1 256 0 gen64" "2 256 0 gen64" "4 64 0 fgan128" "1 64 0 fgan128"; do
  timeout -k 10 120 python trace_convq.py $a >> ../$o/trace.log 2>&1 || { echo "trace $a rc=$?"; tail ../$o/trace.log; exit 1; }
done
grep -v amdgpu.ids ../$o/trace.log
cd ..
unset FFC_LIB_PATH
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timed_shapes.py -x -q --timeout 120 --timeout-method thread -k "fba or block or golden" > $o/tests_block.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests_block.log; exit 1; }
tail -1 $o/tests_block.log
timeout -k 10 200 python bench.py --workload block --steps 200 --warmup 10 --cpu-seconds 5 > $o/bench_block.log 2>&1 || { echo "bench rc=$?"; tail $o/bench_block.log; exit 1; }
grep '^{' $o/bench_block.log | cut -c100-330
