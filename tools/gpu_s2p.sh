#!/bin/bash
# convq staging register slots 2 (cur) / 3 / 4 with the scalar split
set -o pipefail
cd /root/repo && o=gpurun_out/s2p && mkdir -p $o && export TMPDIR=/tmp
for v in sl3 sl4; do
  FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_convq.py -x -q --timeout 200 --timeout-method thread > $o/tests_$v.log 2>&1 || { tail -20 $o/tests_$v.log; exit 1; }
  tail -1 $o/tests_$v.log
done
AB_STEPS=200 bash tools/ab_bench.sh cur sl3 sl4 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur sl3 sl4 2>&1 | tee $o/ab_fgan128.log
