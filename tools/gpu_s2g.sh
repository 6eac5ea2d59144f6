#!/bin/bash
# convq: select-free staging path for interior units vs select-all (r03 form)
set -o pipefail
cd /root/repo && o=gpurun_out/s2g && mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_convq.py tests/test_gpu_timed_shapes.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
AB_STEPS=100 bash tools/ab_bench.sh cur selall 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur selall 2>&1 | tee $o/ab_fgan128.log
