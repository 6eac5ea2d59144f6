#!/bin/bash
# small-M MFMA probes: staging off / MFMA off / deeper staging, gen64 and fgan128
set -o pipefail
cd /root/repo && o=gpurun_out/s2c && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_defer.py -x -q --timeout 200 --timeout-method thread -k "smallm" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
AB_STEPS=100 bash tools/ab_bench.sh cur nostage s3 cur+FFC_SMALLM_MFMA=0 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur nostage s3 2>&1 | tee $o/ab_fgan128.log
