#!/bin/bash
# packed-f32 VALU beside MFMAs: scalar split (nopk) / no SLP packing (noslp) vs current
set -o pipefail
cd /root/repo && o=gpurun_out/s2d && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "smallm" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
AB_STEPS=100 bash tools/ab_bench.sh cur nopk noslp 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur nopk noslp 2>&1 | tee $o/ab_fgan128.log
AB_ARGS="--workload gan64train" AB_STEPS=20 bash tools/ab_bench.sh cur nopk noslp 2>&1 | tee $o/ab_gan64train.log
