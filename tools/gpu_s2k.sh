#!/bin/bash
# BN apply planes: loads first, GELU on the branch-free pair form: full GPU suite + fgan128 A/B
set -o pipefail
cd /root/repo && o=gpurun_out/s2k && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_fgan128.log
AB_ARGS="--workload fgan128train" AB_STEPS=10 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_fgan128train.log
