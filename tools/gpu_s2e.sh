#!/bin/bash
# round session on the current default (scalar split) + A/B: packed split (old), convq static priority
set -o pipefail
cd /root/repo
bash tools/gpu_round3.sh r03s3 || exit $?
o=gpurun_out/s2e && mkdir -p $o
AB_STEPS=100 bash tools/ab_bench.sh cur old prio1 prio2 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur old prio1 prio2 2>&1 | tee $o/ab_fgan128.log
AB_ARGS="--workload gan64train" AB_STEPS=20 bash tools/ab_bench.sh cur old 2>&1 | tee $o/ab_gan64train.log
