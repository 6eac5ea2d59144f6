#!/bin/bash
# whole-library -fno-slp-vectorize (noslp) vs the default build, with the GPU suite on noslp
set -o pipefail
cd /root/repo && o=gpurun_out/s2m && mkdir -p $o && export TMPDIR=/tmp
FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_noslp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests_noslp.log 2>&1 || { tail -30 $o/tests_noslp.log; exit 1; }
tail -1 $o/tests_noslp.log
AB_STEPS=100 bash tools/ab_bench.sh cur noslp 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur noslp 2>&1 | tee $o/ab_fgan128.log
AB_ARGS="--workload gan64train" AB_STEPS=20 bash tools/ab_bench.sh cur noslp 2>&1 | tee $o/ab_gan64train.log
