#!/bin/bash
# ConvT small-M: odd last output channel packed across input rows (v_pk_fma_f32) vs scalar
set -o pipefail
cd /root/repo && o=gpurun_out/s2o && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timed_shapes.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
AB_STEPS=200 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload gan64train" AB_STEPS=20 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_gan64train.log
