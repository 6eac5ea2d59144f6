#!/bin/bash
# session: tests for the C2R column packing, 2-level BN reduce, deferred head; gen64 + fgan128 benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-s5}
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_bn_reduce.py tests/test_gpu_fu2d.py tests/test_gpu_defer.py tests/test_gpu_bn_fold.py tests/test_gpu_sn_fp16.py tests/test_gpu_timed_shapes.py tests/test_gpu_rccl.py tests/test_gpu_syncbn_train.py} \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
for spec in ${BENCHES:-gen64:256 gen64:32 fgan128:512 fgan128:64}; do
  wl=${spec%%:*}; gb=${spec#*:}
  timeout -k 10 240 python bench.py --workload $wl --global-batch $gb --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
    > gpurun_out/${tag}_${wl}_$gb.log 2>&1 || { echo "bench $spec rc=$?"; tail -5 gpurun_out/${tag}_${wl}_$gb.log; exit 1; }
  python tools/bench_summary.py gpurun_out/${tag}_${wl}_$gb.log | head -14
done
