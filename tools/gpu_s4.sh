#!/bin/bash
# session: deferred-head + small-tile ConvT tests, gen64 shard benches, fgan128 defer A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-s4}
timeout -k 10 400 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_timed_shapes.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
for gb in 32 64 256; do
  timeout -k 10 200 python bench.py --global-batch $gb --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_gen64_$gb.log 2>&1 || exit $?
  python tools/bench_summary.py gpurun_out/${tag}_gen64_$gb.log | head -12
done
BATCHES="512" VARIANTS="11 01" bash tools/gpu_ab_fgan.sh ${tag}
