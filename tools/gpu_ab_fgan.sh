#!/bin/bash
# fgan128 A/B session: targeted GPU tests, then bench lines at B=64 and 512 with the deferred head
# (FFC_DEFER_HEAD) and the spilled-Y FU (FFC_FU2D_SPILL) on/off, then rocprof kernel stats at B=64.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${tag}_tests.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${tag}_tests.log | head -30; echo "tests rc=$rc"; exit $rc; }
fi
for gb in ${BATCHES:-64 512}; do
  for v in ${VARIANTS:-11 01 10 00}; do
    d=${v:0:1}; sp=${v:1:1}
    FFC_DEFER_HEAD=$d FFC_FU2D_SPILL=$sp timeout -k 10 240 python bench.py --workload fgan128 --global-batch $gb \
      --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_fgan_${gb}_$v.log 2>&1
    rc=$?
    echo "fgan128 B=$gb defer=$d spill=$sp rc=$rc"
    [ $rc -eq 0 ] || { tail -20 gpurun_out/${tag}_fgan_${gb}_$v.log; exit $rc; }
    python tools/bench_summary.py gpurun_out/${tag}_fgan_${gb}_$v.log 2>/dev/null | head -20 || true
  done
done
if [ -n "${PROF:-}" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
    python3 bench.py --workload fgan128 --global-batch 64 --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 gpurun_out/${tag}_prof.log; exit 1; }
  find gpurun_out/${tag}_prof -name "*kernel_stats*"
fi
