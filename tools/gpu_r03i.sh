#!/bin/bash
# r03 session i: full -m gpu suite + the default bench lines on the retuned persistent convq
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03i; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for w in gen64 fgan128 fgan128sn gan64train; do
  timeout -k 10 300 python bench.py --workload $w --steps 100 --warmup 5 --cpu-seconds 5 > $o/bench_$w.log 2>&1 || { echo "bench $w rc=$?"; tail -20 $o/bench_$w.log; exit 1; }
  grep '^{' $o/bench_$w.log | cut -c100-330
done
