#!/bin/bash
# r03 session b: capture-mode probe per mode, the whole -m gpu suite, block + gen64 + fgan128 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03b; mkdir -p $o
export TMPDIR=/tmp
for m in global thread_local relaxed; do timeout -k 10 60 ./tools/capture_mode_probe $m >> $o/capture_mode_probe.json 2>&1 || exit 1; done
cat $o/capture_mode_probe.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for w in block gen64 fgan128; do
  timeout -k 10 300 python bench.py --workload $w --steps 100 --warmup 5 --cpu-seconds 5 > $o/bench_$w.log 2>&1 || { echo "bench $w rc=$?"; tail -20 $o/bench_$w.log; exit 1; }
  grep '^{' $o/bench_$w.log | cut -c1-400
done
