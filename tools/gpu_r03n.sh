#!/bin/bash
# r03 session n: packed GELU in the deferred head transform: parity, per-kernel A/B (new vs base lib)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03n; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_timed_shapes.py -x -q --timeout 120 --timeout-method thread -k "defer or fgan" > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for v in "" _base "" _base; do
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd$v.so timeout -k 10 300 python bench.py --workload fgan128 --steps 30 --warmup 3 --no-cpu-baseline > $o/bench$v.log 2>&1 || { echo "bench rc=$?"; tail $o/bench$v.log; exit 1; }
  echo "$v $(grep '^{' $o/bench$v.log | cut -c150-230)"
  grep '^{' $o/bench$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  conv3_smallm', d['kernels']['conv3_smallm']['avg_us'])"
done
