#!/bin/bash
# One GPU session: the given pytest selection, then bench lines.  Usage:
#   TESTS="tests/x.py tests/y.py" BENCH="gen64:--global-batch 128;fgan128:" bash tools/gpu_session.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-s}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 180 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1
  rc=$?
  grep -E "PASS|FAIL|ERROR|per-layer|B=|passed|failed|loss" gpurun_out/${tag}_tests.log | tail -60
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
IFS=';' read -ra lines <<< "${BENCH:-}"
i=0
for l in "${lines[@]}"; do
  [ -z "$l" ] && continue
  wl=${l%%:*}; extra=${l#*:}
  i=$((i+1))
  timeout -k 10 300 python bench.py --workload $wl $extra > gpurun_out/${tag}_bench$i.log 2>&1
  rc=$?
  echo "bench $wl $extra rc=$rc"
  grep -h '^{' gpurun_out/${tag}_bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d.get(k) for k in ('value','ms_per_step','n_gpus')}, d['config'].get('global_batch'), d['config'].get('per_gpu_batch'), {k:(d.get('roofline') or {}).get(k) for k in ('kernel','frac','split_frac')}, (d.get('fft_roofline') or {}).get('frac'), d.get('parity'))" || true
  [ $rc -eq 0 ] || exit $rc
done
