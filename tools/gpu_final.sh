#!/bin/bash
# Round measurement session: smoke, the whole -m gpu suite, the four default bench lines (with CPU
# baselines), rocprofv3 kernel stats of the gen64 and fgan128 benches.  Copy gpurun_out/<tag>_* to
# profiles/<round>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-final}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -h '^{' "gpurun_out/${tag}_$name.log" | cut -c1-300
  [ $rc -eq 0 ] || { tail -20 "gpurun_out/${tag}_$name.log"; exit $rc; }
}
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/${tag}_smoke.log
if [ -z "${SKIP_TESTS:-}" ]; then
  run tests 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
  tail -2 gpurun_out/${tag}_tests.log
fi
run bench_gen64 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 10
run bench_fgan128 300 python bench.py --workload fgan128 --steps 20 --warmup 3 --cpu-seconds 10
run bench_fgan128sn 300 python bench.py --workload fgan128sn --steps 20 --warmup 3 --cpu-seconds 10
run bench_gan64train 300 python bench.py --workload gan64train --steps 20 --warmup 3 --cpu-seconds 10
run rocprof_gen64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_gen64 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
run rocprof_fgan128 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_fgan128 -o run -- python3 bench.py --workload fgan128 --steps 10 --warmup 3 --no-cpu-baseline
find gpurun_out/${tag}_prof_* -name "*kernel_stats*"
