#!/bin/bash
# A round's measurement session: smoke, the whole -m gpu suite, the default bench lines (with CPU
# baselines), the gen64 strong-scaling shard steps, rocprofv3 kernel stats of gen64 and fgan128 and
# (PMC=1) the PMC passes of tools/pmc_round.sh.  Usage: [PMC=1] bash tools/gpu_round.sh <tag>
# (one-off experiments use tools/gpu_run.sh; the per-session scripts of earlier rounds are in git history)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-round}
o=gpurun_out/$tag; mkdir -p $o
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$o/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -h '^{' "$o/$name.log" | cut -c1-200
  [ $rc -eq 0 ] || { tail -20 "$o/$name.log"; exit $rc; }
}
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
if [ -z "${SKIP_TESTS:-}" ]; then
  run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
  tail -1 $o/tests.log
fi
run bench_gen64 300 python bench.py --cpu-seconds 10
run bench_fgan128 300 python bench.py --workload fgan128 --steps 50 --warmup 3 --cpu-seconds 10
run bench_fgan128sn 300 python bench.py --workload fgan128sn --steps 30 --warmup 3 --cpu-seconds 10
run bench_gan64train 300 python bench.py --workload gan64train --steps 50 --warmup 3 --cpu-seconds 10
run bench_block 300 python bench.py --workload block --cpu-seconds 10
run rocprof_gen64 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_gen64 -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline
run rocprof_fgan128 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_fgan128 -o run -- python3 bench.py --workload fgan128 --steps 10 --warmup 3 --no-cpu-baseline
run bench_fgan128train 300 python bench.py --workload fgan128train --steps 20 --warmup 3 --cpu-seconds 10
for b in 128 64 32; do
  run bench_gen64_shard_$b 300 python bench.py --batch $b --steps 200 --warmup 5 --no-cpu-baseline --scaling weak
done
if [ -n "${PMC:-}" ]; then ROUND=$tag bash tools/pmc_round.sh gen64 fgan128 || exit $?; fi
