#!/bin/bash
# One measurement session: smoke, every workload's bench line, rocprofv3 kernel stats of the gen64
# bench, PMC HBM traffic (gen64, fgan128) into gpurun_out/ (copy to profiles/<round>/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -h '^{' "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 gpurun_out/smoke.log
run bench_gen64 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 10
run bench_fgan128 300 python bench.py --workload fgan128 --steps 20 --warmup 3 --cpu-seconds 10
run bench_fgan128sn 300 python bench.py --workload fgan128sn --steps 20 --warmup 3 --cpu-seconds 10
run bench_gan64train 300 python bench.py --workload gan64train --steps 20 --warmup 3 --cpu-seconds 10
run rocprof_gen64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gen64 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
find gpurun_out/prof_gen64 -name "*stats*"
ROUND=${ROUND:-pmc} bash tools/pmc_traffic.sh || exit $?
ROUND=${ROUND:-pmc} WORKLOAD=fgan128 bash tools/pmc_traffic.sh || exit $?
cp profiles/${ROUND:-pmc}/pmc_traffic*.json gpurun_out/
