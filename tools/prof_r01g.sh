#!/bin/bash
# rocprofv3 kernel traces/stats: gen64 bench (graph) and one eager gan64train step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gen64 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_gen64.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- python3 bench.py --workload gan64train --steps 2 --warmup 1 --no-graph --profile-steps 1 --no-cpu-baseline > gpurun_out/prof_train.log 2>&1 || exit $?
find gpurun_out/prof_gen64 gpurun_out/prof_train -name "*.csv"
