#!/bin/bash
# r03 session r: per-rank strong-scaling shard steps (gen64 B = 128 / 64 / 32) and the B = 32 kernel list
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03r; mkdir -p $o
export TMPDIR=/tmp
for B in 128 64 32; do
  timeout -k 10 200 python bench.py --batch $B --steps 400 --warmup 10 --no-cpu-baseline > $o/bench_$B.log 2>&1 || { echo "bench rc=$?"; tail $o/bench_$B.log; exit 1; }
  echo "B=$B $(grep '^{' $o/bench_$B.log | cut -c150-250)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof32 -o run -- python3 bench.py --batch 32 --steps 100 --warmup 5 --no-cpu-baseline > $o/prof32.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo ok
