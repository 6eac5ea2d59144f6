#!/bin/bash
# PMC evidence on the session-2 tree (MFMA busy, HBM traffic) + the strong-scaling per-rank shard steps
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
ROUND=r03s bash tools/pmc_round.sh gen64 fgan128 || exit $?
o=gpurun_out/s2h && mkdir -p $o
for b in 128 64 32; do
  timeout -k 10 300 python bench.py --batch $b --steps 200 --warmup 5 --no-cpu-baseline > $o/bench_gen64_shard_$b.log 2>&1 || { tail -20 $o/bench_gen64_shard_$b.log; exit 1; }
  grep -h -o '"ms_per_step": [0-9.]*, "ms_per_step_median": [0-9.]*' $o/bench_gen64_shard_$b.log
done
