#!/bin/bash
# round-3 final measurement on the final tree: smoke, all GPU tests, every bench line, rocprof gen64 +
# fgan128, PMC (MFMA busy, HBM traffic) for gen64 and fgan128, gen64 shard steps
set -o pipefail
cd /root/repo
bash tools/gpu_round3.sh r03final || exit $?
ROUND=r03f bash tools/pmc_round.sh gen64 fgan128 || exit $?
o=gpurun_out/r03final
for b in 128 64 32; do
  timeout -k 10 300 python bench.py --batch $b --steps 200 --warmup 5 --no-cpu-baseline > $o/bench_gen64_shard_$b.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --workload fgan128train --steps 20 --warmup 3 --cpu-seconds 10 > $o/bench_fgan128train.log 2>&1 || exit 1
grep -h '^{' $o/bench_fgan128train.log | cut -c1-200
