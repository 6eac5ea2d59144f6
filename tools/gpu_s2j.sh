#!/bin/bash
# multiply-free j = 0 / quarter-turn butterflies in fft_reg: full GPU suite + bench A/B vs the previous library
set -o pipefail
cd /root/repo && o=gpurun_out/s2j && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
AB_STEPS=100 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_fgan128.log
AB_ARGS="--workload gan64train" AB_STEPS=20 bash tools/ab_bench.sh prev cur 2>&1 | tee $o/ab_gan64train.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline > $o/rocprof.log 2>&1 || { tail -20 $o/rocprof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_f -o run -- python3 bench.py --workload fgan128 --steps 10 --warmup 3 --no-cpu-baseline > $o/rocprof_f.log 2>&1 || { tail -20 $o/rocprof_f.log; exit 1; }
grep -h "fu_\|fu2d" $o/prof/run_kernel_stats.csv $o/prof_f/run_kernel_stats.csv | cut -d, -f1-4
