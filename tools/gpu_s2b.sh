#!/bin/bash
# small-M MFMA kernels: parity tests, gen64 / fgan128 A/B (FFC_SMALLM_MFMA=0 vs on), rocprof kernel stats
set -o pipefail
cd /root/repo && o=gpurun_out/s2b && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_defer.py tests/test_gpu_fu2d.py -x -q --timeout 300 --timeout-method thread -k "smallm or head or defer" > $o/tests.log 2>&1 || { tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_shapes.py -x -q --timeout 300 --timeout-method thread > $o/tests_timed.log 2>&1 || { tail -40 $o/tests_timed.log; exit 1; }
tail -2 $o/tests_timed.log
AB_STEPS=100 bash tools/ab_bench.sh cur+FFC_SMALLM_MFMA=0 cur 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=30 bash tools/ab_bench.sh cur+FFC_SMALLM_MFMA=0 cur 2>&1 | tee $o/ab_fgan128.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_gen64 -o run -- python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline > $o/rocprof_gen64.log 2>&1 || { tail -20 $o/rocprof_gen64.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_fgan128 -o run -- python3 bench.py --workload fgan128 --steps 10 --warmup 3 --no-cpu-baseline > $o/rocprof_fgan128.log 2>&1 || { tail -20 $o/rocprof_fgan128.log; exit 1; }
grep -h "smallm" $o/prof_gen64/run_kernel_stats.csv $o/prof_fgan128/run_kernel_stats.csv | cut -d, -f1-4
