#!/bin/bash
# parity-split C2R: FU tests, fgan128 A/B (fold off / from 64^2 / from 128^2), rocprof kernel stats
set -o pipefail
cd /root/repo && o=gpurun_out/s2a && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fu2d.py tests/test_gpu_parity.py tests/test_gpu_timed_shapes.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
AB_ARGS="--workload fgan128" AB_STEPS=30 bash tools/ab_bench.sh cur+FFC_C2R_FOLD=0 cur cur+FFC_C2R_FOLD=128 2>&1 | tee $o/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --workload fgan128 --steps 10 --warmup 3 --no-cpu-baseline > $o/rocprof.log 2>&1 || { tail -20 $o/rocprof.log; exit 1; }
grep -h "c2r" $o/prof/run_kernel_stats.csv | cut -d, -f1-5
