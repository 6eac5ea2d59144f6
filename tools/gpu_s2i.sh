#!/bin/bash
# fused FU pass 1 split over channel groups (one wave per sample x 64/H channels) vs one workgroup per sample
set -o pipefail
cd /root/repo && o=gpurun_out/s2i && mkdir -p $o && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_timed_shapes.py tests/test_gpu_bn_fold.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
AB_STEPS=100 bash tools/ab_bench.sh cur+FFC_FU_SPLIT=0 cur 2>&1 | tee $o/ab_gen64.log
AB_ARGS="--workload fgan128" AB_STEPS=20 bash tools/ab_bench.sh cur+FFC_FU_SPLIT=0 cur 2>&1 | tee $o/ab_fgan128.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline > $o/rocprof.log 2>&1 || { tail -20 $o/rocprof.log; exit 1; }
grep -h "fu_" $o/prof/run_kernel_stats.csv | cut -d, -f1-4
