#!/bin/bash
# fgan128train diagnostics: D per-layer probe + rocprof kernel stats of the bench line
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r03u
timeout -k 10 300 python -u tools/dtrain_probe.py 64 > gpurun_out/r03u/dprobe.log 2>&1 || { tail -30 gpurun_out/r03u/dprobe.log; exit 1; }
cat gpurun_out/r03u/dprobe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fgan_train.py tests/test_gpu_fgan_d.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u/tests.log 2>&1 || { tail -30 gpurun_out/r03u/tests.log; exit 1; }
tail -3 gpurun_out/r03u/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r03u/prof -o run -- python3 /root/repo/bench.py --workload fgan128train --steps 10 --warmup 2 --no-cpu-baseline > /root/repo/gpurun_out/r03u/bench_prof.log 2>&1 || { tail -30 /root/repo/gpurun_out/r03u/bench_prof.log; exit 1; }
f=$(ls /root/repo/gpurun_out/r03u/prof/*/run_kernel_stats.csv | head -1); head -30 "$f" | cut -c1-220
