#!/bin/bash
# fgan128train: D tests, D per-layer probe under rocprof, the bench line under rocprof (graph replays included)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r03w
timeout -k 10 300 python -u -m pytest tests/test_gpu_fgan_d.py tests/test_gpu_fgan_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03w/tests.log 2>&1 || { tail -30 gpurun_out/r03w/tests.log; exit 1; }
tail -2 gpurun_out/r03w/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/r03w/dprof -o run -- python3 /root/repo/tools/dtrain_probe.py 64 > /root/repo/gpurun_out/r03w/dprobe.log 2>&1 || { tail -30 /root/repo/gpurun_out/r03w/dprobe.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/r03w/prof -o run -- python3 /root/repo/bench.py --workload fgan128train --steps 10 --warmup 2 --no-cpu-baseline --profile-steps 1 > /root/repo/gpurun_out/r03w/bench.log 2>&1 || { tail -30 /root/repo/gpurun_out/r03w/bench.log; exit 1; }
head -c 400 /root/repo/gpurun_out/r03w/bench.log
head -25 /root/repo/gpurun_out/r03w/prof/run_kernel_stats.csv | cut -c1-160
