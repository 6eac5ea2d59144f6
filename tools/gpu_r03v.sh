#!/bin/bash
# D per-layer probe under rocprof kernel trace (which kernels the D's fwd / dgrad / wgrad run)
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r03v
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/r03v/prof -o run -- python3 /root/repo/tools/dtrain_probe.py 64 > /root/repo/gpurun_out/r03v/dprobe.log 2>&1 || { tail -30 /root/repo/gpurun_out/r03v/dprobe.log; exit 1; }
cat /root/repo/gpurun_out/r03v/dprobe.log
f=$(ls /root/repo/gpurun_out/r03v/prof/*/run_kernel_stats.csv /root/repo/gpurun_out/r03v/prof/run_kernel_stats.csv 2>/dev/null | head -1); head -30 "$f" | cut -c1-200
