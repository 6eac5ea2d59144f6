#!/bin/bash
# fgan128 Discriminator / training-iteration parity tests + the fgan128train bench line
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r03t
timeout -k 10 400 python -u -m pytest tests/test_gpu_fgan_d.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r03t/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03t/tests.log; exit 1; }
tail -15 gpurun_out/r03t/tests.log
timeout -k 10 400 python -u bench.py --workload fgan128train --steps 20 --warmup 3 --cpu-seconds 10 \
  > gpurun_out/r03t/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/r03t/bench.log; exit 1; }
tail -c 3000 gpurun_out/r03t/bench.log
