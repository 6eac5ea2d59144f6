#!/bin/bash
# split-once wgrad: kernel tests, A/B probe on gan64train and fgan128train shapes, train parity tests
set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r03z
timeout -k 10 300 python -u tools/wgrad_probe.py 64 fgan128train > gpurun_out/r03z/wgrad_fgan.log 2>&1 || { tail -30 gpurun_out/r03z/wgrad_fgan.log; exit 1; }
tail -3 gpurun_out/r03z/wgrad_fgan.log
timeout -k 10 300 python -u tools/wgrad_probe.py 256 > gpurun_out/r03z/wgrad_gan64.log 2>&1 || { tail -30 gpurun_out/r03z/wgrad_gan64.log; exit 1; }
tail -3 gpurun_out/r03z/wgrad_gan64.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fgan_train.py tests/test_gpu_fgan_d.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z/tests.log 2>&1 || { tail -30 gpurun_out/r03z/tests.log; exit 1; }
tail -2 gpurun_out/r03z/tests.log
timeout -k 10 300 python -u bench.py --workload gan64train --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r03z/gan64train.log 2>&1 || { tail -20 gpurun_out/r03z/gan64train.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload fgan128train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03z/fgan128train.log 2>&1 || { tail -20 gpurun_out/r03z/fgan128train.log; exit 1; }
grep -h -o '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/r03z/gan64train.log gpurun_out/r03z/fgan128train.log
