#!/bin/bash
# r03 session l: C2R single-latency load + residual prefetch: parity, rocprof of the fgan128 step (new vs base lib)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03m; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fu2d.py tests/test_gpu_parity.py tests/test_gpu_bn_fold.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for v in "" _base; do
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof$v -o run -- python3 bench.py --workload fgan128 --steps 10 --warmup 3 --no-cpu-baseline > $o/bench$v.log 2>&1 || { echo "prof rc=$?"; tail $o/bench$v.log; exit 1; }
  grep '^{' $o/bench$v.log | cut -c150-260
  f=$(find $o/prof$v -name "*kernel_stats.csv" | head -1); echo "== $v"; grep -E "c2r|r2c|mix_kernel|convq_kernel|conv3x3|bn_act" $f | cut -d, -f1-4 | sed -e 's/(anonymous namespace):://g' | cut -c1-140
done
