#!/bin/bash
# r03 session s: convq epilogue handed to the staging waves: parity, probes and benches (EPI on / off)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03s; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_convq.py tests/test_gpu_timed_shapes.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for e in 1 0; do
  FFC_CONVQ_EPI=$e timeout -k 10 200 python tools/convq_probe.py 256 gen64 > $o/probe_e$e.log 2>&1 || { echo "probe rc=$?"; tail $o/probe_e$e.log; exit 1; }
  echo "== epi $e"; grep -v amdgpu.ids $o/probe_e$e.log | sed -e 's/\[[^]]*\]//g' | cut -c1-200
  FFC_CONVQ_EPI=$e timeout -k 10 200 python tools/convq_probe.py 512 fgan128 > $o/probef_e$e.log 2>&1 || { echo "probe rc=$?"; tail $o/probef_e$e.log; exit 1; }
  grep -v amdgpu.ids $o/probef_e$e.log | sed -e 's/\[[^]]*\]//g' | cut -c1-60
done
for e in 1 0 1 0; do
  FFC_CONVQ_EPI=$e timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-cpu-baseline > $o/bench_e$e.log 2>&1 || { echo "bench rc=$?"; tail $o/bench_e$e.log; exit 1; }
  echo "gen64 epi $e $(grep '^{' $o/bench_e$e.log | cut -c150-230)"
done
for e in 1 0; do
  FFC_CONVQ_EPI=$e timeout -k 10 200 python bench.py --workload fgan128 --steps 30 --warmup 3 --no-cpu-baseline > $o/benchf_e$e.log 2>&1 || { echo "bench rc=$?"; tail $o/benchf_e$e.log; exit 1; }
  echo "fgan128 epi $e $(grep '^{' $o/benchf_e$e.log | cut -c170-260)"
done
