#!/bin/bash
# A/B of an environment knob: VAR=name VALUES="a b" BENCHES="wl:B ..." bash tools/gpu_ab_env.sh tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-abenv}
for spec in $BENCHES; do
  wl=${spec%%:*}; gb=${spec#*:}
  for val in $VALUES; do
    env "$VAR=$val" timeout -k 10 240 python bench.py --workload $wl --global-batch $gb --steps ${STEPS:-20} --warmup 3 \
      --no-cpu-baseline > gpurun_out/${tag}_${wl}_${gb}_$val.log 2>&1 || { echo "bench $spec $val failed"; exit 1; }
    echo "$VAR=$val"; python tools/bench_summary.py gpurun_out/${tag}_${wl}_${gb}_$val.log | head -${LINES_:-4}
  done
done
