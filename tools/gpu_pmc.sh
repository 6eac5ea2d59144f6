#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run -- \
      python bench.py --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 1 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc/p$i.log; exit $rc; fi
done
