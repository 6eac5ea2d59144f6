#!/bin/bash
# Diagnostic PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a short eager
# bench run of one workload; per-kernel averages -> gpurun_out/pmc_diag_<W>/<i>/ + summary json.
# usage: bash tools/pmc_diag.sh <workload> "<group 1>" "<group 2>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
W=$1; shift
export TMPDIR=/tmp
d=gpurun_out/pmc_diag_$W; mkdir -p $d
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $d/g$i -o run -- \
      python3 bench.py --workload $W --steps 3 --warmup 2 --no-cpu-baseline --no-graph --profile-steps 1 > $d/g$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc ($grp)"
  if [ $rc -ne 0 ]; then tail -20 $d/g$i.log; exit $rc; fi
done
mkdir -p $d/all && rm -rf $d/all/* && for g in $d/g*/; do cp -r $g $d/all/; done
python3 tools/pmc_mfma.py $d/all $d/summary.json > /dev/null
python3 - "$d/summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, v in sorted(d.items(), key=lambda kv: -kv[1]["duration_us"])[:6]:
    print(k[:50], {c: round(x, 1) for c, x in v.items()})
PY
