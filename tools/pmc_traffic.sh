#!/bin/bash
# HBM-side traffic per kernel from rocprofv3 PMC counters (MI355X_MICROARCH.md §HBM):
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), kernel-trace only, over a short
# bench run; bytes/launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE counts half
# of a 16-B/lane stream).  Writes profiles/$ROUND/pmc_traffic.json (gen64) or pmc_traffic_$WORKLOAD.json (read by bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r01}
WORKLOAD=${WORKLOAD:-gen64}
OUT=pmc_traffic.json
[ "$WORKLOAD" != gen64 ] && OUT=pmc_traffic_$WORKLOAD.json
mkdir -p gpurun_out/pmc_traffic_$WORKLOAD profiles/$ROUND
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_traffic_$WORKLOAD/$c -o run -- \
      python bench.py --workload $WORKLOAD --steps 3 --warmup 2 --no-cpu-baseline --no-graph --profile-steps 1 \
      > gpurun_out/pmc_traffic_$WORKLOAD/$c.log 2>&1
  rc=$?
  echo "pass $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc_traffic_$WORKLOAD/$c.log; exit $rc; fi
done
python tools/pmc_traffic.py gpurun_out/pmc_traffic_$WORKLOAD profiles/$ROUND/$OUT
