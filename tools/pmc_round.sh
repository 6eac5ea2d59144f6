#!/bin/bash
# PMC evidence of one round (MI355X_MICROARCH.md recipe: one counter group per rocprofv3 run,
# kernel-trace only, short eager bench runs):
#   MFMA pass     SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -> pmc_mfma_<w>.json
#   traffic       FETCH_SIZE, WRITE_SIZE (separate passes)                              -> pmc_traffic[_<w>].json
# usage: ROUND=r03 bash tools/pmc_round.sh gen64 fgan128 fgan128sn
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r03}
export TMPDIR=/tmp
mkdir -p profiles/$ROUND
for W in "$@"; do
  d=gpurun_out/pmc_$ROUND/$W
  mkdir -p $d
  steps="--steps 3 --warmup 2"
  for pass in "mfma:SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d $d/$name -o run -- \
        python3 bench.py --workload $W $steps --no-cpu-baseline --no-graph --profile-steps 1 > $d/$name.log 2>&1
    rc=$?
    echo "$W pass $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $d/$name.log; exit $rc; fi
  done
  mkdir -p $d/m && rm -rf $d/m/* && cp -r $d/mfma $d/m/mfma && python3 tools/pmc_mfma.py $d/m profiles/$ROUND/pmc_mfma_$W.json | head -6
  mkdir -p $d/traffic && rm -rf $d/traffic/* && cp -r $d/fetch $d/traffic/fetch && cp -r $d/write $d/traffic/write
  out=pmc_traffic.json; [ "$W" != gen64 ] && out=pmc_traffic_$W.json
  python3 tools/pmc_traffic.py $d/traffic profiles/$ROUND/$out | head -6
  cp profiles/$ROUND/pmc_mfma_$W.json profiles/$ROUND/$out gpurun_out/pmc_$ROUND/
done
