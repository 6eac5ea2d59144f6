#!/bin/bash
# Two SQ counter passes (issue / wait / LDS) over short eager bench runs, one rocprofv3 run per pass
# (kernel-trace only): per-kernel averages into profiles/<ROUND>/pmc_diag_<workload>.json.
# usage: ROUND=r06 bash tools/pmc_diag.sh gen64 fgan128
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=${ROUND:-r06}
export TMPDIR=/tmp
mkdir -p profiles/$ROUND
for W in "$@"; do
  d=gpurun_out/pmcdiag_$ROUND/$W
  rm -rf $d; mkdir -p $d
  steps="--steps 2 --warmup 2"
  [ "$W" = gen64 ] && steps="--steps 3 --warmup 2"
  for pass in "a:SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES" \
              "b:SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d $d/$name -o run -- \
        python3 bench.py --workload $W $steps --no-cpu-baseline --no-graph --profile-steps 1 > $d/$name.log 2>&1
    rc=$?
    echo "$W pass $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $d/$name.log; exit $rc; fi
  done
  python3 tools/pmc_mfma.py $d profiles/$ROUND/pmc_diag_$W.json > /dev/null
  cp profiles/$ROUND/pmc_diag_$W.json gpurun_out/pmcdiag_$ROUND/
done
