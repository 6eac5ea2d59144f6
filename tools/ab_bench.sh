#!/bin/bash
# A/B the in-tree library against variants, interleaved, in one GPU session.
# usage: tools/ab_bench.sh <variant>...   variant = cur | <name> (libffc_amd_<name>.so)
#        optionally suffixed +VAR=value (environment for that run), e.g. cur+FFC_TILE_ORDER=interleaved
#        AB_ARGS: extra bench.py arguments (e.g. "--workload fgan128"), AB_STEPS: timed steps,
#        AB_PREFIX: log-name prefix (gpurun_out/<prefix>ab_<variant>.log)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    name=${v%%+*}; envs=""
    if [ "$name" != "$v" ]; then envs=${v#*+}; fi
    if [ "$name" = cur ]; then lib=""; else lib="fastfourierconvolution_amd/libffc_amd_$name.so"; fi
    tag=$(echo "$v" | tr '+=/' '___')
    env FFC_LIB_PATH=$lib $envs timeout -k 10 300 python bench.py --steps ${AB_STEPS:-50} --warmup 5 --no-cpu-baseline ${AB_ARGS:-} \
      > gpurun_out/${AB_PREFIX:-}ab_$tag.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $v rc=$rc"; tail -5 gpurun_out/${AB_PREFIX:-}ab_$tag.log; exit $rc; fi
    python - "${AB_PREFIX:-}ab_$tag" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[1]:36s} {d['value']:10.0f} img/s {d['ms_per_step']:.4f} ms  " +
      " ".join(f"{k}={v['ms_per_step']*1e3:.0f}" for k, v in d["kernels"].items()))
PY
  done
done
