#!/bin/bash
# r03 session g: fgan128 layers on convq (forced, persistent) vs convp
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03g; mkdir -p $o
for B in 512 64; do
timeout -k 10 300 python tools/convq_probe.py $B fgan128 > $o/probe_fgan128_$B.log 2>&1 || { echo "probe rc=$?"; tail $o/probe_fgan128_$B.log; exit 1; }
echo "== B=$B"; grep -v amdgpu.ids $o/probe_fgan128_$B.log | sed -e 's/\[[^]]*\]//g'
done
