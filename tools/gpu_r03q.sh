#!/bin/bash
# r03 session q: convq section trace on the current code (diagnostic build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03q; mkdir -p $o
export FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd_traceq.so
cd tools
for a in "0 256 2 gen64" "1 256 0 gen64" "2 256 0 gen64" "4 64 0 fgan128" "0 64 2 fgan128"; do
  timeout -k 10 120 python trace_convq.py $a >> ../$o/trace.log 2>&1 || { echo "trace $a rc=$?"; tail ../$o/trace.log; exit 1; }
done
grep -v amdgpu.ids ../$o/trace.log
