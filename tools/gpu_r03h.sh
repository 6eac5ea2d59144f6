#!/bin/bash
# r03 session h: re-tune convq (persistent) on every timed shape; write the table to gpurun_out
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03h; mkdir -p $o
cd tools && timeout -k 10 900 python -u tune_convq.py gen64:256,128,64,32 fgan128:1024,512,128,64 --out ../$o/convq_tuned.json > ../$o/tune.log 2>&1 || { echo "tune rc=$?"; tail -20 ../$o/tune.log; exit 1; }
grep -v amdgpu.ids ../$o/tune.log
