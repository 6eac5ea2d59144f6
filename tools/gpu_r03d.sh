#!/bin/bash
# r03 session d: convq section probes (timing only: NOSTAGE / NOMFMA / NOBAR / NOEPI builds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/r03e; mkdir -p $o
for v in "" _p_COALB _p_NOA _p_NOA_COALB _q4 _p_NOSTAGE; do
  FFC_LIB_PATH=$PWD/fastfourierconvolution_amd/libffc_amd$v.so timeout -k 10 200 python tools/convq_probe.py 256 gen64 > $o/probe$v.log 2>&1 || { echo "probe $v rc=$?"; tail $o/probe$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $o/probe$v.log | sed -e 's/\[[^]]*\]//g'
done
