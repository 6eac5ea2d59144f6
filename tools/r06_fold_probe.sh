#!/bin/bash
# Round-6 probe of DESIGN 10c: the per-channel bn1 fold inside fu2d_r2c_mix, variants as libraries
# usage: tools/r06_fold_probe.sh <outdir> <variant>...   ("-" = the default library); env passes through
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
export R2C_PROBE_QUICK=1
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib=fastfourierconvolution_amd/libffc_amd_$v.so
  FFC_LIB_PATH=$lib timeout -k 10 240 python -u tools/experiments/r2cmix_st_repeat.py >> $out/probe.log 2>&1 || { echo "variant $v failed rc=$?" >> $out/probe.log; exit 1; }
done
grep -v amdgpu.ids $out/probe.log
