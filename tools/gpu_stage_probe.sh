#!/bin/bash
# r04: which fu2d kernel differs between a default build and a -fno-slp-vectorize build (tools/slp_stage_probe.py)
# usage: tools/gpu_stage_probe.sh <reference lib tag>:<suspect lib tag> ...
cd /root/repo && o=gpurun_out/slp && mkdir -p $o
for pair in "$@"; do
  ref=${pair%%:*}; sus=${pair#*:}
  FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_$ref.so timeout -k 10 120 python -u tools/slp_stage_probe.py ref $o/stages_$ref.pt || exit $?
  echo "== $sus vs $ref"
  FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_$sus.so timeout -k 10 120 python -u tools/slp_stage_probe.py cmp $o/stages_$ref.pt || exit $?
done
