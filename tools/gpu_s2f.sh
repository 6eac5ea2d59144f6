#!/bin/bash
# which build change broke the generator smoke: packed vs scalar split x SLP on/off
cd /root/repo && o=gpurun_out/s2f && mkdir -p $o
for v in cur pknoslp scslp old; do
  lib=""; [ $v != cur ] && lib=fastfourierconvolution_amd/libffc_amd_$v.so
  FFC_LIB_PATH=$lib timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke_$v.log 2>&1
  echo "$v rc=$? $(grep -h 'normwise' $o/smoke_$v.log | tail -1)"
done
