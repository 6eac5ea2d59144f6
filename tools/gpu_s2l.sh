#!/bin/bash
# which source group, built with -fno-slp-vectorize, breaks the B = 8 generator smoke
cd /root/repo && o=gpurun_out/s2l && mkdir -p $o
for v in "$@"; do
  FFC_LIB_PATH=fastfourierconvolution_amd/libffc_amd_$v.so timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke_$v.log 2>&1
  echo "$v rc=$? $(grep -h 'normwise' $o/smoke_$v.log | tail -1)"
done
