#!/bin/bash
# r04: name the kernel of the no-SLP generator miscompare (old tree 0363812, one file group no-SLP at a time)
cd /root/repo && o=gpurun_out/slp && mkdir -p $o
for v in "$@"; do
  lib=fastfourierconvolution_amd/libffc_amd_$v.so; [ $v = cur ] && lib=""
  FFC_LIB_PATH=$lib timeout -k 10 240 python -u tools/slp_probe.py 8 > $o/probe_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 $o/probe_$v.log)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
