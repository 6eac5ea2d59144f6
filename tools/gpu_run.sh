#!/bin/bash
# One GPU session: named steps, each under its own time limit, logs under gpurun_out/<tag>/.
# Stops at the first step that times out, aborts or crashes (rc 124/134/137/139); a step that
# merely fails (tests red, parity off) does not stop the later steps.
# usage: tools/gpu_run.sh <tag> "<name>:<seconds>:<command>" ...
cd /root/repo && tag=$1 && shift && o=gpurun_out/$tag && mkdir -p $o
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 $secs bash -c "$cmd" > $o/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -3 $o/$name.log
  case $rc in 124|134|137|139) echo "stopping after $name (rc $rc)"; exit $rc;; esac
done
exit 0
