#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; stop at the first step that
# timed out / aborted / segfaulted (never start more GPU work after a fault).
#   bash tools/gpu_steps.sh NAME SECONDS "cmd" [NAME SECONDS "cmd" ...]
# Each step's output goes to gpurun_out/<NAME>.log.
export TMPDIR=/tmp
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
  name="$1"; secs="$2"; cmd="$3"; shift 3
  echo "[step] $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[step] $name rc=$rc"
  tail -n 15 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139|136|135) echo "[step] fatal rc=$rc in $name -- stopping"; exit $rc ;;
  esac
done
exit 0
