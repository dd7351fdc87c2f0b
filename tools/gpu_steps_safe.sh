#!/bin/bash
# Run "name:seconds:command" steps in order; a Python error (exit 1 / 2) does not stop the chain,
# a time limit (124 / 137), abort (134) or segfault (139) -- or anything else -- ends it.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "[step] $name (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[step] $name rc=$rc" | tee -a gpurun_out/steps.log
  case $rc in 0|1|2) ;; *) exit $rc ;; esac
done
