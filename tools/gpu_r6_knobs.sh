#!/bin/bash
# round 6 late knob A/Bs on ResNet-50 (same box, interleaved): 3x3 panel routing, side-stream TN grid
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/knobs
run() {  # tag, env...
  local tag=$1; shift
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py \
    > gpurun_out/r6/knobs/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/knobs/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run def_$r MI355X_DP_PANEL=1 || exit $?
  run p3x3_$r MI355X_DP_PANEL=5 || exit $?
done
