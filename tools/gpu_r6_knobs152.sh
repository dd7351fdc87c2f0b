#!/bin/bash
# ResNet-152 knob A/B (same box, interleaved): fused BN-backward finalize, side-stream TN grid
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/k152
run() {
  local tag=$1; shift
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model resnet152 \
    > gpurun_out/r6/k152/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/k152/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run def_$r MI355X_DP_BN_FUSED_FIN=0 || exit $?
  run fusedfin_$r MI355X_DP_BN_FUSED_FIN=1 || exit $?
  run side512_$r MI355X_DP_TN_BLOCKS_SIDE=512 || exit $?
done
