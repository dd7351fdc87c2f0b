#!/bin/bash
# round 6: ViT-B/16 with the weight-gradient side stream (auto = off for GEMM-bound models) -- same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/vitws
run() {
  local tag=$1; shift
  MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model vit_b_16 "$@" \
    > gpurun_out/r6/vitws/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/vitws/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'], d['config'].get('wgrad_stream'))"
}
for r in a b; do
  run auto_$r || exit $?
  run ws1_$r --wgrad-stream 1 || exit $?
done
