#!/bin/bash
# round 6: ViT-B/16 bs256 -- same-box A/B of the library data-gradient GEMMs (MI355X_DP_BLAS_DGRAD)
# on the round-6 tree, then a steady-state kernel profile
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/vit
run() {
  local tag=$1; shift
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model vit_b_16 \
    > gpurun_out/r6/vit/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/vit/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run vit_def_$r || exit $?
  run vit_blas_$r MI355X_DP_BLAS_DGRAD=1 || exit $?
done
bash tools/r4_prof_grid.sh r6/vit/prof --model vit_b_16 || exit $?
head -40 gpurun_out/r6/vit/prof.summary.md
