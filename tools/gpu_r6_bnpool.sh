#!/bin/bash
# round 6: stem BN+pool backward statistics pass with 2 rows per loop trip -- stem tests, isolated A/B,
# same-box step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/bnpool
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_stem_gpu.py tests/test_determinism_gpu.py > gpurun_out/r6/bnpool/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/bnpool/t.log
[ $rc -eq 0 ] || exit $rc
for r in a b; do
  MI355X_DP_BNPOOL_U=1 timeout -k 10 120 python tools/bench_bnpool.py || exit $?
  MI355X_DP_BNPOOL_U=2 timeout -k 10 120 python tools/bench_bnpool.py || exit $?
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6/bnpool/iso.log
run() {
  local tag=$1; shift
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py \
    > gpurun_out/r6/bnpool/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/bnpool/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b c; do
  run rn50_u1_$r MI355X_DP_BNPOOL_U=1 || exit $?
  run rn50_u2_$r MI355X_DP_BNPOOL_U=2 || exit $?
done
