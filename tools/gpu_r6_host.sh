#!/bin/bash
# round 6: is the ResNet-50 bs256 step host-bound anywhere?  Host time per step at small batches (the GPU
# share shrinks, the host's launch path stays), and the HIP API time of the bs256 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/host
run() {
  local tag=$1; shift
  MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py "$@" \
    > gpurun_out/r6/host/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/host/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
run b16 --batch 16 --steps 30 || exit $?
run b32 --batch 32 --steps 30 || exit $?
run b64 --batch 64 --steps 30 || exit $?
run b256 || exit $?
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/r6/host/tr -o run -- python3 bench.py --steps 6 --warmup 3 \
  > gpurun_out/r6/host/tr.bench.log 2> gpurun_out/r6/host/tr.err || exit $?
db=$(find gpurun_out/r6/host/tr -name '*results.db' | head -1)
python tools/hip_api_top.py $db > gpurun_out/r6/host/api_top.md 2>&1
head -30 gpurun_out/r6/host/api_top.md
python3 - "$db" > gpurun_out/r6/host/schema.txt 2>&1 <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for (n, s) in c.execute("select name, sql from sqlite_master where type in ('table','view')"):
    print(n, "::", (s or "")[:600])
PY
cp $db gpurun_out/r6/host/trace.db 2>/dev/null; ls -la gpurun_out/r6/host/trace.db
rm -rf gpurun_out/r6/host/tr
