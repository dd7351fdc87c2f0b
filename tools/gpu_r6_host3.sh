#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/host
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d /tmp/r6tr -o run -- python3 bench.py --steps 6 --warmup 3 \
  > gpurun_out/r6/host/tr3.bench.log 2> gpurun_out/r6/host/tr3.err || exit $?
db=$(find /tmp/r6tr -name '*results.db' | head -1)
timeout -k 10 300 python tools/host_lead.py $db --step 5 > gpurun_out/r6/host/lead3.md 2>&1
rc=$?
head -120 gpurun_out/r6/host/lead3.md | cut -c1-600
rm -rf /tmp/r6tr
exit $rc
