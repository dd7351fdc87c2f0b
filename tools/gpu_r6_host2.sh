#!/bin/bash
# round 6: where the host loses its run-ahead in the ResNet-50 bs256 step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/host
timeout -k 10 200 python tools/sync_probe.py > gpurun_out/r6/host/sync_probe.log 2>&1 || exit $?
tail -5 gpurun_out/r6/host/sync_probe.log
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d /tmp/r6tr -o run -- python3 bench.py --steps 6 --warmup 3 \
  > gpurun_out/r6/host/tr.bench.log 2> gpurun_out/r6/host/tr.err || exit $?
db=$(find /tmp/r6tr -name '*results.db' | head -1)
python tools/hip_api_top.py $db > gpurun_out/r6/host/api_top.md 2>&1
timeout -k 10 300 python tools/host_lead.py $db --step 5 > gpurun_out/r6/host/lead.md 2>&1
rc=$?
head -60 gpurun_out/r6/host/lead.md
rm -rf /tmp/r6tr
exit $rc
