#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6
bash tools/gpu_r6_emul.sh > gpurun_out/r6/emul.txt 2>&1; rc=$?; echo "emul rc=$rc"; tail -14 gpurun_out/r6/emul.txt | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r6_pmc.sh > gpurun_out/r6/pmc.txt 2>&1; echo "pmc rc=$?"; tail -30 gpurun_out/r6/pmc.txt
